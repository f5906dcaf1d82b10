// Diagnostic: cycle probes inside k_select<2> (tools build only; MCTS_TIMING). Runs B trees
// of hash-prior searches (spl_hash_eval as the network) through the C ABI and reports the
// cycles the first wave of each workgroup spends per stage, summed over the run.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMCTS_TIMING=1 \
//        tools/time_select.hip -Lalphazero-general-ori_amd -lsplendor_amd -o tools/time_select
// Run:   LD_LIBRARY_PATH=alphazero-general-ori_amd tools/time_select
#include "../alphazero-general-ori_amd/csrc/mcts.hip"
#include <cstdio>
#include <vector>
#include <cstdlib>
int main(int argc, char **argv) {
    const int B = 32768, SIMS = 100, MOVES = 3;
    const int emul = argc > 1 ? atoi(argv[1]) : 32;   // edge_cap = emul x node_cap
    spl_ctx *c; spl_ctx_create(2, 10, &c);
    spl_mcts_config cfg{};
    cfg.num_sims = SIMS; cfg.ratio_full = 1; cfg.prob_full = 1.0; cfg.cpuct = 2.5; cfg.fpu = 0.3;
    cfg.node_cap = 4 * SIMS + 64; cfg.edge_cap = emul * cfg.node_cap; cfg.seed = 0x5EED; cfg.temp_threshold = 10;
    cfg.dirichlet_temp = 1.0;
    spl_mcts *m; if (spl_mcts_create(c, B, &cfg, &m)) { printf("create failed\n"); return 1; }
    int8_t *st, *leaf; uint64_t *mk; uint8_t *lv; float *pi, *v;
    (void)hipMalloc(&st, (size_t)B * 392); (void)hipMalloc(&leaf, (size_t)B * 392); (void)hipMalloc(&mk, (size_t)B * 56);
    (void)hipMalloc(&lv, B); (void)hipMalloc(&pi, (size_t)B * 409 * 4); (void)hipMalloc(&v, (size_t)B * 8);
    spl_init(c, B, st, nullptr, nullptr, 0, 0x5EED, 0xFFFFFFFFu, 0, nullptr);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int mv = 0; mv < MOVES; mv++) {
        spl_mcts_set_roots(m, st, mv > 0, 1, nullptr);
        if (mv == MOVES - 1) {
            unsigned long long z[24] = {0};
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_select_timing), z, sizeof(z));
            (void)hipEventRecord(e0);
        }
        for (int s = 0; s < SIMS; s++) {
            spl_mcts_select(m, leaf, mk, lv, nullptr);
            spl_hash_eval(c, B, leaf, mk, pi, v, nullptr);
            spl_mcts_backup(m, mk, pi, v, nullptr);
        }
    }
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[24];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_select_timing), sizeof(h));
    const char *names[] = {"root load", "descend: loop top", "pick_edge: UCB + argmax", "make_move + roll",
                           "fingerprint + hash", "node checks (to next level)", "leaf: store + mask", "headers",
                           "pick_edge: edge loads"};
    const double calls = (double)h[21];
    printf("edge_cap %d, arena %.2f GB\n", cfg.edge_cap, spl_mcts_device_bytes(m) / 1e9);
    printf("%d sims x %d trees: %.1f us per select+hash_eval+backup iteration; %.0f probed waves, %.2f levels/sim\n",
           SIMS, B, ms * 1e3 / SIMS, calls, h[20] / calls);
    for (int k = 0; k < 9; k++) printf("  %-28s %8.0f cycles per select\n", names[k], h[k] / calls);
    return 0;
}
