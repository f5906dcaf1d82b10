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
// value-free leaves (v = 0, like a random-init network's near-zero values): deep trees
__global__ void zero_values(float *v, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = 0.f;
}
int main(int argc, char **argv) {
    // argv: [sims=100] [warm iterations=3000] [timed iterations=1000] [node_cap=2048] [zero values=0]
    // self-play steady state (spl_mcts_commit), genbu args, hash-prior network
    const int B = 32768;
    const int SIMS = argc > 1 ? atoi(argv[1]) : 100;
    const int WARM = argc > 2 ? atoi(argv[2]) : 3000, ITERS = argc > 3 ? atoi(argv[3]) : 1000;
    const int ZV = argc > 5 ? atoi(argv[5]) : 0;   // 1: hash priors, v = 0; 2: SplendorNNet, small random weights
    float *nw = nullptr;
    if (ZV == 2) {
        const int nf = spl_nn_packed_floats(2);
        std::vector<float> hw(nf);
        uint32_t x = 12345;
        for (auto &f : hw) { x = x * 1664525u + 1013904223u; f = ((x >> 8) * (1.0f / 16777216.0f) - 0.5f) * 0.1f; }
        (void)hipMalloc(&nw, (size_t)nf * 4);
        (void)hipMemcpy(nw, hw.data(), (size_t)nf * 4, hipMemcpyHostToDevice);
    }
    spl_ctx *c; spl_ctx_create(2, 10, &c);
    spl_mcts_config cfg{};
    cfg.num_sims = SIMS; cfg.ratio_full = 5; cfg.prob_full = 0.25; cfg.cpuct = 2.5; cfg.fpu = 0.3;
    cfg.node_cap = argc > 4 ? atoi(argv[4]) : 2048; cfg.edge_cap = 32 * cfg.node_cap; cfg.seed = 0x5EED;
    cfg.temp_threshold = 10; cfg.dirichlet_alpha = 0.3; cfg.dirichlet_temp = 1.25; cfg.selfplay = 1;
    cfg.out_cap = 64 * B;
    spl_mcts *m; if (spl_mcts_create(c, B, &cfg, &m)) { printf("create failed\n"); return 1; }
    int8_t *leaf; uint64_t *mk; uint8_t *lv; float *pi, *v; int32_t *cnt;
    (void)hipMalloc(&leaf, (size_t)B * 392); (void)hipMalloc(&mk, (size_t)B * 56);
    (void)hipMalloc(&lv, B); (void)hipMalloc(&pi, (size_t)B * 409 * 4); (void)hipMalloc(&v, (size_t)B * 8);
    (void)hipMalloc(&cnt, 4);
    spl_mcts_reset_games(m, nullptr);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int it = 0; it < WARM + ITERS; it++) {
        if (it == WARM) {
            unsigned long long z[24] = {0};
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_select_timing), z, sizeof(z));
            (void)hipEventRecord(e0);
        }
        spl_mcts_select(m, leaf, mk, lv, nullptr);
        if (ZV == 2) spl_nn_forward(2, B, leaf, mk, nw, pi, v, nullptr);   // small random weights
        else spl_hash_eval(c, B, leaf, mk, pi, v, nullptr);
        if (ZV == 1) zero_values<<<(2 * B + 255) / 256, 256>>>(v, 2 * B);
        spl_mcts_backup(m, mk, pi, v, nullptr);
        spl_mcts_commit(m, nullptr);
        if (it % 500 == 499) spl_mcts_drain_examples(m, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, cnt, nullptr);
    }
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[24];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_select_timing), sizeof(h));
    const char *names[] = {"root load", "descend: loop top", "pick_edge: UCB + argmax", "make_move + roll",
                           "fingerprint + hash", "node checks (to next level)", "leaf: store + mask", "headers",
                           "pick_edge: edge loads"};
    const double calls = (double)h[21];
    printf("node_cap %d edge_cap %d, arena %.2f GB\n", cfg.node_cap, cfg.edge_cap, spl_mcts_device_bytes(m) / 1e9);
    printf("%d sims, %d trees, steady state after %d iterations: %.1f us per select+hash_eval+backup+commit iteration; "
           "%.0f probed waves, %.2f levels/sim\n", SIMS, B, WARM, ms * 1e3 / ITERS, calls, h[20] / calls);
    for (int k = 0; k < 9; k++) printf("  %-28s %8.0f cycles per select\n", names[k], h[k] / calls);
    printf("  levels repeating the previous simulation's path: %.2f per simulation (of %.2f)\n", h[22] / calls,
           h[23] / calls);
    return 0;
}
