// Diagnostic: per-workgroup phase cycle totals of k_rollout<2> over one K-move launch
// (clock64 per phase, wall-clock block lifetime, placement). Timing only.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DROLLOUT_TIMING=1 \
//        -o tools/time_rollout tools/time_rollout.hip
#include "../alphazero-general-ori_amd/csrc/splendor_env.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
#include <cstdlib>
int main(int argc, char **argv) {
    // argv: [K = moves per launch, 100]
    const int B = 32768, NB = B / 64, K = argc > 1 ? atoi(argv[1]) : 100;
    spl_ctx *c; spl_ctx_create(2, 10, &c);
    int8_t *st, *pl; uint64_t *mk; int16_t *ac; float *en; int32_t *gd; uint64_t *tm;
    (void)hipMalloc(&st, (size_t)B * 392); (void)hipMalloc(&pl, B); (void)hipMalloc(&mk, (size_t)K * B * 56);
    (void)hipMalloc(&ac, (size_t)K * 2 * B); (void)hipMalloc(&en, (size_t)K * 8 * B); (void)hipMalloc(&gd, 4 * B);
    (void)hipMalloc(&tm, (size_t)NB * 40 * 8);
    (void)hipMemset(gd, 0, 4 * B);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rollout_timing), &tm, sizeof(tm));
    spl_init(c, B, st, pl, nullptr, 0, 0x5EED, 0xFFFFFFFFu, 0, nullptr);
    for (int k = 0; k < 5; k++) spl_rollout_run(c, B, K, st, pl, mk, ac, en, gd, 0x5EED, K * k, 0, nullptr);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h((size_t)NB * 40);
    // probe slots (splendor_env.hip / splendor_device.h SPL_PROBE)
    // (thread 0 = lane 0 of wave 0: its move-phase slots see the gem-move pipeline)
    const int slots[] = {0, 16, 17, 1, 5, 6, 7, 2, 9, 8, 3, 4};
    const char *names[] = {"load", "predicates (w0)", "predicate sync", "mask words+sync", "select",
                           "mask store+make_move (w0)", "end check (w0)", "outputs (w0)", "deal philox (w0)",
                           "deal board (w0)", "tail to sync", "store"};
    const bool per_move[] = {false, true, true, true, true, true, true, true, true, true, true, false};
    const int NS = 12;
    for (int rep = 0; rep < 2; rep++) {
        spl_rollout_run(c, B, K, st, pl, mk, ac, en, gd, 0x5EED, 200 + K * rep, 0, nullptr);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), tm, h.size() * 8, hipMemcpyDeviceToHost);
        uint64_t w0 = ~0ull, w1 = 0;
        std::vector<double> ph[NS], life;
        for (int b = 0; b < NB; b++) {
            const uint64_t *r = &h[(size_t)b * 40];
            w0 = std::min(w0, r[24]); w1 = std::max(w1, r[25]);
            for (int k = 0; k < NS; k++) ph[k].push_back((double)r[slots[k]] / (per_move[k] ? K : 1));
            life.push_back((double)(r[25] - r[24]) / 100.0);
        }
        printf("rep %d: K=%d moves, kernel span %.2f us (%.2f us/move)\n", rep, K, (w1 - w0) / 100.0, (w1 - w0) / 100.0 / K);
        for (int k = 0; k < NS; k++) {
            std::sort(ph[k].begin(), ph[k].end());
            printf("  %-22s cycles%s p10 %8.0f  p50 %8.0f  p90 %8.0f  max %8.0f\n", names[k],
                   per_move[k] ? "/move" : "     ", ph[k][NB / 10], ph[k][NB / 2], ph[k][NB * 9 / 10], ph[k][NB - 1]);
        }
        std::sort(life.begin(), life.end());
        printf("  block life us p10 %.2f p50 %.2f p90 %.2f max %.2f\n", life[NB / 10], life[NB / 2], life[NB * 9 / 10], life[NB - 1]);
        double xw = 0, xl = 0;
        for (int b = 0; b < NB; b++) { xw += (double)h[(size_t)b * 40 + 18]; xl += (double)h[(size_t)b * 40 + 19]; }
        printf("  exact-path waves per wave-move %.4f, lanes per board-move %.5f\n", xw / (NB * 4.0 * K), xl / (NB * 64.0 * K));
        printf("  move phase per wave (gems / buy / reserve / buy reserved), cycles/move:");
        for (int k = 0; k < 4; k++) {
            double x = 0;
            for (int b = 0; b < NB; b++) x += (double)h[(size_t)b * 40 + 20 + k];
            printf(" %.0f", x / (NB * (double)K));
        }
        printf("\n");
        printf("  move pipeline before deals per wave, cycles/move:");
        for (int k = 0; k < 4; k++) {
            double x = 0;
            for (int b = 0; b < NB; b++) x += (double)h[(size_t)b * 40 + 26 + k];
            printf(" %.0f", x / (NB * (double)K));
        }
        printf("\n  make_move done per wave (lane 0 when it has a board; summed over moves / K):");
        for (int k = 0; k < 4; k++) {
            double x = 0;
            for (int b = 0; b < NB; b++) x += (double)h[(size_t)b * 40 + 30 + k];
            printf(" %.0f", x / (NB * (double)K));
        }
        printf("\n");
    }
    return 0;
}
