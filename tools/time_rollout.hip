// Diagnostic: per-workgroup phase timestamps of k_rollout<2> (clock64 deltas per phase,
// wall-clock block lifetime, XCC / CU placement). Timing only; outputs are not checked.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DROLLOUT_TIMING=1 \
//        -o tools/time_rollout tools/time_rollout.hip
#include "../alphazero-general-ori_amd/csrc/splendor_env.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
int main() {
    const int B = 32768, NB = B / 64;
    spl_ctx *c; spl_ctx_create(2, 10, &c);
    int8_t *st, *pl; uint64_t *mk; int16_t *ac; float *en; int32_t *gd; uint64_t *tm;
    (void)hipMalloc(&st, (size_t)B * 392); (void)hipMalloc(&pl, B); (void)hipMalloc(&mk, (size_t)B * 56);
    (void)hipMalloc(&ac, 2 * B); (void)hipMalloc(&en, 8 * B); (void)hipMalloc(&gd, 4 * B);
    (void)hipMalloc(&tm, (size_t)NB * 8 * 8);
    (void)hipMemset(gd, 0, 4 * B);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rollout_timing), &tm, sizeof(tm));
    spl_init(c, B, st, pl, nullptr, 0, 0x5EED, 0xFFFFFFFFu, 0, nullptr);
    for (int k = 0; k < 120; k++) spl_rollout_step(c, B, st, pl, mk, ac, en, gd, 0x5EED, k, 0, nullptr);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h((size_t)NB * 8);
    const char *names[] = {"load+philox", "mask", "step", "reset", "store(wall)"};
    for (int rep = 0; rep < 3; rep++) {
        spl_rollout_step(c, B, st, pl, mk, ac, en, gd, 0x5EED, 200 + rep, 0, nullptr);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), tm, h.size() * 8, hipMemcpyDeviceToHost);
        uint64_t w0 = ~0ull, w1 = 0;
        std::vector<double> ph[4], life;
        std::vector<int> per_cu(4096, 0);
        for (int b = 0; b < NB; b++) {
            const uint64_t *r = &h[(size_t)b * 8];
            w0 = std::min(w0, r[0]); w1 = std::max(w1, r[6]);
            for (int k = 0; k < 4; k++) ph[k].push_back((double)(r[k + 2] - r[k + 1]));
            life.push_back((double)(r[6] - r[0]) / 100.0);   // wall clock 100 MHz -> us
            const uint32_t hw = (uint32_t)r[7], xcc = (uint32_t)(r[7] >> 32) & 0xF;
            const int cu = (hw >> 8) & 0xF, se = (hw >> 13) & 0x7;
            per_cu[(xcc * 8 + se) * 16 + cu]++;
        }
        printf("rep %d: kernel span (first block start -> last block end) %.2f us\n", rep, (w1 - w0) / 100.0);
        for (int k = 0; k < 4; k++) {
            std::sort(ph[k].begin(), ph[k].end());
            printf("  %-12s cycles p10 %8.0f  p50 %8.0f  p90 %8.0f  max %8.0f\n", names[k], ph[k][NB / 10],
                   ph[k][NB / 2], ph[k][NB * 9 / 10], ph[k][NB - 1]);
        }
        std::sort(life.begin(), life.end());
        printf("  block life us p10 %.2f p50 %.2f p90 %.2f max %.2f\n", life[NB / 10], life[NB / 2], life[NB * 9 / 10], life[NB - 1]);
        int hist[8] = {0};
        for (int v : per_cu) if (v < 8) hist[v]++;
        printf("  CUs by block count: 0:%d 1:%d 2:%d 3:%d 4:%d\n", hist[0], hist[1], hist[2], hist[3], hist[4]);
        // start-time spread
        std::vector<double> st0;
        for (int b = 0; b < NB; b++) st0.push_back((h[(size_t)b * 8] - w0) / 100.0);
        std::sort(st0.begin(), st0.end());
        printf("  block start offset us p50 %.2f p90 %.2f max %.2f\n", st0[NB / 2], st0[NB * 9 / 10], st0[NB - 1]);
    }
    return 0;
}
