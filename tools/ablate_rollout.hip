// Diagnostic: time k_rollout<2> (32768 boards) as one launch per move and as K-move launches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DROLLOUT_ABLATE=<k> \
//        -o tools/ablate_<k> tools/ablate_rollout.hip ; outputs are not checked (timing only).
//        ROLLOUT_ABLATE: 0 = full, 1 = skip mask, 2 = skip move.
#include "../alphazero-general-ori_amd/csrc/splendor_env.hip"
#include <cstdio>
int main() {
    const int B = 32768, T = 200;
    spl_ctx *c; spl_ctx_create(2, 10, &c);
    int8_t *st, *pl; uint64_t *mk; int16_t *ac; float *en; int32_t *gd;
    (void)hipMalloc(&st, (size_t)B * 392); (void)hipMalloc(&pl, B); (void)hipMalloc(&mk, (size_t)T * B * 56);
    (void)hipMalloc(&ac, (size_t)T * 2 * B); (void)hipMalloc(&en, (size_t)T * 8 * B); (void)hipMalloc(&gd, 4 * B);
    (void)hipMemset(gd, 0, 4 * B);
    spl_init(c, B, st, pl, nullptr, 0, 0x5EED, 0xFFFFFFFFu, 0, nullptr);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    uint32_t step = 0;
    for (int K : {1, 1, 10, 20, 50, 200}) {
        spl_rollout_run(c, B, K, st, pl, mk, ac, en, gd, 0x5EED, step, 0, nullptr);   // warm
        step += K;
        (void)hipEventRecord(a);
        for (int k = 0; k < T / K; k++, step += K) spl_rollout_run(c, B, K, st, pl, mk, ac, en, gd, 0x5EED, step, 0, nullptr);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("ablate=%d K=%3d moves/launch: %.2f us/move  %.1f M rollouts/s\n", ROLLOUT_ABLATE, K, ms * 1000 / T,
               (double)B * T / (ms * 1e-3) / 1e6);
    }
    return 0;
}
