// Diagnostic: time k_rollout<2> phase ablations in one process (interleaved rounds).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DROLLOUT_ABLATE=<k> \
//        -o ablate_<k> tools/ablate_rollout.hip ; outputs are not checked (timing only).
#include "../alphazero-general-ori_amd/csrc/splendor_env.hip"
#include <cstdio>
#include <vector>
int main() {
    const int B = 32768, K = 200;
    spl_ctx *c; spl_ctx_create(2, 10, &c);
    int8_t *st, *pl; uint64_t *mk; int16_t *ac; float *en; int32_t *gd;
    (void)hipMalloc(&st, (size_t)B * 392); (void)hipMalloc(&pl, B); (void)hipMalloc(&mk, (size_t)B * 56);
    (void)hipMalloc(&ac, 2 * B); (void)hipMalloc(&en, 8 * B); (void)hipMalloc(&gd, 4 * B);
    (void)hipMemset(gd, 0, 4 * B);
    spl_init(c, B, st, pl, nullptr, 0, 0x5EED, 0xFFFFFFFFu, 0, nullptr);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int r = 0; r < 3; r++) {
        for (int k = 0; k < 20; k++) spl_rollout_step(c, B, st, pl, mk, ac, en, gd, 0x5EED, k, 0, nullptr);
        (void)hipEventRecord(a);
        for (int k = 0; k < K; k++) spl_rollout_step(c, B, st, pl, mk, ac, en, gd, 0x5EED, 100 + k, 0, nullptr);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("ablate=%d round %d: %.2f us/step\n", ROLLOUT_ABLATE, r, ms * 1000 / K);
    }
    return 0;
}
