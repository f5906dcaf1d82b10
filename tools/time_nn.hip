// Diagnostic: per-layer cycle probes of k_nn_forward<2> (NN_TIMING build): 32768 leaves,
// random int8 boards, random packed weights (timing only; values are not checked).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNN_TIMING=1 \
//        -o tools/time_nn tools/time_nn.hip
#include "../alphazero-general-ori_amd/csrc/nnet.hip"
#include <cstdio>
#include <random>
#include <vector>
int main() {
    const int B = 32768, R = 56, ITERS = 20;
    const int nw = spl_nn_packed_floats(2);
    std::vector<float> hw(nw);
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> ud(-0.05f, 0.05f);
    for (auto &x : hw) x = ud(rng);
    std::vector<int8_t> hs((size_t)B * R * 7);
    for (auto &x : hs) x = (int8_t)(rng() % 9);
    std::vector<uint64_t> hm((size_t)B * 7, ~0ull);
    float *w, *pi, *v; int8_t *st; uint64_t *mk;
    (void)hipMalloc(&w, nw * 4); (void)hipMalloc(&pi, (size_t)B * 409 * 4); (void)hipMalloc(&v, (size_t)B * 8);
    (void)hipMalloc(&st, hs.size()); (void)hipMalloc(&mk, hm.size() * 8);
    (void)hipMemcpy(w, hw.data(), nw * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(st, hs.data(), hs.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(mk, hm.data(), hm.size() * 8, hipMemcpyHostToDevice);
    for (int i = 0; i < 5; i++) spl_nn_forward(2, B, st, mk, w, pi, v, nullptr);
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_nn_timing), z, sizeof(z));
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < ITERS; i++) spl_nn_forward(2, B, st, mk, w, pi, v, nullptr);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[16];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_nn_timing), sizeof(h));
    const double wg = (double)((B + 31) / 32) * ITERS;
    const double flops = 2.0 * 595328.0 * B;
    printf("k_nn_forward: %.1f us per launch, %.1f TFLOP/s\n", ms * 1e3 / ITERS, flops / (ms * 1e-3 / ITERS) / 1e12);
    const char *names[] = {"input staging", "dense2d_1 (K=R)", "dense2d_1[3]", "partialgpool_1", "dense2d_3",
                           "col pool", "dense1d_4 (K=704)", "pgp4 + d5a + d5b + pgp5", "heads PI0/V0", "PI1 + V1",
                           "softmax"};
    for (int k = 0; k < 11; k++) printf("  %-26s %8.0f cycles per workgroup\n", names[k], h[k] / wg);
    return 0;
}
