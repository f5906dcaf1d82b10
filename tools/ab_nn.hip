// Diagnostic A/B of k_nn_forward without probes: average launch time over 50 launches
// (HIP events) at B = 32768 and 16384 leaves, 2 and 4 players, random int8 boards and
// weights (timing only). Build against the product kernel or a variant copied next to
// this file (its include of splendor_amd.h adjusted):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-DNNET_SRC='"<file>"'] \
//         -o tools/ab_nn tools/ab_nn.hip
#ifndef NNET_SRC
#define NNET_SRC "../alphazero-general-ori_amd/csrc/nnet.hip"
#endif
#include NNET_SRC
#include <cstdio>
#include <random>
#include <vector>
static void run(int n, int B) {
    const int R = 32 + 10 * n + n * n, ITERS = 50;
    const int nw = spl_nn_packed_floats(n);
    std::vector<float> hw(nw);
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> ud(-0.05f, 0.05f);
    for (auto &x : hw) x = ud(rng);
    std::vector<int8_t> hs((size_t)B * R * 7);
    for (auto &x : hs) x = (int8_t)(rng() % 9);
    std::vector<uint64_t> hm((size_t)B * 7, ~0ull);
    float *w, *pi, *v; int8_t *st; uint64_t *mk;
    (void)hipMalloc(&w, nw * 4); (void)hipMalloc(&pi, (size_t)B * 409 * 4); (void)hipMalloc(&v, (size_t)B * 16);
    (void)hipMalloc(&st, hs.size()); (void)hipMalloc(&mk, hm.size() * 8);
    (void)hipMemcpy(w, hw.data(), nw * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(st, hs.data(), hs.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(mk, hm.data(), hm.size() * 8, hipMemcpyHostToDevice);
    for (int i = 0; i < 20; i++) spl_nn_forward(n, B, st, mk, w, pi, v, nullptr);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < ITERS; i++) spl_nn_forward(n, B, st, mk, w, pi, v, nullptr);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / ITERS;
    printf("%s n=%d B=%d: %.1f us per launch, %.1f TFLOP/s (flops per leaf from bench: 1.19 M at n=2)\n", NNET_SRC, n, B,
           us, 2.0 * 595328.0 * B / (us * 1e-6) / 1e12);
    (void)hipFree(w); (void)hipFree(pi); (void)hipFree(v); (void)hipFree(st); (void)hipFree(mk);
}
int main() {
    run(2, 32768); run(2, 16384); run(4, 16384); run(2, 32768);
    return 0;
}
