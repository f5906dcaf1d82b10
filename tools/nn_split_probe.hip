// nn_split_probe.hip — diagnostic (never the product): is a per-column layer of k_nn_forward
// (224 tokens x 128 outputs x K = 128, one 512-thread workgroup, A in LDS, B from L2) faster on
// bf16 MFMAs with fp32 operands split into three bf16 parts (x = hi + mid + lo exactly to
// 2^-24), and is its error no larger than the f32 MFMA's? Variants:
//   0  v_mfma_f32_32x32x2_f32 (the shipping scheme: K halves on the lane halves, float4 steps)
//   1  v_mfma_f32_32x32x16_bf16, 8 products (all but lo*lo), hi*hi in its own accumulator
//   2  6 products (drops mid*lo, lo*mid), two accumulators
//   3  6 products, one accumulator
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o /tmp/nn_split_probe tools/nn_split_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int T = 224, N = 128, K = 128, XS = 132, NNT = 512;
constexpr int S = K / 2, Q = S / 4, C16 = K / 16;

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; i++) z[i] = 0.f;
    return z;
}
__device__ __forceinline__ int acc_row(int r) { return (r & 3) + 8 * (r >> 2) + 4 * ((threadIdx.x & 63) >> 5); }

// x (8 floats) -> hi, mid, lo bf16 parts (truncations: hi + mid + lo = x to 2^-24 |x|)
__device__ __forceinline__ void split8(const float4 &x0, const float4 &x1, bf16x8 &hi, bf16x8 &mid, bf16x8 &lo) {
    const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    uint32_t h[8], m[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t u = __float_as_uint(xs[j]);
        h[j] = u & 0xFFFF0000u;
        const float r1 = xs[j] - __uint_as_float(h[j]);
        m[j] = __float_as_uint(r1) & 0xFFFF0000u;
        const float r2 = r1 - __uint_as_float(m[j]);
        l[j] = __float_as_uint(r2);
    }
    u32x4 H, M, L;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        H[p] = (h[2 * p] >> 16) | h[2 * p + 1];
        M[p] = (m[2 * p] >> 16) | m[2 * p + 1];
        L[p] = (l[2 * p] >> 16) | (l[2 * p + 1] & 0xFFFF0000u);
    }
    hi = __builtin_bit_cast(bf16x8, H);
    mid = __builtin_bit_cast(bf16x8, M);
    lo = __builtin_bit_cast(bf16x8, L);
}

template <int V>
__global__ __launch_bounds__(NNT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_probe(
    const float *__restrict__ A, const float4 *__restrict__ W32, const bf16x8 *__restrict__ Wb, float *out, int reps, float zr) {
    __shared__ __align__(16) float buf[T * XS];
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int wc = w & 3, wg = w >> 2, t0 = 4 * wg, ntok = wg ? 3 : 4;
    for (int i = tid; i < T * K; i += NNT) buf[(i / K) * XS + i % K] = A[i];
    __syncthreads();
    const int li = lane & 31, h = lane >> 5;
    f32x16 acc[4], acl[4];
#pragma unroll
    for (int t = 0; t < 4; t++) { acc[t] = zero16(); acl[t] = zero16(); }
    for (int rep = 0; rep < reps; rep++) {
        // (zr = 0 at run time: every rep starts from zero, but depends on the previous one)
#pragma unroll
        for (int t = 0; t < 4; t++) { acc[t] *= zr; acl[t] *= zr; }
        if constexpr (V == 0) {
            const float4 *w4 = W32 + (size_t)wc * Q * 64 + lane;
            float4 b = w4[0], bn;
#pragma unroll
            for (int q = 0; q < Q; q++) {
                if (q + 1 < Q) bn = w4[(q + 1) * 64];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    if (t < ntok) {
                        const float4 a = *reinterpret_cast<const float4 *>(buf + ((t0 + t) * 32 + li) * XS + h * S + 4 * q);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc[t], 0, 0, 0);
                    }
                }
                b = bn;
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
            const bf16x8 *wb = Wb + (size_t)wc * C16 * 3 * 64 + lane;
            bf16x8 b0 = wb[0], b1 = wb[64], b2 = wb[128], n0, n1, n2;
#pragma unroll
            for (int c = 0; c < C16; c++) {
                if (c + 1 < C16) { n0 = wb[(3 * (c + 1)) * 64]; n1 = wb[(3 * (c + 1) + 1) * 64]; n2 = wb[(3 * (c + 1) + 2) * 64]; }
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    if (t < ntok) {
                        const float *ap = buf + ((t0 + t) * 32 + li) * XS + 16 * c + 8 * h;
                        bf16x8 a0, a1, a2;
                        split8(*reinterpret_cast<const float4 *>(ap), *reinterpret_cast<const float4 *>(ap + 4), a0, a1, a2);
                        f32x16 &lo = V == 3 ? acc[t] : acl[t];
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[t], 0, 0, 0);
                        lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, lo, 0, 0, 0);
                        lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, lo, 0, 0, 0);
                        lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, lo, 0, 0, 0);
                        lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, lo, 0, 0, 0);
                        lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, lo, 0, 0, 0);
                        if constexpr (V == 1) {
                            lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b2, lo, 0, 0, 0);
                            lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b1, lo, 0, 0, 0);
                        }
                    }
                }
                b0 = n0; b1 = n1; b2 = n2;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    if (blockIdx.x == 0) {
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (t < ntok)
#pragma unroll
                for (int r = 0; r < 16; r++)
                    out[((t0 + t) * 32 + acc_row(r)) * N + 32 * wc + li] = (V == 1 || V == 2) ? acc[t][r] + acl[t][r] : acc[t][r];
    }
}

static uint16_t trunc16(float x) { uint32_t u; memcpy(&u, &x, 4); return (uint16_t)(u >> 16); }
static float f16hi(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char **argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 1024, reps = argc > 2 ? atoi(argv[2]) : 16;
    std::vector<float> A(T * K), B(K * N);
    srand(7);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    for (auto &x : A) x = fmaxf(rnd(), 0.f) * 3.f;           // post-ReLU activations
    for (auto &x : B) x = rnd() * 0.1f;
    // f32 packing: [nt][q][lane] float4 {B[h S + 4q + j][32 nt + (lane & 31)]}
    std::vector<float> W32((size_t)4 * Q * 64 * 4);
    for (int nt = 0; nt < 4; nt++)
        for (int q = 0; q < Q; q++)
            for (int l = 0; l < 64; l++)
                for (int j = 0; j < 4; j++)
                    W32[(((size_t)nt * Q + q) * 64 + l) * 4 + j] = B[((l >> 5) * S + 4 * q + j) * N + 32 * nt + (l & 31)];
    // bf16 parts: [nt][c][part][lane] x 8 {B[16c + 8h + j][col]}
    std::vector<uint16_t> Wb((size_t)4 * C16 * 3 * 64 * 8);
    for (int nt = 0; nt < 4; nt++)
        for (int c = 0; c < C16; c++)
            for (int l = 0; l < 64; l++)
                for (int j = 0; j < 8; j++) {
                    const float x = B[(16 * c + 8 * (l >> 5) + j) * N + 32 * nt + (l & 31)];
                    const uint16_t hh = trunc16(x);
                    const float r1 = x - f16hi(hh);
                    const uint16_t mm = trunc16(r1);
                    const float r2 = r1 - f16hi(mm);
                    const uint16_t ll = trunc16(r2);
                    const uint16_t parts[3] = {hh, mm, ll};
                    for (int p = 0; p < 3; p++) Wb[((((size_t)nt * C16 + c) * 3 + p) * 64 + l) * 8 + j] = parts[p];
                }
    std::vector<double> ref(T * N), mag(T * N);
    for (int i = 0; i < T; i++)
        for (int n = 0; n < N; n++) {
            double s = 0, m = 0;
            for (int k = 0; k < K; k++) { s += (double)A[i * K + k] * B[k * N + n]; m += fabs((double)A[i * K + k] * B[k * N + n]); }
            ref[i * N + n] = s; mag[i * N + n] = m;
        }
    float *dA, *dW32, *dout;
    void *dWb;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dW32, W32.size() * 4); hipMalloc(&dWb, Wb.size() * 2);
    hipMalloc(&dout, T * N * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dW32, W32.data(), W32.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dWb, Wb.data(), Wb.size() * 2, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](int v, int rp) {
        switch (v) {
            case 0: hipLaunchKernelGGL(k_probe<0>, dim3(grid), dim3(NNT), 0, 0, dA, (const float4 *)dW32, (const bf16x8 *)dWb, dout, rp, 0.f); break;
            case 1: hipLaunchKernelGGL(k_probe<1>, dim3(grid), dim3(NNT), 0, 0, dA, (const float4 *)dW32, (const bf16x8 *)dWb, dout, rp, 0.f); break;
            case 2: hipLaunchKernelGGL(k_probe<2>, dim3(grid), dim3(NNT), 0, 0, dA, (const float4 *)dW32, (const bf16x8 *)dWb, dout, rp, 0.f); break;
            default: hipLaunchKernelGGL(k_probe<3>, dim3(grid), dim3(NNT), 0, 0, dA, (const float4 *)dW32, (const bf16x8 *)dWb, dout, rp, 0.f); break;
        }
    };
    for (int v = 0; v < 4; v++) {
        run(v, 1);
        hipDeviceSynchronize();
        std::vector<float> o(T * N);
        hipMemcpy(o.data(), dout, T * N * 4, hipMemcpyDeviceToHost);
        double emax = 0, erel = 0, esum = 0;
        for (int i = 0; i < T * N; i++) {
            const double e = fabs((double)o[i] - ref[i]);
            emax = fmax(emax, e); erel = fmax(erel, e / mag[i]); esum += e / mag[i];
        }
        run(v, reps);
        hipEventRecord(e0);
        for (int it = 0; it < 5; it++) run(v, reps);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1000.0 / 5, flop = 2.0 * T * N * K * (double)grid * reps;
        printf("{\"variant\": %d, \"us\": %.1f, \"tflops_f32_equiv\": %.1f, \"max_abs_err\": %.3e, \"max_rel_err_sum_abs\": %.3e, \"mean_rel\": %.3e}\n",
               v, us, flop / us * 1e-6, emax, erel, esum / (T * N));
    }
    return 0;
}
