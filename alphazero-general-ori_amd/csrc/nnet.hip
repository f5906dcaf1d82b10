// nnet.hip — SplendorNNet inference (SplendorNNet.py:56-159, eval mode) as one fused
// gfx950 kernel: int8 leaf boards + packed legality masks in, masked softmax policy and
// tanh values out (GenericNNetWrapper.predict, :141-168). C ABI: include/splendor_amd.h.
//
// One 512-thread workgroup (8 waves, two per SIMD so one wave's LDS / L2 latency hides
// behind the other's MFMAs) evaluates ML = 32 leaves through all 13 dense layers with every
// activation on chip:
//   * GEMMs on v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation: the reference
//     network's precision). Wave w owns output columns [32(w&3), 32(w&3)+32) of a 128-wide
//     layer; the two wave groups (w>>2) split the token tiles of the per-column layers and
//     the K range of the per-leaf layers (partial sums combined through LDS).
//   * The per-board-column layers (dense2d_1, dense2d_3, partialgpool_1) treat the 7 board
//     columns of the 32 leaves as 7 token tiles of 32 (channel-major), so the per-column
//     BatchNorm affine is uniform across an MFMA tile.
//   * K is split in halves across the two lane halves of the MFMA (lane half h feeds
//     k = s + h*S at step s), so a lane's A operand for 4 steps is one ds_read_b128 and
//     its B operand one coalesced global float4 from the pre-packed weights (pack order in
//     splendor_amd.h, spl_nn_forward).
//   * Activations live in LDS with a 132-float row stride (= 4 mod 64 dwords: the 16 lanes
//     of a ds_read_b128 group hit distinct 16-byte bank slots).
#include <hip/hip_runtime.h>

#include "../../include/splendor_amd.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NNT = 512;       // threads per workgroup (8 waves)
constexpr int ML = 32;         // leaves per workgroup
constexpr int XS = 132;        // activation row stride (floats)
constexpr int LS = 420;        // logits row stride (floats)
constexpr int ACT = 409;

__host__ __device__ constexpr int kpad(int K) { return (K + 7) / 8 * 8; }
__host__ __device__ constexpr int ntiles(int N) { return (N + 31) / 32; }
__host__ __device__ constexpr int wfloats(int N, int K) { return ntiles(N) * 32 * kpad(K); }

// layer order of the packed weights: dense2d_1, dense2d_1[3], partialgpool_1 dense,
// dense2d_3, dense1d_4, partialgpool_4 dense, dense1d_5[0], dense1d_5[3], partialgpool_5
// dense, PI[0], PI[1], V[0], V[1]; then the per-column BN affines s1, t1, sp1, tp1 (7 each)
template <int NP>
struct Net {
    static constexpr int R = 32 + 10 * NP + NP * NP;
    static constexpr int NL = 13;
    static constexpr int Ns[NL] = {128, 128, 120, 128, 128, 120, 128, 128, 120, 128, ACT, 128, NP};
    static constexpr int Ks[NL] = {R, 128, 96, 128, 704, 112, 128, 128, 112, 128, 128, 128, 128};
    static constexpr int woff(int l) {
        int o = 0;
        for (int j = 0; j < l; j++) o += wfloats(Ns[j], Ks[j]) + ntiles(Ns[j]) * 32;
        return o;
    }
    static constexpr int boff(int l) { return woff(l) + wfloats(Ns[l], Ks[l]); }
    static constexpr int AFF = woff(NL);
    static constexpr int TOTAL = AFF + 28;
    static constexpr int X0S = (kpad(R) / 4) % 2 ? kpad(R) : kpad(R) + 4;   // int8 input stride (odd dwords)
};

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; i++) z[i] = 0.f;
    return z;
}

__device__ __forceinline__ void mfma4(const float4 &a, const float4 &b, f32x16 &acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
}

// token tiles t0 .. t0+nt_tok-1 (<= T) x one N tile (column block nt) over K = 2S
// wp: packed weights of the layer; afetch(t, col) -> float4 of A[token tile t][lane row][col..col+3]
template <int T, int S, class AF>
__device__ __forceinline__ void gemm_tiles(const float *__restrict__ wp, int nt, int t0, int nt_tok, AF afetch,
                                           f32x16 acc[T]) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const float4 *w4 = reinterpret_cast<const float4 *>(wp) + (size_t)nt * (S / 4) * 64 + lane;
#pragma unroll
    for (int t = 0; t < T; t++) acc[t] = zero16();
    float4 bn = w4[0];
#pragma unroll 2
    for (int s4 = 0; s4 < S / 4; s4++) {
        const float4 b = bn;
        if (s4 + 1 < S / 4) bn = w4[(s4 + 1) * 64];
#pragma unroll
        for (int t = 0; t < T; t++)
            if (t < nt_tok) mfma4(afetch(t0 + t, h * S + 4 * s4), b, acc[t]);
    }
}

// one token tile x up to NT column blocks {nt0, nt0 + step, ...} < ntot (shared A operand),
// over the step range [q0, q1) of the S/4 float4 steps
template <int NT, int S, class AF>
__device__ __forceinline__ void gemm_cols(const float *__restrict__ wp, int nt0, int step, int ntot, int q0, int q1,
                                          AF afetch, f32x16 acc[NT]) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < NT; j++) acc[j] = zero16();
    const float4 *w4 = reinterpret_cast<const float4 *>(wp) + lane;
#pragma unroll 2
    for (int s4 = q0; s4 < q1; s4++) {
        const float4 a = afetch(0, h * S + 4 * s4);
#pragma unroll
        for (int j = 0; j < NT; j++) {
            const int nt = nt0 + j * step;
            if (nt < ntot) mfma4(a, w4[((size_t)nt * (S / 4) + s4) * 64], acc[j]);
        }
    }
}

// accumulator element r of this lane: (row, col) of the 32x32 tile (C/D map of gfx950)
__device__ __forceinline__ int acc_row(int r) { return (r & 3) + 8 * (r >> 2) + 4 * ((threadIdx.x & 63) >> 5); }
__device__ __forceinline__ int acc_col() { return threadIdx.x & 31; }

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

template <int NP>
__global__ __launch_bounds__(NNT) void k_nn_forward(int B, const int8_t *__restrict__ state,
                                                    const uint64_t *__restrict__ mask,
                                                    const float *__restrict__ W, float *__restrict__ pi_out,
                                                    float *__restrict__ v_out) {
    using Nt = Net<NP>;
    constexpr int R = Nt::R, X0S = Nt::X0S;
    __shared__ __align__(16) float bufA[7 * ML * XS];      // per-column activations / logits
    __shared__ __align__(16) float bufP[ML * XS];          // per-leaf ping
    __shared__ __align__(16) float bufQ[ML * XS];          // per-leaf pong
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, li = lane & 31;
    const int wc = w & 3, wg = w >> 2;                     // column block, wave group
    const int b0 = blockIdx.x * ML, nb = min(ML, B - b0);
    const float *aff = W + Nt::AFF;                        // s1, t1, sp1, tp1
    float *scratch = bufA + 7 * ML * XS - 4 * 16 * 64;     // split-K partials (per-leaf layers)
    const int t0 = 4 * wg, ntok = wg ? 3 : 4;              // this wave's token tiles (per-column layers)

    // ---- input: x[column c][leaf i][row r] = state[leaf][r][c] as int8 (token c*32+i)
    int8_t *x0 = reinterpret_cast<int8_t *>(bufA);
    for (int j = tid; j < 7 * ML * X0S / 4; j += NNT) reinterpret_cast<int32_t *>(x0)[j] = 0;
    __syncthreads();
    for (int j = tid; j < nb * 7 * R; j += NNT) {
        const int i = j / (7 * R), rem = j - i * 7 * R, r = rem / 7, c = rem - 7 * r;
        x0[(c * ML + i) * X0S + r] = state[(size_t)(b0 + i) * 7 * R + rem];
    }
    __syncthreads();

    f32x16 acc[4];
    const int col = 32 * wc + acc_col();
    // per-column epilogue over this wave's token tiles: dst = f(acc, t, n)
    auto store_tiles = [&](int coloff, auto f) {
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (t < ntok)
#pragma unroll
                for (int r = 0; r < 16; r++)
                    bufA[((t0 + t) * ML + acc_row(r)) * XS + coloff] = f(acc[t][r], t0 + t);
    };
    auto fetchA = [&](int col0) {
        return [&, col0](int t, int c) { return ld4(bufA + (t * ML + li) * XS + col0 + c); };
    };
    // ---- dense2d_1: relu(s1[c] * (W1 x + b1) + t1[c])
    {
        constexpr int S = kpad(R) / 2;
        gemm_tiles<4, S>(W + Nt::woff(0), wc, t0, ntok, [&](int t, int c) {
            const int v = *reinterpret_cast<const int32_t *>(x0 + (t * ML + li) * X0S + c);
            return make_float4((float)(int8_t)v, (float)(int8_t)(v >> 8), (float)(int8_t)(v >> 16), (float)(v >> 24));
        }, acc);
        __syncthreads();
        const float bias = W[Nt::boff(0) + col];
        store_tiles(col, [&](float x, int t) { return fmaxf((x + bias) * aff[t] + aff[7 + t], 0.f); });
        __syncthreads();
    }
    // ---- dense2d_1[3]: relu(W2 x + b2)
    {
        gemm_tiles<4, 64>(W + Nt::woff(1), wc, t0, ntok, fetchA(0), acc);
        __syncthreads();
        const float bias = W[Nt::boff(1) + col];
        store_tiles(col, [&](float x, int) { return fmaxf(x + bias, 0.f); });
        __syncthreads();
    }
    // ---- partialgpool_1: [max, mean over 4 groups of 8 of x[0:32]] ++ relu(BN(Wp1 x[32:] + bp1))
    {
        gemm_tiles<4, 48>(W + Nt::woff(2), wc, t0, ntok, fetchA(32), acc);
        constexpr int NQ = (7 * ML * 8 + NNT - 1) / NNT;
        float pv[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int item = tid + NNT * q, tok = item >> 3, j = item & 7, g = j & 3;
            pv[q] = 0.f;
            if (item < 7 * ML * 8) {
                const float *p = bufA + tok * XS + 8 * g;
                float m = p[0], s = p[0];
#pragma unroll
                for (int k = 1; k < 8; k++) { m = fmaxf(m, p[k]); s += p[k]; }
                pv[q] = j < 4 ? m : s / 8.f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int item = tid + NNT * q;
            if (item < 7 * ML * 8) bufA[(item >> 3) * XS + (item & 7)] = pv[q];
        }
        if (col < 120) {
            const float bias = W[Nt::boff(2) + col];
            store_tiles(8 + col, [&](float x, int t) { return fmaxf((x + bias) * aff[14 + t] + aff[21 + t], 0.f); });
        }
        __syncthreads();
    }
    // ---- dense2d_3: relu(W3 x + b3)
    {
        gemm_tiles<4, 64>(W + Nt::woff(3), wc, t0, ntok, fetchA(0), acc);
        __syncthreads();
        const float bias = W[Nt::boff(3) + col];
        store_tiles(col, [&](float x, int) { return fmaxf(x + bias, 0.f); });
        __syncthreads();
    }
    // ---- FlattenAndPartialGPool(64, 5): pool[i] = [max_c<5 x[c][i][0:64], mean_c<5 ...]
    for (int item = tid; item < ML * 64; item += NNT) {
        const int i = item >> 6, f = item & 63;
        float m = bufA[i * XS + f], s = m;
#pragma unroll
        for (int c = 1; c < 5; c++) {
            const float x = bufA[(c * ML + i) * XS + f];
            m = fmaxf(m, x);
            s += x;
        }
        bufP[i * XS + f] = m;
        bufP[i * XS + 64 + f] = s / 5.f;
    }
    __syncthreads();
    // per-leaf layer, 4 column blocks, K split between the wave groups; the summed tile goes to
    // group 0, which applies f(x, n) and writes dst (f returns NaN-free values only for n < nmax)
    auto leaf_layer = [&](auto gemm, float *dst, int dst_off, int nmax, auto f) {
        gemm();
        __syncthreads();
        if (wg) {
#pragma unroll
            for (int r = 0; r < 16; r++) scratch[(wc * 16 + r) * 64 + lane] = acc[0][r];
        }
        __syncthreads();
        if (!wg && col < nmax) {
#pragma unroll
            for (int r = 0; r < 16; r++)
                dst[acc_row(r) * XS + dst_off + col] = f(acc[0][r] + scratch[(wc * 16 + r) * 64 + lane]);
        }
        __syncthreads();
    };
    // ---- dense1d_4 over the 704 flattened features: [pool 128][x[5][:64]][x[6][:64]][x[c][64:128], c<7]
    {
        const float bias = W[Nt::boff(4) + col];
        leaf_layer([&] {
            gemm_cols<1, 352>(W + Nt::woff(4), wc, 4, 4, 44 * wg, 44 * wg + 44, [&](int, int k) {
                if (k < 128) return ld4(bufP + li * XS + k);
                if (k < 256) return ld4(bufA + ((5 + ((k - 128) >> 6)) * ML + li) * XS + ((k - 128) & 63));
                return ld4(bufA + (((k - 256) >> 6) * ML + li) * XS + 64 + ((k - 256) & 63));
            }, acc);
        }, bufQ, 0, 128, [&](float x) { return fmaxf(x + bias, 0.f); });
    }
    // partial pool over 4 groups of 4 of x[0:16] ++ relu(Wp x[16:] + bp) (BN folded): src -> dst
    auto pool44 = [&](const float *src, float *dst, int layer) {
        float pv = 0.f;
        if (tid < ML * 8) {
            const int i = tid >> 3, j = tid & 7, g = j & 3;
            const float *p = src + i * XS + 4 * g;
            pv = j < 4 ? fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3])) : (p[0] + p[1] + p[2] + p[3]) / 4.f;
        }
        const float bias = col < 120 ? W[Nt::boff(layer) + col] : 0.f;
        leaf_layer([&] {
            gemm_cols<1, 56>(W + Nt::woff(layer), wc, 4, 4, 7 * wg, 7 * wg + 7,
                             [&](int, int c) { return ld4(src + li * XS + 16 + c); }, acc);
        }, dst, 8, 120, [&](float x) { return fmaxf(x + bias, 0.f); });
        if (tid < ML * 8) dst[(tid >> 3) * XS + (tid & 7)] = pv;
        __syncthreads();
    };
    auto dense128 = [&](const float *src, float *dst, int layer) {
        const float bias = W[Nt::boff(layer) + col];
        leaf_layer([&] {
            gemm_cols<1, 64>(W + Nt::woff(layer), wc, 4, 4, 8 * wg, 8 * wg + 8,
                             [&](int, int c) { return ld4(src + li * XS + c); }, acc);
        }, dst, 0, 128, [&](float x) { return fmaxf(x + bias, 0.f); });
    };
    pool44(bufQ, bufP, 5);                  // partialgpool_4
    dense128(bufP, bufQ, 6);                // dense1d_5[0] (+BN folded)
    dense128(bufQ, bufP, 7);                // dense1d_5[3]
    pool44(bufP, bufQ, 8);                  // partialgpool_5 -> trunk output in bufQ
    // ---- heads: PI[0] (group 0) and V[0] (group 1), no activation
    {
        const int layer = wg ? 11 : 9;
        gemm_cols<1, 64>(W + Nt::woff(layer), wc, 4, 4, 0, 16, [&](int, int c) { return ld4(bufQ + li * XS + c); },
                         acc);
        __syncthreads();
        const float bias = W[Nt::boff(layer) + col];
        float *dst = wg ? bufA : bufP;
#pragma unroll
        for (int r = 0; r < 16; r++) dst[acc_row(r) * XS + col] = acc[0][r] + bias;
        __syncthreads();
    }
    float *logits = bufA + ML * XS;
    // ---- PI[1] (409 outputs, 13 column blocks over 8 waves) and V[1] (NP outputs, wave 7)
    {
        gemm_cols<2, 64>(W + Nt::woff(10), w, 8, ntiles(ACT), 0, 16, [&](int, int c) { return ld4(bufP + li * XS + c); },
                         acc);
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int nt = w + 8 * j;
            if (nt < ntiles(ACT)) {
                const int n = 32 * nt + acc_col();
                const float bias = W[Nt::boff(10) + n];
#pragma unroll
                for (int r = 0; r < 16; r++) logits[acc_row(r) * LS + n] = acc[j][r] + bias;
            }
        }
        if (w == 7) {
            gemm_cols<1, 64>(W + Nt::woff(12), 0, 1, 1, 0, 16, [&](int, int c) { return ld4(bufA + li * XS + c); },
                             acc);
            const int n = acc_col();
            if (n < NP) {
                const float bias = W[Nt::boff(12) + n];
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int i = acc_row(r);
                    if (i < nb) v_out[(size_t)(b0 + i) * NP + n] = tanhf(acc[0][r] + bias);
                }
            }
        }
        __syncthreads();
    }
    // ---- masked softmax (invalid -> -1e8, as the reference's masked_fill + log_softmax)
    constexpr int PERW = ML / (NNT / 64);
    for (int i = w * PERW; i < (w + 1) * PERW; i++) {
        if (i >= nb) break;
        const uint64_t *mk = mask + (size_t)(b0 + i) * 7;
        float x[7];
        float m = -3.0e38f;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const int a = 64 * k + lane;
            const bool ok = a < ACT && ((mk[k] >> lane) & 1);
            x[k] = a < ACT ? (ok ? logits[i * LS + a] : -1e8f) : -3.0e38f;
            m = fmaxf(m, x[k]);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            x[k] = 64 * k + lane < ACT ? expf(x[k] - m) : 0.f;
            s += x[k];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        const float inv = 1.f / s;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const int a = 64 * k + lane;
            if (a < ACT) pi_out[(size_t)(b0 + i) * ACT + a] = x[k] * inv;
        }
    }
}

inline int check_launch() { return hipGetLastError() == hipSuccess ? 0 : SPL_EDEVICE; }

}  // namespace

extern "C" {

int spl_nn_packed_floats(int n_players) {
    switch (n_players) {
        case 2: return Net<2>::TOTAL;
        case 3: return Net<3>::TOTAL;
        case 4: return Net<4>::TOTAL;
        default: return SPL_EINVAL;
    }
}

int spl_nn_forward(int n_players, int B, const int8_t *leaf_state, const uint64_t *leaf_mask,
                   const float *packed_weights, float *pi, float *v, void *hs) {
    if (n_players < 2 || n_players > 4 || B < 0 || (B && (!leaf_state || !leaf_mask || !packed_weights || !pi || !v)))
        return SPL_EINVAL;
    if (!B) return 0;
    const dim3 grid((unsigned)((B + ML - 1) / ML));
    switch (n_players) {
        case 2: hipLaunchKernelGGL(k_nn_forward<2>, grid, dim3(NNT), 0, (hipStream_t)hs, B, leaf_state, leaf_mask,
                                   packed_weights, pi, v); break;
        case 3: hipLaunchKernelGGL(k_nn_forward<3>, grid, dim3(NNT), 0, (hipStream_t)hs, B, leaf_state, leaf_mask,
                                   packed_weights, pi, v); break;
        default: hipLaunchKernelGGL(k_nn_forward<4>, grid, dim3(NNT), 0, (hipStream_t)hs, B, leaf_state, leaf_mask,
                                    packed_weights, pi, v); break;
    }
    return check_launch();
}

}  // extern "C"
