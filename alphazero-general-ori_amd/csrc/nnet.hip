// nnet.hip — SplendorNNet inference (SplendorNNet.py:56-159, eval mode) as one fused
// gfx950 kernel: int8 leaf boards + packed legality masks in, masked softmax policy and
// tanh values out (GenericNNetWrapper.predict, :141-168). C ABI: include/splendor_amd.h.
//
// One 512-thread workgroup (8 waves, two per SIMD so one wave's LDS / L2 latency hides
// behind the other's MFMAs) evaluates ML = 32 leaves through all 13 dense layers with every
// activation on chip:
//   * GEMMs on f32 MFMA (exact f32 products, f32 accumulation: the reference network's
//     precision). Per-column layers: v_mfma_f32_32x32x2_f32, wave w owns output columns
//     [32(w&3), 32(w&3)+32) for half of the token tiles (w>>2). Per-leaf layers:
//     v_mfma_f32_16x16x4_f32, wave w owns 16-column tile w for both 16-leaf row tiles.
//   * The per-board-column layers (dense2d_1, dense2d_3, partialgpool_1) treat the 7 board
//     columns of the 32 leaves as 7 token tiles of 32 (channel-major), so the per-column
//     BatchNorm affine is uniform across an MFMA tile.
//   * K is split across the MFMA's lane groups (32x32x2: lane half h feeds k = s + h*S;
//     16x16x4: lane quarter g feeds k = s + g*S), so a lane's A operand for 4 steps is one
//     ds_read_b128 and its B operand one coalesced global float4 from the pre-packed
//     weights (pack order in splendor_amd.h, spl_nn_forward).
//   * Activations live in LDS with a 132-float row stride (= 4 mod 64 dwords: the 16 lanes
//     of a ds_read_b128 group hit distinct 16-byte bank slots).
#include <hip/hip_runtime.h>

#include "../../include/splendor_amd.h"

#ifndef NN_TIMING
#define NN_TIMING 0        // diagnostic builds only (tools/time_nn.hip): per-layer cycle probes
#endif
#if NN_TIMING
__shared__ uint64_t nn_probe_acc[16];
__shared__ uint64_t nn_probe_last;
__device__ unsigned long long g_nn_timing[16];
#define NN_PROBE(k)                                                                        \
    if (threadIdx.x == 0) {                                                                \
        const uint64_t c_ = clock64();                                                     \
        nn_probe_acc[k] += c_ - nn_probe_last;                                             \
        nn_probe_last = c_;                                                                \
    }
#else
#define NN_PROBE(k)
#endif

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NNT = 512;       // threads per workgroup (8 waves)
constexpr int ML = 32;         // leaves per workgroup
constexpr int XS = 132;        // activation row stride (floats)
constexpr int LS = 420;        // logits row stride (floats)
constexpr int ACT = 409;

__host__ __device__ constexpr int kpad(int K) { return (K + 7) / 8 * 8; }
__host__ __device__ constexpr int ntiles(int N) { return (N + 31) / 32; }
__host__ __device__ constexpr int ntiles16(int N) { return (N + 15) / 16; }
// packed floats of a layer: the 4 per-column layers use 32x32x2 B fragments (32-column
// tiles, K in 2 halves), the 9 per-leaf layers 16x16x4 B fragments (16-column tiles, K in
// 4 quarters); see splendor_amd.h spl_nn_forward
__host__ __device__ constexpr bool f16(int l) { return l >= 4; }
__host__ __device__ constexpr int colpad(int l, int N) { return f16(l) ? ntiles16(N) * 16 : ntiles(N) * 32; }
__host__ __device__ constexpr int wfloats(int l, int N, int K) { return colpad(l, N) * kpad(K); }

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
        for (int j = 0; j < l; j++) o += wfloats(j, Ns[j], Ks[j]) + colpad(j, Ns[j]);
        return o;
    }
    static constexpr int boff(int l) { return woff(l) + wfloats(l, Ns[l], Ks[l]); }
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma4_16(const float4 &a, const float4 &b, f32x4 &acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
}

// per-leaf GEMM on v_mfma_f32_16x16x4_f32: the 32 leaves as 2 row tiles of 16 x up to NC
// 16-column tiles {c0, c0 + cstep, ...} < ctot, K = 16 * Q4 (lane group g = lane >> 4 feeds
// k = g * 4 Q4 + s at step s). afetch(rt, col) -> float4 of A[row tile rt][lane row][col..+3].
template <int NC, int Q4, class AF>
__device__ __forceinline__ void gemm16(const float *__restrict__ wp, int c0, int cstep, int ctot, AF afetch,
                                       f32x4 acc[NC][2]) {
    // a k-step is only 8 NC MFMAs (~256 NC cycles), shorter than an L2 round trip: the
    // weight fragments are prefetched PF steps ahead, the activations one step ahead
    constexpr int PF = 4;
    const int lane = threadIdx.x & 63, g = lane >> 4;
#pragma unroll
    for (int j = 0; j < NC; j++)
#pragma unroll
        for (int r = 0; r < 2; r++) acc[j][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float4 *w4 = reinterpret_cast<const float4 *>(wp) + lane;
    float4 bq[PF][NC];
#pragma unroll
    for (int p = 0; p < PF; p++)
#pragma unroll
        for (int j = 0; j < NC; j++) {
            const int ct = c0 + j * cstep;
            bq[p][j] = ct < ctot && p < Q4 ? w4[((size_t)ct * Q4 + p) * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    float4 a0 = afetch(0, g * 4 * Q4), a1 = afetch(1, g * 4 * Q4);
    for (int q0 = 0; q0 < Q4; q0 += PF) {
#pragma unroll
        for (int p = 0; p < PF; p++) {
            const int q = q0 + p;
            if (q < Q4) {
                const float4 x0 = a0, x1 = a1;
                if (q + 1 < Q4) {
                    a0 = afetch(0, g * 4 * Q4 + 4 * (q + 1));
                    a1 = afetch(1, g * 4 * Q4 + 4 * (q + 1));
                }
#pragma unroll
                for (int j = 0; j < NC; j++) {
                    const int ct = c0 + j * cstep;
                    if (ct < ctot) {
                        const float4 b = bq[p][j];
                        if (q + PF < Q4) bq[p][j] = w4[((size_t)ct * Q4 + q + PF) * 64];
                        mfma4_16(x0, b, acc[j][0]);
                        mfma4_16(x1, b, acc[j][1]);
                    }
                }
            }
        }
    }
}
// 16x16 accumulator element r of this lane: row (within the row tile) and column
__device__ __forceinline__ int acc16_row(int r) { return ((threadIdx.x & 63) >> 4) * 4 + r; }
__device__ __forceinline__ int acc16_col() { return threadIdx.x & 15; }

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
#if NN_TIMING
    if (tid < 16) nn_probe_acc[tid] = 0;
    if (tid == 0) nn_probe_last = clock64();
#endif
    const int b0 = blockIdx.x * ML, nb = min(ML, B - b0);
    const float *aff = W + Nt::AFF;                        // s1, t1, sp1, tp1
    const int t0 = 4 * wg, ntok = wg ? 3 : 4;              // this wave's token tiles (per-column layers)

    // ---- input: x[column c][leaf i][row r] = state[leaf][r][c] as int8 (token c*32+i)
    int8_t *x0 = reinterpret_cast<int8_t *>(bufA);
    for (int j = tid; j < 7 * ML * X0S / 4; j += NNT) reinterpret_cast<int32_t *>(x0)[j] = 0;
    __syncthreads();
    for (int j = tid; j < nb * R; j += NNT) {              // one board row (7 bytes) per thread
        const int i = j / R, r = j - i * R;
        const int8_t *src = state + ((size_t)(b0 + i) * R + r) * 7;
#pragma unroll
        for (int c = 0; c < 7; c++) x0[(c * ML + i) * X0S + r] = src[c];
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
    NN_PROBE(0)
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
    NN_PROBE(1)
    // ---- dense2d_1[3]: relu(W2 x + b2)
    {
        gemm_tiles<4, 64>(W + Nt::woff(1), wc, t0, ntok, fetchA(0), acc);
        __syncthreads();
        const float bias = W[Nt::boff(1) + col];
        store_tiles(col, [&](float x, int) { return fmaxf(x + bias, 0.f); });
        __syncthreads();
    }
    NN_PROBE(2)
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
    NN_PROBE(3)
    // ---- dense2d_3: relu(W3 x + b3)
    {
        gemm_tiles<4, 64>(W + Nt::woff(3), wc, t0, ntok, fetchA(0), acc);
        __syncthreads();
        const float bias = W[Nt::boff(3) + col];
        store_tiles(col, [&](float x, int) { return fmaxf(x + bias, 0.f); });
        __syncthreads();
    }
    NN_PROBE(4)
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
    // ---- per-leaf layers on 16x16x4 tiles: wave w owns 16-column tile w (both 16-leaf row
    // tiles) of a 128-wide layer; dst[row][dst_off + col] = f(acc, col) for col < nmax
    f32x4 a16[4][2];
    auto store16 = [&](int j, int ct, float *dst, int stride, int dst_off, int nmax, auto f) {
        const int col = 16 * ct + acc16_col();
        if (col < nmax) {
#pragma unroll
            for (int rt = 0; rt < 2; rt++)
#pragma unroll
                for (int r = 0; r < 4; r++) dst[(16 * rt + acc16_row(r)) * stride + dst_off + col] = f(a16[j][rt][r], col);
        }
    };
    auto leaf_fetch = [&](const float *src, int col0) {
        return [=](int rt, int c) { return ld4(src + (16 * rt + (lane & 15)) * XS + col0 + c); };
    };
    NN_PROBE(5)
    // ---- dense1d_4 over the 704 flattened features: [pool 128][x[5][:64]][x[6][:64]][x[c][64:128], c<7]
    {
        gemm16<1, 44>(W + Nt::woff(4), w, 8, 8, [&](int rt, int k) {
            const int i = 16 * rt + (lane & 15);
            if (k < 128) return ld4(bufP + i * XS + k);
            if (k < 256) return ld4(bufA + ((5 + ((k - 128) >> 6)) * ML + i) * XS + ((k - 128) & 63));
            return ld4(bufA + (((k - 256) >> 6) * ML + i) * XS + 64 + ((k - 256) & 63));
        }, a16);
        const float *bias = W + Nt::boff(4);
        store16(0, w, bufQ, XS, 0, 128, [&](float x, int c) { return fmaxf(x + bias[c], 0.f); });
        __syncthreads();
    }
    // partial pool over 4 groups of 4 of x[0:16] ++ relu(Wp x[16:] + bp) (BN folded): src -> dst
    auto pool44 = [&](const float *src, float *dst, int layer) {
        float pv = 0.f;
        if (tid < ML * 8) {
            const int i = tid >> 3, j = tid & 7, g = j & 3;
            const float *p = src + i * XS + 4 * g;
            pv = j < 4 ? fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3])) : (p[0] + p[1] + p[2] + p[3]) / 4.f;
        }
        gemm16<1, 7>(W + Nt::woff(layer), w, 8, 8, leaf_fetch(src, 16), a16);
        const float *bias = W + Nt::boff(layer);
        if (tid < ML * 8) dst[(tid >> 3) * XS + (tid & 7)] = pv;
        store16(0, w, dst, XS, 8, 120, [&](float x, int c) { return fmaxf(x + bias[c], 0.f); });
        __syncthreads();
    };
    auto dense128 = [&](const float *src, float *dst, int layer) {
        gemm16<1, 8>(W + Nt::woff(layer), w, 8, 8, leaf_fetch(src, 0), a16);
        const float *bias = W + Nt::boff(layer);
        store16(0, w, dst, XS, 0, 128, [&](float x, int c) { return fmaxf(x + bias[c], 0.f); });
        __syncthreads();
    };
    NN_PROBE(6)
    pool44(bufQ, bufP, 5);                  // partialgpool_4
    dense128(bufP, bufQ, 6);                // dense1d_5[0] (+BN folded)
    dense128(bufQ, bufP, 7);                // dense1d_5[3]
    pool44(bufP, bufQ, 8);                  // partialgpool_5 -> trunk output in bufQ
    NN_PROBE(7)
    // ---- heads: PI[0] -> bufP, V[0] -> bufA (no activation); wave w: column tile w of both
    {
        gemm16<1, 8>(W + Nt::woff(9), w, 8, 8, leaf_fetch(bufQ, 0), a16);
        gemm16<1, 8>(W + Nt::woff(11), w, 8, 8, leaf_fetch(bufQ, 0), a16 + 1);
        const float *bp = W + Nt::boff(9), *bv = W + Nt::boff(11);
        store16(0, w, bufP, XS, 0, 128, [&](float x, int c) { return x + bp[c]; });
        store16(1, w, bufA, XS, 0, 128, [&](float x, int c) { return x + bv[c]; });
        __syncthreads();
    }
    NN_PROBE(8)
    float *logits = bufA + ML * XS;
    // ---- PI[1] (409 outputs, 26 column tiles over 8 waves) and V[1] (NP outputs, wave 7)
    {
        constexpr int CT = ntiles16(ACT);
        gemm16<4, 8>(W + Nt::woff(10), w, 8, CT, leaf_fetch(bufP, 0), a16);
        const float *bp = W + Nt::boff(10);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (w + 8 * j < CT) store16(j, w + 8 * j, logits, LS, 0, 16 * CT, [&](float x, int c) { return x + bp[c]; });
        if (w == 7) {
            gemm16<1, 8>(W + Nt::woff(12), 0, 1, 1, leaf_fetch(bufA, 0), a16);
            const int n = acc16_col();
            if (n < NP) {
                const float bias = W[Nt::boff(12) + n];
#pragma unroll
                for (int rt = 0; rt < 2; rt++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int i = 16 * rt + acc16_row(r);
                        if (i < nb) v_out[(size_t)(b0 + i) * NP + n] = tanhf(a16[0][rt][r] + bias);
                    }
            }
        }
        __syncthreads();
    }
    NN_PROBE(9)
    // ---- masked softmax (invalid -> -1e8, as the reference's masked_fill + log_softmax);
    // the wave's leaves are processed together so their reductions overlap
    {
        constexpr int PERW = ML / (NNT / 64);
        float x[PERW][7], m[PERW], sum[PERW];
#pragma unroll
        for (int q = 0; q < PERW; q++) {
            const int i = w * PERW + q;
            const uint64_t *mk = mask + (size_t)(b0 + min(i, nb - 1)) * 7;
            m[q] = -3.0e38f;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                const int a = 64 * k + lane;
                const bool ok = a < ACT && ((mk[k] >> lane) & 1);
                x[q][k] = a < ACT ? (ok ? logits[i * LS + a] : -1e8f) : -3.0e38f;
                m[q] = fmaxf(m[q], x[q][k]);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int q = 0; q < PERW; q++) m[q] = fmaxf(m[q], __shfl_xor(m[q], o, 64));
#pragma unroll
        for (int q = 0; q < PERW; q++) {
            sum[q] = 0.f;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                x[q][k] = 64 * k + lane < ACT ? __expf(x[q][k] - m[q]) : 0.f;
                sum[q] += x[q][k];
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int q = 0; q < PERW; q++) sum[q] += __shfl_xor(sum[q], o, 64);
#pragma unroll
        for (int q = 0; q < PERW; q++) {
            const int i = w * PERW + q;
            if (i < nb) {
                const float inv = 1.f / sum[q];
#pragma unroll
                for (int k = 0; k < 7; k++) {
                    const int a = 64 * k + lane;
                    if (a < ACT) pi_out[(size_t)(b0 + i) * ACT + a] = x[q][k] * inv;
                }
            }
        }
    }
#if NN_TIMING
    NN_PROBE(10)
    if (tid == 0)
        for (int k = 0; k < 16; k++) atomicAdd(&g_nn_timing[k], (unsigned long long)nn_probe_acc[k]);
#endif
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
