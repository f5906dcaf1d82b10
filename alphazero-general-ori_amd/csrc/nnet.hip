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

#ifndef NN_PF1
#define NN_PF1 4               // weight-prefetch depth (k steps) of the per-leaf GEMMs
#endif
constexpr int NNT = 512;      // threads per workgroup (8 waves)
constexpr int ML = 32;         // leaves per workgroup
constexpr int XS = 132;        // activation row stride (floats)
constexpr int LS = 420;        // logits row stride (floats)
// per-leaf operands are read by ds_read_b128 with lane l on row l & 15 and k group l >> 4
// 4 floats apart: with rows 8 banks apart, the groups {0-3,12-15,20-27}, ... that share an
// LDS cycle land on disjoint banks (MI355X_MICROARCH.md §LDS)
constexpr int PS = 136;        // per-leaf activation row stride (floats)
constexpr int ZS = 712;        // flattened trunk row stride (704 features)
static_assert(ML * ZS <= 7 * ML * XS && ML * (PS + LS) <= 7 * ML * XS, "bufA overlays");
static_assert(2 * 64 * ML <= ML * PS, "dense2d_3 pool partials fit bufP");
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
// the split copy of a per-column layer: [4][Kp16/16][3][64][8] bf16 (hi, mid, lo parts of
// W[32 nt + l % 32][16 c + 8 (l / 32) + j]), as floats
__host__ __device__ constexpr int kp16(int K) { return (K + 15) / 16 * 16; }
__host__ __device__ constexpr int sfloats(int K) { return 4 * (kp16(K) / 16) * 3 * 64 * 8 / 2; }

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
    // bf16 x 3 copies of the 4 per-column layers (NN_SPLIT), 16-byte aligned after the affines
    static constexpr int SBASE = (AFF + 28 + 3) / 4 * 4;
    static constexpr int soff(int l) {
        int o = SBASE;
        for (int j = 0; j < l; j++) o += sfloats(Ks[j]);
        return o;
    }
    static constexpr int TOTAL = soff(4);
    static constexpr int X0S = (kpad(R) / 4) % 2 ? kpad(R) : kpad(R) + 4;   // int8 input stride (odd dwords)
};

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; i++) z[i] = 0.f;
    return z;
}

[[maybe_unused]] __device__ __forceinline__ void mfma4(const float4 &a, const float4 &b, f32x16 &acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
}

template <int V> struct IntC {
    static constexpr int value = V;
};

// weight-fragment ring of the per-column GEMMs (a k-step is 4 T MFMAs of 64 cycles)
constexpr int PFC = 2;
typedef float4 RingC[PFC];

// first PFC k-steps of column block nt of a per-column layer (K = 2S) into the ring
template <int S>
__device__ __forceinline__ void ringc_load(const float *__restrict__ wp, int nt, RingC &bq) {
    const float4 *w4 = reinterpret_cast<const float4 *>(wp) + (size_t)nt * (S / 4) * 64 + (threadIdx.x & 63);
#pragma unroll
    for (int p = 0; p < PFC; p++) bq[p] = w4[(p < S / 4 ? p : S / 4 - 1) * 64];
}

// token tiles t0 .. t0+T-1 x one N tile (column block nt) over K = 2S; bq holds the first
// PFC steps (ringc_load); afetch(t, col) -> float4 of A[token tile t][lane row][col..col+3];
// next() runs after the last MFMA is issued. Unrolled and branch-free like gemm16.
template <int T, int S, class AF, class NX>
__device__ __forceinline__ void gemm_tiles(const float *__restrict__ wp, int nt, int t0, RingC &bq, AF afetch,
                                           f32x16 *acc, NX next) {
    constexpr int Q = S / 4;
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const float4 *w4 = reinterpret_cast<const float4 *>(wp) + (size_t)nt * Q * 64 + lane;
#pragma unroll
    for (int t = 0; t < T; t++) acc[t] = zero16();
    float4 a[T];
#pragma unroll
    for (int t = 0; t < T; t++) a[t] = afetch(t0 + t, h * S);
#pragma unroll
    for (int q = 0; q < Q; q++) {
        float4 x[T];
#pragma unroll
        for (int t = 0; t < T; t++) x[t] = a[t];
        if (q + 1 < Q)
#pragma unroll
            for (int t = 0; t < T; t++) a[t] = afetch(t0 + t, h * S + 4 * (q + 1));
        const float4 b = bq[q % PFC];
        if (q + PFC < Q) bq[q % PFC] = w4[(q + PFC) * 64];
#pragma unroll
        for (int t = 0; t < T; t++) mfma4(x[t], b, acc[t]);
        __builtin_amdgcn_sched_barrier(0);
    }
    next();
    __builtin_amdgcn_sched_barrier(0);
}


#ifndef NN_SPLIT
#define NN_SPLIT 1      // per-column layers on bf16 MFMAs with operands split in three parts (0: f32 MFMA)
#endif
// Split per-column GEMMs (NN_SPLIT): an f32 x is exactly hi + mid + lo, three bf16 parts
// taken by truncation (hi: the top 8 significant bits, mid: the top 8 of the residual, lo: the
// rest, at most 8 significant bits), and x y = Σ over the parts' products minus the three
// smallest (mid lo, lo mid, lo lo: < 2^-22 |x y| together, ~2^-24 typically). v_mfma_f32_32x32x16_bf16 takes 16 k per instruction at 16 times the f32
// MFMA's rate, so the six products of a 16-k chunk cost 6 x 32 cycles against 8 x 64 for
// v_mfma_f32_32x32x2_f32. Each bf16 product is exact in f32; hi hi goes into the layer's
// accumulator and the five smaller products into a second one (added in the epilogue), so
// the large accumulator rounds once per MFMA (16 k) instead of once per k, and the small one's
// roundings are ~2^-8 smaller: measured against float64 the split layer's error is below the
// f32 MFMA's (tools/nn_split_probe.hip). The int8 boards of dense2d_1 are exact
// in bf16: three products (the weight's parts) into one accumulator.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#ifndef NN_PFS
#define NN_PFS 2
#endif
constexpr int PFS = NN_PFS;            // chunks of weight parts in flight
struct RingS {
    bf16x8 b[PFS][3];
};
struct F8 {
    float4 lo, hi;                     // 8 consecutive k of one lane's A row
};

[[maybe_unused]] __device__ __forceinline__ void split8(const F8 &x, bf16x8 &hi, bf16x8 &mid, bf16x8 &lo) {
    const float xs[8] = {x.lo.x, x.lo.y, x.lo.z, x.lo.w, x.hi.x, x.hi.y, x.hi.z, x.hi.w};
    uint32_t h[8], m[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        h[j] = __float_as_uint(xs[j]) & 0xFFFF0000u;
        const float r1 = xs[j] - __uint_as_float(h[j]);
        m[j] = __float_as_uint(r1) & 0xFFFF0000u;
        l[j] = __float_as_uint(r1 - __uint_as_float(m[j]));
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
// 8 int8 (two dwords) -> 8 bf16, exact
[[maybe_unused]] __device__ __forceinline__ bf16x8 i8_to_bf16x8(int v0, int v1) {
    u32x4 r;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const int v = p < 2 ? v0 : v1, sh = 16 * (p & 1);
        const uint32_t e0 = __float_as_uint((float)(int8_t)(v >> sh)) >> 16;
        const uint32_t e1 = __float_as_uint((float)(int8_t)(v >> (sh + 8))) & 0xFFFF0000u;
        r[p] = e0 | e1;
    }
    return __builtin_bit_cast(bf16x8, r);
}

// first PFS chunks of column block nt of a split layer (C chunks of 16 k) into the ring
template <int C>
__device__ __forceinline__ void rings_load(const float *__restrict__ ws, int nt, RingS &r) {
    const bf16x8 *w = reinterpret_cast<const bf16x8 *>(ws) + (size_t)nt * C * 3 * 64 + (threadIdx.x & 63);
#pragma unroll
    for (int p = 0; p < PFS; p++)
#pragma unroll
        for (int q = 0; q < 3; q++) r.b[p][q] = w[((p < C ? p : C - 1) * 3 + q) * 64];
}

// gemm_tiles on split operands: token tiles t0 .. t0+T-1 x column block nt over C chunks of
// 16 k. INT8: afetch(t, k) -> bf16x8 (exact A, three products); else afetch(t, k) -> F8
// (A split here, six products). Lane l: A[row l % 32][k = 16 c + 8 (l / 32) + j].
template <int T, int C, bool INT8, class AF, class NX>
__device__ __forceinline__ void gemm_split(const float *__restrict__ ws, int nt, int t0, RingS &r, AF afetch,
                                           f32x16 *acc, NX next) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const bf16x8 *w = reinterpret_cast<const bf16x8 *>(ws) + (size_t)nt * C * 3 * 64 + lane;
    f32x16 acl[T];                                       // the five smaller products
#pragma unroll
    for (int t = 0; t < T; t++) { acc[t] = zero16(); acl[t] = zero16(); }
#pragma unroll
    for (int c = 0; c < C; c++) {
        const bf16x8 b0 = r.b[c % PFS][0], b1 = r.b[c % PFS][1], b2 = r.b[c % PFS][2];
        if (c + PFS < C)
#pragma unroll
            for (int q = 0; q < 3; q++) r.b[c % PFS][q] = w[((c + PFS) * 3 + q) * 64];
        if constexpr (INT8) {
            bf16x8 a[T];
#pragma unroll
            for (int t = 0; t < T; t++) a[t] = afetch(t0 + t, 16 * c + 8 * h);
#pragma unroll
            for (int t = 0; t < T; t++) {
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t], b2, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t], b1, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t], b0, acc[t], 0, 0, 0);
            }
        } else {
            F8 x[T];
#pragma unroll
            for (int t = 0; t < T; t++) x[t] = afetch(t0 + t, 16 * c + 8 * h);
#pragma unroll
            for (int t = 0; t < T; t++) {
                bf16x8 a0, a1, a2;
                split8(x[t], a0, a1, a2);
                acl[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acl[t], 0, 0, 0);
                acl[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acl[t], 0, 0, 0);
                acl[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acl[t], 0, 0, 0);
                acl[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acl[t], 0, 0, 0);
                acl[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acl[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[t], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    next();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!INT8)
#pragma unroll
        for (int t = 0; t < T; t++) acc[t] += acl[t];
}


typedef float f32x4 __attribute__((ext_vector_type(4)));

// both row tiles against one B fragment, alternating accumulators: a 16x16x4 f32 MFMA
// issues every 32 cycles but its result is ready for a dependent one only after 40
// (MI355X_MICROARCH.md, cycle constants)
__device__ __forceinline__ void mfma4_16x2(const float4 &a0, const float4 &a1, const float4 &b, f32x4 &c0,
                                          f32x4 &c1) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b.x, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b.x, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b.y, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b.y, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b.z, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b.z, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b.w, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b.w, c1, 0, 0, 0);
}

// workgroup barrier for LDS traffic only: waits for this wave's LDS operations, not for its
// global loads, so weight fragments prefetched for the next layer stay in flight across it
// (__syncthreads() waits vmcnt(0) first); the memory clobber keeps the compiler from moving
// LDS accesses across it
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// weight-fragment ring of the per-leaf GEMMs: PF16 k-steps x up to 4 column tiles
constexpr int PF16 = NN_PF1;
typedef float4 Ring16[PF16][4];

// column tile j of a per-leaf layer: tile min(c0 + j cstep, ctot - 1) (a clamped tile is
// loaded but never multiplied)
template <int Q4>
__device__ __forceinline__ const float4 *tile16(const float *__restrict__ wp, int c0, int cstep, int ctot, int j) {
    return reinterpret_cast<const float4 *>(wp) + (size_t)min(c0 + j * cstep, ctot - 1) * Q4 * 64 + (threadIdx.x & 63);
}

// issue the first PF16 k-steps of a per-leaf layer's weight fragments into the ring; a
// caller does this right after the previous layer's last MFMA, ahead of its epilogue and
// barrier, so no layer starts on an L2 round trip
template <int NC, int Q4>
__device__ __forceinline__ void ring_load(const float *__restrict__ wp, int c0, int cstep, int ctot, Ring16 &bq) {
#pragma unroll
    for (int j = 0; j < NC; j++) {
        const float4 *w4 = tile16<Q4>(wp, c0, cstep, ctot, j);
#pragma unroll
        for (int p = 0; p < PF16; p++) bq[p][j] = w4[(p < Q4 ? p : Q4 - 1) * 64];
    }
}

// per-leaf GEMM on v_mfma_f32_16x16x4_f32: the 32 leaves as 2 row tiles of 16 x NC
// 16-column tiles {c0, c0 + cstep, ...} (all valid: the caller picks NC for its wave),
// K = 16 * Q4 (lane group g = lane >> 4 feeds k = 16 q + 4 g + j at step q, MFMA j).
// bq holds the first PF16 steps (ring_load); afetch(rt, col) -> float4 of
// A[row tile rt][lane row][col..+3]; next() runs after the last MFMA is issued.
// The k loop is fully unrolled with no branch in it: a conditional weight load makes the
// compiler copy the loaded fragment into the ring register under an s_waitcnt vmcnt(0)
// at once, and every step then pays the whole L2 round trip.
template <int NC, int Q4, class AF, class NX>
__device__ __forceinline__ void gemm16(const float *__restrict__ wp, int c0, int cstep, Ring16 &bq, AF afetch,
                                       f32x4 (*acc)[2], NX next) {
    // a k-step is only 8 NC MFMAs (~256 NC cycles), shorter than an L2 round trip: the
    // weight fragments are prefetched PF16 steps ahead, the activations one step ahead
    constexpr int PF = PF16;
    const int lane = threadIdx.x & 63, g = lane >> 4;
#pragma unroll
    for (int j = 0; j < NC; j++)
#pragma unroll
        for (int r = 0; r < 2; r++) acc[j][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float4 *w4[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) w4[j] = tile16<Q4>(wp, c0, cstep, 1 << 30, j);
    float4 a0 = afetch(0, 4 * g), a1 = afetch(1, 4 * g);
#pragma unroll
    for (int q = 0; q < Q4; q++) {
        const float4 x0 = a0, x1 = a1;
        if (q + 1 < Q4) {
            a0 = afetch(0, 4 * g + 16 * (q + 1));
            a1 = afetch(1, 4 * g + 16 * (q + 1));
        }
#pragma unroll
        for (int j = 0; j < NC; j++) {
            const float4 b = bq[q % PF][j];
            if (q + PF < Q4) bq[q % PF][j] = w4[j][(q + PF) * 64];
            mfma4_16x2(x0, x1, b, acc[j][0], acc[j][1]);
        }
        // keep each step's loads in its step: left alone, the scheduler sinks them next to
        // their MFMAs PF steps later (vmcnt(1) waits, the ring gone)
        __builtin_amdgcn_sched_barrier(0);
    }
    next();
    __builtin_amdgcn_sched_barrier(0);
}
struct NoNext {
    __device__ void operator()() const {}
};
// 16x16 accumulator element r of this lane: row (within the row tile) and column
__device__ __forceinline__ int acc16_row(int r) { return ((threadIdx.x & 63) >> 4) * 4 + r; }
__device__ __forceinline__ int acc16_col() { return threadIdx.x & 15; }

// accumulator element r of this lane: (row, col) of the 32x32 tile (C/D map of gfx950)
__device__ __forceinline__ int acc_row(int r) { return (r & 3) + 8 * (r >> 2) + 4 * ((threadIdx.x & 63) >> 5); }
__device__ __forceinline__ int acc_col() { return threadIdx.x & 31; }

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// wave reductions for the softmax: butterfly inside each 16-lane row on DPP (quad_perm
// [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the four row results by readlane
// (uniform result, no LDS round trips)
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float rows_f32(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16 * k));
}
__device__ __forceinline__ float wave_max_f32(float v) {
    v = fmaxf(v, dpp_f32<0xB1>(v));
    v = fmaxf(v, dpp_f32<0x4E>(v));
    v = fmaxf(v, dpp_f32<0x141>(v));
    v = fmaxf(v, dpp_f32<0x140>(v));
    return fmaxf(fmaxf(rows_f32(v, 0), rows_f32(v, 1)), fmaxf(rows_f32(v, 2), rows_f32(v, 3)));
}
__device__ __forceinline__ float wave_sum_f32(float v) {
    v += dpp_f32<0xB1>(v);
    v += dpp_f32<0x4E>(v);
    v += dpp_f32<0x141>(v);
    v += dpp_f32<0x140>(v);
    return (rows_f32(v, 0) + rows_f32(v, 1)) + (rows_f32(v, 2) + rows_f32(v, 3));
}

template <int NP>
// one workgroup per CU (LDS) = 2 waves per SIMD: the register budget is 256, and without
// saying so the scheduler sinks the prefetched weight loads next to their MFMAs
// idx (optional): the kernel evaluates rows idx[0 .. *count) — board / mask / output row
// idx[k] — instead of 0 .. B (the search's NN leaves, compacted by k_leaf_mask); tiles past
// *count exit at once.
__global__ __launch_bounds__(NNT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_nn_forward(int B, const int8_t *__restrict__ state,
                                                    const uint64_t *__restrict__ mask,
                                                    const float *__restrict__ W, float *__restrict__ pi_out,
                                                    float *__restrict__ v_out,
                                                    const int32_t *__restrict__ idx,
                                                    const int32_t *__restrict__ count) {
    using Nt = Net<NP>;
    constexpr int R = Nt::R, X0S = Nt::X0S;
    __shared__ __align__(16) float bufA[7 * ML * XS];      // per-column activations / logits
    __shared__ __align__(16) float bufP[ML * PS];          // per-leaf ping
    __shared__ __align__(16) float bufQ[ML * PS];          // per-leaf pong
    __shared__ uint64_t mskl[ML * 7];                      // legality masks (read at the softmax)
    // wave index in an SGPR: every per-wave choice below is a scalar branch
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, li = lane & 31;
    const int wc = w & 3, wg = w >> 2;                     // column block, wave group
#if NN_TIMING
    if (tid < 16) nn_probe_acc[tid] = 0;
    if (tid == 0) nn_probe_last = clock64();
#endif
    const int b0 = blockIdx.x * ML;
    const int cnt = count ? __builtin_amdgcn_readfirstlane(*count) : B;
    if (b0 >= cnt) return;
    const int nb = min(ML, cnt - b0);
    // row of leaf i of this tile (its board, mask and outputs)
    const auto rowof = [&](int i) -> size_t { return idx ? (size_t)idx[b0 + i] : (size_t)(b0 + i); };
    const float *aff = W + Nt::AFF;                        // s1, t1, sp1, tp1
    const int t0 = 4 * wg, ntok = wg ? 3 : 4;              // this wave's token tiles (per-column layers)
#if NN_SPLIT
    constexpr int C1 = kp16(R) / 16;
    RingS rings;                                           // per-column weight parts, one layer ahead
    rings_load<C1>(W + Nt::soff(0), wc, rings);
#else
    constexpr int S1 = kpad(R) / 2;
    RingC ringc;                                           // per-column weight fragments, one layer ahead
    ringc_load<S1>(W + Nt::woff(0), wc, ringc);
#endif

    // ---- input: x[column c][leaf i][row r] = state[leaf][r][c] as int8 (token c*32+i)
    int8_t *x0 = reinterpret_cast<int8_t *>(bufA);
    for (int j = tid; j < 7 * ML * X0S / 4; j += NNT) reinterpret_cast<int32_t *>(x0)[j] = 0;
    lds_barrier();
    if (tid < nb * 7) mskl[tid] = mask[rowof(tid / 7) * 7 + tid % 7];
    if constexpr ((7 * R) % 4 == 0) {
        // the workgroup's boards: dword loads (a board is a whole number of dwords), all in
        // flight at once, then each byte scattered to its (column, leaf, row) slot
        constexpr int BW = R * 7 / 4;                      // dwords per board
        constexpr int PER = (ML * BW + NNT - 1) / NNT;
        int32_t d[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int j = tid + k * NNT, i = j / BW;
            d[k] = j < nb * BW ? reinterpret_cast<const int32_t *>(state + rowof(i) * R * 7)[j - i * BW] : 0;
        }
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int j = tid + k * NNT;
            if (j < nb * R * 7 / 4) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int o = 4 * j + q, i = o / (R * 7), rem = o - i * (R * 7), r = rem / 7, c = rem - 7 * r;
                    x0[(c * ML + i) * X0S + r] = (int8_t)(d[k] >> (8 * q));
                }
            }
        }
    } else {
        for (int j = tid; j < nb * R; j += NNT) {          // one board row (7 bytes) per thread
            const int i = j / R, r = j - i * R;
            const int8_t *src = state + (rowof(i) * R + r) * 7;
#pragma unroll
            for (int c = 0; c < 7; c++) x0[(c * ML + i) * X0S + r] = src[c];
        }
    }
    lds_barrier();

    f32x16 acc[4];
    const int col = 32 * wc + acc_col();
    // this wave's 4 (group 0) or 3 (group 1) token tiles of column block wc
#if NN_SPLIT
    // (s_const: chunks of 16 k; i8_const: A is the int8 input)
    auto gemm_cols = [&](auto c_const, auto i8_const, const float *ws, auto afetch, auto next) {
        constexpr int C = decltype(c_const)::value;
        constexpr bool I8 = decltype(i8_const)::value != 0;
        if (wg == 0)
            gemm_split<4, C, I8>(ws, wc, 0, rings, afetch, acc, next);
        else
            gemm_split<3, C, I8>(ws, wc, 4, rings, afetch, acc, next);
    };
    auto fetchA8 = [&](int col0) {
        return [&, col0](int t, int c) {
            const float *p = bufA + (t * ML + li) * XS + col0 + c;
            return F8{ld4(p), ld4(p + 4)};
        };
    };
#else
    auto gemm_col = [&](auto s_const, const float *wp, auto afetch, auto next) {
        constexpr int S = decltype(s_const)::value;
        if (wg == 0)
            gemm_tiles<4, S>(wp, wc, 0, ringc, afetch, acc, next);
        else
            gemm_tiles<3, S>(wp, wc, 4, ringc, afetch, acc, next);
    };
#endif
    // per-column epilogue over this wave's token tiles: dst = f(acc, t, n)
    auto store_tiles = [&](int coloff, auto f) {
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (t < ntok)
#pragma unroll
                for (int r = 0; r < 16; r++)
                    bufA[((t0 + t) * ML + acc_row(r)) * XS + coloff] = f(acc[t][r], t0 + t);
    };
#if !NN_SPLIT
    auto fetchA = [&](int col0) {
        return [&, col0](int t, int c) { return ld4(bufA + (t * ML + li) * XS + col0 + c); };
    };
#endif
    NN_PROBE(0)
    // ---- dense2d_1: relu(s1[c] * (W1 x + b1) + t1[c])
    // (each layer's bias is read before its GEMM, ahead of the next layer's ring: vmcnt
    // retires loads in order)
    {
        const float bias = W[Nt::boff(0) + col];
#if NN_SPLIT
        // (k past R reads zero padding or the next row's bytes: their weights are 0)
        gemm_cols(IntC<C1>(), IntC<1>(), W + Nt::soff(0), [&](int t, int c) {
            const int32_t *p = reinterpret_cast<const int32_t *>(x0 + (t * ML + li) * X0S + c);
            return i8_to_bf16x8(p[0], p[1]);
        }, [&] { rings_load<8>(W + Nt::soff(1), wc, rings); });
#else
        gemm_col(IntC<S1>(), W + Nt::woff(0), [&](int t, int c) {
            const int v = *reinterpret_cast<const int32_t *>(x0 + (t * ML + li) * X0S + c);
            return make_float4((float)(int8_t)v, (float)(int8_t)(v >> 8), (float)(int8_t)(v >> 16), (float)(v >> 24));
        }, [&] { ringc_load<64>(W + Nt::woff(1), wc, ringc); });
#endif
        lds_barrier();
        store_tiles(col, [&](float x, int t) { return fmaxf((x + bias) * aff[t] + aff[7 + t], 0.f); });
        lds_barrier();
    }
    NN_PROBE(1)
    // ---- dense2d_1[3]: relu(W2 x + b2)
    {
        const float bias = W[Nt::boff(1) + col];
#if NN_SPLIT
        gemm_cols(IntC<8>(), IntC<0>(), W + Nt::soff(1), fetchA8(0), [&] { rings_load<6>(W + Nt::soff(2), wc, rings); });
#else
        gemm_col(IntC<64>(), W + Nt::woff(1), fetchA(0), [&] { ringc_load<48>(W + Nt::woff(2), wc, ringc); });
#endif
        lds_barrier();
        store_tiles(col, [&](float x, int) { return fmaxf(x + bias, 0.f); });
        lds_barrier();
    }
    NN_PROBE(2)
    // ---- partialgpool_1: [max, mean over 4 groups of 8 of x[0:32]] ++ relu(BN(Wp1 x[32:] + bp1))
    {
        const float bias = W[Nt::boff(2) + col];  // 0-padded to 128 columns
#if NN_SPLIT
        gemm_cols(IntC<6>(), IntC<0>(), W + Nt::soff(2), fetchA8(32), [&] { rings_load<8>(W + Nt::soff(3), wc, rings); });
#else
        gemm_col(IntC<48>(), W + Nt::woff(2), fetchA(32), [&] { ringc_load<64>(W + Nt::woff(3), wc, ringc); });
#endif
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
        lds_barrier();
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int item = tid + NNT * q;
            if (item < 7 * ML * 8) bufA[(item >> 3) * XS + (item & 7)] = pv[q];
        }
        if (col < 120)
            store_tiles(8 + col, [&](float x, int t) { return fmaxf((x + bias) * aff[14 + t] + aff[21 + t], 0.f); });
        lds_barrier();
    }
    NN_PROBE(3)
    // ---- dense2d_3: relu(W3 x + b3), written straight into the flattened per-leaf image
    // Z[leaf][704] = [max_c<5 x[c][:64]][mean_c<5 x[c][:64]][x[5][:64]][x[6][:64]][x[c][64:], c<7]
    // (FlattenAndPartialGPool(64, 5)), so dense1d_4 reads plain rows
    float *Z = bufA;
    Ring16 ring;                           // per-leaf weight fragments, one layer ahead
    {
        const float bias = W[Nt::boff(3) + col];
#if NN_SPLIT
        gemm_cols(IntC<8>(), IntC<0>(), W + Nt::soff(3), fetchA8(0), [&] { ring_load<1, 44>(W + Nt::woff(4), w, 8, 8, ring); });
#else
        gemm_col(IntC<64>(), W + Nt::woff(3), fetchA(0), [&] { ring_load<1, 44>(W + Nt::woff(4), w, 8, 8, ring); });
#endif
        lds_barrier();
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[t][r] = fmaxf(acc[t][r] + bias, 0.f);
        if (col >= 64) {
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (t < ntok)
#pragma unroll
                    for (int r = 0; r < 16; r++) Z[acc_row(r) * ZS + 256 + 64 * (t0 + t) + col - 64] = acc[t][r];
        } else if (wg == 0) {              // channels 0-3: partial max / sum -> bufP
#pragma unroll
            for (int r = 0; r < 16; r++) {
                bufP[acc_row(r) * 128 + col] = fmaxf(fmaxf(acc[0][r], acc[1][r]), fmaxf(acc[2][r], acc[3][r]));
                bufP[acc_row(r) * 128 + 64 + col] = acc[0][r] + acc[1][r] + acc[2][r] + acc[3][r];
            }
        } else {                           // channels 5, 6 pass through
#pragma unroll
            for (int r = 0; r < 16; r++) {
                Z[acc_row(r) * ZS + 128 + col] = acc[1][r];
                Z[acc_row(r) * ZS + 192 + col] = acc[2][r];
            }
        }
        lds_barrier();
        if (col < 64 && wg == 1) {         // channel 4 closes the pool
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int i = acc_row(r);
                Z[i * ZS + col] = fmaxf(bufP[i * 128 + col], acc[0][r]);
                Z[i * ZS + 64 + col] = (bufP[i * 128 + 64 + col] + acc[0][r]) / 5.f;
            }
        }
        lds_barrier();
    }
    NN_PROBE(4)
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
    auto leaf_fetch = [&](const float *src, int col0, int stride = PS) {
        return [=](int rt, int c) { return ld4(src + (16 * rt + (lane & 15)) * stride + col0 + c); };
    };
    // bias of this lane's column in tile ct of a per-leaf layer (biases are 0-padded to whole
    // tiles). Read before the layer's GEMM: vmcnt retires loads in order, so a bias load
    // issued behind the next layer's ring prefetch would wait for the whole ring.
    auto bias16 = [&](int layer, int ct) { return W[Nt::boff(layer) + 16 * ct + acc16_col()]; };
    auto ring7 = [&](int layer) { return [&, layer] { ring_load<1, 7>(W + Nt::woff(layer), w, 8, 8, ring); }; };
    auto ring8 = [&](int layer) { return [&, layer] { ring_load<1, 8>(W + Nt::woff(layer), w, 8, 8, ring); }; };
    constexpr int CT = ntiles16(ACT);      // PI[1] column tiles
    static_assert(CT > 24 && CT <= 32, "PI[1] tiles: 3 or 4 per wave");
    NN_PROBE(5)
    // ---- dense1d_4 over the 704 flattened features Z
    {
        const float bl = bias16(4, w);
        gemm16<1, 44>(W + Nt::woff(4), w, 8, ring, leaf_fetch(Z, 0, ZS), a16, ring7(5));
        store16(0, w, bufQ, PS, 0, 128, [&](float x, int) { return fmaxf(x + bl, 0.f); });
        lds_barrier();
    }
    // partial pool over 4 groups of 4 of x[0:16] ++ relu(Wp x[16:] + bp) (BN folded): src -> dst
    auto pool44 = [&](const float *src, float *dst, int layer, auto next) {
        const float bl = bias16(layer, w);
        float pv = 0.f;
        if (tid < ML * 8) {
            const int i = tid >> 3, j = tid & 7, g = j & 3;
            const float *p = src + i * PS + 4 * g;
            pv = j < 4 ? fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3])) : (p[0] + p[1] + p[2] + p[3]) / 4.f;
        }
        gemm16<1, 7>(W + Nt::woff(layer), w, 8, ring, leaf_fetch(src, 16), a16, next);
        if (tid < ML * 8) dst[(tid >> 3) * PS + (tid & 7)] = pv;
        store16(0, w, dst, PS, 8, 120, [&](float x, int) { return fmaxf(x + bl, 0.f); });
        lds_barrier();
    };
    auto dense128 = [&](const float *src, float *dst, int layer, auto next) {
        const float bl = bias16(layer, w);
        gemm16<1, 8>(W + Nt::woff(layer), w, 8, ring, leaf_fetch(src, 0), a16, next);
        store16(0, w, dst, PS, 0, 128, [&](float x, int) { return fmaxf(x + bl, 0.f); });
        lds_barrier();
    };
    NN_PROBE(6)
    pool44(bufQ, bufP, 5, ring8(6));        // partialgpool_4
    dense128(bufP, bufQ, 6, ring8(7));      // dense1d_5[0] (+BN folded)
    dense128(bufQ, bufP, 7, ring7(8));      // dense1d_5[3]
    pool44(bufP, bufQ, 8, ring8(9));        // partialgpool_5 -> trunk output in bufQ
    NN_PROBE(7)
    // ---- heads: PI[0] -> bufP, V[0] -> bufA (no activation); wave w: column tile w of both
    {
        const float bp = bias16(9, w), bv = bias16(11, w);
        gemm16<1, 8>(W + Nt::woff(9), w, 8, ring, leaf_fetch(bufQ, 0), a16, ring8(11));
        gemm16<1, 8>(W + Nt::woff(11), w, 8, ring, leaf_fetch(bufQ, 0), a16 + 1,
                     [&] { ring_load<4, 8>(W + Nt::woff(10), w, 8, CT, ring); });
        store16(0, w, bufP, PS, 0, 128, [&](float x, int) { return x + bp; });
        store16(1, w, bufA, PS, 0, 128, [&](float x, int) { return x + bv; });
        lds_barrier();
    }
    NN_PROBE(8)
    float *logits = bufA + ML * PS;
    // ---- PI[1] (409 outputs, 26 column tiles: waves 0-1 take 4, the others 3) and V[1]
    // (NP outputs, wave 7, whose ring is loaded behind its last PI[1] MFMA)
    {
        float bp[4];
#pragma unroll
        for (int j = 0; j < 4; j++) bp[j] = bias16(10, min(w + 8 * j, CT - 1));
        const float bv = bias16(12, 0);
        auto store_logits = [&](int nc) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (j < nc) store16(j, w + 8 * j, logits, LS, 0, 16 * CT, [&](float x, int) { return x + bp[j]; });
        };
        if (w + 24 < CT) {
            gemm16<4, 8>(W + Nt::woff(10), w, 8, ring, leaf_fetch(bufP, 0), a16, NoNext());
            store_logits(4);
        } else if (w != 7) {
            gemm16<3, 8>(W + Nt::woff(10), w, 8, ring, leaf_fetch(bufP, 0), a16, NoNext());
            store_logits(3);
        } else {
            gemm16<3, 8>(W + Nt::woff(10), w, 8, ring, leaf_fetch(bufP, 0), a16,
                         [&] { ring_load<1, 8>(W + Nt::woff(12), 0, 1, 1, ring); });
            store_logits(3);
            gemm16<1, 8>(W + Nt::woff(12), 0, 1, ring, leaf_fetch(bufA, 0), a16, NoNext());
            const int n = acc16_col();
            if (n < NP) {
#pragma unroll
                for (int rt = 0; rt < 2; rt++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int i = 16 * rt + acc16_row(r);
                        if (i < nb) v_out[rowof(i) * NP + n] = tanhf(a16[0][rt][r] + bv);
                    }
            }
        }
        lds_barrier();
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
            const uint64_t *mk = mskl + min(i, nb - 1) * 7;
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
        for (int q = 0; q < PERW; q++) m[q] = wave_max_f32(m[q]);
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
        for (int q = 0; q < PERW; q++) sum[q] = wave_sum_f32(sum[q]);
#pragma unroll
        for (int q = 0; q < PERW; q++) {
            const int i = w * PERW + q;
            if (i < nb) {
                const float inv = 1.f / sum[q];
#pragma unroll
                for (int k = 0; k < 7; k++) {
                    const int a = 64 * k + lane;
                    if (a < ACT) pi_out[rowof(i) * ACT + a] = x[q][k] * inv;
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

static int launch_nn(int n_players, int B, const int8_t *leaf_state, const uint64_t *leaf_mask,
                     const float *packed_weights, float *pi, float *v, const int32_t *idx, const int32_t *count,
                     void *hs) {
    if (n_players < 2 || n_players > 4 || B < 0 || (B && (!leaf_state || !leaf_mask || !packed_weights || !pi || !v)))
        return SPL_EINVAL;
    if (!B) return 0;
    const dim3 grid((unsigned)((B + ML - 1) / ML));
    switch (n_players) {
        case 2: hipLaunchKernelGGL(k_nn_forward<2>, grid, dim3(NNT), 0, (hipStream_t)hs, B, leaf_state, leaf_mask,
                                   packed_weights, pi, v, idx, count); break;
        case 3: hipLaunchKernelGGL(k_nn_forward<3>, grid, dim3(NNT), 0, (hipStream_t)hs, B, leaf_state, leaf_mask,
                                   packed_weights, pi, v, idx, count); break;
        default: hipLaunchKernelGGL(k_nn_forward<4>, grid, dim3(NNT), 0, (hipStream_t)hs, B, leaf_state, leaf_mask,
                                    packed_weights, pi, v, idx, count); break;
    }
    return check_launch();
}

int spl_nn_forward(int n_players, int B, const int8_t *leaf_state, const uint64_t *leaf_mask,
                   const float *packed_weights, float *pi, float *v, void *hs) {
    return launch_nn(n_players, B, leaf_state, leaf_mask, packed_weights, pi, v, nullptr, nullptr, hs);
}

int spl_nn_forward_indexed(int n_players, int B, const int8_t *leaf_state, const uint64_t *leaf_mask,
                           const int32_t *leaf_index, const int32_t *leaf_count, const float *packed_weights,
                           float *pi, float *v, void *hs) {
    if (!leaf_index || !leaf_count) return SPL_EINVAL;
    return launch_nn(n_players, B, leaf_state, leaf_mask, packed_weights, pi, v, leaf_index, leaf_count, hs);
}

}  // extern "C"
