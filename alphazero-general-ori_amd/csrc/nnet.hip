// nnet.hip — SplendorNNet inference (SplendorNNet.py:56-159, eval mode) as one fused
// gfx950 kernel: int8 leaf boards + packed legality masks in, masked softmax policy and
// tanh values out (GenericNNetWrapper.predict, :141-168). C ABI: include/splendor_amd.h.
//
// One 512-thread workgroup (8 waves, two per SIMD so one wave's LDS / L2 latency hides
// behind the other's MFMAs) evaluates ML = 32 leaves through all 13 dense layers with every
// activation on chip. f32 arithmetic, the reference network's precision, on bf16 MFMAs: every
// f32 operand is split exactly into three bf16 parts (x = hi + mid + lo by truncation) and
// x y is the sum of six part products (all but the three smallest, < 2^-22 |x y| together),
// the largest in an f32 accumulator of its own. gfx950 has no xf32 and its f32 MFMA runs at
// 1/16 of the bf16 rate, so six bf16 products cost 3/8 of one f32 product's MFMA time.
//   * Per-column layers (dense2d_1, its second linear, partialgpool_1, dense2d_3; round 4)
//     on v_mfma_f32_32x32x16_bf16: the 7 board columns of the 32 leaves as 7 token tiles of
//     32 (channel-major, so the per-column BatchNorm affine is uniform across a tile); wave w
//     owns output column blocks 2(w&1), 2(w&1)+1 of token tiles 2(w>>1), 2(w>>1)+1 (wave 6, 7:
//     tile 6 alone); the activations (f32 LDS rows, 132-float stride) are split in registers,
//     each A fragment once for both column blocks (round 5: 2 splits per token tile, was 4).
//   * Per-leaf layers (round 5) on v_mfma_f32_16x16x32_bf16 over 16-leaf row tiles. Their
//     activations live in LDS ALREADY SPLIT: each producing epilogue writes its outputs as
//     three bf16 planes (SplitAct), split once instead of once per consuming wave (8 waves
//     read every input). dense1d_4's input, the 704-feature flattened image, is too large
//     for three planes: it stays f32 and each wave splits the one row tile it needs (two
//     column tiles per wave, half the splitting of one column tile over both row tiles).
//   * Weights: every layer's parts split and packed once on the host in MFMA B-fragment order
//     (spl_nn_forward in splendor_amd.h), each lane's B operand one coalesced 16-byte load,
//     prefetched a chunk ahead in a register ring; the next layer's ring is issued behind the
//     last MFMA of the current one; barriers wait for LDS only.
#include <hip/hip_runtime.h>

#include "../../include/splendor_amd.h"

// per-layer cycle probes (diagnostic builds only, -DNN_PROBE=1; never the product): wave 0's
// s_memtime at every layer boundary, summed over the workgroups (spl_diag_nn_probe)
#ifndef NN_PROBE
#define NN_PROBE 0
#endif
#if NN_PROBE
__device__ unsigned long long g_nn_probe[16];
#define NPROBE(k)                                                  \
    if (threadIdx.x == 0) {                                        \
        const uint64_t c_ = __builtin_readcyclecounter();          \
        atomicAdd(&g_nn_probe[k], (unsigned long long)(c_ - nlast)); \
        nlast = c_;                                                \
    }
#else
#define NPROBE(k)
#endif

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int NNT = 512;      // threads per workgroup (8 waves)
constexpr int ML = 32;         // leaves per workgroup
constexpr int LS = 420;        // logits row stride (floats)
constexpr int ZS = 712;        // flattened trunk row stride (704 features; 8 mod 64 dwords)
constexpr int ACT = 409;
// split per-leaf activations: three bf16 planes of ML rows, row stride SS bf16 (72 dwords = 8
// mod 64: the 16 rows x 4 k groups of a 16x16x32 operand read, ds_read_b128, spread over the
// banks); columns [128, 144) hold zeros (the pool layers read k = 16 .. 143 against 0 weights)
constexpr int SS = 144;
struct SplitAct {
    uint16_t p[3][ML][SS];
};
constexpr int SAB = (int)sizeof(SplitAct);                 // 27,648 bytes
// Per-column stage (round 6): wave w < 7 owns board column w of the ML leaves (one 32-token
// tile) and keeps its 128-channel activation in registers through all four per-column layers;
// the layers' split weights stream through LDS, once per workgroup, in stages of at most
// RSTAGE 16-k chunks (RSLOT bytes each: 4 column blocks x 3 parts x 64 lanes x 16 B, lane-linear
// MFMA fragments), double-buffered and filled by wave 7 with LDS-DMA loads.
constexpr int RSLOT = 4 * 3 * 1024;
constexpr int RSTAGE = 4;
constexpr int RING = 2 * RSTAGE * RSLOT;                   // 98,304 bytes
constexpr int PS = 64;                                     // pool staging row (floats, 16-B units swizzled)
// bufA (bytes): the int8 input staging and the weight ring (per-column stage), then the
// flattened trunk Z [ML][ZS] with the pool staging P [5][ML][PS] of columns 0-4's channels 0-63
// behind it, then — once dense1d_4 has read Z — split buffers SB1 [0, SAB), SB2 [SAB, 2 SAB)
// and the logits from 2 SAB on; SB0 has its own array (the per-column biases before dense1d_4)
constexpr int ZBYTES = ML * ZS * 4;
constexpr int BUFA = ZBYTES + 5 * ML * PS * 4;             // 132,096 bytes
static_assert(2 * SAB + ML * LS * 4 <= BUFA, "bufA overlays");
static_assert(4 * 128 * 4 <= SAB, "per-column biases fit SB0");

__host__ __device__ constexpr int kpad(int K) { return (K + 7) / 8 * 8; }
__host__ __device__ constexpr int ntiles(int N) { return (N + 31) / 32; }
__host__ __device__ constexpr int ntiles16(int N) { return (N + 15) / 16; }
// f32 copy of every layer (kept in the packed layout: the biases are read from it, the host
// reference and older builds read the rest): the 4 per-column layers in 32x32x2 B fragments,
// the 9 per-leaf layers in 16x16x4 B fragments
__host__ __device__ constexpr bool f16(int l) { return l >= 4; }
__host__ __device__ constexpr int colpad(int l, int N) { return f16(l) ? ntiles16(N) * 16 : ntiles(N) * 32; }
__host__ __device__ constexpr int wfloats(int l, int N, int K) { return colpad(l, N) * kpad(K); }
// the split copy of a per-column layer: [4][Kp16/16][3][64][8] bf16 (hi, mid, lo parts of
// W[32 nt + l % 32][16 c + 8 (l / 32) + j]), as floats
__host__ __device__ constexpr int kp16(int K) { return (K + 15) / 16 * 16; }
__host__ __device__ constexpr int sfloats(int K) { return 4 * (kp16(K) / 16) * 3 * 64 * 8 / 2; }
// the split copy of a per-leaf layer: [NT16][Kp32/32][3][64][8] bf16 (parts of
// W[16 nt + l % 16][32 c + 8 (l / 16) + j]), as floats
__host__ __device__ constexpr int kp32(int K) { return (K + 31) / 32 * 32; }
__host__ __device__ constexpr int lfloats(int N, int K) { return ntiles16(N) * (kp32(K) / 32) * 3 * 64 * 8 / 2; }

// layer order of the packed weights: dense2d_1, dense2d_1[3], partialgpool_1 dense,
// dense2d_3, dense1d_4, partialgpool_4 dense, dense1d_5[0], dense1d_5[3], partialgpool_5
// dense, PI[0], PI[1], V[0], V[1]; then the per-column BN affines s1, t1, sp1, tp1 (7 each);
// then (16-byte aligned) the split copies of all 13 layers
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
    static constexpr int SBASE = (AFF + 28 + 3) / 4 * 4;
    static constexpr int soff(int l) {
        int o = SBASE;
        for (int j = 0; j < l; j++) o += j < 5 ? sfloats(Ks[j]) : lfloats(Ns[j], Ks[j]);
        return o;
    }
    static constexpr int TOTAL = soff(NL);
    static constexpr int X0S = (kpad(R) / 4) % 2 ? kpad(R) : kpad(R) + 4;   // int8 input stride (odd dwords)
    // per-column stage: 16-k chunks per layer, each layer split into one or two LDS stages
    static constexpr int CL[4] = {kp16(R) / 16, 8, 6, 8};
    static constexpr int XR = (7 * ML * X0S + 15) / 16 * 16;  // weight ring offset in bufA (bytes)
    static constexpr int first(int l) { return CL[l] > RSTAGE ? (CL[l] + 1) / 2 : CL[l]; }
    static constexpr int nstages(int l) { return CL[l] > RSTAGE ? 2 : 1; }
    static constexpr int NSTG = nstages(0) + nstages(1) + nstages(2) + nstages(3);
    // stage s: (layer, first chunk, chunks)
    static constexpr int stg_layer(int s) {
        for (int l = 0; l < 4; l++) {
            if (s < nstages(l)) return l;
            s -= nstages(l);
        }
        return -1;
    }
    static constexpr int stg_index(int s) {
        for (int l = 0; l < 4; l++) {
            if (s < nstages(l)) return s;
            s -= nstages(l);
        }
        return -1;
    }
    static constexpr int stg_c0(int s) { return stg_index(s) ? first(stg_layer(s)) : 0; }
    static constexpr int stg_nc(int s) { return stg_index(s) ? CL[stg_layer(s)] - first(stg_layer(s)) : first(stg_layer(s)); }
};
static_assert(Net<4>::XR + RING <= BUFA, "input staging + weight ring fit bufA");

template <int V> struct IntC {
    static constexpr int value = V;
};

// Split per-column GEMMs: an f32 x is exactly hi + mid + lo, three bf16 parts taken by
// truncation (hi: the top 8 significant bits, mid: the top 8 of the residual, lo: the rest, at
// most 8 significant bits), and x y = the sum over the parts' products minus the three smallest
// (mid lo, lo mid, lo lo: < 2^-22 |x y| together, ~2^-24 typically). v_mfma_f32_32x32x16_bf16
// takes 16 k per instruction at 16 times the f32 MFMA's rate, so the six products of a 16-k chunk
// cost 6 x 32 cycles against 8 x 64 for v_mfma_f32_32x32x2_f32. Each bf16 product is exact in
// f32; hi hi goes into the layer's accumulator and the five smaller products into a second one
// (added in the epilogue), so the large accumulator rounds once per MFMA (16 k) instead of once
// per k, and the small one's roundings are ~2^-8 smaller: measured against float64 the split
// layer's error is below the f32 MFMA's (tools/nn_split_probe.hip). The int8
// boards of dense2d_1 are exact in bf16: three products (the weight's parts) into one
// accumulator.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct F8 {
    float4 lo, hi;                     // 8 consecutive k of one lane's A row
};

// the bf16 pair (upper halves of a, b) -> one dword, b low: one v_perm_b32
__device__ __forceinline__ uint32_t hi_pair(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }
__device__ __forceinline__ void split8(const F8 &x, bf16x8 &hi, bf16x8 &mid, bf16x8 &lo) {
    const float xs[8] = {x.lo.x, x.lo.y, x.lo.z, x.lo.w, x.hi.x, x.hi.y, x.hi.z, x.hi.w};
    float r1[8], r2[8];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {                     // (pairs: v_pk_add_f32)
        const f32x2 x2 = {xs[j], xs[j + 1]};
        const f32x2 h2 = {__uint_as_float(__float_as_uint(xs[j]) & 0xFFFF0000u),
                          __uint_as_float(__float_as_uint(xs[j + 1]) & 0xFFFF0000u)};
        const f32x2 a2 = x2 - h2;
        const f32x2 m2 = {__uint_as_float(__float_as_uint(a2[0]) & 0xFFFF0000u),
                          __uint_as_float(__float_as_uint(a2[1]) & 0xFFFF0000u)};
        const f32x2 b2 = a2 - m2;
        r1[j] = a2[0]; r1[j + 1] = a2[1]; r2[j] = b2[0]; r2[j + 1] = b2[1];
    }
    u32x4 H, M, L;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        H[p] = hi_pair(__float_as_uint(xs[2 * p]), __float_as_uint(xs[2 * p + 1]));
        M[p] = hi_pair(__float_as_uint(r1[2 * p]), __float_as_uint(r1[2 * p + 1]));
        L[p] = hi_pair(__float_as_uint(r2[2 * p]), __float_as_uint(r2[2 * p + 1]));
    }
    hi = __builtin_bit_cast(bf16x8, H);
    mid = __builtin_bit_cast(bf16x8, M);
    lo = __builtin_bit_cast(bf16x8, L);
}
// 8 int8 (two dwords) -> 8 bf16, exact
__device__ __forceinline__ bf16x8 i8_to_bf16x8(int v0, int v1) {
    u32x4 r;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const int v = p < 2 ? v0 : v1, sh = 16 * (p & 1);
        r[p] = hi_pair(__float_as_uint((float)(int8_t)(v >> sh)), __float_as_uint((float)(int8_t)(v >> (sh + 8))));
    }
    return __builtin_bit_cast(bf16x8, r);
}

// workgroup barrier for LDS traffic only: waits for this wave's LDS operations, not for its
// global loads, so weight fragments prefetched for the next layer stay in flight across it
// (__syncthreads() waits vmcnt(0) first); the memory clobber keeps the compiler from moving
// LDS accesses across it
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// ------------------------------------------------------------ per-leaf layers
// one f32 into the three planes of a SplitAct (the truncation of split8 and of the host's
// _bf16_parts: hi + mid + lo == x exactly)
__device__ __forceinline__ void put_split(SplitAct *d, int row, int col, float x) {
    const uint32_t h = __float_as_uint(x) & 0xFFFF0000u;
    const float r1 = x - __uint_as_float(h);
    const uint32_t m = __float_as_uint(r1) & 0xFFFF0000u;
    const float r2 = r1 - __uint_as_float(m);
    d->p[0][row][col] = (uint16_t)(h >> 16);
    d->p[1][row][col] = (uint16_t)(m >> 16);
    d->p[2][row][col] = (uint16_t)(__float_as_uint(r2) >> 16);
}
// ... and back, exactly (mid + lo, then + hi, as the split took them apart)
__device__ __forceinline__ float get_split(const SplitAct *s, int row, int col) {
    const float h = __uint_as_float((uint32_t)s->p[0][row][col] << 16);
    const float m = __uint_as_float((uint32_t)s->p[1][row][col] << 16);
    const float l = __uint_as_float((uint32_t)s->p[2][row][col] << 16);
    return h + (m + l);
}

// weight-part ring of a per-leaf GEMM: PF chunks (32 k) x NC column tiles x 3 parts
template <int NC, int PF>
struct RingL {
    static constexpr int P = PF;
    bf16x8 b[PF][NC][3];
};
// column tile j of a per-leaf layer: tile min(c0 + j cstep, ctot - 1) (a clamped tile is
// loaded but never multiplied)
template <int C>
__device__ __forceinline__ const bf16x8 *tilel(const float *__restrict__ ws, int c0, int cstep, int ctot, int j) {
    return reinterpret_cast<const bf16x8 *>(ws) + (size_t)min(c0 + j * cstep, ctot - 1) * C * 3 * 64 + (threadIdx.x & 63);
}
// the first chunks of a per-leaf layer's weight parts into the ring; callers issue this behind
// the previous layer's last MFMA, ahead of its epilogue and barrier, so no layer starts on an
// L2 round trip
template <int C, class RG>
__device__ __forceinline__ void ringl_load(const float *__restrict__ ws, int c0, int cstep, int ctot, RG &r) {
    constexpr int NC = sizeof(r.b[0]) / sizeof(r.b[0][0]);
#pragma unroll
    for (int j = 0; j < NC; j++) {
        const bf16x8 *w = tilel<C>(ws, c0, cstep, ctot, j);
#pragma unroll
        for (int p = 0; p < RG::P; p++)
#pragma unroll
            for (int q = 0; q < 3; q++) r.b[p][j][q] = w[((p < C ? p : C - 1) * 3 + q) * 64];
    }
}
// per-leaf GEMM on v_mfma_f32_16x16x32_bf16: RT row tiles of 16 leaves x NC column tiles
// {c0, c0 + cstep, ...} (NC <= the ring's) over C chunks of 32 k. afetch(t, c, a0, a1, a2):
// the three parts of this lane's A operand for row tile t (row l % 16 of it, k = 32 c +
// 8 (l / 16) .. + 7); the ring holds the first chunks (ringl_load); next() runs after the last
// MFMA is issued. Each (column, row) tile keeps two accumulators, the hi x hi products and
// the five smaller ones, added at the end. Unrolled and branch-free like gemm_split.
template <int NC, int RT, int C, class RG, class AF, class NX>
__device__ __forceinline__ void gemm_leaf(const float *__restrict__ ws, int c0, int cstep, RG &r, AF afetch,
                                          f32x4 (*acc)[2], NX next) {
    constexpr int PF = RG::P;
    const bf16x8 *w[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) w[j] = tilel<C>(ws, c0, cstep, 1 << 30, j);
    f32x4 acl[NC][RT];
#pragma unroll
    for (int j = 0; j < NC; j++)
#pragma unroll
        for (int t = 0; t < RT; t++) {
            acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            acl[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
    for (int c = 0; c < C; c++) {
        bf16x8 a[RT][3];
#pragma unroll
        for (int t = 0; t < RT; t++) afetch(t, c, a[t][0], a[t][1], a[t][2]);
#pragma unroll
        for (int j = 0; j < NC; j++) {
            const bf16x8 b0 = r.b[c % PF][j][0], b1 = r.b[c % PF][j][1], b2 = r.b[c % PF][j][2];
            if (c + PF < C)
#pragma unroll
                for (int q = 0; q < 3; q++) r.b[c % PF][j][q] = w[j][((c + PF) * 3 + q) * 64];
#pragma unroll
            for (int t = 0; t < RT; t++) {
                acl[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][2], b0, acl[j][t], 0, 0, 0);
                acl[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][1], b1, acl[j][t], 0, 0, 0);
                acl[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][0], b2, acl[j][t], 0, 0, 0);
                acl[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][1], b0, acl[j][t], 0, 0, 0);
                acl[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][0], b1, acl[j][t], 0, 0, 0);
                acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t][0], b0, acc[j][t], 0, 0, 0);
            }
        }
        // keep each chunk's loads in its chunk: left alone, the scheduler sinks them next to
        // their MFMAs PF chunks later (vmcnt waits, the ring gone)
        __builtin_amdgcn_sched_barrier(0);
    }
    next();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NC; j++)
#pragma unroll
        for (int t = 0; t < RT; t++) acc[j][t] += acl[j][t];
}
struct NoNext {
    __device__ void operator()() const {}
};
// 16x16 accumulator element r of this lane: row (within the row tile) and column
__device__ __forceinline__ int acc16_row(int r) { return ((threadIdx.x & 63) >> 4) * 4 + r; }
__device__ __forceinline__ int acc16_col() { return threadIdx.x & 15; }


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

// LDS-DMA of one 1 KB MFMA fragment: 16 bytes per lane from src (this lane's address) to the
// wave-uniform LDS base dst (+ 16 x lane); counted by vmcnt, no VGPR destination
__device__ __forceinline__ void glds16(const char *src, char *dst) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)dst, 16, 0, 0);
}
__device__ __forceinline__ f32x4 relu4(f32x4 v) {
    return f32x4{fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)};
}

// The search's NN leaves as k_leaf_mask lists them (ABI 11): segment j (trees 64 j .. 64 j + 63)
// has count[j] leaves at idx[64 j ..]; the list is their concatenation in segment order.
// Wave-collective: returns the list's length; with rowt / offv (ML ints each, the wave's own),
// rowt[i] (i < ML) = the idx position of list entry b0 + i. A lane holds 8 consecutive
// segments' counts (two 16-byte loads) and one DPP scan gives every segment's first entry; each
// segment that reaches into the tile marks the slot where it starts (slot, and 64 j - start
// in offv), and a prefix maximum over the slots gives every slot its segment.
__device__ __forceinline__ int nn_list_rows(const int32_t *__restrict__ count, int nseg, int b0, int *rowt, int *offv) {
    const int lane = threadIdx.x & 63;
    if (rowt && lane < ML) rowt[lane] = -1;
    int base = 0;
    for (int c0 = 0; c0 < nseg; c0 += 512) {
        const int j0 = c0 + 8 * lane;
        int v[8];
        if (j0 + 8 <= nseg) {
            const int4 a = *reinterpret_cast<const int4 *>(count + j0), b = *reinterpret_cast<const int4 *>(count + j0 + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
#pragma unroll
            for (int q = 0; q < 8; q++) v[q] = j0 + q < nseg ? count[j0 + q] : 0;
        }
        int own = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) own += v[q];
        // inclusive scan of the lanes' sums on DPP: row_shr 1 / 2 / 4 / 8 inside each 16-lane
        // row (lanes without a source add 0), then row_bcast 15 (rows 1, 3) and 31 (rows 2, 3)
        int inc = own;
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x111, 0xf, 0xf, true);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x112, 0xf, 0xf, true);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x114, 0xf, 0xf, true);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x118, 0xf, 0xf, true);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x142, 0xa, 0xf, false);
        inc += __builtin_amdgcn_update_dpp(0, inc, 0x143, 0xc, 0xf, false);
        if (rowt) {
            int ex = base + inc - own;                   // first list entry of segment j0
#pragma unroll
            for (int q = 0; q < 8; q++) {
                if (v[q] > 0 && ex + v[q] > b0 && ex < b0 + ML) {
                    const int sl = max(ex - b0, 0);
                    rowt[sl] = sl;
                    offv[sl] = 64 * (j0 + q) - ex;
                }
                ex += v[q];
            }
        }
        base += __builtin_amdgcn_readlane(inc, 63);
    }
    if (rowt) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        int f = lane < ML ? rowt[lane] : -1;             // prefix maximum over slots 0 .. 31
        f = max(f, __builtin_amdgcn_update_dpp(-1, f, 0x111, 0xf, 0xf, false));
        f = max(f, __builtin_amdgcn_update_dpp(-1, f, 0x112, 0xf, 0xf, false));
        f = max(f, __builtin_amdgcn_update_dpp(-1, f, 0x114, 0xf, 0xf, false));
        f = max(f, __builtin_amdgcn_update_dpp(-1, f, 0x118, 0xf, 0xf, false));
        f = max(f, __builtin_amdgcn_update_dpp(-1, f, 0x142, 0xa, 0xf, false));
        const int pos = f >= 0 ? b0 + lane + offv[f] : 0;
        __builtin_amdgcn_wave_barrier();
        if (lane < ML) rowt[lane] = pos;
    }
    return base;
}

template <int NP>
// one workgroup per CU (LDS) = 2 waves per SIMD: the register budget is 256, and without
// saying so the scheduler sinks the prefetched weight loads next to their MFMAs
// idx / count (optional): the kernel evaluates the search's NN leaves as k_leaf_mask lists
// them (nn_list_rows: B trees in segments of 64) — board / mask / output row idx[...] —
// instead of rows 0 .. B; tiles past the list's end exit at once.
__global__ __launch_bounds__(NNT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_nn_forward(int B, const int8_t *__restrict__ state,
                                                    const uint64_t *__restrict__ mask,
                                                    const float *__restrict__ W, float *__restrict__ pi_out,
                                                    float *__restrict__ v_out,
                                                    const int32_t *__restrict__ idx,
                                                    const int32_t *__restrict__ count) {
    using Nt = Net<NP>;
    constexpr int R = Nt::R, X0S = Nt::X0S, NSTG = Nt::NSTG;
    // all LDS in one array (a second __shared__ object beside LDS-DMA targets can make the
    // compiler drain vmcnt before LDS reads): bufA, SB0, the legality masks
    __shared__ __align__(16) char lds[BUFA + SAB + ML * 7 * 8 + 15 * ML * 4];
    float *bufA = reinterpret_cast<float *>(lds);
    SplitAct *SB0 = reinterpret_cast<SplitAct *>(lds + BUFA);
    uint64_t *mskl = reinterpret_cast<uint64_t *>(lds + BUFA + SAB);
    // wave index in an SGPR: every per-wave choice below is a scalar branch
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, li = lane & 31;
    const int h = lane >> 5;
    const int b0 = blockIdx.x * ML;
    const float *aff = W + Nt::AFF;                        // s1, t1, sp1, tp1
    char *ring = lds + Nt::XR;                             // per-column weight stages (2 buffers)
    float *biasL = reinterpret_cast<float *>(SB0);         // [4][128] per-column biases (until dense1d_4)
    // wave 7 (it owns no board column) fills the weight stages: stage S's split weight chunks
    // into buffer S & 1, one 1 KB fragment (column block b, part p, chunk c) per instruction
    auto load_stage = [&](auto s_const) {
        constexpr int S = decltype(s_const)::value;
        if constexpr (S < NSTG) {
            constexpr int L = Nt::stg_layer(S), C0 = Nt::stg_c0(S), NC = Nt::stg_nc(S), C = Nt::CL[L];
            const char *src = reinterpret_cast<const char *>(W + Nt::soff(L)) + lane * 16;
            char *dst = ring + (S & 1) * RSTAGE * RSLOT;
#pragma unroll
            for (int j = 0; j < NC; j++)
#pragma unroll
                for (int b = 0; b < 4; b++)
#pragma unroll
                    for (int p = 0; p < 3; p++)
                        glds16(src + ((b * C + C0 + j) * 3 + p) * 1024, dst + ((j * 4 + b) * 3 + p) * 1024);
        }
    };
    if (w == 7) {                                        // (first: the weights do not depend on
        load_stage(IntC<0>());                           //  the tile's leaves)
        load_stage(IntC<1>());
    }
    // the tile's idx positions (nn_list_rows): a copy per input wave, each mapped by its own
    // wave (no barrier before the input loads; wave 7, which stages no input, needs only the
    // list's length); wave 0 also resolves the rows themselves into rowv for the epilogues
    int *rowt = reinterpret_cast<int *>(lds + BUFA + SAB + ML * 7 * 8);
    int *rowt_w = rowt + (w < 7 ? w : 0) * ML, *rowv = rowt + 7 * ML, *offv_w = rowt + (8 + (w < 7 ? w : 0)) * ML;
    int cnt = B;
    if (count) {
        cnt = __builtin_amdgcn_readfirstlane(
            nn_list_rows(count, (B + 63) >> 6, b0, w < 7 ? rowt_w : nullptr, offv_w));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // (the wave's own LDS writes,
        __builtin_amdgcn_wave_barrier();                        //  read back by its lanes)
    }
    if (b0 >= cnt) {                                     // (past the list: wave 7's stages land
        if (w == 7) __builtin_amdgcn_s_waitcnt(0);       //  before the workgroup's LDS is freed)
        return;
    }
    const int nb = min(ML, cnt - b0);
    // row of leaf i of this tile (its board, mask and outputs): rowin while the wave stages the
    // input, rowof in the epilogues
    const auto rowin = [&](int i) -> size_t { return count ? (size_t)idx[rowt_w[i]] : (size_t)(b0 + i); };
    const auto rowof = [&](int i) -> size_t { return count ? (size_t)rowv[i] : (size_t)(b0 + i); };

#if NN_PROBE
    uint64_t nlast = __builtin_readcyclecounter();
    if (threadIdx.x == 0) atomicAdd(&g_nn_probe[15], 1ull);
#endif
    // ---- input: x[column c][leaf i][row r] = state[leaf][r][c] as int8 (token c*32+i)
    // (no zero fill: the k past R of a row read the row's padding, the next row or, after the
    // last one, the bytes behind it — any int8 is finite and those k have zero weights; rows
    // of missing leaves are never stored)
    int8_t *x0 = reinterpret_cast<int8_t *>(lds);
    // (waves 0-6 stage the input, so wave 7's vmcnt counts its LDS-DMA only)
    constexpr int NS7 = NNT - 64;
    if (w < 7) {
        if (tid < nb * 7) mskl[tid] = mask[rowin(tid / 7) * 7 + tid % 7];
        // per-column biases; partialgpool_1's outputs land on channels 8..127 (its 8 pooled
        // channels come first), so its bias is shifted by 8
        for (int t = tid; t < 4 * 128; t += NS7) {
            const int l = t >> 7, c = t & 127;
            biasL[t] = l == 2 ? (c >= 8 ? W[Nt::boff(2) + c - 8] : 0.f) : W[Nt::boff(l) + c];
        }
        if constexpr ((7 * R) % 4 == 0) {
            // the workgroup's boards: dword loads (a board is a whole number of dwords), all in
            // flight at once, then each byte scattered to its (column, leaf, row) slot
            constexpr int BW = R * 7 / 4;                  // dwords per board
            constexpr int PER = (ML * BW + NS7 - 1) / NS7;
            int32_t d[PER];
#pragma unroll
            for (int k = 0; k < PER; k++) {
                const int j = tid + k * NS7, i = j / BW;
                d[k] = j < nb * BW ? reinterpret_cast<const int32_t *>(state + rowin(i) * R * 7)[j - i * BW] : 0;
            }
#pragma unroll
            for (int k = 0; k < PER; k++) {
                const int j = tid + k * NS7;
                if (j < nb * R * 7 / 4) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int o = 4 * j + q, i = o / (R * 7), rem = o - i * (R * 7), r = rem / 7, c = rem - 7 * r;
                        x0[(c * ML + i) * X0S + r] = (int8_t)(d[k] >> (8 * q));
                    }
                }
            }
        } else {
            for (int j = tid; j < nb * R; j += NS7) {      // one board row (7 bytes) per thread
                const int i = j / R, r = j - i * R;
                const int8_t *src = state + (rowin(i) * R + r) * 7;
#pragma unroll
                for (int c = 0; c < 7; c++) x0[(c * ML + i) * X0S + r] = src[c];
            }
        }
        if (count && w == 0 && lane < nb) rowv[lane] = (int)rowin(lane);   // (after the input loads)
    } else {
        // stage 0 landed (stage 1's 12 x nc fragments may stay in flight): vmcnt(N) encoded as
        // vmcnt[3:0] | vmcnt[5:4] << 14, expcnt and lgkmcnt at their maxima (no wait)
        constexpr int N1 = 12 * Nt::stg_nc(1);
        static_assert(N1 < 64, "vmcnt range");
        __builtin_amdgcn_s_waitcnt((N1 & 15) | ((N1 >> 4) << 14) | (7 << 4) | (15 << 8));
    }
    lds_barrier();
    NPROBE(0)

    // ---- per-column layers (round 6), wave w < 7 = board column w of the ML leaves, in
    // registers: out^T[channel][leaf] = W[channel][k] x^T[k][leaf] on v_mfma_f32_32x32x16_bf16
    // with the weights as the A operand (rows = output channels, 4 blocks of 32) and the
    // activations as B (columns = this tile's 32 leaves). An accumulator's lane l holds leaf
    // l % 32 at channels (r & 3) + 8 (r >> 2) + 4 (l >> 5) of its block, so the next layer's
    // B fragment of a 16-channel chunk (lane l: channels 8 (l >> 5) .. + 7) is two 4-register
    // groups of one block with their 32-lane halves exchanged (4 v_permlane32_swap), then split
    // into three bf16 parts once for all 4 output blocks. Six part products per chunk, hi x hi
    // into the block's accumulator X (started at the bias), the five smaller ones into a second
    // accumulator Xs (round 4's two-accumulator precision, now for every per-column layer).
    f32x16 X[4], Y[4], Ys[4];
    // dense1d_4 (see there): wave w computes output blocks 2 (w & 1), + 1 over K quarter w >> 1;
    // its weight fragments (A operand, 32x32x16 order) PF4 chunks ahead in registers
    constexpr int C4 = 11, PF4 = 2;
    const int bp4 = w & 1, kq4 = w >> 1;
    const bf16x8 *w4 = reinterpret_cast<const bf16x8 *>(W + Nt::soff(4)) + (size_t)(2 * bp4 * 4 * C4 + kq4 * C4) * 3 * 64 + lane;
    constexpr int W4B = 4 * C4 * 3 * 64;                   // the next block's fragments (bf16x8)
    bf16x8 r4[PF4][2][3];
    RingL<1, 2> ring1;                                     // per-leaf layers' weight ring
    auto stage = [&](auto s_const) {
        constexpr int S = decltype(s_const)::value;
        constexpr int L = Nt::stg_layer(S), C0 = Nt::stg_c0(S), NC = Nt::stg_nc(S);
        if (w < 7) {
            if constexpr (C0 == 0) {                       // a layer's first stage: bias, zero
#pragma unroll
                for (int b = 0; b < 4; b++)
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        const f32x4 bb = *reinterpret_cast<const f32x4 *>(biasL + 128 * L + 32 * b + 8 * g + 4 * h);
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            Y[b][4 * g + i] = bb[i];
                            Ys[b][4 * g + i] = 0.f;
                        }
                    }
            }
            const char *buf = ring + (S & 1) * RSTAGE * RSLOT + lane * 16;
#pragma unroll
            for (int j = 0; j < NC; j++) {
                bf16x8 bh, bm, bl;
                if constexpr (L == 0) {                    // int8 boards: exact in one bf16 part
                    const int32_t *px = reinterpret_cast<const int32_t *>(x0 + (w * ML + li) * X0S + 16 * (C0 + j) + 8 * h);
                    bh = i8_to_bf16x8(px[0], px[1]);
                } else {                                   // (partialgpool_1 reads channels 32..127)
                    const int kk = C0 + j + (L == 2 ? 2 : 0), blk = kk >> 1, sh = kk & 1;
                    float v[8];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(X[blk][8 * sh + i]),
                                                                         __float_as_uint(X[blk][8 * sh + 4 + i]), false, false);
                        v[i] = __uint_as_float(r2[0]);
                        v[4 + i] = __uint_as_float(r2[1]);
                    }
                    split8(F8{float4{v[0], v[1], v[2], v[3]}, float4{v[4], v[5], v[6], v[7]}}, bh, bm, bl);
                }
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const char *f = buf + (j * 4 + b) * 3 * 1024;
                    const bf16x8 wh = *reinterpret_cast<const bf16x8 *>(f);
                    const bf16x8 wm = *reinterpret_cast<const bf16x8 *>(f + 1024);
                    const bf16x8 wl = *reinterpret_cast<const bf16x8 *>(f + 2048);
                    if constexpr (L == 0) {
                        Ys[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, bh, Ys[b], 0, 0, 0);
                        Ys[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, bh, Ys[b], 0, 0, 0);
                    } else {
                        Ys[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, bh, Ys[b], 0, 0, 0);
                        Ys[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, bm, Ys[b], 0, 0, 0);
                        Ys[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bl, Ys[b], 0, 0, 0);
                        Ys[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wm, bh, Ys[b], 0, 0, 0);
                        Ys[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bm, Ys[b], 0, 0, 0);
                    }
                    Y[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, bh, Y[b], 0, 0, 0);
                }
            }
        }
        if constexpr (S == NSTG - 1) {
            // dense1d_4's first weight chunks into registers behind the last MFMA (wave 7 has no
            // LDS-DMA in flight any more)
#pragma unroll
            for (int c = 0; c < PF4; c++)
#pragma unroll
                for (int b = 0; b < 2; b++)
#pragma unroll
                    for (int q = 0; q < 3; q++) r4[c][b][q] = w4[b * W4B + (c * 3 + q) * 64];
        } else if (w == 7) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // stage S + 1 landed
        }
        lds_barrier();                                     // buffer S & 1 read by every wave
        if (w == 7) load_stage(IntC<S + 2>());
    };
    auto layer = [&](auto l_const) {
        constexpr int L = decltype(l_const)::value;
        constexpr int S0 = L == 0 ? 0 : (L == 1 ? Nt::nstages(0) : (L == 2 ? Nt::nstages(0) + Nt::nstages(1)
                                                                         : Nt::NSTG - Nt::nstages(3)));
        stage(IntC<S0>());
        if constexpr (Nt::nstages(L) == 2) stage(IntC<S0 + 1>());
    };
    // ---- dense2d_1: relu(s1[c] * (W1 x + b1) + t1[c])
    layer(IntC<0>());
    if (w < 7) {
        const float sc = aff[w], tc = aff[7 + w];
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) X[b][r] = fmaxf((Y[b][r] + Ys[b][r]) * sc + tc, 0.f);
    }
    NPROBE(1)
    // ---- dense2d_1[3]: relu(W2 x + b2)
    layer(IntC<1>());
    if (w < 7) {
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) X[b][r] = fmaxf(Y[b][r] + Ys[b][r], 0.f);
    }
    NPROBE(2)
    // ---- partialgpool_1: [max, mean over 4 groups of 8 of x[0:32]] ++ relu(BN(Wp1 x[32:] + bp1))
    // (the GEMM's outputs on channels 8..127: its weight rows are shifted by 8 on the host)
    layer(IntC<2>());
    if (w < 7) {
        // group g = channels 8g .. 8g+7 of block 0 = registers 4g .. 4g+3 of both lane halves
        float pm[4], ps[4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const float a0 = X[0][4 * g], a1 = X[0][4 * g + 1], a2 = X[0][4 * g + 2], a3 = X[0][4 * g + 3];
            const float m = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)), sm = ((a0 + a1) + a2) + a3;
            const auto rm = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
            const auto rs = __builtin_amdgcn_permlane32_swap(__float_as_uint(sm), __float_as_uint(sm), false, false);
            const float om = __uint_as_float(h ? rm[0] : rm[1]), os = __uint_as_float(h ? rs[0] : rs[1]);
            pm[g] = fmaxf(m, om);
            ps[g] = h ? os + sm : sm + os;                 // (lower half first in both halves)
        }
        const float sc = aff[14 + w], tc = aff[21 + w];
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) X[b][r] = fmaxf((Y[b][r] + Ys[b][r]) * sc + tc, 0.f);
#pragma unroll
        for (int g = 0; g < 4; g++) X[0][g] = h ? ps[g] / 8.f : pm[g];   // channels 0-3 max, 4-7 mean
    }
    NPROBE(3)
    // ---- dense2d_3: relu(W3 x + b3), then the flattened per-leaf image
    // Z[leaf][704] = [max_c<5 x[c][:64]][mean_c<5 x[c][:64]][x[5][:64]][x[6][:64]][x[c][64:], c<7]
    // (FlattenAndPartialGPool(64, 5)), so dense1d_4 reads plain rows
    layer(IntC<3>());
    float *Z = bufA;
    float *P = bufA + ML * ZS;                             // [5][ML][PS]: columns 0-4, channels 0-63
    SplitAct *SB1 = reinterpret_cast<SplitAct *>(bufA);
    SplitAct *SB2 = reinterpret_cast<SplitAct *>(reinterpret_cast<char *>(bufA) + SAB);
    float *logits = reinterpret_cast<float *>(reinterpret_cast<char *>(bufA) + 2 * SAB);
    if (w < 7) {                                           // (the ring is dead: every wave passed
#pragma unroll                                             //  the last stage's barrier)
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const f32x4 v = relu4(f32x4{Y[b][4 * g], Y[b][4 * g + 1], Y[b][4 * g + 2], Y[b][4 * g + 3]} +
                                      f32x4{Ys[b][4 * g], Ys[b][4 * g + 1], Ys[b][4 * g + 2], Ys[b][4 * g + 3]});
                const int ch = 32 * b + 8 * g + 4 * h;     // 4 consecutive channels of leaf li
                if (b >= 2)
                    *reinterpret_cast<f32x4 *>(Z + li * ZS + 256 + 64 * w + ch - 64) = v;
                else if (w < 5)                            // 16-B units swizzled by leaf (banks)
                    *reinterpret_cast<f32x4 *>(P + (w * ML + li) * PS + 4 * ((ch >> 2) ^ (li & 15))) = v;
                else
                    *reinterpret_cast<f32x4 *>(Z + li * ZS + (w == 5 ? 128 : 192) + ch) = v;
            }
    }
    lds_barrier();
    for (int t = tid; t < ML * 64; t += NNT) {             // channels 0-63 of columns 0-4: max, mean
        const int i = t >> 6, c = t & 63, o = i * PS + 4 * ((c >> 2) ^ (i & 15)) + (c & 3);
        const float p0 = P[o], p1 = P[ML * PS + o], p2 = P[2 * ML * PS + o], p3 = P[3 * ML * PS + o],
                    p4 = P[4 * ML * PS + o];
        Z[i * ZS + c] = fmaxf(fmaxf(fmaxf(p0, p1), fmaxf(p2, p3)), p4);
        Z[i * ZS + 64 + c] = ((((p0 + p1) + p2) + p3) + p4) / 5.f;
    }
    lds_barrier();
    NPROBE(4)
    // ---- per-leaf layers: split activations in SB0 / SB1 / SB2 (SplitAct), 16x16x32 tiles
    f32x4 a16[4][2];
    // bias of this lane's column in tile ct of a per-leaf layer (0-padded to whole tiles), read
    // before the layer's GEMM (vmcnt retires loads in order)
    auto bias16 = [&](int layer, int ct) { return W[Nt::boff(layer) + 16 * ct + acc16_col()]; };
    // A operand of a split source: the three planes' 8 bf16 at (row, k) of this lane
    auto split_fetch = [&](const SplitAct *src, int koff) {
        return [=](int t, int c, bf16x8 &a0, bf16x8 &a1, bf16x8 &a2) {
            const int row = 16 * t + (lane & 15), k = koff + 32 * c + 8 * (lane >> 4);
            a0 = *reinterpret_cast<const bf16x8 *>(&src->p[0][row][k]);
            a1 = *reinterpret_cast<const bf16x8 *>(&src->p[1][row][k]);
            a2 = *reinterpret_cast<const bf16x8 *>(&src->p[2][row][k]);
        };
    };
    // epilogue: tile j (column tile ct) of both row tiles into dst, columns < nmax
    auto store_split = [&](int j, int ct, SplitAct *dst, int dst_off, int nmax, auto f) {
        const int c = 16 * ct + acc16_col();
        if (c < nmax) {
#pragma unroll
            for (int t = 0; t < 2; t++)
#pragma unroll
                for (int r = 0; r < 4; r++) put_split(dst, 16 * t + acc16_row(r), dst_off + c, f(a16[j][t][r]));
        }
    };
    // ---- dense1d_4 (round 6) over the 704 flattened features: out^T[128][leaf] = W4 Z^T on
    // v_mfma_f32_32x32x16_bf16 with the weights as the A operand, K split in four quarters: wave
    // w computes output blocks 2 (w & 1), + 1 over chunks 11 (w >> 1) .. + 10, its B fragment (8
    // features of leaf l % 32) read from Z and split here once for both blocks. Every weight
    // fragment is loaded once per workgroup (round 5's row-tile mapping loaded each twice).
    // Two accumulators as in the per-column layers; waves 2-7 hand their partial sums to waves
    // 0-1 through LDS (RED, over the dead Z), which add them in K order, the bias and the relu,
    // and write the split planes of SB0.
    {
        f32x16 D[2], Ds[2];
#pragma unroll
        for (int b = 0; b < 2; b++) {
            const float *b4 = W + Nt::boff(4) + 32 * (2 * bp4 + b) + 4 * h;
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const float4 bb = ld4(b4 + 8 * g);
                D[b][4 * g] = kq4 ? 0.f : bb.x;
                D[b][4 * g + 1] = kq4 ? 0.f : bb.y;
                D[b][4 * g + 2] = kq4 ? 0.f : bb.z;
                D[b][4 * g + 3] = kq4 ? 0.f : bb.w;
            }
#pragma unroll
            for (int r = 0; r < 16; r++) Ds[b][r] = 0.f;
        }
#pragma unroll
        for (int c = 0; c < C4; c++) {
            bf16x8 wv[2][3];
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int q = 0; q < 3; q++) {
                    wv[b][q] = r4[c % PF4][b][q];
                    if (c + PF4 < C4) r4[c % PF4][b][q] = w4[b * W4B + ((c + PF4) * 3 + q) * 64];
                }
            const float *zp = Z + li * ZS + 16 * (kq4 * C4 + c) + 8 * h;
            bf16x8 bh, bm, bl;
            split8(F8{ld4(zp), ld4(zp + 4)}, bh, bm, bl);
#pragma unroll
            for (int b = 0; b < 2; b++) {
                Ds[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wv[b][2], bh, Ds[b], 0, 0, 0);
                Ds[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wv[b][1], bm, Ds[b], 0, 0, 0);
                Ds[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wv[b][0], bl, Ds[b], 0, 0, 0);
                Ds[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wv[b][1], bh, Ds[b], 0, 0, 0);
                Ds[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wv[b][0], bm, Ds[b], 0, 0, 0);
                D[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wv[b][0], bh, D[b], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        ringl_load<4>(W + Nt::soff(5), w, 8, 8, ring1);   // partialgpool_4's first chunks
        __builtin_amdgcn_sched_barrier(0);
        lds_barrier();                                     // (every wave has read Z: RED overlays it)
        float *RED = Z;                                    // [3][2][2][ML][32]: quarters 1-3, block pair, block
        if (kq4) {
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++)
                    *reinterpret_cast<f32x4 *>(RED + ((((kq4 - 1) * 2 + bp4) * 2 + b) * ML + li) * 32 + 8 * g + 4 * h) =
                        f32x4{D[b][4 * g], D[b][4 * g + 1], D[b][4 * g + 2], D[b][4 * g + 3]} +
                        f32x4{Ds[b][4 * g], Ds[b][4 * g + 1], Ds[b][4 * g + 2], Ds[b][4 * g + 3]};
        }
        // SB0's padding columns [128, 144) to zero (it held the per-column biases)
        for (int i = tid; i < 3 * ML * 8; i += NNT)
            reinterpret_cast<uint32_t *>(&SB0->p[i / (ML * 8)][(i >> 3) % ML][128])[i & 7] = 0u;
        lds_barrier();
        if (!kq4) {
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    f32x4 o = f32x4{D[b][4 * g], D[b][4 * g + 1], D[b][4 * g + 2], D[b][4 * g + 3]} +
                              f32x4{Ds[b][4 * g], Ds[b][4 * g + 1], Ds[b][4 * g + 2], Ds[b][4 * g + 3]};
#pragma unroll
                    for (int qq = 0; qq < 3; qq++)         // K quarters 1, 2, 3 in order
                        o += *reinterpret_cast<const f32x4 *>(RED + (((qq * 2 + bp4) * 2 + b) * ML + li) * 32 + 8 * g + 4 * h);
                    const int ch = 32 * (2 * bp4 + b) + 8 * g + 4 * h;
                    uint32_t hi[2], mi[2], lo[2];          // 4 consecutive channels per plane
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const float x = fmaxf(o[i], 0.f);
                        const uint32_t hh = __float_as_uint(x) & 0xFFFF0000u;
                        const float r1 = x - __uint_as_float(hh);
                        const uint32_t mm = __float_as_uint(r1) & 0xFFFF0000u;
                        const uint32_t ll = __float_as_uint(r1 - __uint_as_float(mm)) & 0xFFFF0000u;
                        const int sh = 16 * (i & 1);
                        if (!(i & 1)) hi[i >> 1] = mi[i >> 1] = lo[i >> 1] = 0u;
                        hi[i >> 1] |= (hh >> 16) << sh;
                        mi[i >> 1] |= (mm >> 16) << sh;
                        lo[i >> 1] |= (ll >> 16) << sh;
                    }
                    *reinterpret_cast<uint2 *>(&SB0->p[0][li][ch]) = uint2{hi[0], hi[1]};
                    *reinterpret_cast<uint2 *>(&SB0->p[1][li][ch]) = uint2{mi[0], mi[1]};
                    *reinterpret_cast<uint2 *>(&SB0->p[2][li][ch]) = uint2{lo[0], lo[1]};
                }
        }
        lds_barrier();
        // SB1 / SB2's padding columns to zero (they overlay RED; partialgpool_5 reads SB1's)
        for (int i = tid; i < 2 * 3 * ML * 8; i += NNT) {
            const int b = i / (3 * ML * 8), rem = i - b * 3 * ML * 8, pl = rem / (ML * 8), rr = (rem >> 3) % ML;
            SplitAct *d = b == 0 ? SB1 : SB2;
            reinterpret_cast<uint32_t *>(&d->p[pl][rr][128])[i & 7] = 0u;
        }
    }
    // partial pool over 4 groups of 4 of x[0:16] ++ relu(Wp x[16:] + bp) (BN folded): src -> dst
    auto pool44 = [&](const SplitAct *src, SplitAct *dst, int layer, auto next) {
        const float bl = bias16(layer, w);
        float pv = 0.f;
        if (tid < ML * 8) {
            const int i = tid >> 3, j = tid & 7, g = j & 3;
            const float p0 = get_split(src, i, 4 * g), p1 = get_split(src, i, 4 * g + 1);
            const float p2 = get_split(src, i, 4 * g + 2), p3 = get_split(src, i, 4 * g + 3);
            pv = j < 4 ? fmaxf(fmaxf(p0, p1), fmaxf(p2, p3)) : (p0 + p1 + p2 + p3) / 4.f;
        }
        gemm_leaf<1, 2, 4>(W + Nt::soff(layer), w, 8, ring1, split_fetch(src, 16), a16, next);
        if (tid < ML * 8) put_split(dst, tid >> 3, tid & 7, pv);
        store_split(0, w, dst, 8, 120, [&](float x) { return fmaxf(x + bl, 0.f); });
        lds_barrier();
    };
    auto dense128 = [&](const SplitAct *src, SplitAct *dst, int layer, auto next) {
        const float bl = bias16(layer, w);
        gemm_leaf<1, 2, 4>(W + Nt::soff(layer), w, 8, ring1, split_fetch(src, 0), a16, next);
        store_split(0, w, dst, 0, 128, [&](float x) { return fmaxf(x + bl, 0.f); });
        lds_barrier();
    };
    auto ringn = [&](int layer) { return [&, layer] { ringl_load<4>(W + Nt::soff(layer), w, 8, 8, ring1); }; };
    NPROBE(5)
    pool44(SB0, SB1, 5, ringn(6));          // partialgpool_4
    dense128(SB1, SB2, 6, ringn(7));        // dense1d_5[0] (+BN folded)
    dense128(SB2, SB1, 7, ringn(8));        // dense1d_5[3]
    pool44(SB1, SB0, 8, ringn(9));          // partialgpool_5 -> trunk output in SB0
    NPROBE(6)
    // ---- heads: PI[0] -> SB1, V[0] -> SB2 (no activation); wave w: column tile w of both
    constexpr int CT = ntiles16(ACT);      // PI[1] column tiles
    static_assert(CT > 24 && CT <= 32, "PI[1] tiles: 3 or 4 per wave");
    RingL<4, 1> ring4;
    {
        const float bp = bias16(9, w), bv = bias16(11, w);
        gemm_leaf<1, 2, 4>(W + Nt::soff(9), w, 8, ring1, split_fetch(SB0, 0), a16, ringn(11));
        gemm_leaf<1, 2, 4>(W + Nt::soff(11), w, 8, ring1, split_fetch(SB0, 0), a16 + 1,
                           [&] { ringl_load<4>(W + Nt::soff(10), w, 8, CT, ring4); });
        store_split(0, w, SB1, 0, 128, [&](float x) { return x + bp; });
        store_split(1, w, SB2, 0, 128, [&](float x) { return x + bv; });
        lds_barrier();
    }
    NPROBE(7)
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
                if (j < nc) {
                    const int c = 16 * (w + 8 * j) + acc16_col();
#pragma unroll
                    for (int t = 0; t < 2; t++)
#pragma unroll
                        for (int r = 0; r < 4; r++) logits[(16 * t + acc16_row(r)) * LS + c] = a16[j][t][r] + bp[j];
                }
        };
        if (w + 24 < CT) {
            gemm_leaf<4, 2, 4>(W + Nt::soff(10), w, 8, ring4, split_fetch(SB1, 0), a16, NoNext());
            store_logits(4);
        } else if (w != 7) {
            gemm_leaf<3, 2, 4>(W + Nt::soff(10), w, 8, ring4, split_fetch(SB1, 0), a16, NoNext());
            store_logits(3);
        } else {
            gemm_leaf<3, 2, 4>(W + Nt::soff(10), w, 8, ring4, split_fetch(SB1, 0), a16,
                               [&] { ringl_load<4>(W + Nt::soff(12), 0, 1, 1, ring1); });
            store_logits(3);
            gemm_leaf<1, 2, 4>(W + Nt::soff(12), 0, 1, ring1, split_fetch(SB2, 0), a16, NoNext());
            const int n = acc16_col();
            if (n < NP) {
#pragma unroll
                for (int t = 0; t < 2; t++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int i = 16 * t + acc16_row(r);
                        if (i < nb) v_out[rowof(i) * NP + n] = tanhf(a16[0][t][r] + bv);
                    }
            }
        }
        lds_barrier();
    }
    NPROBE(8)
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
    NPROBE(9)
}

inline int check_launch() { return hipGetLastError() == hipSuccess ? 0 : SPL_EDEVICE; }

}  // namespace

extern "C" {

#if NN_PROBE
// k_nn_forward probes: wave 0's cycles summed over workgroups, [0] input staging [1] dense2d_1
// [2] dense2d_1[3] [3] partialgpool_1 [4] dense2d_3 + flatten [5] dense1d_4 [6] pgp4 .. pgp5
// [7] heads PI[0] / V[0] [8] PI[1] + V[1] [9] softmax, [15] workgroups
int spl_diag_nn_probe(unsigned long long *out16, int reset) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_nn_probe), 16 * 8) != hipSuccess) return SPL_EDEVICE;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_nn_probe), z, sizeof(z)) != hipSuccess) return SPL_EDEVICE;
    }
    return 0;
}
#endif

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
    if (!leaf_index || !leaf_count || reinterpret_cast<uintptr_t>(leaf_count) % 16) return SPL_EINVAL;
    return launch_nn(n_players, B, leaf_state, leaf_mask, packed_weights, pi, v, leaf_index, leaf_count, hs);
}

}  // extern "C"
