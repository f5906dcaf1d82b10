// mcts.hip — device-resident batched MCTS kernels + C ABI (include/splendor_amd.h §MCTS).
// One wave per tree; every tree advances by exactly one simulation per select/backup pair,
// so each tree's sequence of simulations is the reference's sequential search (MCTS.py).
#include <hip/hip_runtime.h>

#include <cmath>
#include <new>

#include "../../include/splendor_amd.h"

#ifndef MCTS_TIMING
#define MCTS_TIMING 0      // diagnostic builds only (tools/time_select.hip): k_select cycle probes
#endif
#if MCTS_TIMING
__shared__ uint64_t spl_probe_acc[24];
__shared__ uint64_t spl_probe_last;
#define SPL_PROBE(k)                                                                       \
    if (threadIdx.x == 0) {                                                                \
        const uint64_t c_ = clock64();                                                     \
        spl_probe_acc[k] += c_ - spl_probe_last;                                           \
        spl_probe_last = c_;                                                               \
    }
__device__ unsigned long long g_select_timing[24];
#endif
#include "mcts_device.h"

#ifndef SELECT_WAVES
#define SELECT_WAVES 6     // k_select waves per SIMD (80 VGPRs; 7 spills)
#endif

using namespace spl;

// Bounds-checked diagnostic builds (-DSPL_BOUNDS_CHECK=1, tools/bounds_check.sh; never the
// product): every node id and global edge index k_select / k_backup derive from the pools,
// the path and the cached links is checked against the pool sizes (and a CSR run against its
// page) before use; a violation is counted, the first one recorded (site, value, tree) and the
// value replaced by a safe one, so the run completes and reports instead of faulting.
#ifndef SPL_BOUNDS_CHECK
#define SPL_BOUNDS_CHECK 0
#endif
#if SPL_BOUNDS_CHECK
__device__ unsigned long long g_bounds[4];
__device__ __noinline__ void bounds_note(int site, long long v, int t) {
    if (atomicAdd(&g_bounds[0], 1ull) == 0) {
        g_bounds[1] = (unsigned long long)v; g_bounds[2] = (unsigned long long)site; g_bounds[3] = (unsigned long long)t;
    }
}
#define BCHK(cond, site, v, t, fix)                                   \
    do {                                                               \
        if (!(cond)) { bounds_note((site), (long long)(v), (t)); fix; } \
    } while (0)
#else
#define BCHK(cond, site, v, t, fix) \
    do {                            \
    } while (0)
#endif

struct spl_ctx {  // must match splendor_env.hip
    int n;
    int token_limit;
};

struct spl_mcts {
    int n, B, S, token_limit;
    SearchCfg cfg;
    Pools P;
    void *arena;
    size_t bytes;                        // the whole arena (spl_mcts_device_bytes)
};

namespace {

#ifndef TREE_WG
#define TREE_WG 1          // waves (trees) per workgroup of the per-tree kernels: trees finish
#endif                     // at different depths, and a 1-wave workgroup frees its slot at once
constexpr int WAVES = TREE_WG;
constexpr int THREADS = 64 * WAVES;

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int l = lane_id();
    return l ? (~0ull >> (64 - l)) : 0ull;
}

// ------------------------------------------------------------ edge selection
// pick_edge for the descent: every edge's (P, N, Q, action, child) is requested in one go
// (up to 2 x 64 edges in registers — more would cost occupancy; wider nodes loop over the
// rest), so a tree level costs one round trip for the edges; the chosen edge's action and
// child come from its lane by shuffle.
struct Pick {
    int e, a, child;
    int cec;                                    // child's cached CSR count (valid when child >= 0)
    int64_t ceb;                                // and base (global edge index)
};
__device__ __forceinline__ int64_t readlane64(int64_t x, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(uint64_t)x, l);
    const int hi = __builtin_amdgcn_readlane((int)((uint64_t)x >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
    return __longlong_as_double(readlane64(__double_as_longlong(x), l));
}

// path_x: a path level's edge offset in its node's CSR run, the run's count and the action
__device__ __forceinline__ int px_pack(int off, int ec, int a) { return off | (ec << 9) | (a << 18); }
__device__ __forceinline__ int px_off(int x) { return x & 0x1ff; }
__device__ __forceinline__ int px_count(int x) { return (x >> 9) & 0x1ff; }
__device__ __forceinline__ int px_action(int x) { return (x >> 18) & 0x1ff; }

__device__ __forceinline__ Pick pick_edge_desc(const Pools &P, const SearchCfg &C, int64_t eb, int ec,
                                               int ns, double qs, bool forced, int step, const Edge &first) {
    const int l = lane_id();
    const EdgePtr E = P.ed + eb;
    float p[2];
    int n[2], a[2], c[2];
    double q[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {               // first: edge l, already requested by the caller
        const int i = 64 * j + l;
        EdgeStat st{0.f, 0, Q_UNSET};
        EdgeLink lk{0, 0, -1};
        if (i < ec) {
            const Edge &ei = j == 0 ? first : E[i];
            st = ei.s; lk = ei.k;
        }
        p[j] = st.p; n[j] = st.n; q[j] = st.q;
        a[j] = lk.a; c[j] = lk.child;
    }
#if MCTS_TIMING
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // split load wait / compute
    SPL_PROBE(8)
#endif
    int bi = -1;
    if (forced) {                               // MCTS.py:208-213: first under-visited edge
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int i = 64 * j + l;
            const bool f = i < ec && (long long)n[j] < (long long)sqrt(0.5 * (double)p[j] * (double)step);
            const uint64_t b = __ballot(f);
            if (bi < 0 && b) bi = 64 * j + __ffsll((unsigned long long)b) - 1;
        }
        for (int base = 128; bi < 0 && base < ec; base += 64) {
            const int i = base + l;
            bool f = false;
            if (i < ec) f = (long long)E[i].s.n < (long long)sqrt(0.5 * (double)E[i].s.p * (double)step);
            const uint64_t b = __ballot(f);
            if (b) bi = base + __ffsll((unsigned long long)b) - 1;
        }
    }
    const double fpu_init = C.fpu > 0 ? qs - C.fpu : C.fpu;
    if (bi < 0 && ec <= 128) {
        // pick_highest_UCB screened in float32: each edge's UCB u (the float64 value the
        // reference computes) lies in [uf - e, uf + e] for its float32 estimate uf (relative
        // error of the estimate <= 7e-7 of |uf| + |q|; e is 3x that). With L = max(uf - e),
        // every edge that can hold the maximum has uf + e >= L; when that is one edge, it is
        // the strict-'>' arg-max and the exact float64 evaluation is skipped. Ties and near
        // ties (several candidates) fall through to the exact path below.
        const float cf = (float)C.cpuct, sqf = sqrtf((float)ns), sqef = sqrtf((float)ns + 1e-8f);
        const float ff = (float)fpu_init;
        float lo[2], hi[2];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            lo[j] = -INFINITY; hi[j] = -INFINITY;
            if (64 * j + l < ec) {
                const bool vis = q[j] != Q_UNSET;
                const float qf = vis ? (float)q[j] : ff;
                const float tf = vis ? cf * p[j] * sqf * __builtin_amdgcn_rcpf(1.f + (float)n[j]) : cf * p[j] * sqef;
                const float uf = qf + tf;
                const float e = 2.1e-6f * (fabsf(uf) + fabsf(qf)) + 1e-30f;
                lo[j] = uf - e; hi[j] = uf + e;
            }
        }
        const float L = wave_max_f32(fmaxf(lo[0], lo[1]));
        const uint64_t c0 = __ballot(hi[0] >= L), c1 = __ballot(hi[1] >= L);
        if (__popcll(c0) + __popcll(c1) == 1)
            bi = uniform(c0 ? __ffsll((unsigned long long)c0) - 1 : 64 + __ffsll((unsigned long long)c1) - 1);
    }
    if (bi < 0) {                               // pick_highest_UCB (MCTS.py:199-219)
        const double sq = sqrt((double)ns), sq_eps = sqrt((double)ns + 1e-8);
        double bu = -INFINITY, uj[2];
        int bj = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int i = 64 * j + l;
            uj[j] = -INFINITY;
            if (i < ec) {
                const double u = q[j] != Q_UNSET ? q[j] + C.cpuct * (double)p[j] * sq / (double)(1 + n[j])
                                                 : fpu_init + C.cpuct * (double)p[j] * sq_eps;
                uj[j] = u;
                if (u > bu) { bu = u; bj = i; }
            }
        }
        if (ec <= 128) {
            // strict '>' scan in action order = the lowest edge index holding the maximum:
            // DPP wave max, then the first lane of the first half that holds it
            const double m = wave_max_f64(bu);
            const uint64_t b0 = __ballot(uj[0] == m);
            bi = b0 ? __ffsll((unsigned long long)b0) - 1
                    : 64 + __ffsll((unsigned long long)__ballot(uj[1] == m)) - 1;
            bi = uniform(bi);
        }
        for (int base = 128; bi < 0 && base < ec; base += 64) {
            const int i = base + l;
            if (i < ec) {
                const double qq = E[i].s.q, pp = (double)E[i].s.p;
                const double u = qq != Q_UNSET ? qq + C.cpuct * pp * sq / (double)(1 + E[i].s.n)
                                               : fpu_init + C.cpuct * pp * sq_eps;
                if (u > bu) { bu = u; bj = i; }
            }
        }
        if (bi < 0) {
            wave_argmax(bu, bj);
            bi = bj;
        }
    }
    const int jb = bi >> 6;
    int av = a[0], cv = c[0];
#pragma unroll
    for (int j = 1; j < 2; j++)
        if (jb == j) { av = a[j]; cv = c[j]; }
    bi = uniform(bi);                           // chosen lane -> SGPRs (readlane, no LDS trip)
    av = __builtin_amdgcn_readlane(av, bi & 63);
    cv = __builtin_amdgcn_readlane(cv, bi & 63);
    if (bi >= 128) { av = E[bi].k.a; cv = E[bi].k.child; }
    return {bi, av, cv, 0, 0};                  // (the child's range: child_range)
}

// pick_highest_UCB's arg-max over a node with at most 64 edges and no forced playouts at this
// level, one edge per lane (lanes >= ec hold anything and take no part), straight-line: the
// float32 screen of pick_edge_desc with the exact float64 arg-max as the fallback. Uniform.
__device__ __forceinline__ int ucb_argmax64(const EdgeStat &e, double cpuct, double fpu, float cf, int ec, int ns,
                                            double qs) {
    const int l = lane_id();
    const bool in = l < ec;
    const double fpu_init = fpu > 0 ? qs - fpu : fpu;
    const bool vis = e.q != Q_UNSET;
    int bi;
    {
        // branch-free estimate; v_sqrt_f32 / v_rcp_f32 (1 ulp) are inside the error bound
        const float nf = (float)ns;
        const float sq = vis ? __builtin_amdgcn_sqrtf(nf) : __builtin_amdgcn_sqrtf(nf + 1e-8f);
        const float rc = vis ? __builtin_amdgcn_rcpf(1.f + (float)e.n) : 1.f;
        const float qf = vis ? (float)e.q : (float)fpu_init;
        const float uf = qf + cf * e.p * sq * rc;
        const float er = 2.1e-6f * (fabsf(uf) + fabsf(qf)) + 1e-30f;
        const float L = wave_max_f32(in ? uf - er : -INFINITY);
        const uint64_t c = __ballot(in && uf + er >= L);
        bi = __popcll(c) == 1 ? __ffsll((unsigned long long)c) - 1 : -1;
    }
    if (bi < 0) {
        const double sq = sqrt((double)ns), sq_eps = sqrt((double)ns + 1e-8);
        double u = -INFINITY;
        if (in)
            u = vis ? e.q + cpuct * (double)e.p * sq / (double)(1 + e.n)
                    : fpu_init + cpuct * (double)e.p * sq_eps;
        const double m = wave_max_f64(u);
        bi = __ffsll((unsigned long long)__ballot(u == m)) - 1;
    }
    return uniform(bi);
}

// the descent's root level in the common case (<= 64 edges, no forced playouts): the arg-max
// and the chosen edge's link by readlane. Same result as pick_edge_desc.
__device__ __forceinline__ Pick pick_edge64(const Edge &e, double cpuct, double fpu, float cf, int ec, int ns,
                                            double qs) {
    const int bi = ucb_argmax64(e.s, cpuct, fpu, cf, ec, ns, qs);
    return {bi, __builtin_amdgcn_readlane((int)e.k.a, bi), __builtin_amdgcn_readlane(e.k.child, bi), 0, 0};
}

// exact pick_highest_UCB arg-max (float64, strict '>' in edge order = lowest index holding the
// maximum) over any number of edges, the edge at offset `off` taking the statistics (on, oq)
// (just written by this wave). Uniform.
__device__ int ucb_argmax_wide(const EdgePtr E, int ec, int ns, double qs, double cpuct, double fpu, int off, int on,
                               double oq) {
    const int l = lane_id();
    const double fpu_init = fpu > 0 ? qs - fpu : fpu;
    const double sq = sqrt((double)ns), sq_eps = sqrt((double)ns + 1e-8);
    double bu = -INFINITY;
    int bj = 0x7fffffff;
    for (int base = 0; base < ec; base += 64) {
        const int i = base + l;
        if (i < ec) {
            EdgeStat e = E[i].s;
            if (i == off) { e.n = on; e.q = oq; }
            const double u = e.q != Q_UNSET ? e.q + cpuct * (double)e.p * sq / (double)(1 + e.n)
                                            : fpu_init + cpuct * (double)e.p * sq_eps;
            if (u > bu) { bu = u; bj = i; }
        }
    }
    wave_argmax(bu, bj);
    return uniform(bj);
}

// ------------------------------------------------------------ prior sums
// numpy pairwise float32 sum of the 409 staged priors (np_sum409 order), 32 lanes:
// lane = 8*block + j accumulates r_j of block `block`; blocks [0,96) [96,200) [200,304)
// [304,409); combine ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) (+ tail), then (b0+b1)+(b2+b3).
__device__ __forceinline__ float wave_np_sum409(const float *a) {
    const int l = lane_id();
    const int blk = (l >> 3) & 3, j = l & 7;
    const int off = blk == 0 ? 0 : (blk == 1 ? 96 : (blk == 2 ? 200 : 304));
    const int len = blk == 0 ? 96 : (blk == 3 ? 105 : 104);
    float r = a[off + j];
    for (int i = 8; i < len - (len % 8); i += 8) r += a[off + i + j];
    float r1 = __shfl_xor(r, 1, 64);
    float p01 = (j & 1) ? r1 + r : r + r1;            // pair sums (r0+r1) etc. on even lanes
    float p23 = __shfl_xor(p01, 2, 64);
    float q = (j & 2) ? p23 + p01 : p01 + p23;        // ((r0+r1)+(r2+r3)) on lane 0 of quad
    float q2 = __shfl_xor(q, 4, 64);
    float res = (j & 4) ? q2 + q : q + q2;            // lane j==0 holds the block result
    float blockv = __shfl(res, 8 * blk, 64);
    if (blk == 3) blockv = blockv + a[off + 104];     // 105 = 13*8 + 1 trailing element
    const float b0 = __shfl(blockv, 0, 64), b1 = __shfl(blockv, 8, 64);
    const float b2 = __shfl(blockv, 16, 64), b3 = __shfl(blockv, 24, 64);
    return (b0 + b1) + (b2 + b3);
}

// ------------------------------------------------------------ Dirichlet root noise
// softmax(Ps, T0) (MCTS.py:245-250) -> applyDirNoise (:180-186) -> normalise (:239-242) on
// the root's priors, for any number of legal actions. Types and orders as the oracle pins
// them against the reference (oracle/splendor_oracle.c or_root_noise): Ps ** (1/T0) in
// float64 (Numba's typing) summed in NumPy's pairwise order, divided and stored float32;
// the mix 0.75*P + 0.25*d in float64 stored float32; normalise in float32 pairwise order.
// The Dirichlet vector replaces the reference's unseeded Generator.dirichlet: det_gamma on
// the Philox sequence (seed, board, stream), counters 4096*i for the i-th legal action,
// normalised like numpy's dirichlet (sequential sum, times its reciprocal).
// pr: LDS scratch of 416 floats for this wave; raw: pr already holds the network's priors
// (a new root, :141-144), else the stored priors of an expanded root are used (:150-154).
__device__ void apply_root_noise(const Pools &P, const SearchCfg &C, int t, int64_t eb, int ec, uint32_t stream,
                                 float *pr, bool raw) {
    const int l = lane_id();
    const EdgePtr ede = P.ed + eb;
    const uint32_t gb = C.board_base + (uint32_t)t;
    if (!raw) {
        for (int a = l; a < 416; a += 64) pr[a] = 0.f;
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        for (int i = l; i < ec; i += 64) pr[ede[i].k.a] = ede[i].s.p;
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
    }
    if (C.dir_temp != 1.0) {
        const double e = 1.0 / C.dir_temp;
        const double s = wave_np_sum409_f64(pr, [e](float x) { return det_pow((double)x, e); });
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        for (int a = l; a < SPL_ACTIONS; a += 64) pr[a] = (float)(det_pow((double)pr[a], e) / s);
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
    }
    // Dirichlet: gammas lane-parallel, their sum sequential in action order; the gammas
    // are drawn again for the mix (deterministic) instead of being kept in registers
    double acc = 0.0;
#pragma unroll 1
    for (int j = 0; j < (ec + 63) / 64; j++) {
        const int i = 64 * j + l;
        const double g = i < ec ? det_gamma(C.dir_alpha, C.seed, gb, stream, (uint32_t)i * 4096u) : 0.0;
        const int m = min(64, ec - 64 * j);
        const int lo = __double2loint(g), hi = __double2hiint(g);
        for (int k = 0; k < m; k++)
            acc = acc + __hiloint2double(__builtin_amdgcn_readlane(hi, k), __builtin_amdgcn_readlane(lo, k));
    }
    const bool ok = acc > 0.0;
    const double inv = ok ? 1.0 / acc : 0.0;
#pragma unroll 1
    for (int j = 0; j < (ec + 63) / 64; j++) {
        const int i = 64 * j + l;
        if (i < ec) {
            const int a = ede[i].k.a;
            const double d = ok ? det_gamma(C.dir_alpha, C.seed, gb, stream, (uint32_t)i * 4096u) * inv
                                : 1.0 / (double)ec;
            pr[a] = (float)(0.75 * (double)pr[a] + 0.25 * d);
        }
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    const float nsum = wave_np_sum409(pr);
    for (int i = l; i < ec; i += 64) ede[i].s.p = pr[ede[i].k.a] / nsum;
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------ page allocation
// Pop a page from a free stack (one lane). Only k_select / k_backup pop, and no launch both
// pops and pushes, so an array stack with one atomic top is exact: a pop that finds the
// stack empty undoes its decrement.
__device__ __forceinline__ int pop_page(int32_t *stack, int32_t *top) {
    const int k = atomicSub(top, 1);
    if (k <= 0) { atomicAdd(top, 1); return -1; }
    return stack[k - 1];
}

// global id of tree t's node slot `id` (its next slot, node_count), taking a node page from
// the pool when the slot opens one; -1 when the tree is at its maximum or the pool is empty.
// Idempotent until node_count advances (a slot reserved by k_select is the one k_backup
// fills). One lane.
__device__ int node_slot(const Pools &P, TreeHdr *H, int t, int id) {
    if (id >= P.nmax) return -1;
    const int pi = id >> NPG_SHIFT;
    int32_t *tab = P.ntab + (size_t)t * P.nptab;
    if (pi >= H->npg) {
        const int pg = pop_page(P.nfree, P.alloc + 0);
        if (pg < 0) { atomicAdd(P.alloc + 2, 1); return -1; }
        tab[pi] = pg;
        P.npidx[pg] = pi;
        H->npg = pi + 1;
    }
    return tab[pi] * NPG + (id & (NPG - 1));
}

// a CSR run of ec edges for a new node (global base), from the tree's current edge page or a
// fresh one (runs never straddle pages); -1 when the tree's edge pages are at their maximum
// or the pool is empty. One lane.
__device__ int64_t edge_run(const Pools &P, TreeHdr *H, int t, int ec) {
    if (H->eleft < ec) {
        if (H->epg >= P.eptab) return -1;
        const int pg = pop_page(P.efree, P.alloc + 1);
        if (pg < 0) { atomicAdd(P.alloc + 3, 1); return -1; }
        P.etab[(size_t)t * P.eptab + H->epg] = pg;
        P.epidx[pg] = H->epg;
        H->epg += 1;
        H->enext = (int64_t)pg * EPG;
        H->eleft = EPG;
    }
    const int64_t eb = H->enext;
    H->enext = eb + ec;
    H->eleft -= ec;
    H->edge_count += ec;
    return eb;
}

// push n page ids (src[0..n)) back to a free stack, wave-collective
__device__ __forceinline__ void push_pages(int32_t *stack, int32_t *top, int cap, const int32_t *src, int n) {
    if (n <= 0) return;
    int base = 0;
    if (lane_id() == 0) base = atomicAdd(top, n);
    base = __shfl(base, 0, 64);
    for (int i = lane_id(); i < n; i += 64)
        if (base + i < cap) stack[base + i] = src[i];    // (never false: a page is pushed once)
}

// ------------------------------------------------------------ garbage collection
// Keep the root and every node whose round counter exceeds the root's: rounds strictly
// increase along every move (SplendorLogicNumba.py:287), so no other node is reachable from
// this root or any later one — an exact subset of the reference's table (which only
// evicts rounds < R-5, MCTS.py:80-85). Compacts the tree's nodes and CSR edges in place (in
// its own page order), remaps child links and their cached ranges, rebuilds the
// transposition table and returns the pages it no longer needs to the pools.
// linked = true (capacity pressure, see begin_search): keep only the root and the nodes
// reachable from it through child links, dropping nodes that only a transposition lookup
// could reach. Wave-collective; runs in k_gc (one wave per tree) with a scratch area of
// gc_ints(nmax) ints.
struct GcScr {
    int32_t *remap;     // old local -> new local (-1: dropped); prune: reachability marks first
    int32_t *nvs;       // old local -> new local edge position of its CSR run
    int32_t *cs;        // new local -> new edge position
    int32_t *cnt;       // new local -> edge count
    int32_t *inv;       // new local -> old local
    int32_t *queue;     // prune: breadth-first queue (old locals)
    int32_t *own;       // new edge position -> new local of its node (-1: page-end gap)
    int64_t *ost;       // new local -> old global edge base
};
__host__ __device__ inline size_t gc_ints(int nmax, int emax) { return 8 * (size_t)(nmax + 2) + (size_t)emax + 64; }
__device__ __forceinline__ GcScr gc_scr(int32_t *base, int nmax) {
    const size_t m = (size_t)nmax + 2;
    GcScr S;
    S.ost = reinterpret_cast<int64_t *>(base);                 // 2m ints, 8-byte aligned
    S.remap = base + 2 * m; S.nvs = S.remap + m; S.cs = S.nvs + m; S.cnt = S.cs + m;
    S.inv = S.cnt + m; S.queue = S.inv + m; S.own = S.queue + m;
    return S;
}

// mark[i] = 1 for the root (local rootl) and every node reachable from it through child
// links, 0 else (breadth-first in batches of up to 64 queued nodes, their edges 64 at a time)
__device__ void mark_linked(const Pools &P, int t, int rootl, int32_t *mark, int32_t *q) {
    const int l = lane_id();
    const int nc = P.hdr[t].node_count;
    for (int i = l; i < nc; i += 64) mark[i] = i == rootl ? 1 : 0;
    if (l == 0) q[0] = rootl;
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    int head = 0, tail = 1;
    while (head < tail) {
        const int nbt = min(64, tail - head);
        int64_t eb = 0;
        int ec = 0;
        if (l < nbt) {
            const int g = node_g(P, t, q[head + l]);
            eb = P.neb[g];
            ec = P.nterm[g] ? 0 : P.nec[g];
        }
        head += nbt;
        int incl = ec;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (l >= o) incl += y;
        }
        const int tot = __shfl(incl, 63, 64), excl = incl - ec;
        for (int c0 = 0; c0 < tot; c0 += 64) {
            const int e = c0 + l;
            int lo = 0;                                  // last lane with excl <= e
#pragma unroll
            for (int step = 32; step > 0; step >>= 1)
                if (__shfl(excl, lo + step, 64) <= e) lo += step;
            const int64_t ebo = __shfl(eb, lo, 64);
            const int exo = __shfl(excl, lo, 64);
            const int c = e < tot ? P.ed[ebo + (e - exo)].k.child : -1;
            const int cl = c >= 0 ? node_l(P, c) : -1;
            const bool fresh = cl >= 0 && atomicCAS(&mark[cl], 0, 1) == 0;
            const uint64_t bm = __ballot(fresh);
            if (fresh) q[tail + __popcll(bm & lanemask_lt())] = cl;
            tail += __popcll(bm);
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
        }
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // (HIP's uint4 struct defeats SROA)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// k_gc collects one tree per workgroup of GCT threads (block-wide scans through LDS), so a
// large tree's collection (config 4: ~40 K nodes, ~1 M edges) is spread over 8 waves
constexpr int GCT = 512, GCW8 = GCT / 64;
struct GcLds {
    int32_t wsum[GCW8];
    int32_t bc[4];
};
__device__ __forceinline__ int block_scan(int x, int &total, GcLds &L) {   // exclusive
    const int l = lane_id(), w = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (l >= o) incl += y;
    }
    if (l == 63) L.wsum[w] = incl;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < GCW8; i++) {
        const int v = L.wsum[i];
        off += i < w ? v : 0;
        tot += v;
    }
    __syncthreads();
    total = tot;
    return off + incl - x;
}
__device__ __forceinline__ int block_min(int x, GcLds &L) {
    const int l = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
    if (l == 0) L.wsum[w] = x;
    __syncthreads();
    int m = L.wsum[0];
#pragma unroll
    for (int i = 1; i < GCW8; i++) m = min(m, L.wsum[i]);
    __syncthreads();
    return m;
}

template <int CR = 4>   // edges per thread per round trip of the edge move (boards: 2 CR units)
__device__ int compact_tree(const Pools &P, int t, int root, int root_round, const GcScr &S, GcLds &L,
                            int bunits, bool linked = false) {
    const int tid = threadIdx.x;
    TreeHdr *H = P.hdr + t;
    const int nc = H->node_count;
    const int rootl = root >= 0 ? node_l(P, root) : -1;
    int32_t *remap = S.remap;
    if (linked) {
        if (tid < 64) mark_linked(P, t, rootl, remap, S.queue);
        __syncthreads();
    }
    int kept = 0;
    for (int base = 0; base < nc; base += GCT) {
        const int i = base + tid;
        bool keep = false;
        if (i < nc) keep = i == rootl || (linked ? remap[i] == 1 : P.nround[node_g(P, t, i)] > root_round);
        int tot;
        const int ex = block_scan(keep ? 1 : 0, tot, L);
        if (i < nc) remap[i] = keep ? kept + ex : -1;
        kept += tot;
    }
    __syncthreads();
    // new edge position of every kept node's CSR run: packed in local order, a run that would
    // straddle an edge page starts the next page (the nodes before the first straddler of a
    // chunk are placed, the rest retried from that page's start). Positions never exceed the
    // old ones, so the in-place moves below read every record before it is overwritten.
    int run = 0;
    for (int base = 0; base < nc; base += GCT) {
        const int i = base + tid;
        int ec = 0;
        if (i < nc && remap[i] >= 0) {
            const int g = node_g(P, t, i);
            ec = P.nterm[g] ? 0 : P.nec[g];
        }
        bool pending = ec > 0;
        int start = run;
        for (;;) {
            const int x = pending ? ec : 0;
            int tot;
            const int ex = block_scan(x, tot, L);
            const int st = run + ex;
            const bool strad = pending && (st & (EPG - 1)) + ec > EPG;
            const int f = block_min(strad ? tid : GCT, L);
            if (f == GCT) {
                if (pending) start = st;
                run += tot;
                break;
            }
            if (pending && tid < f) { start = st; pending = false; }
            if (tid == f) L.bc[0] = (st & ~(EPG - 1)) + EPG;
            __syncthreads();
            run = L.bc[0];
            __syncthreads();
        }
        if (i < nc && remap[i] >= 0) S.nvs[i] = start;
    }
    __syncthreads();
    // node records, chunk by chunk in local order (new slot <= old slot): reads, then writes
    int my_edges = 0;
    for (int base = 0; base < nc; base += GCT) {
        const int i = base + tid;
        const int ni = i < nc ? remap[i] : -1;
        uint64_t k0 = 0, k1 = 0;
        int64_t oeb = 0;
        int ec = 0, rd = 0, vs = 0;
        NodeStat nst{0.0, 0, -1, 0, -1, 0, 0, 0};
        int8_t term = 0;
        float es[4] = {0, 0, 0, 0};
        if (ni >= 0) {
            const int g = node_g(P, t, i);
            k0 = P.nkey0[g]; k1 = P.nkey1[g];
            oeb = P.neb[g]; ec = P.nec[g]; nst = P.nst[g]; rd = P.nround[g];
            term = P.nterm[g];
#pragma unroll
            for (int j = 0; j < 4; j++) es[j] = P.nes[(size_t)g * 4 + j];
            vs = S.nvs[i];
        }
        __syncthreads();
        if (ni >= 0) {
            const int ng = node_g(P, t, ni);
            const int run_ec = term ? 0 : ec;
            P.nkey0[ng] = k0; P.nkey1[ng] = k1;
            P.neb[ng] = run_ec > 0 ? edge_g(P, t, vs) : 0; P.nec[ng] = ec; P.nround[ng] = rd;
            P.nst[ng] = nst; P.nterm[ng] = term;
            S.queue[ni] = nst.bchild;                    // (the arg-max's link, remapped below)
#pragma unroll
            for (int j = 0; j < 4; j++) P.nes[(size_t)ng * 4 + j] = es[j];
            S.cs[ni] = vs; S.cnt[ni] = run_ec; S.inv[ni] = i; S.ost[ni] = oeb;
            my_edges += run_ec;
        }
    }
    int edges;
    (void)block_scan(my_edges, edges, L);
    // the cached arg-max's link (NodeStat) remapped like the edges' links below
    for (int ni = tid; ni < kept; ni += GCT) {
        const int ch = S.queue[ni];
        if (ch >= 0) {
            const int nl = remap[node_l(P, ch)];
            NodeStat *ns = P.nst + node_g(P, t, ni);
            ns->bchild = nl >= 0 ? node_g(P, t, nl) : -1;
            if (nl >= 0) ns->bceb = S.cnt[nl] > 0 ? edge_g(P, t, S.cs[nl]) : 0;
        }
    }
    // the owner of every new edge position (gaps before a page start: -1)
    for (int k = tid; k < run; k += GCT) S.own[k] = -1;
    __syncthreads();
    for (int ni = tid; ni < kept; ni += GCT) {
        const int c0 = S.cs[ni], c = S.cnt[ni];
        for (int e = 0; e < c; e++) S.own[c0 + e] = ni;
    }
    __syncthreads();
    {
        // edge records by new position k, batches of GCT x CR in increasing k (all reads
        // before the writes); child links and their cached ranges remapped
        // (EdgePool layout: per page 1,024 16-byte statistics, then 1,024 8-byte links)
        u32x4 *const e4 = reinterpret_cast<u32x4 *>(P.ed.base);
        u32x2 *const e2 = reinterpret_cast<u32x2 *>(P.ed.base);
        constexpr int64_t PU = EdgePtr::PAGE_BYTES / 16, LU = EdgePtr::PAGE_BYTES / 8;
        const auto su = [&](int64_t i) { return (i >> EPG_SHIFT) * PU + (i & (EPG - 1)); };
        const auto lu = [&](int64_t i) { return (i >> EPG_SHIFT) * LU + 2 * EPG + (i & (EPG - 1)); };
        for (int k0 = 0; k0 < run; k0 += GCT * CR) {
            u32x4 es_[CR];
            u32x2 ek_[CR];
            int nch[CR];
            bool own[CR];
#pragma unroll
            for (int r = 0; r < CR; r++) {
                const int k = k0 + GCT * r + tid;
                const int j = k < run ? S.own[k] : -1;
                own[r] = j >= 0;
                es_[r] = u32x4{0, 0, 0, 0}; ek_[r] = u32x2{0, 0xFFFFFFFFu};
                if (j >= 0) {
                    const int64_t src = S.ost[j] + (k - S.cs[j]);
                    es_[r] = e4[su(src)];
                    ek_[r] = e2[lu(src)];
                }
            }
#pragma unroll
            for (int r = 0; r < CR; r++) {
                nch[r] = -1;
                const int ch = (int)ek_[r].y;
                if (own[r] && ch >= 0) {
                    const int nl = remap[node_l(P, ch)];
                    if (nl >= 0) nch[r] = node_g(P, t, nl);
                }
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < CR; r++) {
                const int k = k0 + GCT * r + tid;
                if (own[r]) {
                    u32x2 o = ek_[r];
                    o.y = (uint32_t)nch[r];
                    const int64_t dst = edge_g(P, t, k);
                    e4[su(dst)] = es_[r];
                    e2[lu(dst)] = o;
                }
            }
            __syncthreads();
        }
    }
    if (P.nbrd) {
        // node boards (bunits 16-byte units each) of new slot nn come from old slot inv[nn]
        // (>= nn), batches in increasing unit with all reads before the writes
        u32x4 *bb = reinterpret_cast<u32x4 *>(P.nbrd);
        const int units = kept * bunits;
        constexpr int R = 2 * CR;
        for (int k0 = 0; k0 < units; k0 += GCT * R) {
            u32x4 d[R];
            size_t dst[R];
            bool mv[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int k = k0 + GCT * r + tid;
                mv[r] = false; dst[r] = 0; d[r] = u32x4{0, 0, 0, 0};
                if (k < units) {
                    const int nn = k / bunits, u = k - nn * bunits, on = S.inv[nn];
                    if (on != nn) {
                        mv[r] = true;
                        dst[r] = (size_t)node_g(P, t, nn) * bunits + u;
                        d[r] = bb[(size_t)node_g(P, t, on) * bunits + u];
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < R; r++)
                if (mv[r]) bb[dst[r]] = d[r];
            __syncthreads();
        }
    }
    // rebuild the transposition table
    int32_t *hs = P.hslot + (size_t)t * P.hcap;
    for (int i = tid; i < P.hcap; i += GCT) hs[i] = -1;
    __syncthreads();
    for (int i = tid; i < kept; i += GCT) {
        const int g = node_g(P, t, i);
        const uint64_t k0 = P.nkey0[g];
        uint32_t h = (uint32_t)(k0 ^ (k0 >> 32)) & (uint32_t)(P.hcap - 1);
        while (atomicCAS(&hs[h], -1, g) != -1) h = (h + 1) & (uint32_t)(P.hcap - 1);
    }
    // pages past the compacted tree go back to the pools
    const int npg = (kept + NPG - 1) >> NPG_SHIFT, epg = (run + EPG - 1) >> EPG_SHIFT;
    const int onpg = H->npg, oepg = H->epg;
    const int nroot = rootl >= 0 && remap[rootl] >= 0 ? node_g(P, t, remap[rootl]) : -1;
    const int eleft = epg * EPG - run;
    const int64_t enext = eleft > 0 ? edge_g(P, t, run) : 0;
    __syncthreads();
    if (tid < 64) {
        push_pages(P.nfree, P.alloc + 0, P.npages, P.ntab + (size_t)t * P.nptab + npg, onpg - npg);
        push_pages(P.efree, P.alloc + 1, P.epages, P.etab + (size_t)t * P.eptab + epg, oepg - epg);
    }
    if (tid == 0) {
        H->node_count = kept; H->edge_count = edges;
        H->npg = npg; H->epg = epg; H->eleft = eleft; H->enext = enext;
        H->live_gc = kept; H->gcs += 1;
    }
    __syncthreads();
    return nroot;
}

// does the next search fit tree t's maxima (budget nodes; 409 root edges plus edge_reserve
// per simulation, in edge positions counting the tail of the current page)
__device__ __forceinline__ bool tree_fits(const Pools &P, const SearchCfg &C, const TreeHdr *H) {
    const long long used = (long long)H->epg * EPG - H->eleft;
    return H->node_count + H->budget + 1 <= P.nmax &&
           used + SPL_ACTIONS + (long long)H->budget * C.edge_reserve <= (long long)P.eptab * EPG;
}
// every page of tree t back to the pools, empty table. Wave-collective.
__device__ void empty_tree(const Pools &P, int t) {
    TreeHdr *H = P.hdr + t;
    const int npg = H->npg, epg = H->epg;
    push_pages(P.nfree, P.alloc + 0, P.npages, P.ntab + (size_t)t * P.nptab, npg);
    push_pages(P.efree, P.alloc + 1, P.epages, P.etab + (size_t)t * P.eptab, epg);
    int32_t *hs = P.hslot + (size_t)t * P.hcap;
    if (H->node_count > 0 || npg > 0)
        for (int i = lane_id(); i < P.hcap; i += 64) hs[i] = -1;
    __builtin_amdgcn_wave_barrier();
    if (lane_id() == 0) {
        H->node_count = 0; H->edge_count = 0; H->npg = 0; H->epg = 0; H->eleft = 0; H->enext = 0;
        H->live_gc = 0;
    }
    __builtin_amdgcn_wave_barrier();
}
// queue tree t for k_gc (one lane); at most one entry per tree (gc_queued), so the queue
// of B entries cannot overflow
__device__ __forceinline__ void gc_push(const Pools &P, TreeHdr *H, int t) {
    if (H->gc_queued) return;
    H->gc_queued = 1;
    const int k = atomicAdd(&P.counters[2], 1);
    P.gcq[k] = t;
}

// ------------------------------------------------------------ search start
// Re-root tree t at the canonical board staged in LDS `s` (MCTS.getActionProb entry,
// :45-56): look the root up in the persistent table (keep) or start empty; draw the
// full/fast search decision (ST_FULL) and arm root noise. Wave-collective.
// Garbage (nodes with rounds <= the root's: unreachable, and no lookup can match them) is
// collected by k_gc, queued here:
//   must (gc_state 3): the search would not fit the tree's maxima (node slots, edge page
//     table), or the arena has no self-play commit (search-only arenas never withdraw a
//     simulation, so every search starts compacted); after compaction k_gc prunes the tree
//     to the nodes linked from the root (prunes++) and empties it if that is still too
//     large (resets++);
//   should (gc_state 5): a tree whose garbage exceeds alpha x its live size, alpha from 4
//     (pools at most half full) down to 1/8 as they fill; k_gc may defer these
//     (GC_SHOULD_CAP per launch).
// Without an event the kept table is exactly the reference's reachable table.
template <int N>
__device__ void begin_search(const Pools &P, const SearchCfg &C, int t, const int8_t *s, bool keep,
                             bool force_full) {
    using Lx = Lay<N>;
    const int l = lane_id();
    TreeHdr *H = P.hdr + t;
    wave_store_board<N>(P.root_state + (size_t)t * Lx::S, s);
    const int mv = H->move_no;
    const bool full = force_full || philox_u01(C.seed, C.board_base + t, ST_FULL | (uint32_t)mv, 0) < C.prob_full;
    const int budget = full ? C.num_sims : C.num_sims / C.ratio_full;
    int root = -1, gcs = 0;
    const int rr = (uint8_t)bt(row(s, 0), 6);
    if (keep && H->node_count > 0) {
        uint64_t k0, k1;
        wave_fingerprint<N>(s, k0, k1);
        root = hash_lookup(P, t, k0, k1);
        const int nc = H->node_count;
        const long long used = (long long)H->epg * EPG - H->eleft;
        const bool must = nc + budget + 1 > P.nmax ||
                          used + SPL_ACTIONS + (long long)budget * C.edge_reserve > (long long)P.eptab * EPG;
        // garbage allowance alpha x the live size (at the last collection): a collection
        // copies the live tree to free its garbage, so a large alpha is cheap per freed node;
        // it shrinks as the shared pools fill (free share f: alpha = 4 down to 1/8)
        const float f = fminf((float)P.alloc[0] / (float)P.npages, (float)P.alloc[1] / (float)P.epages);
        const float alpha = f >= 0.5f ? 4.f : fmaxf(0.125f, 8.f * f);
        const bool should = nc > (int)((1.f + alpha) * (float)H->live_gc) + budget + NPG;
        gcs = must || !C.selfplay ? 3 : (should ? 5 : 0);   // search-only arenas: every search
                                                           // starts compacted (no withdrawals there)
    } else {
        empty_tree(P, t);
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    const int64_t reb = root >= 0 ? P.neb[root] : 0;
    const int rec = root >= 0 ? P.nec[root] : 0;
    if (l == 0) {
        H->root = root;                                  // (a queued GC moves it)
        H->root_eb = reb;
        H->root_ec = rec;
        H->sims_done = 0;
        H->full = full;
        H->budget = budget;
        H->forced = full && C.forced_playouts;
        H->noise_pending = full && C.dirichlet;
        H->leaf_kind = LEAF_NONE;
        H->overflow = 0;
        H->gc_state = gcs;
        H->root_round = rr;
        H->move_no = mv + 1;
        if (gcs) gc_push(P, H, t);
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}

// Garbage collection queued by k_backup (a leaf did not fit mid-search: gc_state 1) and by
// search starts (3 must, 5 should), one workgroup of GCT threads per queued tree, GC_WG
// workgroups sharing the queue (a workgroup's scratch: gc_stride ints of P.gscr). Exactly
// begin_search's policy: compact (rounds > the root's), prune to the linked nodes, empty.
// Queued trees come in bursts (games start together, so trees fill up together): entries
// past GC_SHOULD_CAP that only "should" be collected are skipped this time (their search
// fits; the next search start queues them again), so no launch carries a whole burst.
constexpr int GC_WG = 256;      // one per CU
#ifndef GC_SHOULD_CAP
#define GC_SHOULD_CAP 256
#endif
template <int N>
__global__ __launch_bounds__(GCT) void k_gc(Pools P, SearchCfg C) {
    __shared__ GcLds L;
    const int tid = threadIdx.x;
    const int tail = P.counters[2];                      // no pushes while k_gc runs
    const int ftail = P.counters[5];
    if (tail == 0 && ftail == 0) return;                 // (the usual case)
    const GcScr S = gc_scr(P.gscr + (size_t)blockIdx.x * P.gc_stride, P.nmax);
    for (int k = blockIdx.x; k < tail; k += gridDim.x) {     // garbage collection
        const int t = P.gcq[k];
        TreeHdr *H = P.hdr + t;
        const int st = H->gc_state;
        int root = H->root;
        const int nst = st == 1 ? 2 : 0;
        if (st == 5 && k >= GC_SHOULD_CAP) {
            // deferred (its search fits as it is)
        } else if (st == 1) {                            // the descent then repeats
            root = compact_tree<4>(P, t, root, P.nround[root], S, L, NodeBoard<N>::UNITS);
        } else if (st == 3 || st == 5) {
            const int rr = H->root_round;
            root = compact_tree<4>(P, t, root, rr, S, L, NodeBoard<N>::UNITS);
            if (!tree_fits(P, C, H) && root >= 0) {
                root = compact_tree<4>(P, t, root, rr, S, L, NodeBoard<N>::UNITS, true);
                if (tid == 0) H->prunes += 1;
            }
            __syncthreads();
            if (!tree_fits(P, C, H)) {
                root = -1;
                if (tid < 64) empty_tree(P, t);
                if (tid == 0) H->resets += 1;
            }
        }
        __syncthreads();
        const int64_t reb = root >= 0 ? P.neb[root] : 0;
        const int rec = root >= 0 ? P.nec[root] : 0;
        if (tid == 0) {
            H->root = root;
            H->root_eb = reb;
            H->root_ec = rec;
            H->gc_state = nst;                           // (2: once per search)
            H->gc_queued = 0;
            H->depth = 0;                                // (node ids moved: no path reuse)
        }
        __syncthreads();
    }
    // finished games' example rows (k_commit): the staging rows stay untouched until the
    // tree's next commit, a later iteration
    for (int k = blockIdx.x; k < ftail; k += gridDim.x) {
        const int2 e = P.flq[k];
        const int8_t *bs = P.ex_state + (size_t)e.x * Lay<N>::S;
        int8_t *bd = P.out_state + (size_t)e.y * Lay<N>::S;
        for (int i = tid; i < Lay<N>::S; i += GCT) bd[i] = bs[i];
        const float *src = P.ex_pi + (size_t)e.x * SPL_ACTIONS;
        float *dst = P.out_pi + (size_t)e.y * SPL_ACTIONS;
        for (int i = tid; i < SPL_ACTIONS; i += GCT) dst[i] = src[i];
    }
    __syncthreads();
    if (tid == 0 && atomicAdd(&P.counters[4], 1) == (int)gridDim.x - 1) {
        P.counters[2] = 0;                               // the last workgroup out resets the queues
        P.counters[5] = 0;
        P.counters[4] = 0;
    }
}

// active (optional): trees with active[t] == 0 are left as they are, with no search budget
// (their select/backup are no-ops) — the other player's turn in an Arena game
template <int N>
__global__ __launch_bounds__(THREADS) void k_set_roots(Pools P, SearchCfg C, int B,
                                                       const int8_t *__restrict__ roots,
                                                       const uint8_t *__restrict__ active, int keep,
                                                       int force_full) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    const int w = threadIdx.x >> 6, t = blockIdx.x * WAVES + w;
    if (t >= B) return;
    if (active && !active[t]) {
        if (lane_id() == 0) {
            TreeHdr *H = P.hdr + t;
            H->budget = 0; H->sims_done = 0; H->leaf_kind = LEAF_NONE;
        }
        return;
    }
    int8_t *s = lds[w];
    wave_load_board<N>(s, roots + (size_t)t * Lx::S);
    begin_search<N>(P, C, t, s, keep != 0, force_full != 0);
}

// ------------------------------------------------------------ self-play
// New game on tree t: Board.init_game with ST_DEAL draws, player 0, fresh tree.
template <int N>
__device__ void deal_game(const Pools &P, const SearchCfg &C, int t, int8_t *b, double *ub) {
    TreeHdr *H = P.hdr + t;
    const int g = H->game_no;
    wave_philox_uniforms(ub, C.seed, C.board_base + (uint32_t)t, ST_DEAL | (uint32_t)g, 0, DEAL_DRAWS);
    wave_init_game<N>(b, ub);
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    if (lane_id() == 0) {
        H->game_no = g + 1;
        H->player = 0;
        H->episode_step = 0;
        H->n_examples = 0;
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}

template <int N>
// restart (optional): only the games with restart[t] != 0 are abandoned and re-dealt
__global__ __launch_bounds__(THREADS) void k_reset_games(Pools P, SearchCfg C, int B,
                                                         const uint8_t *__restrict__ restart) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    __shared__ double ub[WAVES][DEAL_DRAWS];
    const int w = threadIdx.x >> 6, t = blockIdx.x * WAVES + w;
    if (t >= B || (restart && !restart[t])) return;
    int8_t *b = lds[w];
    deal_game<N>(P, C, t, b, ub[w]);
    wave_store_board<N>(P.board + (size_t)t * Lx::S, b);
    begin_search<N>(P, C, t, b, false, false);
}

// policy-target pruning of MCTS.py:69-74 applied to one root edge
__device__ __forceinline__ long long pruned_count(long long c, int best, bool forced, float p, int sims) {
    if (forced) {
        if (c != best) c -= (long long)sqrt(0.5 * (double)p * (double)sims);
        if (c <= 1) c = 0;
    }
    return c;
}

// One Coach.executeEpisode iteration (Coach.py:72-100) for every tree whose search is done.
template <int N>
__global__ __launch_bounds__(THREADS) void k_commit(Pools P, SearchCfg C, int B, int lim) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][2][Lx::LS];
    __shared__ double ub[WAVES][DEAL_DRAWS];
    __shared__ double pterm[WAVES][SPL_ACTIONS];         // random_pick's per-edge terms
    __shared__ int16_t pact[WAVES][SPL_ACTIONS];
    const int w = threadIdx.x >> 6, t = blockIdx.x * WAVES + w;
    if (t >= B) return;
    const int l = lane_id();
    TreeHdr *H = P.hdr + t;
    // (a tree whose leaf did not fit waits for k_gc: its simulation was withdrawn, so its
    // search is not done)
    if (H->gc_state == 1 || H->sims_done < H->budget || H->overflow || H->root < 0) return;
    const uint32_t gb = C.board_base + (uint32_t)t;
    const int root = H->root, ec = P.nec[root];
    const bool forced = H->forced;
    const int sims = H->budget, cm = H->move_no;
    const EdgePtr ede = P.ed + P.neb[root];
    int best = 0;
    for (int i = l; i < ec; i += 64) best = max(best, ede[i].s.n);
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
    // policy counts: pruned (MCTS.py:69-74); where the reference would divide 0/0
    // (Coach.py:83 raises) fall back to raw counts, then to uniform
    int mode = forced ? 0 : 1;
    long long tot = 0;
    for (; mode < 3; mode++) {
        tot = 0;
        for (int i = l; i < ec; i += 64)
            tot += mode == 0 ? pruned_count(ede[i].s.n, best, true, ede[i].s.p, sims) : (mode == 1 ? ede[i].s.n : 1);
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (tot > 0) break;
    }
#define POLICY_COUNT(i) (mode == 0 ? pruned_count(ede[i].s.n, best, true, ede[i].s.p, sims) : (mode == 1 ? (long long)ede[i].s.n : 1ll))
    const int step = H->episode_step + 1;
    const int player = H->player;
    int8_t *s = lds[w][0], *b = lds[w][1];
    // training example (Coach.py:76-80): canonical board, player, pi, valids, q
    int nex = H->n_examples;
    if (H->full && nex < P.excap) {
        const size_t x = (size_t)t * P.excap + nex;
        wave_load_board<N>(s, P.root_state + (size_t)t * Lx::S);
        wave_store_board<N>(P.ex_state + x * Lx::S, s);
        float *pi = P.ex_pi + x * SPL_ACTIONS;
        for (int a = l; a < SPL_ACTIONS; a += 64) pi[a] = 0.f;
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        for (int i = l; i < ec; i += 64)   // getSymmetries stores pi as float32 (SplendorGame.py:59-61)
            pi[ede[i].k.a] = (float)((double)POLICY_COUNT(i) / (double)tot);
        uint64_t m[7];
        wave_valid_moves<N>(s, 0, lim, m);
        store_mask(P.ex_valid + x * 7, m);
        if (l == 0) {
            const double q0 = P.nst[root].qs;
            P.ex_player[x] = player;
            for (int i = 0; i < 4; i++)
                P.ex_q[x * 4 + i] = i == 0 ? (float)q0 : (i < N ? (float)(-q0 / (double)(N - 1)) : 0.f);
        }
        nex++;
    }
    // action = random_pick(pi, T) (Coach.py:30-33, 82-83): numpy legacy choice with p
    // (the per-edge terms lane-parallel into LDS, the order-dependent sums on lane 0)
    int action = 408;
    const double T = C.temp_threshold > 0 ? (step < C.temp_threshold ? 2.0 : 0.2) : 1.0;
    for (int i = l; i < ec; i += 64) {
        pterm[w][i] = temp_pow((double)POLICY_COUNT(i) / (double)tot, T);
        pact[w][i] = ede[i].k.a;
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    if (l == 0) {
        const double *pt = pterm[w];
        double sum = 0.0;
        for (int i = 0; i < ec; i++) sum += pt[i];
        double last = 0.0;
        for (int i = 0; i < ec; i++) last += pt[i] / sum;
        const double u = philox_u01(C.seed, gb, ST_PICK | (uint32_t)cm, 0);
        double cdf = 0.0;
        action = pact[w][ec - 1];
        for (int i = 0; i < ec; i++) {
            cdf += pt[i] / sum;
            if (cdf / last > u) { action = pact[w][i]; break; }
        }
    }
    action = __shfl(action, 0, 64);
#undef POLICY_COUNT
    // getNextState with chance (Coach.py:86), getGameEnded (:88)
    wave_load_board<N>(b, P.board + (size_t)t * Lx::S);
    Chance ch{nullptr, C.seed, gb, ST_MOVE | (uint32_t)cm, 0};
    int nxt = make_move<N>(b, action, player, false, ch);
    __builtin_amdgcn_wave_barrier();
    float r[N];
    check_end<N>(b, r);
    bool ended = false;
#pragma unroll
    for (int i = 0; i < N; i++) ended |= r[i] != 0.f;
    if (l == 0) { H->n_examples = nex; H->moves += 1; }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    if (ended) {                                            // Coach.py:89-98
        int f[N];
#pragma unroll
        for (int i = 0; i < N; i++) f[i] = get_score<N>(b, i);
        // the game's examples take queue slots [slot0, slot0 + nex) at once (those past
        // out_cap are dropped and counted); lane per example for the small columns, the
        // board and policy rows are copied by k_post (queued as (staging index, slot) pairs)
        int slot0 = 0;
        if (l == 0) slot0 = atomicAdd(&P.counters[0], nex);
        slot0 = __shfl(slot0, 0, 64);
        const int kept = max(0, min(nex, P.out_cap - slot0));
        int fq0 = 0;
        if (l == 0) {
            if (kept < nex) atomicAdd(&P.counters[1], nex - kept);
            if (kept) fq0 = atomicAdd(&P.counters[5], kept);
        }
        fq0 = __shfl(fq0, 0, 64);
        const int gno = H->game_no - 1;
        for (int j = l; j < kept; j += 64) {
            const size_t x = (size_t)t * P.excap + j;
            const size_t slot = (size_t)slot0 + j;
            const int px = P.ex_player[x];
#pragma unroll
            for (int k = 0; k < 7; k++) P.out_valid[slot * 7 + k] = P.ex_valid[x * 7 + k];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int src = (i + px) % N;
                P.out_winner[slot * 4 + i] = i < N ? r[src < N ? src : 0] : 0.f;
                P.out_scdiff[slot * 4 + i] = i < N ? f[src < N ? src : 0] - f[px < N ? px : 0] : 0;
                P.out_q[slot * 4 + i] = P.ex_q[x * 4 + i];
            }
            P.out_meta[slot * 4 + 0] = (int)gb;
            P.out_meta[slot * 4 + 1] = gno;
            P.out_meta[slot * 4 + 2] = j;
            P.out_meta[slot * 4 + 3] = px;
            P.flq[fq0 + j] = make_int2((int)x, (int)slot);
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        if (l == 0) H->games_done += 1;
        deal_game<N>(P, C, t, b, ub[w]);                        // next episode
        nxt = 0;
    } else if (l == 0) {
        H->player = nxt;
        H->episode_step = step;
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    wave_store_board<N>(P.board + (size_t)t * Lx::S, b);
    wave_roll_players<N>(s, b, nxt);                            // getCanonicalForm (:73)
    begin_search<N>(P, C, t, s, !ended, false);
}

// flat copy of `bytes` bytes (16-byte vectors when both ends allow it), grid-stride
__device__ __forceinline__ void grid_copy(void *dst, const void *src, size_t bytes) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    if (((uintptr_t)dst | (uintptr_t)src) % 16 == 0) {
        const size_t nv = bytes / 16;
        uint4 *d = (uint4 *)dst;
        const uint4 *s = (const uint4 *)src;
        for (size_t i = tid; i < nv; i += nth) d[i] = s[i];
        for (size_t i = nv * 16 + tid; i < bytes; i += nth) ((uint8_t *)dst)[i] = ((const uint8_t *)src)[i];
    } else {
        for (size_t i = tid; i < bytes; i += nth) ((uint8_t *)dst)[i] = ((const uint8_t *)src)[i];
    }
}

// the queue's first k examples into caller buffers: board / pi / valid rows are contiguous
// in both layouts (flat copies), the per-player columns go from 4 to n
__global__ void k_drain_copy(Pools P, int S, int max, int8_t *st, float *pi, uint64_t *valid,
                             float *winner, int32_t *scdiff, float *q, int32_t *meta, int n) {
    const int k = min(P.counters[0], min(max, P.out_cap));
    if (pi) grid_copy(pi, P.out_pi, (size_t)k * SPL_ACTIONS * 4);
    if (st) grid_copy(st, P.out_state, (size_t)k * S);
    if (valid) grid_copy(valid, P.out_valid, (size_t)k * 7 * 8);
    if (meta) grid_copy(meta, P.out_meta, (size_t)k * 4 * 4);
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    for (size_t i = tid; i < (size_t)k * n; i += nth) {
        const size_t e = i / (size_t)n, j = i - e * (size_t)n;
        if (winner) winner[i] = P.out_winner[e * 4 + j];
        if (scdiff) scdiff[i] = P.out_scdiff[e * 4 + j];
        if (q) q[i] = P.out_q[e * 4 + j];
    }
}

__global__ void k_drain_reset(Pools P, int max, int32_t *n_out) {
    const int c = P.counters[0];
    const int k = min(c, min(max, P.out_cap));
    if (n_out) *n_out = k;
    P.counters[1] += min(c, P.out_cap) - k;              // (k_commit counted those past out_cap)
    P.counters[0] = 0;
}

// ------------------------------------------------------------ select
template <int N>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(SELECT_WAVES))) void k_select(Pools P, SearchCfg C, int B, int lim,
                                                    int8_t *__restrict__ leaf_state,
                                                    uint64_t *__restrict__ leaf_mask,
                                                    uint8_t *__restrict__ leaf_valid,
                                                    int32_t *__restrict__ leaf_count) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    __shared__ __align__(16) float lpr[WAVES][416];         // root-noise scratch
    // trees start in P.order (deep descents first: the launch ends with its deepest descent)
    const int w = uniform(threadIdx.x >> 6), slot = blockIdx.x * WAVES + w;
    if (slot >= B) return;
    const int t = uniform(P.order[slot]);
    const int l = lane_id();
    if (slot == 0 && l < 2) P.counters[6 + l] = 0;           // k_leaf_mask's filing counters
    if (slot == 0 && l == 2 && leaf_count) *leaf_count = 0;
    TreeHdr *H = P.hdr + t;
    int8_t *s = lds[w];
    // the root board is requested together with the header (no dependency between them)
    wave_load_board<N>(s, P.root_state + (size_t)t * Lx::S);
    const int sims = H->sims_done;
    if (sims >= H->budget || H->overflow) {
        if (l == 0) { leaf_valid[t] = 0; H->leaf_kind = LEAF_NONE; }
        return;
    }
#if MCTS_TIMING
    if (threadIdx.x == 0) {
        for (int k = 0; k < 24; k++) spl_probe_acc[k] = 0;
        spl_probe_last = clock64();
    }
#endif
    int32_t *path_n = P.path_n + (size_t)t * P.pcap;
    int64_t *path_e = P.path_e + (size_t)t * P.pcap;
    int32_t *path_x = P.path_x + (size_t)t * P.pcap;
    // the previous simulation's path, first 64 levels (lane per level), requested with the header
    int ppn = -1, ppx = 0;
    int64_t ppe = 0;
    if (l < P.pcap) { ppn = path_n[l]; ppx = path_x[l]; ppe = path_e[l]; }
    SPL_PROBE(0)
    int node = H->root, depth = 0, kind = LEAF_NN;
    int miss = -1;                                       // the NN leaf's empty table slot
    uint64_t k0 = 0, k1 = 0;
    float val[4] = {0, 0, 0, 0};
    if (node < 0) {
        wave_fingerprint<N>(s, k0, k1);                  // the root itself is the leaf
    } else {
        // CSR range of the current node: the root's from the header, every child's from the
        // link cached with its parent's arg-max (NodeStat) or on the edge that led to it
        int64_t eb = H->root_eb;
        int ec = H->root_ec;
        const bool noised = sims == 0 && H->noise_pending;
        if (noised) {
            apply_root_noise(P, C, t, eb, ec, ST_DIR | (uint32_t)H->move_no, lpr[w], false);
            if (l == 0) H->noise_pending = 0;           // (a withdrawn simulation must not re-noise)
        }
        const bool forced = H->forced;
        // the root's cached arg-max holds unless its priors were just noised or forced
        // playouts make its pick depend on the simulation index (MCTS.py:208-213)
        const bool root_cache = !forced && !noised;
        // node_boards: a linked child's board is stored, so the descent follows links without
        // the in-tree transition and stages a board only where it needs one (the edge to
        // expand); `bnode` is the node whose board is in LDS (the root's, from root_state)
        const uint64_t *nbrd = reinterpret_cast<const uint64_t *>(P.nbrd);
        int bnode = node;
        // pool bases and search constants of the hot loop, set up once
        const EdgePool ed_t = P.ed;
        const NodeStat *nst_t = P.nst;
        const double cpuct = C.cpuct, fpu = C.fpu;
        const float cf = (float)C.cpuct;
        int pend = -1, pend_n = 0, pend_x = 0;               // path entry not yet stored
        int64_t pend_e = 0;
        // The previous simulation's path (this search's, same root; k_gc clears H->depth when
        // it moves nodes) is this descent's as far as its nodes' cached arg-maxes still pick
        // its edges: k_backup rewrote exactly those nodes' records, so one round trip for the
        // path and one for its nodes' records (lane per level) replace the first levels'
        // dependent loads. The descent resumes at level q = the first level whose node now
        // picks another edge (or the previous leaf's parent), with that node's record in hand.
        bool have = false;
        NodeStat hq{0.0, 0, -1, 0, -1, 0, 0, 0};
        {
            const int pd = min(H->depth, 64);
            const bool ok = sims > 0 && pd > 0 && __builtin_amdgcn_readfirstlane(ppn) == node;
            if (ok) {
                NodeStat h{0.0, 0, -1, 0, -1, 0, 0, 0};
                if (l < pd) h = nst_t[ppn];
                const bool agree = l < pd && h.best == px_off(ppx) && (l > 0 || root_cache);
                const uint64_t dis = ~__ballot(agree) & (pd < 64 ? (1ull << pd) - 1 : ~0ull);
                const int p = dis ? __ffsll((unsigned long long)dis) - 1 : pd;
                const int q = uniform(min(p, pd - 1));
                const int xq = __builtin_amdgcn_readlane(ppx, q);
                node = __builtin_amdgcn_readlane(ppn, q);
                ec = px_count(xq);
                eb = readlane64(ppe, q) - px_off(xq);
                depth = q;
                hq.qs = readlane_f64(h.qs, q);
                hq.ns = __builtin_amdgcn_readlane(h.ns, q);
                hq.best = (int16_t)__builtin_amdgcn_readlane((int)h.best, q);
                hq.ba = (int16_t)__builtin_amdgcn_readlane((int)h.ba, q);
                hq.bchild = __builtin_amdgcn_readlane(h.bchild, q);
                hq.bcec = (int16_t)__builtin_amdgcn_readlane((int)h.bcec, q);
                hq.bceb = readlane64(h.bceb, q);
                have = true;
                if (!nbrd) {
                    // no node boards: the board of the resume node is the root's with the
                    // path's moves applied (the in-tree transition, MCTS.py:227-235)
                    for (int d = 0; d < q; d++) {
                        const int a = px_action(__builtin_amdgcn_readlane(ppx, d));
                        Chance ch{nullptr, 0, 0, 0, 0};
                        int nxt;
                        switch (move_kind_of(a)) {
                            case MK_GEMS: nxt = make_move<N, MK_GEMS>(s, a, 0, true, ch); break;
                            case MK_BUY: nxt = make_move<N, MK_BUY>(s, a, 0, true, ch); break;
                            case MK_RESERVE: nxt = make_move<N, MK_RESERVE>(s, a, 0, true, ch); break;
                            default: nxt = make_move<N, MK_BUY_RESERVED>(s, a, 0, true, ch); break;
                        }
                        __builtin_amdgcn_wave_barrier();
                        if (nxt) wave_roll_players<N>(s, s, nxt);
                    }
                    bnode = node;
                }
            }
        }
        for (;;) {
            SPL_PROBE(1)
            if (depth > 0 && ec < 0) {
                kind = LEAF_TERMINAL;
#pragma unroll
                for (int i = 0; i < 4; i++) val[i] = P.nes[(size_t)node * 4 + i];
                break;
            }
            if (depth >= P.pcap) { kind = LEAF_NONE; if (l == 0) H->overflow = 2; break; }
            // below the root a level is ONE 32-byte load: the node's statistics with its cached
            // arg-max and that edge's link (NodeStat); the root's edges (first 64; lanes past
            // the range read the first edge) are requested with its statistics
#if SPL_BOUNDS_CHECK
            {
                const long long NN = (long long)P.npages * NPG, NE = (long long)P.epages * EPG;
                BCHK(node >= 0 && node < NN, 20, node, t, node = 0);
                BCHK(eb >= 0 && eb < NE && ec <= SPL_ACTIONS && (eb & (EPG - 1)) + ec <= EPG, 21, eb, t,
                     (eb = 0, ec = 0));
            }
#endif
            NodeStat nsq = hq;
            if (!have) nsq = nst_t[node];
            have = false;
            const bool use_cache = depth > 0 || root_cache;
            Edge e64{EdgeStat{0.f, 0, Q_UNSET}, EdgeLink{0, 0, -1}};
            if (!use_cache) e64 = ed_t[eb + (l < ec ? l : 0)];
            // the previous level's path entry is stored behind this level's loads: vmcnt counts
            // stores too, in issue order, so a store issued first would delay the loads' wait
            if (pend >= 0 && l == 0) { path_n[pend] = pend_n; path_e[pend] = pend_e; path_x[pend] = pend_x; }
            pend = -1;
            const int cbest = uniform(nsq.best);
            Pick pk;
            if (use_cache && cbest >= 0) {
                pk = Pick{cbest, uniform(nsq.ba), uniform(nsq.bchild), uniform(nsq.bcec),
                          (int64_t)uniform64((uint64_t)nsq.bceb)};
            } else {
                if (use_cache) e64 = ed_t[eb + (l < ec ? l : 0)];   // (no cached arg-max)
                const int ns = nsq.ns;
                const double qs = nsq.qs;
                pk = ec <= 64 && !(forced && depth == 0)
                         ? pick_edge64(e64, cpuct, fpu, cf, ec, ns, qs)
                         : pick_edge_desc(P, C, eb, ec, ns, qs, forced && depth == 0, sims, e64);
                if (pk.child >= 0) {                     // a scanned level: the child's range
                    pk.ceb = (int64_t)uniform64((uint64_t)P.neb[pk.child]);
                    pk.cec = uniform(P.nterm[pk.child] ? -1 : P.nec[pk.child]);
                }
            }
            BCHK(pk.e >= 0 && pk.e < ec, 22, pk.e, t, pk.e = 0);
            BCHK(pk.child >= -1 && pk.child < (long long)P.npages * NPG, 23, pk.child, t, pk.child = -1);
            const int64_t ge = eb + pk.e;
            pend = depth; pend_n = node; pend_e = ge; pend_x = px_pack(pk.e, ec, pk.a);
            depth++;
            int child = uniform(pk.child);
            int64_t ceb = pk.ceb;
            int cec = uniform(pk.cec);
            SPL_PROBE(2)
            if (child >= 0 && nbrd) {                        // linked: no transition needed
                node = child;
                eb = ceb;
                ec = cec;
                continue;
            }
            if (bnode != node) {                             // stage this node's stored board
                const uint64_t *src = nbrd + (size_t)node * (NodeBoard<N>::BYTES / 8);
                for (int r = l; r < Lx::ROWS; r += 64) row(s, r) = src[r];
                __builtin_amdgcn_wave_barrier();
                bnode = node;
            }
            Chance ch{nullptr, 0, 0, 0, 0};
            int nxt;                                         // MCTS.py:227-235, per kind
            switch (move_kind_of(pk.a)) {                    // (uniform: a scalar branch)
                case MK_GEMS: nxt = make_move<N, MK_GEMS>(s, pk.a, 0, true, ch); break;
                case MK_BUY: nxt = make_move<N, MK_BUY>(s, pk.a, 0, true, ch); break;
                case MK_RESERVE: nxt = make_move<N, MK_RESERVE>(s, pk.a, 0, true, ch); break;
                default: nxt = make_move<N, MK_BUY_RESERVED>(s, pk.a, 0, true, ch); break;
            }
            __builtin_amdgcn_wave_barrier();
            if (nxt) wave_roll_players<N>(s, s, nxt);
            SPL_PROBE(3)
            // a link written here is copied into the node's cached arg-max when that is the edge
            // (k_backup rewrites it anyway; this keeps it exact when the simulation is withdrawn)
            const bool cached = uniform(nsq.best) == pk.e;
            if (child < 0) {
                wave_fingerprint<N>(s, k0, k1);
                k0 = uniform64(k0); k1 = uniform64(k1);
                child = uniform(hash_lookup(P, t, k0, k1, &miss));
                miss = uniform(miss);
                if (child >= 0) {                            // transposition: link + cache
                    ceb = P.neb[child];
                    cec = P.nterm[child] ? -1 : P.nec[child];
                    if (l == 0) {
                        P.ed[ge].k.child = child;
                        if (cached) {
                            P.nst[node].bchild = child; P.nst[node].bcec = (int16_t)cec; P.nst[node].bceb = ceb;
                        }
                    }
                }
            }
            SPL_PROBE(4)
            if (child >= 0) {
                node = child;
                bnode = child;
                eb = ceb;
                ec = cec;
                continue;
            }
            float es[N];
            check_end<N>(s, es);                             // MCTS.py:125
            bool any = false;
#pragma unroll
            for (int i = 0; i < N; i++) any |= es[i] != 0.f;
            if (any) {
                kind = LEAF_TERMINAL;
#pragma unroll
                for (int i = 0; i < N; i++) val[i] = es[i];
                __builtin_amdgcn_wave_barrier();
                if (l == 0) {
                    const int id = H->node_count;
                    const int g = node_slot(P, H, t, id);
                    if (g < 0) {                             // no room: back up, do not store
                        H->unexpanded += 1;
                    } else {
                        P.nkey0[g] = k0; P.nkey1[g] = k1; P.neb[g] = 0;
                        P.nec[g] = 0;
                        P.nst[g] = NodeStat{0.0, 0, -1, 0, -1, 0, 0, 0};
                        P.nround[g] = (uint8_t)bt(row(s, 0), 6); P.nterm[g] = 1;
#pragma unroll
                        for (int i = 0; i < 4; i++) P.nes[(size_t)g * 4 + i] = i < N ? es[i < N ? i : 0] : 0.f;
                        hash_insert(P, t, k0, g);
                        P.ed[ge].k.child = g;
                        if (cached) { P.nst[node].bchild = g; P.nst[node].bcec = -1; P.nst[node].bceb = 0; }
                        H->node_count = id + 1;
                    }
                }
                break;
            }
            break;                                           // new NN leaf
        }
        if (pend >= 0 && l == 0) { path_n[pend] = pend_n; path_e[pend] = pend_e; path_x[pend] = pend_x; }
    }
    __builtin_amdgcn_wave_barrier();
    SPL_PROBE(5)
    if (kind == LEAF_NN) {                                   // its mask: k_leaf_mask
        wave_store_board<N>(leaf_state + (size_t)t * Lx::S, s);
        if (P.nbrd) {                                        // the slot k_backup will insert it at
            int g = -1;
            if (l == 0) g = node_slot(P, H, t, H->node_count);
            g = __shfl(g, 0, 64);
            if (l == 0) H->leaf_slot = g;
            if (g >= 0) {
                uint64_t *dst = reinterpret_cast<uint64_t *>(P.nbrd + (size_t)g * NodeBoard<N>::BYTES);
                for (int r = l; r < Lx::ROWS; r += 64) dst[r] = row(s, r);
            }
        }
    }
    SPL_PROBE(6)
    if (l == 0) {
        H->depth = depth;
        H->leaf_kind = kind;
        H->leaf_hslot = kind == LEAF_NN ? miss : -1;
        if (!P.nbrd || kind != LEAF_NN) H->leaf_slot = -1;
        H->leaf_k0 = k0; H->leaf_k1 = k1;
        H->leaf_round = (uint8_t)bt(row(s, 0), 6);
#pragma unroll
        for (int i = 0; i < 4; i++) H->leaf_v[i] = val[i];
        leaf_valid[t] = kind == LEAF_NN;
    }
#if MCTS_TIMING
    SPL_PROBE(7)
    if (threadIdx.x == 0) {
        for (int k = 0; k < 24; k++) atomicAdd(&g_select_timing[k], (unsigned long long)spl_probe_acc[k]);
        atomicAdd(&g_select_timing[21], 1ull);
    }
#endif
}

// ------------------------------------------------------------ leaf masks
// getValidMoves(leaf, 0) (MCTS.py:136) for every NN leaf of a select, lane per leaf, 64
// leaves per workgroup: the rollout kernel's factorised predicate and mask-word phases
// (splendor_device.h lane_predicates_part / lane_mask_word_fast, exact path for boards
// outside the fast domain), then the pass bit iff nothing else is legal (:263). Replaces
// the wave-per-board mask of the descent kernel (its lanes are idle for it anyway).
// A select's launch time is set by its deepest descents (one dependent round trip per level,
// up to ~115 levels at steady state), so the next select dispatches the trees whose leaf was
// at least DEEP_FIRST deep first: k_leaf_mask files every tree into P.order (one atomic per
// 64 trees and bucket; counters [6] [7] are cleared by k_select).
#ifndef DEEP_FIRST
#define DEEP_FIRST 48
#endif
// leaf_index / leaf_count (optional): the NN leaves listed compactly (any order) for the
// indexed network kernel, one atomic per 64 leaves (the count is cleared by k_select)
template <int N>
__global__ __launch_bounds__(256) void k_leaf_mask(Pools P, int B, int lim, const int8_t *__restrict__ leaf_state,
                                                   const uint8_t *__restrict__ leaf_valid,
                                                   uint64_t *__restrict__ leaf_mask,
                                                   int32_t *__restrict__ leaf_index,
                                                   int32_t *__restrict__ leaf_count) {
    using Lx = Lay<N>;
    using Cv = Conv<N>;
    constexpr int RB = 64, ST = (Lx::ROWS % 2 ? Lx::ROWS : Lx::ROWS + 1) * 8;
    __shared__ __align__(16) int8_t lds[RB * ST];
    __shared__ uint64_t mfac[7 * 116];
    __shared__ uint64_t pf0[4][RB], pf1[RB];
    __shared__ uint32_t pcond[RB];
    __shared__ uint8_t pbad[4][RB];
    __shared__ uint64_t msk[RB][7];
    const int b0 = blockIdx.x * RB, nb = min(RB, B - b0);
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
    if (w == 3) {                                        // launch order of the next select
        const bool in = l < nb;
        const bool deep = in && P.hdr[b0 + l].depth >= DEEP_FIRST;
        const uint64_t bd = __ballot(deep), bs = __ballot(in && !deep);
        int kd = 0, ks = 0;
        if (l == 0) {
            if (bd) kd = atomicAdd(&P.counters[6], __popcll(bd));
            if (bs) ks = atomicAdd(&P.counters[7], __popcll(bs));
        }
        kd = __shfl(kd, 0, 64); ks = __shfl(ks, 0, 64);
        if (deep) P.order[kd + __popcll(bd & lanemask_lt())] = b0 + l;
        else if (in) P.order[B - 1 - (ks + __popcll(bs & lanemask_lt()))] = b0 + l;
    } else if (w == 2 && leaf_index) {                   // the NN leaves, compacted
        const bool v = l < nb && leaf_valid[b0 + l];
        const uint64_t bv = __ballot(v);
        int k = 0;
        if (l == 0 && bv) k = atomicAdd(leaf_count, __popcll(bv));
        k = __shfl(k, 0, 64);
        if (v) leaf_index[k + __popcll(bv & lanemask_lt())] = b0 + l;
    }
    for (int i = tid; i < nb * Cv::UNITS; i += 256) {
        const int b = i / Cv::UNITS, u = i - b * Cv::UNITS;
        Cv::load(lds + b * ST, leaf_state + (size_t)(b0 + b) * Lx::S, u);
    }
    for (int i = tid; i < 7 * 116; i += 256) mfac[i] = (&K_MASK_FACTORS[0][0])[i];
    lds_sync();
    if (l < nb) {                                        // predicates: part w of every leaf
        uint64_t f0, f1;
        uint32_t cc;
        bool bad;
        const int8_t *st = lds + l * ST;
        switch (w) {
            case 0: lane_predicates_part<N, 0>(st, 0, lim, f0, f1, cc, bad); break;
            case 1: lane_predicates_part<N, 1>(st, 0, lim, f0, f1, cc, bad); break;
            case 2: lane_predicates_part<N, 2>(st, 0, lim, f0, f1, cc, bad); break;
            default: lane_predicates_part<N, 3>(st, 0, lim, f0, f1, cc, bad); break;
        }
        pf0[w][l] = f0;
        if (w == 3) pf1[l] = f1;
        if (w == 2) pcond[l] = cc;
        pbad[w][l] = bad;
    }
    lds_sync();
    if (l < nb) {                                        // mask words w and w+4
        const bool bad = pbad[0][l] | pbad[1][l] | pbad[2][l] | pbad[3][l];
        if (bad) {
            const LanePred Pr = lane_predicates_exact<N>(lds + l * ST, 0, lim);
            if (w == 0) { msk[l][0] = lane_mask_word<0>(Pr); msk[l][4] = lane_mask_word<4>(Pr); }
            else if (w == 1) { msk[l][1] = lane_mask_word<1>(Pr); msk[l][5] = lane_mask_word<5>(Pr); }
            else if (w == 2) { msk[l][2] = lane_mask_word<2>(Pr); msk[l][6] = lane_mask_word<6>(Pr); }
            else { msk[l][3] = lane_mask_word<3>(Pr); }
        } else {
            const uint64_t F0 = pf0[0][l] | pf0[1][l] | pf0[2][l];
            const uint32_t Cd = pcond[l], lv = (uint32_t)pf1[l];
            if (w == 0) {
                msk[l][0] = lane_mask_word_fast<0>(Cd, F0, lv, mfac);
                msk[l][4] = lane_mask_word_fast<4>(Cd, F0, lv, mfac);
            } else if (w == 1) {
                msk[l][1] = lane_mask_word_fast<1>(Cd, F0, lv, mfac);
                msk[l][5] = lane_mask_word_fast<5>(Cd, F0, lv, mfac);
            } else if (w == 2) {
                msk[l][2] = lane_mask_word_fast<2>(Cd, F0, lv, mfac);
                msk[l][6] = lane_mask_word_fast<6>(Cd, F0, lv, mfac);
            } else {
                msk[l][3] = lane_mask_word_fast<3>(Cd, F0, lv, mfac);
            }
        }
    }
    lds_sync();
    {                                                    // pass bit, lane l < 16 of wave w
        const int b = 16 * w + l;
        if (l < 16 && b < nb) {
            int cnt = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) cnt += __popcll(msk[b][k]);
            if (!cnt) msk[b][6] |= 1ull << (408 - 384);
        }
    }
    lds_sync();
    for (int i = tid; i < nb * 7; i += 256)
        if (leaf_valid[b0 + i / 7]) leaf_mask[(size_t)b0 * 7 + i] = (&msk[0][0])[i];
}

// k_backup: expansion of the NN leaf, the path backup (MCTS.py:169-176) and every path node's
// cached arg-max (NodeStat), so the next descent through the node reads its pick instead of
// scanning. Lane per level: each lane scans its node's edges (batches of BK_BATCH requested
// together) in one pass of pick_edge_desc's float32 screen — the running maximum L of u - e
// with its edge, and the largest u + e of every other edge; that is below L exactly when one
// edge can hold the maximum, which is then the strict-'>' arg-max. Otherwise (ties, near
// ties) the wave evaluates that level exactly in float64 (ucb_argmax_wide).
#ifndef BK_BATCH
#define BK_BATCH 8
#endif
#ifndef BK_PRELOAD
#define BK_PRELOAD 0       // first batch of every level requested before the expansion
#endif
#ifndef BACKUP_WAVES
#define BACKUP_WAVES 5
#endif

// per-level view of a group of path levels after their update (lane j = level j)
struct LevelV {
    int64_t eb;       // CSR base of the level's node
    int ec, off;      // its edge count, the offset of the edge taken
    int nn, nns;      // the taken edge's and the node's new visit counts
    double nq, nqs;   // their new values
};

// lane-serial screened arg-max of one node, one batch of edges at a time: the running
// maximum L1 of u - e with its edge i1 and its u + e (H1), and the largest u + e of all other
// edges (H2). One edge can hold the maximum exactly when H2 < L1.
struct Screen {
    float L1, H1, H2, cf, ff, sqv, sqe;
    int i1;
};
__device__ __forceinline__ Screen screen_init(int ns, double qs, double cpuct, double fpu) {
    Screen S;
    S.cf = (float)cpuct;
    S.ff = (float)(fpu > 0 ? qs - fpu : fpu);
    const float nf = (float)ns;
    S.sqv = __builtin_amdgcn_sqrtf(nf);
    S.sqe = __builtin_amdgcn_sqrtf(nf + 1e-8f);
    S.L1 = -INFINITY; S.H1 = -INFINITY; S.H2 = -INFINITY;
    S.i1 = 0;
    return S;
}
// edges base .. base + BK_BATCH - 1 (those < ec) in es[]; the edge at `off` takes (on, oq)
// (just written by this wave)
__device__ __forceinline__ void screen_batch(Screen &S, const EdgeStat *es, int base, int ec, int off, int on,
                                             double oq) {
#pragma unroll
    for (int j = 0; j < BK_BATCH; j++) {
        const int i = base + j;
        if (i < ec) {
            EdgeStat st = es[j];
            if (i == off) { st.n = on; st.q = oq; }
            const bool vis = st.q != Q_UNSET;
            const float rc = vis ? __builtin_amdgcn_rcpf(1.f + (float)st.n) : 1.f;
            const float qf = vis ? (float)st.q : S.ff;
            const float uf = qf + S.cf * st.p * (vis ? S.sqv : S.sqe) * rc;
            const float er = 2.1e-6f * (fabsf(uf) + fabsf(qf)) + 1e-30f;
            const float lo = uf - er, hi = uf + er;
            if (lo > S.L1) { S.H2 = fmaxf(S.H2, S.H1); S.L1 = lo; S.H1 = hi; S.i1 = i; }
            else S.H2 = fmaxf(S.H2, hi);
        }
    }
}
__device__ __forceinline__ void batch_load(const EdgePtr E, int base, int ec, EdgeStat *es) {
#pragma unroll
    for (int j = 0; j < BK_BATCH; j++) {
        es[j] = EdgeStat{0.f, 0, Q_UNSET};
        if (base + j < ec) es[j] = E[base + j].s;
    }
}

// KINDS: the leaf kinds this launch backs up (bit 0 NN, bit 1 terminal; spl_mcts_backup_kind)
template <int N, int KINDS>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(BACKUP_WAVES))) void k_backup(Pools P, SearchCfg C, int B,
                                                    const uint64_t *__restrict__ leaf_mask,
                                                    const float *__restrict__ pi,
                                                    const float *__restrict__ v) {
    __shared__ __align__(16) float lpi[WAVES][(KINDS & 1) ? 416 : 4];
    const int w = uniform(threadIdx.x >> 6), t = blockIdx.x * WAVES + w;
    if (t >= B) return;
    const int l = lane_id();
    TreeHdr *H = P.hdr + t;
    const int32_t *path_n = P.path_n + (size_t)t * P.pcap;
    const int64_t *path_e = P.path_e + (size_t)t * P.pcap;
    const int32_t *path_x = P.path_x + (size_t)t * P.pcap;
    // every input that depends on nothing else is requested at once: the header fields, the
    // path's first 64 levels (lane per level), and for an NN leaf its mask, value and policy
    int pnode = path_n[l], px = path_x[l];               // (pcap >= 256)
    int64_t pge = path_e[l];
    const int kind = H->leaf_kind;
    if (kind == LEAF_NONE || !((KINDS >> (kind - 1)) & 1)) return;
    const int depth = H->depth;
    const int h_slot = H->leaf_slot, h_hslot = H->leaf_hslot, h_round = H->leaf_round;
    const uint64_t h_k0 = H->leaf_k0, h_k1 = H->leaf_k1;
    const int h_sims = H->sims_done, h_noise = H->noise_pending, h_gc = H->gc_state;
    const int h_eleft = H->eleft;
    const int64_t h_enext = H->enext;
    float val[4] = {0, 0, 0, 0};
    float piv[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t mw[7] = {0, 0, 0, 0, 0, 0, 0};
    if (kind == LEAF_NN) {
        const float *gp = pi + (size_t)t * SPL_ACTIONS;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            mw[k] = leaf_mask[(size_t)t * 7 + k];
            if (64 * k + l < SPL_ACTIONS) piv[k] = gp[64 * k + l];
        }
#pragma unroll
        for (int i = 0; i < N; i++) val[i] = v[(size_t)t * N + i];
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) val[i] = H->leaf_v[i];
    }
    // the first group's statistics and the first batch of every level's edges, requested
    // before the expansion (which never touches them: the new node is not on its own path)
    int cnt = min(depth, 64);
    LevelV V{0, 0, 0, 0, 0, 0.0, 0.0};
    int pcnt = 0, pns = 0;
    double pq = 0.0, pqs = 0.0;
    EdgeStat b0[BK_BATCH];
#if SPL_BOUNDS_CHECK
    const long long NN = (long long)P.npages * NPG, NE = (long long)P.epages * EPG;
#endif
    if (l < cnt) {
        V.off = px_off(px);
        V.ec = px_count(px);
        BCHK(pnode >= 0 && pnode < NN, 1, pnode, t, pnode = 0);
        BCHK(pge >= 0 && pge < NE, 2, pge, t, pge = 0);
        BCHK(V.ec >= 1 && V.ec <= SPL_ACTIONS && V.off < V.ec && pge - V.off >= 0 &&
                 ((pge - V.off) & (EPG - 1)) + V.ec <= EPG,
             3, V.ec | (V.off << 16), t, (V.ec = 1, V.off = 0, pge = 0));
        V.eb = pge - V.off;
        const EdgeStat st = P.ed[pge].s;
        pcnt = st.n; pq = st.q;
        pns = P.nst[pnode].ns; pqs = P.nst[pnode].qs;
    }
#if BK_PRELOAD
    batch_load(P.ed + V.eb, 0, l < cnt ? V.ec : 0, b0);
#endif
    int lg = -1, lec = 0;                                // the new leaf, linked to the last path edge
    int64_t leb = 0;
    if (kind == LEAF_NN) {
        int ec = 0;
#pragma unroll
        for (int k = 0; k < 7; k++) ec += __popcll(mw[k]);
        // the new node's slot (reserved by k_select with node boards) and CSR run (from the
        // tree's current edge page or a fresh one from the shared pool)
        int g = -1;
        int64_t eb = -1;
        if (l == 0) {
            g = h_slot >= 0 ? h_slot : node_slot(P, H, t, H->node_count);
            if (g >= 0) {
                if (h_eleft >= ec) {
                    eb = h_enext;
                    H->enext = eb + ec;
                    H->eleft = h_eleft - ec;
                    H->edge_count += ec;
                } else {
                    eb = edge_run(P, H, t, ec);
                }
            }
        }
        if (l == 0) {
            BCHK(g < NN, 4, g, t, g = -1);
            BCHK(eb < 0 || ((eb & (EPG - 1)) + ec <= EPG && eb + ec <= NE), 5, eb, t, eb = -1);
        }
        g = __shfl(g, 0, 64);
        eb = readlane64(eb, 0);
        if (eb < 0 && C.selfplay && depth > 0 && h_gc == 0) {
            // garbage is collected lazily (begin_search), so a self-play search may run out
            // of room with dead nodes still held: this simulation is withdrawn (no backup,
            // not counted), k_gc (launched behind every backup of a self-play arena) collects
            // the garbage (exact: nodes with rounds <= the root's) and the next select repeats
            // the same descent. Search-only arenas never withdraw.
            if (l == 0) {
                H->gc_state = 1;
                H->leaf_kind = LEAF_NONE;
                H->withdrawals += 1;
                gc_push(P, H, t);
            }
            return;
        }
        if (eb < 0) {                                    // no room: back up v, do not store
            if (l == 0) H->unexpanded += 1;
        } else {
            float *pr = lpi[w];
#pragma unroll
            for (int k = 0; k < 7; k++)
                if (64 * k + l < SPL_ACTIONS) pr[64 * k + l] = piv[k];
            __builtin_amdgcn_wave_barrier();
            const float sum = wave_np_sum409(pr);                    // normalise (MCTS.py:144)
            // the new node's arg-max: every edge unvisited (Ns = 0, Qs = v), so u = fpu_init +
            // cpuct * P * sqrt(0 + EPS) (MCTS.py:214), evaluated exactly, lowest index on ties
            const double fpu_init = C.fpu > 0 ? (double)val[0] - C.fpu : C.fpu;
            const double sq_eps = sqrt(1e-8);
            double bu = -INFINITY;
            int bj = 0x7fffffff, bact = 0;
            int run = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                const uint64_t wd = mw[k];
                if ((wd >> l) & 1) {
                    const int r = run + __popcll(wd & lanemask_lt());
                    const int a = 64 * k + l;
                    const float p = piv[k] / sum;
                    P.ed[eb + r].k.a = (int16_t)a;
                    P.ed[eb + r].s.p = p;
                    P.ed[eb + r].s.n = 0;
                    P.ed[eb + r].s.q = Q_UNSET;
                    P.ed[eb + r].k.child = -1;
                    const double u = fpu_init + C.cpuct * (double)p * sq_eps;
                    if (u > bu) { bu = u; bj = r; bact = a; }
                }
                run += __popcll(wd);
            }
            const int mine = bj;
            wave_argmax(bu, bj);
            bj = uniform(bj);
            bact = __builtin_amdgcn_readlane(bact, __ffsll((unsigned long long)__ballot(mine == bj)) - 1);
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            // the parent edge: a cross-lane read of lane depth - 1, so it is taken here, with the
            // whole wave active — inside the lane-0 branch below a spilled `pge` is reloaded for
            // lane 0 only and lane depth - 1 reads stale register contents (the round-3
            // aperture violation)
            const int64_t pe = depth > 0 ? readlane64(pge, depth - 1 < 64 ? depth - 1 : 0) : 0;
            if (l == 0) {
                P.nkey0[g] = h_k0; P.nkey1[g] = h_k1;
                P.neb[g] = eb; P.nec[g] = ec;
                // (a new root: its priors may still be noised below, and a root always scans)
                P.nst[g] = NodeStat{(double)val[0], 0, (int16_t)(depth == 0 ? -1 : bj), (int16_t)bact, -1, 0, 0, 0};
                P.nround[g] = h_round; P.nterm[g] = 0;
                if (h_hslot >= 0) P.hslot[(size_t)t * P.hcap + h_hslot] = g;   // the select's lookup ended there
                else hash_insert(P, t, h_k0, g);
                if (depth == 0) { H->root = g; H->root_eb = eb; H->root_ec = ec; }
                else {
                    int64_t pe2 = depth - 1 < 64 ? pe : path_e[depth - 1];
                    BCHK(pe2 >= 0 && pe2 < NE, 8, pe2, t, pe2 = 0);
                    P.ed[pe2].k.child = g;
                }
                H->node_count += 1;
            }
            lg = g; leb = eb; lec = ec;
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            if (depth == 0 && h_sims == 0 && h_noise)    // noise on a new root (raw priors)
                apply_root_noise(P, C, t, eb, ec, ST_DIR | (uint32_t)H->move_no, pr, true);
        }
    }
    // levels in groups of 64, lane per level (the first group's data is in hand)
    for (int g0 = 0; g0 < depth; g0 += 64) {
        const int d = g0 + l;
        if (g0 > 0) {
            cnt = min(64, depth - g0);
            V = LevelV{0, 0, 0, 0, 0, 0.0, 0.0};
            if (l < cnt) {
                pnode = path_n[d]; pge = path_e[d]; px = path_x[d];
                V.off = px_off(px);
                V.ec = px_count(px);
                BCHK(pnode >= 0 && pnode < NN, 9, pnode, t, pnode = 0);
                BCHK(pge >= 0 && pge < NE, 10, pge, t, pge = 0);
                BCHK(V.ec >= 1 && V.ec <= SPL_ACTIONS && V.off < V.ec && pge - V.off >= 0 &&
                         ((pge - V.off) & (EPG - 1)) + V.ec <= EPG,
                     11, V.ec | (V.off << 16), t, (V.ec = 1, V.off = 0, pge = 0));
                V.eb = pge - V.off;
                const EdgeStat st = P.ed[pge].s;
                pcnt = st.n; pq = st.q;
                pns = P.nst[pnode].ns; pqs = P.nst[pnode].qs;
            }
        }
#if BK_PRELOAD
        if (g0 > 0)
#endif
            batch_load(P.ed + V.eb, 0, l < cnt ? V.ec : 0, b0);
        // MCTS.py:169-176: level d sees the leaf value rolled (depth - d) times; the levels
        // touch distinct nodes/edges (rounds strictly increase along a path), so one lane per
        // level applies exactly the sequential update
        if (l < cnt) {
            const int rot = (depth - d) % N, vi = (N - rot) % N;
            float vr = val[0];
#pragma unroll
            for (int i = 1; i < N; i++) vr = vi == i ? val[i] : vr;   // (no dynamic index: scratch)
            const double v0 = (double)vr;
            V.nq = ((double)pcnt * pq + v0) / (double)(pcnt + 1);
            V.nqs = ((double)(pns + 1) * pqs + v0) / (double)(pns + 2);
            V.nn = pcnt + 1;
            V.nns = pns + 1;
            P.ed[pge].s.q = V.nq;
            P.ed[pge].s.n = V.nn;
        }
        // each level's arg-max under its new statistics: screened lane-serial scan, exact
        // float64 for the levels the screen leaves open
        int maxec = l < cnt ? V.ec : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) maxec = max(maxec, __shfl_xor(maxec, o, 64));
        maxec = uniform(maxec);
        const int lec_ = l < cnt ? V.ec : 0;
        Screen S = screen_init(V.nns, V.nqs, C.cpuct, C.fpu);
        screen_batch(S, b0, 0, lec_, V.off, V.nn, V.nq);
        for (int base = BK_BATCH; base < maxec; base += BK_BATCH) {
            EdgeStat es[BK_BATCH];
            batch_load(P.ed + V.eb, base, lec_, es);
            screen_batch(S, es, base, lec_, V.off, V.nn, V.nq);
        }
        int bsel = S.H2 < S.L1 ? S.i1 : -1;
        if (l >= cnt) bsel = 0;
        uint64_t ex = __ballot(l < cnt && bsel < 0);
        while (ex) {
            const int j = __ffsll((unsigned long long)ex) - 1;
            ex &= ex - 1;
            const int b = ucb_argmax_wide(P.ed + readlane64(V.eb, j), __builtin_amdgcn_readlane(V.ec, j),
                                          __builtin_amdgcn_readlane(V.nns, j), readlane_f64(V.nqs, j), C.cpuct, C.fpu,
                                          __builtin_amdgcn_readlane(V.off, j), __builtin_amdgcn_readlane(V.nn, j),
                                          readlane_f64(V.nq, j));
            if (l == j) bsel = b;
        }
        // the node record: statistics, arg-max, that edge's link and its child's CSR range
        // (the new leaf's, else read from the node arrays: lanes in parallel, one round trip)
        if (l < cnt) {
            BCHK(bsel >= 0 && bsel < V.ec, 6, bsel, t, bsel = 0);
            EdgeLink lk = P.ed[V.eb + bsel].k;
            BCHK(lk.child >= -1 && lk.child < NN, 7, lk.child, t, lk.child = -1);
            int64_t cb = 0;
            int cc = 0;
            if (d == depth - 1 && lg >= 0 && bsel == V.off) {
                lk.child = lg; cc = lec; cb = leb;
            } else if (lk.child >= 0) {
                cb = P.neb[lk.child];
                cc = P.nterm[lk.child] ? -1 : P.nec[lk.child];
            }
            P.nst[pnode] = NodeStat{V.nqs, V.nns, (int16_t)bsel, lk.a, lk.child, (int16_t)cc, 0, cb};
        }
    }
    if (l == 0) {
        H->sims_done = h_sims + 1;
        H->noise_pending = 0;
        H->leaf_kind = LEAF_NONE;
        H->depth_max = max(H->depth_max, depth);         // leaf depth statistics (diagnostic)
        H->depth_sum += depth;
    }
}

// ------------------------------------------------------------ arena move
// MCTS.getActionProb(temp=0) (MCTS.py:87-92) followed by Arena's np.argmax of the one-hot:
// the best root count (after policy-target pruning when forced playouts were on, :68-74),
// ties broken uniformly (np.random.choice over bestAs) by the Philox draw
// (seed, board_base + t, ST_BEST | stream, 0) — keyed by the caller's game id and ply, so
// the choice does not depend on how games are batched onto trees.
// With every count 0 the reference ties all 409 actions, and so does this.
__global__ __launch_bounds__(THREADS) void k_pick_best(Pools P, SearchCfg C, int B,
                                                       const uint8_t *__restrict__ active,
                                                       uint32_t board_base, uint32_t stream,
                                                       int16_t *__restrict__ action) {
    const int w = threadIdx.x >> 6, t = blockIdx.x * WAVES + w;
    if (t >= B || (active && !active[t])) return;
    const int l = lane_id();
    TreeHdr *H = P.hdr + t;
    const int root = H->root;
    const double u = philox_u01(C.seed, board_base + (uint32_t)t, ST_BEST | (stream & 0xFFFFFFu), 0);
    if (root < 0) {                                      // no search ran: all counts 0
        if (l == 0) action[t] = (int16_t)(int)(u * (double)SPL_ACTIONS);
        return;
    }
    const EdgePtr E = P.ed + P.neb[root];
    const int ec = P.nec[root];
    const int sims = H->budget;
    const bool forced = H->forced;
    int best = 0;
    for (int i = l; i < ec; i += 64) best = max(best, E[i].s.n);
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
    long long top = 0;
    for (int i = l; i < ec; i += 64)
        top = max(top, pruned_count(E[i].s.n, best, forced, E[i].s.p, sims));
    for (int o = 32; o > 0; o >>= 1) top = max(top, (long long)__shfl_xor(top, o, 64));
    if (top == 0) {
        if (l == 0) action[t] = (int16_t)(int)(u * (double)SPL_ACTIONS);
        return;
    }
    int nbest = 0;
    for (int base = 0; base < ec; base += 64) {
        const int i = base + l;
        const bool hit = i < ec && pruned_count(E[i].s.n, best, forced, E[i].s.p, sims) == top;
        nbest += __popcll(__ballot(hit));
    }
    int k = (int)(u * (double)nbest);                    // k-th best in action order
    for (int base = 0; base < ec; base += 64) {
        const int i = base + l;
        const bool hit = i < ec && pruned_count(E[i].s.n, best, forced, E[i].s.p, sims) == top;
        const uint64_t b = __ballot(hit);
        const int c = __popcll(b);
        if (k < c) {
            uint64_t x = b;
            for (int j = 0; j < k; j++) x &= x - 1;
            const int pos = __ffsll((unsigned long long)x) - 1;
            if (l == 0) action[t] = E[base + pos].k.a;
            return;
        }
        k -= c;
    }
}

// ------------------------------------------------------------ results
// getActionProb tail (MCTS.py:61-97) for temp = 1: root visit counts (with policy-target
// pruning when forced playouts were on), probs, q.
__global__ __launch_bounds__(THREADS) void k_root_stats(Pools P, SearchCfg C, int B, int n,
                                                        int64_t *counts, double *qsa, double *probs,
                                                        double *q, int64_t *adjusted) {
    const int w = threadIdx.x >> 6, t = blockIdx.x * WAVES + w;
    if (t >= B) return;
    const int l = lane_id();
    TreeHdr *H = P.hdr + t;
    const int root = H->root;
    for (int a = l; a < SPL_ACTIONS; a += 64) {
        if (counts) counts[(size_t)t * SPL_ACTIONS + a] = 0;
        if (adjusted) adjusted[(size_t)t * SPL_ACTIONS + a] = 0;
        if (qsa) qsa[(size_t)t * SPL_ACTIONS + a] = Q_UNSET;
        if (probs) probs[(size_t)t * SPL_ACTIONS + a] = 0.0;
    }
    if (root < 0) return;
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    const EdgePtr E = P.ed + P.neb[root];
    const int ec = P.nec[root];
    int best = 0;
    for (int i = l; i < ec; i += 64) best = max(best, E[i].s.n);
    for (int o = 32; o > 0; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
    const int sims = H->budget;
    const bool forced = H->forced;
    long long tot = 0;
    for (int i = l; i < ec; i += 64) {
        const int a = E[i].k.a;
        const long long c = pruned_count(E[i].s.n, best, forced, E[i].s.p, sims);
        if (counts) counts[(size_t)t * SPL_ACTIONS + a] = E[i].s.n;
        if (adjusted) adjusted[(size_t)t * SPL_ACTIONS + a] = c;
        if (qsa) qsa[(size_t)t * SPL_ACTIONS + a] = E[i].s.q;
        tot += c;
    }
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    for (int i = l; i < ec; i += 64) {
        const int a = E[i].k.a;
        const long long c = pruned_count(E[i].s.n, best, forced, E[i].s.p, sims);
        if (probs) probs[(size_t)t * SPL_ACTIONS + a] = (double)c / (double)tot;
    }
    if (q && l == 0) {
        const double q0 = P.nst[root].qs;
        q[(size_t)t * n] = q0;
        for (int i = 1; i < n; i++) q[(size_t)t * n + i] = -q0 / (double)(n - 1);
    }
}

// root priors Ps as stored (MCTS.py:147/176), 409 floats per tree
__global__ __launch_bounds__(THREADS) void k_root_priors(Pools P, int B, float *ps) {
    const int w = threadIdx.x >> 6, t = blockIdx.x * WAVES + w;
    if (t >= B) return;
    const int l = lane_id();
    float *o = ps + (size_t)t * SPL_ACTIONS;
    for (int a = l; a < SPL_ACTIONS; a += 64) o[a] = 0.f;
    const int root = P.hdr[t].root;
    if (root < 0) return;
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    const EdgePtr E = P.ed + P.neb[root];
    const int ec = P.nec[root];
    for (int i = l; i < ec; i += 64) o[E[i].k.a] = E[i].s.p;
}

// leaf int8 [B,R,7] + packed mask -> float32 board and bool mask (predict, :160-161).
// The board is written TRANSPOSED, [B,7,R] (the layout SplendorNNet.forward builds at
// SplendorNNet.py:129), so the first layer is a plain row-major GEMM.
__global__ __launch_bounds__(256) void k_nn_input(int B, int R, const int8_t *__restrict__ st,
                                                  const uint64_t *__restrict__ mask,
                                                  float *__restrict__ x, uint8_t *__restrict__ valid) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t S = (size_t)7 * R, nx = (size_t)B * S, nv = (size_t)B * SPL_ACTIONS;
    if (i < nx) {                       // i indexes x[b][c][r]
        const size_t b = i / S, rem = i % S, c = rem / R, r = rem % R;
        x[i] = (float)st[b * S + r * 7 + c];
    }
    if (valid && i < nv) {
        const size_t b = i / SPL_ACTIONS, a = i % SPL_ACTIONS;
        valid[i] = (uint8_t)((mask[b * 7 + a / 64] >> (a % 64)) & 1);
    }
}

// tree sizes (spl_mcts_tree_sizes): slots in use and the live part of each tree — the root
// and the nodes whose round exceeds the root's (what garbage collection keeps), with their
// CSR edges. Diagnostic (capacity planning), one wave per tree.
__global__ __launch_bounds__(64) void k_tree_sizes(Pools P, int B, int32_t *out) {
    const int t = blockIdx.x;
    if (t >= B) return;
    const int l = lane_id();
    const TreeHdr *H = P.hdr + t;
    const int nc = H->node_count, root = H->root;
    const int rr = root >= 0 ? P.nround[root] : 1 << 30;
    int ln = 0, le = 0;
    for (int i = l; i < nc; i += 64) {
        const int g = node_g(P, t, i);
        if (g == root || P.nround[g] > rr) { ln++; le += P.nterm[g] ? 0 : P.nec[g]; }
    }
    for (int o = 32; o > 0; o >>= 1) { ln += __shfl_xor(ln, o, 64); le += __shfl_xor(le, o, 64); }
    if (l == 0) {
        out[4 * t] = nc; out[4 * t + 1] = H->edge_count;
        out[4 * t + 2] = root >= 0 ? ln : 0; out[4 * t + 3] = root >= 0 ? le : 0;
    }
}

// deterministic hash network (oracle or_fake_predict; used for search-parity tests and
// tree-only throughput runs). mode 0: priors spread over (0, 1], values in [-1, 1); mode 1
// ("peaked"): (w / max w)^256 priors and values near +-1, like the random-init SplendorNNet
// the bench runs — leaves reach the bench's depths
template <int N>
__global__ __launch_bounds__(256) void k_hash_eval(int B, const int8_t *__restrict__ st,
                                                   const uint64_t *__restrict__ mask,
                                                   float *__restrict__ pi, float *__restrict__ v, int mode) {
    const int t = blockIdx.x;
    if (t >= B) return;
    const int8_t *s = st + (size_t)t * Lay<N>::S;
    __shared__ uint64_t hsh;
    __shared__ double wred[4];
    if (threadIdx.x == 0) {
        uint64_t h = 0xCBF29CE484222325ull;
        for (int i = 0; i < Lay<N>::S; i++) { h ^= (uint8_t)s[i]; h *= 0x100000001B3ull; }
        hsh = h;
    }
    __syncthreads();
    const uint64_t h = hsh;
    if (mode == 1) {
        double wm = 0.0;
        for (int a = threadIdx.x; a < SPL_ACTIONS; a += 256)
            if ((mask[(size_t)t * 7 + a / 64] >> (a % 64)) & 1) wm = fmax(wm, (double)(1 + (mix64(h + (uint64_t)a) >> 40)));
        for (int o = 32; o > 0; o >>= 1) wm = fmax(wm, __shfl_xor(wm, o, 64));
        if (lane_id() == 0) wred[threadIdx.x >> 6] = wm;
        __syncthreads();
        wm = fmax(fmax(wred[0], wred[1]), fmax(wred[2], wred[3]));
        for (int a = threadIdx.x; a < SPL_ACTIONS; a += 256) {
            const bool ok = (mask[(size_t)t * 7 + a / 64] >> (a % 64)) & 1;
            double w = (double)(1 + (mix64(h + (uint64_t)a) >> 40)) / wm;
#pragma unroll
            for (int k = 0; k < 8; k++) w = w * w;
            pi[(size_t)t * SPL_ACTIONS + a] = ok ? (float)w : 0.f;
        }
        if (threadIdx.x < N)
            v[(size_t)t * N + threadIdx.x] =
                (float)((threadIdx.x == 0 ? 1.0 : -1.0) *
                        (1.0 - (double)(mix64(h ^ (0xA5A5ull + threadIdx.x)) >> 40) * 0x1p-30));
        return;
    }
    for (int a = threadIdx.x; a < SPL_ACTIONS; a += 256) {
        const bool ok = (mask[(size_t)t * 7 + a / 64] >> (a % 64)) & 1;
        pi[(size_t)t * SPL_ACTIONS + a] =
            ok ? (float)((double)(1 + (mix64(h + (uint64_t)a) >> 40)) * 0x1p-24) : 0.f;
    }
    if (threadIdx.x < N)
        v[(size_t)t * N + threadIdx.x] =
            (float)((double)(mix64(h ^ (0xA5A5ull + threadIdx.x)) >> 40) * 0x1p-23 - 1.0);
}

// free stacks = every page, allocation counters
__global__ void k_init_pools(Pools P, int B) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    for (size_t i = tid; i < (size_t)B; i += nth) P.order[i] = (int32_t)i;
    for (size_t i = tid; i < (size_t)P.npages; i += nth) P.nfree[i] = (int32_t)i;
    for (size_t i = tid; i < (size_t)P.epages; i += nth) P.efree[i] = (int32_t)i;
    if (tid == 0) { P.alloc[0] = P.npages; P.alloc[1] = P.epages; P.alloc[2] = 0; P.alloc[3] = 0; }
}

inline int check_launch() { return hipGetLastError() == hipSuccess ? 0 : SPL_EDEVICE; }
inline dim3 wave_grid(int B) { return dim3((unsigned)((B + WAVES - 1) / WAVES)); }

#define SPL_DISPATCH(n, CALL)                          \
    switch (n) {                                       \
        case 2: { constexpr int N = 2; CALL; break; }  \
        case 3: { constexpr int N = 3; CALL; break; }  \
        default: { constexpr int N = 4; CALL; break; } \
    }

template <class T>
T *carve(char *&p, size_t count) {
    T *r = reinterpret_cast<T *>(p);
    size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
    p += bytes;
    return r;
}

}  // namespace

extern "C" {

// Pool layout of spl_mcts_create (also what spl_mcts_plan_bytes reports).
struct Plan {
    int nmax, emax, hcap, pcap, nptab, eptab, S, excap, out_cap, nbb;   // nbb: bytes per node board
    long long npages, epages;
    size_t bytes;
};
static Plan plan_pools(int n, int B, const spl_mcts_config *cfg) {
    Plan L;
    L.nptab = (cfg->node_cap + NPG - 1) / NPG;
    L.eptab = (cfg->edge_cap + EPG - 1) / EPG;
    L.nmax = L.nptab * NPG; L.emax = L.eptab * EPG;
    // transposition table: power of two with load <= 0.7 at the tree's maximum
    int h = 64;
    while ((long long)h * 7 < (long long)L.nmax * 10) h <<= 1;
    L.hcap = h;
    L.pcap = cfg->num_sims + 64 > 256 ? cfg->num_sims + 64 : 256;
    L.S = 7 * (32 + 10 * n + n * n);
    L.excap = cfg->selfplay ? 62 * n + 2 : 0;
    L.out_cap = cfg->selfplay ? (cfg->out_cap > 0 ? cfg->out_cap : 4 * B) : 0;
    L.nbb = cfg->node_boards ? (8 * (32 + 10 * n + n * n) + 15) & ~15 : 0;
    const long long pn = cfg->pool_nodes > 0 ? cfg->pool_nodes : (long long)B * L.nmax;
    const long long pe = cfg->pool_edges > 0 ? cfg->pool_edges : (long long)B * L.emax;
    L.npages = (pn + NPG - 1) / NPG;
    L.epages = (pe + EPG - 1) / EPG;
    const size_t nn = (size_t)L.npages * NPG, ne = (size_t)L.epages * EPG;
    const size_t nx = (size_t)B * L.excap, no = (size_t)L.out_cap;
    const int gcw = B < GC_WG ? B : GC_WG;
    size_t bytes = 0;
    auto acc = [&](size_t b) { bytes += (b + 255) & ~size_t(255); };
    acc(sizeof(TreeHdr) * B); acc(8 * nn); acc(8 * nn); acc(8 * nn); acc(4 * nn); acc(4 * nn);
    acc(sizeof(NodeStat) * nn); acc(nn); acc(16 * nn); acc((ne / EPG) * EdgePtr::PAGE_BYTES);
    acc(4 * (size_t)B * L.nptab); acc(4 * (size_t)B * L.eptab); acc(4 * (size_t)L.npages); acc(4 * (size_t)L.epages);
    acc(4 * (size_t)L.npages); acc(4 * (size_t)L.epages); acc(64);
    acc(4 * (size_t)B * L.hcap); acc(4 * (size_t)B * L.pcap); acc(8 * (size_t)B * L.pcap); acc(4 * (size_t)B * L.pcap);
    acc(4 * (size_t)gcw * gc_ints(L.nmax, L.emax)); acc((size_t)B * L.S);
    acc((size_t)B * L.S); acc(nx * L.S); acc(4 * nx * SPL_ACTIONS); acc(16 * nx); acc(56 * nx); acc(4 * nx);
    acc(no * L.S); acc(4 * no * SPL_ACTIONS); acc(16 * no); acc(16 * no); acc(56 * no); acc(16 * no);
    acc(16 * no); acc(64); acc((size_t)L.nbb * nn); acc(4 * (size_t)B); acc(8 * no); acc(4 * (size_t)B);
    L.bytes = bytes;
    return L;
}

static bool valid_cfg(const spl_ctx *ctx, int B, const spl_mcts_config *cfg) {
    if (!(ctx && ctx->n >= 2 && ctx->n <= 4 && B > 0 && cfg && cfg->num_sims > 0 && cfg->ratio_full > 0 &&
          cfg->node_cap > 0 && cfg->edge_cap > 0 && cfg->pool_nodes >= 0 && cfg->pool_edges >= 0))
        return false;
    // global node ids are int32; page ids too
    const long long nmax = (long long)((cfg->node_cap + NPG - 1) / NPG) * NPG;
    const long long emax = (long long)((cfg->edge_cap + EPG - 1) / EPG) * EPG;
    const long long pn = cfg->pool_nodes > 0 ? cfg->pool_nodes : (long long)B * nmax;
    const long long pe = cfg->pool_edges > 0 ? cfg->pool_edges : (long long)B * emax;
    return cfg->node_cap <= (1 << 24) && cfg->edge_cap <= (1 << 28) && pn + NPG < (1LL << 31) &&
           pe / EPG + 1 < (1LL << 31);
}

#if MCTS_TIMING
// diagnostic builds only: the k_select probe accumulators (tools/select_reuse.py)
int spl_diag_select_timing(unsigned long long *out24, int reset) {
    if (hipMemcpyFromSymbol(out24, HIP_SYMBOL(g_select_timing), 24 * 8) != hipSuccess) return SPL_EDEVICE;
    if (reset) {
        unsigned long long z[24] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_select_timing), z, sizeof(z)) != hipSuccess) return SPL_EDEVICE;
    }
    return 0;
}
#endif

#if SPL_BOUNDS_CHECK
// bounds-checked builds only: [0] violations, [1] first value, [2] its site, [3] its tree
int spl_diag_bounds(unsigned long long *out4, int reset) {
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_bounds), 4 * 8) != hipSuccess) return SPL_EDEVICE;
    if (reset) {
        unsigned long long z[4] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_bounds), z, sizeof(z)) != hipSuccess) return SPL_EDEVICE;
    }
    return 0;
}
#endif

long long spl_mcts_plan_bytes(const spl_ctx *ctx, int B, const spl_mcts_config *cfg) {
    if (!valid_cfg(ctx, B, cfg)) return SPL_EINVAL;
    return (long long)plan_pools(ctx->n, B, cfg).bytes;
}

int spl_mcts_create(const spl_ctx *ctx, int B, const spl_mcts_config *cfg, spl_mcts **out) {
    if (!valid_cfg(ctx, B, cfg) || !out) return SPL_EINVAL;
    spl_mcts *m = new (std::nothrow) spl_mcts;
    if (!m) return SPL_EINVAL;
    m->n = ctx->n; m->B = B; m->S = 7 * (32 + 10 * ctx->n + ctx->n * ctx->n);
    m->token_limit = ctx->token_limit;
    SearchCfg &C = m->cfg;
    C.cpuct = cfg->cpuct; C.fpu = cfg->fpu; C.dir_alpha = cfg->dirichlet_alpha;
    C.dir_temp = cfg->dirichlet_temp > 0 ? cfg->dirichlet_temp : 1.0;
    C.prob_full = cfg->prob_full; C.num_sims = cfg->num_sims; C.ratio_full = cfg->ratio_full;
    C.forced_playouts = cfg->forced_playouts; C.dirichlet = cfg->dirichlet_alpha > 0;
    C.temp_threshold = cfg->temp_threshold; C.seed = cfg->seed; C.board_base = cfg->board_base;
    C.selfplay = cfg->selfplay;
    C.edge_reserve = 32;
    Pools &P = m->P;
    const Plan L = plan_pools(ctx->n, B, cfg);
    P.nmax = L.nmax; P.emax = L.emax; P.hcap = L.hcap; P.pcap = L.pcap;
    P.nptab = L.nptab; P.eptab = L.eptab;
    P.npages = (int)L.npages; P.epages = (int)L.epages;
    const size_t nn = (size_t)L.npages * NPG, ne = (size_t)L.epages * EPG;
    const int excap = L.excap;
    const size_t nx = (size_t)B * excap, no = (size_t)L.out_cap;
    const int gcw = B < GC_WG ? B : GC_WG;
    void *arena = nullptr;
    if (hipMalloc(&arena, L.bytes) != hipSuccess) { delete m; return SPL_EDEVICE; }
    m->arena = arena;
    m->bytes = L.bytes;
    char *p = (char *)arena;
    P.hdr = carve<TreeHdr>(p, B);
    P.nkey0 = carve<uint64_t>(p, nn); P.nkey1 = carve<uint64_t>(p, nn);
    P.neb = carve<int64_t>(p, nn); P.nec = carve<int32_t>(p, nn); P.nround = carve<int32_t>(p, nn);
    P.nst = carve<NodeStat>(p, nn); P.nterm = carve<int8_t>(p, nn);
    P.nes = carve<float>(p, 4 * nn);
    P.ed.base = carve<char>(p, (ne / EPG) * EdgePtr::PAGE_BYTES);   // EdgeStat | EdgeLink blocks per page
    P.ntab = carve<int32_t>(p, (size_t)B * P.nptab); P.etab = carve<int32_t>(p, (size_t)B * P.eptab);
    P.npidx = carve<int32_t>(p, (size_t)P.npages); P.epidx = carve<int32_t>(p, (size_t)P.epages);
    P.nfree = carve<int32_t>(p, (size_t)P.npages); P.efree = carve<int32_t>(p, (size_t)P.epages);
    P.alloc = carve<int32_t>(p, 16);
    P.hslot = carve<int32_t>(p, (size_t)B * P.hcap);
    P.path_n = carve<int32_t>(p, (size_t)B * P.pcap);
    P.path_e = carve<int64_t>(p, (size_t)B * P.pcap);
    P.path_x = carve<int32_t>(p, (size_t)B * P.pcap);
    P.gc_stride = gc_ints(P.nmax, P.eptab * EPG);
    P.gscr = carve<int32_t>(p, (size_t)gcw * P.gc_stride);
    P.root_state = carve<int8_t>(p, (size_t)B * m->S);
    P.excap = excap; P.out_cap = (int)no;
    P.board = carve<int8_t>(p, (size_t)B * m->S);
    P.ex_state = carve<int8_t>(p, nx * m->S); P.ex_pi = carve<float>(p, nx * SPL_ACTIONS);
    P.ex_q = carve<float>(p, 4 * nx); P.ex_valid = carve<uint64_t>(p, 7 * nx);
    P.ex_player = carve<int32_t>(p, nx);
    P.out_state = carve<int8_t>(p, no * m->S); P.out_pi = carve<float>(p, no * SPL_ACTIONS);
    P.out_winner = carve<float>(p, 4 * no); P.out_q = carve<float>(p, 4 * no);
    P.out_valid = carve<uint64_t>(p, 7 * no); P.out_scdiff = carve<int32_t>(p, 4 * no);
    P.out_meta = carve<int32_t>(p, 4 * no); P.counters = carve<int32_t>(p, 16);
    P.nbrd = L.nbb ? carve<int8_t>(p, (size_t)L.nbb * nn) : nullptr;
    P.gcq = carve<int32_t>(p, (size_t)B);
    P.flq = carve<int2>(p, no);
    P.order = carve<int32_t>(p, (size_t)B);
    // zero the small state (headers, counters); the pools need no initialisation (a slot
    // is written before it is read); free stacks hold every page, tables are empty
    bool ok = hipMemset(P.hdr, 0, sizeof(TreeHdr) * B) == hipSuccess &&
              hipMemset(P.counters, 0, 64) == hipSuccess &&
              hipMemset(P.hslot, 0xFF, 4 * (size_t)B * P.hcap) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_init_pools, dim3(1024), dim3(256), 0, (hipStream_t)0, P, B);
        ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess;
    }
    if (!ok) { (void)hipFree(arena); delete m; return SPL_EDEVICE; }
    *out = m;
    return 0;
}

int spl_mcts_destroy(spl_mcts *m) {
    if (!m) return 0;
    (void)hipFree(m->arena);
    delete m;
    return 0;
}

long long spl_mcts_device_bytes(const spl_mcts *m) {
    if (!m) return SPL_EINVAL;
    return (long long)m->bytes;
}

int spl_mcts_set_roots(spl_mcts *m, const int8_t *roots, int keep_tree, int force_full, void *hs) {
    return spl_mcts_set_roots_active(m, roots, nullptr, keep_tree, force_full, hs);
}

// garbage collection queued by search starts / backups (usually none; in bursts up to
// thousands of trees, GC_WG single-wave workgroups share the queue)
static void launch_gc(spl_mcts *m, hipStream_t hs) {
    const unsigned gcw = (unsigned)(m->B < GC_WG ? m->B : GC_WG);
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_gc<N>, dim3(gcw), dim3(GCT), 0, hs, m->P, m->cfg));
}

int spl_mcts_set_roots_active(spl_mcts *m, const int8_t *roots, const uint8_t *active, int keep_tree,
                              int force_full, void *hs) {
    if (!m || !roots) return SPL_EINVAL;
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_set_roots<N>, wave_grid(m->B), dim3(THREADS), 0,
                                          (hipStream_t)hs, m->P, m->cfg, m->B, roots, active, keep_tree,
                                          force_full));
    launch_gc(m, (hipStream_t)hs);
    return check_launch();
}

int spl_mcts_pick_best(spl_mcts *m, const uint8_t *active, uint32_t board_base, uint32_t stream,
                       int16_t *action, void *hs) {
    if (!m || !action || stream > 0xFFFFFFu) return SPL_EINVAL;
    hipLaunchKernelGGL(k_pick_best, wave_grid(m->B), dim3(THREADS), 0, (hipStream_t)hs, m->P, m->cfg,
                       m->B, active, board_base, stream, action);
    return check_launch();
}

static int launch_select(spl_mcts *m, int8_t *leaf_state, uint64_t *leaf_mask, uint8_t *leaf_valid,
                         int32_t *leaf_index, int32_t *leaf_count, void *hs) {
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_select<N>, wave_grid(m->B), dim3(THREADS), 0,
                                          (hipStream_t)hs, m->P, m->cfg, m->B, m->token_limit,
                                          leaf_state, leaf_mask, leaf_valid, leaf_count));
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_leaf_mask<N>, dim3((unsigned)((m->B + 63) / 64)), dim3(256), 0,
                                          (hipStream_t)hs, m->P, m->B, m->token_limit, leaf_state, leaf_valid,
                                          leaf_mask, leaf_index, leaf_count));
    return check_launch();
}

int spl_mcts_select(spl_mcts *m, int8_t *leaf_state, uint64_t *leaf_mask, uint8_t *leaf_valid,
                    void *hs) {
    if (!m || !leaf_state || !leaf_mask || !leaf_valid) return SPL_EINVAL;
    return launch_select(m, leaf_state, leaf_mask, leaf_valid, nullptr, nullptr, hs);
}

int spl_mcts_select_compact(spl_mcts *m, int8_t *leaf_state, uint64_t *leaf_mask, uint8_t *leaf_valid,
                            int32_t *leaf_index, int32_t *leaf_count, void *hs) {
    if (!m || !leaf_state || !leaf_mask || !leaf_valid || !leaf_index || !leaf_count) return SPL_EINVAL;
    return launch_select(m, leaf_state, leaf_mask, leaf_valid, leaf_index, leaf_count, hs);
}

int spl_mcts_backup_kind(spl_mcts *m, const uint64_t *leaf_mask, const float *pi, const float *v, int kinds,
                         void *hs) {
    if (!m || kinds < 1 || kinds > 3 || ((kinds & SPL_LEAF_NN) && (!leaf_mask || !pi || !v))) return SPL_EINVAL;
    if (kinds == 3) {
        SPL_DISPATCH(m->n, hipLaunchKernelGGL((k_backup<N, 3>), wave_grid(m->B), dim3(THREADS), 0,
                                              (hipStream_t)hs, m->P, m->cfg, m->B, leaf_mask, pi, v));
    } else if (kinds == SPL_LEAF_NN) {
        SPL_DISPATCH(m->n, hipLaunchKernelGGL((k_backup<N, 1>), wave_grid(m->B), dim3(THREADS), 0,
                                              (hipStream_t)hs, m->P, m->cfg, m->B, leaf_mask, pi, v));
    } else {
        SPL_DISPATCH(m->n, hipLaunchKernelGGL((k_backup<N, 2>), wave_grid(m->B), dim3(THREADS), 0,
                                              (hipStream_t)hs, m->P, m->cfg, m->B, leaf_mask, pi, v));
    }
    // trees whose simulation was withdrawn (NN leaves only)
    if (m->cfg.selfplay && (kinds & SPL_LEAF_NN)) launch_gc(m, (hipStream_t)hs);
    return check_launch();
}

int spl_mcts_backup(spl_mcts *m, const uint64_t *leaf_mask, const float *pi, const float *v,
                    void *hs) {
    if (!m || !leaf_mask || !pi || !v) return SPL_EINVAL;
    return spl_mcts_backup_kind(m, leaf_mask, pi, v, 3, hs);
}

int spl_mcts_root_stats(spl_mcts *m, int64_t *counts, double *qsa, double *probs, double *q,
                        int64_t *adjusted, void *hs) {
    if (!m) return SPL_EINVAL;
    hipLaunchKernelGGL(k_root_stats, wave_grid(m->B), dim3(THREADS), 0, (hipStream_t)hs, m->P,
                       m->cfg, m->B, m->n, counts, qsa, probs, q, adjusted);
    return check_launch();
}

int spl_mcts_root_priors(spl_mcts *m, float *ps, void *hs) {
    if (!m || !ps) return SPL_EINVAL;
    hipLaunchKernelGGL(k_root_priors, wave_grid(m->B), dim3(THREADS), 0, (hipStream_t)hs, m->P, m->B, ps);
    return check_launch();
}

int spl_mcts_reset_games(spl_mcts *m, void *hs) {
    if (!m || !m->cfg.selfplay) return SPL_EINVAL;
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_reset_games<N>, wave_grid(m->B), dim3(THREADS), 0,
                                          (hipStream_t)hs, m->P, m->cfg, m->B, nullptr));
    return check_launch();
}

int spl_mcts_restart_games(spl_mcts *m, const uint8_t *restart, void *hs) {
    if (!m || !m->cfg.selfplay || !restart) return SPL_EINVAL;
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_reset_games<N>, wave_grid(m->B), dim3(THREADS), 0,
                                          (hipStream_t)hs, m->P, m->cfg, m->B, restart));
    return check_launch();
}

int spl_mcts_commit(spl_mcts *m, void *hs) {
    if (!m || !m->cfg.selfplay) return SPL_EINVAL;
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_commit<N>, wave_grid(m->B), dim3(THREADS), 0,
                                          (hipStream_t)hs, m->P, m->cfg, m->B, m->token_limit));
    launch_gc(m, (hipStream_t)hs);                        // collections queued by the new searches
    return check_launch();
}

int spl_mcts_drain_examples(spl_mcts *m, int8_t *state, float *pi, uint64_t *valid, float *winner,
                            int32_t *scdiff, float *q, int32_t *meta, int max, int32_t *n_out,
                            void *hs) {
    if (!m || !m->cfg.selfplay || max < 0) return SPL_EINVAL;
    const size_t work = (size_t)(max < m->P.out_cap ? max : m->P.out_cap) * SPL_ACTIONS / 4;   // 16-byte pi vectors
    if (work) {
        const unsigned grid = (unsigned)((work + 255) / 256 > 8192 ? 8192 : (work + 255) / 256);
        hipLaunchKernelGGL(k_drain_copy, dim3(grid), dim3(256), 0, (hipStream_t)hs, m->P, m->S, max,
                           state, pi, valid, winner, scdiff, q, meta, m->n);
    }
    hipLaunchKernelGGL(k_drain_reset, dim3(1), dim3(1), 0, (hipStream_t)hs, m->P, max, n_out);
    return check_launch();
}

int spl_mcts_pool_state(spl_mcts *m, int32_t *out, void *hs) {
    if (!m || !out) return SPL_EINVAL;
    return hipMemcpyAsync(out, m->P.alloc, 4 * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)hs) ==
                   hipSuccess ? 0 : SPL_EDEVICE;
}

int spl_mcts_pool_pages(const spl_mcts *m, long long *out4) {
    if (!m || !out4) return SPL_EINVAL;
    out4[0] = m->P.npages; out4[1] = m->P.epages; out4[2] = NPG; out4[3] = EPG;
    return 0;
}

int spl_mcts_counters(spl_mcts *m, int32_t *out, void *hs) {
    if (!m || !out || !m->cfg.selfplay) return SPL_EINVAL;
    return hipMemcpyAsync(out, m->P.counters, 2 * sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)hs) ==
                   hipSuccess ? 0 : SPL_EDEVICE;
}

int spl_mcts_headers(spl_mcts *m, int32_t *out, void *hs) {
    if (!m || !out) return SPL_EINVAL;
    return hipMemcpyAsync(out, m->P.hdr, sizeof(TreeHdr) * m->B, hipMemcpyDeviceToDevice,
                          (hipStream_t)hs) == hipSuccess ? 0 : SPL_EDEVICE;
}

int spl_mcts_tree_sizes(spl_mcts *m, int32_t *out, void *hs) {
    if (!m || !out) return SPL_EINVAL;
    hipLaunchKernelGGL(k_tree_sizes, dim3((unsigned)m->B), dim3(64), 0, (hipStream_t)hs, m->P, m->B, out);
    return check_launch();
}

int spl_nn_input(const spl_ctx *ctx, int B, const int8_t *state, const uint64_t *mask, float *x,
                 uint8_t *valid, void *hs) {
    if (!ctx || B < 0 || (B && (!state || !x || (valid && !mask)))) return SPL_EINVAL;
    if (!B) return 0;
    const int R = 32 + 10 * ctx->n + ctx->n * ctx->n, S = 7 * R;
    const size_t tot = (size_t)B * (S > SPL_ACTIONS ? S : SPL_ACTIONS);
    hipLaunchKernelGGL(k_nn_input, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       (hipStream_t)hs, B, R, state, mask, x, valid);
    return check_launch();
}

int spl_hash_eval_mode(const spl_ctx *ctx, int B, const int8_t *state, const uint64_t *mask, float *pi,
                       float *v, int mode, void *hs) {
    if (!ctx || B < 0 || mode < 0 || mode > 1 || (B && (!state || !mask || !pi || !v))) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(ctx->n, hipLaunchKernelGGL(k_hash_eval<N>, dim3((unsigned)B), dim3(256), 0,
                                            (hipStream_t)hs, B, state, mask, pi, v, mode));
    return check_launch();
}

int spl_hash_eval(const spl_ctx *ctx, int B, const int8_t *state, const uint64_t *mask, float *pi,
                  float *v, void *hs) {
    return spl_hash_eval_mode(ctx, B, state, mask, pi, v, 0, hs);
}

}  // extern "C"
