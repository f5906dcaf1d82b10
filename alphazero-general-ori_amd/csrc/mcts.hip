// mcts.hip — device-resident batched MCTS kernels + C ABI (include/splendor_amd.h §MCTS).
// Every tree advances by exactly one simulation per select/backup pair (descent lane per
// tree, backup two trees per wave), so each tree's sequence of simulations is the
// reference's sequential search (MCTS.py).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <new>

#include "../../include/splendor_amd.h"

#include "mcts_device.h"

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
__device__ unsigned long long g_bounds[4 + 64];   // count, first (value, site, tree), per-site counts
__device__ __noinline__ void bounds_note(int site, long long v, int t) {
    atomicAdd(&g_bounds[4 + (site & 63)], 1ull);
    if (atomicAdd(&g_bounds[0], 1ull) == 0) {
        g_bounds[1] = (unsigned long long)v; g_bounds[2] = (unsigned long long)site; g_bounds[3] = (unsigned long long)t;
    }
}
#define BCHK(cond, site, v, t, fix)                                   \
    do {                                                               \
        if (!(cond)) { bounds_note((site), (long long)(v), (t)); fix; } \
    } while (0)
// is global node id g one of tree t's first `lim` node slots (its own page)
#define IN_TREE(P, t, g, lim)                                                                          \
    ((g) >= 0 && (g) < (P).npages * NPG && (P).npidx[(g) >> NPG_SHIFT] < (P).hdr[t].npg &&             \
     (P).ntab[(size_t)(t) * (P).nptab + (P).npidx[(g) >> NPG_SHIFT]] == ((g) >> NPG_SHIFT) &&          \
     node_l((P), (g)) < (lim))
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
// A pick: the edge's rank in its node's run, its action, its child (global id, -1: not linked)
// and whether that child is terminal.
struct Pick {
    int e, a, child, cterm;
};
__device__ __forceinline__ int64_t readlane64(int64_t x, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(uint64_t)x, l);
    const int hi = __builtin_amdgcn_readlane((int)((uint64_t)x >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
    return __longlong_as_double(readlane64(__double_as_longlong(x), l));
}
__device__ __forceinline__ int wave_min_i32(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
    return uniform(x);
}
__device__ __forceinline__ int wave_max_i32(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
    return uniform(x);
}

// path_x: a path level's edge: its rank in the node's run and its action
__device__ __forceinline__ int px_pack(int off, int a) { return off | (a << 9); }
__device__ __forceinline__ int px_off(int x) { return x & 0x1ff; }
__device__ __forceinline__ int px_action(int x) { return (x >> 9) & 0x1ff; }

// pick_highest_UCB's two expressions (MCTS.py:214-216) in float64, evaluated in the
// reference's order
__device__ __forceinline__ double ucb_visited(double q, int n, float p, double cpuct, double sq) {
    return q + cpuct * (double)p * sq / (double)(1 + n);
}
__device__ __forceinline__ double ucb_unvisited(float p, double cpuct, double fpu_init, double sq_eps) {
    return fpu_init + cpuct * (double)p * sq_eps;
}
__device__ __forceinline__ double fpu_base(double fpu, double qs) { return fpu > 0 ? qs - fpu : fpu; }

// exact pick_highest_UCB over a whole run (MCTS.py:199-219), wave-wide: lane per edge in
// chunks of 64, statistics from the node's visit block; the reference scans actions in order
// with a strict '>', so ties go to the lowest action. forced (a root with forced playouts,
// :208-213): the lowest action with Nsa < int(sqrt(0.5 P step)) wins outright. Uniform.
__device__ Pick scan_run(const Pools &P, const NodeRun &r, int ns, double qs, double cpuct, double fpu, bool forced,
                         int step) {
    const int l = lane_id();
    const double fpu_init = fpu_base(fpu, qs);
    const double sq = sqrt((double)ns), sq_eps = sqrt((double)ns + 1e-8);
    double bu = -INFINITY;
    int ba = 0x7fffffff, bi = 0, bc = -1;
    int fa = 0x7fffffff, fi = 0, fc = -1;
    for (int base = 0; base < r.ec; base += 64) {
        const int i = base + l;
        if (i < r.ec) {
            const EdgeP e = *P.ep(r.eb + i);
            int n = 0, c = -1;
            double q = Q_UNSET;
            if (e.vi >= 0) {
                const VisitRec v = *P.vr(r.vb + REC_UNITS * e.vi);
                n = v.n; q = v.q; c = v.child;
            }
            if (forced && (long long)n < (long long)sqrt(0.5 * (double)e.p * (double)step) && e.a < fa) {
                fa = e.a; fi = i; fc = c;
            }
            const double u = q != Q_UNSET ? ucb_visited(q, n, e.p, cpuct, sq) : ucb_unvisited(e.p, cpuct, fpu_init, sq_eps);
            if (u > bu || (u == bu && e.a < ba)) { bu = u; ba = e.a; bi = i; bc = c; }
        }
    }
    if (forced) {
        const int m = wave_min_i32(fa);
        if (m != 0x7fffffff) {
            const int ln = __ffsll((unsigned long long)__ballot(fa == m)) - 1;
            return {__builtin_amdgcn_readlane(fi, ln), m, __builtin_amdgcn_readlane(fc, ln), 0};
        }
    }
    const double mu = wave_max_f64(bu);
    const int am = wave_min_i32(bu == mu ? ba : 0x7fffffff);
    const int ln = __ffsll((unsigned long long)__ballot(bu == mu && ba == am)) - 1;
    return {__builtin_amdgcn_readlane(bi, ln), am, __builtin_amdgcn_readlane(bc, ln), 0};
}

// The best unvisited edge of a run, exactly: the candidate (lowest rank without statistics:
// the largest prior, lowest action among equal priors) unless a later unvisited edge with a
// smaller prior rounds to the same float64 u and has a lower action (strict '>' in action
// order). Walks from the candidate while u stays equal (edges of the candidate's prior are
// passed over: their actions are larger); usually one step. One lane; cand < ec.
__device__ __forceinline__ int best_unvisited(const Pools &P, int64_t eb, int ec, int cand, double cpuct,
                                              double fpu_init, double sq_eps, double &u_out, int &a_out) {
    const EdgeP c = *P.ep(eb + cand);
    const double uc = ucb_unvisited(c.p, cpuct, fpu_init, sq_eps);
    int bi = cand, ba = c.a;
    if (c.p > 0.f) {
        for (int j = cand + 1; j < ec; j++) {
            const EdgeP e = *P.ep(eb + j);
            if (e.vi >= 0 || e.p == c.p) continue;
            if (ucb_unvisited(e.p, cpuct, fpu_init, sq_eps) < uc) break;
            if (e.a < ba) { ba = e.a; bi = j; }
        }
    }
    u_out = uc;
    a_out = ba;
    return bi;
}

// The candidate fields of a node record (NodeCold cand / ca / cp / np) for a run whose edges
// before rank `from` all have visit records: cand = the first rank from `from` on without one,
// its action and prior, and np = the prior of the first unvisited edge after it with a smaller
// prior (-1: none; the runs are sorted by prior, so that is the largest smaller prior). One lane.
__device__ __forceinline__ void lane_cand(const Pools &P, int64_t eb, int ec, int from, int &cand, int &ca, float &cp,
                                          float &np) {
    cand = ec; ca = 0; cp = 0.f; np = -1.f;
    bool found = false;
    // eight edges per round trip (their loads issued together), scanned in registers
    for (int c0 = from; c0 < ec; c0 += 8) {
        EdgeP e[8];
#pragma unroll
        for (int k = 0; k < 8; k++) e[k] = c0 + k < ec ? *P.ep(eb + c0 + k) : EdgeP{0.f, 0, 0};
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (c0 + k >= ec) return;
            if (!found) {
                if (e[k].vi < 0) {
                    found = true;
                    cand = c0 + k; ca = e[k].a; cp = e[k].p;
                    if (!(cp > 0.f)) return;
                }
            } else if (e[k].vi < 0 && e[k].p != cp) {
                np = e[k].p;
                return;
            }
        }
    }
}
// the same with `cand` known, wave-collective (ranks lane-parallel); uniform results
__device__ __forceinline__ void wave_cand(const Pools &P, int64_t eb, int ec, int cand, int &ca, float &cp, float &np) {
    ca = 0; cp = 0.f; np = -1.f;
    if (cand >= ec) return;
    const EdgeP c = *P.ep(eb + cand);
    ca = uniform(c.a); cp = __int_as_float(uniform(__float_as_int(c.p)));
    float m = -1.f;
    if (cp > 0.f)
        for (int j = cand + 1 + lane_id(); j < ec; j += 64) {
            const EdgeP e = *P.ep(eb + j);
            if (e.vi < 0 && e.p < cp) m = fmaxf(m, e.p);
        }
    np = wave_max_f32(m);
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

// ------------------------------------------------------------ runs in action order
__device__ __forceinline__ void wave_lds_fence() {
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}
// the same for LDS traffic only: waits for this wave's LDS operations, not for its global stores
// (a __threadfence_block is s_waitcnt vmcnt(0): every outstanding store's acknowledgement)
__device__ __forceinline__ void wave_lds_only_fence() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
// index of action a among the legal actions `bits` (the reference's array order)
__device__ __forceinline__ int order_of(const uint64_t *bits, int a) {
    const int w = a >> 6;
    int k = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) k += j < w ? __popcll(bits[j]) : 0;
    return k + __popcll(bits[w] & ((1ull << (a & 63)) - 1));
}
// the i-th legal action (i < count)
__device__ __forceinline__ int action_at(const uint64_t *bits, int i) {
#pragma unroll 1
    for (int j = 0; j < 7; j++) {
        const int c = __popcll(bits[j]);
        if (i < c) return 64 * j + kth_bit64(bits[j], i);
        i -= c;
    }
    return 408;
}
// the legal-action set of a run into LDS bits[7]. Wave-collective.
__device__ __forceinline__ void run_bits(const Pools &P, const NodeRun &r, uint64_t *bits) {
    const int l = lane_id();
    if (l < 7) bits[l] = 0;
    wave_lds_fence();
    for (int i = l; i < r.ec; i += 64) {
        const int a = P.ep(r.eb + i)->a;
        atomicOr(reinterpret_cast<unsigned long long *>(bits + (a >> 6)), 1ull << (a & 63));
    }
    wave_lds_fence();
}

// A run written sorted by (prior descending, action ascending) from the LDS list cp / ca /
// cvi of its ec edges in ACTION order (cvi: visit record index, nullptr = none yet); visit
// records get their edge's new rank and prior. Returns the lowest rank without a visit
// record (ec: none). Wave-collective.
__device__ int write_sorted_run(const Pools &P, int64_t eb, int64_t vb, int ec, const float *cp, const int16_t *ca,
                                const int16_t *cvi) {
    int cmin = ec;
    for (int i = lane_id(); i < ec; i += 64) {
        const float pi = cp[i];
        int r = 0;
        for (int j = 0; j < ec; j++) {
            const float pj = cp[j];
            r += (pj > pi) || (pj == pi && j < i);
        }
        const int vi = cvi ? cvi[i] : -1;
        *P.ep(eb + r) = EdgeP{pi, ca[i], (int16_t)vi};
        if (vi >= 0) {
            VisitRec *R = P.vr(vb + REC_UNITS * vi);
            R->p = pi;
            R->off = (int16_t)r;
        } else {
            cmin = min(cmin, r);
        }
    }
    return wave_min_i32(cmin);
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
// pr: LDS, the priors by action (0 for illegal actions; 416 floats), replaced by the noised
// ones; bits: the legal actions (LDS), ec of them. Wave-collective.
// gbuf (optional, LDS, gcap doubles, not overlapping pr / bits): when ec <= gcap the legal
// actions' powered priors and then their gammas are kept there, in legal order, instead of
// being evaluated twice (round 6: k_commit noises the kept root of every tree in the commit
// iteration at once; the same values, so the same bits)
__device__ void root_noise_lds(const SearchCfg &C, int t, uint32_t stream, float *pr, const uint64_t *bits, int ec,
                               double *gbuf = nullptr, int gcap = 0) {
    const int l = lane_id();
    const uint32_t gb = C.board_base + (uint32_t)t;
    if (ec > gcap) gbuf = nullptr;
    if (C.dir_temp != 1.0) {
        const double e = 1.0 / C.dir_temp;
        if (gbuf) {
            for (int k = l; k < ec; k += 64) gbuf[k] = det_pow((double)pr[action_at(bits, k)], e);
            wave_lds_fence();
            // (an illegal action's prior is 0 and det_pow(0) = 0: the pairwise sum of the same
            // 409 values)
            const double s = wave_np_sum409_f64_at([&](int p) {
                return (bits[p >> 6] >> (p & 63)) & 1 ? gbuf[order_of(bits, p)] : 0.0;
            });
            for (int k = l; k < ec; k += 64) {
                const int a = action_at(bits, k);
                pr[a] = (float)(gbuf[k] / s);
            }
        } else {
            const double s = wave_np_sum409_f64(pr, [e](float x) { return det_pow((double)x, e); });
            wave_lds_fence();
            for (int a = l; a < SPL_ACTIONS; a += 64) pr[a] = (float)(det_pow((double)pr[a], e) / s);
        }
        wave_lds_fence();
    }
    // Dirichlet: gammas lane-parallel, their sum sequential in action order; without gbuf the
    // gammas are drawn again for the mix (deterministic) instead of being kept in registers
    double acc = 0.0;
#pragma unroll 1
    for (int j = 0; j < (ec + 63) / 64; j++) {
        const int i = 64 * j + l;
        const double g = i < ec ? det_gamma(C.dir_alpha, C.seed, gb, stream, (uint32_t)i * 4096u) : 0.0;
        if (gbuf && i < ec) gbuf[i] = g;
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
            const int a = action_at(bits, i);
            const double g = gbuf ? gbuf[i] : (ok ? det_gamma(C.dir_alpha, C.seed, gb, stream, (uint32_t)i * 4096u) : 0.0);
            const double d = ok ? g * inv : 1.0 / (double)ec;
            pr[a] = (float)(0.75 * (double)pr[a] + 0.25 * d);
        }
    }
    wave_lds_fence();
    const float nsum = wave_np_sum409(pr);
    for (int a = l; a < SPL_ACTIONS; a += 64)
        if ((bits[a >> 6] >> (a & 63)) & 1) pr[a] = pr[a] / nsum;
    wave_lds_fence();
}

// LDS scratch of a wave that re-sorts or stages a run (root noise, move sampling)
struct RunScr {
    uint64_t bits[7];
    float pr[416];                 // priors by action
    float cp[SPL_ACTIONS];         // the run in action order: prior, action, visit record
    int16_t ca[SPL_ACTIONS];
    int16_t cvi[SPL_ACTIONS];
};

// root noise on an expanded root (MCTS.py:150-154, the stored priors): its run re-noised,
// re-sorted, its visit records' priors and ranks updated; returns the new candidate rank.
// LDS scratch: bits[7], pr[416], cp / ca / cvi [409]. Wave-collective.
// gbuf / gcap: root_noise_lds's scratch; callers pass cp (written only after it)
__device__ int noise_kept_root(const Pools &P, const SearchCfg &C, int t, const NodeRun &r, uint32_t stream,
                               uint64_t *bits, float *pr, float *cp, int16_t *ca, int16_t *cvi, double *gbuf = nullptr,
                               int gcap = 0) {
    const int l = lane_id();
    run_bits(P, r, bits);
    for (int a = l; a < 416; a += 64) pr[a] = 0.f;
    wave_lds_fence();
    for (int i = l; i < r.ec; i += 64) {
        const EdgeP e = *P.ep(r.eb + i);
        pr[e.a] = e.p;
        const int k = order_of(bits, e.a);
        ca[k] = e.a;
        cvi[k] = e.vi;
    }
    wave_lds_fence();
    root_noise_lds(C, t, stream, pr, bits, r.ec, gbuf, gcap);
    wave_lds_fence();                                    // (gbuf may overlay cp)
    for (int k = l; k < r.ec; k += 64) cp[k] = pr[ca[k]];
    wave_lds_fence();
    return write_sorted_run(P, r.eb, r.vb, r.ec, cp, ca, cvi);
}
__device__ __forceinline__ int noise_kept_root(const Pools &P, const SearchCfg &C, int t, const NodeRun &r,
                                               uint32_t stream, RunScr &S) {
    return noise_kept_root(P, C, t, r, stream, S.bits, S.pr, S.cp, S.ca, S.cvi);
}

// ------------------------------------------------------------ page allocation
// Home pages (Pools::nhome / ehome): a tree's first SPL_HOME_N node pages (x 64 nodes) and
// SPL_HOME_E edge pages (x 16 KB) are fixed, so a tree of average size (config 3: ~24 node and
// ~18 edge pages) lives in one contiguous stretch per pool and the 64 trees of a wave in a few
// 2 MB translations; pages beyond come from the shared free stacks.
#ifndef SPL_HOME_N
#define SPL_HOME_N 32
#endif
#ifndef SPL_HOME_E
#define SPL_HOME_E 24
#endif
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
__device__ int node_slot(const Pools &P, TreeHdr *H, int t, int id, int *npg_reg = nullptr) {
    if (id >= P.nmax) return -1;
    const int pi = id >> NPG_SHIFT;
    int32_t *tab = P.ntab + (size_t)t * P.nptab;
    if (pi >= (npg_reg ? *npg_reg : H->npg)) {
        const int pg = pi < P.nhome ? t * P.nhome + pi : pop_page(P.nfree, P.alloc + 0);
        if (pg < 0) { atomicAdd(P.alloc + 2, 1); return -1; }
        tab[pi] = pg;
        P.npidx[pg] = pi;
        H->npg = pi + 1;
        if (npg_reg) *npg_reg = pi + 1;
        return pg * NPG + (id & (NPG - 1));
    }
    return node_g(P, t, id);
}

// n contiguous edge units for tree t (a run or a visit block: global base), from the tree's
// current edge page or a fresh one (allocations never straddle pages); -1 when the tree's
// edge pages are at their maximum or the pool is empty. The tree's allocator fields are held
// in registers (k_backup_h loads them with the header's first loads, so an allocation costs
// no dependent header load) and written through on every change. One lane per tree.
struct AllocState {
    int64_t enext;
    int eleft, epg, edge_count;
};
__device__ __forceinline__ AllocState alloc_state(const TreeHdr *H) { return AllocState{H->enext, H->eleft, H->epg, H->edge_count}; }
__device__ int64_t unit_alloc_s(const Pools &P, TreeHdr *H, int t, int n, AllocState &a) {
    if (a.eleft < n) {
        if (a.epg >= P.eptab) return -1;
        const int pg = a.epg < P.ehome ? t * P.ehome + a.epg : pop_page(P.efree, P.alloc + 1);
        if (pg < 0) { atomicAdd(P.alloc + 3, 1); return -1; }
        P.etab[(size_t)t * P.eptab + a.epg] = pg;
        P.epidx[pg] = a.epg;
        a.epg += 1;
        H->epg = a.epg;
        a.enext = (int64_t)pg * UPG;
        a.eleft = UPG;
    }
    const int64_t b = a.enext;
    a.enext = b + n; a.eleft -= n; a.edge_count += n;
    H->enext = a.enext; H->eleft = a.eleft; H->edge_count = a.edge_count;
    return b;
}

// push tree pages [from, to) of a page table (tab) back to a free stack, the home entries
// (< home) excepted, wave-collective
__device__ __forceinline__ void push_pages(int32_t *stack, int32_t *top, int cap, const int32_t *tab, int from, int to,
                                           int home) {
    from = max(from, home);
    const int n = to - from;
    const int32_t *src = tab + from;
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
// evicts rounds < R-5, MCTS.py:80-85). Compacts the tree's nodes (in place, in its own page
// order) and their edge units (each kept node's run followed by its visit records, staged
// through a scratch buffer: runs and visit blocks were allocated in different orders),
// remaps child links, rebuilds the transposition table and returns the pages it no longer
// needs to the pools.
// linked = true (capacity pressure, see begin_search): keep only the root and the nodes
// reachable from it through child links, dropping nodes that only a transposition lookup
// could reach. Runs in k_gc (one workgroup per tree) with a scratch area of gc_ints ints.
struct GcScr {
    int64_t *ost;       // new local -> its old run base (global unit)
    int64_t *ovb;       // new local -> its old visit block base
    uint64_t *buf;      // new unit position -> the unit's value (staging)
    int32_t *remap;     // old local -> new local (-1: dropped); prune: reachability marks first
    int32_t *nvs;       // old local -> new local unit position of its allocation
    int32_t *cs;        // new local -> new unit position
    int32_t *cnt;       // new local -> units
    int32_t *inv;       // new local -> old local
    int32_t *queue;     // prune: breadth-first queue (old locals); then the cached links
    int32_t *oec;       // new local -> its run length (edges)
    int32_t *own;       // new unit position -> new local of its node (-1: page-end gap)
};
__host__ __device__ inline size_t gc_ints(int nmax, int emax) {
    return 11 * (size_t)(nmax + 2) + 3 * (size_t)emax + 64;
}
__device__ __forceinline__ GcScr gc_scr(int32_t *base, int nmax, int emax) {
    const size_t m = (size_t)nmax + 2;                       // (even: nmax is a multiple of 64)
    GcScr S;
    S.ost = reinterpret_cast<int64_t *>(base);
    S.ovb = reinterpret_cast<int64_t *>(base + 2 * m);
    S.buf = reinterpret_cast<uint64_t *>(base + 4 * m);
    int32_t *q = base + 4 * m + 2 * (size_t)emax;
    S.remap = q; S.nvs = q + m; S.cs = q + 2 * m; S.cnt = q + 3 * m;
    S.inv = q + 4 * m; S.queue = q + 5 * m; S.oec = q + 6 * m; S.own = q + 7 * m;
    return S;
}

// mark[i] = 1 for the root (local rootl) and every node reachable from it through child
// links, 0 else (breadth-first in batches of up to 64 queued nodes, their visit records —
// the only linked edges — 64 at a time)
__device__ void mark_linked(const Pools &P, int t, int rootl, int32_t *mark, int32_t *q) {
    const int l = lane_id();
    const int nc = P.hdr[t].node_count;
    for (int i = l; i < nc; i += 64) mark[i] = i == rootl ? 1 : 0;
    if (l == 0) q[0] = rootl;
    wave_lds_fence();
    int head = 0, tail = 1;
    while (head < tail) {
        const int nbt = min(64, tail - head);
        int64_t vb = 0;
        int cnt = 0;
        if (l < nbt) {
            const int g = node_g(P, t, q[head + l]);
            if (!P.nd[g].h.term) {
                const NodeCold c = P.nd[g].c;
                vb = c.vb();
                cnt = c.vcnt();
            }
        }
        head += nbt;
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (l >= o) incl += y;
        }
        const int tot = __shfl(incl, 63, 64), excl = incl - cnt;
        for (int c0 = 0; c0 < tot; c0 += 64) {
            const int e = c0 + l;
            int lo = 0;                                  // last lane with excl <= e
#pragma unroll
            for (int step = 32; step > 0; step >>= 1)
                if (__shfl(excl, lo + step, 64) <= e) lo += step;
            const int64_t vbo = __shfl(vb, lo, 64);
            const int exo = __shfl(excl, lo, 64);
            const int c = e < tot ? P.vr(vbo + REC_UNITS * (e - exo))->child : -1;
            BCHK(c < 0 || IN_TREE(P, t, c, nc), 58, c, t, (void)0);
            const int cl = c >= 0 ? node_l(P, c) : -1;
            const bool fresh = cl >= 0 && atomicCAS(&mark[cl], 0, 1) == 0;
            const uint64_t bm = __ballot(fresh);
            if (fresh) q[tail + __popcll(bm & lanemask_lt())] = cl;
            tail += __popcll(bm);
            wave_lds_fence();
        }
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // (HIP's uint4 struct defeats SROA)

// k_gc collects one tree per workgroup of GCT threads (block-wide scans through LDS), so a
// large tree's collection (config 4: ~40 K nodes, ~0.5 M edge units) is spread over 8 waves
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

// per-phase cycle probes of compact_tree (diagnostic builds only, -DGC_PROBE=1; never the
// product): thread 0 of each workgroup adds its phase cycles into the workgroup's slot
#ifndef GC_PROBE
#define GC_PROBE 0
#endif
#if GC_PROBE
constexpr int GC_WG_MAX_PROBE = 1024;
__device__ unsigned long long g_gc_probe[GC_WG_MAX_PROBE][16];
__device__ unsigned long long g_gc_probe_max[GC_WG_MAX_PROBE][8];   // the slowest collection's phases
#define GPROBE(k)                                                                 \
    if (threadIdx.x == 0) {                                                       \
        const uint64_t c_ = __builtin_readcyclecounter();                         \
        gacc[k] += c_ - glast;                                                    \
        glast = c_;                                                               \
    }
#else
#define GPROBE(k)
#endif
constexpr int GC_NOFIT = -2;   // compact_tree: the compacted tree would not fit the edge pages it holds
#ifndef GC_SR
#define GC_SR 8            // edge units per thread per batch of the unit staging / write-back
#endif
#ifndef GC_CR
#define GC_CR 4            // node-board units per thread per round trip of the board move (x2)
#endif
template <int CR = 4>   // board units per thread per round trip of the node-board move (x2)
__device__ int compact_tree(const Pools &P, int t, int root, int root_round, const GcScr &S, GcLds &L,
                            int bunits, bool linked = false) {
    const int tid = threadIdx.x;
    TreeHdr *H = P.hdr + t;
    const int nc = H->node_count;
    const int rootl = root >= 0 ? node_l(P, root) : -1;
    int32_t *remap = S.remap;
#if GC_PROBE
    uint64_t gacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, glast = __builtin_readcyclecounter();
    const uint64_t gstart = glast;
#endif
    if (linked) {
        if (tid < 64) mark_linked(P, t, rootl, remap, S.queue);
        __syncthreads();
    }
    int kept = 0;
    for (int base = 0; base < nc; base += GCT) {
        const int i = base + tid;
        bool keep = false;
        if (i < nc) keep = i == rootl || (linked ? remap[i] == 1 : P.nd[node_g(P, t, i)].h.round > root_round);
        int tot;
        const int ex = block_scan(keep ? 1 : 0, tot, L);
        if (i < nc) remap[i] = keep ? kept + ex : -1;
        kept += tot;
    }
    __syncthreads();
    GPROBE(0)
    // new unit position of every kept node's allocation (run + visit records): packed in local
    // order, an allocation that would straddle an edge page starts the next page. The sizes
    // are staged (all threads), then ONE wave walks the nodes 64 at a time with wave prefix
    // sums, placing the lanes before the first straddler and retrying the rest from the next
    // page — a few instructions per page boundary instead of block-wide scans (round 4: the
    // block-scan version cost ~6 workgroup barriers per page boundary, most of a collection)
    for (int i = tid; i < nc; i += GCT) {
        int sz = -1;                                     // (-1: dropped)
        if (remap[i] >= 0) {
            sz = 0;
            const int g = node_g(P, t, i);
            const Node nd = P.nd[g];
            if (!nd.h.term) sz = nd.c.ec + REC_UNITS * nd.c.vcnt();
        }
        S.nvs[i] = sz;
    }
    __syncthreads();
    if (tid < 64) {
        const int l = tid;
        int run = 0;
        constexpr int PD = 4;                            // chunks of sizes loaded ahead
        int pre[PD];
#pragma unroll
        for (int d = 0; d < PD; d++) pre[d] = 64 * d + l < nc ? S.nvs[64 * d + l] : -1;
        for (int base = 0; base < nc; base += 64) {
            const int i = base + l;
            const int szk = pre[0];
#pragma unroll
            for (int d = 0; d + 1 < PD; d++) pre[d] = pre[d + 1];
            pre[PD - 1] = base + 64 * PD + l < nc ? S.nvs[base + 64 * PD + l] : -1;
            const bool kept = szk >= 0;
            const int sz = kept ? szk : 0;
            bool pending = sz > 0;
            int start = run;
            for (;;) {
                const int x = pending ? sz : 0;
                int incl = x;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(incl, o, 64);
                    if (l >= o) incl += y;
                }
                const int st = run + incl - x;
                const bool strad = pending && (st & (UPG - 1)) + sz > UPG;
                const uint64_t m = __ballot(strad);
                if (!m) {
                    if (pending) start = st;
                    run += __shfl(incl, 63, 64);
                    break;
                }
                const int f = __ffsll((unsigned long long)m) - 1;
                if (pending && l < f) { start = st; pending = false; }
                run = (__builtin_amdgcn_readlane(st, f) & ~(UPG - 1)) + UPG;
            }
            if (kept) S.nvs[i] = start;
        }
        if (l == 0) L.bc[0] = run;
    }
    __syncthreads();
    const int run = L.bc[0];
    GPROBE(1)
    // packed with page-end gaps in an order other than the allocation order (a node's run and
    // visit block together, by local index), the kept units may need more edge pages than the
    // tree holds (the compaction moves units within its own pages and takes none from the
    // pool: k_gc only pushes pages). Only with almost no garbage: nothing is written yet, the
    // caller falls back to pruning / emptying.
    if (run > H->epg * UPG) return GC_NOFIT;
    __syncthreads();
    // node records, chunk by chunk in local order (new slot <= old slot): reads, then writes
    int my_units = 0;
    for (int base = 0; base < nc; base += GCT) {
        const int i = base + tid;
        const int ni = i < nc ? remap[i] : -1;
        uint64_t k0 = 0, k1 = 0;
        Node nd{};
        int vs = 0;
        if (ni >= 0) {
            const int g = node_g(P, t, i);
            k0 = P.nkey0[g]; k1 = P.nkey1[g];
            nd = P.nd[g];
            vs = S.nvs[i];
        }
        __syncthreads();
        if (ni >= 0) {
            const int ng = node_g(P, t, ni);
            const bool term = nd.h.term;
            const int ec = nd.c.ec, vcnt = term ? 0 : nd.c.vcnt();
            const int sz = term ? 0 : ec + REC_UNITS * vcnt;
            Node w = nd;                                 // (a terminal node's values as they are)
            S.queue[ni] = term ? -1 : nd.h.bchild;       // (the arg-max's link, remapped below)
            S.ost[ni] = nd.c.eb(); S.ovb[ni] = nd.c.vb(); S.oec[ni] = term ? 0 : ec;
            if (!term) {
                w.c.set_eb(ec > 0 ? unit_g(P, t, vs) : 0, vcnt);
                w.c.set_vb(vcnt > 0 ? unit_g(P, t, vs + ec) : 0, vcnt);
            }
            w.h.h2 = -1; w.h.h3 = -1;
            P.nkey0[ng] = k0; P.nkey1[ng] = k1;
            P.nd[ng] = w;
            S.cs[ni] = vs; S.cnt[ni] = sz; S.inv[ni] = i;
            my_units += sz;
        }
    }
    int units;
    (void)block_scan(my_units, units, L);
    GPROBE(2)
    // the cached arg-max's link (NodeStat) remapped like the visit records' links below
    for (int ni = tid; ni < kept; ni += GCT) {
        const int ch = S.queue[ni];
        if (ch >= 0) {
            BCHK(IN_TREE(P, t, ch, nc), 56, ((long long)ni << 32) | (uint32_t)ch, t, (void)0);
            const int nl = remap[node_l(P, ch)];
            P.nd[node_g(P, t, ni)].h.bchild = nl >= 0 ? node_g(P, t, nl) : -1;
            BCHK(nl < 0 || P.nd[node_g(P, t, nl)].h.round == P.nd[node_g(P, t, ni)].h.round + 1, 40,
                 ((long long)ni << 32) | (uint32_t)nl, t, (void)0);
        }
    }
    // the owner of every new unit position (gaps before a page start: -1)
    for (int k = tid; k < run; k += GCT) S.own[k] = -1;
    __syncthreads();
    for (int ni = tid; ni < kept; ni += GCT) {
        const int c0 = S.cs[ni], c = S.cnt[ni];
        for (int e = 0; e < c; e++) S.own[c0 + e] = ni;
    }
    __syncthreads();
    GPROBE(3)
    // units staged by new position (a run's EdgeP units verbatim, visit records with their
    // links remapped), then written back; every thread writes back exactly the positions it
    // staged, so only the workgroup barrier between the two passes is needed. SR positions
    // per thread per batch with each stage's loads issued together (owner -> its old bases ->
    // the unit -> the link's remap: four dependent round trips per batch, not per unit)
    constexpr int SR = GC_SR;
    for (int k0 = 0; k0 < run; k0 += GCT * SR) {
        int j[SR];
#pragma unroll
        for (int r = 0; r < SR; r++) {
            const int k = k0 + GCT * r + tid;
            j[r] = k < run ? S.own[k] : -1;
        }
        int64_t src[SR];
        bool link[SR];
#pragma unroll
        for (int r = 0; r < SR; r++) {
            src[r] = 0; link[r] = false;
            if (j[r] >= 0) {
                const int rel = k0 + GCT * r + tid - S.cs[j[r]], ec = S.oec[j[r]];
                if (rel < ec) {
                    src[r] = S.ost[j[r]] + rel;
                } else {
                    const int rr = rel - ec;
                    src[r] = S.ovb[j[r]] + rr;
                    link[r] = rr % REC_UNITS == REC_LINK_UNIT;   // {child, rank | action}: the link remapped
                }
            }
        }
        uint64_t v[SR];
#pragma unroll
        for (int r = 0; r < SR; r++) v[r] = j[r] >= 0 ? P.eu[src[r]] : 0;
#pragma unroll
        for (int r = 0; r < SR; r++) {
            if (!link[r]) continue;
            const int ch = (int)(uint32_t)v[r];
            int nch = -1;
            if (ch >= 0) {
                BCHK(IN_TREE(P, t, ch, nc), 57, ((long long)j[r] << 32) | (uint32_t)ch, t, (void)0);
                const int nl = remap[node_l(P, ch)];
                if (nl >= 0) nch = node_g(P, t, nl);
                BCHK(nl < 0 || P.nd[nch].h.round == P.nd[node_g(P, t, j[r])].h.round + 1, 41,
                     ((long long)j[r] << 32) | (uint32_t)nl, t, (void)0);
            }
            v[r] = (v[r] & 0xFFFFFFFF00000000ull) | (uint64_t)(uint32_t)nch;
        }
#pragma unroll
        for (int r = 0; r < SR; r++)
            if (j[r] >= 0) S.buf[k0 + GCT * r + tid] = v[r];
    }
    __syncthreads();
    GPROBE(4)
    for (int k0 = 0; k0 < run; k0 += GCT * SR) {
        int j[SR];
        uint64_t v[SR];
#pragma unroll
        for (int r = 0; r < SR; r++) {
            const int k = k0 + GCT * r + tid;
            j[r] = k < run ? S.own[k] : -1;
            v[r] = k < run ? S.buf[k] : 0;
        }
#pragma unroll
        for (int r = 0; r < SR; r++)
            if (j[r] >= 0) P.eu[unit_g(P, t, k0 + GCT * r + tid)] = v[r];
    }
    if (P.nbrd) {
        // node boards (bunits 16-byte units each) of new slot nn come from old slot inv[nn]
        // (>= nn), batches in increasing unit with all reads before the writes
        u32x4 *bb = reinterpret_cast<u32x4 *>(P.nbrd);
        const int bu = kept * bunits;
        constexpr int R = 2 * CR;
        for (int k0 = 0; k0 < bu; k0 += GCT * R) {
            u32x4 d[R];
            size_t dst[R];
            bool mv[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int k = k0 + GCT * r + tid;
                mv[r] = false; dst[r] = 0; d[r] = u32x4{0, 0, 0, 0};
                if (k < bu) {
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
    GPROBE(5)
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
    const int npg = (kept + NPG - 1) >> NPG_SHIFT, epg = (run + UPG - 1) >> UPG_SHIFT;
    const int onpg = H->npg, oepg = H->epg;
    const int nroot = rootl >= 0 && remap[rootl] >= 0 ? node_g(P, t, remap[rootl]) : -1;
    const int eleft = epg * UPG - run;
    const int64_t enext = eleft > 0 ? unit_g(P, t, run) : 0;
    __syncthreads();
    if (tid < 64) {
        push_pages(P.nfree, P.alloc + 0, P.npages, P.ntab + (size_t)t * P.nptab, npg, onpg, P.nhome);
        push_pages(P.efree, P.alloc + 1, P.epages, P.etab + (size_t)t * P.eptab, epg, oepg, P.ehome);
    }
    if (tid == 0) {
        H->node_count = kept; H->edge_count = units;
        H->npg = npg; H->epg = epg; H->eleft = eleft; H->enext = enext;
        H->live_gc = kept; H->units_gc = units; H->gcs += 1;
    }
    __syncthreads();
    GPROBE(6)
#if GC_PROBE
    if (tid == 0) {
        unsigned long long *g = g_gc_probe[blockIdx.x % GC_WG_MAX_PROBE];
        for (int k = 0; k < 7; k++) g[k] += gacc[k];
        g[8] += 1;
        const unsigned long long tot = glast - gstart;
        g[9] += tot;
        if (tot > g[10]) {
            g[10] = tot; g[11] = (unsigned long long)run; g[12] = (unsigned long long)kept; g[13] = (unsigned long long)nc;
            for (int k = 0; k < 7; k++) g_gc_probe_max[blockIdx.x % GC_WG_MAX_PROBE][k] = gacc[k];
        }
    }
#endif
    return nroot;
}

// edge units of tree t in use (counting the unused tail of its current page)
__device__ __forceinline__ long long units_used(const TreeHdr *H) { return (long long)H->epg * UPG - H->eleft; }
// does the next search fit tree t's maxima (budget nodes; a root's run and visit block plus
// edge_reserve units per simulation)
__device__ __forceinline__ bool tree_fits(const Pools &P, const SearchCfg &C, const TreeHdr *H) {
    return H->node_count + H->budget + 1 <= P.nmax &&
           units_used(H) + 4 * SPL_ACTIONS + (long long)H->budget * C.edge_reserve <= (long long)P.eptab * UPG;
}
// every page of tree t back to the pools, empty table. Wave-collective.
__device__ void empty_tree(const Pools &P, int t) {
    TreeHdr *H = P.hdr + t;
    const int npg = H->npg, epg = H->epg;
    push_pages(P.nfree, P.alloc + 0, P.npages, P.ntab + (size_t)t * P.nptab, 0, npg, P.nhome);
    push_pages(P.efree, P.alloc + 1, P.epages, P.etab + (size_t)t * P.eptab, 0, epg, P.ehome);
    int32_t *hs = P.hslot + (size_t)t * P.hcap;
    if (H->node_count > 0 || npg > 0)
        for (int i = lane_id(); i < P.hcap; i += 64) hs[i] = -1;
    __builtin_amdgcn_wave_barrier();
    if (lane_id() == 0) {
        H->node_count = 0; H->edge_count = 0; H->npg = 0; H->epg = 0; H->eleft = 0; H->enext = 0;
        H->live_gc = 0; H->units_gc = 0;
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
// Garbage (nodes with rounds <= the root's: unreachable, and no lookup can match them; runs
// and visit blocks of collected nodes, outgrown visit blocks) is collected by k_gc, queued
// here:
//   must (gc_state 3): the search would not fit the tree's maxima (node slots, edge page
//     table), or the arena has no self-play commit (search-only arenas never withdraw a
//     simulation, so every search starts compacted); after compaction k_gc prunes the tree
//     to the nodes linked from the root (prunes++) and empties it if that is still too
//     large (resets++);
//   should (gc_state 5): a tree whose garbage (nodes or edge units) exceeds alpha x its live
//     size, alpha from 4 (pools at most half full) down to 1/8 as they fill; k_gc may defer
//     these (GC_SHOULD_CAP per launch).
// Without an event the kept table is exactly the reference's reachable table.
#ifndef GC_ALPHA_FREE
#define GC_ALPHA_FREE 8.f  // garbage allowance while the pools are at least 3/4 free
#endif
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
        BCHK(root < 0 || IN_TREE(P, t, root, H->node_count), 54, root, t, (void)0);
        const int nc = H->node_count;
        const long long used = units_used(H);
        const bool must = nc + budget + 1 > P.nmax ||
                          used + 4 * SPL_ACTIONS + (long long)budget * C.edge_reserve > (long long)P.eptab * UPG;
        // garbage allowance alpha x the live size (at the last collection): a collection
        // copies the live tree to free its garbage, so a large alpha is cheap per freed node;
        // it shrinks as the shared pools fill (free share f: alpha = 8 while f >= 3/4, 4 while
        // f >= 1/2, then down to 1/8; config 3: 8 instead of 4 halves the collections, 0.628 ->
        // 0.619 ms per iteration, A/B)
        // (the shared pages: the stacks' capacity)
        const float f = fminf((float)P.alloc[0] / (float)max(P.npages - P.nhome * P.ntrees, 1),
                              (float)P.alloc[1] / (float)max(P.epages - P.ehome * P.ntrees, 1));
        const float alpha = f >= 0.75f ? GC_ALPHA_FREE : (f >= 0.5f ? 4.f : fmaxf(0.125f, 8.f * f));
        const bool should = nc > (int)((1.f + alpha) * (float)H->live_gc) + budget + NPG ||
                            used > (long long)((1.f + alpha) * (float)H->units_gc) +
                                       (long long)budget * C.edge_reserve + UPG;
        gcs = must || !C.selfplay ? 3 : (should ? 5 : 0);   // search-only arenas: every search
                                                           // starts compacted (no withdrawals there)
    } else {
        empty_tree(P, t);
    }
    wave_lds_fence();
    if (l == 0) {
        H->root = root;                                  // (a queued GC moves it)
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
        H->depth = 0;                                    // (a new search: no path reuse)
        H->wd_search = 0;
        if (gcs) gc_push(P, H, t);
    }
    wave_lds_fence();
}

// Garbage collection queued by k_backup (a leaf did not fit mid-search: gc_state 1) and by
// search starts (3 must, 5 should), one workgroup of GCT threads per queued tree, GC_WG
// workgroups sharing the queue (a workgroup's scratch: gc_stride ints of P.gscr). Exactly
// begin_search's policy: compact (rounds > the root's), prune to the linked nodes, empty.
// Queued trees come in bursts (games start together and commit together, so trees fill up
// together): "should" collections beyond GC_SHOULD_CAP per launch stay queued for the next
// launches (k_gc runs behind every self-play backup and commit). That is exact: a deferred
// tree searches on as it is (its search fits), and if a leaf finds no room meanwhile the
// simulation is withdrawn (gc_state 5 -> 1) and the tree collected in the next launch. A
// collection is a chain of dependent phases in one workgroup, so a launch costs about its
// slowest collection however many run beside it: the cap is one round of workgroups (a
// smaller cap spreads a burst over more launches that each pay that latency — round 4
// measured 16 per launch at 195 us per launch, ~390 us per iteration at config 3).
#ifndef GC_WG
#define GC_WG 256               // one per CU (168 VGPRs x 8 waves: a second one does not fit;
#endif                          //  512 measured no change, r05)
#ifndef GC_SHOULD_CAP
#define GC_SHOULD_CAP GC_WG
#endif
template <int N>
__global__ __launch_bounds__(GCT) void k_gc(Pools P, SearchCfg C) {
    __shared__ GcLds L;
    __shared__ int keep_s;
    const int tid = threadIdx.x;
    const int tail = P.counters[2];                      // no pushes while k_gc runs
    const int ftail = P.counters[5];
    if (tail == 0 && ftail == 0) return;                 // (the usual case)
    const GcScr S = gc_scr(P.gscr + (size_t)blockIdx.x * P.gc_stride, P.nmax, P.emax);
    for (int k = blockIdx.x; k < tail; k += gridDim.x) {     // garbage collection
        const int t = P.gcq[k];
        TreeHdr *H = P.hdr + t;
        const int st = H->gc_state;
        if (tid == 0) {
            int keep = 0;
            if (st == 5 && atomicAdd(&P.counters[8], 1) >= GC_SHOULD_CAP) {
                keep = 1;                                // deferred: stays queued
                P.gcq2[atomicAdd(&P.counters[9], 1)] = t;
            }
            keep_s = keep;
        }
        __syncthreads();
        if (keep_s) continue;
        int root = H->root;
        const int nst = st == 1 ? 2 : 0;
        if (st == 1 || st == 3 || st == 5) {
            // mid-search (1: the descent then repeats): rounds above the root's; search start:
            // above the root round
            const int rr = st == 1 && root >= 0 ? P.nd[root].h.round : H->root_round;
            const int r0 = root;
            root = compact_tree<GC_CR>(P, t, r0, rr, S, L, NodeBoard<N>::UNITS);
            // capacity pressure (search start: the search would not fit; any: the compacted
            // layout would not fit the page table): prune to the linked nodes, else empty
            bool prune = root == GC_NOFIT;
            if (!prune && st != 1) prune = !tree_fits(P, C, H) && root >= 0;
            if (prune) {
                root = compact_tree<GC_CR>(P, t, root == GC_NOFIT ? r0 : root, rr, S, L, NodeBoard<N>::UNITS, true);
                if (tid == 0) H->prunes += 1;
            }
            __syncthreads();
            if (root == GC_NOFIT || (st != 1 && !tree_fits(P, C, H))) {
                root = -1;
                if (tid < 64) empty_tree(P, t);
                if (tid == 0) H->resets += 1;
            }
        }
        __syncthreads();
        if (tid == 0) {
            H->gc_queued = 0;
            if (st == 1 || st == 3 || st == 5) {
                H->root = root;
                H->gc_state = nst;                       // (2: collected mid-search)
                H->depth = 0;                            // (node ids moved: no path reuse)
            }
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
    if (tid == 0) {
        __threadfence();                                 // (deferred entries before the count)
        keep_s = atomicAdd(&P.counters[4], 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (keep_s) {                                        // the last workgroup out: the deferred
        __threadfence();                                 // entries become the queue
        const int nk = __hip_atomic_load(&P.counters[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int i = tid; i < nk; i += GCT)
            P.gcq[i] = __hip_atomic_load(&P.gcq2[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (tid == 0) {
            P.counters[2] = nk;
            P.counters[5] = 0;
            P.counters[4] = 0;
            P.counters[8] = 0;
            P.counters[9] = 0;
        }
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
    __shared__ int16_t pact[WAVES][SPL_ACTIONS];         // the root's edges in action order:
    __shared__ int32_t pcnt[WAVES][SPL_ACTIONS];         // action, visit count, prior
    __shared__ __align__(16) float pprior[WAVES][SPL_ACTIONS + 3];   // (rows 16-byte aligned: they
                                                                     //  double as root noise's scratch)
    __shared__ uint64_t pbits[WAVES][7];
    const int w = threadIdx.x >> 6, t = blockIdx.x * WAVES + w;
    if (t >= B) return;
    const int l = lane_id();
    TreeHdr *H = P.hdr + t;
    // (a tree whose leaf did not fit waits for k_gc: its simulation was withdrawn, so its
    // search is not done)
    if (H->gc_state == 1 || H->sims_done < H->budget || H->overflow || H->root < 0) return;
    const uint32_t gb = C.board_base + (uint32_t)t;
    const int root = H->root;
    const NodeRun rr = run_of(P.nd[root].c);
    const int ec = rr.ec;
    const bool forced = H->forced;
    const int sims = H->budget, cm = H->move_no;
    // the root's edges staged in action order (the reference's array order, which the
    // sequential sums of random_pick follow)
    run_bits(P, rr, pbits[w]);
    int best = 0;
    for (int i = l; i < ec; i += 64) {
        const EdgeP e = *P.ep(rr.eb + i);
        const int n = e.vi >= 0 ? P.vr(rr.vb + REC_UNITS * e.vi)->n : 0;
        const int k = order_of(pbits[w], e.a);
        pact[w][k] = e.a; pcnt[w][k] = n; pprior[w][k] = e.p;
        best = max(best, n);
    }
    best = wave_max_i32(best);
    wave_lds_fence();
    // policy counts: pruned (MCTS.py:69-74); where the reference would divide 0/0
    // (Coach.py:83 raises) fall back to raw counts, then to uniform
    int mode = forced ? 0 : 1;
    long long tot = 0;
    for (; mode < 3; mode++) {
        tot = 0;
        for (int i = l; i < ec; i += 64)
            tot += mode == 0 ? pruned_count(pcnt[w][i], best, true, pprior[w][i], sims) : (mode == 1 ? pcnt[w][i] : 1);
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (tot > 0) break;
    }
#define POLICY_COUNT(i) (mode == 0 ? pruned_count(pcnt[w][i], best, true, pprior[w][i], sims) : (mode == 1 ? (long long)pcnt[w][i] : 1ll))
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
            pi[pact[w][i]] = (float)((double)POLICY_COUNT(i) / (double)tot);
        uint64_t m[7];
        wave_valid_moves<N>(s, 0, lim, m);
        store_mask(P.ex_valid + x * 7, m);
        if (l == 0) {
            const double q0 = P.nd[root].h.qs;
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
    // (round 6: the same operations in the same order, but every division off the sequential
    // chain: p[i] = pt[i] / sum lane-parallel, cdf = cumsum(p) on lane 0 (its last entry is
    // the normaliser), the first i with cdf[i] / cdf[-1] > u found lane-parallel)
    for (int i = l; i < ec; i += 64) pterm[w][i] = temp_pow((double)POLICY_COUNT(i) / (double)tot, T);
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    double sum = 0.0;
    if (l == 0) {
        const double *pt = pterm[w];
        for (int i = 0; i < ec; i++) sum += pt[i];
    }
    sum = readlane_f64(sum, 0);
    for (int i = l; i < ec; i += 64) pterm[w][i] = pterm[w][i] / sum;
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    if (l == 0) {
        double *pt = pterm[w];
        double cdf = 0.0;
        for (int i = 0; i < ec; i++) {
            cdf += pt[i];
            pt[i] = cdf;
        }
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    {
        const double last = pterm[w][ec - 1];
        const double u = philox_u01(C.seed, gb, ST_PICK | (uint32_t)cm, 0);
        int first = ec - 1;
        for (int base = 0; base < ec; base += 64) {
            const int i = base + l;
            const uint64_t m = __ballot(i < ec && pterm[w][i] / last > u);
            if (m) { first = base + __ffsll((unsigned long long)m) - 1; break; }
        }
        action = pact[w][first];
    }
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
    // a kept root's Dirichlet noise at its search start: exactly what the search's first
    // select would apply (same stored priors, same stream ST_DIR | move_no), here where every
    // tree has a wave of its own instead of the select's one tree at a time per wave; then
    // the root's arg-max under the noised priors (scan_run, as that select would scan) is
    // cached. Not when a collection is queued (it may move or empty the tree first: the select
    // or the backup of a new root then applies the noise). The move-sampling scratch is free.
    const int nroot = uniform(H->root);
    if (nroot >= 0 && uniform(H->noise_pending) && !uniform(H->gc_queued)) {
        const Node nd0 = P.nd[nroot];
        NodeRun r = run_of(nd0.c);
        r.eb = (int64_t)uniform64((uint64_t)r.eb); r.vb = (int64_t)uniform64((uint64_t)r.vb);
        r.ec = uniform(r.ec);
        const int cand = noise_kept_root(P, C, t, r, ST_DIR | (uint32_t)uniform(H->move_no), pbits[w],
                                         reinterpret_cast<float *>(pterm[w]), pprior[w], pact[w],
                                         reinterpret_cast<int16_t *>(pcnt[w]),
                                         reinterpret_cast<double *>(pprior[w]), (int)(sizeof(pprior[w]) / 8));
        wave_lds_fence();                                        // (the re-sorted run, read below)
        int ca;
        float cp, np;
        wave_cand(P, r.eb, r.ec, cand, ca, cp, np);
        const bool forced = uniform(H->forced) != 0;
        Pick pk{-1, 0, -1, 0};
        if (!forced) pk = scan_run(P, r, nd0.h.ns, nd0.h.qs, C.cpuct, C.fpu, false, 0);
        if (l == 0) {
            H->noise_pending = 0;
            Node w2 = nd0;
            w2.c.cand = (int16_t)cand; w2.c.ca = (int16_t)ca; w2.c.cp = cp; w2.c.np = np;
            w2.h.set_pick(pk.e, pk.a, pk.e >= 0 && pk.child >= 0 ? P.nd[pk.child].h.term : 0);   // (-1: scans)
            w2.h.bchild = pk.e >= 0 ? pk.child : -1;
            w2.h.h2 = -1; w2.h.h3 = -1;
            w2.h.bvi = pk.e >= 0 ? P.ep(r.eb + pk.e)->vi : (int16_t)-1;
            P.nd[nroot] = w2;
        }
    }
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
// a terminal node's end values (its NodeCold's first 16 bytes hold es[4])
__device__ __forceinline__ void term_values(const Pools &P, int g, float v[4]) {
    const float4 e = *reinterpret_cast<const float4 *>(&P.nd[g].c);
    v[0] = e.x; v[1] = e.y; v[2] = e.z; v[3] = e.w;
}
// the record of a new terminal node of round rd with end values v
__device__ __forceinline__ Node term_node(const float v[4], int rd) {
    Node n{};
    n.h.bchild = -1; n.h.h2 = -1; n.h.h3 = -1; n.h.set_pick(-1, 0, 0); n.h.ns = 0;
    n.h.term = 1; n.h.round = (uint8_t)rd; n.h.qs = 0.0;
    *reinterpret_cast<float4 *>(&n.c) = make_float4(v[0], v[1], v[2], v[3]);
    n.h.bvi = -1;
    n.c.ec = 0; n.c.cand = 0; n.c.ca = 0; n.c.pad = 0; n.c.cp = 0.f; n.c.np = -1.f;
    return n;
}

// ------------------------------------------------------------ select, lane per tree
// k_select_lanes: the descent (MCTS.py:99-177 down to the leaf) with one LANE per tree (64
// trees per wave). Below the root a level is one 32-byte NodeStat load (the cached arg-max and
// its link), work for a single lane, so a wave per tree (round 3) left 63 lanes idle and the
// launch was bound by wave slots x the chain latency; lane per tree keeps 64 chains in flight
// per wave. The steps that
// need a board — the in-tree transition at the edge to expand (MCTS.py:227-235), the
// fingerprint lookup (:119-120), the end check (:125) and the new leaf's board — run per lane
// on the lane's own LDS board. Root scans (a root whose priors were just noised, forced
// playouts, a new root) and root noise stay wave-collective, one tree at a time (rare).

// swap_players on a lane's own LDS board, in place: every player block rotated left by its
// stride (gems k, nobles 3k — hard-coded 3, SplendorLogicNumba.py:345 —, cards k, reserved
// 6k rows; wave_roll_players' mapping) by three reversals
template <int N>
__device__ __forceinline__ void lane_roll_players(int8_t *s, int k) {
    using Lx = Lay<N>;
    auto rev = [&](int a, int b) {
        for (--b; a < b; a++, b--) {
            const uint64_t x = row(s, a);
            row(s, a) = row(s, b);
            row(s, b) = x;
        }
    };
    auto rot = [&](int base, int m, int sh) {
        sh %= m;
        if (!sh) return;
        rev(base, base + sh);
        rev(base + sh, base + m);
        rev(base, base + m);
    };
    rot(Lx::GEMS, N, k);
    rot(Lx::GEMS + N, N * Lx::NN, 3 * k);
    rot(Lx::GEMS + N + N * Lx::NN, N, k);
    rot(Lx::GEMS + 2 * N + N * Lx::NN, 6 * N, 6 * k);
}
// the wave_fingerprint of a lane's own board
template <int N>
__device__ __forceinline__ void lane_fingerprint(const int8_t *s, uint64_t &k0, uint64_t &k1) {
    uint64_t a = 0, b = 0;
    for (int i = 0; i < Lay<N>::ROWS; i++) {
        const uint64_t x = row(s, i) | ((uint64_t)i << 56);
        a ^= mix64(x ^ 0x243F6A8885A308D3ull);
        b ^= mix64(x ^ 0x13198A2E03707344ull);
    }
    k0 = a;
    k1 = b | 1ull;
}
// the in-tree transition of one lane's board (MCTS.py:227-235): make_move(a, 0, det) + roll
template <int N>
__device__ __forceinline__ void lane_tree_step(int8_t *s, int a) {
    Chance ch{nullptr, 0, 0, 0, 0};
    int nxt;
    switch (move_kind_of(a)) {
        case MK_GEMS: nxt = make_move<N, MK_GEMS>(s, a, 0, true, ch); break;
        case MK_BUY: nxt = make_move<N, MK_BUY>(s, a, 0, true, ch); break;
        case MK_RESERVE: nxt = make_move<N, MK_RESERVE>(s, a, 0, true, ch); break;
        default: nxt = make_move<N, MK_BUY_RESERVED>(s, a, 0, true, ch); break;
    }
    if (nxt) lane_roll_players<N>(s, nxt);
}

// Per-phase cycle probes of k_select_lanes (diagnostic builds only, -DSELECT_PROBE=1; never
// the product): per wave, s_memtime deltas summed over the waves of every launch
#ifndef SELECT_PROBE
#define SELECT_PROBE 0
#endif
#if SELECT_PROBE
__device__ unsigned long long g_sel_probe[16];
#define SPROBE(k)                                                  \
    {                                                              \
        const uint64_t c_ = __builtin_readcyclecounter();          \
        pacc[k] += c_ - plast;                                     \
        plast = c_;                                                \
    }
#else
#define SPROBE(k)
#endif
#ifndef PATH_CHUNK
#define PATH_CHUNK 8       // previous-path levels a lane checks per round trip
#endif
enum { LS_DESCEND = 0, LS_EXPAND = 1, LS_DONE = 2 };

// The linked run of the descent (levels whose cached pick is linked to a non-terminal child)
// with the descent hints (NodeHot h2 / h3: the cached picks two and three levels down, written
// by k_backup_h): every level requests the record its h3 names — the record three levels down
// most likely needs — so along a correct chain a level's record was requested two levels
// earlier. A lane whose child is not the predicted node loads its child's record on the spot
// (into the same registers: loads return in order). The wave waits for the older load only
// when every active lane's prediction held (vmcnt(8) / (9): the record requested two levels
// ago, behind 8 or 9 younger memory instructions; else vmcnt(3): this level's own load) —
// compiled code cannot express that data-dependent wait (its waits follow the registers: a
// compiled loop-carried prefetch measured 0.606 vs 0.557 ms), so the loop is one assembly block
// with its own registers (v226-v255), three rotating record slots and a unique label set.
// In: lanes in `runm` descend from (node, depth) with rec = node's link record (arrived). Out:
// each lane at the first level that is not a plain link, rec = its record; the path entries
// [depth_in, depth_out) written. The records and path are the C loop's (SELECT_ASM=0).
#ifndef SELECT_ASM
#define SELECT_ASM 1       // (bounds-checked builds too: their check follows the block)
#endif
// The block's waits count memory instructions per level: an optional child-record load (SA),
// the h3 record load (SC) and SEL_STORES path stores, in that order. A lane's child loaded on
// the spot is SEL_W_OWN instructions back; a record requested two levels ago (that level's SC)
// is behind its SEL_STORES stores and the two later levels' SC + stores: SEL_W_HINT, plus one
// when the previous level loaded a child. Change the body and these together.
#define SEL_STORES 2
#define SEL_W_OWN 3
#define SEL_W_HINT 8
#define SEL_W_HINT1 9
static_assert(SEL_W_OWN == 1 + SEL_STORES, "own child load: behind SC + the stores");
static_assert(SEL_W_HINT == SEL_STORES + 2 * (1 + SEL_STORES) && SEL_W_HINT1 == SEL_W_HINT + 1,
              "hinted record: two levels back");
#define SEL_STR2(x) #x
#define SEL_STR(x) SEL_STR2(x)
#define SEL_BODY(SA, SC, K)                                                                     \
    "v_cmp_le_i32 vcc, 0, v240\n"                 /* a linked pick                     */      \
    "v_cmp_le_i32 %[T], 0, v243\n"                /* whose child is not terminal       */      \
    "s_and_b64 vcc, vcc, %[T]\n"                                                               \
    "v_cmp_gt_i32 %[T], %[pcap], v233\n"          /* below the path limit              */      \
    "s_and_b64 vcc, vcc, %[T]\n"                                                               \
    "s_and_b64 exec, exec, vcc\n"                                                              \
    "s_cbranch_execz L_done_%=\n"                                                              \
    "v_cmp_ne_u32 vcc, v240, v234\n"              /* the child is not the predicted node: */    \
    "s_and_saveexec_b64 %[SV], vcc\n"             /* load its record now                */      \
    "s_mov_b64 %[INV], exec\n"                                                                 \
    "s_cbranch_execz L_nf" K "_%=\n"                                                           \
    "v_mad_u64_u32 v[238:239], %[CC], v240, 64, %[nd]\n"                                       \
    "global_load_dwordx4 " SA ", v[238:239], off\n"                                            \
    "L_nf" K "_%=:\n"                                                                          \
    "s_mov_b64 exec, %[SV]\n"                                                                  \
    "v_cmp_gt_u32 vcc, %[lim], v242\n"            /* h3, if a node id (else the child   */      \
    "v_cndmask_b32 v226, v240, v242, vcc\n"       /* again): three levels down          */      \
    "v_mad_u64_u32 v[238:239], %[CC], v226, 64, %[nd]\n"                                       \
    "global_load_dwordx4 " SC ", v[238:239], off\n"                                            \
    "v_mad_u64_u32 v[238:239], %[CC], v233, 4, v[252:253]\n"   /* path_n[depth] = node */      \
    "global_store_dword v[238:239], v232, off\n"                                               \
    "v_and_b32 v236, 0xffff, v243\n"                           /* path_x: rank | a << 9 */     \
    "v_bfe_u32 v237, v243, 16, 15\n"                                                           \
    "v_lshl_or_b32 v236, v237, 9, v236\n"                                                      \
    "v_mad_u64_u32 v[238:239], %[CC], v233, 4, v[254:255]\n"                                   \
    "global_store_dword v[238:239], v236, off\n"                                               \
    "v_add_u32 v233, 1, v233\n"                                                                \
    "v_mov_b32 v232, v240\n"                                                                   \
    "v_mov_b32 v234, v235\n"                      /* predictions: next level, the one after */ \
    "v_mov_b32 v235, v226\n"                                                                   \
    "s_cmp_eq_u64 %[INV], 0\n"                                                                 \
    "s_cbranch_scc1 L_av" K "_%=\n"                                                            \
    "s_waitcnt vmcnt(" SEL_STR(SEL_W_OWN) ")\n"    /* some lane loaded its child now     */      \
    "s_mov_b32 %[F], 1\n"                                                                      \
    "s_branch L_sel" K "_%=\n"                                                                 \
    "L_av" K "_%=:\n"                             /* every record requested two levels  */      \
    "s_cmp_eq_u32 %[F], 0\n"                      /* ago: behind 8 memory instructions, */      \
    "s_cbranch_scc1 L_a8" K "_%=\n"               /* 9 if the last level loaded a child */      \
    "s_waitcnt vmcnt(" SEL_STR(SEL_W_HINT1) ")\n"                                              \
    "s_branch L_a0" K "_%=\n"                                                                  \
    "L_a8" K "_%=:\n"                                                                          \
    "s_waitcnt vmcnt(" SEL_STR(SEL_W_HINT) ")\n"                                               \
    "L_a0" K "_%=:\n"                                                                          \
    "s_mov_b32 %[F], 0\n"                                                                      \
    "L_sel" K "_%=:\n"
#define SEL_TAKE(R)                                                                             \
    "v_mov_b32 v240, v" #R "\n"                                                                \
    "v_mov_b32 v241, v" #R "+1\n"
__device__ __forceinline__ void descend_linked_asm(int &node, int &depth, NodeLink &rec, const Node *nd, int pcap,
                                                   int32_t *path_n, int32_t *path_x, uint64_t runm, int lim) {
    int r0 = rec.bchild, r1 = rec.h2, r2 = rec.h3;
    int r3 = (int)((uint32_t)(uint16_t)rec.best | ((uint32_t)rec.babt << 16));
    uint64_t T, SV, INV, CC, SAVE;
    int F;
    asm volatile(
        "s_mov_b64 %[SAVE], exec\n"
        "s_mov_b32 %[F], 1\n"
        "v_mov_b32 v232, %[node]\n"
        "v_mov_b32 v233, %[depth]\n"
        "v_mov_b32 v240, %[r0]\n"
        "v_mov_b32 v241, %[r1]\n"
        "v_mov_b32 v242, %[r2]\n"
        "v_mov_b32 v243, %[r3]\n"
        "v_mov_b32 v234, -1\n"
        "v_mov_b32 v235, -1\n"
        "v_mov_b64 v[252:253], %[pn]\n"
        "v_mov_b64 v[254:255], %[pxp]\n"
        "s_and_b64 exec, exec, %[runm]\n"
        "s_cbranch_execz L_done_%=\n"
        "L_top_%=:\n"
        SEL_BODY("v[244:247]", "v[228:231]", "0")
        "v_mov_b32 v240, v244\n" "v_mov_b32 v241, v245\n" "v_mov_b32 v242, v246\n" "v_mov_b32 v243, v247\n"
        SEL_BODY("v[248:251]", "v[244:247]", "1")
        "v_mov_b32 v240, v248\n" "v_mov_b32 v241, v249\n" "v_mov_b32 v242, v250\n" "v_mov_b32 v243, v251\n"
        SEL_BODY("v[228:231]", "v[248:251]", "2")
        "v_mov_b32 v240, v228\n" "v_mov_b32 v241, v229\n" "v_mov_b32 v242, v230\n" "v_mov_b32 v243, v231\n"
        "s_branch L_top_%=\n"
        "L_done_%=:\n"
        "s_waitcnt vmcnt(0)\n"
        "s_mov_b64 exec, %[SAVE]\n"
        "v_mov_b32 %[node], v232\n"
        "v_mov_b32 %[depth], v233\n"
        "v_mov_b32 %[r0], v240\n"
        "v_mov_b32 %[r1], v241\n"
        "v_mov_b32 %[r2], v242\n"
        "v_mov_b32 %[r3], v243\n"
        : [node] "+v"(node), [depth] "+v"(depth), [r0] "+v"(r0), [r1] "+v"(r1), [r2] "+v"(r2), [r3] "+v"(r3),
          [T] "=&s"(T), [SV] "=&s"(SV), [INV] "=&s"(INV), [CC] "=&s"(CC), [SAVE] "=&s"(SAVE), [F] "=&s"(F)
        : [nd] "s"(nd), [pcap] "s"(pcap), [pn] "v"(path_n), [pxp] "v"(path_x), [runm] "s"(runm), [lim] "s"(lim)
        : "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238",
          "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251",
          "v252", "v253", "v254", "v255", "vcc", "scc", "memory");
    rec.bchild = r0; rec.h2 = r1; rec.h3 = r2;
    rec.best = (int16_t)(r3 & 0xFFFF); rec.babt = (uint16_t)((uint32_t)r3 >> 16);
}
#undef SEL_BODY
#undef SEL_TAKE

template <int N>
__global__ __launch_bounds__(64) void k_select_lanes(Pools P, SearchCfg C, int B, int lim,
                                                     int8_t *__restrict__ leaf_state,
                                                     uint8_t *__restrict__ leaf_valid) {
    using Lx = Lay<N>;
    constexpr int ST = (Lx::ROWS % 2 ? Lx::ROWS : Lx::ROWS + 1) * 8;   // odd row count per board:
    __shared__ __align__(16) int8_t boards[64 * ST];                    // lanes on distinct banks
    __shared__ RunScr scr;                                              // root noise (one tree)
    const int l = lane_id();
#if SELECT_PROBE
    uint64_t pacc[6] = {0, 0, 0, 0, 0, 0}, plast = __builtin_readcyclecounter();
    const uint64_t pstart = plast;
    int plev = 0, pexp = 0;                              // levels descended, expansion rounds
#endif
    const int slot = blockIdx.x * 64 + l;
    const bool live = slot < B;
    const int t = live ? slot : 0;
    TreeHdr *H = P.hdr + t;
    int8_t *s = boards + l * ST;
    int sims = 0, root = -1, hdepth = 0, mv = 0, hnc = 0, hnpg = 0;
    bool act = false, noise = false, forced = false;
    if (live) {
        sims = H->sims_done;
        act = sims < H->budget && !H->overflow;
        root = H->root; hdepth = H->depth; mv = H->move_no;
        noise = H->noise_pending != 0; forced = H->forced != 0;
        hnc = H->node_count; hnpg = H->npg;          // (k_select's own writes update them)
        if (!act) { leaf_valid[t] = 0; H->leaf_kind = LEAF_NONE; }
    }
    const uint64_t *nbrd = reinterpret_cast<const uint64_t *>(P.nbrd);
    const int32_t pstride = P.pcap + 1;
    int32_t *path_n = P.path_n + (size_t)t * pstride;
    int32_t *path_x = P.path_x + (size_t)t * P.pcap;
    // boards the lane needs from the start: the root's when it is the leaf, or without node
    // boards (the transition then runs at every level, from the root)
    if (act && (root < 0 || !nbrd))
        for (int u = 0; u < Conv<N>::UNITS; u++) Conv<N>::load(s, P.root_state + (size_t)t * Lx::S, u);
    // root noise on kept roots (:150-154), wave-collective one tree at a time
    const bool noised = act && root >= 0 && sims == 0 && noise;
    for (uint64_t m = __ballot(noised); m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        const int tj = __builtin_amdgcn_readlane(t, j), rj = __builtin_amdgcn_readlane(root, j);
        NodeRun r = run_of(P.nd[rj].c);
        r.eb = (int64_t)uniform64((uint64_t)r.eb); r.vb = (int64_t)uniform64((uint64_t)r.vb);
        r.ec = uniform(r.ec);
        const int cand = noise_kept_root(P, C, tj, r, ST_DIR | (uint32_t)__builtin_amdgcn_readlane(mv, j), scr);
        wave_lds_fence();
        int ca;
        float cp, np;
        wave_cand(P, r.eb, r.ec, cand, ca, cp, np);
        if (l == 0) {
            P.hdr[tj].noise_pending = 0;                 // (a withdrawn simulation must not re-noise)
            NodeCold &c = P.nd[rj].c;
            c.cand = (int16_t)cand; c.ca = (int16_t)ca; c.cp = cp; c.np = np;
            P.nd[rj].h.best = -1;                        // ranks moved: the root scans
        }
        wave_lds_fence();
    }
    __threadfence_block();
    const bool root_cache = !forced && !noised;
    int node = root, depth = 0, state = act && root >= 0 ? LS_DESCEND : LS_DONE;
    int kind = act ? LEAF_NN : LEAF_NONE;
    // resume on the previous simulation's path (same search: sims > 0; k_gc clears H->depth
    // when it moves nodes) at the first level whose node's cached pick no longer is the path's
    // edge, or the previous leaf's parent — k_backup, which moved those picks, recorded that
    // level (H->resume); only a backup changes a cached pick between two selects of a search
    if (state == LS_DESCEND && sims > 0 && hdepth > 0) {
        const int q = root_cache ? min(H->resume, hdepth - 1) : 0;
        node = path_n[q];
        depth = q;
        if (!nbrd)                                       // the resume node's board: the path's moves
            for (int d = 0; d < q; d++) lane_tree_step<N>(s, px_action(path_x[d]));
    }
    // the root level scans when its cached pick does not hold (noise, forced playouts, a new
    // root): wave-collective, one tree at a time, before the lanes descend
    Pick pk{0, 0, -1, 0};
    bool have_pk = false;
    NodeHot nsq{-1, -1, -1, -1, 0, 0, 0, 0, -1, 0.0};   // (the first node's whole hot half)
    if (state == LS_DESCEND) nsq = P.nd[node].h;
    const bool scan = state == LS_DESCEND && depth == 0 && (!root_cache || nsq.best < 0);
    for (uint64_t m = __ballot(scan); m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        const int nj = __builtin_amdgcn_readlane(node, j);
        NodeRun r = run_of(P.nd[nj].c);
        r.eb = (int64_t)uniform64((uint64_t)r.eb); r.vb = (int64_t)uniform64((uint64_t)r.vb);
        r.ec = uniform(r.ec);
        const Pick p = scan_run(P, r, __builtin_amdgcn_readlane(nsq.ns, j), readlane_f64(nsq.qs, j), C.cpuct, C.fpu,
                                __builtin_amdgcn_readlane((int)forced, j) != 0, __builtin_amdgcn_readlane(sims, j));
        if (l == j) { pk = p; have_pk = true; }
    }
    if (have_pk) {                                       // the scanned edge's link and whether terminal
        if (pk.child < 0 && pk.e == nsq.best && !noised) { pk.child = nsq.bchild; pk.cterm = nsq.bterm(); }
        else pk.cterm = pk.child >= 0 ? (int)P.nd[pk.child].h.term : 0;
    }
    int bnode = nbrd ? -1 : node;                        // the node whose board the lane holds
    int miss = -1, leaf_node = -1, cbest = -1;
    uint64_t k0 = 0, k1 = 0;
    float val[4] = {0, 0, 0, 0};
    // the descent reads ONE 16-byte link record per level: rec is `node`'s (nsq's at the start)
    NodeLink rec = *reinterpret_cast<const NodeLink *>(&nsq);
    int tv_node = -1;                                    // a stored terminal leaf: its end values
    // descend phase: every lane in DESCEND takes one level per round trip until it reaches the
    // edge it expands (or a terminal child); then the expansions of all lanes run together —
    // the expansion (board staging, transition, fingerprint, lookup) is long, and lanes
    // reaching it at different levels would otherwise run it once per level in turn
    // (measured: 342 us per select at config 3 with the two phases interleaved).
    // The common level — the cached pick is linked and its child is not terminal — runs in a
    // tight loop that carries only (node, depth, rec): a lane issues the child's record load,
    // then its two path stores, and the next level waits for that load alone (gfx950 counts
    // stores in vmcnt: vmcnt(2)); other levels (a scanned root pick, a terminal child, an
    // edge to expand, the path limit) take the general step below it once.
    SPROBE(0)
    while (__ballot(state != LS_DONE)) {
      while (__ballot(state == LS_DESCEND)) {
        bool run = state == LS_DESCEND && !have_pk && nbrd;
#if SELECT_ASM
        {
#if SELECT_PROBE || SPL_BOUNDS_CHECK
            const int d0 = depth;
#endif
            descend_linked_asm(node, depth, rec, P.nd, P.pcap, path_n, path_x, __ballot(run), P.npages * NPG);
#if SELECT_PROBE
            plev += depth - d0;
#endif
#if SPL_BOUNDS_CHECK
            // the assembly descent's new path entries [d0, depth): every level's child in the
            // tree and one round deeper (the C loop's sites 52 / 30)
            for (int d = d0; d < depth; d++) {
                const int pn = path_n[d], c = d + 1 < depth ? path_n[d + 1] : node;
                BCHK(IN_TREE(P, t, c, H->node_count), 52, c, t, (void)0);
                BCHK(P.nd[c].h.round == P.nd[pn].h.round + 1, 30, ((long long)pn << 32) | (uint32_t)c, t, (void)0);
            }
#endif
            run = false;
        }
#endif
        while (__ballot(run)) {
            if (run) {
                const int c = rec.bchild;
                run = c >= 0 && !rec.bterm() && depth < P.pcap;
                if (run) {
                    BCHK(IN_TREE(P, t, c, H->node_count), 52, c, t, (void)0);
                    BCHK(P.nd[c].h.round == P.nd[node].h.round + 1, 30, ((long long)node << 32) | (uint32_t)c, t, (void)0);
                    const NodeLink nx = link_of(P.nd, c);
                    path_n[depth] = node; path_x[depth] = px_pack(rec.best, rec.ba());
                    depth++;
                    node = c;
                    rec = nx;
#if SELECT_PROBE
                    plev++;
#endif
                }
            }
        }
        if (state == LS_DESCEND) {                       // the general step
            if (depth >= P.pcap) {
                state = LS_DONE; kind = LEAF_NONE; H->overflow = 2;
            } else {
                if (!have_pk) pk = Pick{rec.best, rec.ba(), rec.bchild, rec.bterm()};
                have_pk = false;
                cbest = rec.best;
#if SELECT_PROBE
                plev++;
#endif
                path_n[depth] = node; path_x[depth] = px_pack(pk.e, pk.a);
                depth++;
                if (pk.child >= 0 && pk.cterm) {         // a terminal child (MCTS.py:125-132)
                    kind = LEAF_TERMINAL;                // (its end values after the loop)
                    leaf_node = pk.child;
                    tv_node = pk.child;
                    state = LS_DONE;
                } else if (pk.child >= 0 && nbrd) {      // linked (a scanned root pick)
                    BCHK(IN_TREE(P, t, pk.child, H->node_count), 52, pk.child, t, (void)0);
                    rec = link_of(P.nd, pk.child);
                    node = pk.child;
                } else {
                    state = LS_EXPAND;
                }
            }
        }
      }
        SPROBE(1)
        if (state == LS_EXPAND && nbrd && bnode != node) {   // stage this node's stored board
            const uint64_t *src = nbrd + (size_t)node * (NodeBoard<N>::BYTES / 8);
            for (int r = 0; r < Lx::ROWS; r++) row(s, r) = src[r];
#if SPL_BOUNDS_CHECK
            uint64_t f0, f1;
            lane_fingerprint<N>(s, f0, f1);
            BCHK(f0 == P.nkey0[node] && f1 == P.nkey1[node], 36, node, t, (void)0);
#endif
        }
        SPROBE(2)
#if SELECT_PROBE
        pexp += __ballot(state == LS_EXPAND) != 0;
#endif
        if (state == LS_EXPAND) {
            lane_tree_step<N>(s, pk.a);
            int child = pk.child;
            const bool cached = cbest == pk.e;
            if (child < 0) {
                lane_fingerprint<N>(s, k0, k1);
                child = hash_lookup(P, t, k0, k1, &miss);
                if (child >= 0) {                        // transposition: link the cached pick
                    const int ct = P.nd[child].h.term;
                    BCHK(IN_TREE(P, t, child, H->node_count), 53, child, t, (void)0);
                    BCHK(P.nd[child].h.round == P.nd[node].h.round + 1, 37, ((long long)node << 32) | (uint32_t)child, t, (void)0);
                    if (cached) { P.nd[node].h.bchild = child; P.nd[node].h.babt = (uint16_t)(pk.a | (ct << 15)); }
                    if (ct) {
                        kind = LEAF_TERMINAL;
                        tv_node = child;
                        leaf_node = child;
                        state = LS_DONE;
                    }
                }
            }
            if (state == LS_EXPAND) {
                BCHK(child < 0 || P.nd[child].h.round == (uint8_t)bt(row(s, 0), 6), 31,
                     ((long long)node << 32) | (uint32_t)child, t, child = child);
                if (child >= 0) {                        // continue below the linked node
                    rec = link_of(P.nd, child);
                    node = child;
                    bnode = child;
                    state = LS_DESCEND;
                } else {
                    float es[N];
                    check_end<N>(s, es);                 // MCTS.py:125
                    bool any = false;
#pragma unroll
                    for (int i = 0; i < N; i++) any |= es[i] != 0.f;
                    if (any) {
                        kind = LEAF_TERMINAL;
#pragma unroll
                        for (int i = 0; i < N; i++) val[i] = es[i];
                        const int id = hnc;
                        const int g = node_slot(P, H, t, id, &hnpg);
                        if (g < 0) {                     // no room: back up, do not store
                            H->unexpanded += 1;
                        } else {
                            P.nkey0[g] = k0; P.nkey1[g] = k1;
                            P.nd[g] = term_node(val, (uint8_t)bt(row(s, 0), 6));
                            hash_insert(P, t, k0, g);
                            if (cached) { P.nd[node].h.bchild = g; P.nd[node].h.babt = (uint16_t)(pk.a | (1 << 15)); }
                            H->node_count = id + 1;
                            hnc = id + 1;
                        }
                        leaf_node = g;
                    }
                    state = LS_DONE;                     // terminal, or a new NN leaf
                }
            }
        }
        SPROBE(3)
    }
    if (tv_node >= 0) term_values(P, tv_node, val);
    if (act && root < 0) lane_fingerprint<N>(s, k0, k1);   // the root itself is the leaf
    if (act && kind == LEAF_NN) {                        // its board for k_leaf_mask / the network
        for (int u = 0; u < Conv<N>::UNITS; u++) Conv<N>::store(leaf_state + (size_t)t * Lx::S, s, u);
        int g = -1;
        if (P.nbrd) {                                    // the slot k_backup will insert it at
            g = node_slot(P, H, t, hnc, &hnpg);
            if (g >= 0) {
                u32x4 *dst = reinterpret_cast<u32x4 *>(P.nbrd + (size_t)g * NodeBoard<N>::BYTES);
                static_assert(NodeBoard<N>::BYTES % 16 == 0, "node boards: 16-byte stores");
#pragma unroll
                for (int r = 0; r < Lx::ROWS; r += 2) {      // (two rows per 16-byte store)
                    const uint64_t a = row(s, r), b = r + 1 < Lx::ROWS ? row(s, r + 1) : 0;
                    dst[r >> 1] = u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
                }
            }
        }
        H->leaf_slot = g;
    }
    if (act) {
        H->depth = depth;
        H->leaf_kind = kind;
        H->leaf_hslot = kind == LEAF_NN ? miss : -1;
        if (kind != LEAF_NN) H->leaf_slot = -1;
        H->leaf_k0 = k0; H->leaf_k1 = k1;
        H->leaf_round = (uint8_t)bt(row(s, 0), 6);
#pragma unroll
        for (int i = 0; i < 4; i++) H->leaf_v[i] = val[i];
        leaf_valid[t] = kind == LEAF_NN;
        path_n[depth] = kind == LEAF_TERMINAL ? leaf_node : -1;
    }
#if SELECT_PROBE
    SPROBE(4)
    if (l == 0) {
        for (int k = 0; k < 5; k++) atomicAdd(&g_sel_probe[k], (unsigned long long)pacc[k]);
        atomicAdd(&g_sel_probe[5], 1ull);
        atomicMax(&g_sel_probe[6], (unsigned long long)(plast - pstart));
        atomicAdd(&g_sel_probe[7], (unsigned long long)(plast - pstart));
    }
    {
        const int lmax = wave_max_i32(plev);
        int lsum = plev;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o, 64);
        if (l == 0) {
            atomicAdd(&g_sel_probe[8], (unsigned long long)lmax);
            atomicAdd(&g_sel_probe[9], (unsigned long long)lsum);
            atomicMax(&g_sel_probe[10], (unsigned long long)lmax);
            atomicAdd(&g_sel_probe[11], (unsigned long long)pexp);
        }
    }
#endif
}

// ------------------------------------------------------------ leaf masks
// getValidMoves(leaf, 0) (MCTS.py:136) for every NN leaf of a select, lane per leaf, 64
// leaves per workgroup: the rollout kernel's factorised predicate and mask-word phases
// (splendor_device.h lane_predicates_part / lane_mask_word_fast, exact path for boards
// outside the fast domain), then the pass bit iff nothing else is legal (:263). Replaces
// the wave-per-board mask of the descent kernel (its lanes are idle for it anyway).
// (Until late round 6 this kernel also filed the trees whose leaf was deep into the first
// launch slots of the next select, behind one returning atomic per workgroup on a shared
// counter — 10 of its 20 us at config 3, LM_PROBE. A select's 64-lane waves are all resident
// at once, so its launch lasts as long as its deepest descent whatever the grouping: the
// select now takes tree = slot, A/B 0.4471 / 0.4462 vs 0.4486 / 0.4485 ms.)
// leaf_index / leaf_count (optional): the NN leaves for the indexed network kernel, segment by
// segment without atomics: segment j = this kernel's workgroup j (trees 64 j .. 64 j + 63) lists
// its leaves at leaf_index[64 j ..] and their number at leaf_count[j] (nn_list_rows)
// per-workgroup timestamps of the last k_leaf_mask launch (diagnostic builds only,
// -DLM_PROBE=1; never the product): s_memrealtime (100 MHz) at entry, after each of the three
// barriers and at exit
#ifndef LM_PROBE
#define LM_PROBE 0
#endif
#if LM_PROBE
constexpr int LM_PSLOTS = 4096;
__device__ unsigned long long g_lm_probe[LM_PSLOTS][8];
#define LMPROBE(k) \
    if (threadIdx.x == 0 && blockIdx.x < LM_PSLOTS) g_lm_probe[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();
#else
#define LMPROBE(k)
#endif
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
    LMPROBE(0)
    const int b0 = blockIdx.x * RB, nb = min(RB, B - b0);
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
    if (w == 2 && leaf_index) {                          // the segment's NN leaves
        const bool v = l < nb && leaf_valid[b0 + l];
        const uint64_t bv = __ballot(v);
        if (v) leaf_index[b0 + __popcll(bv & lanemask_lt())] = b0 + l;
        if (l == 0) leaf_count[blockIdx.x] = __popcll(bv);
    }
    // the boards and the mask factors: every load issued before the first LDS store (a loop of
    // load -> store pairs waits one round trip per iteration — 17 of this kernel's 19 us at
    // config 3, LM_PROBE; now one)
    constexpr int FW = (7 * 116 + 255) / 256;            // factor words per thread
    uint64_t fw[FW];
#pragma unroll
    for (int k = 0; k < FW; k++) {
        const int i = tid + 256 * k;
        fw[k] = i < 7 * 116 ? (&K_MASK_FACTORS[0][0])[i] : 0;
    }
    if constexpr (Cv::QUAD) {
        constexpr int BU = (RB * Cv::UNITS + 255) / 256;  // board units (4 rows) per thread
        uint32_t d[BU][7];
#pragma unroll
        for (int k = 0; k < BU; k++) {
            const int i = min(tid + 256 * k, nb * Cv::UNITS - 1), b = i / Cv::UNITS, u = i - b * Cv::UNITS;
            const uint32_t *g = reinterpret_cast<const uint32_t *>(leaf_state + (size_t)(b0 + b) * Lx::S) + 7 * u;
#pragma unroll
            for (int q = 0; q < 7; q++) d[k][q] = g[q];
        }
#pragma unroll
        for (int k = 0; k < BU; k++) {
            const int i = tid + 256 * k, b = i / Cv::UNITS, u = i - b * Cv::UNITS;
            if (i < nb * Cv::UNITS) quad_rows_put(d[k], reinterpret_cast<uint64_t *>(lds + b * ST) + 4 * u);
        }
    } else {
        for (int i = tid; i < nb * Cv::UNITS; i += 256) {
            const int b = i / Cv::UNITS, u = i - b * Cv::UNITS;
            Cv::load(lds + b * ST, leaf_state + (size_t)(b0 + b) * Lx::S, u);
        }
    }
#pragma unroll
    for (int k = 0; k < FW; k++)
        if (tid + 256 * k < 7 * 116) mfac[tid + 256 * k] = fw[k];
    lds_sync();
    LMPROBE(1)
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
    LMPROBE(2)
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
    LMPROBE(3)
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
    LMPROBE(4)
    for (int i = tid; i < nb * 7; i += 256)
        if (leaf_valid[b0 + i / 7]) leaf_mask[(size_t)b0 * 7 + i] = (&msk[0][0])[i];
    LMPROBE(5)
}

// k_backup_h: expansion of the NN leaf, the path backup (MCTS.py:169-176) and every path node's
// cached arg-max (NodeStat), so the next descent through the node reads its pick instead of
// scanning. Lane per level. A level's arg-max needs only its visited edges (the visit block)
// and its best unvisited edge (the run's candidate: MCTS.py:214 is monotone in P), plus the
// next unvisited edge of a smaller prior so the float32 screen can rule out a float64
// rounding tie: each lane screens its level's records (batches of BK_BATCH requested
// together) in one pass — the running maximum L of u - e with its edge, and the largest u + e
// of every other item; that is below L exactly when one edge can hold the maximum, which is
// then the strict-'>' arg-max. Otherwise (ties, near ties) and for levels with more than
// BK_WIDE records (roots) the wave evaluates the level exactly in float64.
#ifndef BK_PF
#define BK_PF 4            // visit-record heads requested together by the screen
#endif
#ifndef BK_WIDE
#define BK_WIDE 12
#endif
#ifndef BACKUP_WAVES
#define BACKUP_WAVES 4
#endif

struct Screen {
    float L1, H1, H2, cf, ff, sqv, sqe;
    int off, a, child, vi;    // the leading item: rank, action, link, visit record (-1: none)
};
__device__ __forceinline__ Screen screen_init(int ns, double qs, double cpuct, double fpu) {
    Screen S;
    S.cf = (float)cpuct;
    S.ff = (float)fpu_base(fpu, qs);
    const float nf = (float)ns;
    S.sqv = __builtin_amdgcn_sqrtf(nf);
    S.sqe = __builtin_amdgcn_sqrtf(nf + 1e-8f);
    S.L1 = -INFINITY; S.H1 = -INFINITY; S.H2 = -INFINITY;
    S.off = 0; S.a = 0; S.child = -1; S.vi = -1;
    return S;
}
// one edge's float32 UCB estimate with its error bound (|estimate - the reference's float64
// value| <= e = 2.1e-6 (|u| + |q|), tests/test_ucb_screen.py)
__device__ __forceinline__ void screen_item(Screen &S, bool vis, float p, int n, double q, int off, int a, int child,
                                            int vi = -1) {
    const float rc = vis ? __builtin_amdgcn_rcpf(1.f + (float)n) : 1.f;
    const float qf = vis ? (float)q : S.ff;
    const float uf = qf + S.cf * p * (vis ? S.sqv : S.sqe) * rc;
    const float er = 2.1e-6f * (fabsf(uf) + fabsf(qf)) + 1e-30f;
    const float lo = uf - er, hi = uf + er;
    if (lo > S.L1) {
        S.H2 = fmaxf(S.H2, S.H1); S.L1 = lo; S.H1 = hi;
        S.off = off; S.a = a; S.child = child; S.vi = vi;
    } else {
        S.H2 = fmaxf(S.H2, hi);
    }
}

// screen_item for a visited edge in branch-free form (the backup's record loop: no branch may
// separate a record's load from its use, or the compiler waits vmcnt(0) at every use and the
// prefetch is lost); a visited leader is kept by its record index only
__device__ __forceinline__ void screen_visited(Screen &S, bool valid, float p, int n, double q, int vi) {
    const float rc = __builtin_amdgcn_rcpf(1.f + (float)n);
    const float qf = (float)q;
    const float uf = qf + S.cf * p * S.sqv * rc;
    const float er = 2.1e-6f * (fabsf(uf) + fabsf(qf)) + 1e-30f;
    const float lo = uf - er, hi = uf + er;
    const bool lead = valid && lo > S.L1;
    S.H2 = valid ? fmaxf(S.H2, lead ? S.H1 : hi) : S.H2;
    S.L1 = lead ? lo : S.L1;
    S.H1 = lead ? hi : S.H1;
    S.vi = lead ? vi : S.vi;
}

// exact arg-max of one level (wave-uniform arguments): its visit records lane-parallel, the
// record `vidx` taking (n1, q1) (just written by the level's lane), and its best unvisited
// edge (uc, ac, rc; has_c) as computed by that lane. Ties: lowest action.
__device__ void exact_level(const Pools &P, int64_t vb, int vcnt, int ns, double cpuct, int vidx, int n1, double q1,
                            bool has_c, double uc, int ac, int rc, int &rank, int &act, int &child, int &rvi) {
    const int l = lane_id();
    const double sq = sqrt((double)ns);
    double bu = -INFINITY;
    int ba = 0x7fffffff, bo = 0, bc = -1, bv = -1;
    if (l == 0 && has_c) { bu = uc; ba = ac; bo = rc; }
    for (int base = 0; base < vcnt; base += 64) {
        const int k = base + l;
        if (k < vcnt) {
            const VisitRec v = *P.vr(vb + REC_UNITS * k);
            const int n = k == vidx ? n1 : v.n;
            const double q = k == vidx ? q1 : v.q;
            const double u = ucb_visited(q, n, v.p, cpuct, sq);
            if (u > bu || (u == bu && v.a < ba)) { bu = u; ba = v.a; bo = v.off; bc = v.child; bv = k; }
        }
    }
    const double mu = wave_max_f64(bu);
    const int am = wave_min_i32(bu == mu ? ba : 0x7fffffff);
    const int ln = __ffsll((unsigned long long)__ballot(bu == mu && ba == am)) - 1;
    rank = __builtin_amdgcn_readlane(bo, ln);
    act = am;
    child = __builtin_amdgcn_readlane(bc, ln);
    rvi = __builtin_amdgcn_readlane(bv, ln);
}

// per-level state of a group of path levels (lane j = level g0 + j)
struct Level {
    int node, off, act, child;  // the node, the edge taken (rank, action), the node it led to
    int ns;                     // Ns before the update
    double qs;
    NodeRun r;                  // the node's run / visit block
    int16_t ca;                 // its candidate's action (prior cp, screen bound np), its round
    uint8_t round;
    float cp, np;
    EdgeP e;                    // the edge taken
    int n;                      // its Nsa (0 without a visit record)
    double q;                   // its Qsa
    int rchild;                 // its record's link
    int grow;                   // new visit-block capacity (0: no new block needed)
    int64_t nb;                 // the new block (grow)
};

// the loads of one group: path entries, node records, the edges taken and their records
// (level d of tree t on this lane)
__device__ __forceinline__ void load_levels_at(const Pools &P, int t, int d, int depth, int lid, Level &V, bool in) {
    const int32_t *path_n = P.path_n + (size_t)t * (P.pcap + 1);
    const int32_t *path_x = P.path_x + (size_t)t * P.pcap;
    V.node = 0; V.off = 0; V.act = 0; V.child = -1; V.ns = 0; V.qs = 0.0;
    V.r = NodeRun{0, 0, 0, 0, 0, 0}; V.e = EdgeP{0.f, 0, -1}; V.n = 0; V.q = Q_UNSET; V.rchild = -1;
    V.grow = 0; V.nb = -1; V.ca = 0; V.round = 0; V.cp = 0.f; V.np = -1.f;
    if (!in) return;
    V.node = path_n[d];
    const int px = path_x[d];
    V.child = d + 1 < depth ? path_n[d + 1] : lid;
    V.off = px_off(px); V.act = px_action(px);
    const Node nd = P.nd[V.node];                        // the level's one record (64 bytes)
    V.ns = nd.h.ns; V.qs = nd.h.qs; V.round = nd.h.round;
    V.r = run_of(nd.c);
    V.ca = nd.c.ca; V.cp = nd.c.cp; V.np = nd.c.np;
    // the path edge is the node's cached pick (the descent followed it) unless the root
    // level scanned: its visit record is then known without the EdgeP (whose prior only a
    // new record needs)
    if (nd.h.best == V.off && nd.h.bvi >= 0) V.e = EdgeP{0.f, (int16_t)V.act, nd.h.bvi};
    else V.e = *P.ep(V.r.eb + V.off);
    if (V.e.vi >= 0) {
        const VisitRec v = *P.vr(V.r.vb + REC_UNITS * V.e.vi);
        V.n = v.n; V.q = v.q; V.rchild = v.child;
    } else if (V.r.vcnt == V.r.vcap) {
        // blocks double; a root's takes room for every edge at once (a root gains visited
        // edges fastest, and its block then never moves again during the search)
        V.grow = d == 0 ? (int)V.r.ec : (V.r.vcap == 0 ? 1 : min(2 * (int)V.r.vcap, (int)V.r.ec));
    }
}

// pass A's view of a deeper group's level d: the new visit-block capacity its backup needs
// (load_levels_at's V.grow) from the fields that decide it only
__device__ __forceinline__ int grow_at(const Pools &P, int t, int d, bool in) {
    if (!in) return 0;
    const int node = P.path_n[(size_t)t * (P.pcap + 1) + d];
    const int off = px_off(P.path_x[(size_t)t * P.pcap + d]);
    const Node *nd = P.nd + node;
    const int best = nd->h.best, bvi = nd->h.bvi;
    const uint64_t ebq = nd->c.ebq, vbq = nd->c.vbq;
    const int ec = nd->c.ec, vcap = (int)(ebq >> 48), vcnt = (int)(vbq >> 48);
    const int vi = best == off && bvi >= 0 ? bvi : P.ep((int64_t)(ebq & LOW48) + off)->vi;
    if (vi >= 0 || vcnt != vcap) return 0;
    return d == 0 ? ec : (vcap == 0 ? 1 : min(2 * vcap, ec));
}

// per-phase cycle probes of k_backup_h (diagnostic builds only, -DBACKUP_PROBE=1; never the
// product): per wave, s_memtime deltas summed over the waves of every launch
#ifndef BACKUP_PROBE
#define BACKUP_PROBE 0
#endif
#if BACKUP_PROBE
// one slot per wave of a launch (plain read-modify-writes: launches run one after another), so
// the probes add no atomic contention of their own; spl_diag_backup_probe sums the slots
constexpr int BK_PSLOTS = 32768;
__device__ unsigned long long g_bk_probe[BK_PSLOTS][16];
#define BPROBE(k)                                                  \
    {                                                              \
        const uint64_t c_ = __builtin_readcyclecounter();          \
        bacc[k] += c_ - blast;                                     \
        blast = c_;                                                \
    }
#else
#define BPROBE(k)
#endif

#ifndef WD_MAX
#define WD_MAX 4           // withdrawals per search (k_backup)
#endif
// ------------------------------------------------------------ backup, two trees per wave
// k_backup_h: each wave's halves back up two trees (lanes [32h, 32h + 32) on tree 2 w + h,
// lane per path level, levels in groups of 32). A wave-per-tree backup's time scales with
// the number of trees at a fixed occupancy (latency of ~15-20 dependent round trips per
// tree, 4 waves per SIMD by registers); two trees per wave double the trees in flight. Per-tree
// collective steps (the policy staging and prior sums, the sorted run, the new node's
// arg-max, allocations, the resume level) run on 32-lane halves; steps that need the whole
// wave (root noise, the exact evaluation of a level, block copies) take the two trees' items
// in turn. Same arithmetic, same order of every sum as the sequential reference.
__device__ __forceinline__ int hbase() { return lane_id() & 32; }
__device__ __forceinline__ int half_min_i32(int x) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ __forceinline__ int half_sum_i32(int x) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ double half_max_f64(double x) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        const int lo = __shfl_xor(__double2loint(x), o, 64), hi = __shfl_xor(__double2hiint(x), o, 64);
        x = fmax(x, __hiloint2double(hi, lo));
    }
    return x;
}
__device__ __forceinline__ float half_max_f32(float x) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ __forceinline__ int64_t shfl64(int64_t x, int src) {
    const int lo = __shfl((int)(uint32_t)(uint64_t)x, src, 64), hi = __shfl((int)((uint64_t)x >> 32), src, 64);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// wave_np_sum409 on a half: the same blocks and combining order, lanes hbase() + 0 .. 31
__device__ __forceinline__ float half_np_sum409(const float *a) {
    const int l = lane_id() & 31, hb = hbase();
    const int blk = (l >> 3) & 3, j = l & 7;
    const int off = blk == 0 ? 0 : (blk == 1 ? 96 : (blk == 2 ? 200 : 304));
    const int len = blk == 0 ? 96 : (blk == 3 ? 105 : 104);
    float r = a[off + j];
    for (int i = 8; i < len - (len % 8); i += 8) r += a[off + i + j];
    float r1 = __shfl_xor(r, 1, 64);
    float p01 = (j & 1) ? r1 + r : r + r1;
    float p23 = __shfl_xor(p01, 2, 64);
    float q = (j & 2) ? p23 + p01 : p01 + p23;
    float q2 = __shfl_xor(q, 4, 64);
    float res = (j & 4) ? q2 + q : q + q2;
    float blockv = __shfl(res, hb + 8 * blk, 64);
    if (blk == 3) blockv = blockv + a[off + 104];
    const float b0 = __shfl(blockv, hb, 64), b1 = __shfl(blockv, hb + 8, 64);
    const float b2 = __shfl(blockv, hb + 16, 64), b3 = __shfl(blockv, hb + 24, 64);
    return (b0 + b1) + (b2 + b3);
}
// write_sorted_run of a new node (no visit records yet) on a half: edge i's rank is the number
// of edges with a larger prior or an equal one earlier in action order. cp: 16-byte aligned,
// -inf past ec up to a multiple of 4 (never counted: priors are >= 0), read 4 at a time.
__device__ __forceinline__ void half_write_new_run(const Pools &P, int64_t eb, int ec, const float *cp,
                                                   const int16_t *ca) {
    const float4 *c4 = reinterpret_cast<const float4 *>(cp);
    const int n4 = (ec + 3) >> 2;
    for (int i = lane_id() & 31; i < ec; i += 32) {
        const float pi = cp[i];
        int r = 0;
        for (int q = 0; q < n4; q++) {
            const float4 v = c4[q];
            const int j = 4 * q;
            r += (v.x > pi) || (v.x == pi && j < i);
            r += (v.y > pi) || (v.y == pi && j + 1 < i);
            r += (v.z > pi) || (v.z == pi && j + 2 < i);
            r += (v.w > pi) || (v.w == pi && j + 3 < i);
        }
        *P.ep(eb + r) = EdgeP{pi, ca[i], (int16_t)-1};
    }
}
struct __align__(16) BkScr {           // a half's scratch: the leaf's policy and mask, its run
    float pr[416];
    float cp[416];                     // (float4 reads: -inf pads past ec)
    uint64_t bits[7];
    int16_t ca[SPL_ACTIONS];
};

template <int N, int KINDS>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(BACKUP_WAVES))) void k_backup_h(
    Pools P, SearchCfg C, int B, const uint64_t *__restrict__ leaf_mask, const float *__restrict__ pi,
    const float *__restrict__ v) {
    __shared__ BkScr scr[2 * WAVES];
    const int w = uniform(threadIdx.x >> 6), l = lane_id(), hl = l & 31, hb = l & 32, half = l >> 5;
    const int t = 2 * (blockIdx.x * WAVES + w) + half;
    const bool tv = t < B;
    TreeHdr *H = P.hdr + (tv ? t : 0);
    const int kind0 = tv ? H->leaf_kind : LEAF_NONE;
    const bool act = kind0 != LEAF_NONE && ((KINDS >> (kind0 - 1)) & 1);
    if (!__ballot(act)) return;
    bool done = !act;                                    // this half's tree has nothing (more) to do
    const int kind = act ? kind0 : LEAF_NONE;
    const int depth = act ? H->depth : 0;
    const int h_slot = H->leaf_slot, h_hslot = H->leaf_hslot, h_round = H->leaf_round;
    const uint64_t h_k0 = H->leaf_k0, h_k1 = H->leaf_k1;
    const int h_sims = H->sims_done, h_noise = H->noise_pending, h_gc = H->gc_state;
    AllocState al = alloc_state(H);                      // (used by the tree's lane 0 / 32)
    int h_nc = H->node_count, h_npg = H->npg;
    const int32_t *path_n = P.path_n + (size_t)(tv ? t : 0) * (P.pcap + 1);
    float val[4] = {0, 0, 0, 0};
    int lid = -1;
    BkScr &S = scr[2 * w + half];
    // the leaf's policy and mask: loaded here, staged in LDS after pass A's loads are issued
    // (an LDS store would wait for them first: one round trip less per tree)
#ifndef BK_DEFER_PI
#define BK_DEFER_PI 1
#endif
    float prv[13];
    uint64_t mbits = 0;
    if (kind == LEAF_NN) {
        const float *gp = pi + (size_t)t * SPL_ACTIONS;
#pragma unroll
        for (int k = 0; k < 13; k++) prv[k] = 32 * k + hl < SPL_ACTIONS ? gp[32 * k + hl] : 0.f;
        if (hl < 7) mbits = leaf_mask[(size_t)t * 7 + hl];
        if (!BK_DEFER_PI) {
#pragma unroll
            for (int k = 0; k < 13; k++)
                if (32 * k + hl < SPL_ACTIONS) S.pr[32 * k + hl] = prv[k];
            if (hl < 7) S.bits[hl] = mbits;
        }
#pragma unroll
        for (int i = 0; i < N; i++) val[i] = v[(size_t)t * N + i];
    } else if (kind == LEAF_TERMINAL) {
#pragma unroll
        for (int i = 0; i < N; i++) val[i] = H->leaf_v[i];
        lid = path_n[depth];
    }
    // The two trees' path levels packed over the wave's 64 lanes: position p < dA is tree A's
    // (half 0) level p, dA <= p < dA + dB tree B's level p - dA, 64 positions per iteration
    // (halves of 32 levels each took max(dA, dB) / 32 iterations: 1.64 per wave at config 3,
    // packed 1.31). A level lane reads its tree's values from the tree's lane 0 / 32.
    const int dA = __builtin_amdgcn_readlane(depth, 0), dB = __builtin_amdgcn_readlane(depth, 32);
    const int tA = __builtin_amdgcn_readlane(t, 0), tB = __builtin_amdgcn_readlane(t, 32);
    const int tot = dA + dB, iters = (tot + 63) >> 6;
    const auto lev = [&](int k, int &sel, int &d) {      // this lane's level in iteration k
        const int p = 64 * k + l;
        sel = p >= dA;
        d = sel ? p - dA : p;
        return p < tot;
    };
#if BACKUP_PROBE
    uint64_t bacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, blast = __builtin_readcyclecounter();
    int bexact = 0, bgroups = 0;
#endif
    // ---- pass A (as k_backup)
    Level V;
    int sel0, d0;
    const bool in0 = lev(0, sel0, d0);
    {
        const int lidA = __builtin_amdgcn_readlane(lid, 0), lidB = __builtin_amdgcn_readlane(lid, 32);
        load_levels_at(P, sel0 ? tB : tA, d0, sel0 ? dB : dA, sel0 ? lidB : lidA, V, in0);
    }
    bool fail = false;
    for (int k = 0; k < iters; k++) {
        int sel, d;
        const bool inl = lev(k, sel, d);
        const int tk = sel ? tB : tA;
        const int grow = k == 0 ? V.grow : grow_at(P, tk, d, inl);
        uint64_t gm = __ballot(grow > 0);
        int64_t nb = -1;
        while (gm) {                                     // (both trees' blocks in turn, each by
            const int j = __ffsll((unsigned long long)gm) - 1;   //  its tree's lane 0 / 32)
            gm &= gm - 1;
            const int units = REC_UNITS * __builtin_amdgcn_readlane(grow, j);
            const int owner = __builtin_amdgcn_readlane(sel, j) ? 32 : 0;
            const bool mine = hb == owner;
            int64_t b = -1;
            if (l == owner && !fail) b = unit_alloc_s(P, H, t, units, al);
            b = readlane64(b, owner);
            if (mine && b < 0) fail = true;
            if (l == j) nb = b;
        }
        if (k == 0) V.nb = nb;
        else if (grow > 0) P.path_b[(size_t)tk * P.pcap + d] = nb;
    }
    BPROBE(0)
    int g = -1, ec = 0;
    int64_t eb = -1;
    if (kind == LEAF_NN) {
        if (BK_DEFER_PI) {
#pragma unroll
            for (int k = 0; k < 13; k++)
                if (32 * k + hl < SPL_ACTIONS) S.pr[32 * k + hl] = prv[k];
            if (hl < 7) S.bits[hl] = mbits;
        }
        wave_lds_only_fence();
#pragma unroll
        for (int k = 0; k < 7; k++) ec += __popcll(S.bits[k]);
        if (!fail && hl == 0) {
            g = h_slot >= 0 ? h_slot : node_slot(P, H, t, h_nc, &h_npg);
            if (g >= 0) eb = unit_alloc_s(P, H, t, ec, al);
        }
    }
    g = __shfl(g, hb, 64);
    eb = shfl64(eb, hb);
    BPROBE(6)
    if (act && (fail || (kind == LEAF_NN && eb < 0)) && C.selfplay && depth > 0 &&
        (h_gc == 0 || h_gc == 5 || (h_gc == 2 && H->wd_search < WD_MAX))) {
        if (hl == 0) {                                   // withdrawn (see k_backup)
            H->gc_state = 1;
            H->leaf_kind = LEAF_NONE;
            H->withdrawals += 1;
            H->wd_search += 1;
            gc_push(P, H, t);
        }
        done = true;
    }
    if (!done && fail && hl == 0) H->unexpanded += 1;
    const bool expand = !done && kind == LEAF_NN && eb >= 0;
    if (!done && kind == LEAF_NN && eb < 0 && hl == 0) H->unexpanded += 1;
    // root noise on a new root (whole wave, one tree at a time)
    const bool noise = expand && depth == 0 && h_sims == 0 && h_noise;
    for (uint64_t nm = __ballot(noise && hl == 0); nm; nm &= nm - 1) {
        const int j = __ffsll((unsigned long long)nm) - 1;
        BkScr &Sj = scr[2 * w + (j >> 5)];
        root_noise_lds(C, __builtin_amdgcn_readlane(t, j), ST_DIR | (uint32_t)__builtin_amdgcn_readlane(H->move_no, j),
                       Sj.pr, Sj.bits, __builtin_amdgcn_readlane(ec, j));
    }
    // the normalisation (Ps * valids / sum, MCTS.py:117-121) of the legal priors only, as
    // the run is built (root noise normalises its own)
    float psum = 1.f;
    if (expand && !noise) psum = half_np_sum409(S.pr);
    BPROBE(7)
    if (expand) {
        float *pr = S.pr;
        int run = 0;
#pragma unroll
        for (int k = 0; k < 7; k++) {
            const uint64_t wd = S.bits[k];
#pragma unroll
            for (int hh = 0; hh < 2; hh++) {
                const int bit = 32 * hh + hl;
                if ((wd >> bit) & 1) {
                    const int r = run + __popcll(wd & ((1ull << bit) - 1));
                    S.cp[r] = noise ? pr[64 * k + bit] : pr[64 * k + bit] / psum;
                    S.ca[r] = (int16_t)(64 * k + bit);
                }
            }
            run += __popcll(wd);
        }
        if (hl < 4) S.cp[ec + hl] = -INFINITY;
        wave_lds_only_fence();
        half_write_new_run(P, eb, ec, S.cp, S.ca);
    }
    BPROBE(8)
    {                                                    // the new node's arg-max (see k_backup)
        int bsel = -1, bact = 0;
        double bu = -INFINITY;
        int ba = 0x7fffffff;
        float pm = -1.f;                                 // its candidate's prior (rank 0)
        const bool narg = expand && depth > 0;
        if (expand) {
            const double fpu_init = fpu_base(C.fpu, (double)val[0]), sq_eps = sqrt(1e-8);
            for (int i = hl; i < ec; i += 32) {
                const float p = S.cp[i];
                pm = fmaxf(pm, p);
                if (narg) {
                    const double u = ucb_unvisited(p, C.cpuct, fpu_init, sq_eps);
                    if (u > bu || (u == bu && S.ca[i] < ba)) { bu = u; ba = S.ca[i]; }
                }
            }
        }
        const double mu = half_max_f64(bu);
        bact = half_min_i32(bu == mu ? ba : 0x7fffffff);
        pm = half_max_f32(pm);
        // its rank; the candidate (rank 0: the largest prior, lowest action among equals) and
        // the screen bound np (the largest smaller prior)
        int r = 0, cam = 0x7fffffff;
        float npm = -1.f;
        if (expand) {
            const float pb = narg ? S.pr[bact] / psum : 0.f;     // (narg: depth > 0, no noise)
            for (int i = hl; i < ec; i += 32) {
                const float p = S.cp[i];
                const int a = S.ca[i];
                r += (p > pb) || (p == pb && a < bact);
                if (p == pm) cam = min(cam, a);
                else npm = fmaxf(npm, p);
            }
        }
        r = half_sum_i32(r);
        cam = half_min_i32(cam);
        npm = half_max_f32(npm);
        if (narg) bsel = r;
        else bact = 0;
        BPROBE(9)
        if (expand && hl == 0) {
            P.nkey0[g] = h_k0; P.nkey1[g] = h_k1;
            Node nn;
            nn.h.bchild = -1; nn.h.h2 = -1; nn.h.h3 = -1;
            nn.h.set_pick(bsel, bact, 0); nn.h.ns = 0;
            nn.h.term = 0; nn.h.round = (uint8_t)h_round; nn.h.bvi = -1;
            nn.h.qs = (double)val[0];
            nn.c.set_eb(eb, 0); nn.c.set_vb(0, 0);
            nn.c.ec = (int16_t)ec; nn.c.cand = 0; nn.c.ca = (int16_t)cam; nn.c.pad = 0;
            nn.c.cp = pm; nn.c.np = pm > 0.f ? npm : -1.f;
            P.nd[g] = nn;
            if (h_hslot >= 0) P.hslot[(size_t)t * P.hcap + h_hslot] = g;
            else hash_insert(P, t, h_k0, g);
            if (depth == 0) H->root = g;
            H->node_count = h_nc + 1;
        }
        if (expand) lid = g;
    }
    // per-tree values of the level lanes (after the expansion and the withdrawals)
    const int lidA = __builtin_amdgcn_readlane(lid, 0), lidB = __builtin_amdgcn_readlane(lid, 32);
    const int kindA = __builtin_amdgcn_readlane(kind, 0), kindB = __builtin_amdgcn_readlane(kind, 32);
    const int doneA = __builtin_amdgcn_readlane((int)done, 0), doneB = __builtin_amdgcn_readlane((int)done, 32);
    float valA[4], valB[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        valA[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(val[i]), 0));
        valB[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(val[i]), 32));
    }
    if (in0 && !(sel0 ? doneB : doneA) && (sel0 ? kindB : kindA) == LEAF_NN && d0 == (sel0 ? dB : dA) - 1)
        V.child = sel0 ? lidB : lidA;                    // (the new leaf below its parent's level)
    BPROBE(1)
    // ---- pass B (as k_backup), the packed levels 64 per iteration
    int moved = 0x7fffffff, n_wide_lo = 0, n_wide_hi = 0, n_big_lo = 0, n_big_hi = 0;
    for (int k = 0; k < iters; k++) {
        int sel, d;
        const bool inl = lev(k, sel, d);
        const int tk = sel ? tB : tA, depk = sel ? dB : dA, kk = sel ? kindB : kindA, lk = sel ? lidB : lidA;
        const bool in = !(sel ? doneB : doneA) && inl;
        const uint64_t selm = __ballot(sel);             // (tree B's lanes)
        if (k > 0) {
            load_levels_at(P, tk, d, depk, lk, V, in);
            if (in && V.grow > 0) V.nb = P.path_b[(size_t)tk * P.pcap + d];
        }
        const bool reloc = in && V.e.vi < 0 && V.grow > 0 && V.nb >= 0 && V.r.vcnt > 0;
        {                                                // (per-tree counts, in SGPRs)
            const uint64_t bm = __ballot(reloc && V.grow >= 128);
            n_big_lo += __popcll(bm & ~selm); n_big_hi += __popcll(bm & selm);
        }
        for (uint64_t gm = __ballot(reloc); gm; gm &= gm - 1) {
            const int j = __ffsll((unsigned long long)gm) - 1;
            const int64_t ob = readlane64(V.r.vb, j), nb = readlane64(V.nb, j);
            const int nu = REC_UNITS * __builtin_amdgcn_readlane((int)V.r.vcnt, j);
            for (int k = l; k < nu; k += 64) P.eu[nb + k] = P.eu[ob + k];
        }
        // (no fence, round 6: the screen below reads the block as it was before this level's
        // update — a moved block's old copy stays until the tree's next collection — so only
        // the exact evaluation, which reads other lanes' records, waits for these stores)
        const int64_t ovb = V.r.vb;
        const int ovc = V.r.vcnt;
        int n1 = 0, vidx = -1, nns = 0;
        double q1 = 0.0, nqs = 0.0;
        if (in) {
            const int rot = (depk - d) % N, vi = (N - rot) % N;
            float vr = sel ? valB[0] : valA[0];
#pragma unroll
            for (int i = 1; i < N; i++) vr = vi == i ? (sel ? valB[i] : valA[i]) : vr;
            const double v0 = (double)vr;
            nqs = ((double)(V.ns + 1) * V.qs + v0) / (double)(V.ns + 2);
            nns = V.ns + 1;
            q1 = ((double)V.n * V.q + v0) / (double)(V.n + 1);
            n1 = V.n + 1;
            if (V.e.vi >= 0) {
                vidx = V.e.vi;
                VisitRec *R = P.vr(V.r.vb + REC_UNITS * vidx);
                R->q = q1;
                R->n = n1;
                if (V.rchild < 0 && V.child >= 0) R->child = V.child;
            } else if (V.grow > 0 && V.nb < 0) {
                vidx = -1;
            } else {
                if (V.grow > 0) {
                    V.r.vb = V.nb;
                    V.r.vcap = (int16_t)V.grow;
                }
                vidx = V.r.vcnt;
                *P.vr(V.r.vb + REC_UNITS * vidx) = VisitRec{q1, n1, V.e.p, V.child, (int16_t)V.off, (int16_t)V.act};
                P.ep(V.r.eb + V.off)->vi = (int16_t)vidx;
                V.r.vcnt = (int16_t)(vidx + 1);
                // (a record elsewhere leaves np an upper bound: the screen stays exact)
                if (V.off == V.r.cand) {
                    int cd, ca;
                    lane_cand(P, V.r.eb, V.r.ec, V.off + 1, cd, ca, V.cp, V.np);
                    V.r.cand = (int16_t)cd; V.ca = (int16_t)ca;
                }
                NodeCold c;                              // the record's second half (run / block)
                c.set_eb(V.r.eb, V.r.vcap); c.set_vb(V.r.vb, V.r.vcnt);
                c.ec = (int16_t)V.r.ec; c.cand = (int16_t)V.r.cand; c.ca = (int16_t)V.ca; c.pad = 0;
                c.cp = V.cp; c.np = V.np;
                P.nd[V.node].c = c;
            }
            V.rchild = V.rchild >= 0 ? V.rchild : V.child;
        }
        BPROBE(2)
#if BACKUP_PROBE
        bgroups++;
#endif
        const bool wide = in && V.r.vcnt > BK_WIDE;
        {
            const uint64_t wm = __ballot(wide && d > 0);
            n_wide_lo += __popcll(wm & ~selm); n_wide_hi += __popcll(wm & selm);
        }
        Screen Sc = screen_init(nns, nqs, C.cpuct, C.fpu);
        bool has_c = false;
        double uc = 0.0;
        int ac = 0, rc = 0;
        if (in && V.r.cand < V.r.ec) {                  // the best unvisited edge, and the bound
            has_c = true;                                // on every other one (cached in the record)
            rc = V.r.cand; ac = V.ca;
            screen_item(Sc, false, V.cp, 0, 0.0, rc, V.ca, -1);
            if (V.np >= 0.f) screen_item(Sc, false, V.np, 0, 0.0, 0, 0, -1);   // (never leads: np < cp)
        }
        // the level's visit records (round 6): only their 16-byte heads {Qsa, Nsa, P}, BK_PF
        // requested ahead (round 5 waited one round trip per record); a visited leader is kept
        // by index, its link / rank / action read afterwards (only when it is not the path edge,
        // whose values the lane holds)
        // (the block before the update, ovb: records [0, ovc); a new record, index ovc, is the
        // level's own — its values are the lane's)
        const int myv = in && !wide ? V.r.vcnt : 0;
        const int maxv = wave_max_i32(myv);
        {
            const int64_t vb0 = myv && ovc ? ovb : 0;
            const auto head = [&](int i) { return *P.vh(vb0 + REC_UNITS * (i < myv && i < ovc ? i : 0)); };
            VisitHead hd[BK_PF];
#pragma unroll
            for (int k = 0; k < BK_PF; k++) hd[k] = head(k);
            for (int base = 0; base < maxv; base += BK_PF) {
#pragma unroll
                for (int k = 0; k < BK_PF; k++) {
                    const int i = base + k;
                    const bool mine = i == vidx;
                    screen_visited(Sc, i < myv, mine && i >= ovc ? V.e.p : hd[k].p, mine ? n1 : hd[k].n,
                                   mine ? q1 : hd[k].q, i);
                    hd[k] = head(base + BK_PF + k);       // (unconditional: see screen_visited)
                }
            }
        }
        if (Sc.vi >= 0) {                                // a visited leader: its link, rank, action
            if (Sc.vi == vidx) {
                Sc.off = V.off; Sc.a = V.act; Sc.child = V.rchild;
            } else {
                const VisitTail tl = *P.vt(ovb + REC_UNITS * Sc.vi);
                Sc.off = tl.off; Sc.a = tl.a; Sc.child = tl.child;
            }
        }
        bool open = in && (wide || !(Sc.H2 < Sc.L1));
        int bsel = Sc.off, bact = Sc.a, bch = Sc.child, bvi = Sc.vi;
        if (open && has_c) {
            double u;
            rc = best_unvisited(P, V.r.eb, V.r.ec, V.r.cand, C.cpuct, fpu_base(C.fpu, nqs), sqrt((double)nns + 1e-8),
                                u, ac);
            uc = u;
        }
        if (__ballot(open)) wave_lds_fence();             // (exact_level reads every lane's records)
        BPROBE(3)
#if BACKUP_PROBE
        bexact += __popcll(__ballot(open));
#endif
        for (uint64_t ex = __ballot(open); ex; ex &= ex - 1) {
            const int j = __ffsll((unsigned long long)ex) - 1;
            int rk, ak, ck, vk;
            exact_level(P, readlane64(V.r.vb, j), __builtin_amdgcn_readlane((int)V.r.vcnt, j),
                        __builtin_amdgcn_readlane(nns, j), C.cpuct, __builtin_amdgcn_readlane(vidx, j),
                        __builtin_amdgcn_readlane(n1, j), readlane_f64(q1, j),
                        __builtin_amdgcn_readlane((int)has_c, j) != 0, readlane_f64(uc, j),
                        __builtin_amdgcn_readlane(ac, j), __builtin_amdgcn_readlane(rc, j), rk, ak, ck, vk);
            if (l == j) { bsel = rk; bact = ak; bch = ck; bvi = vk; }
        }
        BPROBE(4)
        const bool stay = in && bsel == V.off;
        if (stay) { bch = V.rchild; bvi = vidx; }
        // the descent hints: a level whose pick stays on the path edge names the next two path
        // levels' new picks (lanes l + 1, l + 2: the same tree while d + 1 / d + 2 < its depth;
        // none across an iteration boundary)
        const int nb1 = __shfl(bch, min(l + 1, 63), 64), nb2 = __shfl(bch, min(l + 2, 63), 64);
        const int ns1 = __shfl((int)stay, min(l + 1, 63), 64);
        const int hh2 = stay && l < 63 && d + 1 < depk ? nb1 : -1;
        const int hh3 = hh2 >= 0 && ns1 && l < 62 && d + 2 < depk ? nb2 : -1;
        if (in) {                                        // the level's record, written once
            int bt_;
            if (stay) bt_ = kk == LEAF_TERMINAL && bch >= 0 && bch == lk;     // (the path's child:
            else bt_ = bch >= 0 ? (int)P.nd[bch].h.term : 0;                   //  terminal only as the leaf)
            NodeHot w;                                   // (the second half: written with a new record)
            w.bchild = bch; w.h2 = hh2; w.h3 = hh3;
            w.set_pick(bsel, bact, bt_); w.ns = nns;
            w.term = 0; w.round = (uint8_t)V.round; w.bvi = (int16_t)bvi;
            w.qs = nqs;
            P.nd[V.node].h = w;
        }
        {                                                // first level per tree whose pick moved
            const uint64_t mv = __ballot(in && bsel != V.off);
            const uint64_t mA = mv & ~selm, mB = mv & selm;
            const int mvA = mA ? 64 * k + __ffsll((unsigned long long)mA) - 1 : 0x7fffffff;
            const int mvB = mB ? 64 * k + __ffsll((unsigned long long)mB) - 1 - dA : 0x7fffffff;
            moved = min(moved, half ? mvB : mvA);
        }
    }
    const int n_wide = hb ? n_wide_hi : n_wide_lo, n_big = hb ? n_big_hi : n_big_lo;
    if (!done && hl == 0) {
        H->sims_done = h_sims + 1;
        H->noise_pending = 0;
        H->leaf_kind = LEAF_NONE;
        H->depth_max = max(H->depth_max, depth);
        H->depth_sum += depth;
        H->resume = min(moved, max(depth - 1, 0));
        H->sims_backed += 1;
        if (n_wide) H->exact_wide += n_wide;
        if (n_big) H->big_moves += n_big;
    }
#if BACKUP_PROBE
    BPROBE(5)
    // (the level-group iterations the two trees' levels would take packed into 64 lanes)
    const int pdv = act ? depth : 0;
    const int pdA = __builtin_amdgcn_readlane(pdv, 0), pdB = __builtin_amdgcn_readlane(pdv, 32);
    if (l == 0) {
        unsigned long long *g = g_bk_probe[(blockIdx.x * WAVES + w) % BK_PSLOTS];
        for (int k = 0; k < 10; k++) g[k] += bacc[k];
        g[12] += 1;
        g[13] += bexact;
        g[14] += bgroups;
        g[15] += (unsigned long long)((pdA + pdB + 63) / 64);
    }
#endif
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
    __shared__ uint64_t hb[WAVES][7];                    // the best actions (bitmap, action order)
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
    const NodeRun r = run_of(P.nd[root].c);
    const int sims = H->budget;
    const bool forced = H->forced;
    auto count = [&](int i, float &p, int &a) {
        const EdgeP e = *P.ep(r.eb + i);
        p = e.p; a = e.a;
        return e.vi >= 0 ? P.vr(r.vb + REC_UNITS * e.vi)->n : 0;
    };
    int best = 0;
    for (int i = l; i < r.ec; i += 64) { float p; int a; best = max(best, count(i, p, a)); }
    best = wave_max_i32(best);
    long long top = 0;
    for (int i = l; i < r.ec; i += 64) {
        float p; int a;
        const int n = count(i, p, a);
        top = max(top, pruned_count(n, best, forced, p, sims));
    }
    for (int o = 32; o > 0; o >>= 1) top = max(top, (long long)__shfl_xor(top, o, 64));
    if (top == 0) {
        if (l == 0) action[t] = (int16_t)(int)(u * (double)SPL_ACTIONS);
        return;
    }
    if (l < 7) hb[w][l] = 0;
    wave_lds_fence();
    for (int i = l; i < r.ec; i += 64) {
        float p; int a;
        const int n = count(i, p, a);
        if (pruned_count(n, best, forced, p, sims) == top)
            atomicOr(reinterpret_cast<unsigned long long *>(&hb[w][a >> 6]), 1ull << (a & 63));
    }
    wave_lds_fence();
    int nbest = 0;
#pragma unroll
    for (int j = 0; j < 7; j++) nbest += __popcll(hb[w][j]);
    const int k = (int)(u * (double)nbest);              // k-th best in action order
    if (l == 0) action[t] = (int16_t)action_at(hb[w], k);
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
    const NodeRun r = run_of(P.nd[root].c);
    int best = 0;
    for (int i = l; i < r.ec; i += 64) {
        const EdgeP e = *P.ep(r.eb + i);
        best = max(best, e.vi >= 0 ? P.vr(r.vb + REC_UNITS * e.vi)->n : 0);
    }
    best = wave_max_i32(best);
    const int sims = H->budget;
    const bool forced = H->forced;
    long long tot = 0;
    for (int i = l; i < r.ec; i += 64) {
        const EdgeP e = *P.ep(r.eb + i);
        int cn = 0;
        double cq = Q_UNSET;
        if (e.vi >= 0) {
            const VisitRec v = *P.vr(r.vb + REC_UNITS * e.vi);
            cn = v.n; cq = v.q;
        }
        const long long c = pruned_count(cn, best, forced, e.p, sims);
        if (counts) counts[(size_t)t * SPL_ACTIONS + e.a] = cn;
        if (adjusted) adjusted[(size_t)t * SPL_ACTIONS + e.a] = c;
        if (qsa) qsa[(size_t)t * SPL_ACTIONS + e.a] = cq;
        tot += c;
    }
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    for (int i = l; i < r.ec; i += 64) {
        const EdgeP e = *P.ep(r.eb + i);
        const int cn = e.vi >= 0 ? P.vr(r.vb + REC_UNITS * e.vi)->n : 0;
        const long long c = pruned_count(cn, best, forced, e.p, sims);
        if (probs) probs[(size_t)t * SPL_ACTIONS + e.a] = (double)c / (double)tot;
    }
    if (q && l == 0) {
        const double q0 = P.nd[root].h.qs;
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
    const NodeRun r = run_of(P.nd[root].c);
    for (int i = l; i < r.ec; i += 64) {
        const EdgeP e = *P.ep(r.eb + i);
        o[e.a] = e.p;
    }
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
// edge units (runs and visit records). Diagnostic (capacity planning), one wave per tree.
__global__ __launch_bounds__(64) void k_tree_sizes(Pools P, int B, int32_t *out) {
    const int t = blockIdx.x;
    if (t >= B) return;
    const int l = lane_id();
    const TreeHdr *H = P.hdr + t;
    const int nc = H->node_count, root = H->root;
    const int rr = root >= 0 ? P.nd[root].h.round : 1 << 30;
    int ln = 0, le = 0;
    for (int i = l; i < nc; i += 64) {
        const int g = node_g(P, t, i);
        const Node nd = P.nd[g];
        if (g == root || nd.h.round > rr) {
            ln++;
            if (!nd.h.term) le += nd.c.ec + REC_UNITS * nd.c.vcnt();   // (content: block slack depends
        }                                                           //  on the collection history)
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
    // free stacks: every page past the home pages, lowest on top
    const int nsh = P.npages - P.nhome * B, esh = P.epages - P.ehome * B;
    for (size_t i = tid; i < (size_t)nsh; i += nth) P.nfree[i] = (int32_t)(P.npages - 1 - i);
    for (size_t i = tid; i < (size_t)esh; i += nth) P.efree[i] = (int32_t)(P.epages - 1 - i);
    if (tid == 0) { P.alloc[0] = nsh; P.alloc[1] = esh; P.alloc[2] = 0; P.alloc[3] = 0; }
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
    L.eptab = (cfg->edge_cap + UPG - 1) / UPG;
    L.nmax = L.nptab * NPG; L.emax = L.eptab * UPG;
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
    L.epages = (pe + UPG - 1) / UPG;
    const size_t nn = (size_t)L.npages * NPG, ne = (size_t)L.epages * UPG;
    const size_t nx = (size_t)B * L.excap, no = (size_t)L.out_cap;
    const int gcw = B < GC_WG ? B : GC_WG;
    size_t bytes = 0;
    auto acc = [&](size_t b) { bytes += (b + 255) & ~size_t(255); };
    acc(sizeof(TreeHdr) * B); acc(8 * nn); acc(8 * nn);
    acc(sizeof(Node) * nn); acc(8 * ne);
    acc(4 * (size_t)B * L.nptab); acc(4 * (size_t)B * L.eptab); acc(4 * (size_t)L.npages); acc(4 * (size_t)L.epages);
    acc(4 * (size_t)L.npages); acc(4 * (size_t)L.epages); acc(64);
    acc(4 * (size_t)B * L.hcap); acc(4 * (size_t)B * (L.pcap + 1)); acc(4 * (size_t)B * L.pcap); acc(8 * (size_t)B * L.pcap);
    acc(4 * (size_t)gcw * gc_ints(L.nmax, L.emax)); acc((size_t)B * L.S);
    acc((size_t)B * L.S); acc(nx * L.S); acc(4 * nx * SPL_ACTIONS); acc(16 * nx); acc(56 * nx); acc(4 * nx);
    acc(no * L.S); acc(4 * no * SPL_ACTIONS); acc(16 * no); acc(16 * no); acc(56 * no); acc(16 * no);
    acc(16 * no); acc(64); acc((size_t)L.nbb * nn); acc(4 * (size_t)B); acc(4 * (size_t)B); acc(8 * no);
    L.bytes = bytes;
    return L;
}

static bool valid_cfg(const spl_ctx *ctx, int B, const spl_mcts_config *cfg) {
    if (!(ctx && ctx->n >= 2 && ctx->n <= 4 && B > 0 && cfg && cfg->num_sims > 0 && cfg->ratio_full > 0 &&
          cfg->node_cap > 0 && cfg->edge_cap > 0 && cfg->pool_nodes >= 0 && cfg->pool_edges >= 0))
        return false;
    // global node ids are int32; page ids too
    const long long nmax = (long long)((cfg->node_cap + NPG - 1) / NPG) * NPG;
    const long long emax = (long long)((cfg->edge_cap + UPG - 1) / UPG) * UPG;
    const long long pn = cfg->pool_nodes > 0 ? cfg->pool_nodes : (long long)B * nmax;
    const long long pe = cfg->pool_edges > 0 ? cfg->pool_edges : (long long)B * emax;
    return cfg->node_cap <= (1 << 24) && cfg->edge_cap <= (1 << 28) && pn + NPG < (1LL << 31) &&
           pe / UPG + 1 < (1LL << 31);
}

#if SELECT_PROBE
// k_select_lanes phase probes: [0] prologue [1] descents [2] board staging [3] expansions
// [4] leaf outputs (cycles summed over waves), [5] waves, [6] max wave cycles, [7] total,
// [8] the deepest lane's levels summed over waves, [9] levels of all lanes, [10] most levels of
// one lane, [11] expansion rounds summed over waves
int spl_diag_select_probe(unsigned long long *out16, int reset) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_sel_probe), 16 * 8) != hipSuccess) return SPL_EDEVICE;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sel_probe), z, sizeof(z)) != hipSuccess) return SPL_EDEVICE;
    }
    return 0;
}
#endif

#if GC_PROBE
// compact_tree phase probes (cycles summed over collections): [0] keep / remap scan [1] sizes +
// page packing [2] node records moved [3] arg-max links + owner map [4] unit staging [5]
// write-back + node boards [6] table rebuild + pages; [8] collections [9] total cycles [10]
// the slowest collection's cycles, [11] its units, [12] its kept nodes, [13] its nodes before
int spl_diag_gc_probe(unsigned long long *out24, int reset) {
    static unsigned long long h[GC_WG_MAX_PROBE][16], hm[GC_WG_MAX_PROBE][8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_gc_probe), sizeof(h)) != hipSuccess) return SPL_EDEVICE;
    if (hipMemcpyFromSymbol(hm, HIP_SYMBOL(g_gc_probe_max), sizeof(hm)) != hipSuccess) return SPL_EDEVICE;
    for (int k = 0; k < 24; k++) out24[k] = 0;
    for (int i = 0; i < GC_WG_MAX_PROBE; i++) {
        for (int k = 0; k < 10; k++) out24[k] += h[i][k];
        if (h[i][10] > out24[10]) {
            for (int k = 10; k < 14; k++) out24[k] = h[i][k];
            for (int k = 0; k < 7; k++) out24[16 + k] = hm[i][k];   // [16 ..] its phases
        }
    }
    if (reset) {
        memset(h, 0, sizeof(h));
        memset(hm, 0, sizeof(hm));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_gc_probe), h, sizeof(h)) != hipSuccess) return SPL_EDEVICE;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_gc_probe_max), hm, sizeof(hm)) != hipSuccess) return SPL_EDEVICE;
    }
    return 0;
}
#endif

#if LM_PROBE
// the last k_leaf_mask launch's per-workgroup timestamps (LM_PSLOTS x 8)
int spl_diag_lm_probe(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lm_probe), sizeof(g_lm_probe)) == hipSuccess ? 0 : SPL_EDEVICE;
}
#endif

#if BACKUP_PROBE
// k_backup_h phase probes (cycles summed over waves): [0] header + pass A [1] expansion's node
// record / table insert [2] pass B loads / updates [3] screen [4] exact levels [5] record writes
// + end, expansion's [6] allocations [7] noise + normalisation [8] sorted run [9] arg-max; [12]
// waves, [13] levels evaluated exactly, [14] level groups
int spl_diag_backup_probe(unsigned long long *out16, int reset) {
    static unsigned long long h[BK_PSLOTS][16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bk_probe), sizeof(h)) != hipSuccess) return SPL_EDEVICE;
    for (int k = 0; k < 16; k++) out16[k] = 0;
    for (int i = 0; i < BK_PSLOTS; i++)
        for (int k = 0; k < 16; k++) out16[k] += h[i][k];
    if (reset) {
        memset(h, 0, sizeof(h));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_bk_probe), h, sizeof(h)) != hipSuccess) return SPL_EDEVICE;
    }
    return 0;
}
#endif

#if SPL_BOUNDS_CHECK
// bounds-checked builds only: [0] violations, [1] first value, [2] its site, [3] its tree
int spl_diag_bounds(unsigned long long *out4, int reset) {
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_bounds), 68 * 8) != hipSuccess) return SPL_EDEVICE;
    if (reset) {
        unsigned long long z[68] = {0};
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
    C.edge_reserve = 48;                                  // units: a new node's run (~20 edges) +
                                                          // visit records and their growth
    Pools &P = m->P;
    const Plan L = plan_pools(ctx->n, B, cfg);
    P.nmax = L.nmax; P.emax = L.emax; P.hcap = L.hcap; P.pcap = L.pcap;
    P.nptab = L.nptab; P.eptab = L.eptab;
    P.npages = (int)L.npages; P.epages = (int)L.epages;
    // home pages: at most a quarter of each pool, SPL_HOME_N / SPL_HOME_E per tree
    P.ntrees = B;
    P.nhome = min(min(SPL_HOME_N, P.nptab), (int)(L.npages / (4 * (long long)B)));
    while (P.nhome & (P.nhome - 1)) P.nhome &= P.nhome - 1;   // (a power of two: node_l masks)
    P.ehome = min(min(SPL_HOME_E, P.eptab), (int)(L.epages / (4 * (long long)B)));
    const size_t nn = (size_t)L.npages * NPG, ne = (size_t)L.epages * UPG;
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
    P.nd = carve<Node>(p, nn);
    P.eu = carve<uint64_t>(p, ne);                                   // EdgeP runs, VisitRec blocks
    P.ntab = carve<int32_t>(p, (size_t)B * P.nptab); P.etab = carve<int32_t>(p, (size_t)B * P.eptab);
    P.npidx = carve<int32_t>(p, (size_t)P.npages); P.epidx = carve<int32_t>(p, (size_t)P.epages);
    P.nfree = carve<int32_t>(p, (size_t)P.npages); P.efree = carve<int32_t>(p, (size_t)P.epages);
    P.alloc = carve<int32_t>(p, 16);
    P.hslot = carve<int32_t>(p, (size_t)B * P.hcap);
    P.path_n = carve<int32_t>(p, (size_t)B * (P.pcap + 1));
    P.path_x = carve<int32_t>(p, (size_t)B * P.pcap);
    P.path_b = carve<int64_t>(p, (size_t)B * P.pcap);
    P.gc_stride = gc_ints(P.nmax, P.emax);
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
    P.gcq2 = carve<int32_t>(p, (size_t)B);
    P.flq = carve<int2>(p, no);
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
    SPL_DISPATCH(m->n, hipLaunchKernelGGL(k_select_lanes<N>, dim3((unsigned)((m->B + 63) / 64)), dim3(64), 0,
                                          (hipStream_t)hs, m->P, m->cfg, m->B, m->token_limit,
                                          leaf_state, leaf_valid));
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
    const bool defer_gc = (kinds & SPL_BACKUP_DEFER_GC) != 0;
    kinds &= ~SPL_BACKUP_DEFER_GC;
    if (!m || kinds < 1 || kinds > 3 || ((kinds & SPL_LEAF_NN) && (!leaf_mask || !pi || !v))) return SPL_EINVAL;
    const dim3 grid = wave_grid((m->B + 1) / 2);
    if (kinds == 3) {
        SPL_DISPATCH(m->n, hipLaunchKernelGGL((k_backup_h<N, 3>), grid, dim3(THREADS), 0, (hipStream_t)hs, m->P,
                                              m->cfg, m->B, leaf_mask, pi, v));
    } else if (kinds == SPL_LEAF_NN) {
        SPL_DISPATCH(m->n, hipLaunchKernelGGL((k_backup_h<N, 1>), grid, dim3(THREADS), 0, (hipStream_t)hs, m->P,
                                              m->cfg, m->B, leaf_mask, pi, v));
    } else {
        SPL_DISPATCH(m->n, hipLaunchKernelGGL((k_backup_h<N, 2>), grid, dim3(THREADS), 0, (hipStream_t)hs, m->P,
                                              m->cfg, m->B, leaf_mask, pi, v));
    }
    // trees whose simulation was withdrawn (NN leaves only; deferred: the caller's commit
    // collects them before the next select)
    if (m->cfg.selfplay && (kinds & SPL_LEAF_NN) && !defer_gc) launch_gc(m, (hipStream_t)hs);
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
    out4[0] = m->P.npages; out4[1] = m->P.epages; out4[2] = NPG; out4[3] = UPG;
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
