// splendor_env.hip — batched Splendor environment kernels for gfx950 + the C ABI
// declared in include/splendor_amd.h.
//
// Mapping: one 64-lane wave per board, 4 boards per 256-thread workgroup; each wave stages
// its board in its own LDS slot (Lay<N>::LS bytes, 8-byte rows), so boards never share LDS
// and no workgroup barrier is needed (waves exit independently). The fused rollout kernel
// instead owns 64 boards per workgroup (see k_rollout). Device logic: splendor_device.h.
#include <hip/hip_runtime.h>

#include <new>

#include "../../include/splendor_amd.h"

#ifndef ROLLOUT_ABLATE
#define ROLLOUT_ABLATE 0   // diagnostic builds only (tools/ablate_rollout.hip): 1 = skip mask, 2 = skip move
#endif
#ifndef ROLLOUT_PRIO
#define ROLLOUT_PRIO 1     // k_rollout: raise the wave priority of each phase's longest pipeline (0 = off, A/B)
#endif
#ifndef ROLLOUT_TIMING
#define ROLLOUT_TIMING 0   // diagnostic builds only (tools/time_rollout.hip): per-block cycle totals
#endif
#if ROLLOUT_TIMING
// block-shared cycle accumulators; SPL_PROBE(k) charges the cycles since the previous probe
// to slot k (thread 0's view; in product builds SPL_PROBE expands to nothing)
__shared__ uint64_t spl_probe_acc[32];
__shared__ uint64_t spl_probe_last;
#define SPL_PROBE(k)                                                                       \
    if (threadIdx.x == 0) {                                                                \
        const uint64_t c_ = clock64();                                                     \
        spl_probe_acc[k] += c_ - spl_probe_last;                                           \
        spl_probe_last = c_;                                                               \
    }
__device__ uint64_t *g_rollout_timing;
#endif
#include "splendor_device.h"

using namespace spl;

struct spl_ctx {
    int n;
    int token_limit;
};

namespace {

constexpr int WAVES = 4;            // boards per workgroup
constexpr int THREADS = 64 * WAVES;

// ---------------------------------------------------------------- kernels
template <int N>
__global__ __launch_bounds__(THREADS) void k_init(int B, int8_t *__restrict__ state,
                                                  int8_t *__restrict__ player,
                                                  const double *__restrict__ u, int ustride,
                                                  uint64_t seed, uint32_t stream, uint32_t bbase) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    __shared__ double ub[WAVES][DEAL_DRAWS];
    const int w = threadIdx.x >> 6, b = blockIdx.x * WAVES + w;
    if (b >= B) return;
    int8_t *s = lds[w];
    const double *du = u ? u + (size_t)b * ustride : ub[w];
    if (!u) wave_philox_uniforms(ub[w], seed, bbase + (uint32_t)b, stream, 0, DEAL_DRAWS);
    wave_init_game<N>(s, du);
    wave_store_board<N>(state + (size_t)b * Lx::S, s);
    if (player && lane_id() == 0) player[b] = 0;
}

template <int N>
__global__ __launch_bounds__(THREADS) void k_valid(int B, const int8_t *__restrict__ state,
                                                   const int8_t *__restrict__ player, int lim,
                                                   uint64_t *__restrict__ mask) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    const int w = threadIdx.x >> 6, b = blockIdx.x * WAVES + w;
    if (b >= B) return;
    int8_t *s = lds[w];
    wave_load_board<N>(s, state + (size_t)b * Lx::S);
    const int p = player ? player[b] : 0;
    uint64_t m[7];
    wave_valid_moves<N>(s, p, lim, m);
    store_mask(mask + (size_t)b * 7, m);
}

template <int N>
__global__ __launch_bounds__(THREADS) void k_step(int B, int8_t *__restrict__ state,
                                                  const int8_t *__restrict__ player,
                                                  const int16_t *__restrict__ action,
                                                  int8_t *__restrict__ next_player, int det,
                                                  const double *__restrict__ u, int ustride,
                                                  uint64_t seed, uint32_t stream, uint32_t bbase,
                                                  int32_t *err) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    const int w = threadIdx.x >> 6, b = blockIdx.x * WAVES + w;
    if (b >= B) return;
    const int a = action[b];
    const int p = player ? player[b] : 0;
    if (a < 0 || a >= SPL_ACTIONS) {
        if (err && lane_id() == 0) atomicOr(err, SPL_ERR_BAD_ACTION);
        if (next_player && lane_id() == 0) next_player[b] = (int8_t)p;
        return;
    }
    int8_t *s = lds[w];
    int8_t *g = state + (size_t)b * Lx::S;
    wave_load_board<N>(s, g);
    Chance ch{u ? u + (size_t)b * ustride : nullptr, seed, bbase + (uint32_t)b, stream, 0};
    const int nxt = make_move<N>(s, a, p, det != 0, ch);
    __builtin_amdgcn_wave_barrier();
    wave_store_board<N>(g, s);
    if (next_player && lane_id() == 0) next_player[b] = (int8_t)nxt;
}

// end / score / round read ~20 bytes per board: one lane per board straight from HBM
template <int N>
__global__ __launch_bounds__(256) void k_ended(int B, const int8_t *__restrict__ state,
                                               float *__restrict__ out) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    float e[N];
    check_end_rows<N>(HbmRows{state + (size_t)b * Lay<N>::S}, e);
#pragma unroll
    for (int i = 0; i < N; i++) out[(size_t)b * N + i] = e[i];
}

template <int N>
__global__ __launch_bounds__(256) void k_score_round(int B, const int8_t *__restrict__ state,
                                                     int32_t *__restrict__ score,
                                                     int32_t *__restrict__ round) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    const int8_t *s = state + (size_t)b * Lay<N>::S;
    if (score)
#pragma unroll
        for (int p = 0; p < N; p++) score[(size_t)b * N + p] = score_rows<N>(HbmRows{s}, p);
    if (round) round[b] = (uint8_t)s[6];
}

template <int N>
__global__ __launch_bounds__(THREADS) void k_canonical(int B, const int8_t *__restrict__ state,
                                                       const int8_t *__restrict__ player,
                                                       int8_t *out) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    const int w = threadIdx.x >> 6, b = blockIdx.x * WAVES + w;
    if (b >= B) return;
    int8_t *s = lds[w];
    wave_load_board<N>(s, state + (size_t)b * Lx::S);
    const int p = player ? player[b] : 0;
    if (p) wave_roll_players<N>(s, s, p);
    wave_store_board<N>(out + (size_t)b * Lx::S, s);
}

template <int N>
__global__ __launch_bounds__(THREADS) void k_tree_step(int B, const int8_t *__restrict__ parent,
                                                       const int16_t *__restrict__ action,
                                                       int8_t *__restrict__ child, int32_t *err) {
    using Lx = Lay<N>;
    __shared__ __align__(16) int8_t lds[WAVES][Lx::LS];
    const int w = threadIdx.x >> 6, b = blockIdx.x * WAVES + w;
    if (b >= B) return;
    int8_t *s = lds[w];
    wave_load_board<N>(s, parent + (size_t)b * Lx::S);
    const int a = action[b];
    if (a < 0 || a >= SPL_ACTIONS) {
        if (err && lane_id() == 0) atomicOr(err, SPL_ERR_BAD_ACTION);
    } else {
        Chance ch{nullptr, 0, 0, 0, 0};
        const int nxt = make_move<N>(s, a, 0, true, ch);
        __builtin_amdgcn_wave_barrier();
        if (nxt) wave_roll_players<N>(s, s, nxt);
    }
    wave_store_board<N>(child + (size_t)b * Lx::S, s);
}

// Fused random-policy self-play (splendor_amd.h spl_rollout_step / spl_rollout_run).
// A 256-thread workgroup owns RB = 64 consecutive boards and keeps them in LDS, as 8-byte
// rows at an odd-qword stride (conflict-free lane-per-board ds_read_b64/ds_write_b64), for
// all K moves of the launch:
//   load     HBM -> LDS, one 4-row quad per thread (7 dwords -> 4 qwords), deck tables
//   per move t (step = step0 + t), four phases between LDS-only barriers:
//     preds  lane-per-board legality predicates on the real board for the player to move
//            (== the canonical form's mask: it only reads player p's rows), part w in wave
//            w (cards 0-5 / cards 6-11 / reserved cards, decks, conditions / colour
//            levels); wave 3 also draws Philox blocks 0-1 of every board's step stream
//            (draw 0 picks the action, 1-2 feed a deck draw)
//     mask   mask words w, w+4 in wave w (factorised words, lane_mask_word_fast)
//     select lane l < 16 of wave w = board 16w + l: pass bit (:263), uniform action draw;
//            boards filed by move kind
//     move   the masks go to HBM; wave k makes the moves of kind k (gem vectors / buy /
//            reserve / buy reserved), lane per board: chance, end check, per-move outputs;
//            then it re-deals the games its moves finished (wave-collective, draws 3..)
//   store    boards, players, game counters LDS -> HBM
#ifndef ROLLOUT_RB
#define ROLLOUT_RB 64
#endif
constexpr int RB = ROLLOUT_RB;   // boards per workgroup (<= 64: lane per board)
#define RT_MARK(k) SPL_PROBE(k)
// v of lane I of this lane's quad (DPP quad_perm broadcast; every lane must be active)
template <int I>
__device__ __forceinline__ int quad_bcast(int v) {
    return __builtin_amdgcn_update_dpp(v, v, I | I << 2 | I << 4 | I << 6, 0xF, 0xF, false);
}
template <int N>
struct RolloutLds {
    static constexpr int STRIDE = (Lay<N>::ROWS % 2 ? Lay<N>::ROWS : Lay<N>::ROWS + 1) * 8;
};

// COUNT elements of a table held in registers across the workgroup's THREADS threads:
// fetch() issues every load (clamped indices, no branch, so they all go out back to back),
// put() stores them into LDS after the other fetches
template <class T, int COUNT>
struct StageRegs {
    static constexpr int IT = (COUNT + THREADS - 1) / THREADS;
    T v[IT];
    __device__ __forceinline__ void fetch(const T *src, int tid) {
#pragma unroll
        for (int k = 0; k < IT; k++) v[k] = src[min(tid + k * THREADS, COUNT - 1)];
    }
    __device__ __forceinline__ void put(T *dst, int tid) const {
#pragma unroll
        for (int k = 0; k < IT; k++)
            if (tid + k * THREADS < COUNT) dst[tid + k * THREADS] = v[k];
    }
};

template <int N>
__global__ __launch_bounds__(THREADS) void k_rollout(int B, int K, int8_t *__restrict__ state,
                                                     int8_t *__restrict__ player, int lim,
                                                     uint64_t *__restrict__ mask_out,
                                                     int16_t *__restrict__ action_out,
                                                     float *__restrict__ ended_out,
                                                     int32_t *__restrict__ games_done,
                                                     uint64_t seed, uint32_t step0, uint32_t bbase) {
    using Lx = Lay<N>;
    using Cv = Conv<N>;
    constexpr int ST = RolloutLds<N>::STRIDE;
    constexpr int PER = RB / WAVES;
    static_assert(PER * 4 == 64, "select: four lanes per board, one wave per PER boards");
    __shared__ __align__(16) int8_t lds[RB * ST];
    __shared__ uint64_t msk[RB][7];    // legality masks (odd qword stride: conflict-free)
    __shared__ int8_t pl[RB];
    __shared__ int32_t gdone[RB];
    __shared__ double ud[RB][4];       // draws 0..3 of each board's step stream
    __shared__ double ub[WAVES][DEAL_DRAWS];
    __shared__ TabsLds tabs;
    __shared__ uint64_t mfac[7 * 116];  // K_MASK_FACTORS (lane_mask_word_fast)
    __shared__ uint32_t klist[4][RB];  // per move kind: board | action << 8 | player << 20
    __shared__ int kcount[4];
    __shared__ uint64_t pf0[WAVES][RB], pf1[RB];
    __shared__ uint32_t pcond[RB];
    __shared__ uint8_t pbad[WAVES][RB];
    __shared__ DealRec drec[2][RB];     // deals of games gd0+1, gd0+2 of every board
    __shared__ int32_t gd0[RB];
    const int b0 = blockIdx.x * RB, nb = min(RB, B - b0);
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
    int8_t *const gst = state + (size_t)b0 * Lx::S;
#if ROLLOUT_TIMING
    if (tid < 32) spl_probe_acc[tid] = 0;
    if (tid == 0) spl_probe_last = clock64();
    const uint64_t wall0 = wall_clock64();
#endif
    // prologue: every global load (boards, players, game counters, the LDS tables) is issued
    // before the first LDS store. Strided copy loops waited one L2 / HBM round trip per
    // iteration: 13 of them, 15.5 K cycles of a 20-move launch's ~210 K (tools/time_rollout).
    {
        // (the deal tasks' game counters first: vmcnt retires loads in order, so the deals
        // below wait for these alone)
        int32_t gt[2];
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int b = ((tid + j * THREADS) >> 2) % RB;
            gt[j] = games_done[b0 + min(b, nb - 1)];      // (never null: spl_rollout_run checks)
        }
        StageRegs<double, 41 * 9> q_quot;
        StageRegs<uint64_t, 240> q_cards;
        StageRegs<uint64_t, 409> q_take, q_give;
        StageRegs<int8_t, 409> q_rsv;
        StageRegs<uint64_t, 7 * 116> q_fac;
        q_quot.fetch(&K_QUOT[0][0], tid);
        q_cards.fetch(&K_CARD_ROWS[0][0], tid);
        q_take.fetch(K_ACT_TAKE, tid);
        q_give.fetch(K_ACT_GIVE, tid);
        q_rsv.fetch(K_ACT_RSV, tid);
        q_fac.fetch(&K_MASK_FACTORS[0][0], tid);
        const double recip = K_RECIP[min(tid, 8)];
        const int bi = min(tid, nb - 1);
        const int8_t p0 = player[b0 + bi];
        const int32_t g0 = games_done[b0 + bi];
        constexpr int BI = Cv::QUAD ? (RB * Cv::UNITS + THREADS - 1) / THREADS : 1;
        uint32_t d[BI][7];
        if constexpr (Cv::QUAD) {
#pragma unroll
            for (int k = 0; k < BI; k++) {              // clamped index: every load is valid
                const int i = min(tid + k * THREADS, nb * Cv::UNITS - 1), b = i / Cv::UNITS, u = i - b * Cv::UNITS;
                const uint32_t *g = reinterpret_cast<const uint32_t *>(gst + (size_t)b * Lx::S) + 7 * u;
#pragma unroll
                for (int j = 0; j < 7; j++) d[k][j] = g[j];
            }
        }
        // the next deals of every board (one for launches of 4-47 moves, two beyond),
        // computed up front by four lanes per deal (3 tiers + nobles, lane_deal_part) so that
        // ending a game costs a row expansion, not the draws; a game ending beyond them draws
        // its deal on the spot (same keys). They read the constant tables and their own game
        // counters, so they run while the loads above are in flight.
        const int pre = K >= 48 ? 2 : (K >= 4 ? 1 : 0);
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int task = tid + j * THREADS, part = task & 3, rec = task >> 2, k = rec / RB, b = rec - k * RB;
            if (task < pre * RB * 4 && b < nb)
                lane_deal_part<N>(seed, bbase + (uint32_t)(b0 + b), (uint32_t)(gt[j] + 1 + k), part, Tabs{}, drec[k][b]);
        }
        if constexpr (Cv::QUAD) {
#pragma unroll
            for (int k = 0; k < BI; k++) {
                const int i = tid + k * THREADS, b = i / Cv::UNITS, u = i - b * Cv::UNITS;
                if (i < nb * Cv::UNITS) quad_rows_put(d[k], reinterpret_cast<uint64_t *>(lds + b * ST) + 4 * u);
            }
        } else {
            for (int i = tid; i < nb * Cv::UNITS; i += THREADS) {
                const int b = i / Cv::UNITS, u = i - b * Cv::UNITS;
                Cv::load(lds + b * ST, gst + (size_t)b * Lx::S, u);
            }
        }
        if (tid < nb) {
            pl[tid] = p0;
            gdone[tid] = g0;
            gd0[tid] = g0;
        }
        if (tid < 4) kcount[tid] = 0;
        q_quot.put(&tabs.quot[0][0], tid);
        q_cards.put(&tabs.cards[0][0], tid);
        q_take.put(tabs.act_take, tid);
        q_give.put(tabs.act_give, tid);
        q_rsv.put(tabs.act_rsv, tid);
        q_fac.put(mfac, tid);
        if (tid < 9) tabs.recip[tid] = recip;
    }
    const int pre = K >= 48 ? 2 : (K >= 4 ? 1 : 0);
    // every barrier of the move loop orders LDS only: the per-move outputs are write-only
    // HBM streams, and waiting for their stores (__syncthreads) cost ~2K cycles a barrier
    lds_sync();
    RT_MARK(0)
    for (int t = 0; t < K; t++) {
        const uint32_t step = step0 + (uint32_t)t;
        const size_t ob = (size_t)t * B + b0;            // this move's output row base
        if (tid < 4) kcount[tid] = 0;                    // (last read in the previous move phase)
        // draws 0-3 of every board's step stream, on wave 3 (its predicate part is the lightest)
        // wave priority: the SIMD's other waves (the co-resident workgroup's) yield issue
        // slots to the wave on this phase's critical path (predicate part 2; buy / reserve
        // moves below): 8.17 -> 8.7 G rollouts/s, tools/ab_rollout.sh
        if (ROLLOUT_PRIO && w == 2) __builtin_amdgcn_s_setprio(1);
        if (w == 3 && l < nb) {
#pragma unroll
            for (int k = 0; k < 2; k++)
                philox_pair(seed, bbase + (uint32_t)(b0 + l), step, k, ud[l][2 * k], ud[l][2 * k + 1]);
        }
        // predicates: wave w computes part w of every board's predicate set (lane per board)
        if (ROLLOUT_ABLATE != 1 && l < nb) {
            uint64_t f0, f1;
            uint32_t cc;
            bool bad;
            const int8_t *s = lds + l * ST;
            switch (w) {
                case 0: lane_predicates_part<N, 0>(s, pl[l], lim, f0, f1, cc, bad); break;
                case 1: lane_predicates_part<N, 1>(s, pl[l], lim, f0, f1, cc, bad); break;
                case 2: lane_predicates_part<N, 2>(s, pl[l], lim, f0, f1, cc, bad); break;
                default: lane_predicates_part<N, 3>(s, pl[l], lim, f0, f1, cc, bad); break;
            }
            pf0[w][l] = f0;
            if (w == 3) pf1[l] = f1;
            if (w == 2) pcond[l] = cc;
            pbad[w][l] = bad;
        }
        if (ROLLOUT_PRIO) __builtin_amdgcn_s_setprio(0);
        RT_MARK(16)
        lds_sync();
        RT_MARK(17)
        // mask words w and w+4 of every board: factorised words from the card predicates,
        // condition bits and colour levels; boards outside the fast domain take the exact
        // predicates and the per-action descriptor words
        if (ROLLOUT_ABLATE != 1 && l < nb) {
            const bool bad = pbad[0][l] | pbad[1][l] | pbad[2][l] | pbad[3][l];
#if ROLLOUT_TIMING
            {   // diagnostic: waves that take the exact predicate path (slot 18), lanes (19)
                const uint64_t bm = __ballot(bad);
                if (l == 0 && bm) { atomicAdd((unsigned long long *)&spl_probe_acc[18], 1ull);
                                    atomicAdd((unsigned long long *)&spl_probe_acc[19], (unsigned long long)__popcll(bm)); }
            }
#endif
            if (bad) {
                const LanePred P = lane_predicates_exact<N>(lds + l * ST, pl[l], lim);
                if (w == 0) { msk[l][0] = lane_mask_word<0>(P); msk[l][4] = lane_mask_word<4>(P); }
                else if (w == 1) { msk[l][1] = lane_mask_word<1>(P); msk[l][5] = lane_mask_word<5>(P); }
                else if (w == 2) { msk[l][2] = lane_mask_word<2>(P); msk[l][6] = lane_mask_word<6>(P); }
                else { msk[l][3] = lane_mask_word<3>(P); }
            } else {
                const uint64_t F0 = pf0[0][l] | pf0[1][l] | pf0[2][l];
                const uint32_t C = pcond[l], lv = (uint32_t)pf1[l];
                if (w == 0) {
                    msk[l][0] = lane_mask_word_fast<0>(C, F0, lv, mfac);
                    msk[l][4] = lane_mask_word_fast<4>(C, F0, lv, mfac);
                } else if (w == 1) {
                    msk[l][1] = lane_mask_word_fast<1>(C, F0, lv, mfac);
                    msk[l][5] = lane_mask_word_fast<5>(C, F0, lv, mfac);
                } else if (w == 2) {
                    msk[l][2] = lane_mask_word_fast<2>(C, F0, lv, mfac);
                    msk[l][6] = lane_mask_word_fast<6>(C, F0, lv, mfac);
                } else {
                    msk[l][3] = lane_mask_word_fast<3>(C, F0, lv, mfac);
                }
            }
        }
        lds_sync();
        RT_MARK(1)
        // select: four lanes per board (board w*16 + l/4; lane q = l%4 holds mask words 2q,
        // 2q+1): quad-wide counts by DPP, then the lane whose words hold the drawn index
        // finds its bit, so no lane walks all seven words. Pass bit (:263) when nothing is
        // legal; the board is filed by move kind.
        {
            const int b = w * PER + (l >> 2), q = l & 3;
            const bool on = ROLLOUT_ABLATE != 2 && b < nb;
            uint64_t x0 = 0, x1 = 0;
            if (on) {
                x0 = msk[b][2 * q];
                if (q < 3) x1 = msk[b][2 * q + 1];
            }
            const int c0 = __popcll(x0), c = c0 + __popcll(x1);
            const int k0 = quad_bcast<0>(c), k1 = quad_bcast<1>(c), k2 = quad_bcast<2>(c), k3 = quad_bcast<3>(c);
            const int cnt = k0 + k1 + k2 + k3;
            const int pre = (q > 0 ? k0 : 0) + (q > 1 ? k1 : 0) + (q > 2 ? k2 : 0);
            int a = -1;
            if (on) {
                if (ROLLOUT_ABLATE == 1) {
                    if (q == 0) a = 30 + (int)((step + b) % 5);
                } else if (cnt == 0) {
                    if (q == 3) {
                        a = 408;
                        x0 |= 1ull << (408 - 384);
                    }
                } else {
                    const int r = (int)(ud[b][0] * (double)cnt) - pre;
                    if (r >= 0 && r < c) {
                        const bool hi = r >= c0;
                        a = 128 * q + (hi ? 64 : 0) + kth_bit64(hi ? x1 : x0, hi ? r - c0 : r);
                    }
                }
            }
            // the move's final mask goes to HBM from these registers (no LDS re-read)
            if (mask_out && on && ROLLOUT_ABLATE != 1) {
                uint64_t *mo = mask_out + (ob + b) * 7 + 2 * q;
                mo[0] = x0;
                if (q < 3) mo[1] = x1;
            }
            if (a >= 0) {
                const int kind = move_kind_of(a);
                klist[kind][atomicAdd(&kcount[kind], 1)] = (uint32_t)b | (uint32_t)a << 8 | (uint32_t)pl[b] << 20;
            }
        }
        lds_sync();
        RT_MARK(5)
        // move phase. Wave w makes every move
        // of kind w (one pipeline specialisation per wave, so no wave carries the stages of
        // other kinds): chance draws 1-2, end check, outputs. Then the wave re-deals the games
        // its own moves finished (wave-collective; draws 3.. of the step stream) — mostly the
        // gem-move wave, which has the shortest pipeline, so the deals fill its wait for the
        // other kinds instead of taking a phase of their own.
#if ROLLOUT_TIMING
        const uint64_t mv0 = clock64();
#endif
        {
            int b = 0;
            bool ended = false;
            const int kc = kcount[w];
            const uint32_t ke = klist[w][l];                 // (read before the count is known)
            if (ROLLOUT_PRIO && (w == MK_BUY || w == MK_RESERVE)) __builtin_amdgcn_s_setprio(2);
            if (ROLLOUT_ABLATE != 2 && l < kc) {
                b = ke & 0xFF;
                const int a = (ke >> 8) & 0xFFF, p = ke >> 20;
                int8_t *s = lds + b * ST;
                const int r = (uint8_t)(bt(row(s, Lx::BANK), 6) + 1);   // the round after the move
                Chance ch{&ud[b][0], 0, 0, 0, 1, 0.0, false, tabs.view()};
                int nxt;
                switch (w) {
                    case MK_GEMS: nxt = make_move<N, MK_GEMS>(s, a, p, false, ch); break;
                    case MK_BUY: nxt = make_move<N, MK_BUY>(s, a, p, false, ch); break;
                    case MK_RESERVE: nxt = make_move<N, MK_RESERVE>(s, a, p, false, ch); break;
                    default: nxt = make_move<N, MK_BUY_RESERVED>(s, a, p, false, ch); break;
                }
                RT_MARK(6)
#if ROLLOUT_TIMING
                // per wave: move pipeline up to make_move's end (slots 28+w, lane 0's board)
                if (l == 0) atomicAdd((unsigned long long *)&spl_probe_acc[28 + w], (unsigned long long)(clock64() - mv0));
#endif
                float e[N];
                check_end_round<N>(s, r, e);
#pragma unroll
                for (int i = 0; i < N; i++) {
                    ended |= e[i] != 0.f;
                    ended_out[(ob + b) * N + i] = e[i];
                }
                RT_MARK(7)
                action_out[ob + b] = (int16_t)a;
                if (ended) {
                    nxt = 0;
                    gdone[b] += 1;
                }
                pl[b] = (int8_t)nxt;
            }
            RT_MARK(2)
#if ROLLOUT_TIMING
            {   // per wave: move pipeline up to the deals (24+w)
                if (l == 0) atomicAdd((unsigned long long *)&spl_probe_acc[24 + w], (unsigned long long)(clock64() - mv0));
            }
#endif
            for (uint64_t rm = __ballot(ended); rm; rm &= rm - 1) {
                const int rb = __shfl(b, __ffsll((unsigned long long)rm) - 1);
                const int g = gdone[rb];                      // the new game's number
                const int slot = g - gd0[rb] - 1;
                if (slot < pre) {
                    wave_apply_deal<N>(lds + rb * ST, drec[slot][rb], tabs.view());
                    RT_MARK(8)
                } else {
                    wave_philox_uniforms(ub[w], seed, bbase + (uint32_t)(b0 + rb), DEAL_STREAM | (uint32_t)g, 0,
                                         DEAL_DRAWS);
                    RT_MARK(9)
                    wave_init_game<N>(lds + rb * ST, ub[w], tabs.view());
                    RT_MARK(8)
                }
            }
#if ROLLOUT_TIMING
            if (l == 0) atomicAdd((unsigned long long *)&spl_probe_acc[20 + w], (unsigned long long)(clock64() - mv0));
#endif
            if (ROLLOUT_PRIO) __builtin_amdgcn_s_setprio(0);
        }
        lds_sync();
        RT_MARK(3)
    }
    for (int i = tid; i < nb * Cv::UNITS; i += THREADS) {
        const int b = i / Cv::UNITS, u = i - b * Cv::UNITS;
        Cv::store(gst + (size_t)b * Lx::S, lds + b * ST, u);
    }
    if (tid < nb) {
        player[b0 + tid] = pl[tid];
        if (games_done) games_done[b0 + tid] = gdone[tid];
    }
#if ROLLOUT_TIMING
    __syncthreads();
    RT_MARK(4)
    if (threadIdx.x == 0) {
        uint64_t *o = g_rollout_timing + (size_t)blockIdx.x * 40;   // tools/time_rollout.hip row
        for (int k = 0; k < 24; k++) o[k] = spl_probe_acc[k];
        o[24] = wall0;
        o[25] = wall_clock64();
        for (int k = 24; k < 32; k++) o[k + 2] = spl_probe_acc[k];   // o[26..29] pre-deal, o[30..33] make_move done
    }
#endif
}

// Board.get_symmetries (SplendorLogicNumba.py:349-395) for E examples, one wave per
// example. Variant k of K = 10 + 2n: 0 = identity; 1..9 = tier t = (k-1)/3 visible cards
// permuted by cards_symmetries[(k-1)%3] (SplendorLogic.py:283) with buy/reserve actions
// permuted alike; 10 + 2p + q = player p's reserved cards permuted by
// reserve_symmetries[#reserved][q] (:284-295; present only when defined), buy-reserve
// actions permuted for p == 0. present[e][k] marks emitted variants (reference order).
__constant__ int8_t K_CARD_SYM[3][4] = {{1, 3, 0, 2}, {2, 0, 3, 1}, {3, 2, 1, 0}};
__constant__ int8_t K_RSV_SYM[4][2][3] = {{{-1, -1, -1}, {-1, -1, -1}}, {{-1, -1, -1}, {-1, -1, -1}},
                                          {{1, 0, 2}, {-1, -1, -1}}, {{1, 2, 0}, {2, 0, 1}}};

template <int N>
__global__ __launch_bounds__(THREADS) void k_symmetries(int E, const int8_t *__restrict__ state,
                                                        const float *__restrict__ pi,
                                                        const uint64_t *__restrict__ valid,
                                                        int8_t *__restrict__ ostate, float *__restrict__ opi,
                                                        uint64_t *__restrict__ ovalid,
                                                        uint8_t *__restrict__ present) {
    using Lx = Lay<N>;
    constexpr int K = 10 + 2 * N;
    __shared__ __align__(16) int8_t lds[WAVES][(Lx::S + 15) & ~15];   // raw 7-byte rows
    const int w = threadIdx.x >> 6, e = blockIdx.x * WAVES + w;
    if (e >= E) return;
    const int l = lane_id();
    int8_t *s = lds[w];
    wave_copy_bytes(s, state + (size_t)e * Lx::S, Lx::S);
    int nres[N];
#pragma unroll
    for (int p = 0; p < N; p++) {        // _nb_of_reserved_cards (:770-774)
        nres[p] = 3;
        for (int c = 2; c >= 0; c--)
            if (sum5(HbmRows{s}(Lx::RSV + 6 * p + 2 * c)) == 0) nres[p] = c;
    }
    for (int k = 0; k < K; k++) {
        int tier = -1, p = -1;
        const int8_t *perm = nullptr;
        if (k >= 1 && k <= 9) { tier = (k - 1) / 3; perm = K_CARD_SYM[(k - 1) % 3]; }
        if (k >= 10) {
            p = (k - 10) / 2;
            perm = K_RSV_SYM[nres[p]][(k - 10) % 2];
            if (perm[0] < 0) { if (l == 0) present[(size_t)e * K + k] = 0; continue; }
        }
        if (l == 0) present[(size_t)e * K + k] = 1;
        int8_t *os = ostate + ((size_t)e * K + k) * Lx::S;
        // state bytes: rows of the permuted block come from the source row pair
        for (int i = l; i < Lx::S; i += 64) {
            int src = i;
            const int r = i / 7, c = i - 7 * (i / 7);
            if (tier >= 0 && r >= Lx::TIERS + 8 * tier && r < Lx::TIERS + 8 * tier + 8) {
                const int rr = r - Lx::TIERS - 8 * tier;
                src = 7 * (Lx::TIERS + 8 * tier + 2 * perm[rr >> 1] + (rr & 1)) + c;
            }
            if (p >= 0 && r >= Lx::RSV + 6 * p && r < Lx::RSV + 6 * p + 6) {
                const int rr = r - Lx::RSV - 6 * p;
                src = 7 * (Lx::RSV + 6 * p + 2 * perm[rr >> 1] + (rr & 1)) + c;
            }
            os[i] = s[src];
        }
        // policy and legality: action a takes the source action's entry
        const float *ip = pi + (size_t)e * SPL_ACTIONS;
        float *op = opi + ((size_t)e * K + k) * SPL_ACTIONS;
        const uint64_t *iv = valid + (size_t)e * 7;
#pragma unroll
        for (int ch = 0; ch < 7; ch++) {
            const int a = 64 * ch + l;
            int src = a;
            if (tier >= 0) {
                if (a >= 4 * tier && a < 4 * tier + 4) src = 4 * tier + perm[a - 4 * tier];
                if (a >= 12 + 4 * tier && a < 16 + 4 * tier) src = 12 + 4 * tier + perm[a - 12 - 4 * tier];
            }
            if (p == 0 && a >= 27 && a < 30) src = 27 + perm[a - 27];
            if (a < SPL_ACTIONS) op[a] = ip[src];
            const bool bit = a < SPL_ACTIONS && ((iv[src >> 6] >> (src & 63)) & 1);
            const uint64_t word = __ballot(bit);
            if (l == 0) ovalid[((size_t)e * K + k) * 7 + ch] = word;
        }
    }
}

// ---------------------------------------------------------------- launch helpers
inline int check_launch() { return hipGetLastError() == hipSuccess ? 0 : SPL_EDEVICE; }
inline dim3 wave_grid(int B) { return dim3((unsigned)((B + WAVES - 1) / WAVES)); }
inline dim3 lane_grid(int B) { return dim3((unsigned)((B + 255) / 256)); }
inline bool ok_ctx(const spl_ctx *c) { return c && c->n >= 2 && c->n <= 4; }

#define SPL_DISPATCH(n, CALL)            \
    switch (n) {                         \
        case 2: { constexpr int N = 2; CALL; break; } \
        case 3: { constexpr int N = 3; CALL; break; } \
        default: { constexpr int N = 4; CALL; break; } \
    }

}  // namespace

// ---------------------------------------------------------------- C ABI
extern "C" {

int spl_abi_version(void) { return SPL_ABI_VERSION; }

int spl_ctx_create(int n, int token_limit, spl_ctx **out) {
    if (!out || n < 2 || n > 4 || token_limit < 3 || token_limit > 100) return SPL_EINVAL;
    spl_ctx *c = new (std::nothrow) spl_ctx;
    if (!c) return SPL_EINVAL;
    c->n = n;
    c->token_limit = token_limit;
    *out = c;
    return 0;
}

int spl_ctx_destroy(spl_ctx *ctx) {
    delete ctx;
    return 0;
}

int spl_state_rows(const spl_ctx *c) { return ok_ctx(c) ? 32 + 10 * c->n + c->n * c->n : SPL_EINVAL; }
int spl_state_bytes(const spl_ctx *c) { return ok_ctx(c) ? 7 * spl_state_rows(c) : SPL_EINVAL; }

int spl_init(const spl_ctx *c, int B, int8_t *state, int8_t *player_out, const double *u,
             int u_stride, uint64_t seed, uint32_t stream, uint32_t board_base, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && !state) || (u && u_stride < 29)) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_init<N>, wave_grid(B), dim3(THREADS), 0,
                                          (hipStream_t)hs, B, state, player_out, u, u_stride,
                                          seed, stream, board_base));
    return check_launch();
}

int spl_valid_moves(const spl_ctx *c, int B, const int8_t *state, const int8_t *player,
                    uint64_t *mask, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && (!state || !mask))) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_valid<N>, wave_grid(B), dim3(THREADS), 0,
                                          (hipStream_t)hs, B, state, player, c->token_limit, mask));
    return check_launch();
}

int spl_step(const spl_ctx *c, int B, int8_t *state, const int8_t *player, const int16_t *action,
             int8_t *next_player, int det, const double *u, int u_stride, uint64_t seed,
             uint32_t stream, uint32_t board_base, int32_t *err, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && (!state || !action)) || (u && u_stride < 2)) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_step<N>, wave_grid(B), dim3(THREADS), 0,
                                          (hipStream_t)hs, B, state, player, action, next_player,
                                          det, u, u_stride, seed, stream, board_base, err));
    return check_launch();
}

int spl_game_ended(const spl_ctx *c, int B, const int8_t *state, float *out, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && (!state || !out))) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_ended<N>, lane_grid(B), dim3(256), 0,
                                          (hipStream_t)hs, B, state, out));
    return check_launch();
}

int spl_canonical(const spl_ctx *c, int B, const int8_t *state, const int8_t *player,
                  int8_t *out, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && (!state || !out))) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_canonical<N>, wave_grid(B), dim3(THREADS), 0,
                                          (hipStream_t)hs, B, state, player, out));
    return check_launch();
}

int spl_score(const spl_ctx *c, int B, const int8_t *state, int32_t *out, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && (!state || !out))) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_score_round<N>, lane_grid(B), dim3(256), 0,
                                          (hipStream_t)hs, B, state, out, (int32_t *)nullptr));
    return check_launch();
}

int spl_round(const spl_ctx *c, int B, const int8_t *state, int32_t *out, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && (!state || !out))) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_score_round<N>, lane_grid(B), dim3(256), 0,
                                          (hipStream_t)hs, B, state, (int32_t *)nullptr, out));
    return check_launch();
}

int spl_tree_step(const spl_ctx *c, int B, const int8_t *parent, const int16_t *action,
                  int8_t *child, int32_t *err, void *hs) {
    if (!ok_ctx(c) || B < 0 || (B && (!parent || !action || !child))) return SPL_EINVAL;
    if (!B) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_tree_step<N>, wave_grid(B), dim3(THREADS), 0,
                                          (hipStream_t)hs, B, parent, action, child, err));
    return check_launch();
}

int spl_ctx_set_token_limit(spl_ctx *c, int token_limit) {
    if (!ok_ctx(c) || token_limit < 3 || token_limit > 100) return SPL_EINVAL;
    c->token_limit = token_limit;
    return 0;
}

int spl_symmetries(const spl_ctx *c, int E, const int8_t *state, const float *pi,
                   const uint64_t *valid, int8_t *out_state, float *out_pi, uint64_t *out_valid,
                   uint8_t *present, void *hs) {
    if (!ok_ctx(c) || E < 0 || (E && (!state || !pi || !valid || !out_state || !out_pi || !out_valid ||
                                      !present)))
        return SPL_EINVAL;
    if (!E) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_symmetries<N>, wave_grid(E), dim3(THREADS), 0,
                                          (hipStream_t)hs, E, state, pi, valid, out_state, out_pi,
                                          out_valid, present));
    return check_launch();
}

int spl_rollout_run(const spl_ctx *c, int B, int K, int8_t *state, int8_t *player, uint64_t *mask_out,
                    int16_t *action_out, float *ended_out, int32_t *games_done, uint64_t seed,
                    uint32_t step0, uint32_t board_base, void *hs) {
    if (!ok_ctx(c) || B < 0 || K < 0 || (B && K && (!state || !player || !action_out || !ended_out || !games_done)))
        return SPL_EINVAL;
    if (!B || !K) return 0;
    SPL_DISPATCH(c->n, hipLaunchKernelGGL(k_rollout<N>, dim3((unsigned)((B + RB - 1) / RB)), dim3(THREADS), 0,
                                          (hipStream_t)hs, B, K, state, player, c->token_limit,
                                          mask_out, action_out, ended_out, games_done, seed,
                                          step0, board_base));
    return check_launch();
}

int spl_rollout_step(const spl_ctx *c, int B, int8_t *state, int8_t *player, uint64_t *mask_out,
                     int16_t *action_out, float *ended_out, int32_t *games_done, uint64_t seed,
                     uint32_t step, uint32_t board_base, void *hs) {
    if (B && !mask_out) return SPL_EINVAL;
    return spl_rollout_run(c, B, 1, state, player, mask_out, action_out, ended_out, games_done, seed,
                           step, board_base, hs);
}

}  // extern "C"
