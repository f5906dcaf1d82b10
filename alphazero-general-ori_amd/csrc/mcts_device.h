// mcts_device.h — device-resident batched PUCT tree (one tree per game, one wave per tree).
//
// Restates MCTS.py (search :99-177, pick_highest_UCB :199-219, backup :171-176,
// getActionProb :45-97) as three stream-ordered kernels per simulation wave:
//   select  : descend from the root with a wave arg-max over the node's CSR edges, apply
//             the deterministic in-tree transition in LDS, resolve the child through the
//             per-tree transposition table; emit one leaf per tree (NN leaf or terminal).
//   backup  : expand the NN leaf (CSR edges over legal actions, priors normalised in NumPy's
//             pairwise order), insert it, then walk the path updating Q/N with the
//             per-level value rotation (np.roll, :169).
//   commit  : (self-play) play the move, record the example, re-root, collect garbage.
// Arithmetic types follow the deployed reference: Q, Qs, UCB in float64; P float32.
#pragma once
#include "splendor_device.h"

namespace spl {

constexpr double Q_UNSET = -42.0;   // MCTS.py:9 NAN sentinel

struct TreeHdr {
    int32_t node_count, edge_count, root, sims_done;
    int32_t budget, full, noise_pending, depth;
    int32_t leaf_kind, player, episode_step, move_no;
    int32_t game_no, overflow, n_examples, leaf_round;
    uint64_t leaf_k0, leaf_k1;
    float leaf_v[4];
    int32_t games_done, forced, pad0, pad1;
};
enum { LEAF_NONE = 0, LEAF_NN = 1, LEAF_TERMINAL = 2 };

// Edge records, two 16-byte halves: what the UCB scan reads for every edge, and what is
// read only for the chosen one (loaded in the same round trip).
struct __align__(16) EdgeStat {
    float p;       // prior Ps[a] (float32)
    int32_t n;     // Nsa
    double q;      // Qsa (Q_UNSET = the reference's -42 sentinel)
};
struct __align__(16) EdgeLink {
    int16_t a;     // action
    int16_t cec;   // cached child CSR count (-1: terminal child); valid when child >= 0
    int32_t child; // child node (-1: not linked yet)
    int32_t ceb;   // cached child CSR base
    int32_t pad;
};
__device__ __forceinline__ int2 get_cr(const EdgeLink &e) { return make_int2(e.ceb, e.cec); }
__device__ __forceinline__ void set_cr(EdgeLink &e, int eb, int ec) { e.ceb = eb; e.cec = (int16_t)ec; }

// per-tree SoA pools; tree t owns [t*ncap, (t+1)*ncap) nodes, [t*ecap, ...) edges
struct Pools {
    int ncap, ecap, hcap, pcap;          // nodes, edges, hash slots (pow2), path depth
    TreeHdr *hdr;
    uint64_t *nkey0, *nkey1;
    int32_t *neb, *nec, *nns, *nround;
    double *nqs;
    int8_t *nterm;
    float *nes;                          // ncap x 4 terminal values
    EdgeStat *es;                        // UCB inputs of every edge (one 16-byte load)
    EdgeLink *el;                        // action, child and the child's cached CSR range
    int32_t *hslot;
    int32_t *path;                       // pcap x 2 (node, edge)
    int32_t *remap, *remap_eb;           // ncap scratch for compaction (new index, new CSR base)
    int8_t *root_state;                  // B x S (canonical root)
    // self-play (Coach.executeEpisode) state
    int excap, out_cap;                  // staged examples per tree, finished-example queue
    int8_t *board;                       // B x S real (non-canonical) boards
    int8_t *ex_state;                    // B x excap x S
    float *ex_pi, *ex_q;                 // B x excap x 409, B x excap x 4
    uint64_t *ex_valid;                  // B x excap x 7
    int32_t *ex_player;                  // B x excap
    int8_t *out_state;                   // out_cap x S
    float *out_pi, *out_winner, *out_q;  // out_cap x 409 / 4 / 4
    uint64_t *out_valid;                 // out_cap x 7
    int32_t *out_scdiff, *out_meta;      // out_cap x 4, out_cap x 4 (board id, game, index, player)
    int32_t *counters;                   // [0] queued examples [1] dropped
};

struct SearchCfg {
    double cpuct, fpu, dir_alpha, dir_temp, prob_full;
    int num_sims, ratio_full, forced_playouts, dirichlet;
    int temp_threshold, selfplay;
    uint64_t seed;
    uint32_t board_base;
};

// RNG streams for the search / self-play decisions (Philox counter word 2)
enum : uint32_t { ST_FULL = 1u << 24, ST_DIR = 2u << 24, ST_PICK = 3u << 24, ST_MOVE = 4u << 24,
                  ST_DEAL = 5u << 24, ST_BEST = 6u << 24 };

// --------------------------------------------------------------- wave reductions
__device__ __forceinline__ uint64_t wave_xor64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
    return x;
}

// arg-max with lowest-index tie-break (strict '>' scan order of MCTS.py:216)
__device__ __forceinline__ void wave_argmax(double &u, int &i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        double u2 = __shfl_xor(u, o, 64);
        int i2 = __shfl_xor(i, o, 64);
        if (u2 > u || (u2 == u && i2 < i)) { u = u2; i = i2; }
    }
}

// wave maximum of a double, uniform result: butterfly within each 16-lane row on DPP
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: no LDS round trips), then
// the four row maxima by readlane. Exact (max returns one of its operands).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, CTRL, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(lo, lo, CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ double wave_max_f64(double v) {
    v = fmax(v, dpp_f64<0xB1>(v));
    v = fmax(v, dpp_f64<0x4E>(v));
    v = fmax(v, dpp_f64<0x141>(v));
    v = fmax(v, dpp_f64<0x140>(v));
    const int lo = __double2loint(v), hi = __double2hiint(v);
    double r[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        r[k] = __hiloint2double(__builtin_amdgcn_readlane(hi, 16 * k), __builtin_amdgcn_readlane(lo, 16 * k));
    return fmax(fmax(r[0], r[1]), fmax(r[2], r[3]));
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// 128-bit fingerprint of the state staged in LDS (8-byte rows, zero pad byte); the
// transposition key of MCTS.py:119 (board.tobytes()). Row r enters as its 7 bytes with r
// in the pad byte. Wave-collective.
template <int N>
__device__ __forceinline__ void wave_fingerprint(const int8_t *s, uint64_t &k0, uint64_t &k1) {
    const int l = lane_id();
    uint64_t a = 0, b = 0;
    for (int i = l; i < Lay<N>::ROWS; i += 64) {
        const uint64_t x = row(s, i) | ((uint64_t)i << 56);
        a ^= mix64(x ^ 0x243F6A8885A308D3ull);
        b ^= mix64(x ^ 0x13198A2E03707344ull);
    }
    k0 = wave_xor64(a);
    k1 = wave_xor64(b) | 1ull;  // never equal to an empty key
}

__device__ __forceinline__ int hash_lookup(const Pools &P, int t, uint64_t k0, uint64_t k1) {
    const int32_t *hs = P.hslot + (size_t)t * P.hcap;
    const uint64_t *K0 = P.nkey0 + (size_t)t * P.ncap, *K1 = P.nkey1 + (size_t)t * P.ncap;
    uint32_t h = (uint32_t)(k0 ^ (k0 >> 32)) & (uint32_t)(P.hcap - 1);
    for (int probe = 0; probe < P.hcap; probe++) {
        const int c = hs[h];
        if (c < 0) return -1;
        if (K0[c] == k0 && K1[c] == k1) return c;
        h = (h + 1) & (uint32_t)(P.hcap - 1);
    }
    return -1;
}

// single-writer insert (uniform code; the wave owns the tree)
__device__ __forceinline__ void hash_insert(const Pools &P, int t, uint64_t k0, int id) {
    int32_t *hs = P.hslot + (size_t)t * P.hcap;
    uint32_t h = (uint32_t)(k0 ^ (k0 >> 32)) & (uint32_t)(P.hcap - 1);
    while (hs[h] >= 0) h = (h + 1) & (uint32_t)(P.hcap - 1);
    hs[h] = id;
}

// --------------------------------------------------------------- priors
// normalise (MCTS.py:239-242): x / np.sum(x), np.sum = NumPy pairwise float32 order over
// all 409 entries. One lane per 8-wide accumulator block; the block tree is fixed for 409.
__device__ __forceinline__ float pw_block(const float *a, int len) {
    if (len < 8) { float r = 0.f; for (int i = 0; i < len; i++) r += a[i]; return r; }
    float r[8]; int i;
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = a[j];
    for (i = 8; i < len - (len % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] += a[i + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < len; i++) res += a[i];
    return res;
}
// pairwise(409) = ((pw[0,96) + pw[96,200)) + (pw[200,304) + pw[304,409)))
__device__ __forceinline__ float np_sum409(const float *a) {
    return (pw_block(a, 96) + pw_block(a + 96, 104)) + (pw_block(a + 200, 104) + pw_block(a + 304, 105));
}

// x ** (1/T) of applyTemperatureAndNormalize (Coach.py:25) with an exactly specified
// evaluation shared with the oracle: sqrt for 1/T = 0.5, left-to-right products for small
// integer 1/T (T = 0.2 -> x^5), pow otherwise.
__host__ __device__ inline double temp_pow(double x, double T) {
    if (T == 1.0) return x;
    const double e = 1.0 / T;
    if (e == 0.5) return sqrt(x);
    const int k = (int)e;
    if ((double)k == e && k >= 1 && k <= 8) {
        double r = x;
        for (int j = 1; j < k; j++) r = r * x;
        return r;
    }
    return pow(x, e);
}

}  // namespace spl
