// mcts_device.h — device-resident batched PUCT trees (one tree per game) in a shared arena.
//
// Restates MCTS.py (search :99-177, pick_highest_UCB :199-219, backup :171-176,
// getActionProb :45-97) as stream-ordered kernels per simulation wave:
//   select  : (k_select_lanes, lane per tree) descend from the root along each node's cached
//             arg-max (one 32-byte NodeStat per level), apply the deterministic in-tree
//             transition at the expanded edge, resolve the child through the per-tree
//             transposition table; emit one leaf per tree (NN leaf or terminal).
//   backup  : (k_backup, wave per tree, lane per level) expand the NN leaf (its run of edges
//             sorted by prior, priors normalised in NumPy's pairwise order), insert it, then
//             update every path level (visit record, Ns / Qs, with the per-level value
//             rotation, np.roll :169) and recompute its cached arg-max.
//   commit  : (self-play) play the move, record the example, re-root; k_gc collects garbage.
// Arithmetic types follow the deployed reference: Q, Qs, UCB in float64; P float32.
#pragma once
#include "splendor_device.h"

namespace spl {

constexpr double Q_UNSET = -42.0;   // MCTS.py:9 NAN sentinel

struct TreeHdr {
    int32_t node_count, edge_count, root, sims_done;   // node_count: the tree's node slots in use
    int32_t budget, full, noise_pending, depth;         // (local order), edge_count: edge units in
    int32_t leaf_kind, player, episode_step, move_no;   // use (runs, visit blocks, garbage)
    int32_t game_no, overflow, n_examples, leaf_round;
    uint64_t leaf_k0, leaf_k1;
    float leaf_v[4];
    int32_t games_done, forced, moves, wd_search;   // wd_search: withdrawals in this search
    // capacity events: searches that started on a tree pruned to the nodes
    // linked from the root / on an emptied tree, and simulations whose leaf did not fit
    // (evaluated and backed up without being stored)
    int32_t prunes, resets, unexpanded, gc_state;
    int64_t units_gc;                    // edge units kept by the last collection
    int64_t enext;                       // next free unit of the tree's current edge page
    int32_t npg, epg, eleft, live_gc;    // node / edge pages held, units left in the current
                                         // edge page, nodes kept by the last collection
    int32_t root_round, gc_queued, withdrawals, gcs;   // root round (deferred GC), queued for
                                         // k_gc, simulations withdrawn for GC, collections run
    int32_t leaf_hslot, leaf_slot;       // the NN leaf's empty table slot (found by the
                                         // select's lookup) and reserved node slot, or -1
    int32_t depth_max, depth_sum;        // leaf depths of the simulations backed up: maximum, sum
    int32_t resume;                      // the next descent's first new level (k_backup: the first
                                         // path level whose cached pick moved, else the leaf's parent)
    // search-path coverage counters (cumulative; tests assert the large-budget paths ran):
    // simulations backed up, non-root levels with more than BK_WIDE visit records evaluated
    // exactly, visit blocks relocated to a capacity of at least 128 records
    int32_t sims_backed, exact_wide, big_moves;
};
static_assert(sizeof(TreeHdr) == 208, "TreeHdr layout (splendor/mcts.py HDR_DTYPE)");
// gc_state: 0 none; 1 a leaf did not fit mid-search (withdrawn, k_gc collects, the descent
// repeats); 2 collected mid-search (a further withdrawal is allowed while wd_search < WD_MAX); 3 collection before this search (must: the
// search does not fit the tree's maxima); 5 collection before this search (should: garbage
// or pool pressure; k_gc may skip it, see GC_SHOULD_CAP)
enum { LEAF_NONE = 0, LEAF_NN = 1, LEAF_TERMINAL = 2 };

// ---------------------------------------------------------------- two-tier edges
// The edge pool is a pool of 8-byte units handed out in pages of UPG units. A node owns
//   a run: one EdgeP (8 B) per legal action — what an unvisited edge needs, the prior and the
//     action — sorted by (prior descending, action ascending), so the best unvisited edge of
//     a node is its lowest-ranked edge without statistics (pick_highest_UCB, MCTS.py:214:
//     an unvisited edge's u = fpu_init + cpuct P sqrt(Ns + EPS) is monotone in P);
//   a visit block: one VisitRec (24 B = 3 units) per edge with statistics (Nsa, Qsa, the
//     link), appended on the edge's first backup; the block grows by doubling (relocated;
//     the old one is garbage until the tree's next collection).
// Measured live trees keep statistics on ~6 % of their edges, so an edge costs ~9 bytes
// instead of a full 24-byte record (what lets BASELINE config 4's trees fit).
struct EdgeP {
    float p;       // prior Ps[a] (float32)
    int16_t a;     // action
    int16_t vi;    // its VisitRec in the node's block, -1: none (Nsa = 0, Qsa = -42)
};
static_assert(sizeof(EdgeP) == 8, "EdgeP layout");
// (round 6: the fields the backup's float32 screen reads — Qsa, Nsa, the prior — are the first
// 16 bytes, one dwordx4 per record; the link, rank and action, which only the level's new pick
// needs, are the third unit)
struct VisitRec {
    double q;      // Qsa
    int32_t n;     // Nsa
    float p;       // the edge's prior (copy of its EdgeP)
    int32_t child; // link: child node (global id), -1: not linked
    int16_t off;   // its rank in the run
    int16_t a;     // its action
};
static_assert(sizeof(VisitRec) == 24, "VisitRec layout");
constexpr int REC_UNITS = 3;
constexpr int REC_LINK_UNIT = 2;   // the unit holding the link (low 32 bits), rank and action
struct VisitHead {                 // the first 16 bytes of a VisitRec
    double q;
    int32_t n;
    float p;
};
struct VisitTail {                 // its third unit
    int32_t child;
    int16_t off;
    int16_t a;
};

// A node is one 64-byte record (round 5; round 4 kept a 32-byte NodeStat, a 24-byte NodeRun, a
// round and a terminal flag in four arrays: three to four lines per path level for k_backup).
// pick_highest_UCB (MCTS.py:199-219) at a non-root node reads only that node's Ns, Qs and its
// edges' P, N, Q; all of them change only when a simulation backs up through the node (priors
// change only at a root: Dirichlet noise, :150-154; forced playouts are root-only, :157). So the
// arg-max k_backup computes right after a node's update is exactly the edge the next descent
// through the node picks: the descent follows `best` and its link (one load of the record's first
// half per level, no edge scan). The root level scans when its priors were just noised or forced
// playouts are on. Invariant (k_backup, k_select's links, k_gc's remap): bchild is the child of
// edge `best` (-1: not linked), bterm whether that child is terminal.
// Descent hints (round 5): h2 / h3 name the nodes two / three levels down along the cached
// picks as the last backup through the node saw them (k_backup_h; -1: none; k_gc clears them).
// They may be stale (a transposition's other parent moved a pick), so the descent uses them only
// as prefetch addresses, checked against the authoritative link above (descend_linked_asm).
struct NodeHot {             // first half: the descent reads its first 16 bytes per level
    int32_t bchild;          // cached arg-max's child (global id, -1: not linked)
    int32_t h2, h3;          // descent hints (-1: none)
    int16_t best;            // cached arg-max: rank of the edge in the run (-1: unknown, scan)
    uint16_t babt;           // its action | (1: that child is terminal) << 15
    int32_t ns;              // Ns
    uint8_t term;            // 1: this node is terminal (end values in NodeCold's first 16 bytes)
    uint8_t round;           // the node's round counter (GC: rounds <= the root's are garbage)
    int16_t bvi;             // the visit record of edge `best` (-1: none yet), so k_backup finds the
                             // path edge's record without loading its EdgeP
    double qs;               // Qs
    __device__ __forceinline__ int ba() const { return babt & 0x7FFF; }
    __device__ __forceinline__ int bterm() const { return babt >> 15; }
    __device__ __forceinline__ void set_pick(int rank, int a, int term_child) {
        best = (int16_t)rank;
        babt = (uint16_t)(a | (term_child << 15));
    }
};
// the descent's view of a record (NodeHot's first 16 bytes: one dwordx4 load)
struct __align__(16) NodeLink {
    int32_t bchild, h2, h3;
    int16_t best;
    uint16_t babt;
    __device__ __forceinline__ int ba() const { return babt & 0x7FFF; }
    __device__ __forceinline__ int bterm() const { return babt >> 15; }
};
constexpr uint64_t LOW48 = (1ull << 48) - 1;
struct NodeCold {            // second half: the run / visit block, the best unvisited edge
    uint64_t ebq;            // run base (global unit, 48 bits) | visit-block capacity << 48
    uint64_t vbq;            // visit-block base | visit records in use << 48
    int16_t ec;              // edges (legal actions; 0: terminal)
    int16_t cand;            // lowest rank without a visit record (ec: none) = the best unvisited edge
    int16_t ca;              // its action
    int16_t pad;
    float cp;                // its prior
    float np;                // an upper bound on the priors below cp of the unvisited edges after
                             // cand (-1: none; 0 when cp is 0): the float32 screen's bound on every
                             // other unvisited edge (equal priors tie cand and lose on the action)
    __device__ __forceinline__ int64_t eb() const { return (int64_t)(ebq & LOW48); }
    __device__ __forceinline__ int64_t vb() const { return (int64_t)(vbq & LOW48); }
    __device__ __forceinline__ int vcap() const { return (int)(ebq >> 48); }
    __device__ __forceinline__ int vcnt() const { return (int)(vbq >> 48); }
    __device__ __forceinline__ void set_eb(int64_t eb, int vcap) { ebq = (uint64_t)eb | ((uint64_t)vcap << 48); }
    __device__ __forceinline__ void set_vb(int64_t vb, int vcnt) { vbq = (uint64_t)vb | ((uint64_t)vcnt << 48); }
};
struct __align__(64) Node {
    NodeHot h;
    NodeCold c;
};
static_assert(sizeof(NodeHot) == 32 && sizeof(NodeCold) == 32 && sizeof(Node) == 64 && sizeof(NodeLink) == 16,
              "Node layout");
__device__ __forceinline__ NodeLink link_of(const Node *nd, int g) {
    return *reinterpret_cast<const NodeLink *>(&nd[g].h);
}

// a node's run / visit block in registers (the packed NodeCold unpacked)
struct NodeRun {
    int64_t eb, vb;
    int16_t ec, vcnt, vcap, cand;
};
__device__ __forceinline__ NodeRun run_of(const NodeCold &c) {
    return NodeRun{c.eb(), c.vb(), c.ec, (int16_t)c.vcnt(), (int16_t)c.vcap(), c.cand};
}

// Per-GPU shared arena. Nodes and edge units live in pools shared by all trees
// and are handed out in pages: node page = NPG consecutive global node ids, edge page = UPG
// consecutive global unit indices. A tree holds a list of node pages and a list of edge pages
// (its page tables, in allocation order) and addresses everything by GLOBAL id: child links,
// the path, the root and the transposition table hold global ids, so the descent never
// translates. A tree's "local" node index (0 .. node_count) is its allocation order (slot i =
// page ntab[i / NPG], offset i % NPG). Runs and visit blocks never straddle an edge page. Pages
// are popped from the free stacks by k_select / k_backup only and pushed back by k_gc /
// k_commit / k_set_roots / k_reset_games only, so pops and pushes never share a launch (an
// array stack with one atomic top is then exact).
constexpr int NPG_SHIFT = 6, NPG = 1 << NPG_SHIFT;     // nodes per node page
constexpr int UPG_SHIFT = 11, UPG = 1 << UPG_SHIFT;    // units per edge page (16 KB): a node's
                                                       // run + block is at most 409 x (1 + 3)
static_assert(UPG >= 4 * 409, "a node's allocation fits one edge page");

struct Pools {
    int nmax, emax, hcap, pcap;          // per tree: node slots, edge units (page tables), hash
                                         // slots, path levels
    int nptab, eptab;                    // page-table entries per tree (nmax / NPG, emax / UPG)
    int npages, epages;                  // pages in the pools
    int ntrees;                          // B
    int nhome, ehome;                    // home pages per tree (nhome a power of two or 0): tree t's page-table entries
                                         // i < nhome are node pages t nhome + i (edge pages
                                         // t ehome + i), never on the free stacks, so a tree's
                                         // first nodes and edges sit together and a wave's
                                         // consecutive trees share translations (VERDICT r04:
                                         // LIFO stacks scattered the live set over 230 GiB)
    TreeHdr *hdr;
    uint64_t *nkey0, *nkey1;             // node pool, indexed by global node id: fingerprints
    Node *nd;                            // the nodes' records
    uint64_t *eu;                        // edge unit pool (EdgeP runs, VisitRec blocks)
    int32_t *ntab, *etab;                // B x nptab / B x eptab page tables
    int32_t *npidx, *epidx;              // per page: its index in the owning tree's page table
    int32_t *nfree, *efree;              // free page stacks
    int32_t *alloc;                      // [0] / [1] free shared node / edge pages (stack tops),
                                         // [2] / [3] failed node / edge page requests
    int32_t *hslot;                      // B x hcap transposition table (global node ids)
    int32_t *path_n;                     // B x (pcap + 1) descent path: node (global id); entry
                                         // `depth` = the leaf's node when it is stored
    int32_t *path_x;                     // B x pcap the edge taken: rank | action << 9
    int64_t *path_b;                     // B x pcap k_backup scratch: a level's new visit block
    int32_t *gscr;                       // k_gc scratch, GC_WG x gc_stride ints
    size_t gc_stride;
    int8_t *nbrd;                        // per node slot its canonical board (LDS row format), or
                                         // nullptr (node_boards = 0: the descent re-applies moves)
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
    int32_t *counters;                   // [0] queued examples [1] dropped [2] GC queue
                                         // [5] example-row queue [4] k_gc workgroups done
                                         // [6] [7] unused
                                         // [8] should-collections taken by this k_gc launch
                                         // [9] deferred entries (gcq2)
    int32_t *gcq;                        // B: trees whose garbage collection k_gc runs
    int32_t *gcq2;                       // B: entries deferred to the next k_gc launch
    int2 *flq;                           // out_cap: (staging row, queue slot) rows k_gc copies

    __device__ __forceinline__ EdgeP *ep(int64_t u) const { return reinterpret_cast<EdgeP *>(eu + u); }
    __device__ __forceinline__ VisitRec *vr(int64_t u) const { return reinterpret_cast<VisitRec *>(eu + u); }
    __device__ __forceinline__ const VisitHead *vh(int64_t u) const { return reinterpret_cast<const VisitHead *>(eu + u); }
    __device__ __forceinline__ const VisitTail *vt(int64_t u) const {
        return reinterpret_cast<const VisitTail *>(eu + u + REC_LINK_UNIT);
    }
};

// tree t's local node slot i / local (virtual) unit position v -> global
// (a home page needs no table load: tree t's page i < nhome is t nhome + i; nhome is a power
// of two, so the reverse map of a home page is a mask)
__device__ __forceinline__ int node_g(const Pools &P, int t, int i) {
    const int pi = i >> NPG_SHIFT;
    const int pg = pi < P.nhome ? t * P.nhome + pi : P.ntab[(size_t)t * P.nptab + pi];
    return pg * NPG + (i & (NPG - 1));
}
__device__ __forceinline__ int node_l(const Pools &P, int g) {
    const int pg = g >> NPG_SHIFT;
    const int pi = pg < P.nhome * P.ntrees ? (pg & (P.nhome - 1)) : P.npidx[pg];
    return pi * NPG + (g & (NPG - 1));
}
__device__ __forceinline__ int64_t unit_g(const Pools &P, int t, int v) {
    const int pi = v >> UPG_SHIFT;
    const int64_t pg = pi < P.ehome ? (int64_t)t * P.ehome + pi : (int64_t)P.etab[(size_t)t * P.eptab + pi];
    return pg * UPG + (v & (UPG - 1));
}

// per-node board slot (Pools::nbrd): the LDS row format padded to 16 bytes
template <int N>
struct NodeBoard {
    static constexpr int BYTES = (Lay<N>::LS + 15) & ~15;
    static constexpr int UNITS = BYTES / 16;
};

struct SearchCfg {
    double cpuct, fpu, dir_alpha, dir_temp, prob_full;
    int num_sims, ratio_full, forced_playouts, dirichlet;
    int temp_threshold, selfplay;
    int edge_reserve;                    // edge units reserved per simulation at search start
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

// wave maximum of a float through order-preserving int keys (v_max_i32 folds the DPP row
// moves; no canonicalisation), uniform result. No NaNs; -0 < +0 here (callers compare the
// result back in float).
__device__ __forceinline__ int fkey(float x) {
    const int b = __float_as_int(x);
    return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float wave_max_f32(float x) {
    int k = fkey(x);
    k = max(k, __builtin_amdgcn_mov_dpp(k, 0xB1, 0xF, 0xF, true));   // bound_ctrl: foldable
    k = max(k, __builtin_amdgcn_mov_dpp(k, 0x4E, 0xF, 0xF, true));    // into v_max_i32_dpp
    k = max(k, __builtin_amdgcn_mov_dpp(k, 0x141, 0xF, 0xF, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, 0x140, 0xF, 0xF, true));
    const int m = max(max(__builtin_amdgcn_readlane(k, 0), __builtin_amdgcn_readlane(k, 16)),
                      max(__builtin_amdgcn_readlane(k, 32), __builtin_amdgcn_readlane(k, 48)));
    return __int_as_float(m ^ ((m >> 31) & 0x7fffffff));
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

// miss_slot (optional): on a miss, the empty slot that ended the probe — where an insert
// of this key goes while the table is unchanged
__device__ __forceinline__ int hash_lookup(const Pools &P, int t, uint64_t k0, uint64_t k1, int *miss_slot = nullptr) {
    const int32_t *hs = P.hslot + (size_t)t * P.hcap;
    const uint64_t *K0 = P.nkey0, *K1 = P.nkey1;
    uint32_t h = (uint32_t)(k0 ^ (k0 >> 32)) & (uint32_t)(P.hcap - 1);
    if (miss_slot) *miss_slot = -1;
    for (int probe = 0; probe < P.hcap; probe++) {
        const int c = hs[h];
        if (c < 0) {
            if (miss_slot) *miss_slot = (int)h;
            return -1;
        }
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

// pairwise(409) of a double-valued function of a 409-float array (NumPy's float64 pairwise
// order, the block tree of np_sum409); 32 lanes, lane = 8*block + j, uniform result.
// (the element at position p is g(p))
template <class G>
__device__ __forceinline__ double wave_np_sum409_f64_at(G g) {
    const int l = lane_id();
    const int blk = (l >> 3) & 3, j = l & 7;
    const int off = blk == 0 ? 0 : (blk == 1 ? 96 : (blk == 2 ? 200 : 304));
    const int len = blk == 0 ? 96 : (blk == 3 ? 105 : 104);
    double r = g(off + j);
    for (int i = 8; i < len - (len % 8); i += 8) r += g(off + i + j);
    const double r1 = __shfl_xor(r, 1, 64);
    const double p01 = (j & 1) ? r1 + r : r + r1;
    const double p23 = __shfl_xor(p01, 2, 64);
    const double q = (j & 2) ? p23 + p01 : p01 + p23;
    const double q2 = __shfl_xor(q, 4, 64);
    const double res = (j & 4) ? q2 + q : q + q2;
    double blockv = __shfl(res, 8 * blk, 64);
    if (blk == 3) blockv = blockv + g(off + 104);
    const double b0 = __shfl(blockv, 0, 64), b1 = __shfl(blockv, 8, 64);
    const double b2 = __shfl(blockv, 16, 64), b3 = __shfl(blockv, 24, 64);
    return (b0 + b1) + (b2 + b3);
}
template <class F>
__device__ __forceinline__ double wave_np_sum409_f64(const float *a, F f) {
    const int l = lane_id();
    const int blk = (l >> 3) & 3, j = l & 7;
    const int off = blk == 0 ? 0 : (blk == 1 ? 96 : (blk == 2 ? 200 : 304));
    const int len = blk == 0 ? 96 : (blk == 3 ? 105 : 104);
    double r = f(a[off + j]);
    for (int i = 8; i < len - (len % 8); i += 8) r += f(a[off + i + j]);
    const double r1 = __shfl_xor(r, 1, 64);
    const double p01 = (j & 1) ? r1 + r : r + r1;
    const double p23 = __shfl_xor(p01, 2, 64);
    const double q = (j & 2) ? p23 + p01 : p01 + p23;
    const double q2 = __shfl_xor(q, 4, 64);
    const double res = (j & 4) ? q2 + q : q + q2;
    double blockv = __shfl(res, 8 * blk, 64);
    if (blk == 3) blockv = blockv + f(a[off + 104]);
    const double b0 = __shfl(blockv, 0, 64), b1 = __shfl(blockv, 8, 64);
    const double b2 = __shfl(blockv, 16, 64), b3 = __shfl(blockv, 24, 64);
    return (b0 + b1) + (b2 + b3);
}

// ----------------------------------------------------------- deterministic transcendentals
// The Dirichlet sampler and the noise softmax use a logarithm / exponential built from
// + - * / only, so the device, the C oracle (oracle/splendor_oracle.c det_*) and the
// fixture generator (tests/golden/detrand.py) compute identical bits (no libm / ocml
// rounding differences; the library is built with -ffp-contract=off).
constexpr double DET_LN2_HI = 6.93147180369123816490e-01;
constexpr double DET_LN2_LO = 1.90821492927058770002e-10;
constexpr double DET_INV_LN2 = 1.44269504088896338700e+00;

__device__ inline double det_log(double x) {         // x > 0, normal
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    double m = __longlong_as_double((long long)((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull));
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    const double f = (m - 1.0) / (m + 1.0), s = f * f;
    double p = 1.0 / 23.0;
    p = p * s + 1.0 / 21.0; p = p * s + 1.0 / 19.0; p = p * s + 1.0 / 17.0;
    p = p * s + 1.0 / 15.0; p = p * s + 1.0 / 13.0; p = p * s + 1.0 / 11.0;
    p = p * s + 1.0 / 9.0; p = p * s + 1.0 / 7.0; p = p * s + 1.0 / 5.0; p = p * s + 1.0 / 3.0;
    const double t = 2.0 * f, r = t + t * (s * p);
    return (double)e * DET_LN2_HI + (r + (double)e * DET_LN2_LO);
}
__device__ inline double det_exp(double x) {
    if (x < -700.0) return 0.0;
    const double kf = floor(x * DET_INV_LN2 + 0.5);
    const double r = (x - kf * DET_LN2_HI) - kf * DET_LN2_LO;
    double p = 1.0 / 6227020800.0;
    p = p * r + 1.0 / 479001600.0; p = p * r + 1.0 / 39916800.0; p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0; p = p * r + 1.0 / 40320.0; p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0; p = p * r + 1.0 / 120.0; p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0; p = p * r + 0.5; p = p * r + 1.0; p = p * r + 1.0;
    return ldexp(p, (int)kf);
}
__device__ inline double det_pow(double x, double y) { return x == 0.0 ? 0.0 : det_exp(y * det_log(x)); }

// Gamma(alpha) for the Dirichlet draw: Marsaglia-Tsang with polar normals (and the alpha<1
// boost), uniforms ctr, ctr+1, ... of the Philox sequence (seed, board, stream).
__device__ inline double det_gamma(double alpha, uint64_t seed, uint32_t board, uint32_t stream,
                                   uint32_t ctr) {
    const double a = alpha < 1.0 ? alpha + 1.0 : alpha;
    const double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
    double g = 0.0;
    for (int it = 0; it < 64; it++) {
        double z = 0.0;
        for (int j = 0; j < 16; j++) {
            const double u1 = 2.0 * philox_u01(seed, board, stream, ctr) - 1.0;
            const double u2 = 2.0 * philox_u01(seed, board, stream, ctr + 1) - 1.0;
            ctr += 2;
            const double s = u1 * u1 + u2 * u2;
            if (s < 1.0 && s > 0.0) { z = u1 * sqrt(-2.0 * det_log(s) / s); break; }
        }
        double v = 1.0 + c * z;
        if (v <= 0.0) continue;
        v = v * v * v;
        double u = philox_u01(seed, board, stream, ctr++);
        if (u < 1e-300) u = 1e-300;
        if (det_log(u) < 0.5 * z * z + d - d * v + d * det_log(v)) { g = d * v; break; }
    }
    if (alpha < 1.0) {
        double u = philox_u01(seed, board, stream, ctr++);
        if (u < 1e-300) u = 1e-300;
        g = g * det_exp(det_log(u) / alpha);
    }
    return g;
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
