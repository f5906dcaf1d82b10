// splendor_device.h — gfx950 device implementation of the Splendor rules.
//
// Board representation on chip: the reference's int8 (R,7) state (SplendorLogicNumba.py:
// 291-303; 7 bytes per row in HBM, identical to board.tobytes()) is staged in LDS as
// R x 8-byte rows (7 columns + a zero pad byte). Every row is one aligned 64-bit word, so
// a row read/write/copy is a single ds_read_b64/ds_write_b64 and gem arithmetic is
// byte-wise SIMD-within-a-register on whole rows.
//
// Kernels use two mappings: WAVE-per-board (the 409-action legality mask is 7 chunks of
// 64 lanes packed by ballots) and LANE-per-board (transitions: the serial rule logic of 64
// boards runs in one wave). Functions named wave_* are wave-collective; all others are
// per-lane and run either uniformly across a wave or one board per lane.
//
// Semantics follow the reference bit for bit (incl. the Numba int8 wraps); every function
// cites the lines it restates. Parity: tests/ compare against the CPU oracle (oracle/),
// itself pinned to golden vectors recorded from the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "splendor_tables.h"

#ifndef SPL_PROBE
#define SPL_PROBE(k)   // diagnostic cycle probes (tools/time_rollout.hip); empty in product builds
#endif

namespace spl {

// condition codes of K_ACTION_DESC (gen_tables.py)
enum { C_ALWAYS, C_RSV_LIMIT, C_TAKE1, C_TAKE2D, C_TAKE3, C_TAKE2S, C_EX8, C_EX9, C_EX10,
       C_EX10G, C_NEVER };

template <int N>
struct Lay {  // row offsets of the (R,7) state (SplendorLogicNumba.py:296-303)
    static constexpr int NN = N + 1;                 // nobles on the table
    static constexpr int ROWS = 32 + 10 * N + N * N;
    static constexpr int S = 7 * ROWS;               // bytes per board in HBM (7-byte rows)
    static constexpr int LS = 8 * ROWS;              // bytes per board in LDS (8-byte rows)
    static constexpr int BANK = 0, TIERS = 1, DECKS = 25, NOBLES = 31;
    static constexpr int GEMS = 32 + N, PNOB = 32 + 2 * N, CARDS = 32 + 3 * N + N * N;
    static constexpr int RSV = 32 + 4 * N + N * N;
    static constexpr int PROWS = ROWS - GEMS;        // player-specific rows
    static constexpr int MAXMOVES = 62 * N;
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }
// wave-uniform value moved to an SGPR (lets dependent loads use the scalar cache)
__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32);
}

// workgroup barrier ordering LDS traffic only: waits for this wave's LDS (and scalar)
// operations, not its global ones. __syncthreads() first waits vmcnt(0), i.e. for every
// global store of the wave to be acknowledged by memory (~2K cycles for HBM). Use it where
// no wave reads global memory another wave wrote before the barrier. The memory clobber
// keeps the compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ------------------------------------------------------------------ row words
__device__ __forceinline__ uint64_t &row(int8_t *s, int r) { return *reinterpret_cast<uint64_t *>(s + 8 * r); }
__device__ __forceinline__ uint64_t row(const int8_t *s, int r) { return *reinterpret_cast<const uint64_t *>(s + 8 * r); }
__device__ __forceinline__ int bt(uint64_t w, int c) { return (int8_t)(uint8_t)(w >> (8 * c)); }
__device__ __forceinline__ uint64_t with_bt(uint64_t w, int c, int v) {
    return (w & ~(0xFFull << (8 * c))) | ((uint64_t)(uint8_t)v << (8 * c));
}
__device__ __forceinline__ int sum5(uint64_t w) { return bt(w, 0) + bt(w, 1) + bt(w, 2) + bt(w, 3) + bt(w, 4); }
__device__ __forceinline__ int sum7(uint64_t w) { return sum5(w) + bt(w, 5) + bt(w, 6); }
// byte-wise add / sub modulo 256 in every byte (the int8 wrap), no carries between bytes
__device__ __forceinline__ uint64_t bytes_add(uint64_t a, uint64_t b) {
    const uint64_t H = 0x8080808080808080ull;
    return ((a & ~H) + (b & ~H)) ^ ((a ^ b) & H);
}
__device__ __forceinline__ uint64_t bytes_sub(uint64_t a, uint64_t b) {
    const uint64_t H = 0x8080808080808080ull;
    return ((a | H) - (b & ~H)) ^ ((a ^ ~b) & H);
}
// each of the first 5 signed bytes of x >= the matching signed byte of v
__device__ __forceinline__ bool ge5(uint64_t x, uint64_t v) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 5; c++) ok &= bt(x, c) >= bt(v, c);
    return ok;
}

// ------------------------------------------------------------------ chance source
// Philox4x32-10 (Salmon et al. 2011); identical to oracle/splendor_oracle.c. Uniform d of
// a (seed, board, stream) sequence is one half of counter block d/2: output words (0,1)
// for even d, (2,3) for odd d, 53 bits each.
__device__ __forceinline__ void philox_pair(uint64_t seed, uint32_t board, uint32_t stream,
                                            uint32_t blk, double &a, double &b) {
    uint32_t c0 = blk, c1 = board, c2 = stream, c3 = 0x53504C44u;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    a = ((double)(c0 >> 5) * 67108864.0 + (double)(c1 >> 6)) * (1.0 / 9007199254740992.0);
    b = ((double)(c2 >> 5) * 67108864.0 + (double)(c3 >> 6)) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ double philox_u01(uint64_t seed, uint32_t board, uint32_t stream, uint32_t d) {
    double a, b;
    philox_pair(seed, board, stream, d >> 1, a, b);
    return (d & 1) ? b : a;
}

// The transition tables (deck draws, per-action gem vectors). Default: constant memory;
// a kernel may stage them in LDS (stage_tabs) and pass the LDS copy.
struct Tabs {
    const double (*quot)[9] = K_QUOT;
    const double *recip = K_RECIP;
    const uint64_t (*cards)[2] = K_CARD_ROWS;
    const uint64_t *act_take = K_ACT_TAKE, *act_give = K_ACT_GIVE;
    const int8_t *act_rsv = K_ACT_RSV;
};
struct TabsLds {          // LDS image of Tabs
    double quot[41][9];
    double recip[9];
    uint64_t cards[120][2];
    uint64_t act_take[409], act_give[409];
    int8_t act_rsv[409];
    __device__ __forceinline__ Tabs view() const { return Tabs{quot, recip, cards, act_take, act_give, act_rsv}; }
};
// cooperative copy of the tables into LDS by `nthreads` threads (caller synchronises)
__device__ __forceinline__ void stage_tabs(TabsLds &t, int tid, int nthreads) {
    for (int i = tid; i < 41 * 9; i += nthreads) (&t.quot[0][0])[i] = (&K_QUOT[0][0])[i];
    for (int i = tid; i < 240; i += nthreads) (&t.cards[0][0])[i] = (&K_CARD_ROWS[0][0])[i];
    for (int i = tid; i < 409; i += nthreads) {
        t.act_take[i] = K_ACT_TAKE[i];
        t.act_give[i] = K_ACT_GIVE[i];
        t.act_rsv[i] = K_ACT_RSV[i];
    }
    if (tid < 9) t.recip[tid] = K_RECIP[tid];
}

// Either an explicit stream of doubles (parity with recorded reference draws) or Philox.
// Sequential draws reuse the second half of a Philox block. The transition tables travel
// with the chance source.
struct Chance {
    const double *u;   // explicit uniforms for this board, or nullptr -> Philox
    uint64_t seed;
    uint32_t board, stream, next;
    double spare = 0.0;
    bool have_spare = false;
    Tabs tab = Tabs{};
    __device__ __forceinline__ double draw() {
        if (u) return u[next++];
        double r;
        if ((next & 1) && have_spare) {
            r = spare;
        } else {
            double a, b;
            philox_pair(seed, board, stream, next >> 1, a, b);
            r = (next & 1) ? b : a;
            spare = b;
        }
        have_spare = !(next & 1);
        ++next;
        return r;
    }
};

// ------------------------------------------------------------------ HBM <-> LDS
// HBM boards have 7-byte rows; LDS boards 8-byte rows with a zero pad byte. Four rows are
// 28 HBM bytes = 7 dwords; one lane converts such a quad in registers (funnel shifts), so
// a board moves as 7-dword global accesses and 64-bit LDS accesses. Boards whose row count
// is not a multiple of 4 (3 players) go byte by byte.
// (the 7 dwords already in registers -> the 4 LDS rows)
__device__ __forceinline__ void quad_rows_put(const uint32_t (&d)[7], uint64_t *o) {
    const uint64_t M = 0x00FFFFFFFFFFFFFFull;
    o[0] = ((uint64_t)d[0] | (uint64_t)d[1] << 32) & M;
    o[1] = ((uint64_t)d[1] >> 24 | (uint64_t)d[2] << 8 | (uint64_t)d[3] << 40) & M;
    o[2] = ((uint64_t)d[3] >> 16 | (uint64_t)d[4] << 16 | (uint64_t)d[5] << 48) & M;
    o[3] = ((uint64_t)d[5] >> 8 | (uint64_t)d[6] << 24) & M;
}
__device__ __forceinline__ void quad_to_rows(const uint32_t *g, uint64_t *o) {
    uint32_t d[7];
#pragma unroll
    for (int k = 0; k < 7; k++) d[k] = g[k];
    quad_rows_put(d, o);
}
__device__ __forceinline__ void rows_to_quad(const uint64_t *r, uint32_t *g) {
    const uint64_t r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
    g[0] = (uint32_t)r0;
    g[1] = (uint32_t)(r0 >> 32 | r1 << 24);
    g[2] = (uint32_t)(r1 >> 8);
    g[3] = (uint32_t)(r1 >> 40 | r2 << 16);
    g[4] = (uint32_t)(r2 >> 16);
    g[5] = (uint32_t)(r2 >> 48 | r3 << 8);
    g[6] = (uint32_t)(r3 >> 24);
}
// quad-or-byte unit u of a board (units per board: Conv<N>::UNITS)
template <int N>
struct Conv {
    static constexpr bool QUAD = Lay<N>::ROWS % 4 == 0;
    static constexpr int UNITS = QUAD ? Lay<N>::ROWS / 4 : Lay<N>::S;
    static __device__ __forceinline__ void load(int8_t *lds, const int8_t *g, int u) {
        if constexpr (QUAD) {
            quad_to_rows(reinterpret_cast<const uint32_t *>(g) + 7 * u, reinterpret_cast<uint64_t *>(lds) + 4 * u);
        } else {
            lds[8 * (u / 7) + u % 7] = g[u];
            if (u % 7 == 6) lds[8 * (u / 7) + 7] = 0;
        }
    }
    static __device__ __forceinline__ void store(int8_t *g, const int8_t *lds, int u) {
        if constexpr (QUAD) rows_to_quad(reinterpret_cast<const uint64_t *>(lds) + 4 * u, reinterpret_cast<uint32_t *>(g) + 7 * u);
        else g[u] = lds[8 * (u / 7) + u % 7];
    }
};
template <int N>
__device__ __forceinline__ void wave_load_board(int8_t *lds, const int8_t *g) {
    for (int u = lane_id(); u < Conv<N>::UNITS; u += 64) Conv<N>::load(lds, g, u);
    __builtin_amdgcn_wave_barrier();
}
template <int N>
__device__ __forceinline__ void wave_store_board(int8_t *g, const int8_t *lds) {
    __builtin_amdgcn_wave_barrier();
    for (int u = lane_id(); u < Conv<N>::UNITS; u += 64) Conv<N>::store(g, lds, u);
}
// plain byte copies in one layout (HBM->HBM, or byte-permuting kernels)
__device__ __forceinline__ void wave_copy_bytes(int8_t *dst, const int8_t *src, int bytes) {
    const int l = lane_id();
    if ((bytes & 3) == 0 && ((uintptr_t)dst & 3) == 0 && ((uintptr_t)src & 3) == 0) {
        for (int i = 4 * l; i < bytes; i += 256)
            *reinterpret_cast<int32_t *>(dst + i) = *reinterpret_cast<const int32_t *>(src + i);
    } else {
        for (int i = l; i < bytes; i += 64) dst[i] = src[i];
    }
    __builtin_amdgcn_wave_barrier();
}
// LDS -> LDS board copy (8-byte rows)
template <int N>
__device__ __forceinline__ void wave_copy_lds_board(int8_t *dst, const int8_t *src) {
    for (int r = lane_id(); r < Lay<N>::ROWS; r += 64) row(dst, r) = row(src, r);
    __builtin_amdgcn_wave_barrier();
}

// swap_players (SplendorLogicNumba.py:338-347): roll each player block so that player k
// becomes player 0 (gems by k, nobles by 3k — hard-coded 3, :345 —, cards by k, reserved
// by 6k). Wave: one lane per row. dst may equal src.
template <int N>
__device__ __forceinline__ void wave_roll_players(int8_t *dst, const int8_t *src, int k) {
    using Lx = Lay<N>;
    constexpr int IT = (Lx::ROWS + 63) / 64;
    const int l = lane_id();
    uint64_t v[IT];
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const int r = l + 64 * j;
        v[j] = 0;
        if (r < Lx::ROWS) {
            int sr = r;
            const int q = r - Lx::GEMS;
            if (q >= 0) {
                if (q < N) sr = Lx::GEMS + (q + k) % N;
                else if (q < N + N * Lx::NN) sr = Lx::GEMS + N + (q - N + 3 * k) % (N * Lx::NN);
                else if (q < 2 * N + N * Lx::NN) sr = Lx::GEMS + N + N * Lx::NN + (q - N - N * Lx::NN + k) % N;
                else sr = Lx::GEMS + 2 * N + N * Lx::NN + (q - 2 * N - N * Lx::NN + 6 * k) % (6 * N);
            }
            v[j] = row(src, sr);
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const int r = l + 64 * j;
        if (r < Lx::ROWS && (dst != src || r >= Lx::GEMS)) row(dst, r) = v[j];
    }
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ legality mask
// Board.valid_moves (SplendorLogicNumba.py:251-265). Wave-collective over an LDS board;
// returns the packed 409-bit mask in w[0..6] (bit a%64 of word a/64), same in every lane.
//
// Phase 1 packs 120 per-board predicates into two ballots:
//   F0: 0-11 _valid_buy (:476-501)  12-26 _valid_reserve(is_limit=False) (:508-515)
//       27-29 _valid_buy_reserve (:538-552)  30-54 bank holds DIFF3[i] (:562-568)
//       55-59 bank[c] >= 4 (:578-583)
//   F1: 0-19 _valid_give_gems(+identical) (:595-613)  20-59 _valid_give_gems3 (:602-607)
// Phase 2 evaluates one action per lane from K_ACTION_DESC: flag0 & flag1 & condition,
// the conditions restating the token-count branches of _valid_get_gems (:570-574) and
// _valid_exchange (:615-680). Pass (408) is set iff nothing else is legal (:263).
// Board-independent per-lane operands of the mask (action descriptors and the gem vector
// each predicate lane compares against), loaded once per kernel instead of per board.
struct MaskLane {
    uint32_t desc[7];
    uint64_t take, give;
    __device__ __forceinline__ static MaskLane load() {
        const int l = lane_id();
        MaskLane m;
#pragma unroll
        for (int k = 0; k < 7; k++) m.desc[k] = 64 * k + l < 409 ? K_ACTION_DESC[64 * k + l] : (uint32_t)(C_NEVER << 16);
        m.take = l >= 30 && l < 55 ? K_TAKE_ROW[l - 30] : 0;
        m.give = l < 15 ? K_GIVE_ROW[l] : (l >= 20 && l < 60 ? K_SPEC3_ROW[l - 20] : 0);
        return m;
    }
};

template <int N>
__device__ __forceinline__ void wave_valid_moves(const int8_t *s, int p, int lim, uint64_t w[7], const MaskLane &ml) {
    using Lx = Lay<N>;
    const int l = lane_id();
    const uint64_t bank = row(s, Lx::BANK), gems = row(s, Lx::GEMS + p), cards = row(s, Lx::CARDS + p);
    const int T = sum7(gems), gold = bt(gems, 5), bgold = bt(bank, 5);
    int nspec = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) nspec += bt(bank, c) != 0;
    const bool slot_free = sum5(row(s, Lx::RSV + 6 * p + 5)) == 0;   // third slot's gain row (:514)

    bool f = false;
    if (l < 12 || (l >= 27 && l < 30)) {          // affordability (visible or reserved card)
        const uint64_t cost = row(s, l < 12 ? Lx::TIERS + 2 * l : Lx::RSV + 6 * p + 2 * (l - 27));
        int miss = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            const int d = bt(cost, c) - bt(gems, c) - bt(cards, c);
            miss += d > 0 ? d : 0;
        }
        f = miss <= gold && sum5(cost) != 0;
    } else if (l < 27) {                          // reservable slot non-empty
        const int i = l - 12;
        f = sum5(row(s, i < 12 ? Lx::TIERS + 2 * i : Lx::DECKS + 2 * (i - 12))) != 0 && slot_free;
    } else if (l < 55) {                          // bank can supply take vector
        f = ge5(bank, ml.take);
    } else if (l < 60) {
        f = bt(bank, l - 55) >= 4;
    }
    const uint64_t F0 = __ballot(f);
    f = false;
    if (l >= 15 && l < 20) f = bt(gems, l - 15) >= 2;                 // two identical gems
    else if (l < 60) f = ge5(gems, ml.give);
    const uint64_t F1 = __ballot(f);

    const bool ex_any = T > 7;
    const bool ex8 = ex_any && T == lim - 2;
    const bool ex9 = ex_any && !ex8 && T == lim - 1;
    const bool ex10 = ex_any && !ex8 && !ex9;
    uint32_t cond = 1u << C_ALWAYS;
    cond |= (uint32_t)(!(T == lim && bgold > 0)) << C_RSV_LIMIT;
    cond |= (uint32_t)(T + 1 <= lim && (T == 9 || nspec == 1)) << C_TAKE1;
    cond |= (uint32_t)(T + 2 <= lim && (T == 8 || nspec == 2)) << C_TAKE2D;
    cond |= (uint32_t)(T + 3 <= lim) << C_TAKE3;
    cond |= (uint32_t)(T + 2 <= lim) << C_TAKE2S;
    cond |= (uint32_t)ex8 << C_EX8;
    cond |= (uint32_t)ex9 << C_EX9;
    cond |= (uint32_t)ex10 << C_EX10;
    cond |= (uint32_t)(ex10 && bgold > 0) << C_EX10G;

    uint64_t any = 0;
#pragma unroll
    for (int k = 0; k < 7; k++) {
        const uint32_t d = ml.desc[k];
        const bool f0 = !((d >> 6) & 1) || ((F0 >> (d & 63)) & 1);
        const bool f1 = !((d >> 14) & 1) || ((F1 >> ((d >> 8) & 63)) & 1);
        const bool c = (cond >> ((d >> 16) & 15)) & 1;
        w[k] = __ballot(f0 && f1 && c);
        any |= w[k];
    }
    if (!any) w[6] |= 1ull << (408 - 384);
}
template <int N>
__device__ __forceinline__ void wave_valid_moves(const int8_t *s, int p, int lim, uint64_t w[7]) {
    wave_valid_moves<N>(s, p, lim, w, MaskLane::load());
}

// Lane-per-board form of the same mask: one lane evaluates every predicate and action of
// its own board with compile-time bit positions (KC_* tables), ~20x fewer instructions
// per board than the wave form; used where 64 boards share a wave.
struct LanePred {
    uint64_t F0, F1;   // the two predicate sets of wave_valid_moves
    uint32_t C;        // condition bits, indexed by condition code
};

// threshold mask of the 5 colours of a row: bit 5t+c <-> byte c >= t (t = 0..4)
__device__ __forceinline__ uint32_t thresh5(uint64_t w) {
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const int v = bt(w, c);
#pragma unroll
        for (int t = 0; t < 5; t++) m |= (uint32_t)(v >= t) << (5 * t + c);
    }
    return m;
}

// condition bits (the token-count branches of wave_valid_moves)
__device__ __forceinline__ uint32_t lane_cond(int T, int lim, int nspec, int bgold) {
    const bool ex_any = T > 7;
    const bool ex8 = ex_any && T == lim - 2;
    const bool ex9 = ex_any && !ex8 && T == lim - 1;
    const bool ex10 = ex_any && !ex8 && !ex9;
    uint32_t C = 1u << C_ALWAYS;
    C |= (uint32_t)(!(T == lim && bgold > 0)) << C_RSV_LIMIT;
    C |= (uint32_t)(T + 1 <= lim && (T == 9 || nspec == 1)) << C_TAKE1;
    C |= (uint32_t)(T + 2 <= lim && (T == 8 || nspec == 2)) << C_TAKE2D;
    C |= (uint32_t)(T + 3 <= lim) << C_TAKE3;
    C |= (uint32_t)(T + 2 <= lim) << C_TAKE2S;
    C |= (uint32_t)ex8 << C_EX8;
    C |= (uint32_t)ex9 << C_EX9;
    C |= (uint32_t)ex10 << C_EX10;
    C |= (uint32_t)(ex10 && bgold > 0) << C_EX10G;
    return C;
}

// exact predicates for any int8 board (threshold masks over signed bytes)
template <int N>
__device__ __noinline__ LanePred lane_predicates_exact(const int8_t *s, int p, int lim) {
    using Lx = Lay<N>;
    const uint64_t bank = row(s, Lx::BANK), gems = row(s, Lx::GEMS + p), cards = row(s, Lx::CARDS + p);
    const int T = sum7(gems), gold = bt(gems, 5), bgold = bt(bank, 5);
    int nspec = 0, have[5];
#pragma unroll
    for (int c = 0; c < 5; c++) {
        nspec += bt(bank, c) != 0;
        have[c] = bt(gems, c) + bt(cards, c);
    }
    const bool slot_free = sum5(row(s, Lx::RSV + 6 * p + 5)) == 0;
    LanePred P{0, 0, 0};
    // F0 0-11 buy a visible card, 12-23 reserve it (:476-515)
#pragma unroll
    for (int i = 0; i < 12; i++) {
        const uint64_t cost = row(s, Lx::TIERS + 2 * i);
        int miss = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            const int d = bt(cost, c) - have[c];
            miss += d > 0 ? d : 0;
        }
        const bool any = sum5(cost) != 0;
        P.F0 |= (uint64_t)(miss <= gold && any) << i;
        P.F0 |= (uint64_t)(any && slot_free) << (12 + i);
    }
    // F0 24-26 reserve from a deck, 27-29 buy a reserved card (:508-552)
#pragma unroll
    for (int t = 0; t < 3; t++) {
        P.F0 |= (uint64_t)(sum5(row(s, Lx::DECKS + 2 * t)) != 0 && slot_free) << (24 + t);
        const uint64_t cost = row(s, Lx::RSV + 6 * p + 2 * t);
        int miss = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            const int d = bt(cost, c) - have[c];
            miss += d > 0 ? d : 0;
        }
        P.F0 |= (uint64_t)(miss <= gold && sum5(cost) != 0) << (27 + t);
    }
    // F0 30-59 bank supplies, F1 0-59 player can give (threshold masks, KC_REQ*)
    const uint32_t nb = ~thresh5(bank), ng = ~thresh5(gems);
#pragma unroll
    for (int i = 30; i < 60; i++) P.F0 |= (uint64_t)((KC_REQ0[i] & nb) == 0) << i;
#pragma unroll
    for (int i = 0; i < 60; i++) P.F1 |= (uint64_t)((KC_REQ1[i] & ng) == 0) << i;
    P.C = lane_cond(T, lim, nspec, bgold);
    return P;
}

// colours whose byte is >= t
__device__ __forceinline__ uint32_t ge_set(uint64_t w, int t) {
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) m |= (uint32_t)(bt(w, c) >= t) << c;
    return m;
}

// Predicates of lane_predicates_exact, computed with byte arithmetic for boards whose
// colour bytes (bank, the player's gems and cards, card costs, deck counts, reserve slot)
// are non-negative — every board reachable from init_game. Affordability uses byte SADs:
// sum max(cost - have, 0) = (sum |cost - have| + sum cost - sum have) / 2; the gem-vector
// predicates are subset / level table lookups (K_LUT_DIFF, K_LUT_SPEC3). Other boards take
// the exact path.
template <int N>
__device__ __forceinline__ LanePred lane_predicates(const int8_t *s, int p, int lim,
                                                    const uint32_t *lut_diff = K_LUT_DIFF,
                                                    const uint64_t *lut_s3 = K_LUT_SPEC3) {
    using Lx = Lay<N>;
    constexpr uint64_t M5 = 0xFFFFFFFFFFull, H5 = 0x8080808080ull;
    const uint64_t bank = row(s, Lx::BANK), gems = row(s, Lx::GEMS + p), cards = row(s, Lx::CARDS + p);
    const uint64_t slot5 = row(s, Lx::RSV + 6 * p + 5);
    uint64_t cost[15], deck[3];
    uint64_t any = bank | gems | cards | slot5;
#pragma unroll
    for (int i = 0; i < 15; i++) {
        cost[i] = row(s, i < 12 ? Lx::TIERS + 2 * i : Lx::RSV + 6 * p + 2 * (i - 12));
        any |= cost[i];
    }
#pragma unroll
    for (int t = 0; t < 3; t++) {
        deck[t] = row(s, Lx::DECKS + 2 * t);
        any |= deck[t];
    }
    if (any & H5) return lane_predicates_exact<N>(s, p, lim);
    const uint64_t have = (gems & M5) + (cards & M5);          // bytes < 256: no carries
    const uint32_t hlo = (uint32_t)have, hhi = (uint32_t)(have >> 32);
    const int gold = bt(gems, 5);
    const int rhs = 2 * gold + (int)__builtin_amdgcn_sad_u8(hlo, 0u, hhi);
    const bool slot_free = (slot5 & M5) == 0;
    LanePred P{0, 0, 0};
#pragma unroll
    for (int i = 0; i < 15; i++) {
        const uint32_t clo = (uint32_t)cost[i], chi = (uint32_t)(cost[i] >> 32) & 0xFF;
        const uint32_t absd = __builtin_amdgcn_sad_u8(clo, hlo, __builtin_amdgcn_sad_u8(chi, hhi, 0u));
        const int lhs = (int)__builtin_amdgcn_sad_u8(clo, 0u, absd + chi);   // sum|c-h| + sum c
        const bool nz = (cost[i] & M5) != 0;
        const bool buy = lhs <= rhs && nz;
        if (i < 12) {
            P.F0 |= (uint64_t)buy << i;
            P.F0 |= (uint64_t)(nz && slot_free) << (12 + i);
        } else {
            P.F0 |= (uint64_t)buy << (27 + i - 12);
        }
    }
#pragma unroll
    for (int t = 0; t < 3; t++) P.F0 |= (uint64_t)((deck[t] & M5) != 0 && slot_free) << (24 + t);
    const uint32_t b1 = ge_set(bank, 1), g1 = ge_set(gems, 1);
    uint32_t lvl = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) lvl |= (uint32_t)min(bt(gems, c), 3) << (2 * c);
    P.F0 |= (uint64_t)lut_diff[b1] << 30 | (uint64_t)ge_set(bank, 4) << 55;
    P.F1 = (uint64_t)(lut_diff[g1] & 0x7FFFu) | (uint64_t)ge_set(gems, 2) << 15 | lut_s3[lvl] << 20;
    P.C = lane_cond(sum7(gems), lim, __popc(b1), bt(bank, 5));
    return P;
}

// packed level indices of lane_mask_word_fast: bank levels (0 / 1-3 / >= 4 gems) and gem
// levels (min(gems, 3)) of colours 0-2 and 3-4, as table row offsets
__device__ __forceinline__ uint32_t lane_levels(uint64_t bank, uint64_t gems) {
    int lam[5], ell[5];
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const int b = bt(bank, c);
        lam[c] = b >= 4 ? 2 : (b >= 1 ? 1 : 0);
        ell[c] = min(bt(gems, c), 3);
    }
    return (uint32_t)(lam[0] + 3 * lam[1] + 9 * lam[2]) | (uint32_t)(lam[3] + 3 * lam[4]) << 5 |
           (uint32_t)(ell[0] + 4 * ell[1] + 16 * ell[2]) << 9 | (uint32_t)(ell[3] + 4 * ell[4]) << 15;
}

// Mask word K of a board in the fast domain from its card predicates (F0 bits 0-29),
// condition bits C and levels lv (lane_levels): the gem-vector predicates of
// lane_predicates depend on the board only through the colour levels, so per word they
// factor into four level-table rows (K_MASK_FACTORS, staged at fac) ANDed with the gates
// of the word's condition codes and its card-predicate runs (gen_tables.py mask_factors,
// which checks the factorisation against the descriptor formula of lane_mask_word).
template <int K>
__device__ __forceinline__ uint64_t lane_mask_word_fast(uint32_t C, uint64_t F0, uint32_t lv, const uint64_t *fac) {
    const uint64_t *r = fac + 116 * K;
    const uint64_t m = r[lv & 31] & r[27 + ((lv >> 5) & 15)] & r[36 + ((lv >> 9) & 63)] & r[100 + ((lv >> 15) & 15)];
    uint64_t gate = 0;
#pragma unroll
    for (int c = 0; c < 11; c++)
        if (KC_MASK_GATE[K][c]) gate |= ((C >> c) & 1) ? KC_MASK_GATE[K][c] : 0ull;
    uint64_t card = ~0ull;
#pragma unroll
    for (int b = 0; b < KC_CARD_NBLK; b++) {
        if (KC_CARD_BLK[b][0] != K) continue;
        const int j0 = KC_CARD_BLK[b][1], n = KC_CARD_BLK[b][2], f0 = KC_CARD_BLK[b][3];
        const uint64_t span = ((1ull << n) - 1) << j0;
        const uint64_t src = KC_CARD_BLK[b][4] ? (((F0 >> f0) & 1) ? span : 0ull) : ((F0 >> f0) << j0) & span;
        card &= ~span | src;
    }
    return m & gate & card;
}

// One quarter of lane_predicates' fast path, so four waves can share a board's predicate
// work: PART 0 / 1 = buy and reserve bits of visible cards 0-5 / 6-11, PART 2 = reserved
// cards, deck reserves and the condition bits, PART 3 = the colour levels (returned in F1)
// that lane_mask_word_fast turns into the gem-vector predicates. F0 / C of the parts OR
// together; `bad` flags rows outside the fast domain (the caller then uses
// lane_predicates_exact and lane_mask_word for the board).
template <int N, int PART>
__device__ __forceinline__ void lane_predicates_part(const int8_t *s, int p, int lim, uint64_t &F0, uint64_t &F1,
                                                     uint32_t &C, bool &bad) {
    using Lx = Lay<N>;
    constexpr uint64_t M5 = 0xFFFFFFFFFFull, H5 = 0x8080808080ull;
    const uint64_t bank = row(s, Lx::BANK), gems = row(s, Lx::GEMS + p);
    F0 = 0; F1 = 0; C = 0;
    if constexpr (PART == 3) {
        bad = ((bank | gems) & H5) != 0;
        F1 = lane_levels(bank, gems);
    } else {
        constexpr int I0 = PART == 0 ? 0 : (PART == 1 ? 6 : 12), NI = PART == 2 ? 3 : 6;
        const uint64_t cards = row(s, Lx::CARDS + p), slot5 = row(s, Lx::RSV + 6 * p + 5);
        uint64_t cost[NI];
        uint64_t any = gems | cards | slot5;
#pragma unroll
        for (int k = 0; k < NI; k++) {
            const int i = I0 + k;
            cost[k] = row(s, i < 12 ? Lx::TIERS + 2 * i : Lx::RSV + 6 * p + 2 * (i - 12));
            any |= cost[k];
        }
        uint64_t deck[3] = {0, 0, 0};
        if constexpr (PART == 2) {
#pragma unroll
            for (int t = 0; t < 3; t++) {
                deck[t] = row(s, Lx::DECKS + 2 * t);
                any |= deck[t];
            }
            any |= bank;
        }
        bad = (any & H5) != 0;
        const uint64_t have = (gems & M5) + (cards & M5);
        const uint32_t hlo = (uint32_t)have, hhi = (uint32_t)(have >> 32);
        const int rhs = 2 * bt(gems, 5) + (int)__builtin_amdgcn_sad_u8(hlo, 0u, hhi);
        const bool slot_free = (slot5 & M5) == 0;
#pragma unroll
        for (int k = 0; k < NI; k++) {
            const int i = I0 + k;
            const uint32_t clo = (uint32_t)cost[k], chi = (uint32_t)(cost[k] >> 32) & 0xFF;
            const uint32_t absd = __builtin_amdgcn_sad_u8(clo, hlo, __builtin_amdgcn_sad_u8(chi, hhi, 0u));
            const int lhs = (int)__builtin_amdgcn_sad_u8(clo, 0u, absd + chi);
            const bool nz = (cost[k] & M5) != 0;
            const bool buy = lhs <= rhs && nz;
            if (i < 12) {
                F0 |= (uint64_t)buy << i;
                F0 |= (uint64_t)(nz && slot_free) << (12 + i);
            } else {
                F0 |= (uint64_t)buy << (27 + i - 12);
            }
        }
        if constexpr (PART == 2) {
#pragma unroll
            for (int t = 0; t < 3; t++) F0 |= (uint64_t)((deck[t] & M5) != 0 && slot_free) << (24 + t);
            C = lane_cond(sum7(gems), lim, __popc(ge_set(bank, 1)), bt(bank, 5));
        }
    }
}

// mask word K (actions 64K .. 64K+63) from the predicates; the pass bit is not included
template <int K>
__device__ __forceinline__ uint64_t lane_mask_word(const LanePred &P) {
    uint64_t w = 0;
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const int a = 64 * K + j;
        if (a >= 405) break;                       // 405-408: never set here
        const uint32_t d = KC_ACTION_DESC[a];
        uint64_t bit = (uint64_t)(P.C >> ((d >> 16) & 15));
        if ((d >> 6) & 1) bit &= P.F0 >> (d & 63);
        if ((d >> 14) & 1) bit &= P.F1 >> ((d >> 8) & 63);
        w |= (bit & 1) << j;
    }
    return w;
}

// k-th set bit (k < popcount) of a lane-private 64-bit word, by halving
__device__ __forceinline__ int kth_bit64(uint64_t x, int k) {
    int pos = 0;
#pragma unroll
    for (int h = 32; h >= 1; h >>= 1) {
        const int c = __popcll(x & ((1ull << h) - 1));
        if (k >= c) { k -= c; x >>= h; pos += h; }
    }
    return pos;
}

// ------------------------------------------------------------------ transition
// _get_deck_card (SplendorLogicNumba.py:400-420): colour ~ remaining count, then card ~
// remaining bit, each by searchsorted(cumsum(p), U, 'right') (:39-41); K_QUOT / K_RECIP
// hold the correctly rounded quotients the reference divides out. The bitfield is stored
// as int8 (packbits wrap, :44-46). Returns false if the tier's deck is empty.
// Colour pick with true divisions, for counts outside K_QUOT (unreachable boards); kept out
// of line so the common path carries no division code.
__device__ __noinline__ int pick_color_div(uint64_t cnt, int tot, double u) {
    double c = 0.0;
    for (int k = 0; k < 5; k++) {
        c += (double)bt(cnt, k) / (double)tot;
        if (c > u) return k;
    }
    return 4;
}

// Colour / card picks of _get_deck_card. The reference compares fp cumulative sums of the
// quotients cnt_k / tot (and 1 / nbits) with u; those sums equal the exact fractions
// C_k / tot to within 1e-15, so away from a boundary the pick is the integer count of
// prefix sums C_k <= u * tot. Draws with u * tot within 1e-9 of an integer (which covers
// every boundary |C_k - u * tot| < 1e-9; about 2 in 1e9) take the reference's fp sums over
// the exact quotient tables instead.
__device__ __noinline__ int pick_color_fp(uint64_t cnt, int tot, double u, const double (*quot)[9]) {
    const double *q = quot[tot];
    double c = 0.0;
    for (int k = 0; k < 5; k++) {
        c += q[bt(cnt, k)];
        if (c > u) return k;
    }
    return 4;
}
__device__ __noinline__ int pick_card_fp(uint32_t b, double u, const double *recip) {
    const double inv = recip[__builtin_popcount(b)];
    double c = 0.0;
    for (int k = 0; k < 8; k++) {
        c += ((b >> (7 - k)) & 1) ? inv : 0.0;
        if (c > u) return k;
    }
    return 7;
}

// floor(x) of x >= 0, and whether x lies within 1e-9 of an integer (x - floor(x) and
// floor(x) + 1 - x are exact in f64). For an integer prefix count C, C <= x iff
// C <= floor(x), so the picks below count in integers; "near" is a superset of the
// boundary draws |C_k - x| < 1e-9 and sends them (and ~2e-9 of all draws) to the fp path.
__device__ __forceinline__ int floor_near(double x, bool &near) {
    const double f = floor(x);
    near = x - f < 1e-9 || f + 1.0 - x < 1e-9;
    return (int)f;
}

// the colour and card index one draw takes from a tier deck's count / bit rows (tot > 0),
// given the draw's two uniforms; deck_take removes that card from the rows
__device__ __forceinline__ void deck_pick(uint64_t cnt, uint64_t bits, double u0, double u1, const Tabs &tab,
                                          int &color_out, int &idx_out) {
    const int tot = sum5(cnt);
    bool dom = true;
#pragma unroll
    for (int k = 0; k < 5; k++) dom &= (unsigned)bt(cnt, k) <= 8u;
    int color;
    if (dom) {
        bool amb;
        const int fx = floor_near(u0 * (double)tot, amb);
        int ck = 0, n_le = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            ck += bt(cnt, k);
            n_le += ck <= fx;
        }
        color = amb ? pick_color_fp(cnt, tot, u0, tab.quot) : min(n_le, 4);
    } else {
        color = pick_color_div(cnt, tot, u0);
    }
    const uint32_t b = (uint8_t)bt(bits, color);
    const int nb = __builtin_popcount(b);
    bool amb;
    const int fx = floor_near(u1 * (double)nb, amb);
    int pk = 0, n_le = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        pk += (b >> (7 - k)) & 1;
        n_le += pk <= fx;
    }
    // nb == 0 (reference: 0/0 sums, no index above u -> the last card) gives x = 0, near an
    // integer, and is resolved by the fp path, which returns the last card as well
    color_out = color;
    idx_out = amb ? pick_card_fp(b, u1, tab.recip) : min(n_le, 7);
}
__device__ __forceinline__ void deck_take(uint64_t &cnt, uint64_t &bits, int color, int idx) {
    bits = with_bt(bits, color, (int)((uint8_t)bt(bits, color) & ~(1u << (7 - idx))));
    cnt = with_bt(cnt, color, bt(cnt, color) - 1);
}

template <int N>
__device__ __forceinline__ bool deck_card(int8_t *s, int tier, Chance &ch, uint64_t &cost, uint64_t &gain) {
    using Lx = Lay<N>;
    uint64_t cnt = row(s, Lx::DECKS + 2 * tier), bits = row(s, Lx::DECKS + 2 * tier + 1);
    if (sum5(cnt) == 0) return false;
    const double u0 = ch.draw();
    const double u1 = ch.draw();
    int color, idx;
    deck_pick(cnt, bits, u0, u1, ch.tab, color, idx);
    deck_take(cnt, bits, color, idx);
    row(s, Lx::DECKS + 2 * tier + 1) = bits;
    row(s, Lx::DECKS + 2 * tier) = cnt;
    cost = ch.tab.cards[tier * 40 + color * 8 + idx][0];
    gain = ch.tab.cards[tier * 40 + color * 8 + idx][1];
    return true;
}

template <int N>
__device__ __forceinline__ void fill_new_card(int8_t *s, int tier, int idx, bool det, Chance &ch) {
    const int r = Lay<N>::TIERS + 8 * tier + 2 * idx;
    uint64_t cost = 0, gain = 0;
    if (!det) deck_card<N>(s, tier, ch, cost, gain);   // _fill_new_card (:445-450)
    row(s, r) = cost;
    row(s, r + 1) = gain;
}

// _give_nobles_if_earned (:763-768): every qualifying noble, stored at row nn*p+i
template <int N>
__device__ __forceinline__ void give_nobles(int8_t *s, int p) {
    using Lx = Lay<N>;
    const uint64_t cards = row(s, Lx::CARDS + p);
    uint64_t nob[Lx::NN];                    // all noble rows read before any write
#pragma unroll
    for (int i = 0; i < Lx::NN; i++) nob[i] = row(s, Lx::NOBLES + i);
#pragma unroll
    for (int i = 0; i < Lx::NN; i++) {
        if (sum5(nob[i]) > 0 && ge5(cards, nob[i])) {
            row(s, Lx::PNOB + Lx::NN * p + i) = nob[i];
            row(s, Lx::NOBLES + i) = 0;
        }
    }
}

// _buy_card (:458-474): pay coloured gems, then gold for what is missing; take the gain
template <int N>
__device__ __forceinline__ void buy_card(int8_t *s, int cost_row, int p) {
    using Lx = Lay<N>;
    const uint64_t cost = row(s, cost_row), gain = row(s, cost_row + 1);
    uint64_t gems = row(s, Lx::GEMS + p), bank = row(s, Lx::BANK);
    const uint64_t cards = row(s, Lx::CARDS + p);
    int miss = 0;
    uint64_t paid = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const int cc = bt(cost, c), gc = bt(gems, c), kc = bt(cards, c);
        const int d = cc - gc - kc;
        miss += d > 0 ? d : 0;
        int need = cc - kc;
        need = need > 0 ? need : 0;
        paid |= (uint64_t)(uint8_t)(need < gc ? need : gc) << (8 * c);
    }
    gems = bytes_sub(gems, paid);
    bank = bytes_add(bank, paid);
    row(s, Lx::GEMS + p) = with_bt(gems, 5, bt(gems, 5) - miss);
    row(s, Lx::BANK) = with_bt(bank, 5, bt(bank, 5) + miss);
    row(s, Lx::CARDS + p) = bytes_add(cards, gain);
    SPL_PROBE(15)
    give_nobles<N>(s, p);
}

// Board.make_move (:267-289) as one fixed pipeline of row operations, so boards that take
// different kinds of moves share every stage (lane-per-board kernels run the pipeline once,
// not once per move kind):
//   buy     _buy_card (:458-474) for a visible (0-11) or reserved (27-29) card
//   reserve _reserve (:517-536): first empty slot; a visible card moves there
//   draw    one deck draw: refill the bought / reserved visible slot (_fill_new_card,
//           zeros when the deck is empty or in the tree), or a deck reserve into the slot
//           (nothing in the tree: deterministic reserve-from-deck draws no card)
//   shift   _buy_reserve (:554-560) closes the bought card's slot
//   gems    reserving grants a gold if the bank has one; then the action's take vector
//           (_get_gems :585-593) and summed give-back vectors (_give_gems :685-694,
//           exchanges :697-761) as one byte-wise row update
//   round   round counter +1, int8 (:287)
// Actions 405..408 are a no-op + round increment (the reference's select-noble stub does
// not parse and pass reads give_ids3 out of bounds; DESIGN.md "Defined deviations").
// Returns the next player.
// KIND (move_kind_of) >= 0 specialises the pipeline to one kind of move when the caller knows
// it: the stages that kind never uses are compiled out.
enum { MK_GEMS = 0, MK_BUY = 1, MK_RESERVE = 2, MK_BUY_RESERVED = 3 };
// same classification without the table: the reserve actions are 12-26 (visible / deck)
// and 290-364 (reserve-and-give-back), the rows of K_ACT_RSV >= 0 (gen_tables.py)
__device__ __forceinline__ int move_kind_of(int a) {
    return a < 12 ? MK_BUY : (a < 27 ? MK_RESERVE : (a < 30 ? MK_BUY_RESERVED :
                                                     (a >= 290 && a < 365 ? MK_RESERVE : MK_GEMS)));
}

// make_move for a visible-card buy (KIND == MK_BUY) with every row it touches read up front
// and kept in registers: the same stages and results as the fixed pipeline below (_buy_card
// :458-474, _give_nobles_if_earned :763-768, _fill_new_card :445-450, round +1 :287), but
// one LDS round trip for the reads instead of a chain of write-then-reread steps (the buy
// wave is the longest move pipeline of the rollout kernel).
template <int N>
__device__ __forceinline__ int make_move_buy(int8_t *s, int a, int p, bool det, Chance &ch) {
    using Lx = Lay<N>;
    const int r = Lx::TIERS + 2 * a, tier = a >> 2;
    const uint64_t cost = row(s, r), gain = row(s, r + 1);
    uint64_t gems = row(s, Lx::GEMS + p), bank = row(s, Lx::BANK);
    const uint64_t cards = row(s, Lx::CARDS + p);
    uint64_t nob[Lx::NN];
#pragma unroll
    for (int i = 0; i < Lx::NN; i++) nob[i] = row(s, Lx::NOBLES + i);
    uint64_t cnt = row(s, Lx::DECKS + 2 * tier), bits = row(s, Lx::DECKS + 2 * tier + 1);
    const bool draw = !det && sum5(cnt) != 0;
    double u0 = 0.0, u1 = 0.0;
    if (draw) { u0 = ch.draw(); u1 = ch.draw(); }
    // _buy_card: coloured gems first, gold for what is missing
    int miss = 0;
    uint64_t paid = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const int cc = bt(cost, c), gc = bt(gems, c), kc = bt(cards, c);
        const int d = cc - gc - kc;
        miss += d > 0 ? d : 0;
        int need = cc - kc;
        need = need > 0 ? need : 0;
        paid |= (uint64_t)(uint8_t)(need < gc ? need : gc) << (8 * c);
    }
    gems = bytes_sub(gems, paid);
    bank = bytes_add(bank, paid);
    gems = with_bt(gems, 5, bt(gems, 5) - miss);
    bank = with_bt(bank, 5, bt(bank, 5) + miss);
    const uint64_t ncards = bytes_add(cards, gain);
    // _fill_new_card: one deck draw into the bought slot (zeros when the deck is empty)
    uint64_t ncost = 0, ngain = 0;
    if (draw) {
        int color, idx;
        deck_pick(cnt, bits, u0, u1, ch.tab, color, idx);
        deck_take(cnt, bits, color, idx);
        ncost = ch.tab.cards[tier * 40 + color * 8 + idx][0];
        ngain = ch.tab.cards[tier * 40 + color * 8 + idx][1];
    }
    row(s, Lx::CARDS + p) = ncards;
#pragma unroll
    for (int i = 0; i < Lx::NN; i++) {
        if (sum5(nob[i]) > 0 && ge5(ncards, nob[i])) {
            row(s, Lx::PNOB + Lx::NN * p + i) = nob[i];
            row(s, Lx::NOBLES + i) = 0;
        }
    }
    if (draw) {
        row(s, Lx::DECKS + 2 * tier + 1) = bits;
        row(s, Lx::DECKS + 2 * tier) = cnt;
    }
    row(s, r) = ncost;
    row(s, r + 1) = ngain;
    row(s, Lx::GEMS + p) = gems;
    row(s, Lx::BANK) = with_bt(bank, 6, bt(bank, 6) + 1);
    return (p + 1) % N;
}

// make_move for a reserve (KIND == MK_RESERVE) in the same register-resident form: the
// player's reserve slots, the reserved visible card, the tier's deck, gems and bank read in
// one LDS round trip, then the same stages as the fixed pipeline below (_reserve
// :517-536: first free slot, visible card or a deck draw, the gold, the action's take /
// give-back vectors, round +1), all writes at the end (every row written is distinct).
template <int N>
__device__ __forceinline__ int make_move_reserve(int8_t *s, int a, int p, bool det, Chance &ch) {
    using Lx = Lay<N>;
    const int rsv = (int)ch.tab.act_rsv[a];
    const uint64_t take = ch.tab.act_take[a], give = ch.tab.act_give[a];
    const bool vis = rsv < 12;
    const int tier = vis ? rsv >> 2 : rsv - 12, R = Lx::RSV + 6 * p;
    const int vr = Lx::TIERS + 2 * (vis ? rsv : 0);
    const uint64_t c0 = row(s, R), c1 = row(s, R + 2), c2 = row(s, R + 4);
    const uint64_t vcost = row(s, vr), vgain = row(s, vr + 1);
    uint64_t cnt = row(s, Lx::DECKS + 2 * tier), bits = row(s, Lx::DECKS + 2 * tier + 1);
    uint64_t gems = row(s, Lx::GEMS + p), bank = row(s, Lx::BANK);
    const int slot = sum5(c0) == 0 ? R : (sum5(c1) == 0 ? R + 2 : (sum5(c2) == 0 ? R + 4 : -1));
    const bool draw = !det && sum5(cnt) != 0;
    uint64_t cost = 0, gain = 0;
    if (draw) {
        const double u0 = ch.draw(), u1 = ch.draw();
        int color, idx;
        deck_pick(cnt, bits, u0, u1, ch.tab, color, idx);
        deck_take(cnt, bits, color, idx);
        cost = ch.tab.cards[tier * 40 + color * 8 + idx][0];
        gain = ch.tab.cards[tier * 40 + color * 8 + idx][1];
    }
    if (bt(bank, 5) > 0) {
        gems = with_bt(gems, 5, bt(gems, 5) + 1);
        bank = with_bt(bank, 5, bt(bank, 5) - 1);
    }
    gems = bytes_sub(bytes_add(gems, take), give);
    bank = bytes_add(bytes_sub(bank, take), give);
    if (vis) {
        if (slot >= 0) {
            row(s, slot) = vcost;
            row(s, slot + 1) = vgain;
        }
        row(s, vr) = cost;
        row(s, vr + 1) = gain;
    } else if (draw && slot >= 0) {
        row(s, slot) = cost;
        row(s, slot + 1) = gain;
    }
    if (draw) {
        row(s, Lx::DECKS + 2 * tier + 1) = bits;
        row(s, Lx::DECKS + 2 * tier) = cnt;
    }
    row(s, Lx::GEMS + p) = gems;
    row(s, Lx::BANK) = with_bt(bank, 6, bt(bank, 6) + 1);
    return (p + 1) % N;
}

template <int N, int KIND = -1>
__device__ __forceinline__ int make_move(int8_t *s, int a, int p, bool det, Chance &ch) {
    using Lx = Lay<N>;
    if constexpr (KIND == MK_BUY) return make_move_buy<N>(s, a, p, det, ch);
    if constexpr (KIND == MK_RESERVE) return make_move_reserve<N>(s, a, p, det, ch);
    constexpr bool ANY = KIND < 0;
    const int rsv = ANY || KIND == MK_RESERVE ? (int)ch.tab.act_rsv[a] : -1;
    const bool vec = ANY || KIND == MK_GEMS || KIND == MK_RESERVE;
    const uint64_t take = vec ? ch.tab.act_take[a] : 0, give = vec ? ch.tab.act_give[a] : 0;
    const bool buy_vis = ANY ? a < 12 : KIND == MK_BUY;
    const bool buy_rsv = ANY ? (a >= 27 && a < 30) : KIND == MK_BUY_RESERVED;
    SPL_PROBE(10)
    if (buy_vis || buy_rsv) buy_card<N>(s, buy_vis ? Lx::TIERS + 2 * a : Lx::RSV + 6 * p + 2 * (a - 27), p);
    SPL_PROBE(11)
    int slot = -1;
    if (rsv >= 0) {
        for (int k = 2; k >= 0; k--)
            if (sum5(row(s, Lx::RSV + 6 * p + 2 * k)) == 0) slot = Lx::RSV + 6 * p + 2 * k;
        if (rsv < 12 && slot >= 0) {
            const int r = Lx::TIERS + 2 * rsv;
            row(s, slot) = row(s, r);
            row(s, slot + 1) = row(s, r + 1);
        }
    }
    SPL_PROBE(12)
    const int tier = buy_vis ? a >> 2 : (rsv >= 0 ? (rsv < 12 ? rsv >> 2 : rsv - 12) : -1);
    if (tier >= 0) {
        uint64_t cost = 0, gain = 0;
        const bool got = !det && deck_card<N>(s, tier, ch, cost, gain);
        if (buy_vis || rsv < 12) {
            const int r = Lx::TIERS + 2 * (buy_vis ? a : rsv);
            row(s, r) = cost;
            row(s, r + 1) = gain;
        } else if (got && slot >= 0) {
            row(s, slot) = cost;
            row(s, slot + 1) = gain;
        }
    }
    SPL_PROBE(13)
    if (buy_rsv) {
        for (int r = Lx::RSV + 6 * p + 2 * (a - 27); r < Lx::RSV + 6 * p + 4; r++) row(s, r) = row(s, r + 2);
        row(s, Lx::RSV + 6 * p + 4) = 0;
        row(s, Lx::RSV + 6 * p + 5) = 0;
    }
    uint64_t bank = row(s, Lx::BANK), gems = row(s, Lx::GEMS + p);
    if (rsv >= 0 && bt(bank, 5) > 0) {
        gems = with_bt(gems, 5, bt(gems, 5) + 1);
        bank = with_bt(bank, 5, bt(bank, 5) - 1);
    }
    gems = bytes_sub(bytes_add(gems, take), give);
    bank = bytes_add(bytes_sub(bank, take), give);
    row(s, Lx::GEMS + p) = gems;
    row(s, Lx::BANK) = with_bt(bank, 6, bt(bank, 6) + 1);
    SPL_PROBE(14)
    return (p + 1) % N;
}

// ------------------------------------------------------------------ end of game
// Row views: an LDS board (8-byte rows) or an HBM board (7-byte rows, byte-assembled).
struct LdsRows {
    const int8_t *s;
    __device__ __forceinline__ uint64_t operator()(int r) const { return row(s, r); }
};
struct HbmRows {
    const int8_t *s;
    __device__ __forceinline__ uint64_t operator()(int r) const {
        uint64_t v = 0;
#pragma unroll
        for (int c = 0; c < 7; c++) v |= (uint64_t)(uint8_t)s[7 * r + c] << (8 * c);
        return v;
    }
};

template <int N, class V>
__device__ __forceinline__ int score_rows(const V &rows, int p) {   // :217-220 (hard-coded 3)
    using Lx = Lay<N>;
    int v = bt(rows(Lx::CARDS + p), 6);
    for (int i = 0; i < 3; i++) v += bt(rows(Lx::PNOB + 3 * p + i), 6);
    return v;
}

// check_end_game + judge (:320-334, :306-318)
template <int N, class V>
__device__ __forceinline__ void check_end_rows(const V &rows, float out[N]) {
    using Lx = Lay<N>;
#pragma unroll
    for (int i = 0; i < N; i++) out[i] = 0.f;
    const int r = (uint8_t)bt(rows(Lx::BANK), 6);
    if (r % N != 0) return;
    int sc[N], mx = -1000;
#pragma unroll
    for (int p = 0; p < N; p++) {
        sc[p] = (int8_t)score_rows<N>(rows, p);
        mx = sc[p] > mx ? sc[p] : mx;
    }
    if (!(mx >= 15 || r >= Lx::MAXMOVES)) return;
    int nmax = 0;
#pragma unroll
    for (int p = 0; p < N; p++) nmax += sc[p] == mx;
    if (nmax == 1) {
#pragma unroll
        for (int p = 0; p < N; p++) out[p] = sc[p] == mx ? 1.f : -1.f;
        return;
    }
    int m[N], mn = 127;
#pragma unroll
    for (int p = 0; p < N; p++) {
        m[p] = (int8_t)sum5(rows(Lx::CARDS + p));
        if (sc[p] < mx) m[p] = -25;                          // int8(999) (:313)
        mn = m[p] < mn ? m[p] : mn;
    }
    int cnt = 0;
#pragma unroll
    for (int p = 0; p < N; p++) cnt += m[p] == mn;
#pragma unroll
    for (int p = 0; p < N; p++) out[p] = m[p] == mn ? (cnt > 1 ? 0.01f : 1.f) : -1.f;
}
template <int N>
__device__ __forceinline__ void check_end(const int8_t *lds, float out[N]) { check_end_rows<N>(LdsRows{lds}, out); }

// check_end with the round counter after the move given (r, uint8: the caller read it
// before the move), so the common no-end case reads no row the move wrote
template <int N>
__device__ __forceinline__ void check_end_round(const int8_t *lds, int r, float out[N]) {
    if (r % N != 0) {
#pragma unroll
        for (int i = 0; i < N; i++) out[i] = 0.f;
        return;
    }
    check_end<N>(lds, out);
}
template <int N>
__device__ __forceinline__ int get_score(const int8_t *lds, int p) { return score_rows<N>(LdsRows{lds}, p); }

// ------------------------------------------------------------------ new game
// Board.init_game (:222-246) on a zeroed board. Card draws use the chance source; the
// noble draw is a partial Fisher-Yates on the same stream (the reference's
// np.random.choice is unseeded). The decks start full, so each of the 12 visible cards
// takes exactly two draws: uniforms 8t..8t+7 deal tier t, 24..24+nn-1 pick the nobles.
// The four parts touch disjoint rows and are dealt concurrently by lanes 0-3.
constexpr int DEAL_DRAWS = 29;                    // 24 card draws + up to 5 nobles

// The four draws of a tier touch only its deck rows: they run on registers (deck rows and
// the 8 uniforms loaded once), and the deck and visible-card rows are written at the end.
template <int N>
__device__ __forceinline__ void deal_tier(int8_t *s, int t, const double *u, const Tabs &tab) {
    using Lx = Lay<N>;
    const uint64_t len = t == 0 ? 8 : (t == 1 ? 6 : 4);
    uint64_t cnt = len * 0x0000000101010101ull;
    uint64_t bits = (uint8_t)(0xFFu << (8 - len)) * 0x0000000101010101ull;
    double uu[8];
#pragma unroll
    for (int k = 0; k < 8; k++) uu[k] = u[8 * t + k];
    int card[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int color, idx;
        deck_pick(cnt, bits, uu[2 * i], uu[2 * i + 1], tab, color, idx);
        deck_take(cnt, bits, color, idx);
        card[i] = t * 40 + color * 8 + idx;
    }
    row(s, Lx::DECKS + 2 * t) = cnt;
    row(s, Lx::DECKS + 2 * t + 1) = bits;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        row(s, Lx::TIERS + 8 * t + 2 * i) = tab.cards[card[i]][0];
        row(s, Lx::TIERS + 8 * t + 2 * i + 1) = tab.cards[card[i]][1];
    }
}
template <int N>
__device__ __forceinline__ void deal_nobles_bank(int8_t *s, const double *u) {
    using Lx = Lay<N>;
    const uint64_t g = N == 2 ? 4 : (N == 3 ? 5 : 7);
    row(s, Lx::BANK) = g * 0x0000000101010101ull | (5ull << 40);
    uint64_t perm = 0x9876543210ull;              // 10 nibbles: partial Fisher-Yates
    for (int i = 0; i < Lx::NN; i++) {
        const int j = i + (int)floor(u[24 + i] * (double)(10 - i));
        const uint64_t pi = (perm >> (4 * i)) & 15, pj = (perm >> (4 * j)) & 15;
        perm &= ~((15ull << (4 * i)) | (15ull << (4 * j)));
        perm |= (pj << (4 * i)) | (pi << (4 * j));
    }
    for (int i = 0; i < Lx::NN; i++) row(s, Lx::NOBLES + i) = K_NOBLE_ROWS[(perm >> (4 * i)) & 15];
}

// uniforms d0 .. d0+n-1 of a Philox sequence into dst (n <= 126), one block per lane
__device__ __forceinline__ void wave_philox_uniforms(double *dst, uint64_t seed, uint32_t board,
                                                     uint32_t stream, uint32_t d0, int n) {
    const int l = lane_id();
    const uint32_t blk = (d0 >> 1) + l;
    if ((int)(2 * blk) < (int)(d0 + n)) {
        double a, b;
        philox_pair(seed, board, stream, blk, a, b);
        const int i = (int)(2 * blk) - (int)d0;
        if (i >= 0) dst[i] = a;
        if (i + 1 < n) dst[i + 1] = b;
    }
    __builtin_amdgcn_wave_barrier();
}

// ---- rollout deals keyed by game number (spl_rollout_run): the deal of board b's game g
// (games counted from the initial deal = 0) takes uniforms 0..DEAL_DRAWS-1 of Philox stream
// DEAL_STREAM | g, so it can be computed before the game that precedes it ends.
constexpr uint32_t DEAL_STREAM = 0x80000000u;
struct DealRec {                      // a dealt board in 72 bytes
    uint64_t cnt[3], bits[3];         // deck rows after the 12 visible cards are drawn
    uint64_t perm;                    // noble permutation (nibbles, partial Fisher-Yates)
    uint8_t card[12];                 // visible cards, tier*40 + colour*8 + index
    uint32_t pad;
};
// lane-per-board: the same draws as deal_tier / deal_nobles_bank, kept as a record
template <int N>
__device__ __forceinline__ void lane_deal_record(uint64_t seed, uint32_t board, uint32_t game, const Tabs &tab,
                                                 DealRec &r) {
    double u[DEAL_DRAWS + 1];
#pragma unroll
    for (int k = 0; k < (DEAL_DRAWS + 1) / 2; k++) philox_pair(seed, board, DEAL_STREAM | game, k, u[2 * k], u[2 * k + 1]);
#pragma unroll
    for (int t = 0; t < 3; t++) {
        const uint64_t len = t == 0 ? 8 : (t == 1 ? 6 : 4);
        uint64_t cnt = len * 0x0000000101010101ull;
        uint64_t bits = (uint8_t)(0xFFu << (8 - len)) * 0x0000000101010101ull;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int color, idx;
            deck_pick(cnt, bits, u[8 * t + 2 * i], u[8 * t + 2 * i + 1], tab, color, idx);
            deck_take(cnt, bits, color, idx);
            r.card[4 * t + i] = (uint8_t)(t * 40 + color * 8 + idx);
        }
        r.cnt[t] = cnt;
        r.bits[t] = bits;
    }
    uint64_t perm = 0x9876543210ull;
#pragma unroll
    for (int i = 0; i < Lay<N>::NN; i++) {
        const int j = i + (int)floor(u[24 + i] * (double)(10 - i));
        const uint64_t pi = (perm >> (4 * i)) & 15, pj = (perm >> (4 * j)) & 15;
        perm &= ~((15ull << (4 * i)) | (15ull << (4 * j)));
        perm |= (pj << (4 * i)) | (pi << (4 * j));
    }
    r.perm = perm;
}
// one quarter of lane_deal_record: part t < 3 deals tier t (draws 8t .. 8t+7: Philox
// blocks 4t .. 4t+3), part 3 the nobles (draws 24 .. 28: blocks 12 .. 14). The parts write
// disjoint fields, so four lanes build a record together at a quarter of the latency.
template <int N>
__device__ __forceinline__ void lane_deal_part(uint64_t seed, uint32_t board, uint32_t game, int part,
                                               const Tabs &tab, DealRec &r) {
    if (part < 3) {
        const int t = part;
        double u[8];
#pragma unroll
        for (int k = 0; k < 4; k++) philox_pair(seed, board, DEAL_STREAM | game, 4 * t + k, u[2 * k], u[2 * k + 1]);
        const uint64_t len = t == 0 ? 8 : (t == 1 ? 6 : 4);
        uint64_t cnt = len * 0x0000000101010101ull;
        uint64_t bits = (uint8_t)(0xFFu << (8 - len)) * 0x0000000101010101ull;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int color, idx;
            deck_pick(cnt, bits, u[2 * i], u[2 * i + 1], tab, color, idx);
            deck_take(cnt, bits, color, idx);
            r.card[4 * t + i] = (uint8_t)(t * 40 + color * 8 + idx);
        }
        r.cnt[t] = cnt;
        r.bits[t] = bits;
    } else {
        double u[6];
#pragma unroll
        for (int k = 0; k < 3; k++) philox_pair(seed, board, DEAL_STREAM | game, 12 + k, u[2 * k], u[2 * k + 1]);
        uint64_t perm = 0x9876543210ull;
#pragma unroll
        for (int i = 0; i < Lay<N>::NN; i++) {
            const int j = i + (int)floor(u[i] * (double)(10 - i));
            const uint64_t pi = (perm >> (4 * i)) & 15, pj = (perm >> (4 * j)) & 15;
            perm &= ~((15ull << (4 * i)) | (15ull << (4 * j)));
            perm |= (pj << (4 * i)) | (pi << (4 * j));
        }
        r.perm = perm;
    }
}
// wave-collective: the board a record describes (every row written once; = wave_init_game)
template <int N>
__device__ __forceinline__ void wave_apply_deal(int8_t *s, const DealRec &r, const Tabs &tab) {
    using Lx = Lay<N>;
    const uint64_t g = N == 2 ? 4 : (N == 3 ? 5 : 7);
    for (int i = lane_id(); i < Lx::ROWS; i += 64) {
        uint64_t v = 0;
        if (i == Lx::BANK) {
            v = g * 0x0000000101010101ull | (5ull << 40);
        } else if (i >= Lx::TIERS && i < Lx::TIERS + 24) {
            const int k = i - Lx::TIERS;
            v = tab.cards[r.card[4 * (k >> 3) + ((k & 7) >> 1)]][k & 1];
        } else if (i >= Lx::DECKS && i < Lx::DECKS + 6) {
            const int k = i - Lx::DECKS;
            v = (k & 1) ? r.bits[k >> 1] : r.cnt[k >> 1];
        } else if (i >= Lx::NOBLES && i < Lx::NOBLES + Lx::NN) {
            v = K_NOBLE_ROWS[(r.perm >> (4 * (i - Lx::NOBLES))) & 15];
        }
        row(s, i) = v;
    }
    __builtin_amdgcn_wave_barrier();
}

// wave-collective new game from DEAL_DRAWS uniforms u (LDS or HBM)
template <int N>
__device__ __forceinline__ void wave_init_game(int8_t *s, const double *u, const Tabs &tab = Tabs{}) {
    const int l = lane_id();
    for (int r = l; r < Lay<N>::ROWS; r += 64) row(s, r) = 0;
    __builtin_amdgcn_wave_barrier();
    if (l < 3) deal_tier<N>(s, l, u, tab);
    else if (l == 3) deal_nobles_bank<N>(s, u);
    __builtin_amdgcn_wave_barrier();
}

// store a wave-uniform packed mask (7 words) from lane 0 (no per-lane word selection:
// selecting w[lane] makes hipcc spill the array to scratch)
__device__ __forceinline__ void store_mask(uint64_t *dst, const uint64_t w[7]) {
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < 7; k++) dst[k] = w[k];
    }
}

// k-th set bit of the packed mask (k < popcount): the word by prefix popcounts, then one
// halving search inside it (no runtime-indexed arrays: those go to scratch)
__device__ __forceinline__ int select_bit(const uint64_t w[7], int k) {
    uint64_t x = w[6];
    int base = 384, rem = k;
    int pre = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const int c = __popcll(w[j]);
        const bool here = k >= pre && k < pre + c;
        x = here ? w[j] : x;
        base = here ? 64 * j : base;
        rem = here ? k - pre : rem;
        pre += c;
    }
    if (base == 384) rem = k - pre;
    return base + kth_bit64(x, rem);
}

}  // namespace spl
