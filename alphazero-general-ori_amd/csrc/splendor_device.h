// splendor_device.h — gfx950 device implementation of the Splendor rules.
//
// Execution model: ONE WAVE (64 lanes) PER BOARD. The board record (7*R int8, the
// reference's (R,7) state, SplendorLogicNumba.py:291-303) is staged in LDS; the wave
// evaluates the 409-action legality mask as 7 x 64-lane chunks and packs each with a
// ballot, and applies a transition with wave-uniform control flow (no divergence, every
// lane runs the same instructions on broadcast LDS reads).
//
// Semantics follow the reference bit-for-bit (incl. Numba int8 wraps); each function
// cites the reference lines it restates. Parity is checked against the CPU oracle
// (oracle/) which is itself pinned to golden vectors recorded from the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "splendor_tables.h"

namespace spl {

// condition codes of K_ACTION_DESC (gen_tables.py)
enum { C_ALWAYS, C_RSV_LIMIT, C_TAKE1, C_TAKE2D, C_TAKE3, C_TAKE2S, C_EX8, C_EX9, C_EX10,
       C_EX10G, C_NEVER };

template <int N>
struct Lay {  // row offsets of the (R,7) state (SplendorLogicNumba.py:296-303)
    static constexpr int NN = N + 1;                 // nobles on the table
    static constexpr int ROWS = 32 + 10 * N + N * N;
    static constexpr int S = 7 * ROWS;               // bytes per board
    static constexpr int SPAD = (S + 15) & ~15;      // LDS slot (16-B aligned)
    static constexpr int BANK = 0, TIERS = 1, DECKS = 25, NOBLES = 31;
    static constexpr int GEMS = 32 + N, PNOB = 32 + 2 * N, CARDS = 32 + 3 * N + N * N;
    static constexpr int RSV = 32 + 4 * N + N * N;
    static constexpr int PROWS = ROWS - GEMS;        // player-specific rows
    static constexpr int MAXMOVES = 62 * N;
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ int sum5(const int8_t *r) { return r[0] + r[1] + r[2] + r[3] + r[4]; }
__device__ __forceinline__ int sum7(const int8_t *r) { return sum5(r) + r[5] + r[6]; }

// ------------------------------------------------------------------ chance source
// Philox4x32-10 (Salmon et al. 2011); identical to oracle/splendor_oracle.c or_philox4x32.
__device__ __forceinline__ double philox_u01(uint64_t seed, uint32_t board, uint32_t stream,
                                             uint32_t draw) {
    uint32_t c0 = draw, c1 = board, c2 = stream, c3 = 0x53504C44u;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return ((double)(c0 >> 5) * 67108864.0 + (double)(c1 >> 6)) * (1.0 / 9007199254740992.0);
}

// Either an explicit stream of doubles (parity with recorded reference draws) or Philox.
struct Chance {
    const double *u;   // explicit uniforms for this board, or nullptr -> Philox
    uint64_t seed;
    uint32_t board, stream, next;
    __device__ __forceinline__ double draw() {
        double r = u ? u[next] : philox_u01(seed, board, stream, next);
        ++next;
        return r;
    }
};

// my_random_choice: searchsorted(cumsum(prob), U, side="right") (SplendorLogicNumba.py:39-41)
__device__ __forceinline__ int rand_choice(const double *p, int len, double u) {
    double c = 0.0;
    for (int i = 0; i < len; i++) {
        c += p[i];
        if (c > u) return i;
    }
    return len;
}

// ------------------------------------------------------------------ gem vectors
__device__ __forceinline__ void move_gems(int8_t *bank, int8_t *gems, const int8_t *v, int sign) {
#pragma unroll
    for (int c = 0; c < 5; c++) {
        bank[c] = (int8_t)(bank[c] - sign * v[c]);
        gems[c] = (int8_t)(gems[c] + sign * v[c]);
    }
}

// ------------------------------------------------------------------ wave helpers
// copy `bytes` (multiple of 4, 4-aligned) between global and LDS with dword lanes
__device__ __forceinline__ void wave_copy4(int8_t *dst, const int8_t *src, int bytes) {
    const int l = lane_id();
    for (int i = 4 * l; i < bytes; i += 256)
        *reinterpret_cast<int32_t *>(dst + i) = *reinterpret_cast<const int32_t *>(src + i);
}
__device__ __forceinline__ void wave_copy1(int8_t *dst, const int8_t *src, int bytes) {
    const int l = lane_id();
    for (int i = l; i < bytes; i += 64) dst[i] = src[i];
}
template <int N>
__device__ __forceinline__ void wave_copy_board(int8_t *dst, const int8_t *src) {
    if constexpr (Lay<N>::S % 4 == 0) wave_copy4(dst, src, Lay<N>::S);
    else wave_copy1(dst, src, Lay<N>::S);
    __builtin_amdgcn_wave_barrier();
}

// swap_players (SplendorLogicNumba.py:338-347): roll each player block so that player k
// becomes player 0. Noble block rolls by 3k (hard-coded 3, :345). dst may equal src.
template <int N>
__device__ __forceinline__ void wave_roll_players(int8_t *dst, const int8_t *src, int k) {
    using Lx = Lay<N>;
    constexpr int PB = 7 * Lx::PROWS;
    constexpr int ITER = (PB + 63) / 64;
    const int l = lane_id();
    int8_t v[ITER];
#pragma unroll
    for (int j = 0; j < ITER; j++) {
        int i = l + 64 * j;
        v[j] = 0;
        if (i < PB) {
            int r = i / 7, c = i - 7 * (i / 7), sr;
            if (r < N) sr = (r + k) % N;
            else if (r < N + N * Lx::NN) sr = N + (r - N + 3 * k) % (N * Lx::NN);
            else if (r < 2 * N + N * Lx::NN) sr = N + N * Lx::NN + (r - N - N * Lx::NN + k) % N;
            else sr = 2 * N + N * Lx::NN + (r - 2 * N - N * Lx::NN + 6 * k) % (6 * N);
            v[j] = src[7 * (Lx::GEMS + sr) + c];
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < ITER; j++) {
        int i = l + 64 * j;
        if (i < PB) dst[7 * Lx::GEMS + i] = v[j];
    }
    if (dst != src) {  // shared (non-player) rows
        for (int i = l; i < 7 * Lx::GEMS; i += 64) dst[i] = src[i];
    }
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ legality mask
// Board.valid_moves (SplendorLogicNumba.py:251-265). Wave-collective; returns the packed
// 409-bit mask in w[0..6] (bit a%64 of word a/64), identical in every lane.
//
// Phase 1 packs 120 per-board predicates into two ballots:
//   F0: 0-11 _valid_buy (:476-501)  12-26 _valid_reserve(is_limit=False) (:508-515)
//       27-29 _valid_buy_reserve (:538-552)  30-54 bank holds DIFF3[i] (:562-568)
//       55-59 bank[c] >= 4 (:578-583)
//   F1: 0-19 _valid_give_gems(+identical) (:595-613)  20-59 _valid_give_gems3 (:602-607)
// Phase 2 evaluates one action per lane from K_ACTION_DESC: flag0 & flag1 & condition,
// the conditions restating the token-count branches of _valid_get_gems (:570-574) and
// _valid_exchange (:615-680). Pass (408) is set iff nothing else is legal (:263).
template <int N>
__device__ __forceinline__ void wave_valid_moves(const int8_t *s, int p, int lim, uint64_t w[7]) {
    using Lx = Lay<N>;
    const int l = lane_id();
    const int8_t *bank = s;
    const int8_t *gems = s + 7 * (Lx::GEMS + p);
    const int8_t *cards = s + 7 * (Lx::CARDS + p);
    const int8_t *rsv = s + 7 * (Lx::RSV + 6 * p);
    const int T = sum7(gems), gold = gems[5], bgold = bank[5];
    int nspec = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) nspec += bank[c] != 0;
    const bool slot_free = sum5(rsv + 35) == 0;   // third slot's gain row (:514)

    bool f = false;
    if (l < 12 || (l >= 27 && l < 30)) {          // affordability (cards or reserved)
        const int8_t *cost = l < 12 ? s + 7 * (Lx::TIERS + 2 * l) : rsv + 14 * (l - 27);
        int miss = 0, tot = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            int d = cost[c] - gems[c] - cards[c];
            miss += d > 0 ? d : 0;
            tot += cost[c];
        }
        f = miss <= gold && tot != 0;
    } else if (l < 27) {                          // reservable slot non-empty
        int i = l - 12;
        const int8_t *row = i < 12 ? s + 7 * (Lx::TIERS + 2 * i) : s + 7 * (Lx::DECKS + 2 * (i - 12));
        f = sum5(row) != 0 && slot_free;
    } else if (l < 55) {                          // bank can supply take vector
        const int8_t *v = K_TAKE[l - 30];
        bool ok = true;
#pragma unroll
        for (int c = 0; c < 5; c++) ok &= (bank[c] - v[c]) >= 0;
        f = ok;
    } else if (l < 60) {
        f = bank[l - 55] >= 4;
    }
    const uint64_t F0 = __ballot(f);
    f = false;
    if (l >= 15 && l < 20) {                      // two identical gems
        f = gems[l - 15] >= 2;
    } else if (l < 60) {                          // player can give back vector
        const int8_t *v = l < 15 ? K_GIVE[l] : K_SPEC3[l - 20];
        bool ok = true;
#pragma unroll
        for (int c = 0; c < 5; c++) ok &= (gems[c] - v[c]) >= 0;
        f = ok;
    }
    const uint64_t F1 = __ballot(f);

    // wave-uniform condition bits, indexed by condition code
    const bool ex_any = T > 7;
    const bool ex8 = ex_any && T == lim - 2;
    const bool ex9 = ex_any && !ex8 && T == lim - 1;
    const bool ex10 = ex_any && !ex8 && !ex9;
    uint32_t cond = 0;
    cond |= 1u << C_ALWAYS;
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
        const int a = 64 * k + l;
        const uint32_t d = a < 409 ? K_ACTION_DESC[a] : (uint32_t)(C_NEVER << 16);
        const bool f0 = !((d >> 6) & 1) || ((F0 >> (d & 63)) & 1);
        const bool f1 = !((d >> 14) & 1) || ((F1 >> ((d >> 8) & 63)) & 1);
        const bool c = (cond >> ((d >> 16) & 15)) & 1;
        w[k] = __ballot(f0 && f1 && c);
        any |= w[k];
    }
    if (!any) w[6] |= 1ull << (408 - 384);
}

// ------------------------------------------------------------------ transition
// _get_deck_card (SplendorLogicNumba.py:400-420): colour ~ remaining count, then card ~
// remaining bit; bitfield stored as int8 (packbits wrap, :44-46). Returns false if empty.
template <int N>
__device__ __forceinline__ bool deck_card(int8_t *s, int tier, Chance &ch, int8_t out[14]) {
    using Lx = Lay<N>;
    int8_t *cnt = s + 7 * (Lx::DECKS + 2 * tier), *bits = cnt + 7;
    const int tot = sum5(cnt);
    if (tot == 0) return false;
    // searchsorted(cumsum(cnt / tot), u, 'right'), evaluated on the fly (no local arrays)
    const double u0 = ch.draw();
    int color = 4;
    double c = 0.0;
#pragma unroll
    for (int k = 0; k < 5; k++) {
        c += (double)cnt[k] / (double)tot;
        if (c > u0) { color = k; break; }
    }
    const uint32_t b = (uint8_t)bits[color];
    const double nbits = (double)__builtin_popcount(b);
    const double u1 = ch.draw();
    int idx = 7;
    c = 0.0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        c += (double)((b >> (7 - k)) & 1) / nbits;
        if (c > u1) { idx = k; break; }
    }
    bits[color] = (int8_t)(b & ~(1u << (7 - idx)));
    cnt[color] = (int8_t)(cnt[color] - 1);
    const int8_t *cd = K_CARDS[tier * 40 + color * 8 + idx];
#pragma unroll
    for (int c = 0; c < 14; c++) out[c] = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) out[c] = cd[c];
    out[7 + cd[5]] = 1;
    out[13] = cd[6];
    return true;
}

template <int N>
__device__ __forceinline__ void fill_new_card(int8_t *s, int tier, int idx, bool det, Chance &ch) {
    int8_t *slot = s + 7 * (Lay<N>::TIERS + 8 * tier + 2 * idx);
    int8_t c[14];
    const bool got = !det && deck_card<N>(s, tier, ch, c);
#pragma unroll
    for (int i = 0; i < 14; i++) slot[i] = got ? c[i] : 0;   // _fill_new_card (:445-450)
}

// _give_nobles_if_earned (:763-768): every qualifying noble, stored at row nn*p+i
template <int N>
__device__ __forceinline__ void give_nobles(int8_t *s, int p) {
    using Lx = Lay<N>;
    const int8_t *cards = s + 7 * (Lx::CARDS + p);
    for (int i = 0; i < Lx::NN; i++) {
        int8_t *nob = s + 7 * (Lx::NOBLES + i);
        bool ok = sum5(nob) > 0;
#pragma unroll
        for (int c = 0; c < 5; c++) ok &= cards[c] >= nob[c];
        if (ok) {
            int8_t *dst = s + 7 * (Lx::PNOB + Lx::NN * p + i);
#pragma unroll
            for (int c = 0; c < 7; c++) { dst[c] = nob[c]; }
#pragma unroll
            for (int c = 0; c < 7; c++) nob[c] = 0;
        }
    }
}

// _buy_card (:458-474)
template <int N>
__device__ __forceinline__ void buy_card(int8_t *s, int cost_row, int p) {
    using Lx = Lay<N>;
    int8_t *bank = s, *gems = s + 7 * (Lx::GEMS + p), *cards = s + 7 * (Lx::CARDS + p);
    int8_t cost[5], gain[7];
#pragma unroll
    for (int c = 0; c < 5; c++) cost[c] = s[7 * cost_row + c];
#pragma unroll
    for (int c = 0; c < 7; c++) gain[c] = s[7 * cost_row + 7 + c];
    int miss = 0;
#pragma unroll
    for (int c = 0; c < 5; c++) {
        int d = cost[c] - gems[c] - cards[c];
        miss += d > 0 ? d : 0;
    }
#pragma unroll
    for (int c = 0; c < 5; c++) {
        int need = cost[c] - cards[c];
        need = need > 0 ? need : 0;
        int paid = need < gems[c] ? need : gems[c];
        gems[c] = (int8_t)(gems[c] - paid);
        bank[c] = (int8_t)(bank[c] + paid);
    }
    gems[5] = (int8_t)(gems[5] - miss);
    bank[5] = (int8_t)(bank[5] + miss);
#pragma unroll
    for (int c = 0; c < 7; c++) cards[c] = (int8_t)(cards[c] + gain[c]);
    give_nobles<N>(s, p);
}

// _reserve (:517-536)
template <int N>
__device__ __forceinline__ void reserve(int8_t *s, int i, int p, bool det, Chance &ch) {
    using Lx = Lay<N>;
    int slot = -1;
    for (int k = 2; k >= 0; k--)
        if (sum5(s + 7 * (Lx::RSV + 6 * p + 2 * k)) == 0) slot = Lx::RSV + 6 * p + 2 * k;
    if (i < 12) {
        const int tier = i >> 2, idx = i & 3;
        const int8_t *src = s + 7 * (Lx::TIERS + 8 * tier + 2 * idx);
        if (slot >= 0) {
#pragma unroll
            for (int c = 0; c < 14; c++) s[7 * slot + c] = src[c];
        }
        fill_new_card<N>(s, tier, idx, det, ch);
    } else if (!det) {
        int8_t c14[14];
        if (deck_card<N>(s, i - 12, ch, c14) && slot >= 0) {
#pragma unroll
            for (int c = 0; c < 14; c++) s[7 * slot + c] = c14[c];
        }
    }
    if (s[5] > 0) {
        s[7 * (Lx::GEMS + p) + 5] += 1;
        s[5] -= 1;
    }
}

// Board.make_move (:267-289); actions 405..408 are a no-op + round increment (the
// reference's select-noble stub does not parse and pass reads give_ids3 out of bounds;
// see DESIGN.md "Defined deviations"). Returns the next player.
template <int N>
__device__ __forceinline__ int make_move(int8_t *s, int a, int p, bool det, Chance &ch) {
    using Lx = Lay<N>;
    int8_t *bank = s, *gems = s + 7 * (Lx::GEMS + p);
    if (a < 12) {
        buy_card<N>(s, Lx::TIERS + 2 * a, p);
        fill_new_card<N>(s, a >> 2, a & 3, det, ch);
    } else if (a < 27) {
        reserve<N>(s, a - 12, p, det, ch);
    } else if (a < 30) {                                   // _buy_reserve (:554-560)
        const int i = a - 27, st = Lx::RSV + 6 * p + 2 * i;
        buy_card<N>(s, st, p);
        for (int r = st; r < Lx::RSV + 6 * p + 4; r++)
#pragma unroll
            for (int c = 0; c < 7; c++) s[7 * r + c] = s[7 * (r + 2) + c];
#pragma unroll
        for (int c = 0; c < 14; c++) s[7 * (Lx::RSV + 6 * p + 4) + c] = 0;
    } else if (a < 60) {                                   // _get_gems (:585-593)
        move_gems(bank, gems, K_TAKE[a - 30], +1);
    } else if (a < 405) {                                  // exchanges (:697-761)
        const uint8_t *e = K_EXCHANGE[a - 60];
        if (e[3] != 255) reserve<N>(s, e[3], p, det, ch);
        if (e[0] != 255) move_gems(bank, gems, K_TAKE[e[0]], +1);
        move_gems(bank, gems, K_GIVE[e[1]], -1);
        if (e[2] != 255) move_gems(bank, gems, K_GIVE[e[2]], -1);
    }
    s[6] = (int8_t)(s[6] + 1);                             // round counter (:287)
    return (p + 1) % N;
}

// ------------------------------------------------------------------ end of game
// check_end_game + judge + get_score (:320-334, :306-318, :217-220)
template <int N>
__device__ __forceinline__ void check_end(const int8_t *s, float out[N]) {
    using Lx = Lay<N>;
#pragma unroll
    for (int i = 0; i < N; i++) out[i] = 0.f;
    const int r = (uint8_t)s[6];
    if (r % N != 0) return;
    int sc[N], mx = -1000;
#pragma unroll
    for (int p = 0; p < N; p++) {
        int v = s[7 * (Lx::CARDS + p) + 6];
        for (int i = 0; i < 3; i++) v += s[7 * (Lx::PNOB + 3 * p + i) + 6];  // hard-coded 3
        sc[p] = (int8_t)v;
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
        m[p] = (int8_t)sum5(s + 7 * (Lx::CARDS + p));
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
__device__ __forceinline__ int get_score(const int8_t *s, int p) {
    using Lx = Lay<N>;
    int v = s[7 * (Lx::CARDS + p) + 6];
    for (int i = 0; i < 3; i++) v += s[7 * (Lx::PNOB + 3 * p + i) + 6];
    return v;
}

// ------------------------------------------------------------------ new game
// Board.init_game (:222-246). Card draws use the chance source; the noble draw is a
// partial Fisher-Yates on the same stream (the reference's np.random.choice is unseeded).
template <int N>
__device__ __forceinline__ void init_fill(int8_t *s, Chance &ch) {   // s already zeroed
    using Lx = Lay<N>;
    const int g = N == 2 ? 4 : (N == 3 ? 5 : 7);
#pragma unroll
    for (int c = 0; c < 5; c++) s[c] = (int8_t)g;
    s[5] = 5;
#pragma unroll
    for (int t = 0; t < 3; t++) {
        const int len = t == 0 ? 8 : (t == 1 ? 6 : 4);
        const int8_t bits = (int8_t)(uint8_t)(0xFFu << (8 - len));
#pragma unroll
        for (int c = 0; c < 5; c++) {
            s[7 * (Lx::DECKS + 2 * t) + c] = (int8_t)len;
            s[7 * (Lx::DECKS + 2 * t + 1) + c] = bits;
        }
    }
    for (int t = 0; t < 3; t++)
        for (int i = 0; i < 4; i++) fill_new_card<N>(s, t, i, false, ch);
    uint64_t perm = 0x9876543210ull;              // 10 nibbles: partial Fisher-Yates
    for (int i = 0; i < Lx::NN; i++) {
        const int j = i + (int)floor(ch.draw() * (double)(10 - i));
        const uint64_t pi = (perm >> (4 * i)) & 15, pj = (perm >> (4 * j)) & 15;
        perm &= ~((15ull << (4 * i)) | (15ull << (4 * j)));
        perm |= (pj << (4 * i)) | (pi << (4 * j));
    }
    for (int i = 0; i < Lx::NN; i++) {
        int8_t *r = s + 7 * (Lx::NOBLES + i);
        const int8_t *nb = K_NOBLES[(perm >> (4 * i)) & 15];
#pragma unroll
        for (int c = 0; c < 7; c++) r[c] = nb[c];
    }
}

// wave-collective new game
template <int N>
__device__ __forceinline__ void init_game(int8_t *s, Chance &ch) {
    const int l = lane_id();
    for (int i = l; i < Lay<N>::S; i += 64) s[i] = 0;
    __builtin_amdgcn_wave_barrier();
    init_fill<N>(s, ch);
    __builtin_amdgcn_wave_barrier();
}

// single-lane new game (lane-per-board code paths)
template <int N>
__device__ __forceinline__ void init_game_lane(int8_t *s, Chance &ch) {
    for (int i = 0; i < Lay<N>::S; i++) s[i] = 0;
    init_fill<N>(s, ch);
}

// store a wave-uniform packed mask (7 words) from lane 0 (no per-lane word selection:
// selecting w[lane] makes hipcc spill the array to scratch)
__device__ __forceinline__ void store_mask(uint64_t *dst, const uint64_t w[7]) {
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < 7; k++) dst[k] = w[k];
    }
}

// k-th set bit of the packed mask (k < popcount); fully unrolled (no runtime indexing)
__device__ __forceinline__ int select_bit(const uint64_t w[7], int k) {
    int res = 408;
    bool done = false;
#pragma unroll
    for (int j = 0; j < 7; j++) {
        const int c = __popcll(w[j]);
        if (!done && k < c) {
            uint64_t x = w[j];
            for (int t = 0; t < k; t++) x &= x - 1;
            res = 64 * j + __ffsll((unsigned long long)x) - 1;
            done = true;
        }
        if (!done) k -= c;
    }
    return res;
}

}  // namespace spl
