/*
 * splendor_oracle.c — scalar CPU restatement of the reference Splendor hot path.
 *
 * TEST INFRASTRUCTURE (parity checker + CPU baseline). See splendor_oracle.h for the
 * usage rule and the list of reference functions restated. Pinned against the golden
 * vectors in tests/golden (recorded from the reference itself by make_golden.py).
 *
 * Build: make -C oracle   (gcc -O2 -ffp-contract=off: strict IEEE order, no FMA, so
 *        the float arithmetic matches the Python-recorded golden vectors bit-exactly)
 */
#include "splendor_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <pthread.h>
#include <string.h>

/* ------------------------------------------------------------------ game tables
 * Card / noble data: SplendorLogic.py:320-473. Cards are [color][k] -> (cost[5], pts);
 * the gain row is one-hot(color) + points (SplendorLogic.py:336-467).               */
static const int8_t NOBLES[10][5] = {
    {0,0,4,4,0},{0,0,0,4,4},{0,4,4,0,0},{4,0,0,0,4},{4,4,0,0,0},
    {3,0,0,3,3},{3,3,3,0,0},{0,0,3,3,3},{0,3,3,3,0},{3,3,0,0,3}};
/* deck colour order in the tables: blue, red, black, white, green (gain colours) */
static const int8_t DECK_GAIN_COLOR[5] = {1, 3, 4, 0, 2};
static const int8_t T1[5][8][6] = {
 {{0,0,0,0,3,0},{1,0,0,0,2,0},{0,0,2,0,2,0},{1,0,2,2,0,0},{0,1,3,1,0,0},{1,0,1,1,1,0},{1,0,1,2,1,0},{0,0,0,4,0,1}},
 {{3,0,0,0,0,0},{0,2,1,0,0,0},{2,0,0,2,0,0},{2,0,1,0,2,0},{1,0,0,1,3,0},{1,1,1,0,1,0},{2,1,1,0,1,0},{4,0,0,0,0,1}},
 {{0,0,3,0,0,0},{0,0,2,1,0,0},{2,0,2,0,0,0},{2,2,0,1,0,0},{0,0,1,3,1,0},{1,1,1,1,0,0},{1,2,1,1,0,0},{0,4,0,0,0,1}},
 {{0,3,0,0,0,0},{0,0,0,2,1,0},{0,2,0,0,2,0},{0,2,2,0,1,0},{3,1,0,0,1,0},{0,1,1,1,1,0},{0,1,2,1,1,0},{0,0,4,0,0,1}},
 {{0,0,0,3,0,0},{2,1,0,0,0,0},{0,2,0,2,0,0},{0,1,0,2,2,0},{1,3,1,0,0,0},{1,1,0,1,1,0},{1,1,0,1,2,0},{0,0,0,0,4,1}}};
static const int8_t T2[5][6][6] = {
 {{0,2,2,3,0,1},{0,2,3,0,3,1},{0,5,0,0,0,2},{5,3,0,0,0,2},{2,0,0,1,4,2},{0,6,0,0,0,3}},
 {{2,0,0,2,3,1},{0,3,0,2,3,1},{0,0,0,0,5,2},{3,0,0,0,5,2},{1,4,2,0,0,2},{0,0,0,6,0,3}},
 {{3,2,2,0,0,1},{3,0,3,0,2,1},{5,0,0,0,0,2},{0,0,5,3,0,2},{0,1,4,2,0,2},{0,0,0,0,6,3}},
 {{0,0,3,2,2,1},{2,3,0,3,0,1},{0,0,0,5,0,2},{0,0,0,5,3,2},{0,0,1,4,2,2},{6,0,0,0,0,3}},
 {{2,3,0,0,2,1},{3,0,2,3,0,1},{0,0,5,0,0,2},{0,5,3,0,0,2},{4,2,0,0,1,2},{0,0,6,0,0,3}}};
static const int8_t T3[5][4][6] = {
 {{3,0,3,3,5,3},{7,0,0,0,0,4},{6,3,0,0,3,4},{7,3,0,0,0,5}},
 {{3,5,3,0,3,3},{0,0,7,0,0,4},{0,3,6,3,0,4},{0,0,7,3,0,5}},
 {{3,3,5,3,0,3},{0,0,0,7,0,4},{0,0,3,6,3,4},{0,0,0,7,3,5}},
 {{0,3,3,5,3,3},{0,0,0,0,7,4},{3,0,0,3,6,4},{3,0,0,0,7,5}},
 {{5,3,0,3,3,3},{0,7,0,0,0,4},{3,6,3,0,0,4},{0,7,3,0,0,5}}};
static const int8_t DECK_LEN[3] = {8, 6, 4};

static const int8_t *card_of(int tier, int color, int k) {
    if (tier == 0) return T1[color][k];
    if (tier == 1) return T2[color][k];
    return T3[color][k];
}

/* gem combinations (SplendorLogic.py:250-280): itertools.combinations order */
static int8_t DIFF3[25][5];     /* np_different_gems_up_to_3 */
static int8_t SPEC3[40][5];     /* np_2specs_gems_up_to_3   */
/* Board.give_ids (SplendorLogicNumba.py:100-166), used slices only */
static const int8_t GIVE0[10][2] = {{3,4},{2,4},{2,3},{1,4},{1,3},{1,2},{0,4},{0,3},{0,2},{0,1}};
static const int8_t GIVE1[10][3] = {{14,18,19},{13,17,19},{12,17,18},{11,16,19},{10,16,18},
                                    {9,16,17},{8,15,19},{7,15,18},{6,15,17},{5,15,16}};
static const int8_t GIVE2[10][6] = {{12,13,14,17,18,19},{10,11,14,16,18,19},{9,11,13,17,16,19},
                                    {9,10,12,17,16,18},{7,8,14,15,19,18},{6,8,13,15,19,17},
                                    {6,7,12,15,18,17},{5,8,11,15,19,16},{5,7,10,15,18,16},
                                    {6,5,9,15,16,17}};
static const int8_t GIVE3[5][10] = {{9,12,13,10,11,14,17,16,18,19},{6,7,8,12,13,14,15,17,18,19},
                                    {5,7,8,10,11,14,15,16,18,19},{6,5,8,9,13,11,15,17,16,19},
                                    {6,5,7,9,12,10,15,17,16,18}};
static const int8_t GIVE4[10][3] = {{2,3,4},{1,3,4},{1,2,4},{1,2,3},{0,3,4},{0,2,4},{0,2,3},
                                    {0,1,4},{0,1,3},{0,1,2}};
static const int8_t GIVE5[5][4] = {{1,2,3,4},{0,2,3,4},{0,1,3,4},{0,1,2,4},{0,1,2,3}};
static const int8_t GIVE_T1[20] = {1,2,3,4, 0,2,3,4, 0,1,3,4, 0,1,2,4, 0,1,2,3};
/* give_ids3 (SplendorLogicNumba.py:169-210): (take3 id, give id, give id) */
static const int8_t GIVE_IDS3[40][3] = {
 {0,3,18},{0,18,4},{0,3,19},{0,19,4},{1,2,17},{1,17,4},{1,2,19},{1,19,4},{2,2,17},{2,17,3},
 {2,2,18},{2,18,3},{3,1,16},{3,16,4},{3,1,19},{3,19,4},{4,1,16},{4,16,3},{4,1,18},{4,18,3},
 {5,1,16},{5,16,2},{5,1,17},{5,17,2},{6,0,15},{6,15,4},{6,0,19},{6,19,4},{7,0,15},{7,15,3},
 {7,0,18},{7,18,3},{8,0,15},{8,15,2},{8,0,17},{8,17,2},{9,0,15},{9,15,1},{9,0,16},{9,16,1}};

/* give option g in [0,20): 0..14 = DIFF3[0..14] (up-to-2 different), 15..19 = 2 of one */
static void give_vec(int g, int8_t v[5]) {
    memset(v, 0, 5);
    if (g < 15) memcpy(v, DIFF3[g], 5); else v[g - 15] = 2;
}
static void take_vec(int t, int8_t v[5]) {  /* t in [0,30): 25 different + 5 identical */
    memset(v, 0, 5);
    if (t < 25) memcpy(v, DIFF3[t], 5); else v[t - 25] = 2;
}

static int tables_ready = 0;
static void build_tables(void) {
    if (tables_ready) return;
    int k = 0;
    for (int c = 0; c < 5; c++) { memset(DIFF3[k], 0, 5); DIFF3[k][c] = 1; k++; }
    for (int a = 0; a < 5; a++) for (int b = a + 1; b < 5; b++) {
        memset(DIFF3[k], 0, 5); DIFF3[k][a] = DIFF3[k][b] = 1; k++; }
    for (int a = 0; a < 5; a++) for (int b = a + 1; b < 5; b++) for (int c = b + 1; c < 5; c++) {
        memset(DIFF3[k], 0, 5); DIFF3[k][a] = DIFF3[k][b] = DIFF3[k][c] = 1; k++; }
    for (int i = 0; i < 40; i++) {
        int8_t g1[5], g2[5];
        give_vec(GIVE_IDS3[i][1], g1); give_vec(GIVE_IDS3[i][2], g2);
        for (int c = 0; c < 5; c++) SPEC3[i][c] = (int8_t)(g1[c] + g2[c]);
    }
    tables_ready = 1;
}

/* ------------------------------------------------------------------ layout */
typedef struct { int n, nn, bank, tiers, decks, nobles, gems, pnobles, cards, rsv, rows; } lay_t;
static lay_t lay(int n) {
    lay_t L; L.n = n; L.nn = n + 1;
    L.bank = 0; L.tiers = 1; L.decks = 25; L.nobles = 31; L.gems = 32 + n;
    L.pnobles = 32 + 2 * n; L.cards = 32 + 3 * n + n * n; L.rsv = 32 + 4 * n + n * n;
    L.rows = 32 + 10 * n + n * n;
    return L;
}
#define RW(s, r) ((s) + 7 * (r))

int or_rows(int n) { return 32 + 10 * n + n * n; }
int or_get_round(const int8_t *s) { return (uint8_t)s[6]; }

int or_get_score(int n, const int8_t *s, int p) {
    lay_t L = lay(n);
    int sc = RW(s, L.cards + p)[6];
    for (int i = 0; i < 3; i++) sc += RW(s, L.pnobles + 3 * p + i)[6];  /* hard-coded 3 :219 */
    return sc;
}

static int sum7(const int8_t *r) { int t = 0; for (int c = 0; c < 7; c++) t += r[c]; return t; }
static int sum5(const int8_t *r) { int t = 0; for (int c = 0; c < 5; c++) t += r[c]; return t; }

/* ------------------------------------------------------------------ chance */
/* my_random_choice: searchsorted(cumsum(prob), U, side='right') (:39-41) */
static int rand_choice(const double *prob, int len, double u) {
    double c = 0.0;
    for (int i = 0; i < len; i++) { c += prob[i]; if (c > u) return i; }
    return len;
}

typedef struct { const double *u; int used; } chance_t;
static double draw(chance_t *ch) { return ch->u[ch->used++]; }

/* _get_deck_card (:400-420). Returns 0 if the deck is empty. */
static int deck_card(lay_t L, int8_t *s, int tier, chance_t *ch, int8_t out[14]) {
    int8_t *cnt = RW(s, L.decks + 2 * tier), *bits = RW(s, L.decks + 2 * tier + 1);
    int tot = sum5(cnt);
    if (tot == 0) return 0;
    double p[8];
    for (int c = 0; c < 5; c++) p[c] = (double)cnt[c] / (double)tot;
    int color = rand_choice(p, 5, draw(ch));
    if (color > 4) color = 4;                     /* unreachable (prob ~1e-16) */
    uint8_t b = (uint8_t)bits[color];
    int nb = 0; int on[8];
    for (int k = 0; k < 8; k++) { on[k] = (b >> (7 - k)) & 1; nb += on[k]; }
    for (int k = 0; k < 8; k++) p[k] = (double)on[k] / (double)nb;
    int idx = rand_choice(p, 8, draw(ch));
    if (idx > 7) idx = 7;
    b &= (uint8_t)~(1u << (7 - idx));
    bits[color] = (int8_t)b;                      /* packbits + int8 wrap (:44-46) */
    cnt[color] -= 1;
    const int8_t *cd = card_of(tier, color, idx);
    memset(out, 0, 14);
    memcpy(out, cd, 5);
    out[7 + DECK_GAIN_COLOR[color]] = 1;
    out[7 + 6] = cd[5];
    return 1;
}

void or_card(int tier, int color, int k, int8_t *out) {
    const int8_t *cd = card_of(tier, color, k);
    memset(out, 0, 14); memcpy(out, cd, 5);
    out[7 + DECK_GAIN_COLOR[color]] = 1; out[13] = cd[5];
}

static void fill_new_card(lay_t L, int8_t *s, int tier, int idx, int det, chance_t *ch) {
    int8_t *slot = RW(s, L.tiers + 8 * tier + 2 * idx);
    memset(slot, 0, 14);
    if (!det) { int8_t c[14]; if (deck_card(L, s, tier, ch, c)) memcpy(slot, c, 14); }
}

void or_init(int n, int8_t *s, const double *u, int *used) {
    build_tables();
    lay_t L = lay(n);
    chance_t ch = {u, 0};
    memset(s, 0, (size_t)7 * L.rows);
    int g = n == 2 ? 4 : (n == 3 ? 5 : 7);
    for (int c = 0; c < 5; c++) s[c] = (int8_t)g;
    s[5] = 5;
    for (int t = 0; t < 3; t++) {
        uint8_t bits = (uint8_t)(0xFFu << (8 - DECK_LEN[t]));
        for (int c = 0; c < 5; c++) {
            RW(s, L.decks + 2 * t)[c] = DECK_LEN[t];
            RW(s, L.decks + 2 * t + 1)[c] = (int8_t)bits;   /* 255/252/240 -> -1/-4/-16 */
        }
    }
    for (int t = 0; t < 3; t++)
        for (int i = 0; i < 4; i++) fill_new_card(L, s, t, i, 0, &ch);
    int perm[10]; for (int i = 0; i < 10; i++) perm[i] = i;
    for (int i = 0; i < L.nn; i++) {       /* injected noble draw (make_golden.py) */
        int j = i + (int)floor(draw(&ch) * (10 - i));
        int t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }
    for (int i = 0; i < L.nn; i++) {
        int8_t *r = RW(s, L.nobles + i);
        memcpy(r, NOBLES[perm[i]], 5); r[5] = 0; r[6] = 3;
    }
    if (used) *used = ch.used;
}

/* ------------------------------------------------------------------ valid moves */
void or_valid_moves(int n, const int8_t *s, int p, uint8_t *res) {
    build_tables();
    lay_t L = lay(n);
    const int8_t *bank = RW(s, 0), *gems = RW(s, L.gems + p), *cards = RW(s, L.cards + p);
    int T = sum7(gems), gold = gems[5];
    memset(res, 0, OR_ACTIONS);
    /* _valid_buy :476-501 */
    for (int i = 0; i < 12; i++) {
        const int8_t *cost = RW(s, L.tiers + 2 * i);
        int miss = 0;
        for (int c = 0; c < 5; c++) { int d = cost[c] - gems[c] - cards[c]; if (d > 0) miss += d; }
        res[i] = (miss <= gold) && sum5(cost) != 0;
    }
    /* _valid_reserve :508-515 (no-limit flags kept for the exchange block) */
    uint8_t rsv[15];
    int slot_free = sum5(RW(s, L.rsv + 6 * p + 5)) == 0;
    for (int i = 0; i < 15; i++) {
        const int8_t *r = i < 12 ? RW(s, L.tiers + 2 * i) : RW(s, L.decks + 2 * (i - 12));
        rsv[i] = (sum5(r) != 0) && slot_free;
    }
    int limited = (T == 10 && bank[5] > 0);
    for (int i = 0; i < 15; i++) res[12 + i] = limited ? 0 : rsv[i];
    /* _valid_buy_reserve :538-552 */
    for (int i = 0; i < 3; i++) {
        const int8_t *cost = RW(s, L.rsv + 6 * p + 2 * i);
        int miss = 0;
        for (int c = 0; c < 5; c++) { int d = cost[c] - gems[c] - cards[c]; if (d > 0) miss += d; }
        res[27 + i] = (miss <= gold) && sum5(cost) != 0;
    }
    /* _valid_get_gems / _identical :562-583 */
    uint8_t get[30];
    int nspec = 0;
    for (int c = 0; c < 5; c++) nspec += bank[c] != 0;
    for (int i = 0; i < 25; i++) {
        int ok = 1, k = 0;
        for (int c = 0; c < 5; c++) { ok &= (bank[c] - DIFF3[i][c]) >= 0; k += DIFF3[i][c]; }
        get[i] = (uint8_t)ok;
        int lim = ok && (T + k <= 10);
        if (i < 5 && T != 9 && nspec != 1) lim = 0;
        if (i >= 5 && i < 15 && T != 8 && nspec != 2) lim = 0;
        res[30 + i] = (uint8_t)lim;
    }
    for (int c = 0; c < 5; c++) {
        get[25 + c] = bank[c] >= 4;
        res[55 + c] = get[25 + c] && (T + 2 <= 10);
    }
    /* give flags :595-613 */
    uint8_t giv[20], giv3[40];
    for (int g = 0; g < 20; g++) {
        int8_t v[5]; give_vec(g, v); int ok = 1;
        for (int c = 0; c < 5; c++) ok &= (gems[c] - v[c]) >= 0;
        giv[g] = (uint8_t)ok;
    }
    for (int k = 0; k < 40; k++) {
        int ok = 1;
        for (int c = 0; c < 5; c++) ok &= (gems[c] - SPEC3[k][c]) >= 0;
        giv3[k] = (uint8_t)ok;
    }
    /* _valid_exchange :615-680 */
    uint8_t *ex = res + 60;
    const uint8_t *dif2 = get + 5, *dif3 = get + 15, *same2 = get + 25;
    if (T == 8) {
        for (int k = 0; k < 20; k++) ex[k] = dif3[k / 2] && giv[GIVE0[k / 2][k % 2]];
    } else if (T == 9) {
        for (int k = 0; k < 30; k++) ex[20 + k] = dif3[k / 3] && giv[GIVE1[k / 3][k % 3]];
        for (int k = 0; k < 30; k++) ex[160 + k] = dif2[k / 3] && giv[GIVE4[k / 3][k % 3]];
        for (int k = 0; k < 20; k++) ex[190 + k] = same2[k / 4] && giv[GIVE5[k / 4][k % 4]];
    } else if (T >= 10) {
        for (int k = 0; k < 60; k++) ex[50 + k] = dif2[k / 6] && giv[GIVE2[k / 6][k % 6]];
        for (int k = 0; k < 50; k++) ex[110 + k] = same2[k / 10] && giv[GIVE3[k / 10][k % 10]];
        for (int k = 0; k < 20; k++) ex[210 + k] = get[k / 4] && giv[GIVE_T1[k]];
        for (int k = 0; k < 40; k++) ex[305 + k] = dif3[k / 4] && giv3[k];
        if (bank[5] > 0)
            for (int k = 0; k < 75; k++) ex[230 + k] = rsv[k / 5] && giv[k % 5];
    }
    /* select-noble 405..407 never valid (WIP stub :682); pass iff nothing else */
    int any = 0;
    for (int a = 0; a < 408; a++) any |= res[a];
    res[408] = !any;
}

/* ------------------------------------------------------------------ make move */
static void give_nobles(lay_t L, int8_t *s, int p) {      /* :763-768 */
    for (int i = 0; i < L.nn; i++) {
        int8_t *nob = RW(s, L.nobles + i);
        const int8_t *cards = RW(s, L.cards + p);
        if (sum5(nob) > 0) {
            int ok = 1;
            for (int c = 0; c < 5; c++) ok &= cards[c] >= nob[c];
            if (ok) { memcpy(RW(s, L.pnobles + L.nn * p + i), nob, 7); memset(nob, 0, 7); }
        }
    }
}

static void buy_card(lay_t L, int8_t *s, const int8_t *cost, const int8_t *gain, int p) {
    int8_t *bank = RW(s, 0), *gems = RW(s, L.gems + p), *cards = RW(s, L.cards + p);
    int miss = 0;
    for (int c = 0; c < 5; c++) { int d = cost[c] - gems[c] - cards[c]; if (d > 0) miss += d; }
    for (int c = 0; c < 5; c++) {
        int need = cost[c] - cards[c]; if (need < 0) need = 0;
        int paid = need < gems[c] ? need : gems[c];
        gems[c] = (int8_t)(gems[c] - paid);
        bank[c] = (int8_t)(bank[c] + paid);
    }
    gems[5] = (int8_t)(gems[5] - miss);
    bank[5] = (int8_t)(bank[5] + miss);
    int8_t g[7]; memcpy(g, gain, 7);           /* gain may alias a row we write below */
    for (int c = 0; c < 7; c++) cards[c] = (int8_t)(cards[c] + g[c]);
    give_nobles(L, s, p);
}

static void move_gems(lay_t L, int8_t *s, const int8_t v[5], int p, int sign) {
    int8_t *bank = RW(s, 0), *gems = RW(s, L.gems + p);
    for (int c = 0; c < 5; c++) {
        bank[c] = (int8_t)(bank[c] - sign * v[c]);
        gems[c] = (int8_t)(gems[c] + sign * v[c]);
    }
}
static void get_gems(lay_t L, int8_t *s, int t, int p) { int8_t v[5]; take_vec(t, v); move_gems(L, s, v, p, +1); }
static void give_gems(lay_t L, int8_t *s, int g, int p) { int8_t v[5]; give_vec(g, v); move_gems(L, s, v, p, -1); }

static void reserve(lay_t L, int8_t *s, int i, int p, int det, chance_t *ch) {   /* :517-536 */
    int slot = -1;
    for (int k = 0; k < 3; k++)
        if (sum5(RW(s, L.rsv + 6 * p + 2 * k)) == 0) { slot = L.rsv + 6 * p + 2 * k; break; }
    if (i < 12) {
        int tier = i / 4, idx = i % 4;
        if (slot >= 0) memcpy(RW(s, slot), RW(s, L.tiers + 8 * tier + 2 * idx), 14);
        fill_new_card(L, s, tier, idx, det, ch);
    } else if (!det) {
        int8_t c[14];
        if (deck_card(L, s, i - 12, ch, c) && slot >= 0) memcpy(RW(s, slot), c, 14);
    }
    if (s[5] > 0) { RW(s, L.gems + p)[5] += 1; s[5] -= 1; }
}

static void give_and_get(lay_t L, int8_t *s, int i, int p) {     /* :697-756 */
    if (i < 20)       { get_gems(L, s, i / 2 + 15, p); give_gems(L, s, GIVE0[i / 2][i % 2], p); }
    else if (i < 50)  { i -= 20;  get_gems(L, s, i / 3 + 15, p); give_gems(L, s, GIVE1[i / 3][i % 3], p); }
    else if (i < 110) { i -= 50;  get_gems(L, s, i / 6 + 5, p);  give_gems(L, s, GIVE2[i / 6][i % 6], p); }
    else if (i < 160) { i -= 110; get_gems(L, s, i / 10 + 25, p); give_gems(L, s, GIVE3[i / 10][i % 10], p); }
    else if (i < 190) { i -= 160; get_gems(L, s, i / 3 + 5, p);  give_gems(L, s, GIVE4[i / 3][i % 3], p); }
    else if (i < 210) { i -= 190; get_gems(L, s, i / 4 + 25, p); give_gems(L, s, GIVE5[i / 4][i % 4], p); }
    else if (i < 230) { i -= 210; get_gems(L, s, i / 4, p);      give_gems(L, s, GIVE_T1[i], p); }
    else {
        i -= 305;
        get_gems(L, s, GIVE_IDS3[i][0] + 15, p);
        give_gems(L, s, GIVE_IDS3[i][1], p);
        give_gems(L, s, GIVE_IDS3[i][2], p);
    }
}

int or_make_move(int n, int8_t *s, int a, int p, int det, const double *u, int *used) {
    build_tables();
    lay_t L = lay(n);
    chance_t ch = {u, 0};
    if (a < 12) {
        buy_card(L, s, RW(s, L.tiers + 2 * a), RW(s, L.tiers + 2 * a + 1), p);
        fill_new_card(L, s, a / 4, a % 4, det, &ch);
    } else if (a < 27) {
        reserve(L, s, a - 12, p, det, &ch);
    } else if (a < 30) {
        int i = a - 27, st = L.rsv + 6 * p + 2 * i;
        buy_card(L, s, RW(s, st), RW(s, st + 1), p);
        if (i < 2) memmove(RW(s, st), RW(s, st + 2), (size_t)7 * (6 * p + 4 + L.rsv - st));
        memset(RW(s, L.rsv + 6 * p + 4), 0, 14);
    } else if (a < 60) {
        get_gems(L, s, a - 30, p);
    } else if (a < 290) {
        give_and_get(L, s, a - 60, p);
    } else if (a < 365) {
        int i = a - 290;
        reserve(L, s, i / 5, p, det, &ch);
        give_gems(L, s, i % 5, p);
    } else if (a < 405) {
        give_and_get(L, s, a - 60, p);
    } /* 405..408: no-op (undefined at HEAD, see make_golden.py P5) */
    s[6] = (int8_t)(s[6] + 1);
    if (used) *used = ch.used;
    return (p + 1) % n;
}

/* ------------------------------------------------------------------ end / swap */
void or_check_end(int n, const int8_t *s, float *out) {
    lay_t L = lay(n);
    for (int i = 0; i < n; i++) out[i] = 0.f;
    int r = (uint8_t)s[6];
    if (r % n != 0) return;
    int sc[4], mx = -1000;
    for (int p = 0; p < n; p++) { sc[p] = (int8_t)or_get_score(n, s, p); if (sc[p] > mx) mx = sc[p]; }
    if (!(mx >= 15 || r >= 62 * n)) return;
    int nmax = 0;
    for (int p = 0; p < n; p++) nmax += sc[p] == mx;
    if (nmax == 1) { for (int p = 0; p < n; p++) out[p] = sc[p] == mx ? 1.f : -1.f; return; }
    int8_t masked[4], mn = 127;
    for (int p = 0; p < n; p++) {
        masked[p] = (int8_t)sum5(RW(s, L.cards + p));
        if (sc[p] < mx) masked[p] = (int8_t)-25;  /* int8(999) (:313) */
        if (masked[p] < mn) mn = masked[p];
    }
    int cnt = 0;
    for (int p = 0; p < n; p++) cnt += masked[p] == mn;
    for (int p = 0; p < n; p++) out[p] = masked[p] == mn ? (cnt > 1 ? 0.01f : 1.f) : -1.f;
}

static void roll_rows(int8_t *blk, int rows, int shift) {
    int8_t tmp[7 * 40];
    memcpy(tmp, blk, (size_t)7 * rows);
    for (int i = 0; i < rows; i++) memcpy(blk + 7 * i, tmp + 7 * ((i + shift) % rows), 7);
}

void or_swap_players(int n, int8_t *s, int k) {
    lay_t L = lay(n);
    roll_rows(RW(s, L.gems), n, k);
    roll_rows(RW(s, L.pnobles), n * (n + 1), 3 * k);  /* hard-coded 3 (:345) */
    roll_rows(RW(s, L.cards), n, k);
    roll_rows(RW(s, L.rsv), 6 * n, 6 * k);
}

int or_tree_step(int n, const int8_t *parent, int a, int8_t *child) {
    memcpy(child, parent, (size_t)7 * or_rows(n));
    int nxt = or_make_move(n, child, a, 0, 1, NULL, NULL);
    if (nxt != 0) or_swap_players(n, child, nxt);
    return nxt;
}

/* ------------------------------------------------------------------ symmetries */
static const int8_t CARD_SYM[3][4] = {{1,3,0,2},{2,0,3,1},{3,2,1,0}};   /* SplendorLogic.py:283 */
static const int8_t RSV_SYM[4][2][3] = {{{-1,-1,-1},{-1,-1,-1}},{{-1,-1,-1},{-1,-1,-1}},
                                        {{1,0,2},{-1,-1,-1}},{{1,2,0},{2,0,1}}};

int or_symmetries(int n, const int8_t *s, const float *pi, const uint8_t *va,
                  int8_t *os, float *op, uint8_t *ov) {
    lay_t L = lay(n);
    int S = 7 * L.rows, cnt = 0;
#define EMIT_BASE() do { memcpy(os + (size_t)cnt * S, s, S); memcpy(op + cnt * 409, pi, 409 * 4); \
                         memcpy(ov + cnt * 409, va, 409); } while (0)
    EMIT_BASE(); cnt++;
    for (int t = 0; t < 3; t++) for (int q = 0; q < 3; q++) {
        EMIT_BASE();
        int8_t *st = os + (size_t)cnt * S;
        for (int i = 0; i < 4; i++) {
            int src = CARD_SYM[q][i];
            memcpy(RW(st, L.tiers + 8 * t + 2 * i), RW(s, L.tiers + 8 * t + 2 * src), 14);
            op[cnt * 409 + 4 * t + i] = pi[4 * t + src];
            op[cnt * 409 + 12 + 4 * t + i] = pi[12 + 4 * t + src];
            ov[cnt * 409 + 4 * t + i] = va[4 * t + src];
            ov[cnt * 409 + 12 + 4 * t + i] = va[12 + 4 * t + src];
        }
        cnt++;
    }
    for (int p = 0; p < n; p++) {
        int nb = 3;
        for (int c = 0; c < 3; c++) if (sum5(RW(s, L.rsv + 6 * p + 2 * c)) == 0) { nb = c; break; }
        for (int q = 0; q < 2; q++) {
            const int8_t *perm = RSV_SYM[nb][q];
            if (perm[0] < 0) continue;
            EMIT_BASE();
            int8_t *st = os + (size_t)cnt * S;
            for (int i = 0; i < 3; i++)
                memcpy(RW(st, L.rsv + 6 * p + 2 * i), RW(s, L.rsv + 6 * p + 2 * perm[i]), 14);
            if (p == 0)
                for (int i = 0; i < 3; i++) {
                    op[cnt * 409 + 27 + i] = pi[27 + perm[i]];
                    ov[cnt * 409 + 27 + i] = va[27 + perm[i]];
                }
            cnt++;
        }
    }
#undef EMIT_BASE
    return cnt;
}

/* ------------------------------------------------------------------ Philox */
void or_philox4x32(uint32_t k0, uint32_t k1, const uint32_t in[4], uint32_t out[4]) {
    uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* uniform d of a (seed, board, stream) sequence: half of counter block d/2 (words 0,1 for
 * even d, 2,3 for odd d), 53 bits */
double or_uniform(uint64_t seed, uint32_t board, uint32_t stream, uint32_t d) {
    uint32_t ctr[4] = {d >> 1, board, stream, 0x53504C44u /* 'SPLD' */}, o[4];
    or_philox4x32((uint32_t)seed, (uint32_t)(seed >> 32), ctr, o);
    const uint32_t *w = o + 2 * (d & 1);
    return ((double)(w[0] >> 5) * 67108864.0 + (double)(w[1] >> 6)) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------------ fake NN */
uint64_t or_state_hash(const int8_t *st, int bytes) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (int i = 0; i < bytes; i++) { h ^= (uint8_t)st[i]; h *= 0x100000001B3ull; }
    return h;
}
static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
/* Hash network of the search-parity tests (device: k_hash_eval). Mode 0: priors spread over
 * (0, 1], values in [-1, 1) — shallow trees (leaf depth ~3). Mode 1 ("peaked"): each legal
 * action's hash weight w in [1, 2^24] divided by the largest legal one and raised to the
 * 256th power, so priors are (w / max w)^256 — one or a few actions dominate and many are
 * exactly 0 in float32 — and values are +-(1 - h 2^-30), i.e. within 2^-6 of +-1 (player 0
 * positive). The search then commits to lines and leaves reach the depths of the bench's
 * steady state (mean > 15, max > 64). */
static int g_fake_mode = 0;
void or_set_fake_mode(int mode) { g_fake_mode = mode; }
void or_fake_predict(int n, const int8_t *st, const uint8_t *va, float *pi, float *v) {
    uint64_t h = or_state_hash(st, 7 * or_rows(n));
    if (g_fake_mode == 1) {
        double wmax = 0.0;                                  /* like a softmax: the top legal */
        for (int a = 0; a < 409; a++)                       /* action's weight is 1          */
            if (va[a]) wmax = fmax(wmax, (double)(1 + (splitmix64(h + (uint64_t)a) >> 40)));
        for (int a = 0; a < 409; a++) {
            double w = (double)(1 + (splitmix64(h + (uint64_t)a) >> 40)) / wmax;
            for (int k = 0; k < 8; k++) w = w * w;          /* w^256: peaked, many exact zeros */
            pi[a] = va[a] ? (float)w : 0.f;
        }
        for (int i = 0; i < n; i++)
            v[i] = (float)((i == 0 ? 1.0 : -1.0) * (1.0 - (double)(splitmix64(h ^ (0xA5A5ull + (uint64_t)i)) >> 40) * 0x1p-30));
        return;
    }
    for (int a = 0; a < 409; a++)
        pi[a] = va[a] ? (float)((double)(1 + (splitmix64(h + (uint64_t)a) >> 40)) * 0x1p-24) : 0.f;
    for (int i = 0; i < n; i++)
        v[i] = (float)((double)(splitmix64(h ^ (0xA5A5ull + (uint64_t)i)) >> 40) * 0x1p-23 - 1.0);
}

/* leaf depths of the searches since the last reset (edges from the root to the leaf each
 * simulation evaluated or found terminal): sum, maximum, simulations */
static long long g_depth_sum = 0, g_depth_max = 0, g_depth_cnt = 0;
void or_depth_stats(long long *out3, int reset) {
    if (out3) { out3[0] = g_depth_sum; out3[1] = g_depth_max; out3[2] = g_depth_cnt; }
    if (reset) g_depth_sum = g_depth_max = g_depth_cnt = 0;
}
static void note_depth(int d) {
    g_depth_sum += d; g_depth_cnt += 1;
    if (d > g_depth_max) g_depth_max = d;
}

static float pw_sum(const float *a, int len) {   /* numpy pairwise_sum, float32 */
    if (len < 8) { float r = 0.f; for (int i = 0; i < len; i++) r += a[i]; return r; }
    if (len <= 128) {
        float r[8]; int i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < len - (len % 8); i += 8) for (int j = 0; j < 8; j++) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < len; i++) res += a[i];
        return res;
    }
    int n2 = len / 2; n2 -= n2 % 8;
    return pw_sum(a, n2) + pw_sum(a + n2, len - n2);
}
float or_np_sum_f32(const float *x, int len) { return pw_sum(x, len); }

static double pw_sum_f64(const double *a, int len) {   /* numpy pairwise_sum, float64 */
    if (len < 8) { double r = 0.0; for (int i = 0; i < len; i++) r += a[i]; return r; }
    if (len <= 128) {
        double r[8]; int i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < len - (len % 8); i += 8) for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < len; i++) res += a[i];
        return res;
    }
    int n2 = len / 2; n2 -= n2 % 8;
    return pw_sum_f64(a, n2) + pw_sum_f64(a + n2, len - n2);
}

/* ------------------------------------------------------------------ Dirichlet noise
 * The reference draws Dirichlet noise from an unseeded numpy Generator (MCTS.py:40,181),
 * so the sampler itself is this build's own definition, shared bit-for-bit with the
 * device (csrc/mcts_device.h det_*) and with tests/golden/detrand.py: logarithm and
 * exponential from +,-,*,/ only (no libm, so host and device agree), Marsaglia-Tsang Gamma
 * with polar normals on the Philox stream (seed, board, stream), counters i*4096 for the
 * i-th legal action, normalised as numpy's Generator.dirichlet does (sequential sum,
 * multiply by its reciprocal). What the reference does with the vector — softmax(Ps, T0)
 * (MCTS.py:245-250, float64 as Numba types Ps ** (1./T)), the 0.75/0.25 mix over the
 * valid actions (:180-186, float64 then stored float32) and normalise (:239-242) — is
 * pinned against the reference by tests/golden/noise_*.npz. */
#define DET_LN2_HI 6.93147180369123816490e-01
#define DET_LN2_LO 1.90821492927058770002e-10
#define DET_INV_LN2 1.44269504088896338700e+00
#define DET_SQRT2 1.4142135623730951

static double det_log(double x) {          /* x > 0, normal */
    uint64_t b; memcpy(&b, &x, 8);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    uint64_t mb = (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m; memcpy(&m, &mb, 8);
    if (m > DET_SQRT2) { m = m * 0.5; e = e + 1; }
    double f = (m - 1.0) / (m + 1.0), s = f * f;
    double p = 1.0 / 23.0;
    p = p * s + 1.0 / 21.0; p = p * s + 1.0 / 19.0; p = p * s + 1.0 / 17.0;
    p = p * s + 1.0 / 15.0; p = p * s + 1.0 / 13.0; p = p * s + 1.0 / 11.0;
    p = p * s + 1.0 / 9.0; p = p * s + 1.0 / 7.0; p = p * s + 1.0 / 5.0; p = p * s + 1.0 / 3.0;
    double t = 2.0 * f, r = t + t * (s * p);
    return (double)e * DET_LN2_HI + (r + (double)e * DET_LN2_LO);
}
static double det_exp(double x) {
    if (x < -700.0) return 0.0;
    double kf = floor(x * DET_INV_LN2 + 0.5);
    double r = (x - kf * DET_LN2_HI) - kf * DET_LN2_LO;
    double p = 1.0 / 6227020800.0;
    p = p * r + 1.0 / 479001600.0; p = p * r + 1.0 / 39916800.0; p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0; p = p * r + 1.0 / 40320.0; p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0; p = p * r + 1.0 / 120.0; p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0; p = p * r + 0.5; p = p * r + 1.0; p = p * r + 1.0;
    return ldexp(p, (int)kf);
}
static double det_pow(double x, double y) { return x == 0.0 ? 0.0 : det_exp(y * det_log(x)); }

static double det_gamma(double alpha, uint64_t seed, uint32_t board, uint32_t stream, uint32_t ctr) {
    const double a = alpha < 1.0 ? alpha + 1.0 : alpha;
    const double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
    double g = 0.0;
    for (int it = 0; it < 64; it++) {
        double z = 0.0;
        for (int j = 0; j < 16; j++) {
            double u1 = 2.0 * or_uniform(seed, board, stream, ctr++) - 1.0;
            double u2 = 2.0 * or_uniform(seed, board, stream, ctr++) - 1.0;
            double s = u1 * u1 + u2 * u2;
            if (s < 1.0 && s > 0.0) { z = u1 * sqrt(-2.0 * det_log(s) / s); break; }
        }
        double v = 1.0 + c * z;
        if (v <= 0.0) continue;
        v = v * v * v;
        double u = or_uniform(seed, board, stream, ctr++);
        if (u < 1e-300) u = 1e-300;
        if (det_log(u) < 0.5 * z * z + d - d * v + d * det_log(v)) { g = d * v; break; }
    }
    if (alpha < 1.0) {
        double u = or_uniform(seed, board, stream, ctr++);
        if (u < 1e-300) u = 1e-300;
        g = g * det_exp(det_log(u) / alpha);
    }
    return g;
}

void or_dirichlet(double alpha, uint64_t seed, uint32_t board, uint32_t stream, int count, double *out) {
    double acc = 0.0;
    for (int i = 0; i < count; i++) {
        out[i] = det_gamma(alpha, seed, board, stream, (uint32_t)i * 4096u);
        acc = acc + out[i];
    }
    if (acc > 0.0) { double inv = 1.0 / acc; for (int i = 0; i < count; i++) out[i] = out[i] * inv; }
    else for (int i = 0; i < count; i++) out[i] = 1.0 / (double)count;
}

/* softmax(Ps, T0) -> applyDirNoise(Ps, Vs) -> normalise(Ps) (MCTS.py:141-144 / :150-154)
 * on ps[409] in place, dir[] = one value per valid action in action order. */
void or_root_noise(float *ps, const uint8_t *vs, const double *dir, double temp0) {
    if (temp0 != 1.0) {                                 /* softmax (:245-250) */
        double sp[409];
        for (int a = 0; a < 409; a++) sp[a] = det_pow((double)ps[a], 1.0 / temp0);
        double s = pw_sum_f64(sp, 409);
        for (int a = 0; a < 409; a++) ps[a] = (float)(sp[a] / s);
    }
    int k = 0;                                          /* applyDirNoise (:180-186) */
    for (int a = 0; a < 409; a++)
        if (vs[a]) { ps[a] = (float)(0.75 * (double)ps[a] + 0.25 * dir[k]); k++; }
    float sum = pw_sum(ps, 409);                        /* normalise (:239-242) */
    for (int a = 0; a < 409; a++) ps[a] = ps[a] / sum;
}

/* ------------------------------------------------------------------ MCTS */
#define NAN_Q (-42.0)
typedef struct {
    int8_t *key;              /* state bytes */
    int terminal, has_ps;
    float es[4];
    uint8_t vs[409];
    float ps[409];
    long long ns;
    double qsa[409];
    long long nsa[409];
    double qs;
} node_t;

struct or_mcts {
    int n, S, sims, forced;
    double cpuct, fpu;
    node_t **slots; int cap, count;
    int step;
    /* root Dirichlet noise (MCTS.py:58, :141-154): applied at step 0 when alpha > 0 */
    double dir_alpha, dir_temp;
    uint64_t dir_seed; uint32_t dir_board, dir_stream;
    int neg_v;                /* second hash network (values negated), arena fixtures */
};

or_mcts *or_mcts_new(int n, int sims, double cpuct, double fpu, int forced) {
    build_tables();
    or_mcts *m = (or_mcts *)calloc(1, sizeof(or_mcts));
    m->n = n; m->S = 7 * or_rows(n); m->sims = sims; m->cpuct = cpuct; m->fpu = fpu;
    m->forced = forced; m->cap = 1 << 12;
    m->slots = (node_t **)calloc((size_t)m->cap, sizeof(node_t *));
    return m;
}
void or_mcts_set_noise(or_mcts *m, double alpha, double temp0, uint64_t seed, uint32_t board,
                       uint32_t stream) {
    m->dir_alpha = alpha; m->dir_temp = temp0; m->dir_seed = seed; m->dir_board = board;
    m->dir_stream = stream;
}
void or_mcts_set_net(or_mcts *m, int neg_v) { m->neg_v = neg_v; }
static void mcts_noise(or_mcts *m, node_t *nd) {
    double dir[409];
    int cnt = 0;
    for (int a = 0; a < 409; a++) cnt += nd->vs[a] != 0;
    or_dirichlet(m->dir_alpha, m->dir_seed, m->dir_board, m->dir_stream, cnt, dir);
    or_root_noise(nd->ps, nd->vs, dir, m->dir_temp);
}
void or_mcts_free(or_mcts *m) {
    for (int i = 0; i < m->cap; i++) if (m->slots[i]) { free(m->slots[i]->key); free(m->slots[i]); }
    free(m->slots); free(m);
}
static node_t **lookup(or_mcts *m, const int8_t *st) {
    uint64_t h = or_state_hash(st, m->S);
    int i = (int)(h & (uint64_t)(m->cap - 1));
    while (m->slots[i] && memcmp(m->slots[i]->key, st, (size_t)m->S) != 0) i = (i + 1) & (m->cap - 1);
    return &m->slots[i];
}
static node_t *insert(or_mcts *m, const int8_t *st) {
    if (2 * (m->count + 1) > m->cap) {
        node_t **old = m->slots; int oc = m->cap;
        m->cap *= 2; m->slots = (node_t **)calloc((size_t)m->cap, sizeof(node_t *));
        for (int i = 0; i < oc; i++) if (old[i]) *lookup(m, old[i]->key) = old[i];
        free(old);
    }
    node_t **slot = lookup(m, st);
    node_t *nd = (node_t *)calloc(1, sizeof(node_t));
    nd->key = (int8_t *)malloc((size_t)m->S); memcpy(nd->key, st, (size_t)m->S);
    *slot = nd; m->count++;
    return nd;
}

/* pick_highest_UCB (MCTS.py:199-219), float64 as Numba types it */
static int pick_ucb(or_mcts *m, node_t *nd, int forced) {
    double best = -INFINITY; int ba = -1;
    double fpu_init = m->fpu > 0 ? nd->qs - m->fpu : m->fpu;
    for (int a = 0; a < 409; a++) {
        if (!nd->vs[a]) continue;
        double P = (double)nd->ps[a];
        if (forced && (double)nd->nsa[a] < (double)(long long)sqrt(0.5 * P * (double)m->step)) return a;
        double u;
        if (nd->qsa[a] != NAN_Q) u = nd->qsa[a] + m->cpuct * P * sqrt((double)nd->ns) / (double)(1 + nd->nsa[a]);
        else u = fpu_init + m->cpuct * P * sqrt((double)nd->ns + 1e-8);
        if (u > best) { best = u; ba = a; }
    }
    return ba;
}

static void search(or_mcts *m, const int8_t *st, int forced, int noise, float *vout, int depth) {
    int n = m->n;
    node_t *nd = *lookup(m, st);
    if (!nd) {
        float es[4]; or_check_end(n, st, es);
        int any = 0; for (int i = 0; i < n; i++) any |= es[i] != 0.f;
        nd = insert(m, st);
        memcpy(nd->es, es, sizeof es);
        if (any) { nd->terminal = 1; memcpy(vout, es, sizeof(float) * n); note_depth(depth); return; }
    } else if (nd->terminal) { memcpy(vout, nd->es, sizeof(float) * n); note_depth(depth); return; }
    if (!nd->has_ps) {
        note_depth(depth);
        or_valid_moves(n, st, 0, nd->vs);
        float v[4];
        or_fake_predict(n, st, nd->vs, nd->ps, v);
        if (m->neg_v) for (int i = 0; i < n; i++) v[i] = -v[i];
        if (noise) mcts_noise(m, nd);           /* softmax + noise + normalise (:141-144) */
        else {
            float sum = pw_sum(nd->ps, 409);    /* normalise (MCTS.py:239-242) */
            for (int a = 0; a < 409; a++) nd->ps[a] = nd->ps[a] / sum;
        }
        nd->has_ps = 1; nd->ns = 0; nd->qs = (double)v[0];
        for (int a = 0; a < 409; a++) { nd->qsa[a] = NAN_Q; nd->nsa[a] = 0; }
        memcpy(vout, v, sizeof(float) * n);
        return;
    }
    if (noise) mcts_noise(m, nd);               /* re-noised stored priors (:150-154) */
    int a = pick_ucb(m, nd, forced);
    int8_t *child = (int8_t *)malloc((size_t)m->S);
    int nxt = or_tree_step(n, st, a, child);
    float vc[4];
    search(m, child, 0, 0, vc, depth + 1);
    free(child);
    nd = *lookup(m, st);                       /* table may have been rehashed */
    for (int i = 0; i < n; i++) vout[i] = vc[((i - nxt) % n + n) % n];   /* np.roll */
    double v0 = (double)vout[0];
    nd->qsa[a] = ((double)nd->nsa[a] * nd->qsa[a] + v0) / (double)(nd->nsa[a] + 1);
    nd->qs = ((double)(nd->ns + 1) * nd->qs + v0) / (double)(nd->ns + 2);
    nd->nsa[a] += 1; nd->ns += 1;
}

int or_mcts_search(or_mcts *m, const int8_t *root, int64_t *counts, double *qsa,
                   double *probs, double *q) {
    float v[4];
    for (m->step = 0; m->step < m->sims; m->step++)
        search(m, root, m->forced, m->step == 0 && m->dir_alpha > 0, v, 0);
    node_t *nd = *lookup(m, root);
    long long c[409], best = 0;
    for (int a = 0; a < 409; a++) { c[a] = nd->nsa[a]; if (c[a] > best) best = c[a]; }
    if (m->forced) {                                  /* MCTS.py:69-74 */
        for (int a = 0; a < 409; a++) {
            if (c[a] != best) c[a] -= (long long)sqrt(0.5 * (double)nd->ps[a] * (double)m->sims);
            if (c[a] <= 1) c[a] = 0;
        }
    }
    long long tot = 0;
    for (int a = 0; a < 409; a++) tot += c[a];
    for (int a = 0; a < 409; a++) {
        counts[a] = nd->nsa[a]; qsa[a] = nd->qsa[a];
        probs[a] = (double)c[a] / (double)tot;
    }
    q[0] = nd->qs;
    for (int i = 1; i < m->n; i++) q[i] = -nd->qs / (double)(m->n - 1);
    return m->count;
}

/* ------------------------------------------------------------------ self-play loop */
/* Coach.executeEpisode (Coach.py:50-100) driven exactly like the device (spl_mcts_commit):
 * one MCTS simulation per iteration per game; when a search's budget is spent the move is
 * committed. Random decisions use Philox streams shared with the device:
 *   full/fast search ST_FULL|move, action pick ST_PICK|move, chance ST_MOVE|move,
 *   deals ST_DEAL|game, root Dirichlet noise ST_DIR|move (at the first simulation of a
 *   full search when dir_alpha > 0). */
#define ST_FULL (1u << 24)
#define ST_DIR  (2u << 24)
#define ST_PICK (3u << 24)
#define ST_MOVE (4u << 24)
#define ST_DEAL (5u << 24)

static double temp_pow(double x, double T) {       /* mcts_device.h temp_pow */
    if (T == 1.0) return x;
    double e = 1.0 / T;
    if (e == 0.5) return sqrt(x);
    int k = (int)e;
    if ((double)k == e && k >= 1 && k <= 8) { double r = x; for (int j = 1; j < k; j++) r = r * x; return r; }
    return pow(x, e);
}

static long long pruned(long long c, long long best, int forced, float p, int sims) {
    if (forced) {
        if (c != best) c -= (long long)sqrt(0.5 * (double)p * (double)sims);
        if (c <= 1) c = 0;
    }
    return c;
}

typedef struct {
    int8_t st[7 * 88]; int player; float q[4];
    float pi[409]; uint8_t va[409];
} or_ex_t;

int or_selfplay_run(int n, int B, int iters, uint64_t seed, uint32_t board_base, int num_sims,
                    int ratio_full, double prob_full, double cpuct, double fpu, int forced_po,
                    int temp_threshold, double dir_alpha, double dir_temp, int8_t *board_out,
                    int32_t *hdr_out, int max_ex, int8_t *ex_state, float *ex_pi, uint64_t *ex_valid,
                    float *ex_winner, int32_t *ex_scdiff, float *ex_q, int32_t *ex_meta) {
    build_tables();
    int S = 7 * or_rows(n), n_out = 0;
    or_ex_t *stage = (or_ex_t *)malloc(sizeof(or_ex_t) * (62 * n + 2));
    for (int t = 0; t < B; t++) {
        uint32_t gb = board_base + (uint32_t)t;
        int8_t board[7 * 88], canon[7 * 88];
        double u[40];
        int player = 0, step = 0, move_no = 0, game_no = 0, games_done = 0, moves = 0, nex = 0;
        for (int d = 0; d < 29; d++) u[d] = or_uniform(seed, gb, ST_DEAL | (uint32_t)game_no, (uint32_t)d);
        or_init(n, board, u, NULL);
        game_no++;
        or_mcts *m = or_mcts_new(n, num_sims, cpuct, fpu, forced_po);
        int full = 0, budget = 0, forced = 0, sims_done = 0;
#define BEGIN_SEARCH() do {                                                            \
            memcpy(canon, board, (size_t)S);                                           \
            if (player) or_swap_players(n, canon, player);                             \
            full = or_uniform(seed, gb, ST_FULL | (uint32_t)move_no, 0) < prob_full;   \
            move_no++;                                                                 \
            budget = full ? num_sims : num_sims / ratio_full;                          \
            forced = full && forced_po; sims_done = 0;                                 \
            or_mcts_set_noise(m, dir_alpha, dir_temp, seed, gb, ST_DIR | (uint32_t)move_no); \
        } while (0)
        BEGIN_SEARCH();
        for (int it = 0; it < iters; it++) {
            float v[4];
            m->step = sims_done;
            search(m, canon, forced, sims_done == 0 && full && dir_alpha > 0, v, 0);
            sims_done++;
            if (sims_done < budget) continue;
            /* commit */
            node_t *nd = *lookup(m, canon);
            long long best = 0, tot = 0, c[409];
            for (int a = 0; a < 409; a++) if (nd->vs[a] && nd->nsa[a] > best) best = nd->nsa[a];
            for (int mode = forced ? 0 : 1; mode < 3; mode++) {   /* 0/0 fallback */
                tot = 0;
                for (int a = 0; a < 409; a++) {
                    c[a] = !nd->vs[a] ? 0 : mode == 0 ? pruned(nd->nsa[a], best, 1, nd->ps[a], budget)
                                                      : mode == 1 ? nd->nsa[a] : 1;
                    tot += c[a];
                }
                if (tot > 0) break;
            }
            step++;
            if (full && nex < 62 * n + 2) {
                or_ex_t *x = &stage[nex++];
                memcpy(x->st, canon, (size_t)S);
                x->player = player;
                for (int a = 0; a < 409; a++) x->pi[a] = (float)((double)c[a] / (double)tot);
                or_valid_moves(n, canon, 0, x->va);
                x->q[0] = (float)nd->qs;
                for (int i = 1; i < 4; i++) x->q[i] = i < n ? (float)(-nd->qs / (double)(n - 1)) : 0.f;
            }
            double T = temp_threshold > 0 ? (step < temp_threshold ? 2.0 : 0.2) : 1.0;
            double sum = 0.0, last = 0.0, cdf = 0.0;
            for (int a = 0; a < 409; a++) if (c[a] || nd->vs[a]) sum += temp_pow((double)c[a] / (double)tot, T);
            for (int a = 0; a < 409; a++) if (c[a] || nd->vs[a]) last += temp_pow((double)c[a] / (double)tot, T) / sum;
            double uu = or_uniform(seed, gb, ST_PICK | (uint32_t)move_no, 0);
            int action = 408;
            for (int a = 408; a >= 0; a--) if (nd->vs[a]) { action = a; break; }
            for (int a = 0; a < 409; a++) {
                if (!(c[a] || nd->vs[a])) continue;
                cdf += temp_pow((double)c[a] / (double)tot, T) / sum;
                if (cdf / last > uu) { action = a; break; }
            }
            u[0] = or_uniform(seed, gb, ST_MOVE | (uint32_t)move_no, 0);
            u[1] = or_uniform(seed, gb, ST_MOVE | (uint32_t)move_no, 1);
            int nxt = or_make_move(n, board, action, player, 0, u, NULL);
            moves++;
            float r[4];
            or_check_end(n, board, r);
            int any = 0;
            for (int i = 0; i < n; i++) any |= r[i] != 0.f;
            if (any) {
                int f[4];
                for (int i = 0; i < n; i++) f[i] = or_get_score(n, board, i);
                for (int j = 0; j < nex; j++) {
                    if (n_out < max_ex) {
                        or_ex_t *x = &stage[j];
                        int px = x->player;
                        memcpy(ex_state + (size_t)n_out * S, x->st, (size_t)S);
                        memcpy(ex_pi + (size_t)n_out * 409, x->pi, 409 * 4);
                        uint64_t w[7] = {0};
                        for (int a = 0; a < 409; a++) if (x->va[a]) w[a >> 6] |= 1ull << (a & 63);
                        memcpy(ex_valid + (size_t)n_out * 7, w, sizeof w);
                        for (int i = 0; i < n; i++) {
                            ex_winner[(size_t)n_out * n + i] = r[(i + px) % n];
                            ex_scdiff[(size_t)n_out * n + i] = f[(i + px) % n] - f[px];
                            ex_q[(size_t)n_out * n + i] = x->q[i];
                        }
                        int32_t meta[4] = {(int32_t)gb, game_no - 1, j, px};
                        memcpy(ex_meta + (size_t)n_out * 4, meta, sizeof meta);
                    }
                    n_out++;
                }
                games_done++;
                for (int d = 0; d < 29; d++) u[d] = or_uniform(seed, gb, ST_DEAL | (uint32_t)game_no, (uint32_t)d);
                or_init(n, board, u, NULL);
                game_no++;
                player = 0; step = 0; nex = 0;
                or_mcts_free(m);                          /* MCTS.reset_all_search_trees */
                m = or_mcts_new(n, num_sims, cpuct, fpu, forced_po);
            } else {
                player = nxt;
            }
            BEGIN_SEARCH();
        }
#undef BEGIN_SEARCH
        if (board_out) memcpy(board_out + (size_t)t * S, board, (size_t)S);
        if (hdr_out) {
            int32_t h[8] = {player, step, move_no, game_no, games_done, moves, sims_done, budget};
            memcpy(hdr_out + (size_t)t * 8, h, sizeof h);
        }
        or_mcts_free(m);
    }
    free(stage);
    return n_out;
}

/* ------------------------------------------------------------------ rollout loop */
/* The fused random-policy env step of spl_rollout_step (include/splendor_amd.h), run
 * for B boards x steps. Outputs are optional (NULL = skip). Returns board-steps done. */
long long or_rollout_run(int n, int B, int steps, uint64_t seed, uint32_t board_base,
                         int8_t *state_out, int8_t *player_out, int16_t *actions,
                         float *ended, int32_t *games, uint64_t *mask_fold, uint64_t *masks) {
    build_tables();
    int S = 7 * or_rows(n);
    int8_t *st = (int8_t *)malloc((size_t)B * S), canon[7 * 88];
    int *pl = (int *)calloc((size_t)B, sizeof(int));
    uint32_t *gm = (uint32_t *)calloc((size_t)B, sizeof(uint32_t));   /* games ended per board */
    uint8_t mask[409];
    double u[40];
    long long done = 0;
    for (int b = 0; b < B; b++) {
        uint32_t gb = board_base + (uint32_t)b;
        for (int d = 0; d < 29; d++) u[d] = or_uniform(seed, gb, 0xFFFFFFFFu, (uint32_t)d);
        or_init(n, st + (size_t)b * S, u, NULL);
        if (games) games[b] = 0;
        if (mask_fold) mask_fold[b] = 0;
    }
    for (int t = 0; t < steps; t++) {
        for (int b = 0; b < B; b++) {
            uint32_t gb = board_base + (uint32_t)b;
            int8_t *s = st + (size_t)b * S;
            memcpy(canon, s, (size_t)S);
            if (pl[b]) or_swap_players(n, canon, pl[b]);
            or_valid_moves(n, canon, 0, mask);
            int cnt = 0;
            uint64_t w[7] = {0};
            for (int a = 0; a < 409; a++) { cnt += mask[a]; if (mask[a]) w[a >> 6] |= 1ull << (a & 63); }
            if (mask_fold) for (int j = 0; j < 7; j++) mask_fold[b] ^= (w[j] * (2 * (uint64_t)j + 1)) ^ ((uint64_t)t << 40);
            if (masks) memcpy(masks + ((size_t)t * B + b) * 7, w, sizeof w);
            int k = (int)(or_uniform(seed, gb, (uint32_t)t, 0) * (double)cnt), a;
            for (a = 0; a < 409; a++) if (mask[a] && k-- == 0) break;
            if (a == 409) a = 408;
            u[0] = or_uniform(seed, gb, (uint32_t)t, 1);
            u[1] = or_uniform(seed, gb, (uint32_t)t, 2);
            pl[b] = or_make_move(n, s, a, pl[b], 0, u, NULL);
            float e[4];
            or_check_end(n, s, e);
            int any = 0;
            for (int i = 0; i < n; i++) any |= e[i] != 0.f;
            if (actions) actions[(size_t)t * B + b] = (int16_t)a;
            if (ended) for (int i = 0; i < n; i++) ended[((size_t)t * B + b) * n + i] = e[i];
            if (any) {   /* game g's deal: uniforms 0..28 of stream 0x80000000 | g */
                gm[b] += 1;
                for (int d = 0; d < 29; d++) u[d] = or_uniform(seed, gb, 0x80000000u | gm[b], (uint32_t)d);
                or_init(n, s, u, NULL);
                pl[b] = 0;
                if (games) games[b] += 1;
            }
            done++;
        }
    }
    if (state_out) memcpy(state_out, st, (size_t)B * S);
    if (player_out) for (int b = 0; b < B; b++) player_out[b] = (int8_t)pl[b];
    free(st); free(pl); free(gm);
    return done;
}

/* boards are independent and every draw is keyed by the global board id, so contiguous
 * board ranges run on separate threads give exactly the single-thread result */
typedef struct { int n, B, steps; uint64_t seed; uint32_t base; long long done; } rr_job;
static void *rr_thread(void *p) {
    rr_job *j = (rr_job *)p;
    j->done = or_rollout_run(j->n, j->B, j->steps, j->seed, j->base, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    return NULL;
}
long long or_random_rollouts(int n, int B, int steps, uint64_t seed, int threads) {
    if (threads <= 1 || B < 2)
        return or_rollout_run(n, B, steps, seed, 0, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    if (threads > B) threads = B;
    build_tables();                              /* shared tables, built before the threads */
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    rr_job *jobs = (rr_job *)malloc(sizeof(rr_job) * (size_t)threads);
    int start = 0;
    for (int k = 0; k < threads; k++) {
        const int cnt = B / threads + (k < B % threads);
        jobs[k] = (rr_job){n, cnt, steps, seed, (uint32_t)start, 0};
        start += cnt;
        pthread_create(&tid[k], NULL, rr_thread, &jobs[k]);
    }
    long long done = 0;
    for (int k = 0; k < threads; k++) { pthread_join(tid[k], NULL); done += jobs[k].done; }
    free(tid); free(jobs);
    return done;
}
