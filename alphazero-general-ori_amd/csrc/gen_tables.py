#!/usr/bin/env python3
"""Emits splendor_tables.h: the device constant tables of the Splendor engine.

Card / noble data are the game's published component lists (reference data tables at
SplendorLogic.py:320-473). Gem-combination tables follow SplendorLogic.py:250-280
(itertools.combinations order). The 409-entry action descriptor table encodes
SplendorLogicNumba.valid_moves (:251-265) as "flag0 AND flag1 AND condition", so a wave
evaluates 64 actions per instruction stream with no divergence.

Run:  python gen_tables.py > splendor_tables.h
"""
import itertools

NOBLES = [(0, 0, 4, 4, 0), (0, 0, 0, 4, 4), (0, 4, 4, 0, 0), (4, 0, 0, 0, 4), (4, 4, 0, 0, 0),
          (3, 0, 0, 3, 3), (3, 3, 3, 0, 0), (0, 0, 3, 3, 3), (0, 3, 3, 3, 0), (3, 3, 0, 0, 3)]
# deck column c holds cards whose gain colour is GAIN[c]
GAIN = (1, 3, 4, 0, 2)
# (cost white, blue, green, red, black, points) per [deck column][card]
TIER1 = [
    [(0,0,0,0,3,0),(1,0,0,0,2,0),(0,0,2,0,2,0),(1,0,2,2,0,0),(0,1,3,1,0,0),(1,0,1,1,1,0),(1,0,1,2,1,0),(0,0,0,4,0,1)],
    [(3,0,0,0,0,0),(0,2,1,0,0,0),(2,0,0,2,0,0),(2,0,1,0,2,0),(1,0,0,1,3,0),(1,1,1,0,1,0),(2,1,1,0,1,0),(4,0,0,0,0,1)],
    [(0,0,3,0,0,0),(0,0,2,1,0,0),(2,0,2,0,0,0),(2,2,0,1,0,0),(0,0,1,3,1,0),(1,1,1,1,0,0),(1,2,1,1,0,0),(0,4,0,0,0,1)],
    [(0,3,0,0,0,0),(0,0,0,2,1,0),(0,2,0,0,2,0),(0,2,2,0,1,0),(3,1,0,0,1,0),(0,1,1,1,1,0),(0,1,2,1,1,0),(0,0,4,0,0,1)],
    [(0,0,0,3,0,0),(2,1,0,0,0,0),(0,2,0,2,0,0),(0,1,0,2,2,0),(1,3,1,0,0,0),(1,1,0,1,1,0),(1,1,0,1,2,0),(0,0,0,0,4,1)]]
TIER2 = [
    [(0,2,2,3,0,1),(0,2,3,0,3,1),(0,5,0,0,0,2),(5,3,0,0,0,2),(2,0,0,1,4,2),(0,6,0,0,0,3)],
    [(2,0,0,2,3,1),(0,3,0,2,3,1),(0,0,0,0,5,2),(3,0,0,0,5,2),(1,4,2,0,0,2),(0,0,0,6,0,3)],
    [(3,2,2,0,0,1),(3,0,3,0,2,1),(5,0,0,0,0,2),(0,0,5,3,0,2),(0,1,4,2,0,2),(0,0,0,0,6,3)],
    [(0,0,3,2,2,1),(2,3,0,3,0,1),(0,0,0,5,0,2),(0,0,0,5,3,2),(0,0,1,4,2,2),(6,0,0,0,0,3)],
    [(2,3,0,0,2,1),(3,0,2,3,0,1),(0,0,5,0,0,2),(0,5,3,0,0,2),(4,2,0,0,1,2),(0,0,6,0,0,3)]]
TIER3 = [
    [(3,0,3,3,5,3),(7,0,0,0,0,4),(6,3,0,0,3,4),(7,3,0,0,0,5)],
    [(3,5,3,0,3,3),(0,0,7,0,0,4),(0,3,6,3,0,4),(0,0,7,3,0,5)],
    [(3,3,5,3,0,3),(0,0,0,7,0,4),(0,0,3,6,3,4),(0,0,0,7,3,5)],
    [(0,3,3,5,3,3),(0,0,0,0,7,4),(3,0,0,3,6,4),(3,0,0,0,7,5)],
    [(5,3,0,3,3,3),(0,7,0,0,0,4),(3,6,3,0,0,4),(0,7,3,0,0,5)]]

# exchange give tables (Board.give_ids slices actually read, SplendorLogicNumba.py:100-166)
GIVE0 = [[3,4],[2,4],[2,3],[1,4],[1,3],[1,2],[0,4],[0,3],[0,2],[0,1]]
GIVE1 = [[14,18,19],[13,17,19],[12,17,18],[11,16,19],[10,16,18],[9,16,17],[8,15,19],[7,15,18],[6,15,17],[5,15,16]]
GIVE2 = [[12,13,14,17,18,19],[10,11,14,16,18,19],[9,11,13,17,16,19],[9,10,12,17,16,18],[7,8,14,15,19,18],
         [6,8,13,15,19,17],[6,7,12,15,18,17],[5,8,11,15,19,16],[5,7,10,15,18,16],[6,5,9,15,16,17]]
GIVE3 = [[9,12,13,10,11,14,17,16,18,19],[6,7,8,12,13,14,15,17,18,19],[5,7,8,10,11,14,15,16,18,19],
         [6,5,8,9,13,11,15,17,16,19],[6,5,7,9,12,10,15,17,16,18]]
GIVE4 = [[2,3,4],[1,3,4],[1,2,4],[1,2,3],[0,3,4],[0,2,4],[0,2,3],[0,1,4],[0,1,3],[0,1,2]]
GIVE5 = [[1,2,3,4],[0,2,3,4],[0,1,3,4],[0,1,2,4],[0,1,2,3]]
GIVE_T1 = [1,2,3,4, 0,2,3,4, 0,1,3,4, 0,1,2,4, 0,1,2,3]
GIVE_IDS3 = [(0,3,18),(0,18,4),(0,3,19),(0,19,4),(1,2,17),(1,17,4),(1,2,19),(1,19,4),(2,2,17),(2,17,3),
             (2,2,18),(2,18,3),(3,1,16),(3,16,4),(3,1,19),(3,19,4),(4,1,16),(4,16,3),(4,1,18),(4,18,3),
             (5,1,16),(5,16,2),(5,1,17),(5,17,2),(6,0,15),(6,15,4),(6,0,19),(6,19,4),(7,0,15),(7,15,3),
             (7,0,18),(7,18,3),(8,0,15),(8,15,2),(8,0,17),(8,17,2),(9,0,15),(9,15,1),(9,0,16),(9,16,1)]


def combos():
    out = []
    for k in (1, 2, 3):
        for c in itertools.combinations(range(5), k):
            out.append(tuple(1 if i in c else 0 for i in range(5)))
    return out


DIFF = combos()                      # 25 (first 15 = up to 2 different)
TAKE = DIFF + [tuple(2 if i == c else 0 for i in range(5)) for c in range(5)]  # 30
GIVE = DIFF[:15] + [tuple(2 if i == c else 0 for i in range(5)) for c in range(5)]  # 20
SPEC3 = [tuple(GIVE[a][c] + GIVE[b][c] for c in range(5)) for (_, a, b) in GIVE_IDS3]

# condition codes (must match splendor_device.h)
C_ALWAYS, C_RSV_LIMIT, C_TAKE1, C_TAKE2D, C_TAKE3, C_TAKE2S, C_EX8, C_EX9, C_EX10, C_EX10G, C_NEVER = range(11)


def desc(i0, i1, cond):
    d = cond << 16
    if i0 is not None:
        d |= (1 << 6) | i0
    if i1 is not None:
        d |= (1 << 14) | (i1 << 8)
    return d


def action_table():
    t = []
    for a in range(12):
        t.append(desc(a, None, C_ALWAYS))
    for a in range(12, 27):
        t.append(desc(a, None, C_RSV_LIMIT))
    for a in range(27, 30):
        t.append(desc(a, None, C_ALWAYS))
    for a in range(30, 35):
        t.append(desc(a, None, C_TAKE1))
    for a in range(35, 45):
        t.append(desc(a, None, C_TAKE2D))
    for a in range(45, 55):
        t.append(desc(a, None, C_TAKE3))
    for a in range(55, 60):
        t.append(desc(a, None, C_TAKE2S))
    t += [desc(45 + k // 2, GIVE0[k // 2][k % 2], C_EX8) for k in range(20)]          # 60-79
    t += [desc(45 + k // 3, GIVE1[k // 3][k % 3], C_EX9) for k in range(30)]          # 80-109
    t += [desc(35 + k // 6, GIVE2[k // 6][k % 6], C_EX10) for k in range(60)]         # 110-169
    t += [desc(55 + k // 10, GIVE3[k // 10][k % 10], C_EX10) for k in range(50)]      # 170-219
    t += [desc(35 + k // 3, GIVE4[k // 3][k % 3], C_EX9) for k in range(30)]          # 220-249
    t += [desc(55 + k // 4, GIVE5[k // 4][k % 4], C_EX9) for k in range(20)]          # 250-269
    t += [desc(30 + k // 4, GIVE_T1[k], C_EX10) for k in range(20)]                   # 270-289
    t += [desc(12 + k // 5, k % 5, C_EX10G) for k in range(75)]                       # 290-364
    t += [desc(45 + k // 4, 20 + k, C_EX10) for k in range(40)]                       # 365-404
    t += [desc(None, None, C_NEVER)] * 4                                              # 405-408
    assert len(t) == 409
    return t


# move decode for _give_and_get_gems / _reserve_and_give (SplendorLogicNumba.py:697-761):
# for exchange action a in [60,405): (take id in TAKE, give id 1 in GIVE, give id 2 or 255,
# reserve index or 255)
def exchange_table():
    t = []
    for a in range(60, 405):
        i = a - 60
        if a >= 290 and a < 365:
            j = a - 290
            t.append((255, j % 5, 255, j // 5))
        elif i < 20:
            t.append((i // 2 + 15, GIVE0[i // 2][i % 2], 255, 255))
        elif i < 50:
            k = i - 20; t.append((k // 3 + 15, GIVE1[k // 3][k % 3], 255, 255))
        elif i < 110:
            k = i - 50; t.append((k // 6 + 5, GIVE2[k // 6][k % 6], 255, 255))
        elif i < 160:
            k = i - 110; t.append((k // 10 + 25, GIVE3[k // 10][k % 10], 255, 255))
        elif i < 190:
            k = i - 160; t.append((k // 3 + 5, GIVE4[k // 3][k % 3], 255, 255))
        elif i < 210:
            k = i - 190; t.append((k // 4 + 25, GIVE5[k // 4][k % 4], 255, 255))
        elif i < 230:
            k = i - 210; t.append((k // 4, GIVE_T1[k], 255, 255))
        else:
            k = i - 305; tk, g1, g2 = GIVE_IDS3[k]; t.append((tk + 15, g1, g2, 255))
    return t


def take_need(t):
    """bank level needed per colour by take t (F0 bit 30 + t): level 1 = >= 1 gem, 2 = >= 4."""
    return TAKE[t] if t < 25 else tuple(2 if c == t - 25 else 0 for c in range(5))


def give_need(g):
    """gem level (min(gems, 3)) needed per colour by give set g (F1 bit g)."""
    return GIVE[g] if g < 20 else SPEC3[g - 20]


def mask_factors():
    """Factorised mask words for reachable boards (splendor_device.h lane_mask_word_fast):
    word K = gate(C) & card(F0 bits 0-29) & U1[bank levels c0-2] & U2[c3-4] & V1[gem levels
    c0-2] & V2[c3-4]. Bank level = 0 / 1 (1-3 gems) / 2 (>= 4); gem level = min(gems, 3).
    Returns (per-word table rows, per-word condition masks, card blocks)."""
    desc = action_table()
    rows, gates, blocks = [], [], []
    for K in range(7):
        acts = [(j, desc[64 * K + j]) for j in range(64) if 64 * K + j < 409]

        def table(colours, base, need_of):
            out = []
            for idx in range(base ** len(colours)):
                lv = [(idx // base ** i) % base for i in range(len(colours))]
                m = 0
                for j, d in acts:
                    need = need_of(d)
                    if need is None or all(lv[i] >= need[c] for i, c in enumerate(colours)):
                        m |= 1 << j
                # bits past action 408 are 1 here; the gates never set them
                out.append(m | (((1 << 64) - 1) ^ sum(1 << j for j, _ in acts)))
            return out

        tk = lambda d: take_need((d & 63) - 30) if (d >> 6) & 1 and (d & 63) >= 30 else None
        gv = lambda d: give_need((d >> 8) & 63) if (d >> 14) & 1 else None
        rows.append(table((0, 1, 2), 3, tk) + table((3, 4), 3, tk) + table((0, 1, 2), 4, gv) + table((3, 4), 4, gv))
        gates.append([sum(1 << j for j, d in acts if (d >> 16) & 15 == c) for c in range(11)])
        # card predicate bits (F0 < 30): runs copied (f0 rises with j) or replicated (same f0)
        uses = [(j, d & 63) for j, d in acts if (d >> 6) & 1 and (d & 63) < 30]
        i = 0
        while i < len(uses):
            j0, f0 = uses[i]
            n = 1
            if i + 1 < len(uses) and uses[i + 1] == (j0 + 1, f0 + 1):
                while i + n < len(uses) and uses[i + n] == (j0 + n, f0 + n):
                    n += 1
                blocks.append((K, j0, n, f0, 0))        # copy F0[f0 .. f0+n) to j0 ..
            else:
                while i + n < len(uses) and uses[i + n] == (j0 + n, f0):
                    n += 1
                blocks.append((K, j0, n, f0, 1))        # replicate F0[f0] over j0 .. j0+n
            i += n
    return rows, gates, blocks


def check_mask_factors(rows, gates, blocks, trials=20000):
    """The factorised words equal the descriptor formula C & F0 & F1 on random predicates."""
    import random
    rnd = random.Random(7)
    desc = action_table()
    for _ in range(trials):
        bank = [rnd.randint(0, 7) for _ in range(5)]
        gems = [rnd.randint(0, 5) for _ in range(5)]
        cards = rnd.getrandbits(30)
        C = rnd.getrandbits(10)
        lam = [0 if b < 1 else (1 if b < 4 else 2) for b in bank]
        ell = [min(g, 3) for g in gems]
        F0 = cards
        for t in range(30):
            need = take_need(t)
            if all(bank[c] >= (4 if need[c] == 2 else need[c]) for c in range(5)):
                F0 |= 1 << (30 + t)
        F1 = sum(1 << g for g in range(60) if all(gems[c] >= give_need(g)[c] for c in range(5)))
        for K in range(7):
            want = 0
            for j in range(64):
                a = 64 * K + j
                if a >= 409:
                    continue
                d = desc[a]
                bit = (C >> ((d >> 16) & 15)) & 1
                if (d >> 6) & 1:
                    bit &= F0 >> (d & 63)
                if (d >> 14) & 1:
                    bit &= F1 >> ((d >> 8) & 63)
                want |= (bit & 1) << j
            r = rows[K]
            got = r[lam[0] + 3 * lam[1] + 9 * lam[2]] & r[27 + lam[3] + 3 * lam[4]]
            got &= r[36 + ell[0] + 4 * ell[1] + 16 * ell[2]] & r[100 + ell[3] + 4 * ell[4]]
            gate = 0
            for c in range(11):
                if (C >> c) & 1:
                    gate |= gates[K][c]
            card = (1 << 64) - 1
            for (k, j0, n, f0, rep) in blocks:
                if k != K:
                    continue
                span = ((1 << n) - 1) << j0
                src = (((cards >> f0) & 1) * ((1 << n) - 1) if rep else (cards >> f0) & ((1 << n) - 1)) << j0
                card &= ~span | src
            got &= gate & card
            assert got == want, (K, hex(got), hex(want))


def arr(name, ctype, rows, fmt=str):
    body = ",\n  ".join("{" + ",".join(fmt(x) for x in r) + "}" if isinstance(r, (list, tuple)) else fmt(r)
                        for r in rows)
    return f"{name} = {{\n  {body}}};\n"


def main():
    out = ["// GENERATED by gen_tables.py — do not edit by hand.",
           "#pragma once", "#include <stdint.h>", ""]
    cards = []
    for tier, tab in enumerate((TIER1, TIER2, TIER3)):
        for col in range(5):
            for k in range(8):
                if k < len(tab[col]):
                    cost = tab[col][k][:5]
                    pts = tab[col][k][5]
                    cards.append(list(cost) + [GAIN[col], pts, 0])
                else:
                    cards.append([0] * 8)
    out.append("// [tier*40 + deckcol*8 + k] -> cost[5], gain colour, points, pad")
    out.append(arr("static __constant__ int8_t K_CARDS[120][8]", None, cards))
    out.append(arr("static __constant__ int8_t K_NOBLES[10][8]", None, [list(n) + [0, 3, 0] for n in NOBLES]))
    out.append(arr("static __constant__ int8_t K_TAKE[30][8]", None, [list(v) + [sum(v), 0, 0] for v in TAKE]))
    out.append(arr("static __constant__ int8_t K_GIVE[20][8]", None, [list(v) + [sum(v), 0, 0] for v in GIVE]))
    out.append(arr("static __constant__ int8_t K_SPEC3[40][8]", None, [list(v) + [0, 0, 0] for v in SPEC3]))
    out.append("// action descriptor: bits0-5 flag0 idx, bit6 use flag0, bits8-13 flag1 idx, bit14 use flag1,")
    out.append("// bits16-19 condition code")
    out.append(arr("static __constant__ uint32_t K_ACTION_DESC[409]", None, action_table(), lambda x: f"0x{x:06x}u"))
    out.append("// exchange actions 60..404: take id, give id, give id (255 none), reserve index (255 none)")
    out.append(arr("static __constant__ uint8_t K_EXCHANGE[345][4]", None, exchange_table()))
    # ---- packed forms for the 8-byte-row LDS layout (splendor_device.h)
    def pack(vals):
        v = 0
        for i, x in enumerate(vals):
            v |= (x & 0xFF) << (8 * i)
        return v
    rows = []
    for tier, tab in enumerate((TIER1, TIER2, TIER3)):
        for col in range(5):
            for k in range(8):
                if k < len(tab[col]):
                    cost = list(tab[col][k][:5])
                    gain = [0] * 7
                    gain[GAIN[col]] = 1
                    gain[6] = tab[col][k][5]
                    rows.append((pack(cost), pack(gain)))
                else:
                    rows.append((0, 0))
    out.append("// [tier*40 + deckcol*8 + k] -> (cost row, gain row) as packed 8-byte rows")
    out.append(arr("static __constant__ uint64_t K_CARD_ROWS[120][2]", None, rows, lambda x: f"0x{x:016x}ull"))
    out.append(arr("static __constant__ uint64_t K_NOBLE_ROWS[10]", None, [pack(list(n) + [0, 3]) for n in NOBLES],
                   lambda x: f"0x{x:016x}ull"))
    out.append(arr("static __constant__ uint64_t K_TAKE_ROW[30]", None, [pack(v) for v in TAKE], lambda x: f"0x{x:016x}ull"))
    out.append(arr("static __constant__ uint64_t K_GIVE_ROW[20]", None, [pack(v) for v in GIVE], lambda x: f"0x{x:016x}ull"))
    out.append(arr("static __constant__ uint64_t K_SPEC3_ROW[40]", None, [pack(v) for v in SPEC3], lambda x: f"0x{x:016x}ull"))
    out.append("// exact IEEE quotients for the deck draw: K_QUOT[tot][cnt] = cnt / tot, K_RECIP[n] = 1 / n")
    quot = [[(c / t if t else 0.0) for c in range(9)] for t in range(41)]
    out.append(arr("static __constant__ double K_QUOT[41][9]", None, quot, lambda x: float(x).hex()))
    out.append(arr("static __constant__ double K_RECIP[9]", None, [0.0] + [1.0 / n for n in range(1, 9)],
                   lambda x: float(x).hex()))
    # ---- per-action gem vectors for the flattened make_move: take / give rows (give = sum of
    # the exchange's give vectors) and the reserve index (-1: none)
    act_take, act_give, act_rsv = [0] * 409, [0] * 409, [-1] * 409
    for a in range(12, 27):
        act_rsv[a] = a - 12
    for a in range(30, 60):
        act_take[a] = pack(TAKE[a - 30])
    for a, (tk, g1, g2, rv) in zip(range(60, 405), exchange_table()):
        if tk != 255:
            act_take[a] = pack(TAKE[tk])
        gv = [GIVE[g1][c] + (GIVE[g2][c] if g2 != 255 else 0) for c in range(5)]
        assert max(gv) < 128
        act_give[a] = pack(gv)
        if rv != 255:
            act_rsv[a] = rv
    out.append("// per action: gems taken / given back (packed rows) and reserve index (-1 none)")
    out.append(arr("static __constant__ uint64_t K_ACT_TAKE[409]", None, act_take, lambda x: f"0x{x:016x}ull"))
    out.append(arr("static __constant__ uint64_t K_ACT_GIVE[409]", None, act_give, lambda x: f"0x{x:016x}ull"))
    out.append(arr("static __constant__ int8_t K_ACT_RSV[409]", None, act_rsv))
    # ---- compile-time forms for the lane-per-board mask (splendor_device.h lane_predicates)
    # threshold masks: bit 5t+c <-> value_c >= t (t = 0..4); a predicate "x >= v in every
    # colour" holds iff REQ(v) & ~THRESH(x) == 0
    def req(v):
        assert max(v) <= 4
        return sum(1 << (5 * t + c) for c in range(5) for t in range(v[c] + 1))
    req0 = [0] * 30 + [req(TAKE[i]) for i in range(25)] + [1 << (20 + c) for c in range(5)]
    req1 = [req(GIVE[i]) for i in range(15)] + [1 << (10 + c) for c in range(5)] + [req(v) for v in SPEC3]
    # subset / level lookup tables for non-negative gem rows (lane_predicates fast path):
    # LUT_DIFF[m] bit i <-> DIFF[i] within colour set m; LUT_SPEC3[l] bit j <-> SPEC3[j] <=
    # levels l (2 bits per colour: min(count, 3))
    lut_diff = [sum(1 << i for i, v in enumerate(DIFF) if all(v[c] <= ((m >> c) & 1) for c in range(5)))
                for m in range(32)]
    assert max(max(v) for v in SPEC3) <= 3
    lut_s3 = [sum(1 << j for j, v in enumerate(SPEC3) if all(v[c] <= ((l >> (2 * c)) & 3) for c in range(5)))
              for l in range(1024)]
    out.append(arr("static __constant__ uint32_t K_LUT_DIFF[32]", None, lut_diff, lambda x: f"0x{x:07x}u"))
    out.append(arr("static __constant__ uint64_t K_LUT_SPEC3[1024]", None, lut_s3, lambda x: f"0x{x:010x}ull"))
    out.append("// compile-time copies for fully unrolled lane-per-board evaluation")
    out.append(arr("static constexpr uint32_t KC_ACTION_DESC[409]", None, action_table(), lambda x: f"0x{x:06x}u"))
    out.append("// F0 bits 30..59 / F1 bits 0..59: required threshold bits (bit 5t+c: colour c >= t)")
    out.append(arr("static constexpr uint32_t KC_REQ0[60]", None, req0, lambda x: f"0x{x:07x}u"))
    out.append(arr("static constexpr uint32_t KC_REQ1[60]", None, req1, lambda x: f"0x{x:07x}u"))
    # ---- factorised mask words (lane_mask_word_fast)
    rows, gates, blocks = mask_factors()
    check_mask_factors(rows, gates, blocks)
    out.append("// factorised mask words: per word K, 116 rows = U1[27] (bank levels c0-2, base 3),")
    out.append("// U2[9] (c3-4), V1[64] (gem levels c0-2, base 4), V2[16] (c3-4); level tables AND to")
    out.append("// the take / give feasibility of every action of the word (1 where unused)")
    out.append(arr("static __constant__ uint64_t K_MASK_FACTORS[7][116]", None, rows, lambda x: f"0x{x:016x}ull"))
    out.append("// per word K: actions gated by condition code c")
    out.append(arr("static constexpr uint64_t KC_MASK_GATE[7][11]", None, gates, lambda x: f"0x{x:016x}ull"))
    out.append("// card-predicate runs: word, first bit, length, F0 bit, replicate (1) or copy (0)")
    out.append(f"static constexpr int KC_CARD_NBLK = {len(blocks)};")
    out.append(arr(f"static constexpr uint8_t KC_CARD_BLK[{len(blocks)}][5]", None, blocks))
    print("\n".join(out))


if __name__ == "__main__":
    main()
