"""Python statement of the build's keyed random streams (test infrastructure).

Used by make_golden.py to inject into the reference exactly the draws that the device and
the oracle make, so that reference runs with injected randomness can be compared with
them bit for bit:

* `uniform(seed, board, stream, d)`: uniform d of a (seed, board, stream) sequence =
  half d&1 of Philox4x32-10 block (counter d>>1, board, stream, 'SPLD'), 53 bits
  (oracle or_uniform, device philox_u01);
* `dirichlet(alpha, seed, board, stream, k)`: the Dirichlet sampler that replaces the
  reference's unseeded `Generator.dirichlet` (MCTS.py:181): Marsaglia-Tsang Gamma with
  polar normals, logarithm / exponential from + - * / only (identical on every platform),
  normalised like numpy's dirichlet (sequential sum, times its reciprocal).

Python floats are IEEE doubles and Python never contracts a*b+c into an FMA, so these
functions give the same bits as the C oracle (-ffp-contract=off) and the device.
"""
import math
import struct

M32 = 0xFFFFFFFF


def philox4x32(k0, k1, c):
    c0, c1, c2, c3 = c
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        hi0, lo0 = (p0 >> 32) & M32, p0 & M32
        hi1, lo1 = (p1 >> 32) & M32, p1 & M32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3


def uniform(seed, board, stream, d):
    o = philox4x32(seed & M32, (seed >> 32) & M32, (d >> 1, board & M32, stream & M32, 0x53504C44))
    w0, w1 = (o[0], o[1]) if (d & 1) == 0 else (o[2], o[3])
    return (float(w0 >> 5) * 67108864.0 + float(w1 >> 6)) * (1.0 / 9007199254740992.0)


class Stream:
    """Sequential draws 0, 1, 2, ... of one (seed, board, stream) sequence."""

    def __init__(self, seed, board, stream, start=0):
        self.key = (seed, board, stream)
        self.d = start

    def random(self):
        u = uniform(*self.key, self.d)
        self.d += 1
        return u


LN2_HI = 6.93147180369123816490e-01
LN2_LO = 1.90821492927058770002e-10
INV_LN2 = 1.44269504088896338700e+00
SQRT2 = 1.4142135623730951


def det_log(x):
    b = struct.unpack("<Q", struct.pack("<d", x))[0]
    e = ((b >> 52) & 0x7FF) - 1023
    m = struct.unpack("<d", struct.pack("<Q", (b & 0x000FFFFFFFFFFFFF) | 0x3FF0000000000000))[0]
    if m > SQRT2:
        m = m * 0.5
        e = e + 1
    f = (m - 1.0) / (m + 1.0)
    s = f * f
    p = 1.0 / 23.0
    for k in (21.0, 19.0, 17.0, 15.0, 13.0, 11.0, 9.0, 7.0, 5.0, 3.0):
        p = p * s + 1.0 / k
    t = 2.0 * f
    r = t + t * (s * p)
    return float(e) * LN2_HI + (r + float(e) * LN2_LO)


def det_exp(x):
    if x < -700.0:
        return 0.0
    kf = float(math.floor(x * INV_LN2 + 0.5))
    r = (x - kf * LN2_HI) - kf * LN2_LO
    p = 1.0 / 6227020800.0
    for c in (1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0, 1.0 / 362880.0, 1.0 / 40320.0,
              1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0):
        p = p * r + c
    return math.ldexp(p, int(kf))


def det_pow(x, y):
    return 0.0 if x == 0.0 else det_exp(y * det_log(x))


def det_gamma(alpha, seed, board, stream, ctr):
    a = alpha + 1.0 if alpha < 1.0 else alpha
    d = a - 1.0 / 3.0
    c = 1.0 / math.sqrt(9.0 * d)
    g = 0.0
    for _ in range(64):
        z = 0.0
        for _ in range(16):
            u1 = 2.0 * uniform(seed, board, stream, ctr) - 1.0
            u2 = 2.0 * uniform(seed, board, stream, ctr + 1) - 1.0
            ctr += 2
            s = u1 * u1 + u2 * u2
            if 0.0 < s < 1.0:
                z = u1 * math.sqrt(-2.0 * det_log(s) / s)
                break
        v = 1.0 + c * z
        if v <= 0.0:
            continue
        v = v * v * v
        u = max(uniform(seed, board, stream, ctr), 1e-300)
        ctr += 1
        if det_log(u) < 0.5 * z * z + d - d * v + d * det_log(v):
            g = d * v
            break
    if alpha < 1.0:
        u = max(uniform(seed, board, stream, ctr), 1e-300)
        g = g * det_exp(det_log(u) / alpha)
    return g


def dirichlet(alpha, seed, board, stream, count):
    g = [det_gamma(alpha, seed, board, stream, i * 4096) for i in range(count)]
    acc = 0.0
    for x in g:
        acc = acc + x
    if acc > 0.0:
        inv = 1.0 / acc
        return [x * inv for x in g]
    return [1.0 / count] * count
