"""The descent's float32 UCB screen (csrc/mcts.hip pick_edge64 / pick_edge_desc): every
edge's float32 estimate uf must lie within e = 2.1e-6 (|uf| + |qf|) of the float64 value
the reference computes (MCTS.py:199-219), so the arg-max taken from the screen — the one
edge whose [uf - e, uf + e] can reach max(uf - e) — is the reference's strict-'>' arg-max.
NumPy float32 emulation of the device arithmetic, with v_sqrt_f32 / v_rcp_f32 pushed a
full ulp the wrong way (their accuracy), over random and boundary cases (CPU)."""
import numpy as np

E_REL = np.float32(2.1e-6)


def screen(q, p, n, ns, vis, fpu_init, cpuct):
    f = np.float32
    nf = ns.astype(f)
    sq = np.where(vis, np.sqrt(nf), np.sqrt(nf + f(1e-8))).astype(f)
    rc = np.where(vis, (f(1) / (f(1) + n.astype(f))).astype(f), f(1)).astype(f)
    # 1-ulp hardware approximations, worst direction
    sq = np.nextafter(sq, f(np.inf)).astype(f)
    rc = np.where(vis, np.nextafter(rc, f(np.inf)), rc).astype(f)
    qf = np.where(vis, q.astype(f), fpu_init.astype(f)).astype(f)
    cf = f(cpuct)
    uf = (qf + ((cf * p).astype(f) * sq).astype(f) * rc).astype(f)
    e = (E_REL * (np.abs(uf) + np.abs(qf)) + f(1e-30)).astype(f)
    return uf, e


def exact(q, p, n, ns, vis, fpu_init, cpuct):
    sq = np.sqrt(ns.astype(np.float64))
    sqe = np.sqrt(ns.astype(np.float64) + 1e-8)
    return np.where(vis, q + cpuct * p.astype(np.float64) * sq / (1 + n), fpu_init + cpuct * p.astype(np.float64) * sqe)


def test_estimate_error_within_a_third_of_the_bound():
    rng = np.random.default_rng(7)
    N = 2_000_000
    q = rng.uniform(-1, 1, N)
    q[:1000] = rng.choice([-1.0, 1.0, 0.0, 1e-300], 1000)
    p = (rng.random(N) ** 3).astype(np.float32)
    p[1000:2000] = 0
    n = rng.integers(0, 5000, N)
    ns = n + rng.integers(0, 20000, N)
    ns[2000:3000] = 0
    vis = rng.random(N) < 0.6
    vis[2000:3000] = False                      # a never-visited node: unvisited edges only
    fpu_init = rng.uniform(-1.3, 1.0, N)
    for cpuct in (2.5, 1.5, 0.5, 4.0):
        uf, e = screen(q, p, n, ns, vis, fpu_init, cpuct)
        u = exact(q, p, n, ns, vis, fpu_init, cpuct)
        err = np.abs(uf.astype(np.float64) - u)
        assert (err <= e.astype(np.float64) / 3).all(), float((err / e).max())


def test_screen_never_drops_the_argmax():
    """Random nodes: whenever the screen names a single candidate it is the float64 arg-max
    (lowest index on ties); near ties leave several candidates (the exact path)."""
    rng = np.random.default_rng(11)
    single = 0
    for _ in range(3000):
        ec = int(rng.integers(1, 65))
        ns = int(rng.integers(0, 400))
        vis = rng.random(ec) < (0.0 if ns == 0 else 0.5)
        q = np.where(vis, rng.uniform(-1, 1, ec), -42.0)
        if rng.random() < 0.3:                   # flat priors: many exact ties among unvisited edges
            p = np.full(ec, np.float32(1.0 / ec))
        else:
            p = rng.dirichlet(np.ones(ec)).astype(np.float32)
        n = np.where(vis, rng.integers(1, max(2, ns + 1), ec), 0)
        qs = rng.uniform(-1, 1)
        fpu_init = np.full(ec, qs - 0.3)
        nsa = np.full(ec, ns)
        uf, e = screen(q, p, n, nsa, vis, fpu_init, 2.5)
        u = exact(q, p, n, nsa, vis, fpu_init, 2.5)
        L = (uf - e).max()
        cand = np.flatnonzero(uf + e >= L)
        want = int(np.flatnonzero(u == u.max())[0])
        assert want in cand
        if len(cand) == 1:
            single += 1
            assert cand[0] == want
    assert single > 1000
