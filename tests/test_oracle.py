"""CPU: the oracle against the reference's golden vectors and against numpy
(the third-party RNG the reference calls).  No GPU needed."""
import numpy as np
import pytest

from conftest import IM_GOLDENS, NET_GOLDENS, NV_GOLDENS, im_kwargs, load_golden, nv_kwargs


def _bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b).astype(a.dtype)
    return np.array_equal(a.view(np.uint8), b.view(np.uint8))


# ---------------------------------------------------------------- RNG
def test_rng_kat_fixture(oracle):
    fx, cfg = load_golden("rng_kat")
    for i, s in enumerate(int(x) for x in cfg["seeds"]):
        st = oracle.pcg64_init(s)
        assert (st == fx["init_state"][i]).all(), s
        raw = [oracle.lib().orc_next64(oracle._p(st)) for _ in range(16)]
        assert (np.array(raw, np.uint64) == fx["random_raw"][i]).all()
        st = oracle.pcg64_init(s)
        dbl = [oracle.lib().orc_next_double(oracle._p(st)) for _ in range(16)]
        assert _bits_equal(np.array(dbl), fx["random_double"][i])
        for j, lam in enumerate(cfg["lams"]):
            out, st = oracle.poisson_stream(s, lam, 1000)
            assert (out == fx["poisson"][i, j]).all(), (s, lam)
            assert (st[:2] == fx["poisson_end_state"][i, j]).all()
    out, _ = oracle.poisson_stream(42, 20, 100)      # reference test.py:1-11
    assert (out == fx["testpy_poisson20"]).all()


@pytest.mark.parametrize("lam", [1e-3, 0.5, 3.3, 9.999999, 10.0, 10.5, 20, 47.25, 200.0, 1234.5, 1e6])
def test_poisson_vs_numpy(oracle, lam):
    for seed in (7, 99991, 2**33 + 1):
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        exp = np.array([g.poisson(lam) for _ in range(3000)])
        out, st = oracle.poisson_stream(seed, lam, 3000)
        assert np.array_equal(out, exp)
        s = g.bit_generator.state["state"]["state"]
        assert int(st[0]) == s >> 64 and int(st[1]) == s & (2**64 - 1)


def test_seedsequence_vs_numpy(oracle):
    rng = np.random.default_rng(0)
    seeds = [0, 1, 2**32 - 1, 2**32, 2**64 - 1, 2**64, 2**96 + 5, 2**128 - 1]
    seeds += [int(x) for x in rng.integers(0, 2**63, 40)]
    for s in seeds:
        d = np.random.PCG64(np.random.SeedSequence(s)).state["state"]
        st = oracle.pcg64_init(s)
        assert int(st[0]) == d["state"] >> 64 and int(st[1]) == d["state"] & (2**64 - 1)
        assert int(st[2]) == d["inc"] >> 64 and int(st[3]) == d["inc"] & (2**64 - 1)


def test_loggam_known_values(oracle):
    import math
    for x in (1.0, 2.0, 3.0, 6.5, 7.0, 20.0, 101.0, 1e4):
        assert abs(oracle.lib().orc_loggam(x) - math.lgamma(x)) < 1e-9 * max(1, abs(math.lgamma(x)))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_numpy_sum_order(oracle, dtype):
    """numpy add.reduce order (sequential < 8, 8 accumulators <= 128, pairwise split)."""
    rng = np.random.default_rng(1)
    fn = oracle.lib().orc_sum_f32 if dtype == np.float32 else oracle.lib().orc_sum_f64
    for n in list(range(0, 40)) + [127, 128, 129, 200, 300]:
        for _ in range(20):
            a = (rng.standard_normal(n) * 10.0 ** rng.integers(-3, 8, n)).astype(dtype)
            got = fn(oracle._p(a), n)
            assert _bits_equal(np.array(got, dtype), a.sum()), n


def test_numpy_clip_semantics():
    """newsvendor.py:132 clips a Python float with np.clip -> np.float64 (NaN kept)."""
    assert np.isnan(np.clip(float("nan"), 0, 2000))
    assert np.clip(float("inf"), 0, 2000) == 2000.0
    assert np.signbit(np.clip(-0.0, 0, 2000))           # numpy keeps -0.0 (oracle/kernel do too)
    assert np.clip(-5e-324, 0, 2000) == 0.0 and not np.signbit(np.clip(-5e-324, 0, 2000))


# ---------------------------------------------------------------- envs vs goldens
def drive(env, fx, cfg):
    n, n_ep, L = cfg["n_env"], cfg["n_ep"], cfg["ep_len"]
    env.seed([cfg["base_seed"] + i for i in range(n)])
    for ep in range(n_ep):
        o = env.reset()
        assert _bits_equal(o, fx["reset_obs"][:, ep])
        for k in range(L):
            s = ep * L + k
            res = env.step(fx["actions"][:, s])
            assert _bits_equal(res[0], fx["obs"][:, s]), f"obs step {s}"
            assert _bits_equal(res[1], fx["reward"][:, s]), f"reward step {s}"
            assert np.array_equal(res[2], fx["truncated"][:, s])


@pytest.mark.parametrize("name", NV_GOLDENS)
def test_oracle_newsvendor_golden(oracle, name):
    fx, cfg = load_golden(name)
    env = oracle.OracleNewsvendor(cfg["n_env"], **nv_kwargs(cfg))
    drive(env, fx, cfg)
    assert _bits_equal(env.params(), fx["params"][:, -1])


@pytest.mark.parametrize("name", IM_GOLDENS)
def test_oracle_invmgmt_golden(oracle, name):
    fx, cfg = load_golden(name)
    env = oracle.OracleInvMgmt(cfg["n_env"], **im_kwargs(cfg))
    drive(env, fx, cfg)


def test_oracle_invmgmt_info_golden(oracle):
    fx, cfg = load_golden("invmgmt_backlog_default")
    env = oracle.OracleInvMgmt(cfg["n_env"], **im_kwargs(cfg))
    env.seed([cfg["base_seed"] + i for i in range(cfg["n_env"])])
    env.reset()
    for s in range(cfg["ep_len"]):
        _, _, _, info = env.step(fx["actions"][:, s], info=True)
        assert np.array_equal(info["demand"], fx["demand"][:, s])
        assert np.array_equal(info["sales"], fx["sales"][:, s])
        assert np.array_equal(info["unfulfilled"], fx["unfulfilled"][:, s])
        assert np.array_equal(info["ending_inventory"], fx["ending_inventory"][:, s])
        assert np.array_equal(info["backlog_next"], fx["backlog_next"][:, s])


@pytest.mark.parametrize("name", NET_GOLDENS)
def test_oracle_net_golden(oracle, name):
    fx, cfg = load_golden(name)
    g = oracle.custom_graph() if cfg["module"].endswith("custom") else oracle.default_graph()
    env = oracle.OracleNet(cfg["n_env"], graph=g, num_periods=cfg.get("num_periods", 30),
                           backlog=cfg["topology"]["backlog"], alpha=cfg.get("alpha", 1.0))
    assert env.obs_dim == cfg["topology"]["obs_dim"]
    n = cfg["n_env"]
    env.seed([cfg["base_seed"] + i for i in range(n)])
    L = cfg["ep_len"]
    for ep in range(cfg["n_ep"]):
        assert _bits_equal(env.reset(), fx["reset_obs"][:, ep])
        for k in range(L):
            s = ep * L + k
            o, r, tr, info = env.step(fx["actions"][:, s], info=True)
            assert _bits_equal(o, fx["obs"][:, s]) and _bits_equal(r, fx["reward"][:, s])
            for key in ("X", "U", "D", "R", "Y", "P"):
                if key in fx.files:
                    assert _bits_equal(info[key], fx[key][:, s]), (key, s)


def test_golden_coverage_of_quirk_branches():
    """The fixtures reach the reference's edge branches (so parity means something)."""
    fx, _ = load_golden("invmgmt_backlog_default")
    assert (fx["ending_inventory"] < 0).any(), "off-by-one supplier decrement driving I < 0"
    assert (fx["backlog_next"][:, :, 1:] > 10**11).any(), "huge requests -> huge backlog"
    fx, _ = load_golden("newsvendor_capped_L9")
    assert (fx["obs"][:, :, 5:].sum(-1) >= 550).any(), "inventory cap branch (f32 cap) reached"
    fx, _ = load_golden("newsvendor_default")
    assert np.isnan(fx["actions"]).any() and np.isinf(fx["actions"]).any()
    fx, _ = load_golden("net_master_truelost_alpha")
    assert (fx["U"] == 0).all(), "true lost sales keeps U at 0"
    fx, _ = load_golden("net_lostsales_default")
    assert (fx["U"] > 0).any(), "reference LostSales class runs backlog=True"


# ---------------------------------------------------------------- numpy demand samplers (dist 2-4)
def _npg(seed):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


@pytest.mark.parametrize("seed", [0, 7, 123456])
def test_standard_exponential_vs_numpy(oracle, seed):
    a, _ = oracle.exponential_stream(seed, 100000)
    assert np.array_equal(a.view(np.uint64), _npg(seed).standard_exponential(100000).view(np.uint64))


@pytest.mark.parametrize("lo,hi", [(0, 11), (5, 300), (-50, 50), (0, 2**32), (0, 2**32 + 1), (0, 2**40),
                                   (-2**62, 2**62), (3, 4)])
def test_integers_vs_numpy(oracle, lo, hi):
    a, _, _ = oracle.dist_stream(3, 3, 20001, lo, hi)
    g = _npg(3)
    assert np.array_equal(a, np.array([g.integers(lo, hi) for _ in range(20001)]))


@pytest.mark.parametrize("n,p", [(10, 0.5), (100, 0.2), (100, 0.35), (1000, 0.5), (20, 0.9), (1000, 0.97),
                                 (50, 0.01), (5000, 0.3), (7, 1.0), (0, 0.3), (40, 0.0)])
def test_binomial_vs_numpy(oracle, n, p):
    a, _, _ = oracle.dist_stream(11, 2, 20000, n, 0, p)
    g = _npg(11)
    assert np.array_equal(a, np.array([g.binomial(n, p) for _ in range(20000)]))


@pytest.mark.parametrize("p", [1.0, 0.5, 0.34, 1 / 3, 0.3333333333333333, 0.2, 0.05, 0.001, 1e-9])
def test_geometric_vs_numpy(oracle, p):
    a, _, _ = oracle.dist_stream(5, 4, 20000, 0, 0, p)
    g = _npg(5)
    assert np.array_equal(a, np.array([g.geometric(p) for _ in range(20000)]))


@pytest.mark.parametrize("dist,dp", [(2, {"n": 40, "p": 0.5}), (2, {"n": 400, "p": 0.05}),
                                     (3, {"low": 0, "high": 40}), (4, {"p": 0.05}), (4, {"p": 0.5})])
def test_oracle_invmgmt_demand_stream_is_numpys(oracle, dist, dp):
    """The env draws np_random.<sampler>(...) once per step (inventory_management.py:173-182,
    :280): env i's demand sequence is numpy's sequence for seed base + i (the
    32-bit buffer of integers() carried across steps; reset without seed keeps it)."""
    n, base = 6, 321
    orc = oracle.OracleInvMgmt(n, dist=dist, dist_param=dp)
    orc.seed(range(base, base + n))
    orc.reset()
    a = np.full((n, 3), 60, np.int64)
    dem = []
    for ep in range(2):
        if ep:
            orc.reset()
        for _ in range(30):
            dem.append(orc.step(a, info=True)[3]["demand"])
    dem = np.stack(dem, 1)
    for i in range(n):
        g = _npg(base + i)
        if dist == 2:
            e = [g.binomial(dp["n"], dp["p"]) for _ in range(60)]
        elif dist == 3:
            e = [g.integers(dp["low"], dp["high"] + 1) for _ in range(60)]
        else:
            e = [g.geometric(dp["p"]) for _ in range(60)]
        assert np.array_equal(dem[i], np.maximum(np.array(e), 0)), i


@pytest.mark.parametrize("fam", ["nv", "im", "net"])
def test_oracle_thread_count_independent(oracle, fam):
    """The OpenMP env loop (bench.py's multi-core cpu_baseline) gives the same
    trajectories as the single-thread loop."""
    n, T = 301, 12
    outs = []
    for threads in (1, 4):
        oracle.set_threads(threads)
        rng = np.random.default_rng(3)
        if fam == "nv":
            env = oracle.OracleNewsvendor(n)
            acts = [rng.uniform(0, 400, size=n).astype(np.float32) for _ in range(T)]
        elif fam == "im":
            env = oracle.OracleInvMgmt(n, backlog=True)
            acts = [rng.integers(0, 231, size=(n, 3)).astype(np.int64) for _ in range(T)]
        else:
            env = oracle.OracleNet(n)
            acts = [rng.uniform(0, 200, size=(n, 11)).astype(np.float32) for _ in range(T)]
        env.seed(range(5, 5 + n))
        rec = [env.reset()]
        for a in acts:
            rec.extend(np.asarray(x).copy() for x in env.step(a)[:3])
        outs.append(rec)
    oracle.set_threads(1)
    for x, y in zip(*outs):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))


@pytest.mark.parametrize("fn,dp", [("binomial", {"n": 40, "p": 0.5}), ("binomial", {"n": 400, "p": 0.05}),
                                   ("integers", {"low": 3, "high": 45}), ("integers", {"low": 25}),
                                   ("geometric", {"p": 0.05}), ("poisson", {"lam": 7.5})])
def test_oracle_net_market_samplers_vs_numpy(oracle, fn, dp):
    """A market link whose demand_dist_func calls np_random.<fn>(**dist_param)
    (network_management.py:257-263): the market draws are the only consumer of
    the env's Generator, so D[t] of env i is numpy's own <fn> stream of seed i
    through max(0, int(round(.)))."""
    from invsim.topology import custom_graph
    g = custom_graph()
    orc = None
    for e in list(g.edges()):
        if "L" not in g.edges[e]:
            g.edges[e]["dist_param"] = dict(dp)
            # the reference's lambda shape for poisson (:125), over the env itself
            # (bound below: the oracle env plays the reference's `self`), a method
            # name otherwise
            g.edges[e]["demand_dist_func"] = (lambda **p: orc.np_random.poisson(**p)) if fn == "poisson" else fn
    n, T = 16, 12
    orc = oracle.OracleNet(n, graph=g, num_periods=T)
    orc.seed(range(100, 100 + n))
    orc.reset()
    D = []
    for _ in range(T):
        _, _, _, info = orc.step(np.full((n, orc.act_dim), 30.0, np.float32), info=True)
        D.append(info["D"])
    D = np.stack(D, 1)                              # [n, T, markets]
    for i in range(n):
        gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(100 + i)))
        exp = [[max(0, int(round(getattr(gen, fn)(**dp)))) for _ in range(3)] for _ in range(T)]
        assert np.array_equal(D[i], np.array(exp, np.float64)), (fn, i)
