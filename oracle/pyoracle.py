"""ctypes front-end of the CPU oracle (test infrastructure only).

ONLY tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg may import this module.  The product package never does.

Classes mirror the reference env classes batch-wise (one oracle env per
instance, stepped in a C loop):

* ``OracleNewsvendor``  <- newsvendor.py:13-230
* ``OracleInvMgmt``     <- inventory_management.py:19-451
* ``OracleNet``         <- network_management.py:26-770 (graph classification
  restated in :func:`net_tables` from :146-195)

Seeding follows gymnasium.utils.seeding.np_random -> numpy SeedSequence(seed):
integer seeds are split into little-endian 32-bit entropy words
(numpy ``_coerce_to_uint32_array``), at most 4 words (seeds < 2**128).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
MAXADJ = 16


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _lib():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    lib.orc_seed_pcg64.argtypes = [P, C.c_int, P]
    lib.orc_next64.argtypes = [P]
    lib.orc_next64.restype = C.c_uint64
    lib.orc_next_double.argtypes = [P]
    lib.orc_next_double.restype = C.c_double
    lib.orc_poisson.argtypes = [P, C.c_double]
    lib.orc_poisson.restype = C.c_int64
    lib.orc_poisson_fill.argtypes = [P, C.c_double, P, C.c_int64]
    lib.orc_dist_fill.argtypes = [P, P, C.c_int, C.c_int64, C.c_int64, C.c_double, P, C.c_int64]
    lib.orc_exponential_fill.argtypes = [P, P, C.c_int64]
    lib.orc_exponential_fill.restype = C.c_double
    lib.orc_loggam.argtypes = [C.c_double]
    lib.orc_loggam.restype = C.c_double
    lib.orc_sum_f32.argtypes = [P, C.c_int64]
    lib.orc_sum_f32.restype = C.c_float
    lib.orc_sum_f64.argtypes = [P, C.c_int64]
    lib.orc_sum_f64.restype = C.c_double
    lib.orc_set_threads.argtypes = [C.c_int]
    lib.orc_max_threads.restype = C.c_int
    for fam in ("nv", "im", "net"):
        getattr(lib, f"orc_{fam}_create").argtypes = [P, C.c_int64]
        getattr(lib, f"orc_{fam}_create").restype = P
        getattr(lib, f"orc_{fam}_destroy").argtypes = [P]
        getattr(lib, f"orc_{fam}_seed").argtypes = [P, P, P]
        getattr(lib, f"orc_{fam}_reset").argtypes = [P, P]
        getattr(lib, f"orc_{fam}_rng").argtypes = [P, P]
    lib.orc_nv_step.argtypes = [P] * 6
    lib.orc_nv_get_params.argtypes = [P, P]
    lib.orc_im_step.argtypes = [P] * 10
    lib.orc_net_step.argtypes = [P] * 12
    lib.orc_net_obs_dim.argtypes = [P]
    lib.orc_net_obs_dim.restype = C.c_int32
    return lib


LIB = None


def set_threads(n):
    """Threads of the oracle's env-parallel batch loops (OpenMP; default 1)."""
    lib().orc_set_threads(int(n))


def max_threads():
    return int(lib().orc_max_threads())


def lib():
    global LIB
    if LIB is None:
        LIB = _lib()
    return LIB


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def seed_words(seeds):
    """Python-int seeds -> (words uint32[n,4], nwords int32[n]) as numpy SeedSequence sees them."""
    seeds = list(seeds)
    words = np.zeros((len(seeds), 4), np.uint32)
    nw = np.zeros(len(seeds), np.int32)
    for i, s in enumerate(seeds):
        s = int(s)
        if s < 0 or s >= 2**128:
            raise ValueError("seed must be in [0, 2**128)")
        k = 0
        while True:
            words[i, k] = s & 0xFFFFFFFF
            k += 1
            s >>= 32
            if s == 0:
                break
        nw[i] = k
    return words, nw


# ---------------------------------------------------------------- RNG helpers
def pcg64_init(seed):
    w, n = seed_words([seed])
    st = np.zeros(4, np.uint64)
    lib().orc_seed_pcg64(_p(w[0]), int(n[0]), _p(st))
    return st


def poisson_stream(seed, lam, n):
    st = pcg64_init(seed)
    out = np.zeros(n, np.int64)
    lib().orc_poisson_fill(_p(st), float(lam), _p(out), n)
    return out, st


def dist_stream(seed, dist, n, n_or_low=0, high=0, p=0.0):
    """numpy Generator(PCG64(seed)) draws: dist 2 binomial(n_or_low, p),
    3 integers(n_or_low, high), 4 geometric(p).  Returns (draws, state, buf)."""
    st = pcg64_init(seed)
    buf = np.zeros(2, np.uint32)
    out = np.zeros(n, np.int64)
    lib().orc_dist_fill(_p(st), _p(buf), int(dist), int(n_or_low), int(high), float(p), _p(out), n)
    return out, st, buf


def exponential_stream(seed, n):
    st = pcg64_init(seed)
    out = np.zeros(n, np.float64)
    lib().orc_exponential_fill(_p(st), _p(out), n)
    return out, st


# ---------------------------------------------------------------- structs
class NVCfg(C.Structure):
    _fields_ = [("lead_time", C.c_int32), ("step_limit", C.c_int32),
                ("max_inventory", C.c_double), ("max_order_quantity", C.c_double),
                ("p_max", C.c_double), ("h_max", C.c_double), ("k_max", C.c_double),
                ("mu_max", C.c_double)]


class IMCfg(C.Structure):
    _fields_ = [("num_stages", C.c_int32), ("periods", C.c_int32), ("backlog", C.c_int32),
                ("dist", C.c_int32), ("mu", C.c_double), ("alpha", C.c_double),
                ("I0", C.c_void_p), ("unit_price", C.c_void_p), ("unit_cost", C.c_void_p),
                ("demand_cost", C.c_void_p), ("holding_cost", C.c_void_p),
                ("supply_capacity", C.c_void_p), ("lead_time", C.c_void_p), ("user_D", C.c_void_p),
                ("dist_n", C.c_int64), ("dist_p", C.c_double), ("dist_low", C.c_int64), ("dist_high", C.c_int64)]


class NetCfg(C.Structure):
    _fields_ = [("J", C.c_int32), ("E", C.c_int32), ("RL", C.c_int32), ("num_periods", C.c_int32),
                ("backlog", C.c_int32), ("alpha", C.c_double)] + [
        (n, C.c_void_p) for n in ("I0", "h", "C", "o", "v", "is_factory", "is_retail", "sup", "pur",
                                  "L", "sup_is_factory", "lp", "lg", "rl_node", "rl_p", "rl_b",
                                  "rl_lam", "rl_user", "user_D", "succ_n", "succ_kind", "succ_idx",
                                  "pred_n", "pred_idx", "rl_dist", "rl_n", "rl_high", "rl_dp")]


class _Base:
    fam = None

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            getattr(lib(), f"orc_{self.fam}_destroy")(h)
            self.h = None

    def seed(self, seeds):
        w, nw = seed_words(seeds)
        assert len(w) == self.n
        getattr(lib(), f"orc_{self.fam}_seed")(self.h, _p(w), _p(nw))

    def rng_state(self):
        """[n][4] uint64 (state hi, state lo, inc hi, inc lo) of every env's PCG64."""
        out = np.zeros((self.n, 4), np.uint64)
        getattr(lib(), f"orc_{self.fam}_rng")(self.h, _p(out))
        return out

    _NULLS = {"nv": 1, "im": 5, "net": 7}

    def run_returns(self, action_pool, T, ret=None):
        """T steps under NEXT_STEP autoreset (the call after a truncation is a
        reset: reward 0, no step), call k taking action_pool[k % P], without
        observations.  Returns (per-env sum of rewards added in call order,
        f64; truncations seen).  The env must be freshly reset."""
        n = self.n
        pool = [np.ascontiguousarray(a) for a in action_pool]
        rew = np.zeros(n, np.float64)
        tr = np.zeros(n, np.uint8)
        ret = np.zeros(n, np.float64) if ret is None else ret
        zero = np.zeros(n, np.float64)
        f = getattr(lib(), f"orc_{self.fam}_step")
        nulls = [None] * self._NULLS[self.fam]
        pending, ntr = False, 0
        for k in range(T):
            if pending:
                getattr(lib(), f"orc_{self.fam}_reset")(self.h, None)
                ret += zero
                pending = False
                continue
            f(self.h, _p(pool[k % len(pool)]), None, _p(rew), _p(tr), *nulls)
            ret += rew
            if tr.any():
                assert tr.all(), "lock-step episodes"
                pending, ntr = True, ntr + 1
        return ret, ntr


# ---------------------------------------------------------------- Newsvendor
class OracleNewsvendor(_Base):
    """newsvendor.py:52-97 constructor defaults."""
    fam = "nv"

    def __init__(self, n, lead_time=5, max_inventory=4000, max_order_quantity=2000, step_limit=40,
                 p_max=100.0, h_max=5.0, k_max=10.0, mu_max=200.0, gamma=1.0):
        self.n = n
        self.L = max(0, int(lead_time))
        self.obs_dim = self.L + 5
        self.cfg = NVCfg(int(lead_time), int(step_limit), float(max_inventory),
                         float(max_order_quantity), float(p_max), float(h_max), float(k_max),
                         float(mu_max))
        self.h = lib().orc_nv_create(C.byref(self.cfg), n)

    def reset(self):
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        lib().orc_nv_reset(self.h, _p(obs))
        return obs

    def step(self, action):
        action = np.ascontiguousarray(np.asarray(action, np.float32).reshape(self.n))
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        rew = np.zeros(self.n, np.float64)
        tr = np.zeros(self.n, np.uint8)
        dem = np.zeros(self.n, np.int64)
        lib().orc_nv_step(self.h, _p(action), _p(obs), _p(rew), _p(tr), _p(dem))
        return obs, rew, tr.astype(bool), dem

    def params(self):
        p = np.zeros((self.n, 5), np.float64)
        lib().orc_nv_get_params(self.h, _p(p))
        return p


# ---------------------------------------------------------------- InvMgmt
class OracleInvMgmt(_Base):
    """inventory_management.py:48-141 parameter processing restated."""
    fam = "im"

    def __init__(self, n, periods=30, I0=(100, 150, 200), p=20, r=(15, 10, 7, 5),
                 k=(0.10, 0.075, 0.05, 0.025), h=(0.15, 0.10, 0.05), c=(100, 200, 230),
                 L=(1, 5, 10), backlog=True, dist=1, dist_param=None, alpha=0.97, user_D=None,
                 env_config=None, **_ignored):
        kw = dict(periods=periods, I0=I0, p=p, r=r, k=k, h=h, c=c, L=L, backlog=backlog, dist=dist,
                  dist_param=dist_param if dist_param is not None else {"mu": 20}, alpha=alpha,
                  user_D=user_D)
        if env_config:
            kw.update(env_config)                                   # :83-84
        self.n = n
        self.m = len(kw["I0"]) + 1
        self._keep = dict(
            I0=np.array(list(kw["I0"]), np.int32).astype(np.int64),
            up=np.append(kw["p"], kw["r"][:-1]).astype(np.float32),   # :89
            uc=np.array(kw["r"], np.float32),
            kc=np.array(kw["k"], np.float32),
            hc=np.append(kw["h"], 0).astype(np.float32),
            c=np.array(list(kw["c"]), np.int64),
            L=np.array(list(kw["L"]), np.int64),
            uD=np.array(list(kw["user_D"] or [0] * kw["periods"]), np.int64))
        self.lt_max = int(self._keep["L"].max()) if self.m > 1 else 0
        self.obs_dim = (self.m - 1) * (self.lt_max + 1)
        self.periods = int(kw["periods"])
        dp, dist = kw["dist_param"], kw["dist"]
        mu = float(dp.get("mu", 0)) if dist == 1 else 0.0
        k = self._keep
        self.cfg = IMCfg(self.m, int(kw["periods"]), int(bool(kw["backlog"])), int(dist), mu,
                         float(kw["alpha"]), _p(k["I0"]).value, _p(k["up"]).value,
                         _p(k["uc"]).value, _p(k["kc"]).value, _p(k["hc"]).value,
                         _p(k["c"]).value, _p(k["L"]).value, _p(k["uD"]).value,
                         int(dp["n"]) if dist == 2 else 0, float(dp["p"]) if dist in (2, 4) else 0.0,
                         int(dp["low"]) if dist == 3 else 0, int(dp["high"]) if dist == 3 else 0)
        self.h = lib().orc_im_create(C.byref(self.cfg), n)

    def reset(self):
        obs = np.zeros((self.n, self.obs_dim), np.int64)
        lib().orc_im_reset(self.h, _p(obs))
        return obs

    def step(self, action, info=False):
        action = np.ascontiguousarray(np.asarray(action, np.int64).reshape(self.n, self.m - 1))
        obs = np.zeros((self.n, self.obs_dim), np.int64)
        rew = np.zeros(self.n, np.float64)
        tr = np.zeros(self.n, np.uint8)
        if not info:
            lib().orc_im_step(self.h, _p(action), _p(obs), _p(rew), _p(tr), *([None] * 5))
            return obs, rew, tr.astype(bool)
        m = self.m
        d = np.zeros(self.n, np.int64)
        S = np.zeros((self.n, m), np.int64)
        U = np.zeros((self.n, m), np.int64)
        Ie = np.zeros((self.n, m - 1), np.int64)
        B = np.zeros((self.n, m), np.int64)
        lib().orc_im_step(self.h, _p(action), _p(obs), _p(rew), _p(tr), _p(d), _p(S), _p(U),
                          _p(Ie), _p(B))
        return obs, rew, tr.astype(bool), dict(demand=d, sales=S, unfulfilled=U,
                                               ending_inventory=Ie, backlog_next=B)


# ---------------------------------------------------------------- NetInvMgmt
def default_graph():
    """network_management.py:108-139 default topology; the market's
    `lambda **p: self.np_random.poisson(**p)` (:125) is named by its method."""
    import networkx as nx
    g = nx.DiGraph()
    g.add_nodes_from([0])
    g.add_nodes_from([1], I0=100, h=0.030)
    g.add_nodes_from([2], I0=110, h=0.020)
    g.add_nodes_from([3], I0=80, h=0.015)
    g.add_nodes_from([4], I0=400, C=90, o=0.010, v=1.000, h=0.012)
    g.add_nodes_from([5], I0=350, C=90, o=0.015, v=1.000, h=0.013)
    g.add_nodes_from([6], I0=380, C=80, o=0.012, v=1.000, h=0.011)
    g.add_nodes_from([7, 8])
    g.add_edges_from([
        (1, 0, {"p": 2.000, "b": 0.100, "demand_dist_func": "poisson", "dist_param": {"lam": 20}}),
        (2, 1, {"L": 5, "p": 1.500, "g": 0.010}),
        (3, 1, {"L": 3, "p": 1.600, "g": 0.015}),
        (4, 2, {"L": 8, "p": 1.000, "g": 0.008}),
        (4, 3, {"L": 10, "p": 0.800, "g": 0.006}),
        (5, 2, {"L": 9, "p": 0.700, "g": 0.005}),
        (6, 2, {"L": 11, "p": 0.750, "g": 0.007}),
        (6, 3, {"L": 12, "p": 0.800, "g": 0.004}),
        (7, 4, {"L": 0, "p": 0.150, "g": 0.000}),
        (7, 5, {"L": 1, "p": 0.050, "g": 0.005}),
        (8, 5, {"L": 2, "p": 0.070, "g": 0.002}),
        (8, 6, {"L": 0, "p": 0.200, "g": 0.000})])
    return g


def custom_graph():
    """network_management_custom.py:108-139 topology."""
    import networkx as nx
    g = nx.DiGraph()
    g.add_nodes_from([0])
    g.add_nodes_from([1, 2, 3], I0=120, h=0.200)
    g.add_nodes_from([4], I0=900, h=0.200)
    g.add_nodes_from([5], I0=1200, C=80, o=0.012, v=1.000, h=0.100)
    g.add_nodes_from([6])
    g.add_edges_from([
        (1, 0, {"p": 25.000, "b": 0.200, "demand_dist_func": "poisson", "dist_param": {"lam": 20}}),
        (2, 0, {"p": 25.000, "b": 0.200, "demand_dist_func": "poisson", "dist_param": {"lam": 20}}),
        (3, 0, {"p": 25.000, "b": 0.200, "demand_dist_func": "poisson", "dist_param": {"lam": 20}}),
        (4, 1, {"L": 1, "p": 5.500, "g": 0.010}),
        (4, 2, {"L": 1, "p": 5.500, "g": 0.010}),
        (4, 3, {"L": 1, "p": 5.500, "g": 0.010}),
        (5, 4, {"L": 1, "p": 1.2, "g": 0.015}),
        (6, 5, {"L": 0, "p": 0.500, "g": 0.000})])
    return g


def market_sampler(attrs):
    """(kind, lam, n_or_low, high, p) of a market link's demand source
    (network_management.py:257-267): only an edge with BOTH `demand_dist_func`
    and `dist_param` draws, `demand_dist_func(**dist_param)`; any other market
    has demand 0 and makes no draw, which is kind 1 with lam 0 (numpy's
    poisson(0) returns 0 without consuming a uniform).  The method is a
    string, a Generator's bound method, or the method name in the reference's
    lambda (`self.np_random.<method>(**p)`, read from its code names); kind 1
    poisson (numpy default lam 1.0), 2 binomial, 3 integers [low, high), 4
    geometric."""
    if "demand_dist_func" not in attrs or "dist_param" not in attrs:
        return 1, 0.0, 0, 0, 0.0
    f = attrs["demand_dist_func"]
    names = {"poisson", "binomial", "integers", "geometric"}
    if isinstance(f, str):
        name = f
    elif hasattr(f, "__self__"):
        name = f.__name__
    else:
        co = getattr(getattr(f, "__code__", None), "co_names", ())
        hit = names & set(co)
        name = hit.pop() if len(hit) == 1 and "np_random" in co else None
    dp = dict(attrs["dist_param"])
    if name == "poisson":
        return 1, float(dp.get("lam", 1.0)), 0, 0, 0.0
    if name == "binomial":
        return 2, 0.0, int(dp["n"]), 0, float(dp["p"])
    if name == "integers":
        lo, hi = (0, int(dp["low"])) if "high" not in dp else (int(dp["low"]), int(dp["high"]))
        return 3, 0.0, lo, hi, 0.0
    if name == "geometric":
        return 4, 0.0, 0, 0, float(dp["p"])
    raise ValueError(f"unsupported market demand source {attrs!r}")


def net_tables(g, num_periods, user_D=None, sample_path=None):
    """Restates network_management.py:146-195 (node/link classification and
    ordering) and the market demand sources of :149-163, :246-267: a link in
    `user_D` with a positive sum and sample_path False replays it, every other
    market link takes `market_sampler`."""
    nodes = list(g.nodes())
    market = [j for j in nodes if not list(g.successors(j))]
    rawmat = [j for j in nodes if not list(g.predecessors(j))]
    factory = [j for j in nodes if "C" in g.nodes[j]]
    distrib = [j for j in nodes if "I0" in g.nodes[j] and "C" not in g.nodes[j] and j not in rawmat]
    retail = [j for j in distrib if any(s in market for s in g.successors(j))]
    main = sorted(set(distrib + factory))
    reorder = sorted([e for e in g.edges() if "L" in g.edges[e]])
    retail_links = [e for e in g.edges() if "L" not in g.edges[e]]
    mi = {j: i for i, j in enumerate(main)}
    ei = {e: i for i, e in enumerate(reorder)}
    ri = {e: i for i, e in enumerate(retail_links)}
    J, E, RL = len(main), len(reorder), len(retail_links)
    t = {}
    t["I0"] = np.array([g.nodes[j].get("I0", 0) for j in main], np.float64)
    t["h"] = np.array([g.nodes[j].get("h", 0) for j in main], np.float64)
    t["C"] = np.array([g.nodes[j].get("C", 0) for j in main], np.float64)
    t["o"] = np.array([g.nodes[j].get("o", 0) for j in main], np.float64)
    t["v"] = np.array([g.nodes[j].get("v", 1.0) for j in main], np.float64)
    t["is_factory"] = np.array([j in factory for j in main], np.int32)
    t["is_retail"] = np.array([j in retail for j in main], np.int32)
    t["sup"] = np.array([mi[s] if s not in rawmat else -1 for s, _ in reorder], np.int32)
    t["pur"] = np.array([mi[p] for _, p in reorder], np.int32)
    t["L"] = np.array([g.edges[e]["L"] for e in reorder], np.int32)
    t["sup_is_factory"] = np.array([s in factory for s, _ in reorder], np.int32)
    t["lp"] = np.array([g.edges[e]["p"] for e in reorder], np.float64)
    t["lg"] = np.array([g.edges[e]["g"] for e in reorder], np.float64)
    t["rl_node"] = np.array([mi[r] for r, _ in retail_links], np.int32)
    t["rl_p"] = np.array([g.edges[e]["p"] for e in retail_links], np.float64)
    t["rl_b"] = np.array([g.edges[e]["b"] for e in retail_links], np.float64)
    ms = [market_sampler(g.edges[e]) for e in retail_links]
    t["rl_lam"] = np.array([m[1] for m in ms], np.float64)
    t["rl_dist"] = np.array([m[0] for m in ms] or [1], np.int32)
    t["rl_n"] = np.array([m[2] for m in ms] or [0], np.int64)
    t["rl_high"] = np.array([m[3] for m in ms] or [0], np.int64)
    t["rl_dp"] = np.array([m[4] for m in ms] or [0.0], np.float64)
    uD = np.zeros((max(RL, 1), num_periods), np.float64)
    rl_user = np.zeros(max(RL, 1), np.int32)
    for e, r in ri.items():
        if e in (user_D or {}):
            d, sp = user_D[e], (sample_path or {}).get(e, False)
        else:
            d, sp = g.edges[e].get("user_D", ()), g.edges[e].get("sample_path", False)
        if len(d) and np.sum(d) > 0 and not sp:
            uD[r] = np.asarray(d, np.float64)
            rl_user[r] = 1
    t["rl_user"], t["user_D"] = rl_user, uD
    sn = np.zeros(J, np.int32)
    sk = np.zeros((J, MAXADJ), np.int32)
    sx = np.zeros((J, MAXADJ), np.int32)
    pn = np.zeros(J, np.int32)
    px = np.zeros((J, MAXADJ), np.int32)
    for j in main:
        a = mi[j]
        for k in g.successors(j):
            e = (j, k)
            sk[a, sn[a]], sx[a, sn[a]] = (0, ei[e]) if e in ei else (1, ri[e])
            sn[a] += 1
        for k in g.predecessors(j):
            e = (k, j)
            if e in ei:
                px[a, pn[a]] = ei[e]
                pn[a] += 1
    t.update(succ_n=sn, succ_kind=sk, succ_idx=sx, pred_n=pn, pred_idx=px)
    return dict(J=J, E=E, RL=RL, tables=t, main=main, reorder=reorder, retail_links=retail_links)


class OracleNet(_Base):
    """NetInvMgmtMasterEnv(graph, num_periods, backlog, alpha).  NOTE the reference
    NetInvMgmtLostSalesEnv runs with backlog=True (network_management.py:83-85 vs :755-761):
    callers pass the *effective* backlog flag here."""
    fam = "net"

    def __init__(self, n, graph=None, num_periods=30, backlog=True, alpha=1.0, user_D=None, sample_path=None):
        if graph is None:
            graph = default_graph()
        self.n = n
        self.topo = net_tables(graph, num_periods, user_D, sample_path)
        self._t = {k: np.ascontiguousarray(v) for k, v in self.topo["tables"].items()}
        t = self._t
        self.cfg = NetCfg(self.topo["J"], self.topo["E"], self.topo["RL"], int(num_periods),
                          int(bool(backlog)), float(alpha),
                          *[_p(t[k]).value for k in ("I0", "h", "C", "o", "v", "is_factory",
                                                     "is_retail", "sup", "pur", "L", "sup_is_factory",
                                                     "lp", "lg", "rl_node", "rl_p", "rl_b", "rl_lam",
                                                     "rl_user", "user_D", "succ_n", "succ_kind",
                                                     "succ_idx", "pred_n", "pred_idx", "rl_dist", "rl_n",
                                                     "rl_high", "rl_dp")])
        self.h = lib().orc_net_create(C.byref(self.cfg), n)
        self.obs_dim = int(lib().orc_net_obs_dim(self.h))
        self.act_dim = self.topo["E"]

    def reset(self):
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        lib().orc_net_reset(self.h, _p(obs))
        return obs

    def step(self, action, info=False):
        action = np.ascontiguousarray(np.asarray(action, np.float32).reshape(self.n, self.act_dim))
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        rew = np.zeros(self.n, np.float64)
        tr = np.zeros(self.n, np.uint8)
        if not info:
            lib().orc_net_step(self.h, _p(action), _p(obs), _p(rew), _p(tr), *([None] * 7))
            return obs, rew, tr.astype(bool)
        J, E, RL = self.topo["J"], self.topo["E"], self.topo["RL"]
        X = np.zeros((self.n, J)); U = np.zeros((self.n, RL)); D = np.zeros((self.n, RL))
        R = np.zeros((self.n, E)); Y = np.zeros((self.n, E)); P = np.zeros((self.n, J))
        S = np.zeros((self.n, RL))
        lib().orc_net_step(self.h, _p(action), _p(obs), _p(rew), _p(tr), _p(X), _p(U), _p(D), _p(R),
                           _p(Y), _p(P), _p(S))
        return obs, rew, tr.astype(bool), dict(X=X, U=U, D=D, R=R, Y=Y, P=P, S=S)
