"""Supply-network topology compiler for NetInvMgmt (host side).

Turns a networkx ``DiGraph`` (or the reference's default/custom graphs) into
the index tables the HIP kernel walks.  Every ordering rule of the reference
is reproduced because float sums and sequential inventory consumption depend
on it (network_management.py:146-195):

* main nodes  = sorted(distributors + factories)                        (:176)
* reorder links = sorted(edges with an 'L' attribute)   -> action order (:179)
* retail links  = edges without 'L' in graph.edges() insertion order    (:158)
* successor / predecessor lists in graph adjacency (insertion) order    (:518, :582-609)
* market = no successors, rawmat = no predecessors, factory = has 'C',
  distributor = has 'I0', no 'C', not rawmat, retail = distributor with a
  market successor                                                      (:168-174)
"""
from dataclasses import dataclass, field

import numpy as np

from ._capi import NET_TABLE_FIELDS, NetInvMgmtSpec


def default_graph(demand_lam=20):
    """network_management.py:108-139."""
    import networkx as nx
    g = nx.DiGraph()
    g.add_nodes_from([0])                                                   # market
    g.add_nodes_from([1], I0=100, h=0.030)                                  # retailer
    g.add_nodes_from([2], I0=110, h=0.020)                                  # distributors
    g.add_nodes_from([3], I0=80, h=0.015)
    g.add_nodes_from([4], I0=400, C=90, o=0.010, v=1.000, h=0.012)          # manufacturers
    g.add_nodes_from([5], I0=350, C=90, o=0.015, v=1.000, h=0.013)
    g.add_nodes_from([6], I0=380, C=80, o=0.012, v=1.000, h=0.011)
    g.add_nodes_from([7, 8])                                                # raw materials
    g.add_edges_from([
        (1, 0, {"p": 2.000, "b": 0.100, "dist_param": {"lam": demand_lam}}),
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


def custom_graph(demand_lam=20):
    """network_management_custom.py:108-139 (3 retailers, 1 distributor, 1 factory)."""
    import networkx as nx
    g = nx.DiGraph()
    g.add_nodes_from([0])
    g.add_nodes_from([1, 2, 3], I0=120, h=0.200)
    g.add_nodes_from([4], I0=900, h=0.200)
    g.add_nodes_from([5], I0=1200, C=80, o=0.012, v=1.000, h=0.100)
    g.add_nodes_from([6])
    g.add_edges_from([
        (1, 0, {"p": 25.000, "b": 0.200, "dist_param": {"lam": demand_lam}}),
        (2, 0, {"p": 25.000, "b": 0.200, "dist_param": {"lam": demand_lam}}),
        (3, 0, {"p": 25.000, "b": 0.200, "dist_param": {"lam": demand_lam}}),
        (4, 1, {"L": 1, "p": 5.500, "g": 0.010}),
        (4, 2, {"L": 1, "p": 5.500, "g": 0.010}),
        (4, 3, {"L": 1, "p": 5.500, "g": 0.010}),
        (5, 4, {"L": 1, "p": 1.2, "g": 0.015}),
        (6, 5, {"L": 0, "p": 0.500, "g": 0.000})])
    return g


MARKET_SAMPLERS = {"poisson": 1, "binomial": 2, "integers": 3, "geometric": 4}


def market_sampler(attrs):
    """Demand source of a market link -> (kind, lam, n_or_low, high, p).

    The reference stores a sampler lambda, `demand_dist_func`, called with
    `dist_param` (network_management.py:125-127, 257-263): numpy poisson in its
    own graphs, any np_random method in a user's.  The device runs numpy's
    poisson, binomial, integers and geometric samplers, so the method is read
    from `demand_dist_func` -- a method name, or the name the lambda's code
    references (`lambda **p: self.np_random.binomial(**p)`) -- else from the
    keys of `dist_param`: {lam} poisson, {n, p} binomial, {low[, high]}
    integers, {p} geometric.  integers(low, high) draws [low, high), and
    integers(low) [0, low), as numpy's Generator.integers."""
    f = attrs.get("demand_dist_func")
    name = f if isinstance(f, str) else None
    if name is None and f is not None:
        hit = set(MARKET_SAMPLERS) & set(getattr(getattr(f, "__code__", None), "co_names", ()))
        if len(hit) != 1:
            raise ValueError(f"demand_dist_func must call one of np_random.{sorted(MARKET_SAMPLERS)}")
        name = hit.pop()
    dp = dict(attrs.get("dist_param", {}))
    if name is None:
        keys = set(dp)
        name = ("poisson" if keys <= {"lam"} else "binomial" if keys == {"n", "p"} else
                "integers" if keys in ({"low"}, {"low", "high"}) else "geometric" if keys == {"p"} else None)
    if name not in MARKET_SAMPLERS:
        raise ValueError(f"unsupported market demand source: {name!r} with dist_param {dp}")
    try:
        if name == "poisson":
            return 1, float(dp.get("lam", 1.0)), 0, 0, 0.0
        if name == "binomial":
            return 2, 0.0, int(dp["n"]), 0, float(dp["p"])
        if name == "integers":
            lo, hi = (0, int(dp["low"])) if "high" not in dp else (int(dp["low"]), int(dp["high"]))
            return 3, 0.0, lo, hi, 0.0
        return 4, 0.0, 0, 0, float(dp["p"])
    except KeyError as e:
        raise ValueError(f"{name} market demand needs dist_param {e.args[0]!r}") from None


@dataclass
class Topology:
    main_nodes: list
    reorder_links: list
    retail_links: list
    network_links: list
    market: list
    rawmat: list
    factory: list
    distrib: list
    retail: list
    lead_times: dict
    num_periods: int
    tables: dict = field(default_factory=dict)

    @property
    def obs_dim(self):
        return len(self.retail_links) + len(self.main_nodes) + sum(self.lead_times.values())

    @property
    def lt_max(self):
        return max(self.lead_times.values()) if self.lead_times else 0

    def spec(self, backlog, alpha):
        """ctypes NetInvMgmtSpec; keep the Topology alive while the spec is used."""
        t = self.tables
        ptrs = [t[k].ctypes.data if t[k] is not None else None for k in NET_TABLE_FIELDS]
        return NetInvMgmtSpec(len(self.main_nodes), len(self.reorder_links), len(self.retail_links),
                              int(self.num_periods), int(bool(backlog)), float(alpha), *ptrs)


def compile_graph(g, num_periods, user_D=None, sample_path=None):
    user_D = user_D or {}
    sample_path = sample_path or {}
    nodes = list(g.nodes())
    market = [j for j in nodes if not list(g.successors(j))]
    rawmat = [j for j in nodes if not list(g.predecessors(j))]
    factory = [j for j in nodes if "C" in g.nodes[j]]
    distrib = [j for j in nodes if "I0" in g.nodes[j] and "C" not in g.nodes[j] and j not in rawmat]
    retail = [j for j in distrib if any(s in market for s in g.successors(j))]
    main = sorted(set(distrib + factory))
    reorder = sorted(e for e in g.edges() if "L" in g.edges[e])
    retail_links = [e for e in g.edges() if "L" not in g.edges[e]]
    network_links = sorted(g.edges())
    mi = {j: i for i, j in enumerate(main)}
    ei = {e: i for i, e in enumerate(reorder)}
    ri = {e: i for i, e in enumerate(retail_links)}
    for s, _ in reorder:
        if s not in mi and s not in rawmat:
            raise ValueError(f"supplier {s} is neither a main node nor a raw material")
    for r, _ in retail_links:
        if r not in mi:
            raise ValueError(f"retail link source {r} must be a main (inventory) node")
    nattr = lambda j, k, d=0.0: g.nodes[j].get(k, d)  # noqa: E731
    T = int(num_periods)
    t = {
        "I0": np.array([nattr(j, "I0") for j in main], np.float64),
        "h": np.array([nattr(j, "h") for j in main], np.float64),
        "C": np.array([nattr(j, "C") for j in main], np.float64),
        "o": np.array([nattr(j, "o") for j in main], np.float64),
        "v": np.array([nattr(j, "v", 1.0) for j in main], np.float64),
        "is_factory": np.array([j in factory for j in main], np.int32),
        "is_retail": np.array([j in retail for j in main], np.int32),
        "sup": np.array([mi.get(s, -1) if s not in rawmat else -1 for s, _ in reorder], np.int32),
        "pur": np.array([mi[p] for _, p in reorder], np.int32),
        "sup_is_factory": np.array([s in factory for s, _ in reorder], np.int32),
        "L": np.array([g.edges[e]["L"] for e in reorder], np.int32),
        "lp": np.array([g.edges[e]["p"] for e in reorder], np.float64),
        "lg": np.array([g.edges[e]["g"] for e in reorder], np.float64),
        "rl_node": np.array([mi[r] for r, _ in retail_links], np.int32),
        "rl_p": np.array([g.edges[e]["p"] for e in retail_links], np.float64),
        "rl_b": np.array([g.edges[e]["b"] for e in retail_links], np.float64),
    }
    # demand source per market link (network_management.py:240-267)
    lam = np.zeros(len(retail_links), np.float64)
    use = np.zeros(len(retail_links), np.int32)
    kind = np.ones(max(len(retail_links), 1), np.int32)
    n_lo = np.zeros(max(len(retail_links), 1), np.int64)
    high = np.zeros(max(len(retail_links), 1), np.int64)
    prob = np.zeros(max(len(retail_links), 1), np.float64)
    uD = np.zeros((max(len(retail_links), 1), T), np.float64)
    for e, r in ri.items():
        attrs = g.edges[e]
        d = user_D.get(e, attrs.get("user_D"))
        sp = sample_path.get(e, attrs.get("sample_path", False))
        if d is not None and np.sum(d) > 0 and not sp:
            d = np.asarray(d, np.float64)
            if len(d) != T:
                raise ValueError(f"Edge {e}: user_D length {len(d)} != num_periods {T}")
            uD[r] = d
            use[r] = 1
        else:
            kind[r], lam[r], n_lo[r], high[r], prob[r] = market_sampler(attrs)
    t["rl_lam"], t["rl_user"], t["user_D"] = lam, use, uD
    t["rl_dist"], t["rl_n"], t["rl_high"], t["rl_dp"] = kind, n_lo, high, prob
    sp_, sk, sx, pp, px = [0], [], [], [0], []
    for j in main:
        for k in g.successors(j):
            e = (j, k)
            sk.append(0 if e in ei else 1)
            sx.append(ei[e] if e in ei else ri[e])
        sp_.append(len(sk))
        for k in g.predecessors(j):
            if (k, j) in ei:
                px.append(ei[(k, j)])
        pp.append(len(px))
    t["succ_ptr"] = np.array(sp_, np.int32)
    t["succ_kind"] = np.array(sk or [0], np.int32)
    t["succ_idx"] = np.array(sx or [0], np.int32)
    t["pred_ptr"] = np.array(pp, np.int32)
    t["pred_idx"] = np.array(px or [0], np.int32)
    for k, v in t.items():
        t[k] = np.ascontiguousarray(v) if v.size else np.zeros(1, v.dtype)
    return Topology(main, reorder, retail_links, network_links, market, rawmat, factory, distrib,
                    retail, {e: int(g.edges[e]["L"]) for e in reorder}, T, t)
