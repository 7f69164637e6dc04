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
        (1, 0, {"p": 2.000, "b": 0.100, "demand_dist_func": "poisson", "dist_param": {"lam": demand_lam}}),
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
        (1, 0, {"p": 25.000, "b": 0.200, "demand_dist_func": "poisson", "dist_param": {"lam": demand_lam}}),
        (2, 0, {"p": 25.000, "b": 0.200, "demand_dist_func": "poisson", "dist_param": {"lam": demand_lam}}),
        (3, 0, {"p": 25.000, "b": 0.200, "demand_dist_func": "poisson", "dist_param": {"lam": demand_lam}}),
        (4, 1, {"L": 1, "p": 5.500, "g": 0.010}),
        (4, 2, {"L": 1, "p": 5.500, "g": 0.010}),
        (4, 3, {"L": 1, "p": 5.500, "g": 0.010}),
        (5, 4, {"L": 1, "p": 1.2, "g": 0.015}),
        (6, 5, {"L": 0, "p": 0.500, "g": 0.000})])
    return g


MARKET_SAMPLERS = {"poisson": 1, "binomial": 2, "integers": 3, "geometric": 4}
# the keyword arguments each numpy Generator method takes here (dist_param keys)
SAMPLER_KWARGS = {"poisson": {"lam"}, "binomial": {"n", "p"}, "integers": {"low", "high"}, "geometric": {"p"}}
# demand 0 without a draw: numpy's poisson(0) returns 0 and consumes no uniform,
# which is the reference's `lambda: 0` fallback (network_management.py:264-267)
ZERO_DEMAND = (1, 0.0, 0, 0, 0.0)

_SKIP_OPS = {"RESUME", "COPY_FREE_VARS", "CACHE", "NOP", "PUSH_NULL", "PRECALL", "MAKE_CELL"}


def _lambda_parts(f):
    """(method, receiver opcode, receiver name) of
    ``lambda **p: <receiver>.np_random.<method>(**p)`` (network_management.py:125),
    read from the bytecode; None for any other shape (arithmetic on the draw,
    another generator, positional arguments, ...).  The receiver is a free
    variable (LOAD_DEREF) or a module global (LOAD_GLOBAL): the two ways a
    lambda written outside the env can name it."""
    import dis
    import inspect
    code = getattr(f, "__code__", None)
    if code is None or code.co_argcount or code.co_kwonlyargcount or code.co_posonlyargcount:
        return None
    if not code.co_flags & inspect.CO_VARKEYWORDS or code.co_flags & inspect.CO_VARARGS:
        return None
    kw = code.co_varnames[0]
    ins = [i for i in dis.get_instructions(f) if i.opname not in _SKIP_OPS]
    if len(ins) < 5:
        return None
    recv, attr, meth = ins[:3]
    if recv.opname not in ("LOAD_DEREF", "LOAD_GLOBAL"):
        return None
    if attr.opname != "LOAD_ATTR" or attr.argval != "np_random":
        return None
    if meth.opname not in ("LOAD_ATTR", "LOAD_METHOD") or meth.argval not in MARKET_SAMPLERS:
        return None
    calls = kwloads = 0
    for i in ins[3:]:
        if i.opname == "LOAD_FAST" and i.argval == kw:
            kwloads += 1
        elif i.opname in ("CALL_FUNCTION_EX",):
            calls += 1
        elif not ((i.opname == "LOAD_CONST" and i.argval == ()) or (i.opname == "BUILD_TUPLE" and i.arg == 0)
                  or (i.opname == "BUILD_MAP" and i.arg == 0) or i.opname in ("DICT_MERGE", "RETURN_VALUE")):
            return None
    if calls != 1 or kwloads != 1 or ins[-1].opname != "RETURN_VALUE" or ins[-2].opname != "CALL_FUNCTION_EX":
        return None
    return meth.argval, recv.opname, recv.argval


def sampler_method(f):
    """Name of the numpy Generator method a market's ``demand_dist_func`` calls.

    Accepted: a method name (``"poisson"``, the package's own graphs) or the
    reference's lambda shape ``lambda **p: <recv>.np_random.poisson(**p)``
    (network_management.py:125).  The reference calls the lambda as written
    (:263), so it draws from ``<recv>``'s generator: the device can only
    reproduce that when ``<recv>`` is the env itself, which
    ``check_market_receivers`` verifies at every ``reset()`` (the name may be
    bound after the graph is built).  A Generator's bound method
    (``rng.poisson``) is refused: its generator is a host object that is never
    the env's own stream.  Anything else raises: the device cannot run an
    arbitrary Python callable."""
    if isinstance(f, str):
        name = f
    elif getattr(f, "__self__", None) is not None and type(f.__self__).__name__ == "Generator":
        raise ValueError(f"unsupported demand_dist_func {f!r}: a bound method of a host numpy Generator "
                         f"draws from that generator (network_management.py:263), which the device "
                         f"cannot; name the method ('poisson') or use "
                         f"`lambda **p: <env>.np_random.<method>(**p)` over the env itself")
    else:
        parts = _lambda_parts(f)
        name = parts[0] if parts else None
    if name not in MARKET_SAMPLERS:
        raise ValueError(f"unsupported demand_dist_func {f!r}: it must be one of "
                         f"{sorted(MARKET_SAMPLERS)} by name, or "
                         f"`lambda **p: <env>.np_random.<method>(**p)` over the env itself")
    return name


_UNBOUND = object()


def lambda_receiver(f):
    """The object a reference-shape market lambda names as ``<recv>`` in
    ``<recv>.np_random.<method>(**p)``, resolved now, as the reference resolves
    it when it calls the lambda (network_management.py:263); None for a method
    name; ``_UNBOUND`` for a free variable or global with no value yet (or
    None, on which the reference's call raises AttributeError)."""
    if isinstance(f, str):
        return None
    parts = _lambda_parts(f)
    if parts is None:
        raise ValueError(f"unsupported demand_dist_func {f!r}")
    _, op, name = parts
    recv = _UNBOUND
    if op == "LOAD_DEREF":
        code = f.__code__
        if name in code.co_freevars and f.__closure__ is not None:
            try:
                recv = f.__closure__[code.co_freevars.index(name)].cell_contents
            except ValueError:                # empty cell
                pass
    else:
        import builtins
        g = getattr(f, "__globals__", {})
        recv = g[name] if name in g else getattr(builtins, name, _UNBOUND)
    return _UNBOUND if recv is None else recv   # None.np_random: the reference raises


def is_env_receiver(recv, env):
    """True when ``recv`` is ``env`` or a view over it (``invsim.compat``'s
    single-env views keep the vector env as ``_v``; a wrapper may expose it as
    ``unwrapped``)."""
    if recv is env:
        return True
    for attr in ("_v", "unwrapped"):
        try:
            if recv is not None and object.__getattribute__(recv, attr) is env:
                return True
        except AttributeError:
            pass
    return False


def check_market_receivers(g, retail_links, env):
    """network_management.py:257-263: a market whose demand_dist_func is the
    reference's lambda draws from ``<recv>.np_random``.  The device draws every
    market from the env's own per-env stream, so ``<recv>`` must resolve to the
    env: anything else (another object's generator, a name still unbound)
    raises ValueError instead of silently drawing from the wrong stream.
    Markets whose demand is user_D or zero never call the lambda and are not
    checked (:250-255, :264-267)."""
    tabs = env.topology.tables
    for r, e in enumerate(retail_links):
        attrs = g.edges[e]
        if tabs["rl_user"][r] or "demand_dist_func" not in attrs or "dist_param" not in attrs:
            continue
        recv = lambda_receiver(attrs["demand_dist_func"])
        if recv is None:
            continue
        if recv is _UNBOUND:
            raise ValueError(f"market link {e}: the demand_dist_func lambda's receiver is not bound at "
                             f"reset(); bind it to the env before resetting")
        if not is_env_receiver(recv, env):
            raise ValueError(f"market link {e}: demand_dist_func draws from {type(recv).__name__} "
                             f"object's np_random, not this env's; the reference would call that "
                             f"generator (network_management.py:263), the device can only draw from the "
                             f"env's own stream -- bind the lambda to the env")


def market_sampler(attrs):
    """Demand source of a market link -> (kind, lam, n_or_low, high, p).

    network_management.py:257-267: a market draws only if the edge has both
    ``demand_dist_func`` and ``dist_param`` (the sampler is called with
    ``**dist_param``); otherwise its demand is 0 and no draw is made
    (``ZERO_DEMAND``).  The device runs numpy's poisson, binomial, integers and
    geometric samplers; ``integers(low, high)`` draws [low, high) and
    ``integers(low)`` [0, low), as numpy's Generator.integers, and
    ``poisson()`` without ``lam`` is numpy's default lam=1.0."""
    if "demand_dist_func" not in attrs or "dist_param" not in attrs:
        return ZERO_DEMAND
    name = sampler_method(attrs["demand_dist_func"])
    dp = dict(attrs["dist_param"])
    extra = set(dp) - SAMPLER_KWARGS[name]
    if extra:
        raise ValueError(f"{name} market demand: unsupported dist_param keys {sorted(extra)}")
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


def classify(g):
    """network_management.py:158-181: (market, rawmat, factory, distrib, retail,
    main_nodes, reorder_links, retail_links, network_links)."""
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
    return market, rawmat, factory, distrib, retail, main, reorder, retail_links, network_links


def market_demand_attrs(g, e, user_D, sample_path, num_periods):
    """The (user_D, sample_path) a market link carries after the reference's
    `_initialize_graph_dependent_attributes` (network_management.py:149-163):
    an entry of the `user_D` argument overrides the edge's own attribute and
    brings its `sample_path` entry (default False) with it; a market link with
    neither gets zeros(num_periods) and False."""
    if e in user_D:
        d = user_D[e]
        return (list(d) if not isinstance(d, (list, np.ndarray)) else d), sample_path.get(e, False)
    attrs = g.edges[e]
    d = attrs["user_D"] if "user_D" in attrs else np.zeros(num_periods)
    return d, attrs.get("sample_path", False)


def validate_inputs(g, num_periods, user_D=None, sample_path=None):
    """network_management.py:197-233, node then edge attribute checks, with the
    reference's AssertionError messages.  (The scalar checks of :236-238 are the
    env constructor's.)"""
    user_D = user_D or {}
    sample_path = sample_path or {}
    market, rawmat, factory, distrib, _, main, reorder, retail_links, _ = classify(g)
    classified = set(market) | set(distrib) | set(factory) | set(rawmat)
    if set(g.nodes()) != classified:
        print(f"Warning: Some nodes not classified: {set(g.nodes()) - classified}")
    for link in user_D:
        if link not in g.edges:
            print(f"Warning: Link {link} from user_D not found in graph.")
    main_s, factory_s, reorder_s, retail_s = set(main), set(factory), set(reorder), set(retail_links)
    for j in g.nodes():
        attrs = g.nodes[j]
        if j in main_s:
            assert "I0" in attrs and attrs["I0"] >= 0, f"Node {j}: Invalid or missing I0>=0"
            assert "h" in attrs and attrs["h"] >= 0, f"Node {j}: Invalid or missing h>=0"
        if j in factory_s:
            assert "C" in attrs and attrs["C"] > 0, f"Node {j}: Invalid or missing C>0"
            assert "o" in attrs and attrs["o"] >= 0, f"Node {j}: Invalid or missing o>=0"
            assert "v" in attrs and 0 < attrs["v"] <= 1, f"Node {j}: Invalid or missing v in (0, 1]"
    for u, v, attrs in g.edges(data=True):
        edge = (u, v)
        if edge in reorder_s:
            assert "L" in attrs and attrs["L"] >= 0, f"Edge {edge}: Invalid or missing L>=0"
            assert "p" in attrs and attrs["p"] >= 0, f"Edge {edge}: Invalid or missing p>=0"
            assert "g" in attrs and attrs["g"] >= 0, f"Edge {edge}: Invalid or missing g>=0"
        if edge in retail_s:
            assert "p" in attrs and attrs["p"] >= 0, f"Edge {edge}: Invalid or missing p>=0 (price)"
            assert "b" in attrs and attrs["b"] >= 0, f"Edge {edge}: Invalid or missing b>=0 (backlog cost)"
            d, sp = market_demand_attrs(g, edge, user_D, sample_path, num_periods)
            # every market link carries user_D by now (:159-161), so this never fires
            assert "demand_dist_func" in attrs or d is not None, \
                f"Edge {edge}: Missing demand source ('demand_dist_func' or 'user_D')"
            if "demand_dist_func" in attrs:
                assert "dist_param" in attrs, f"Edge {edge}: Missing 'dist_param' for 'demand_dist_func'"
            if np.sum(d) > 0 and not sp:
                assert len(d) == num_periods, f"Edge {edge}: user_D length {len(d)} != num_periods {num_periods}"


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


def compile_graph(g, num_periods, user_D=None, sample_path=None, validate=True):
    """Validate (network_management.py:197-233; skipped with validate=False by a
    caller that already did) and compile a graph to the kernel's tables."""
    user_D = user_D or {}
    sample_path = sample_path or {}
    if validate:
        validate_inputs(g, num_periods, user_D, sample_path)
    market, rawmat, factory, distrib, retail, main, reorder, retail_links, network_links = classify(g)
    mi = {j: i for i, j in enumerate(main)}
    ei = {e: i for i, e in enumerate(reorder)}
    ri = {e: i for i, e in enumerate(retail_links)}
    for s, _ in reorder:
        if s not in mi and s not in rawmat:
            raise ValueError(f"supplier {s} is neither a main node nor a raw material")
    for r, _ in retail_links:
        if r not in mi:
            raise ValueError(f"retail link source {r} must be a main (inventory) node")
    nattr = lambda j, k: g.nodes[j].get(k, 0.0)  # noqa: E731  (C, o, v only on factories)
    T = int(num_periods)
    t = {
        "I0": np.array([g.nodes[j]["I0"] for j in main], np.float64),
        "h": np.array([g.nodes[j]["h"] for j in main], np.float64),
        "C": np.array([nattr(j, "C") for j in main], np.float64),
        "o": np.array([nattr(j, "o") for j in main], np.float64),
        # distributors consume order_fulfilled / 1.0 (:484)
        "v": np.array([g.nodes[j]["v"] if j in factory else 1.0 for j in main], np.float64),
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
    # demand source per market link (network_management.py:246-267)
    lam = np.zeros(len(retail_links), np.float64)
    use = np.zeros(len(retail_links), np.int32)
    kind = np.ones(max(len(retail_links), 1), np.int32)
    n_lo = np.zeros(max(len(retail_links), 1), np.int64)
    high = np.zeros(max(len(retail_links), 1), np.int64)
    prob = np.zeros(max(len(retail_links), 1), np.float64)
    uD = np.zeros((max(len(retail_links), 1), T), np.float64)
    for e, r in ri.items():
        attrs = g.edges[e]
        d, sp = market_demand_attrs(g, e, user_D, sample_path, T)
        if np.sum(d) > 0 and not sp:                                   # :250-255
            uD[r] = np.asarray(d, np.float64)
            use[r] = 1
        else:                                                          # :257-267
            src = market_sampler(attrs)
            if src is ZERO_DEMAND:
                print(f"Warning: No valid demand source for edge {e}. Defaulting to 0.")
            kind[r], lam[r], n_lo[r], high[r], prob[r] = src
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
