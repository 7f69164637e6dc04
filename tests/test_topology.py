"""CPU: the NetInvMgmt topology compiler reproduces the reference's graph
classification and ordering rules (network_management.py:146-195), checked
against the golden fixtures' recorded topology and the oracle's independent
restatement."""
import numpy as np
import pytest

from conftest import NET_GOLDENS, load_golden


@pytest.mark.parametrize("name", NET_GOLDENS)
def test_topology_matches_reference_fixture(name):
    from invsim.topology import compile_graph, custom_graph, default_graph
    fx, cfg = load_golden(name)
    g = custom_graph() if cfg["module"].endswith("custom") else default_graph()
    t = compile_graph(g, cfg.get("num_periods", 30))
    topo = cfg["topology"]
    assert t.obs_dim == topo["obs_dim"]
    assert [list(e) for e in t.reorder_links] == topo["reorder_links"]
    assert [list(e) for e in t.retail_links] == topo["retail_links"]
    assert t.main_nodes == topo["main_nodes"]


@pytest.mark.parametrize("which", ["default", "custom"])
def test_topology_matches_oracle_tables(oracle, which):
    from invsim.topology import compile_graph, custom_graph, default_graph
    g = default_graph() if which == "default" else custom_graph()
    t = compile_graph(g, 30)
    o = oracle.net_tables(g, 30)
    ot = o["tables"]
    for k in ("I0", "h", "C", "o", "v", "is_factory", "is_retail", "sup", "pur", "L",
              "sup_is_factory", "lp", "lg", "rl_node", "rl_p", "rl_b", "rl_lam"):
        assert np.array_equal(t.tables[k][: len(ot[k])], ot[k]), k
    # CSR adjacency == oracle's padded adjacency
    J = o["J"]
    for j in range(J):
        a, b = t.tables["succ_ptr"][j], t.tables["succ_ptr"][j + 1]
        assert b - a == ot["succ_n"][j]
        assert np.array_equal(t.tables["succ_kind"][a:b], ot["succ_kind"][j, : b - a])
        assert np.array_equal(t.tables["succ_idx"][a:b], ot["succ_idx"][j, : b - a])
        a, b = t.tables["pred_ptr"][j], t.tables["pred_ptr"][j + 1]
        assert b - a == ot["pred_n"][j]
        assert np.array_equal(t.tables["pred_idx"][a:b], ot["pred_idx"][j, : b - a])


def test_default_graph_facts():
    from invsim.topology import compile_graph, default_graph
    t = compile_graph(default_graph(), 30)
    assert t.obs_dim == 68 and len(t.reorder_links) == 11 and t.lt_max == 12
    assert t.retail == [1] and t.factory == [4, 5, 6] and sorted(t.rawmat) == [7, 8]
    assert sum(t.lead_times.values()) == 61


def test_user_demand_table():
    from invsim.topology import compile_graph, default_graph
    d = np.arange(30, dtype=float)
    t = compile_graph(default_graph(), 30, user_D={(1, 0): d})
    assert t.tables["rl_user"][0] == 1 and np.array_equal(t.tables["user_D"][0], d)
    t = compile_graph(default_graph(), 30, user_D={(1, 0): d}, sample_path={(1, 0): True})
    assert t.tables["rl_user"][0] == 0 and t.tables["rl_lam"][0] == 20
    with pytest.raises(AssertionError, match=r"Edge \(1, 0\): user_D length 5 != num_periods 30"):
        compile_graph(default_graph(), 30, user_D={(1, 0): np.ones(5)})


def test_market_sampler_sources():
    """network_management.py:257-267: a market draws demand_dist_func(**dist_param)
    only when it has both; the method comes from a name, a Generator's bound
    method or the reference's lambda shape; anything else is demand 0 with no
    draw (ZERO_DEMAND = Poisson(0))."""
    import networkx as nx
    from invsim.topology import ZERO_DEMAND, compile_graph, market_sampler

    class Env:
        np_random = np.random.default_rng(0)
    env = Env()
    assert market_sampler({"demand_dist_func": "poisson", "dist_param": {"lam": 20}})[:2] == (1, 20.0)
    assert market_sampler({"demand_dist_func": lambda **p: env.np_random.poisson(**p),
                           "dist_param": {"lam": 3}})[:2] == (1, 3.0)
    assert market_sampler({"demand_dist_func": lambda **p: env.np_random.binomial(**p),
                           "dist_param": {"n": 5, "p": 0.5}}) == (2, 0.0, 5, 0, 0.5)
    assert market_sampler({"demand_dist_func": lambda **p: env.np_random.integers(**p),
                           "dist_param": {"low": 4, "high": 9}}) == (3, 0.0, 4, 9, 0.0)
    # a host Generator's bound method draws from that generator, never the env's stream
    with pytest.raises(ValueError, match="bound method of a host numpy Generator"):
        market_sampler({"demand_dist_func": env.np_random.integers, "dist_param": {"low": 4, "high": 9}})
    assert market_sampler({"demand_dist_func": "integers", "dist_param": {"low": 9}}) == (3, 0.0, 0, 9, 0.0)
    assert market_sampler({"demand_dist_func": "geometric", "dist_param": {"p": 0.25}}) == (4, 0.0, 0, 0, 0.25)
    assert market_sampler({"demand_dist_func": "poisson", "dist_param": {}}) == (1, 1.0, 0, 0, 0.0)
    # no demand_dist_func, or no dist_param: demand 0, no draw (:264-267)
    assert market_sampler({"dist_param": {"lam": 20}}) is ZERO_DEMAND
    assert market_sampler({"dist_param": {"n": 5, "p": 0.5}}) is ZERO_DEMAND
    assert market_sampler({"demand_dist_func": "poisson"}) is ZERO_DEMAND
    assert market_sampler({}) is ZERO_DEMAND
    with pytest.raises(ValueError):
        market_sampler({"demand_dist_func": lambda **p: env.np_random.gamma(**p), "dist_param": {"shape": 2}})
    with pytest.raises(ValueError, match="needs dist_param"):
        market_sampler({"demand_dist_func": "binomial", "dist_param": {"n": 5}})
    with pytest.raises(ValueError, match="unsupported dist_param"):
        market_sampler({"demand_dist_func": "poisson", "dist_param": {"lam": 5, "size": 3}})
    g = nx.DiGraph()
    g.add_node(0)
    g.add_node(1, I0=10, h=0.1)
    g.add_node(2)
    g.add_edge(1, 0, p=1.0, b=0.1, demand_dist_func="binomial", dist_param={"n": 5, "p": 0.5})
    g.add_edge(2, 1, L=1, p=0.5, g=0.0)
    t = compile_graph(g, 10).tables
    assert t["rl_dist"].tolist() == [2] and t["rl_n"].tolist() == [5] and t["rl_dp"].tolist() == [0.5]


def test_lambda_shapes_outside_the_reference_form_are_refused():
    """Only `lambda **p: <recv>.np_random.<method>(**p)` names a device sampler:
    arithmetic on the draw, numpy's global RandomState or fixed arguments
    would change the values or the stream, so they raise."""
    from invsim.topology import market_sampler

    class Env:
        np_random = np.random.default_rng(0)
    self = Env()
    ok = [lambda **p: self.np_random.poisson(**p), lambda **kw: self.np_random.geometric(**kw)]
    for f in ok:
        assert market_sampler({"demand_dist_func": f, "dist_param": {"lam": 2} if f is ok[0] else {"p": .5}})
    bad = [lambda **p: 2 * self.np_random.poisson(**p),
           lambda **p: np.random.poisson(**p),
           lambda **p: self.np_random.poisson(lam=4),
           lambda **p: self.np_random.poisson(3, **p),
           lambda **p: self.other.poisson(**p),
           lambda **p: self.np_random.poisson(**p) + 1,
           lambda lam: self.np_random.poisson(lam),
           np.random.poisson]
    for f in bad:
        with pytest.raises(ValueError, match="unsupported demand_dist_func"):
            market_sampler({"demand_dist_func": f, "dist_param": {"lam": 2}})


def _three_market_graph():
    """The custom graph with one source-less market, one dist_param-only market
    and one reference-style lambda market, whose receiver is a free variable
    that `bind(env)` sets to the env (network_management.py:125 names the env
    itself; check_market_receivers refuses any other receiver at reset)."""
    from invsim.topology import custom_graph
    env = None

    def bind(e):
        nonlocal env
        env = e
    g = custom_graph()
    a, b, c = [e for e in g.edges() if "L" not in g.edges[e]]
    del g.edges[a]["dist_param"], g.edges[a]["demand_dist_func"]
    del g.edges[b]["demand_dist_func"]
    g.edges[c]["demand_dist_func"] = lambda **p: env.np_random.poisson(**p)
    return g, bind


_GLOBAL_RECV = None


def test_market_lambda_receiver_must_be_the_env():
    """VERDICT r04 item 1 (network_management.py:257-263, :125): the reference
    calls the market lambda as written, so `<recv>.np_random.<m>(**p)` draws
    from <recv>'s generator.  The device draws from the env's own stream, so a
    receiver that is not the env (or a view over it) raises at reset instead of
    silently drawing different demands; the receiver is resolved at reset, as a
    late-bound global or closure only binds after the graph is built."""
    global _GLOBAL_RECV
    from invsim.topology import check_market_receivers, compile_graph, custom_graph

    class FakeEnv:                      # stands in for the vector env (no GPU here)
        pass

    class Holder:                       # some other object with a generator
        np_random = np.random.default_rng(0)

    class View:                         # invsim.compat's single-env view keeps the env as _v
        def __init__(self, v):
            self._v = v

    def graph_with(f):
        g = custom_graph()
        c = [e for e in g.edges() if "L" not in g.edges[e]][2]
        g.edges[c]["demand_dist_func"] = f
        return g

    def check(g):
        env = FakeEnv()
        env.topology = compile_graph(g, 30)
        return env, (lambda: check_market_receivers(g, env.topology.retail_links, env))

    # closure receiver bound to the env after construction: accepted
    g, bind = _three_market_graph()
    env, run = check(g)
    with pytest.raises(ValueError, match="not bound at reset"):
        run()
    bind(env)
    run()
    bind(View(env))                     # the compat view over the env
    run()
    for foreign in (Holder(), View(FakeEnv()), FakeEnv()):
        bind(foreign)
        with pytest.raises(ValueError, match="not this env's"):
            run()
    bind(None)
    with pytest.raises(ValueError, match="not bound at reset"):
        run()
    # a module-global receiver, resolved at check time, not at compile time
    g = graph_with(lambda **p: _GLOBAL_RECV.np_random.poisson(**p))
    env, run = check(g)
    _GLOBAL_RECV = Holder()
    with pytest.raises(ValueError, match="Holder object's np_random"):
        run()
    _GLOBAL_RECV = env
    run()
    _GLOBAL_RECV = None
    with pytest.raises(ValueError, match="not bound at reset"):
        run()
    # numpy's global RandomState and a default_rng holder's bound method never compile
    with pytest.raises(ValueError, match="unsupported demand_dist_func"):
        compile_graph(graph_with(lambda **p: np.random.poisson(**p)), 30)
    with pytest.raises(ValueError, match="bound method of a host numpy Generator"):
        compile_graph(graph_with(np.random.default_rng(1).poisson), 30)
    # a market replaying user_D never calls its lambda: not checked (:250-255)
    h = Holder()
    g = graph_with(lambda **p: h.np_random.poisson(**p))
    c = [e for e in g.edges() if "L" not in g.edges[e]][2]
    env = FakeEnv()
    env.topology = compile_graph(g, 30, user_D={c: np.arange(30.0)})
    check_market_receivers(g, env.topology.retail_links, env)


def test_source_less_and_dist_param_only_markets_draw_nothing(oracle):
    """the product and the oracle both give demand 0 with no
    draw (Poisson(0)) to a market without demand_dist_func or without
    dist_param, and Poisson(lam) to the lambda market; user_D with sum 0 or
    sample_path=True falls through to the same rule."""
    from invsim.topology import compile_graph
    g, _ = _three_market_graph()
    t = compile_graph(g, 30).tables
    assert t["rl_dist"].tolist() == [1, 1, 1]
    assert t["rl_lam"].tolist() == [0.0, 0.0, 20.0]
    assert t["rl_user"].tolist() == [0, 0, 0]
    o = oracle.net_tables(g, 30)["tables"]
    for k in ("rl_dist", "rl_lam", "rl_n", "rl_high", "rl_dp", "rl_user"):
        assert np.array_equal(t[k][:3], o[k][:3]), k
    d = np.arange(30.0)
    a = [e for e in g.edges() if "L" not in g.edges[e]][0]
    t = compile_graph(g, 30, user_D={a: d}, sample_path={a: True}).tables
    o = oracle.net_tables(g, 30, user_D={a: d}, sample_path={a: True})["tables"]
    assert t["rl_user"][0] == 0 == o["rl_user"][0] and t["rl_lam"][0] == 0.0 == o["rl_lam"][0]
    t = compile_graph(g, 30, user_D={a: d}).tables
    o = oracle.net_tables(g, 30, user_D={a: d})["tables"]
    assert t["rl_user"][0] == 1 == o["rl_user"][0] and np.array_equal(t["user_D"][0], o["user_D"][0])


def test_reference_demand_rule_source_text():
    """Parity UNPINNED by execution (the reference cannot be imported here):
    this reads network_management.py's `_setup_demand_distributions` as text
    (ast, nothing executed) and checks the rule restated above -- user_D when
    its sum is positive and sample_path is False, else a draw only when BOTH
    'demand_dist_func' and 'dist_param' are on the edge, else `lambda: 0`."""
    import ast
    import os
    path = "/root/reference/network_management.py"
    if not os.path.exists(path):
        pytest.skip("reference source not present")
    tree = ast.parse(open(path).read())
    fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "_setup_demand_distributions")
    ifs = [n for n in ast.walk(fn) if isinstance(n, ast.If) and ast.unparse(n.test) == "use_user_d"]
    assert len(ifs) == 1
    elif_ = ifs[0].orelse[0]
    assert isinstance(elif_, ast.If)
    assert ast.unparse(elif_.test) == "'demand_dist_func' in data and 'dist_param' in data"
    fallback = ast.unparse(elif_.orelse[-1])
    assert fallback.replace(' ', '') == "data['_sample_demand']=lambda:0"
    use = next(n for n in ast.walk(fn) if isinstance(n, ast.Assign) and ast.unparse(n.targets[0]) == "use_user_d")
    assert ast.unparse(use.value) == ("'user_D' in data and np.sum(data['user_D']) > 0 and "
                                      "(not data.get('sample_path', False))")
