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
    with pytest.raises(ValueError):
        compile_graph(default_graph(), 30, user_D={(1, 0): np.ones(5)})


def test_market_sampler_sources():
    """network_management.py:257-263: the numpy method a market's demand_dist_func
    calls (by name or from the lambda's code), else dist_param's keys."""
    import networkx as nx
    from invsim.topology import compile_graph, market_sampler

    class Env:
        np_random = np.random.default_rng(0)
    env = Env()
    assert market_sampler({"dist_param": {"lam": 20}})[:2] == (1, 20.0)
    assert market_sampler({"demand_dist_func": lambda **p: env.np_random.poisson(**p),
                           "dist_param": {"lam": 3}})[:2] == (1, 3.0)
    assert market_sampler({"demand_dist_func": lambda **p: env.np_random.binomial(**p),
                           "dist_param": {"n": 5, "p": 0.5}}) == (2, 0.0, 5, 0, 0.5)
    assert market_sampler({"dist_param": {"low": 4, "high": 9}}) == (3, 0.0, 4, 9, 0.0)
    assert market_sampler({"demand_dist_func": "integers", "dist_param": {"low": 9}}) == (3, 0.0, 0, 9, 0.0)
    assert market_sampler({"dist_param": {"p": 0.25}}) == (4, 0.0, 0, 0, 0.25)
    with pytest.raises(ValueError):
        market_sampler({"demand_dist_func": lambda **p: env.np_random.gamma(**p), "dist_param": {"shape": 2}})
    with pytest.raises(ValueError, match="needs dist_param"):
        market_sampler({"demand_dist_func": "binomial", "dist_param": {"n": 5}})
    g = nx.DiGraph()
    g.add_node(0)
    g.add_node(1, I0=10, h=0.1)
    g.add_node(2)
    g.add_edge(1, 0, p=1.0, b=0.1, dist_param={"n": 5, "p": 0.5})
    g.add_edge(2, 1, L=1, p=0.5, g=0.0)
    t = compile_graph(g, 10).tables
    assert t["rl_dist"].tolist() == [2] and t["rl_n"].tolist() == [5] and t["rl_dp"].tolist() == [0.5]
