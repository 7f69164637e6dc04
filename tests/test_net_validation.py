"""CPU: NetInvMgmt input validation restates network_management.py:197-238 --
node asserts, then edge asserts, then the scalar ones, each with the
reference's AssertionError message.  Every case fails in
the constructor before any GPU work, so these run without a GPU."""
import os

import numpy as np
import pytest

REF = "/root/reference/network_management.py"


def _env(graph=None, **kw):
    import invsim
    return invsim.NetInvMgmtMasterEnv(1, graph=graph, **kw)


def _g():
    from invsim.topology import default_graph
    return default_graph()


def _drop_node(j, k):
    g = _g()
    del g.nodes[j][k]
    return g


def _set_node(j, k, v):
    g = _g()
    g.nodes[j][k] = v
    return g


def _drop_edge(e, k):
    g = _g()
    del g.edges[e][k]
    return g


def _set_edge(e, k, v):
    g = _g()
    g.edges[e][k] = v
    return g


CASES = [
    # node checks (:208-216)
    (lambda: _set_node(1, "I0", -1), {}, "Node 1: Invalid or missing I0>=0"),
    (lambda: _set_node(2, "I0", float("nan")), {}, "Node 2: Invalid or missing I0>=0"),
    (lambda: _drop_node(4, "I0"), {}, "Node 4: Invalid or missing I0>=0"),
    (lambda: _drop_node(3, "h"), {}, "Node 3: Invalid or missing h>=0"),
    (lambda: _set_node(6, "h", -0.5), {}, "Node 6: Invalid or missing h>=0"),
    (lambda: _set_node(5, "C", 0), {}, "Node 5: Invalid or missing C>0"),
    (lambda: _drop_node(4, "o"), {}, "Node 4: Invalid or missing o>=0"),
    (lambda: _set_node(6, "o", -1e-3), {}, "Node 6: Invalid or missing o>=0"),
    (lambda: _drop_node(5, "v"), {}, "Node 5: Invalid or missing v in (0, 1]"),
    (lambda: _set_node(4, "v", 1.5), {}, "Node 4: Invalid or missing v in (0, 1]"),
    (lambda: _set_node(4, "v", 0.0), {}, "Node 4: Invalid or missing v in (0, 1]"),
    # reorder-link checks (:221-224)
    (lambda: _set_edge((2, 1), "L", -1), {}, "Edge (2, 1): Invalid or missing L>=0"),
    (lambda: _drop_edge((4, 3), "p"), {}, "Edge (4, 3): Invalid or missing p>=0"),
    (lambda: _set_edge((7, 5), "p", -0.1), {}, "Edge (7, 5): Invalid or missing p>=0"),
    (lambda: _drop_edge((8, 6), "g"), {}, "Edge (8, 6): Invalid or missing g>=0"),
    # market-link checks (:225-233)
    (lambda: _drop_edge((1, 0), "p"), {}, "Edge (1, 0): Invalid or missing p>=0 (price)"),
    (lambda: _set_edge((1, 0), "b", -2), {}, "Edge (1, 0): Invalid or missing b>=0 (backlog cost)"),
    (lambda: _drop_edge((1, 0), "dist_param"), {}, "Edge (1, 0): Missing 'dist_param' for 'demand_dist_func'"),
    (_g, {"user_D": {(1, 0): np.ones(7)}}, "Edge (1, 0): user_D length 7 != num_periods 30"),
    (lambda: _set_edge((1, 0), "user_D", [3] * 12), {}, "Edge (1, 0): user_D length 12 != num_periods 30"),
    # scalar checks (:236-238)
    (_g, {"backlog": 1}, "backlog must be boolean"),
    (_g, {"alpha": 0.0}, "alpha must be in (0, 1]"),
    (_g, {"alpha": 1.01}, "alpha must be in (0, 1]"),
    (_g, {"num_periods": 0}, "num_periods must be positive"),
]


@pytest.mark.parametrize("make,kw,msg", CASES, ids=[c[2][:40] + f"#{i}" for i, c in enumerate(CASES)])
def test_bad_graph_raises_reference_assert(make, kw, msg):
    with pytest.raises(AssertionError) as ei:
        _env(graph=make(), **kw)
    assert str(ei.value) == msg


def test_first_failing_check_wins_in_reference_order():
    """Nodes before edges, in graph order; the scalar checks come last."""
    g = _drop_edge((2, 1), "p")
    g.nodes[6]["h"] = -1
    with pytest.raises(AssertionError, match=r"^Node 6: Invalid or missing h>=0$"):
        _env(graph=g, alpha=5.0)
    g = _drop_edge((2, 1), "p")
    with pytest.raises(AssertionError, match=r"^Edge \(2, 1\): Invalid or missing p>=0$"):
        _env(graph=g, alpha=5.0)


def test_sample_path_or_zero_user_d_skips_length_check():
    """:232: the length is only checked for a user_D that will be replayed."""
    from invsim.topology import validate_inputs
    validate_inputs(_g(), 30, user_D={(1, 0): np.ones(7)}, sample_path={(1, 0): True})
    validate_inputs(_g(), 30, user_D={(1, 0): np.zeros(7)})
    g = _g()
    g.edges[1, 0]["user_D"] = [1] * 5
    g.edges[1, 0]["sample_path"] = True
    validate_inputs(g, 30)


def test_missing_attributes_are_not_defaulted():
    """compile_graph no longer fills a missing h / v."""
    from invsim.topology import compile_graph
    with pytest.raises(AssertionError, match="Node 1: Invalid or missing h>=0"):
        compile_graph(_drop_node(1, "h"), 30)
    with pytest.raises(AssertionError, match=r"Node 6: Invalid or missing v in \(0, 1\]"):
        compile_graph(_drop_node(6, "v"), 30)


def _reference_messages():
    """The assert message templates of the reference's _validate_inputs, read
    as text with ast (nothing executed)."""
    import ast
    tree = ast.parse(open(REF).read())
    fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "_validate_inputs")
    out = []
    for n in ast.walk(fn):
        if isinstance(n, ast.Assert) and n.msg is not None:
            if isinstance(n.msg, ast.JoinedStr):
                parts = []
                for v in n.msg.values:
                    parts.append(v.value if isinstance(v, ast.Constant) else "{}")
                out.append("".join(parts))
            else:
                out.append(n.msg.value)
    return out


def test_messages_match_reference_source_text():
    """Every message template in network_management.py:197-238 is one this
    module checks above (placeholders filled)."""
    if not os.path.exists(REF):
        pytest.skip("reference source not present")
    import re
    ref = _reference_messages()
    assert len(ref) == 16
    ours = {c[2] for c in CASES} | {"Edge (1, 0): Missing demand source ('demand_dist_func' or 'user_D')"}
    for tmpl in ref:
        pat = "^" + re.escape(tmpl).replace(r"\{\}", ".+") + "$"
        assert any(re.match(pat, m) for m in ours), tmpl
