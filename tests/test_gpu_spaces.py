"""Observation / action Box bounds of the five env classes against the values
the reference's own space definitions give for its default configurations,
worked out by hand from those lines (the fixtures carry no spaces, and the
reference is not imported: parity of these bounds is pinned by the cited
arithmetic, not by generated vectors):

* newsvendor.py:75-88 -- obs low 0, high [p_max, p_max, h_max, k_max, mu_max] +
  [max_order_quantity] * L (float32); action [0, max_order_quantity] (float32)
* inventory_management.py:111-128 -- action [0, c] int64; obs bound
  inv_capacity_sum = sum(c) * periods * 2, low -bound (backlog) or 0 (lost
  sales), shape (m-1)(lt_max+1)
* network_management.py:193-195, 270-298, 755-770 -- order_cap_heuristic =
  max I0 + 5 max C; action [0, 2 ocap] float32; obs high ocap * T * 2, low
  -high when backlogged (the LostSales class still runs backlog=True, :84),
  the first len(retail_links) entries low 0
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _eq(box, low, high, dtype, shape):
    assert box.dtype == np.dtype(dtype) and tuple(box.shape) == shape
    assert np.array_equal(np.asarray(box.low), np.asarray(low, dtype=dtype))
    assert np.array_equal(np.asarray(box.high), np.asarray(high, dtype=dtype))


def test_newsvendor_spaces(gpu):
    import invsim
    env = invsim.NewsvendorEnv(4, device=gpu)                   # defaults: L 5, p 100, h 5, k 10, mu 200, q 2000
    _eq(env.single_observation_space, np.zeros(10), [100, 100, 5, 10, 200] + [2000] * 5, np.float32, (10,))
    _eq(env.single_action_space, [0], [2000], np.float32, (1,))
    env = invsim.NewsvendorEnv(4, device=gpu, lead_time=0, p_max=7.5, max_order_quantity=33)
    _eq(env.single_observation_space, np.zeros(5), [7.5, 7.5, 5, 10, 200], np.float32, (5,))
    _eq(env.single_action_space, [0], [33], np.float32, (1,))


@pytest.mark.parametrize("cls,low", [("InvManagementBacklogEnv", -31800), ("InvManagementLostSalesEnv", 0)])
def test_invmgmt_spaces(gpu, cls, low):
    import invsim
    env = getattr(invsim, cls)(4, device=gpu)                  # c = [100, 200, 230], periods 30, lt_max 10
    bound = (100 + 200 + 230) * 30 * 2                           # 31 800
    _eq(env.single_action_space, [0, 0, 0], [100, 200, 230], np.int64, (3,))
    _eq(env.single_observation_space, np.full(33, low), np.full(33, bound), np.int64, (33,))


@pytest.mark.parametrize("cls", ["NetInvMgmtBacklogEnv", "NetInvMgmtLostSalesEnv"])
def test_net_spaces(gpu, cls):
    import invsim
    env = getattr(invsim, cls)(4, device=gpu)                  # default graph: max I0 400, max C 90, T 30
    ocap = 400 + 90 * 5                                          # 850
    _eq(env.single_action_space, np.zeros(11), np.full(11, 2 * ocap), np.float32, (11,))
    hi = ocap * 30 * 2                                           # 51 000
    O = 1 + 6 + 61                                               # retail links + main nodes + sum of L
    low = np.full(O, -hi, np.float32)
    low[0] = 0.0
    _eq(env.single_observation_space, low, np.full(O, hi), np.float32, (O,))
