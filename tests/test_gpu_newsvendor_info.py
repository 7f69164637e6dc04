"""Newsvendor step info: the cost components of newsvendor.py:149-170 that the
reference returns in ``info`` (:195-199), from the kernels' step record.

The expected values are restated here from the reference expressions with
NumPy-2 scalars (NEP 50: np.float32 op Python float stays float32, Python
min/max return one of their operands), driven by the golden fixtures' states,
actions and demands: same values bit for bit and the same scalar type (Python
float / np.float32 / np.float64) as the reference produces."""
import numpy as np
import pytest
import torch

from conftest import NV_GOLDENS, load_golden, nv_kwargs

pytestmark = pytest.mark.gpu

KINDS = (float, np.float32, np.float64, int)


def ref_components(prev_obs, action, demand, params, cfg):
    """newsvendor.py:128-167 for one env, NumPy-2 scalar semantics."""
    L = max(0, int(cfg.get("lead_time", 5)))
    max_q = cfg.get("max_order_quantity", 2000)
    max_inv = cfg.get("max_inventory", 4000)
    price, cost, h, k = (float(x) for x in params[:4])
    price = 1 if price == 1.0 else price                              # max(1, .) -> the Python int 1 (:105-106)
    cost = 1 if cost == 1.0 else cost
    state = np.asarray(prev_obs, np.float32)
    order_qty = np.clip(float(action), 0, max_q)                        # :130-131
    cur = state[5:].sum()                                              # :134
    inv = state[5] if L > 0 else order_qty                             # :135-141
    order_qty = max(0, min(order_qty, max_inv - cur))                  # :143
    d = int(demand)
    sales = min(inv, d)                                                # :149
    revenue = sales * price                                            # :150
    excess = max(0, inv - d)                                           # :152
    short = max(0, d - inv)                                            # :153
    purchase = order_qty * cost                                        # :162
    holding = excess * h                                               # :166
    penalty = short * k                                                # :167
    return revenue, purchase, holding, penalty


def _kind(x):
    return 1 if isinstance(x, np.float32) else 2 if isinstance(x, np.float64) else 3 if type(x) is int else 0


@pytest.mark.parametrize("name", NV_GOLDENS)
def test_newsvendor_step_info_costs_vs_reference_expressions(gpu, name):
    from invsim import NewsvendorEnv
    fx, cfg = load_golden(name)
    n, n_ep, T = cfg["n_env"], cfg["n_ep"], cfg["ep_len"]
    env = NewsvendorEnv(n, device=gpu, autoreset_mode="disabled", record_demand=True, record_info=True,
                        **nv_kwargs(cfg))
    names = ("revenue", "purchase_cost", "holding_cost", "lost_sales_penalty")
    seen = set()
    for ep in range(n_ep):
        env.reset(seed=cfg["base_seed"]) if ep == 0 else env.reset()
        prev = fx["reset_obs"][:, ep]
        for t in range(T):
            s = ep * T + t
            a = torch.from_numpy(np.ascontiguousarray(fx["actions"][:, s])).to(gpu)
            _, r, _, _, info = env.step(a)
            got = {k: info[k].cpu().numpy() for k in names}
            kinds = {k: info[k + "_kind"].cpu().numpy() for k in names}
            for i in range(n):
                exp = ref_components(prev[i], fx["actions"][i, s].reshape(-1)[0], fx["demand"][i, s],
                                     fx["params"][i, ep], cfg)
                for k, x in zip(names, exp):
                    assert np.float64(x).view(np.int64) == got[k][i].view(np.int64) or (x != x and got[k][i] != got[k][i]), \
                        f"{k} env {i} step {s}: {x!r} vs {got[k][i]!r}"
                    assert kinds[k][i] == _kind(x), f"{k} kind env {i} step {s}"
                    seen.add((k, _kind(x)))
            prev = fx["obs"][:, s]
    assert ("revenue", 1) in seen or ("revenue", 0) in seen


@pytest.mark.parametrize("p_max", [100.0, 0.5])
def test_newsvendor_compat_view_info_types(gpu, p_max):
    """The single-env view's info carries the components with the reference's
    scalar types (p_max = 0.5: price and cost are the Python int 1 of max(1, .),
    so revenue and a zero order's purchase cost are Python ints)."""
    from invsim import compat
    env = compat.make("NewsvendorEnv", device=gpu, lead_time=2, step_limit=6, p_max=p_max)
    obs, info = env.reset(seed=3)
    prev = obs.copy()
    for a in (50.0, 0.0, 3000.0, 7.5, 0.0):
        obs, r, te, tr, info = env.step(np.array([a], np.float32))
        exp = ref_components(prev, a, info["demand"], [info["price"], info["cost"], info["holding_cost_rate"],
                                                       info["penalty_cost_rate"]], dict(lead_time=2))
        for k, x in zip(("revenue", "purchase_cost", "holding_cost", "lost_sales_penalty"), exp):
            assert type(info[k]) is type(x), (k, type(info[k]), type(x))
            assert np.float64(info[k]) == np.float64(x)
        assert r == float(((exp[0] - exp[1]) - exp[2]) - exp[3])
        prev = obs.copy()
    if p_max < 1:
        assert type(info["price"]) is int and type(info["cost"]) is int
