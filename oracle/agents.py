"""CPU restatement of the reference's heuristic agents and evaluate_agent sums
(TEST INFRASTRUCTURE: the checker for invsim_rollout_policy; never shipped).

Restated from the source text of the reference's benchmark scripts, vectorised
over N oracle envs with numpy, evaluating every expression in the dtypes numpy
uses there:

* base_stock       BaseStockAgent.get_action  benchmark_InvManagementBacklogEnv.py:152-198
* order_up_to      OrderUpToHeuristicAgent    benchmark_newsvendor.py:103-111
* classic_nv       ClassicNewsvendorAgent     benchmark_newsvendor.py:121-161 (calls the
                   third-party scipy.stats.poisson.ppf itself, as the reference does)
* ss_policy        sSPolicyAgent              benchmark_newsvendor_sb3_rllib.py:363-371
* constant_order   ConstantOrderAgent         benchmark_NetInvMgmtBacklogEnv.py:127-135
* run_*            evaluate_agent's per-episode sums
                   benchmark_InvManagementBacklogEnv.py:364-399,
                   benchmark_NetInvMgmtLostSalesEnv.py:259-276, benchmark_newsvendor.py:232-242

PARITY UNPINNED against the reference itself: importing the reference's
benchmark modules to generate fixtures was refused in this environment
(DESIGN.md §2); the env steps underneath are the golden-pinned oracle.
"""
import numpy as np


def base_stock(obs, t, log, L, mu, sf, c):
    """obs [N, O] int64 (obs[:, :M1] = I[t]); log [t, N, M1] requested orders
    action_log[0..t); L, c int64 [M1]; mu as env.dist_param['mu'] (int or float)."""
    M1 = len(L)
    pos = obs[:, :M1].astype(np.int64).copy()                  # inventory_position = on hand
    for i in range(M1):
        Li = int(L[i])
        if Li == 0:
            continue
        s = max(0, t - Li)
        if t > 0 and s < t:
            pos[:, i] += log[s:t, :, i].sum(axis=0)             # action_log[s:t, i].sum()
    target = (np.asarray(L, np.int64) + 1) * mu * sf            # (lead_times + 1) * mu * sf
    q = np.maximum(0, target - pos)
    q = np.clip(q, np.zeros(M1, np.int64), np.asarray(c, np.int64))
    return q.astype(np.int64)


def order_up_to(obs, lead_time, sf, max_order):
    """obs [N, 5 + L] float32 -> action [N, 1] float32 (per-env numpy float32 scalars)."""
    out = np.zeros((obs.shape[0], 1), np.float32)
    for n in range(obs.shape[0]):
        mu = obs[n, 4]
        pipeline = obs[n, 5:]
        target = mu * (lead_time + 1) * sf
        pos = pipeline.sum()
        q = max(0, target - pos)
        out[n, 0] = np.clip(q, np.float32(0), np.float32(max_order))
    return out


def classic_nv(obs, lead_time, sf, max_order, cr_method="k_vs_h"):
    """obs [N, 5 + L] float32 -> action [N, 1] float32, per-env numpy scalars."""
    from scipy.stats import poisson
    out = np.zeros((obs.shape[0], 1), np.float32)
    for n in range(obs.shape[0]):
        price, cost, h, k, mu = obs[n, :5]
        pipeline = obs[n, 5:]
        fallback = False
        if cr_method == "profit_margin":
            under = price - cost + k
            over = h
            if under + over <= 1e-6 or under <= 0 or over <= 0:
                fallback = True
            else:
                cr = under / (under + over)
        else:
            if h + k <= 1e-6 or k < 0 or h < 0:
                fallback = True
            else:
                cr = k / (h + k)
        if fallback:
            target = mu * (lead_time + 1)
            q = max(0, target - pipeline.sum())
        else:
            eff = mu * (lead_time + 1) * sf
            level = poisson.ppf(cr, mu=max(1e-6, eff))
            q = max(0, level - pipeline.sum())
        out[n, 0] = np.array([np.clip(q, np.float32(0), np.float32(max_order))], dtype=np.float32)[0]
    return out


def ss_policy(obs, lead_time, S_buffer_factor, max_order):
    from scipy.stats import poisson
    out = np.zeros((obs.shape[0], 1), np.float32)
    for n in range(obs.shape[0]):
        price, cost, h, k, mu = obs[n, :5]
        pipe = obs[n, 5:]
        s_lvl = 0
        if h + k > 1e-6:
            cr_s = k / (h + k)
            eff = mu * (lead_time + 1)
            s_lvl = poisson.ppf(np.clip(cr_s, 0.001, 0.999), mu=max(1e-6, eff))
        s_level = max(0, s_lvl)
        S_level = s_level * S_buffer_factor
        pos = pipe.sum()
        order = 0
        if pos < s_level:
            order = max(0, S_level - pos)
        out[n, 0] = np.array([np.clip(order, np.float32(0), np.float32(max_order))], dtype=np.float32)[0]
    return out


def constant_order(high, fraction, dtype):
    high = np.array(high, copy=True)
    high[high == np.inf] = 1000
    return (high * fraction).astype(dtype)


def run_invmgmt(orc, obs, steps, L, mu, sf, c, period0=0):
    """Drive an OracleInvMgmt with BaseStock for `steps` periods from `obs`
    (period period0); returns (actions, rewards, obs list, sums [N, 6])."""
    N, M1 = obs.shape[0], len(L)
    log = np.zeros((0, N, M1), np.int64)
    sums = np.zeros((N, 6))
    acts, rews, obss = [], [], []
    for k in range(steps):
        t = period0 + k
        a = base_stock(obs, t, log, L, mu, sf, c)
        obs, r, tr, info = orc.step(a, info=True)
        log = np.concatenate([log, np.maximum(a, 0)[None]], axis=0)   # action_log[t] (:250, :268)
        sums[:, 0] += r
        sums[:, 1] += 1
        sums[:, 2] += info["demand"]
        sums[:, 3] += info["sales"][:, 0]
        sums[:, 4] += info["unfulfilled"][:, 0]
        sums[:, 5] += np.maximum(0, info["ending_inventory"]).sum(axis=1)
        acts.append(a), rews.append(r), obss.append(obs)
    return np.stack(acts), np.stack(rews), np.stack(obss), sums


def run_newsvendor(orc, obs, steps, lead_time, sf, max_order, agent="order_up_to", cr_method="k_vs_h"):
    N = obs.shape[0]
    sums = np.zeros((N, 2))
    acts, rews, obss = [], [], []
    for _ in range(steps):
        if agent == "classic_nv":
            a = classic_nv(obs, lead_time, sf, max_order, cr_method)
        elif agent == "ss":
            a = ss_policy(obs, lead_time, sf, max_order)
        else:
            a = order_up_to(obs, lead_time, sf, max_order)
        obs, r, tr, _ = orc.step(a)
        sums[:, 0] += r
        sums[:, 1] += 1
        acts.append(a), rews.append(r), obss.append(obs)
    return np.stack(acts), np.stack(rews), np.stack(obss), sums


def run_net(orc, obs, steps, action):
    N = obs.shape[0]
    J = orc.topo["J"]
    sums = np.zeros((N, 5 + J))
    a = np.broadcast_to(action, (N, len(action))).astype(np.float32)
    rews, obss = [], []
    for _ in range(steps):
        obs, r, tr, info = orc.step(a, info=True)
        sums[:, 0] += r
        sums[:, 1] += 1
        for q in range(info["D"].shape[1]):   # the kernel's order (exact either way for integer flows)
            sums[:, 2] += info["D"][:, q]
            sums[:, 3] += info["S"][:, q]
            sums[:, 4] += info["U"][:, q]
        sums[:, 5:] += info["X"]
        rews.append(r), obss.append(obs)
    return np.stack(rews), np.stack(obss), sums
