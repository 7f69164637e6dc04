"""In-kernel heuristic agents (invsim_rollout_policy) and batched evaluate_agent
against the CPU restatement in oracle/agents.py.

The agents' own parity with the reference is UNPINNED (importing
the reference benchmark modules was refused); the env dynamics underneath are
the golden-pinned ones.  GPU tests compare device and oracle bit for bit.
"""
import numpy as np
import pytest

import agents


def test_base_stock_restatement_hand_case():
    # 2 stages, L = [1, 3], mu = 20, sf = 1.0, capacities [50, 200]
    obs = np.array([[10, -5, 0, 0, 0, 0, 0, 0]], np.int64)
    log = np.array([[[4, 7]], [[6, 1]], [[2, 9]]], np.int64)     # action_log[0..3)
    a = agents.base_stock(obs, 3, log, np.array([1, 3]), 20, 1.0, np.array([50, 200]))
    # stage 0: target 40, position 10 + log[2,0] = 12 -> 28
    # stage 1: target 80, position -5 + (7 + 1 + 9) = 12 -> 68
    assert a.tolist() == [[28, 68]]
    a = agents.base_stock(obs, 3, log, np.array([1, 3]), 20, 1.37, np.array([50, 200]))
    assert a.tolist() == [[int(40 * 1.37 - 12), int(80 * 1.37 - 12)]]
    assert agents.base_stock(obs * 0 - 500, 0, log[:0], np.array([1, 3]), 20, 1.0,
                             np.array([50, 200])).tolist() == [[50, 200]]    # clipped to capacity


def test_order_up_to_restatement_float32():
    obs = np.zeros((2, 10), np.float32)
    obs[:, 4] = [37.25, 150.5]
    obs[0, 5:] = [10, 20, 30, 40, 50]
    obs[1, 5:] = 1000
    a = agents.order_up_to(obs, 5, 1.0, 2000)
    assert a.dtype == np.float32
    assert a[0, 0] == np.float32(np.float32(37.25) * 6) - np.float32(150)
    assert a[1, 0] == 0.0                                          # max(0, negative)


@pytest.mark.gpu
@pytest.mark.parametrize("cls,sf,mu", [("InvManagementBacklogEnv", 1.0, 20), ("InvManagementBacklogEnv", 1.37, 20),
                                       ("InvManagementLostSalesEnv", 1.0, 20),
                                       ("InvManagementBacklogEnv", 0.8, 12.5)])
def test_base_stock_vs_oracle(gpu, oracle, cls, sf, mu):
    import torch
    import invsim
    n = 1000
    env = getattr(invsim, cls)(n, device=gpu, dist_param={"mu": mu}, autoreset_mode="disabled")
    kw = dict(backlog=(cls != "InvManagementLostSalesEnv"), dist_param={"mu": mu})
    orc = oracle.OracleInvMgmt(n, **kw)
    orc.seed(range(500, 500 + n))
    o0 = orc.reset()
    env.reset(seed=500)
    M = invsim.policies.metrics_dim(env)
    met = torch.zeros((n, M), dtype=torch.float64, device=gpu)
    out = env.rollout_policy(invsim.BaseStockAgent(sf), 30, obs=True, actions=True, metrics=met)
    e_act, e_rew, e_obs, e_sum = agents.run_invmgmt(orc, o0, 30, env.lead_time, mu, sf, env.supply_capacity)
    assert np.array_equal(out["actions"].cpu().numpy(), e_act)
    assert np.array_equal(out["obs"].cpu().numpy(), e_obs)
    assert np.array_equal(out["reward"].cpu().numpy().view(np.uint64), e_rew.view(np.uint64))
    assert np.array_equal(met.cpu().numpy().view(np.uint64), e_sum.view(np.uint64))
    assert bool(out["truncated"][-1].all()) and not bool(out["truncated"][:-1].any())


@pytest.mark.gpu
@pytest.mark.parametrize("sf,L", [(1.0, 5), (1.2, 5), (1.0, 0), (0.9, 7)])
def test_order_up_to_vs_oracle(gpu, oracle, sf, L):
    import torch
    import invsim
    n = 700
    env = invsim.NewsvendorEnv(n, device=gpu, lead_time=L, autoreset_mode="disabled")
    orc = oracle.OracleNewsvendor(n, lead_time=L)
    orc.seed(range(900, 900 + n))
    o0 = orc.reset()
    env.reset(seed=900)
    met = torch.zeros((n, 2), dtype=torch.float64, device=gpu)
    out = env.rollout_policy(invsim.OrderUpToHeuristicAgent(sf), 40, obs=True, actions=True, metrics=met)
    e_act, e_rew, e_obs, e_sum = agents.run_newsvendor(orc, o0, 40, L, sf, 2000)
    assert np.array_equal(out["actions"].cpu().numpy().view(np.uint32), e_act.view(np.uint32))
    assert np.array_equal(out["obs"].cpu().numpy().view(np.uint32), e_obs.view(np.uint32))
    assert np.array_equal(out["reward"].cpu().numpy().view(np.uint64), e_rew.view(np.uint64))
    assert np.array_equal(met.cpu().numpy().view(np.uint64), e_sum.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("graph,frac", [("default", 0.1), ("custom", 0.1), ("default", 0.013)])
def test_constant_order_net_vs_oracle(gpu, oracle, graph, frac):
    import torch
    import invsim
    from invsim.topology import custom_graph, default_graph
    n = 640
    g = default_graph() if graph == "default" else custom_graph()
    env = invsim.NetInvMgmtBacklogEnv(n, device=gpu, graph=g, autoreset_mode="disabled")
    agent = invsim.ConstantOrderAgent(frac)
    a = agent.action(env)
    assert a.dtype == np.float32
    orc = oracle.OracleNet(n, graph=g)
    orc.seed(range(31, 31 + n))
    o0 = orc.reset()
    env.reset(seed=31)
    met = torch.zeros((n, invsim.policies.metrics_dim(env)), dtype=torch.float64, device=gpu)
    out = env.rollout_policy(agent, 30, obs=True, actions=True, metrics=met)
    e_rew, e_obs, e_sum = agents.run_net(orc, o0, 30, a)
    assert np.array_equal(out["actions"].cpu().numpy(), np.broadcast_to(a, (30, n, len(a))))
    assert np.array_equal(out["obs"].cpu().numpy().view(np.uint32), e_obs.view(np.uint32))
    assert np.array_equal(out["reward"].cpu().numpy().view(np.uint64), e_rew.view(np.uint64))
    assert np.array_equal(met.cpu().numpy().view(np.uint64), e_sum.view(np.uint64))


@pytest.mark.gpu
def test_policy_rollout_chains_and_replays(gpu):
    """Metrics accumulate across launches; the actions the agent took, replayed
    through the ordinary rollout on a clone, give the same trajectory (incl.
    NEXT_STEP autoresets)."""
    import torch
    import invsim
    n = 513
    e1 = invsim.InvManagementBacklogEnv(n, device=gpu)
    e2 = invsim.InvManagementBacklogEnv(n, device=gpu)
    e3 = invsim.InvManagementBacklogEnv(n, device=gpu)
    for e in (e1, e2, e3):
        e.reset(seed=77)
    ag = invsim.BaseStockAgent(1.1)
    m1 = torch.zeros((n, 6), dtype=torch.float64, device=gpu)
    m2 = torch.zeros_like(m1)
    full = e1.rollout_policy(ag, 75, obs=True, actions=True, metrics=m1)
    p1 = e2.rollout_policy(ag, 20, obs=True, metrics=m2)
    p2 = e2.rollout_policy(ag, 55, obs=True, metrics=m2)
    assert torch.equal(m1, m2)
    assert torch.equal(full["obs"], torch.cat([p1["obs"], p2["obs"]]))
    obs, rew, te, tr = e3.rollout(full["actions"])
    assert torch.equal(obs, full["obs"]) and torch.equal(rew, full["reward"]) and torch.equal(tr, full["truncated"])
    assert torch.equal(e1.get_state(), e3.get_state())


@pytest.mark.gpu
def test_evaluate_agent_columns(gpu, oracle):
    import invsim
    res = invsim.evaluate_agent(invsim.BaseStockAgent(1.0), invsim.InvManagementBacklogEnv,
                                {"periods": 30}, n_episodes=200, seed_offset=1000, device=gpu)
    orc = oracle.OracleInvMgmt(200)
    orc.seed(range(1000, 1200))
    o0 = orc.reset()
    _, _, _, s = agents.run_invmgmt(orc, o0, 30, np.array([1, 5, 10]), 20, 1.0, np.array([100, 200, 230]))
    assert np.array_equal(res["TotalReward"], s[:, 0])
    assert res["Steps"].tolist() == [30] * 200
    sl = [sa / max(1e-6, d) if d > 1e-6 else 1.0 for sa, d in zip(s[:, 3], s[:, 2])]
    assert np.array_equal(res["AvgServiceLevel"], np.array(sl))
    assert np.array_equal(res["AvgEndingInv"], s[:, 5] / 30)
    assert res["Seed"].tolist() == list(range(1000, 1200)) and res["Agent"][0] == "BaseStock_SF=1.0"
