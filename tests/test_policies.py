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


def _two_retailer_graph():
    """A graph outside the compiled specialisations (generic kernel): the
    default network with a second retailer off distributor 3."""
    from invsim.topology import default_graph
    g = default_graph()
    g.add_nodes_from([9], I0=60, h=0.025)
    g.add_edge(9, 0, p=2.5, b=0.2, demand_dist_func="poisson", dist_param={"lam": 7})
    g.add_edge(3, 9, L=2, p=1.4, g=0.012)
    return g


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["two_retailer", "forced_generic"])
def test_constant_order_generic_kernel_vs_oracle(gpu, oracle, monkeypatch, which):
    """ConstantOrderAgent rollouts on the table-walking kernel (any graph):
    same actions, obs, rewards and evaluate_agent metrics as the oracle."""
    import torch
    import invsim
    from invsim.topology import default_graph
    n = 300
    if which == "forced_generic":
        monkeypatch.setenv("INVSIM_NET_GENERIC", "1")
        g = default_graph()
    else:
        g = _two_retailer_graph()
    env = invsim.NetInvMgmtBacklogEnv(n, device=gpu, graph=g, autoreset_mode="next_step", num_periods=12)
    assert env.kernel_variant == 0
    agent = invsim.ConstantOrderAgent(0.07)
    a = agent.action(env)
    orc = oracle.OracleNet(n, graph=g, num_periods=12)
    orc.seed(range(44, 44 + n))
    o0 = orc.reset()
    env.reset(seed=44)
    met = torch.zeros((n, invsim.policies.metrics_dim(env)), dtype=torch.float64, device=gpu)
    out = env.rollout_policy(agent, 12, obs=True, actions=True, metrics=met)
    e_rew, e_obs, e_sum = agents.run_net(orc, o0, 12, a)
    assert np.array_equal(out["actions"].cpu().numpy(), np.broadcast_to(a, (12, n, len(a))))
    assert np.array_equal(out["obs"].cpu().numpy().view(np.uint32), e_obs.view(np.uint32))
    assert np.array_equal(out["reward"].cpu().numpy().view(np.uint64), e_rew.view(np.uint64))
    assert np.array_equal(met.cpu().numpy().view(np.uint64), e_sum.view(np.uint64))
    # metrics only (no per-step outputs), across the NEXT_STEP autoreset, chained
    met2 = torch.zeros_like(met)
    env.reset(seed=44)
    env.rollout_policy(agent, 5, metrics=met2)
    env.rollout_policy(agent, 7, metrics=met2)
    assert torch.equal(met2, met)
    out = env.rollout_policy(agent, 2, obs=True)
    assert (out["reward"][0] == 0).all()             # the reset step of NEXT_STEP


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


# ---- ClassicNewsvendorAgent / sSPolicyAgent: scipy.stats.poisson.ppf on device ----
# The third-party scipy (1.15.3 here and on the GPU box) is the pin: the agents'
# oracle calls poisson.ppf itself, as the reference does.  tests/ppf_model.py
# is the device algorithm in Python.

def _ppf_boundary_cases(rng, n_mu):
    """(q, mu) float32 pairs where scipy's float32 loops decide: q a few ulps
    around CDF(j), and q putting pdtrik's root x* just below / above the f32
    rounding midpoint above an integer."""
    from scipy import special
    f32 = np.float32
    out = []
    for _ in range(n_mu):
        mu = f32(rng.random() * 1200 + 0.5)
        j = int(max(0, round(float(mu) + rng.normal() * np.sqrt(float(mu)) * 2)))
        q0 = f32(special.pdtr(j, float(mu)))
        for d in range(-3, 4):
            q = q0
            for _ in range(abs(d)):
                q = np.nextafter(q, f32(1) if d > 0 else f32(0))
            out.append((q, mu))
        if j >= 1:
            half = 2.0 ** (np.floor(np.log2(j)) - 24)
            for t in (0.5, 0.9, 1.1, 1.5):
                out.append((f32(special.gammaincc(j + 1 + half * t, float(mu))), mu))
    return [(q, mu) for q, mu in out if 0 < q < 1]


def test_ppf_model_vs_scipy_random():
    from scipy.stats import poisson
    import ppf_model
    f32 = np.float32
    rng = np.random.default_rng(5)
    for it in range(3000):
        h, k, mu = f32(rng.random() * 5), f32(rng.random() * 10), f32(rng.random() * 200)
        L, sf = [0, 1, 5, 9][it % 4], [1.0, 1.2, 0.8, 2.0][(it // 4) % 4]
        q = k / (h + k)
        eff = mu * (L + 1) * sf
        m = max(1e-6, eff)
        exp = float(poisson.ppf(q, mu=m))
        assert ppf_model.ppf(float(q), float(m), isinstance(m, np.float32)) == exp, (q, m)


def test_ppf_model_vs_scipy_float32_boundaries():
    """Near the boundaries scipy's float32 loops decide the answer: the model
    matches scipy where a float64 inverse does not."""
    from scipy.stats import poisson
    import ppf_model
    cases = _ppf_boundary_cases(np.random.default_rng(11), 400)
    assert len(cases) > 3000
    plain_wrong = 0
    for q, mu in cases:
        exp = float(poisson.ppf(q, mu=mu))
        assert ppf_model.ppf(float(q), float(mu), True) == exp, (float(q), float(mu))
        plain_wrong += ppf_model.ppf(float(q), float(mu), False) != exp
    assert plain_wrong > len(cases) // 10


def test_classic_nv_restatement_hand_cases():
    from scipy.stats import poisson
    f32 = np.float32
    obs = np.zeros((4, 7), np.float32)
    obs[:, :5] = [[50, 20, 2, 6, 30], [50, 20, 0, 0, 30], [10, 20, 1, 3, 12.5], [50, 20, 2, 6, 30]]
    obs[3, 5:] = [400, 500]
    a = agents.classic_nv(obs, 2, 1.0, 2000)
    assert a.dtype == np.float32
    assert a[0, 0] == poisson.ppf(f32(6) / f32(8), mu=f32(90))              # k / (h + k)
    assert a[1, 0] == f32(30) * 3                                           # h + k = 0: fallback
    assert a[3, 0] == 0.0                                                   # position above the level
    b = agents.classic_nv(obs, 2, 1.0, 2000, "profit_margin")
    assert b[2, 0] == f32(12.5) * 3                                         # p - c + k <= 0: fallback
    u = f32(50) - f32(20) + f32(6)
    assert b[0, 0] == poisson.ppf(u / (u + f32(2)), mu=f32(90))
    s = agents.ss_policy(obs, 2, 1.2, 2000)
    lvl = poisson.ppf(f32(0.75), mu=f32(90))
    assert s[0, 0] == f32(lvl * 1.2) and s[1, 0] == 0.0 and s[3, 0] == 0.0


def _nv_pair(gpu, oracle, n, L, seed):
    import invsim
    env = invsim.NewsvendorEnv(n, device=gpu, lead_time=L, autoreset_mode="disabled")
    orc = oracle.OracleNewsvendor(n, lead_time=L)
    orc.seed(range(seed, seed + n))
    o0 = orc.reset()
    env.reset(seed=seed)
    return env, orc, o0


@pytest.mark.gpu
@pytest.mark.parametrize("cr,sf,L", [("k_vs_h", 1.0, 5), ("k_vs_h", 1.3, 2), ("profit_margin", 1.0, 5),
                                     ("profit_margin", 0.7, 0), ("other", 1.0, 9)])
def test_classic_nv_vs_oracle(gpu, oracle, cr, sf, L):
    import torch
    import invsim
    n = 500
    env, orc, o0 = _nv_pair(gpu, oracle, n, L, 2000)
    met = torch.zeros((n, 2), dtype=torch.float64, device=gpu)
    out = env.rollout_policy(invsim.ClassicNewsvendorAgent(cr, sf), 40, obs=True, actions=True, metrics=met)
    e_act, e_rew, e_obs, e_sum = agents.run_newsvendor(orc, o0, 40, L, sf, 2000, "classic_nv", cr)
    assert np.array_equal(out["actions"].cpu().numpy().view(np.uint32), e_act.view(np.uint32))
    assert np.array_equal(out["obs"].cpu().numpy().view(np.uint32), e_obs.view(np.uint32))
    assert np.array_equal(out["reward"].cpu().numpy().view(np.uint64), e_rew.view(np.uint64))
    assert np.array_equal(met.cpu().numpy().view(np.uint64), e_sum.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("sbf,L", [(1.2, 5), (1.0, 0), (2.5, 3)])
def test_ss_policy_vs_oracle(gpu, oracle, sbf, L):
    import torch
    import invsim
    n = 500
    env, orc, o0 = _nv_pair(gpu, oracle, n, L, 3000)
    met = torch.zeros((n, 2), dtype=torch.float64, device=gpu)
    out = env.rollout_policy(invsim.sSPolicyAgent(0.5, sbf), 40, obs=True, actions=True, metrics=met)
    e_act, e_rew, e_obs, e_sum = agents.run_newsvendor(orc, o0, 40, L, sbf, 2000, "ss")
    assert np.array_equal(out["actions"].cpu().numpy().view(np.uint32), e_act.view(np.uint32))
    assert np.array_equal(out["reward"].cpu().numpy().view(np.uint64), e_rew.view(np.uint64))
    assert np.array_equal(met.cpu().numpy().view(np.uint64), e_sum.view(np.uint64))


@pytest.mark.gpu
def test_classic_nv_ppf_boundaries_on_device(gpu):
    """Episode params injected (set_state) so that k / (h + k) and mu sit on
    the float32 decision boundaries of scipy's ppf; the first action is the
    ppf level itself (empty pipeline, L = 0)."""
    import invsim
    import ppf_model
    f32 = np.float32
    pairs = []
    for q, mu in _ppf_boundary_cases(np.random.default_rng(23), 250):
        k = f32(float(q) / (1.0 - float(q)))
        for _ in range(8):                                  # f32 k with f32(k / (1 + k)) == q
            r = k / (f32(1) + k)
            if r == q:
                pairs.append((k, mu))
                break
            k = np.nextafter(k, f32(np.inf) if r < q else f32(0))
    assert len(pairs) > 1000
    n = len(pairs)
    env = invsim.NewsvendorEnv(n, device=gpu, lead_time=0, autoreset_mode="disabled")
    env.reset(seed=1)
    blob = env.get_state()
    par = env.state_fields(blob)["params"]                  # [5, N] f64 bits
    p = np.zeros((5, n))
    p[0], p[1], p[2] = 50.0, 20.0, 1.0
    p[3] = [float(k) for k, _ in pairs]
    p[4] = [float(mu) for _, mu in pairs]
    par.copy_(torch_from(p, par))
    env.set_state(blob)
    out = env.rollout_policy(invsim.ClassicNewsvendorAgent(), 1, rewards=False, actions=True)
    got = out["actions"][0, :, 0].cpu().numpy()
    obs = np.zeros((n, 5), np.float32)
    obs[:] = p.T
    exp = agents.classic_nv(obs, 0, 1.0, 2000)[:, 0]
    model = np.array([ppf_model.ppf(float(k / (f32(1) + k)), float(mu), True) for k, mu in pairs], np.float32)
    assert np.array_equal(got, model)
    assert np.array_equal(got, exp)


def torch_from(a, like):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).view(torch.int64).to(like.device)


@pytest.mark.gpu
def test_classic_nv_across_autoresets(gpu, oracle):
    """NEXT_STEP autoreset inside one policy launch: the per-episode ppf level
    is recomputed for the new episode's params."""
    import invsim
    n, L = 300, 5
    env = invsim.NewsvendorEnv(n, device=gpu, lead_time=L, step_limit=12)
    orc = oracle.OracleNewsvendor(n, lead_time=L, step_limit=12)
    orc.seed(range(70, 70 + n))
    o0 = orc.reset()
    env.reset(seed=70)
    out = env.rollout_policy(invsim.ClassicNewsvendorAgent("k_vs_h", 1.1), 25, obs=True, actions=True)
    a1, r1, ob1, _ = agents.run_newsvendor(orc, o0, 12, L, 1.1, 2000, "classic_nv")
    o1 = orc.reset()
    a2, r2, ob2, _ = agents.run_newsvendor(orc, o1, 12, L, 1.1, 2000, "classic_nv")
    acts = out["actions"].cpu().numpy()
    assert np.array_equal(acts[:12], a1) and np.array_equal(acts[13:], a2)
    obs = out["obs"].cpu().numpy()
    assert np.array_equal(obs[12], o1) and np.array_equal(obs[13:], ob2)
    rew = out["reward"].cpu().numpy()
    assert np.array_equal(rew[:12], r1) and np.array_equal(rew[13:], r2) and not rew[12].any()


def test_summary_table_matches_reference_aggregation():
    """summary_table restates process_and_report_results
    (benchmark_InvManagementBacklogEnv.py:474-516): per agent mean / median /
    sample std / min / max of TotalReward, means of the per-episode metrics,
    counts and success rate, sorted by AvgReward."""
    from invsim.policies import summary_table
    rng = np.random.default_rng(3)

    def res(name, n):
        return {"Agent": [name] * n, "Episode": np.arange(1, n + 1), "TotalReward": rng.normal(size=n),
                "Steps": np.full(n, 30), "AvgServiceLevel": rng.uniform(size=n),
                "TotalStockoutQty": rng.uniform(size=n) * 9, "AvgEndingInv": rng.uniform(size=n) * 50,
                "Time": np.full(n, 1e-4), "Seed": np.arange(n), "Error": [None] * n}
    rs = [res("BaseStock", 7), res("Constant", 5)]
    t = summary_table(rs)
    for r in rs:
        row = t.loc[r["Agent"][0]]
        x = r["TotalReward"]
        assert row["AvgReward"] == pytest.approx(x.mean())
        assert row["MedianReward"] == pytest.approx(np.median(x))
        assert row["StdReward"] == pytest.approx(x.std(ddof=1))
        assert row["MinReward"] == x.min() and row["MaxReward"] == x.max()
        assert row["AvgServiceLevel"] == pytest.approx(r["AvgServiceLevel"].mean())
        assert row["AvgStockoutQty"] == pytest.approx(r["TotalStockoutQty"].mean())
        assert row["AvgEndInv"] == pytest.approx(r["AvgEndingInv"].mean())
        assert row["SuccessfulEpisodes"] == len(x) == row["EpisodesAttempted"]
        assert row["SuccessRate(%)"] == 100.0
    assert list(t.index) == sorted(t.index, key=lambda a: -t.loc[a, "AvgReward"])


@pytest.mark.gpu
@pytest.mark.parametrize("cls", ["InvManagementBacklogEnv", "InvManagementLostSalesEnv"])
@pytest.mark.parametrize("agent", ["base_stock_1.0", "base_stock_1.3", "constant"])
@pytest.mark.parametrize("n", [4096, 65536])
def test_policy_on_fused_rollout_equals_run_kernel(gpu, monkeypatch, cls, agent, n):
    """BaseStock / ConstantOrder inside the fused 2-role rollout kernel
    (im_roll3_kernel<..., POL>) give the one-wave run kernel's outputs, actions,
    metrics and final state bit for bit, across NEXT_STEP autoresets and
    chained launches (every output optional).  At 4 096 envs the 3-role
    kernel runs, once more with two groups per workgroup (INVSIM_IM_ROLL3O_G2)."""
    import torch
    import invsim
    ag = invsim.ConstantOrderAgent(0.3) if agent == "constant" else invsim.BaseStockAgent(float(agent[-3:]))
    res = []
    for roll in ("0", "1", "g2"):
        monkeypatch.setenv("INVSIM_IM_POL_ROLL", "0" if roll == "0" else "1")
        monkeypatch.setenv("INVSIM_IM_ROLL3O_G2", "1" if roll == "g2" else "0")
        env = getattr(invsim, cls)(n, device=gpu)
        env.reset(seed=21)
        m = torch.zeros((n, 6), dtype=torch.float64, device=gpu)
        a = env.rollout_policy(ag, 45, obs=True, actions=True, metrics=m)
        b = env.rollout_policy(ag, 40, obs=False, rewards=False, metrics=m)
        c = env.rollout_policy(ag, 30, obs=True, metrics=m)
        res.append((a, b, c, m, env.get_state()))
    a2, b2, c2, m2, s2 = res[0]                       # the one-wave run kernel
    for a1, b1, c1, m1, s1 in res[1:]:
        for k in a1:
            assert torch.equal(a1[k], a2[k]), k
        for k in c1:
            assert torch.equal(c1[k], c2[k]), k
        assert torch.equal(m1.view(torch.int64), m2.view(torch.int64))
        assert torch.equal(s1, s2)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["default", "custom"])
@pytest.mark.parametrize("n", [4096, 32768])
def test_constant_order_on_fused_net_rollout_equals_spec_kernel(gpu, monkeypatch, graph, n):
    """ConstantOrder inside the 3-role Net rollout kernel (net_roll3o_kernel<...,
    POL>) gives net_spec_kernel's outputs, actions, metrics and state bit for bit."""
    import torch
    import invsim
    from invsim.topology import custom_graph, default_graph
    ag = invsim.ConstantOrderAgent(0.15)
    res = []
    for roll in ("1", "0"):
        monkeypatch.setenv("INVSIM_NET_POL_ROLL", roll)
        g = default_graph() if graph == "default" else custom_graph()
        env = invsim.NetInvMgmtBacklogEnv(n, device=gpu, graph=g)
        env.reset(seed=8)
        m = torch.zeros((n, invsim.policies.metrics_dim(env)), dtype=torch.float64, device=gpu)
        a = env.rollout_policy(ag, 45, obs=True, actions=True, metrics=m)
        b = env.rollout_policy(ag, 40, obs=False, rewards=False, metrics=m)
        c = env.rollout_policy(ag, 30, obs=True, metrics=m)
        res.append((a, b, c, m, env.get_state()))
    (a1, b1, c1, m1, s1), (a2, b2, c2, m2, s2) = res
    for k in a1:
        assert torch.equal(a1[k], a2[k]), k
    for k in c1:
        assert torch.equal(c1[k], c2[k]), k
    assert torch.equal(m1.view(torch.int64), m2.view(torch.int64))
    assert torch.equal(s1, s2)


@pytest.mark.gpu
@pytest.mark.parametrize("agent", ["order_up_to", "classic_nv", "ss", "constant"])
@pytest.mark.parametrize("n,L,limit", [(4096, 5, 40), (65536, 5, 40), (5000, 2, 12), (3000, 9, 17)])
def test_newsvendor_policy_on_fused_rollout_equals_run_kernel(gpu, monkeypatch, agent, n, L, limit):
    """OrderUpTo / ClassicNV / (s, S) / ConstantOrder inside the 3-wave
    Newsvendor rollout kernel (nv_roll_kernel<LT, POL>) give nv_run_kernel's
    outputs, actions, metrics and final state bit for bit, across NEXT_STEP
    autoresets (the per-episode ppf level recomputed) and chained launches."""
    import torch
    import invsim
    ag = {"order_up_to": lambda: invsim.OrderUpToHeuristicAgent(1.2),
          "classic_nv": lambda: invsim.ClassicNewsvendorAgent("profit_margin", 0.9),
          "ss": lambda: invsim.sSPolicyAgent(0.5, 1.4),
          "constant": lambda: invsim.ConstantOrderAgent(0.05)}[agent]()
    res = []
    for roll in ("1", "0"):
        monkeypatch.setenv("INVSIM_NV_POL_ROLL", roll)
        env = invsim.NewsvendorEnv(n, device=gpu, lead_time=L, step_limit=limit)
        env.reset(seed=31)
        m = torch.zeros((n, 2), dtype=torch.float64, device=gpu)
        a = env.rollout_policy(ag, 45, obs=True, actions=True, metrics=m)
        b = env.rollout_policy(ag, 40, obs=False, rewards=False, metrics=m)
        c = env.rollout_policy(ag, 30, obs=True, metrics=m)
        res.append((a, b, c, m, env.get_state()))
    (a1, b1, c1, m1, s1), (a2, b2, c2, m2, s2) = res
    for k in a1:
        assert torch.equal(a1[k], a2[k]), k
    for k in c1:
        assert torch.equal(c1[k], c2[k]), k
    assert torch.equal(m1.view(torch.int64), m2.view(torch.int64))
    assert torch.equal(s1, s2)
