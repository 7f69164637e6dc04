"""Single-env views (invsim.compat) and the SB3 VecEnv adapter (invsim.sb3):
the reference's per-env API, step-info dicts and history attributes, checked
against the CPU oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_invmgmt_view_histories_and_info(gpu, oracle):
    import invsim.compat as compat
    env = compat.make("InvManagementBacklogEnv", device=gpu)
    orc = oracle.OracleInvMgmt(1)
    orc.seed([2024])
    o0 = orc.reset()
    obs, info = env.reset(seed=2024)
    assert np.array_equal(obs, o0[0]) and info["period"] == 0
    assert env.num_stages == 4 and env.lt_max == 10 and env.dist_param == {"mu": 20}
    rng = np.random.default_rng(0)
    for t in range(30):
        a = rng.integers(-5, 150, size=3)
        obs, r, te, tr, info = env.step(a)
        e_obs, e_rew, e_tr, ei = orc.step(a[None], info=True)
        assert np.array_equal(obs, e_obs[0]) and r == float(e_rew[0]) and tr == bool(e_tr[0])
        S, U = ei["sales"][0], ei["unfulfilled"][0]
        assert np.array_equal(env.S[t], S) and np.array_equal(info["sales"], S)
        assert np.array_equal(info["unfulfilled"], U) and env.D[t] == ei["demand"][0] == info["demand_realized"]
        assert np.array_equal(env.I[t + 1], ei["ending_inventory"][0]) and np.array_equal(env.B[t + 1], U)
        assert np.array_equal(env.action_log[t], np.maximum(a, 0)) and np.array_equal(env.R[t], S[1:])
        assert env.P[t] == np.float32(r) and env.period == t + 1
        # the reference's cost components, recomputed with numpy from S, U, I (inventory_management.py:314-320)
        rev = env.unit_price * S
        pro = env.unit_cost * S
        hol = env.holding_cost * np.maximum(0, np.append(env.I[t + 1], 0))
        pen = env.demand_cost * U
        assert info["revenue"] == rev.sum() and info["procurement_cost"] == pro.sum()
        assert info["holding_cost"] == hol.sum() and info["penalty_cost"] == pen.sum()
        assert info["period_profit"] == np.sum(rev - pro - hol - pen)
    with pytest.raises(IndexError):
        env.step(np.array([1, 1, 1]))


@pytest.mark.parametrize("graph", ["default", "custom"])
def test_net_view_dataframes(gpu, oracle, graph):
    import invsim.compat as compat
    from invsim.topology import custom_graph, default_graph
    g = default_graph() if graph == "default" else custom_graph()
    env = compat.make("NetInvMgmtBacklogEnv", device=gpu, graph=g)
    orc = oracle.OracleNet(1, graph=g)
    orc.seed([7])
    o0 = orc.reset()
    obs, info = env.reset(seed=7)
    assert np.array_equal(obs, o0[0])
    rng = np.random.default_rng(1)
    for t in range(30):
        a = rng.uniform(0, 150, size=env.action_space.shape).astype(np.float32)
        obs, r, te, tr, info = env.step(a)
        e_obs, e_rew, e_tr, ei = orc.step(a[None], info=True)
        assert np.array_equal(obs.view(np.uint32), e_obs[0].view(np.uint32)) and r == float(e_rew[0])
        assert np.array_equal(env.X.iloc[t + 1].to_numpy(), ei["X"][0])
        assert np.array_equal(env.U.iloc[t + 1].to_numpy(), ei["U"][0])
        assert np.array_equal(env.D.iloc[t].to_numpy(), ei["D"][0])
        assert np.array_equal(env.R.iloc[t].to_numpy(), ei["R"][0])
        assert np.array_equal(env.Y.iloc[t + 1].to_numpy(), ei["Y"][0])
        assert np.array_equal(env.P.iloc[t].to_numpy(), ei["P"][0])
        assert np.array_equal(env.S.loc[t, env.retail_links].to_numpy(dtype=np.float64), ei["S"][0])
        assert info["period"] == t + 1 and "demand_prev" in info


def test_newsvendor_view(gpu, oracle):
    import invsim.compat as compat
    env = compat.make("NewsvendorEnv", device=gpu)
    orc = oracle.OracleNewsvendor(1)
    orc.seed([99])
    o0 = orc.reset()
    obs, info = env.reset(seed=99)
    assert np.array_equal(obs.view(np.uint32), o0[0].view(np.uint32))
    assert info["price"] == orc.params()[0][0] and info["lead_time"] == 5
    for t in range(40):
        a = np.array([37.5 + t], np.float32)
        obs, r, te, tr, info = env.step(a)
        e_obs, e_rew, e_tr, e_dem = orc.step(a[None])
        assert np.array_equal(obs.view(np.uint32), e_obs[0].view(np.uint32)) and r == float(e_rew[0])
        assert info["demand"] == e_dem[0] and info["step_count"] == t + 1 and tr == bool(e_tr[0])


def test_sb3_vecenv_autoreset_semantics(gpu):
    import torch
    import invsim
    from invsim.sb3 import InvSimVecEnv
    n = 8
    venv = InvSimVecEnv(invsim.InvManagementBacklogEnv, n, device=gpu, seed=3)
    ref = invsim.InvManagementBacklogEnv(n, device=gpu, autoreset_mode="next_step")
    obs = venv.reset()
    r_obs, _ = ref.reset(seed=3)
    assert isinstance(obs, np.ndarray) and np.array_equal(obs, r_obs.cpu().numpy())
    a = np.full((n, 3), 40, np.int64)
    for t in range(30):
        obs, rew, dones, infos = venv.step(a)
        r_obs, r_rew, _, r_tr, _ = ref.step(torch.as_tensor(a, device=gpu))
        assert rew.dtype == np.float32 and np.array_equal(rew, r_rew.cpu().numpy().astype(np.float32))
        if t < 29:
            assert not dones.any() and np.array_equal(obs, r_obs.cpu().numpy())
    assert dones.all() and all(i["TimeLimit.truncated"] for i in infos)
    assert np.array_equal(np.stack([i["terminal_observation"] for i in infos]), r_obs.cpu().numpy())
    r_obs, *_ = ref.step(torch.as_tensor(a, device=gpu))      # NEXT_STEP: the reset happens now
    assert np.array_equal(obs, r_obs.cpu().numpy())            # SB3: the reset obs came with the done step
    assert venv.get_attr("num_stages") == [4] * n and venv.env_is_wrapped(object) == [False] * n


def test_rllib_env_creator(gpu):
    from invsim.sb3 import rllib_env_creator
    env = rllib_env_creator({"env_class": "NetInvMgmtLostSalesEnv", "num_periods": 30, "device": gpu})
    obs, info = env.reset(seed=1)
    assert obs.shape == env.observation_space.shape and env.num_periods == 30
    obs, r, te, tr, info = env.step(env.action_space.sample() if hasattr(env.action_space, "sample")
                                    else np.zeros(env.action_space.shape, np.float32))
    assert isinstance(r, float) and env.period == 1
