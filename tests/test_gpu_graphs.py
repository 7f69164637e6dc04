"""HIP-graph capture of a step loop (invsim.graphs.StepGraph over
invsim_capture_begin / _end): replays of a captured policy + env.step loop are
bit-identical to the same loop run eagerly on a twin env, for every family and
autoreset mode; captures that would not replay from where they were recorded,
and calls that cannot be captured, are refused loudly."""
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 4096


def _im_policy(o):
    return o[:, :3] % 97 + 5                               # int64 [N, 3]


def _nv_policy(o):
    return o[:, 4:5] * 1.1 + o[:, 5:6] * 0.25              # f32 [N, 1], mu and a pipeline slot


def _net_policy(o):
    return torch.remainder(o[:, :11], 50.0) + 10.0         # f32 [N, 11]


def _make(family, gpu, autoreset="next_step", **kw):
    import invsim
    if family == "invmgmt":
        return invsim.InvManagementBacklogEnv(N, device=gpu, autoreset_mode=autoreset, **kw), _im_policy
    if family == "lostsales":
        return invsim.InvManagementLostSalesEnv(N, device=gpu, autoreset_mode=autoreset, **kw), _im_policy
    if family == "newsvendor":
        return invsim.NewsvendorEnv(N, device=gpu, autoreset_mode=autoreset, **kw), _nv_policy
    return invsim.NetInvMgmtBacklogEnv(N, device=gpu, autoreset_mode=autoreset, **kw), _net_policy


def _cycle(env):
    h = env._horizon()
    return h + 1 if env.autoreset_mode == "next_step" else h


def _loop(env, policy, obs, steps):
    def fn():
        o, rews, dones = obs, [], []
        for _ in range(steps):
            o, r, te, tr, _ = env.step(policy(o))
            rews.append(r)
            dones.append(tr)
        obs.copy_(o)
        return torch.stack(rews), torch.stack(dones)
    return fn


@pytest.mark.parametrize("family,autoreset", [("invmgmt", "next_step"), ("invmgmt", "same_step"),
                                              ("lostsales", "next_step"), ("newsvendor", "next_step"),
                                              ("net", "next_step"), ("net", "same_step")])
def test_graph_replays_equal_eager_loop(gpu, family, autoreset):
    env, policy = _make(family, gpu, autoreset)
    twin, _ = _make(family, gpu, autoreset)
    C = _cycle(env)
    obs_g = env.reset(seed=11)[0].clone()
    obs_e = twin.reset(seed=11)[0].clone()
    g = env.capture(_loop(env, policy, obs_g, C), warmup=1)
    assert g.steps == C
    eager = _loop(twin, policy, obs_e, C)
    eager()                                                # the twin of the capture's warm-up run
    for rep in range(3):
        rew_g, done_g = g.replay()
        rew_e, done_e = eager()
        torch.cuda.synchronize(gpu)
        assert torch.equal(rew_g.view(torch.int64), rew_e.view(torch.int64)), f"rewards differ in replay {rep}"
        assert torch.equal(done_g, done_e)
        assert torch.equal(obs_g, obs_e), f"obs differ after replay {rep}"
        assert int(done_g.sum()) == N                      # one episode boundary per cycle
    assert env.position() == g.position == twin.position()


def test_graph_of_rollout_and_explicit_reset(gpu):
    """DISABLED autoreset: fn = reset + one fused K-step rollout; and a NEXT_STEP
    rollout graph. Both equal their eager twins."""
    import invsim
    env = invsim.InvManagementBacklogEnv(N, device=gpu, autoreset_mode="disabled")
    twin = invsim.InvManagementBacklogEnv(N, device=gpu, autoreset_mode="disabled")
    env.reset(seed=5)
    twin.reset(seed=5)
    H = env._horizon()
    acts = torch.randint(0, 150, (H, N, 3), device=gpu, dtype=torch.int64)

    def mk(e):
        def fn():
            o0, _ = e.reset()
            o, r, te, tr = e.rollout(acts)
            return o0, o, r, tr
        return fn
    g = env.capture(mk(env))
    eager = mk(twin)
    eager()
    for _ in range(2):
        out_g = g.replay()
        out_e = eager()
        torch.cuda.synchronize(gpu)
        for a, b in zip(out_g, out_e):
            assert torch.equal(a.view(torch.uint8), b.view(torch.uint8))

    env2 = invsim.NetInvMgmtBacklogEnv(N, device=gpu)
    twin2 = invsim.NetInvMgmtBacklogEnv(N, device=gpu)
    env2.reset(seed=8)
    twin2.reset(seed=8)
    C = env2._horizon() + 1
    acts2 = torch.rand((C, N, 11), device=gpu) * 120
    g2 = env2.capture(lambda: env2.rollout(acts2))
    twin2.rollout(acts2)
    for _ in range(2):
        out_g = g2.replay()
        out_e = twin2.rollout(acts2)
        torch.cuda.synchronize(gpu)
        for a, b in zip(out_g, out_e):
            assert torch.equal(a.view(torch.uint8), b.view(torch.uint8))


def test_graph_of_device_policy_rollout(gpu):
    import invsim
    env = invsim.InvManagementLostSalesEnv(N, device=gpu)
    twin = invsim.InvManagementLostSalesEnv(N, device=gpu)
    env.reset(seed=2)
    twin.reset(seed=2)
    C = env._horizon() + 1
    agent = invsim.BaseStockAgent()
    g = env.capture(lambda: env.rollout_policy(agent, C, obs=True))
    twin.rollout_policy(agent, C, obs=True)
    for _ in range(2):
        og = g.replay()
        oe = twin.rollout_policy(agent, C, obs=True)
        torch.cuda.synchronize(gpu)
        for k in og:
            if isinstance(og[k], torch.Tensor):
                assert torch.equal(og[k], oe[k]), k


def test_graph_refuses_partial_cycle_and_keeps_position(gpu):
    import invsim
    env, policy = _make("invmgmt", gpu)
    twin, _ = _make("invmgmt", gpu)
    obs = env.reset(seed=3)[0].clone()
    obs_t = twin.reset(seed=3)[0].clone()
    _loop(twin, policy, obs_t, 10)()                       # the failed capture's warm-up run
    with pytest.raises(invsim._capi.InvsimError, match="whole number of episode cycles"):
        env.capture(_loop(env, policy, obs, 10))
    pos = env.position()
    assert pos == twin.position()
    # nothing ran during the refused capture: eager steps still match the twin
    for _ in range(5):
        a = policy(obs)
        o1, r1, _, _, _ = env.step(a)
        o2, r2, _, _, _ = twin.step(policy(obs_t))
        assert torch.equal(o1, o2) and torch.equal(r1, r2)
        obs, obs_t = o1, o2


def test_graph_refusals(gpu):
    import invsim
    env, policy = _make("newsvendor", gpu, demand_stream="philox")
    env.reset(seed=1)
    with pytest.raises(invsim._capi.InvsimError, match="numpy demand stream"):
        env.capture(lambda: env.step(torch.zeros((N, 1), device=gpu)), warmup=0)

    env2, policy2 = _make("invmgmt", gpu)
    obs = env2.reset(seed=1)[0]
    a = policy2(obs)
    env2.step(a)
    # a capture of env.step outside the begin/end bracket fails loudly
    g = torch.cuda.CUDAGraph()
    with pytest.raises(Exception, match="invsim_capture_begin"):
        with torch.cuda.graph(g):
            env2.step(a)
    # host-synchronising calls inside the bracket are refused
    lib, h = env2._lib, env2._h
    assert lib.invsim_capture_begin(h) == 0
    try:
        with pytest.raises(invsim._capi.InvsimError, match="cannot be captured"):
            env2.get_state()
        with pytest.raises(invsim._capi.InvsimError, match="cannot be captured"):
            env2.set_demand_stream("philox")
    finally:
        assert lib.invsim_capture_end(h, None) == 0


def test_replay_checks_position(gpu):
    env, policy = _make("invmgmt", gpu)
    obs = env.reset(seed=4)[0].clone()
    g = env.capture(_loop(env, policy, obs, _cycle(env)))
    g.replay()
    env.step(policy(obs))                                  # one eager step: a partial cycle
    with pytest.raises(RuntimeError, match="position"):
        g.replay()
    for _ in range(_cycle(env) - 1):                       # close the cycle eagerly
        env.step(policy(obs))
    g.replay()
    torch.cuda.synchronize(gpu)
