"""NetInvMgmt rollouts for small per-GPU shards (SURVEY row h*, VERDICT r05
item 3): net_roll4_kernel puts the period profit on a wave of its own (the
default up to 16 384 envs), and net_rollq_kernel (opt-in) spreads one env's
edge work over a 16-lane row (clamp-scan over each supplier's links, row
gathers for the per-node sums, a node-order scan for the period profit;
netspec.hip).  Bar: bit-identical to the one-env-per-lane 3-role
net_roll3o_kernel (INVSIM_NET_ROLL4_MAX_N=0 / INVSIM_NET_ROLLQ_MAX_N=0) and
to the C oracle stepping the same seeds (network_management.py:436-635)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _eq_bits(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.uint8), b.astype(a.dtype).view(np.uint8))
    return np.array_equal(a, b)


CASES = [
    ("default", True, 4096, 30, "next_step", "numpy"),     # config 5 over 8 GPUs: 4 096 envs per rank
    ("default", True, 4099, 30, "next_step", "numpy"),     # a partial 16-env workgroup
    ("default", False, 8192, 30, "next_step", "numpy"),
    ("default", True, 1000, 4, "next_step", "numpy"),      # several resets per chunk, t < L at every step
    ("default", True, 1000, 30, "disabled", "numpy"),
    ("custom", True, 2000, 30, "next_step", "numpy"),      # three markets, three links on one supplier
    ("custom", False, 777, 3, "next_step", "numpy"),
    ("default", True, 4096, 30, "next_step", "philox"),
]


def _pair(gpu, monkeypatch, kernel, graph, backlog, n, periods, mode, stream):
    """(env on `kernel`, env on net_roll3o_kernel) with the same configuration"""
    import invsim
    from invsim.topology import custom_graph, default_graph
    mk_g = default_graph if graph == "default" else custom_graph
    mk = (lambda: invsim.NetInvMgmtMasterEnv(n, device=gpu, graph=mk_g(), backlog=backlog, num_periods=periods,
                                             autoreset_mode=mode, demand_stream=stream))
    monkeypatch.setenv("INVSIM_NET_ROLL4_MAX_N", "0")
    monkeypatch.setenv("INVSIM_NET_ROLLQ_MAX_N", "0")
    ref = mk()
    if kernel == "rollq":
        monkeypatch.setenv("INVSIM_NET_ROLLQ_MAX_N", "100000")
    else:
        monkeypatch.setenv("INVSIM_NET_ROLL4_MAX_N", "100000")
    env = mk()
    monkeypatch.delenv("INVSIM_NET_ROLL4_MAX_N")
    monkeypatch.delenv("INVSIM_NET_ROLLQ_MAX_N")
    return [env, ref]


@pytest.mark.parametrize("kernel", ["roll4", "rollq"])
@pytest.mark.parametrize("graph,backlog,n,periods,mode,stream", CASES)
def test_small_shard_rollout_equals_roll3o(gpu, monkeypatch, kernel, graph, backlog, n, periods, mode, stream):
    envs = _pair(gpu, monkeypatch, kernel, graph, backlog, n, periods, mode, stream)
    for env in envs:
        env.reset(seed=31)
    A = envs[0].action_dim
    g = torch.Generator(device=gpu).manual_seed(8)
    a = torch.rand((n, A), device=gpu, generator=g) * 250
    for env in envs:
        env.step(a)                                   # start the rollouts mid-episode
    Ks = (75, 9, 2) if mode == "next_step" else (8, 17)
    for K in Ks:
        a = torch.rand((K, n, A), device=gpu, generator=g) * 300 - 5
        a[:, ::37, 0] = 2.5                           # half-to-even ties
        a[:, ::41, 1] = 1e30                          # orders far past any inventory
        outs = [env.rollout(a) for env in envs]
        for x, y in zip(outs[0], outs[1]):
            assert torch.equal(x, y), K
        assert torch.equal(envs[0].get_state(), envs[1].get_state()), K
    if mode == "next_step":
        a = torch.rand((n, A), device=gpu, generator=g) * 250
        for x, y in zip(envs[0].step(a)[:4], envs[1].step(a)[:4]):
            assert torch.equal(x, y)


@pytest.mark.parametrize("kernel", ["roll4", "rollq"])
@pytest.mark.parametrize("graph", ["default", "custom"])
def test_small_shard_rollout_vs_oracle(gpu, oracle, monkeypatch, kernel, graph):
    """4 096 envs (one rank's shard of config 5 over 8 GPUs): a 61-step fused
    rollout across the NEXT_STEP reset, step by step against the oracle."""
    import invsim
    from invsim.topology import custom_graph, default_graph
    n, T, K = 4096, 30, 61
    g = default_graph() if graph == "default" else custom_graph()
    if kernel == "rollq":
        monkeypatch.setenv("INVSIM_NET_ROLLQ_MAX_N", "100000")   # net_rollq_kernel (opt-in)
    env = invsim.NetInvMgmtBacklogEnv(n, device=gpu, graph=g)   # net_roll4_kernel by default at this size
    monkeypatch.delenv("INVSIM_NET_ROLLQ_MAX_N", raising=False)
    orc = oracle.OracleNet(n, graph=g)
    orc.seed(range(500, 500 + n))
    e_obs = orc.reset()
    obs, _ = env.reset(seed=500)
    assert _eq_bits(obs.cpu().numpy(), e_obs)
    rng = np.random.default_rng(12)
    acts = rng.uniform(-5, 300, size=(K, n, env.action_dim)).astype(np.float32)
    acts[:, ::53, 0] = 7.5
    o, r, te, tr = env.rollout(torch.from_numpy(acts).to(gpu))
    o, r, tr = o.cpu().numpy(), r.cpu().numpy(), tr.cpu().numpy()
    t = 0
    for k in range(K):
        if t >= T:
            assert _eq_bits(o[k], orc.reset()), k
            assert (r[k] == 0).all() and not tr[k].any(), k
            t = 0
            continue
        res = orc.step(acts[k])
        assert _eq_bits(o[k], res[0]), f"obs step {k}"
        assert _eq_bits(r[k], res[1]), f"reward step {k}: max|diff| {np.abs(r[k] - res[1]).max()}"
        assert np.array_equal(tr[k], res[2]), k
        t += 1
