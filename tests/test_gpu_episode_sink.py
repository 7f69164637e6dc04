"""The episode sink (invsim_set_episode_sink): the
evaluation harness's running returns (benchmark_InvManagementBacklogEnv.py:
371, 386, 434) folded inside the step / rollout kernels.

* fused == fold: an env with the sink attached and a twin env whose outputs
  are folded afterwards by invsim_episode_fold_groups, launch by launch, give
  the same running returns and the same per-group partials, bit for bit (the
  kernels run the fold's per-lane code on the rows they produce);
* returns == oracle: the per-env running returns equal the C oracle's rewards
  summed in step order, bit for bit, and the finished-episode statistics its
  episode sums;
* the other families (no in-kernel fold) take the fallback fold of their
  outputs, with the same bits as an explicit fold.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.detach().cpu().numpy().view(np.int64)


def _twins(cls, n, seed, gpu):
    from invsim.distributed import EpisodeStats
    a, b = cls(n, device=gpu), cls(n, device=gpu)
    a.reset(seed=seed)
    b.reset(seed=seed)
    sa, sb = EpisodeStats(n, gpu), EpisodeStats(n, gpu)
    sa.attach(a)
    return a, b, sa, sb


def _im_actions(g, K, n, gpu):
    shape = (K, n, 3) if K else (n, 3)
    return torch.randint(-5, 240, shape, device=gpu, generator=g)


def _check(sa, sb, where):
    torch.cuda.synchronize()
    assert np.array_equal(_bits(sa.ret), _bits(sb.ret)), f"{where}: running returns"
    assert np.array_equal(_bits(sa.part), _bits(sb.part)), f"{where}: group partials"


@pytest.mark.parametrize("cls_name,n", [("InvManagementBacklogEnv", 65536),      # im_split + im_roll3
                                        ("InvManagementBacklogEnv", 4099),       # im_roll3o, a partial group
                                        ("InvManagementLostSalesEnv", 32768)])   # im_roll3o (config 4 shard)
def test_sink_fused_equals_fold(gpu, cls_name, n):
    import invsim
    a, b, sa, sb = _twins(getattr(invsim, cls_name), n, 41, gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(n)
    # single steps across a NEXT_STEP reset (steps 0..29, the reset step, 0..8)
    for k in range(40):
        act = _im_actions(g, 0, n, gpu)
        a.step(act)
        _, r, te, tr, _ = b.step(act)
        sb.update_block(r.reshape(1, -1), te.reshape(1, -1), tr.reshape(1, -1))
        if k in (0, 29, 30, 39):
            _check(sa, sb, f"step {k}")
    # fused rollouts of several lengths, across resets, then steps again
    for K in (30, 17, 45, 2):
        act = _im_actions(g, K, n, gpu)
        a.rollout(act)
        _, r, te, tr = b.rollout(act)
        sb.update_block(r.contiguous(), te.contiguous(), tr.contiguous())
        _check(sa, sb, f"rollout K={K}")
    for k in range(5):
        act = _im_actions(g, 0, n, gpu)
        a.step(act)
        _, r, te, tr, _ = b.step(act)
        sb.update_block(r.reshape(1, -1), te.reshape(1, -1), tr.reshape(1, -1))
    _check(sa, sb, "steps after the rollouts")
    assert float(sa.acc[2]) == 4 * n            # four episodes finished (steps 29; rollouts 30 and 45 twice)
    sa.detach()
    a.step(_im_actions(g, 0, n, gpu))            # detached: nothing more is folded
    _check(sa, sb, "after detach")


def test_sink_policy_rollout_equals_fold(gpu):
    """in-kernel BaseStock agent (im_roll3 / im_roll3o with POL): the sink
    folds the rewards the kernel computes"""
    import invsim
    from invsim.policies import BaseStockAgent
    for n in (65536, 8192):
        a, b, sa, sb = _twins(invsim.InvManagementBacklogEnv, n, 5, gpu)
        for K in (30, 31, 7):
            a.rollout_policy(BaseStockAgent(1.0), K)
            out = b.rollout_policy(BaseStockAgent(1.0), K)
            r, te, tr = out["reward"], out["terminated"], out["truncated"]
            sb.update_block(r.contiguous(), te.contiguous(), tr.contiguous())
            _check(sa, sb, f"policy n={n} K={K}")


@pytest.mark.parametrize("cls_name", ["NewsvendorEnv", "NetInvMgmtBacklogEnv"])
def test_sink_fallback_families(gpu, cls_name):
    """families without the in-kernel fold: the library folds each launch's
    output rows (invsim_episode_fold_groups on the launch stream)"""
    import invsim
    n = 4096 + 3
    cls = getattr(invsim, cls_name)
    a, b, sa, sb = _twins(cls, n, 9, gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(1)
    A = b.action_dim
    hi = 300.0
    T = a._horizon() + 1
    for k in range(T + 3):
        act = torch.rand((n, A), device=gpu, generator=g) * hi
        a.step(act)
        _, r, te, tr, _ = b.step(act)
        sb.update_block(r.reshape(1, -1), te.reshape(1, -1), tr.reshape(1, -1))
    act = torch.rand((2 * T, n, A), device=gpu, generator=g) * hi
    a.rollout(act)
    _, r, te, tr = b.rollout(act)
    sb.update_block(r.contiguous(), te.contiguous(), tr.contiguous())
    _check(sa, sb, cls_name)
    assert float(sa.acc[2]) == 3 * n


def test_sink_returns_vs_oracle(gpu, oracle):
    """running returns bit-exact against the oracle's rewards summed in step
    order; finished-episode sums against the oracle's episodes"""
    import invsim
    from invsim.distributed import EpisodeStats
    n = 2048 + 5
    env = invsim.InvManagementBacklogEnv(n, device=gpu)
    st = EpisodeStats(n, gpu)
    env.reset(seed=123)
    st.attach(env)
    orc = oracle.OracleInvMgmt(n, backlog=True)
    orc.seed(range(123, 123 + n))
    orc.reset()
    rng = np.random.default_rng(2)
    acts = rng.integers(0, 230, size=(80, n, 3)).astype(np.int64)
    dev = torch.from_numpy(acts).to(gpu)
    env.rollout(dev[:25])                      # periods 0..24
    for k in range(25, 50):                    # 25..29, reset, 0..18
        env.step(dev[k])
    env.rollout(dev[50:80])                    # 19..29, reset, 0..17
    ret = np.zeros(n)
    fin = []
    t = 0
    for k in range(80):
        if t >= 30:
            orc.reset()
            t = 0
            continue
        _, r, tr = orc.step(acts[k])
        ret = ret + r
        t += 1
        if tr.all():
            fin.append(ret)
            ret = np.zeros(n)
    torch.cuda.synchronize()
    assert np.array_equal(st.ret.cpu().numpy().view(np.int64), ret.view(np.int64))
    fin = np.stack(fin)
    res = st.allreduce()
    assert res["episodes"] == fin.size
    assert res["sum"] == pytest.approx(fin.sum(), rel=1e-12)
    assert res["sum_sq"] == pytest.approx((fin * fin).sum(), rel=1e-12)


def test_sink_refuses_missing_rewards(gpu):
    import invsim
    from invsim.distributed import EpisodeStats
    n = 256
    env = invsim.InvManagementBacklogEnv(n, device=gpu)
    env.reset(seed=0)
    st = EpisodeStats(n, gpu)
    st.attach(env)
    a = torch.zeros((n, 3), dtype=torch.int64, device=gpu)
    obs = torch.empty((n, env.obs_dim), dtype=torch.int64, device=gpu)
    rc = env._lib.invsim_step(env._h, a.data_ptr(), obs.data_ptr(), None, None, None, None, None)
    assert rc == -22                                     # INVSIM_EINVAL: no reward outputs to fold
    with pytest.raises(ValueError):
        EpisodeStats(n + 1, gpu).attach(env)
