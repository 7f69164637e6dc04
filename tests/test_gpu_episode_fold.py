"""HIP episodic-return fold (invsim_episode_fold) against a numpy restatement
of EpisodeStats' arithmetic, and against the returns of a real rollout."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _numpy_fold(rew, done, ret0):
    ret = ret0.copy()
    s = s2 = c = 0.0
    for k in range(rew.shape[0]):
        ret += rew[k]
        d = done[k]
        s += ret[d].sum()
        s2 += (ret[d] ** 2).sum()
        c += d.sum()
        ret[d] = 0.0
    return ret, np.array([s, s2, c, rew.sum()])


@pytest.mark.parametrize("N", [1, 63, 65536 + 17])
def test_episode_fold_kernel_vs_numpy(gpu, N):
    from invsim.distributed import EpisodeStats
    rng = np.random.default_rng(N)
    K = 31
    st = EpisodeStats(N, gpu)
    ret0 = np.zeros(N)
    acc = np.zeros(4)
    for rep in range(3):
        rew = rng.normal(size=(K, N)) * 1e3
        term = rng.random((K, N)) < 0.02
        trunc = rng.random((K, N)) < 0.04
        tt = torch.from_numpy(term).to(gpu) if rep != 1 else None       # a NULL flag stream
        if rep == 1:
            term[:] = False
        st.update_block(torch.from_numpy(rew).to(gpu), tt, torch.from_numpy(trunc).to(gpu))
        ret0, a = _numpy_fold(rew, term | trunc, ret0)
        acc += a
    torch.cuda.synchronize()
    # per-env running returns: same additions in the same order -> exact
    assert np.array_equal(st.ret.cpu().numpy(), ret0)
    got = st.acc.cpu().numpy()
    assert got[2] == acc[2]
    assert np.allclose(got, acc, rtol=1e-12, atol=1e-6)


def test_episode_fold_matches_rollout_returns(gpu):
    import invsim
    N, K = 4096, 62
    env = invsim.InvManagementBacklogEnv(N, device=gpu)
    env.reset(seed=3)
    g = torch.Generator(device=gpu)
    g.manual_seed(0)
    acts = torch.randint(0, 100, (K, N, 3), device=gpu, generator=g)
    obs, rew, term, trunc = env.rollout(acts)[:4]
    from invsim.distributed import EpisodeStats
    st = EpisodeStats(N, gpu)
    st.update_block(rew.contiguous(), term.contiguous(), trunc.contiguous())
    r = rew.cpu().numpy()
    ep = r[:30].sum(0)          # periods 1..30; step 30 is the NEXT_STEP reset, 31..60 the second episode
    ep2 = r[31:61].sum(0)
    res = st.allreduce()
    assert res["episodes"] == 2 * N
    assert res["sum"] == pytest.approx(ep.sum() + ep2.sum(), rel=1e-12)
    assert res["sum_sq"] == pytest.approx((ep * ep).sum() + (ep2 * ep2).sum(), rel=1e-12)
