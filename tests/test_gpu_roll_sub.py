"""The 2-role InvMgmt rollout (im_roll3_kernel) as back-to-back launches over
sub-ranges of the env groups (INVSIM_IM_ROLL_SUB, a launch-shape knob): the
same outputs, state and episode-sink partials as one launch over every group
(INVSIM_IM_ROLL_SUB=0),
bit for bit (inventory_management.py:224-352 per env; the groups are
independent)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,sub", [(65536 + 3 * 64 + 5, 4096), (40000, 16384),
                                   (2 * 65536 + 5 * 64 + 3, None)])   # None: the default, 65 536
def test_roll_sub_launches_equal_one_launch(gpu, monkeypatch, n, sub):
    import invsim
    from invsim.distributed import EpisodeStats
    monkeypatch.setenv("INVSIM_IM_ROLL3O_MAX_N", "0")       # the 2-role kernel at every size
    monkeypatch.setenv("INVSIM_IM_ROLL_SUB", "0")           # one launch over every group
    ref = invsim.InvManagementBacklogEnv(n, device=gpu)
    if sub is None:
        monkeypatch.delenv("INVSIM_IM_ROLL_SUB")
    else:
        monkeypatch.setenv("INVSIM_IM_ROLL_SUB", str(sub))
    env = invsim.InvManagementBacklogEnv(n, device=gpu)
    monkeypatch.delenv("INVSIM_IM_ROLL_SUB", raising=False)
    monkeypatch.delenv("INVSIM_IM_ROLL3O_MAX_N")
    stats = []
    for x in (env, ref):
        x.reset(seed=77)
        st = EpisodeStats(n, gpu)
        st.attach(x)
        stats.append(st)
    g = torch.Generator(device=gpu).manual_seed(3)
    for K in (30, 17, 45):
        a = torch.randint(-5, 240, (K, n, 3), device=gpu, generator=g)
        outs = [x.rollout(a) for x in (env, ref)]
        for p, q in zip(outs[0], outs[1]):
            assert torch.equal(p, q), K
        assert torch.equal(env.get_state(), ref.get_state()), K
    torch.cuda.synchronize()
    for name in ("ret", "part"):
        u, v = (getattr(st, name).cpu().numpy().view(np.int64) for st in stats)
        assert np.array_equal(u, v), name
