"""VectorEnv host-side fast paths on the GPU: the kernels run on torch's
current stream (the raw stream lookup equals torch.cuda.current_stream), and
actions already in the kernel's dtype / device / layout are passed through
without a copy while other inputs are converted as before."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_raw_stream_is_torch_current_stream(gpu):
    import invsim
    env = invsim.NewsvendorEnv(64, device=gpu)
    assert env._stream() == torch.cuda.current_stream(gpu).cuda_stream
    s = torch.cuda.Stream(device=gpu)
    with torch.cuda.stream(s):
        assert env._stream() == s.cuda_stream
        env.reset(seed=1)
        o, r, te, tr, _ = env.step(torch.full((64, 1), 50.0, device=gpu))
    s.synchronize()
    env2 = invsim.NewsvendorEnv(64, device=gpu)
    env2.reset(seed=1)
    o2, r2, _, _, _ = env2.step(torch.full((64, 1), 50.0, device=gpu))
    assert torch.equal(o, o2) and torch.equal(r, r2)


def test_action_fast_path_and_conversions(gpu):
    import invsim
    n = 256
    envs = [invsim.InvManagementBacklogEnv(n, device=gpu) for _ in range(3)]
    for e in envs:
        e.reset(seed=3)
    a = torch.randint(-5, 120, (n, 3), device=gpu, dtype=torch.int64)
    assert envs[0]._actions(a, (n,)) is a                         # passed through
    outs = [envs[0].step(a), envs[1].step(a.cpu().numpy()), envs[2].step(a.to(torch.float64))]
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
    nc = a.t().contiguous().t()                                 # non-contiguous view: converted
    assert not nc.is_contiguous() and envs[0]._actions(nc, (n,)).is_contiguous()
