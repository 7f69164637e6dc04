"""Host cost of one invsim_step call through ctypes, split into its parts.

InvMgmt Backlog, 65 536 envs.  Prints host microseconds per call for:
  noop    a ctypes call of a trivial export (invsim_kernel_variant)
  step    invsim_step (host time only: 10 calls into an idle queue, then sync)
  step1   the first invsim_step after an idle, synchronised GPU (what a timed
          region pays once, before the launches overlap the kernels)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))

import torch  # noqa: E402

import invsim  # noqa: E402
from invsim import _capi  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N = 65536
    env = invsim.InvManagementBacklogEnv(N, device=dev, copy=False)
    env.reset(seed=0)
    a = torch.randint(0, 100, (N, 3), device=dev, dtype=torch.int64)
    obs = torch.empty((N, env.obs_dim), dtype=torch.int64, device=dev)
    rew = torch.empty(N, dtype=torch.float64, device=dev)
    te = torch.empty(N, dtype=torch.bool, device=dev)
    tr = torch.empty(N, dtype=torch.bool, device=dev)
    lib, h = env._lib, env._h
    sp = torch.cuda.current_stream(dev).cuda_stream
    args = (a.data_ptr(), obs.data_ptr(), rew.data_ptr(), te.data_ptr(), tr.data_ptr(), None, sp)
    C = _capi.C
    v = C.c_int32()
    for _ in range(100):
        lib.invsim_step(h, *args)
    torch.cuda.synchronize(dev)

    def noop():
        t0 = time.perf_counter()
        for _ in range(1000):
            lib.invsim_kernel_variant(h, C.byref(v))
        return (time.perf_counter() - t0) / 1000

    def step():
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(10):
            lib.invsim_step(h, *args)
        el = (time.perf_counter() - t0) / 10
        torch.cuda.synchronize(dev)
        return el

    def step1():
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        lib.invsim_step(h, *args)
        el = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
        return el

    for name, fn in (("noop", noop), ("step", step), ("step1", step1)):
        xs = sorted(fn() * 1e6 for _ in range(41))
        print(f"{name:6s} host us/call  p10={xs[4]:6.2f} med={xs[20]:6.2f} p90={xs[36]:6.2f}", flush=True)


if __name__ == "__main__":
    main()
