"""Host cost of the Python VectorEnv.step() around the C ABI call (InvMgmt
Backlog, 65 536 envs): wall time per step of K back-to-back env.step() calls
(copy=True: fresh output tensors per step; copy=False: reused buffers) against
K raw invsim_step calls, and the kernel time from events.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))

import torch  # noqa: E402

import invsim  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, K = 65536, 2000
    g = torch.Generator(device=dev).manual_seed(1)
    hi = torch.tensor([101.0, 201.0, 231.0], device=dev, dtype=torch.float64)
    acts = [torch.floor(torch.rand((n, 3), device=dev, dtype=torch.float64, generator=g) * hi).to(torch.int64)
            for _ in range(16)]
    for copy in (True, False):
        env = invsim.InvManagementBacklogEnv(n, device=dev, copy=copy)
        env.reset(seed=0)
        for i in range(50):
            env.step(acts[i % 16])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            env.step(acts[i % 16])
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        print(f"env.step copy={copy}: host enqueue {t_enq / K * 1e6:.2f} us/step, wall {t_all / K * 1e6:.2f} us/step",
              flush=True)
    lib, h = env._lib, env._h
    obs = torch.empty((n, env.obs_dim), dtype=torch.int64, device=dev)
    rew = torch.empty(n, dtype=torch.float64, device=dev)
    te = torch.empty(n, dtype=torch.bool, device=dev)
    tr = torch.empty(n, dtype=torch.bool, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    ptrs = [a.data_ptr() for a in acts]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        lib.invsim_step(h, ptrs[i % 16], obs.data_ptr(), rew.data_ptr(), te.data_ptr(), tr.data_ptr(), None, sp)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"raw ABI: host enqueue {t_enq / K * 1e6:.2f} us/step, wall {t_all / K * 1e6:.2f} us/step")


if __name__ == "__main__":
    main()
