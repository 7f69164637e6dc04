"""Per-wave timeline of the InvMgmt lock-step step (im_split_kernel with the
demand lookahead): lookahead workgroups vs the step's window and dynamics
waves (profiling only; needs the TIMING build, csrc `make timing`).

  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so python tools/timing_im_step.py [N] [lostsales]

Probes (s_memrealtime, 100 MHz): 0 workgroup entry (thread 0); lookahead
1 loads + RHS table in LDS, 2 demand drawn, 5 exit; step 3 / 4 dynamics wave
entry / exit, 1 its loads in and d handed over, 2 its step computed (tile
complete), 6 / 5 window wave: rows landed / exit.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))


def main():
    import invsim
    from invsim import _capi
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    cls = invsim.InvManagementLostSalesEnv if "lostsales" in sys.argv[2:] else invsim.InvManagementBacklogEnv
    env = cls(num_envs=n)
    env.reset(seed=0)
    g = torch.Generator(device="cuda").manual_seed(1)
    hi = torch.as_tensor(env.single_action_space.high, device=env.device)
    for _ in range(12):
        a = torch.floor(torch.rand((n, 3), device=env.device, generator=g, dtype=torch.float64) * (hi + 1))
        env.step(a.to(torch.int64))
    torch.cuda.synchronize()
    buf = np.zeros((8192, 8), dtype=np.uint64)
    rc = _capi.lib().invsim_debug_timing(buf.ctypes.data_as(C.c_void_p), C.c_int64(buf.nbytes))
    assert rc == 0, rc
    b = buf.astype(np.int64)
    gla = (n + 127) // 128
    nst = (n + 63) // 64
    tot = gla + nst
    t0 = b[:tot, 0].min()
    pct = [0, 10, 50, 90, 100]
    fmt = lambda x: " ".join(f"{v * 10.0:7.0f}" for v in np.percentile(x, pct))
    print("ns percentiles          p0      p10     p50     p90     max")
    la, st = b[:gla], b[gla:tot]
    print(f"-- lookahead: {gla} workgroups")
    print("  entry             " + fmt(la[:, 0] - t0))
    print("  entry->loaded     " + fmt(la[:, 1] - la[:, 0]))
    print("  draw              " + fmt(la[:, 2] - la[:, 1]))
    print("  exit              " + fmt(la[:, 5] - t0))
    print(f"-- step: {nst} workgroups")
    print("  entry             " + fmt(st[:, 0] - t0))
    print("  window exit       " + fmt(st[:, 5] - t0))
    print("  window rows in    " + fmt(st[:, 6] - t0))
    print("  dynamics entry    " + fmt(st[:, 3] - t0))
    print("  dynamics loads in " + fmt(st[:, 1] - t0))
    print("  dynamics computed " + fmt(st[:, 2] - t0))
    print("  dynamics exit     " + fmt(st[:, 4] - t0))
    print("  (computed - d in) " + fmt(st[:, 2] - st[:, 1]))
    print("  (exit - computed) " + fmt(st[:, 4] - st[:, 2]))
    print("  (d in - entry)    " + fmt(st[:, 1] - st[:, 3]))
    print(f"kernel span {(np.maximum(b[:tot, 5], b[:tot, 4]).max() - t0) * 10.0:.0f} ns")


if __name__ == "__main__":
    main()
