"""Per-wave timeline of the Newsvendor lock-step step (nv_step1_kernel with the
demand lookahead): lookahead workgroups (PTRS / multiplication branch) vs step
workgroups (profiling only; needs the TIMING build, csrc `make timing`).

  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so python tools/timing_nv_step.py

Probes (s_memrealtime, 100 MHz, lane 0 of each one-wave workgroup): 0 entry,
lookahead 1 constants loaded / 2 demand drawn, step 1-3 inside nv_step_regs,
4 obs tile stores issued, 5 exit (stores drained).
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
    n = 65536
    env = invsim.NewsvendorEnv(num_envs=n)
    env.reset(seed=0)
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(12):
        env.step(torch.rand((n, 1), device=env.device, generator=g) * 400)
    torch.cuda.synchronize()
    buf = np.zeros((8192, 8), dtype=np.uint64)
    rc = _capi.lib().invsim_debug_timing_nv(buf.ctypes.data_as(C.c_void_p), C.c_int64(buf.nbytes))
    assert rc == 0, rc
    b = buf.astype(np.int64)
    gla = 2 * (n // 64)
    t0 = b[:3072, 0].min()
    pct = [0, 10, 50, 90, 100]
    fmt = lambda x: " ".join(f"{v * 10.0:7.0f}" for v in np.percentile(x, pct))
    print("ns percentiles       p0      p10     p50     p90     max")
    for name, sel in (("lookahead PTRS", b[0:gla:2]), ("lookahead mult", b[1:gla:2]), ("step", b[gla:gla + n // 64])):
        print(f"-- {name}: {len(sel)} waves")
        print("  entry          " + fmt(sel[:, 0] - t0))
        print("  exit           " + fmt(sel[:, 5] - t0))
        print("  lifetime       " + fmt(sel[:, 5] - sel[:, 0]))
        if name.startswith("lookahead"):
            live = sel[sel[:, 1] > 0]
            if len(live):
                print("  entry->loaded  " + fmt(live[:, 1] - live[:, 0]))
                print("  draw           " + fmt(live[:, 2] - live[:, 1]))
                if name.endswith("PTRS"):
                    c = live[(live[:, 3] > live[:, 1]) & (live[:, 3] < live[:, 2])]
                    print(f"  (compaction probes in {len(c)} waves)")
                    if len(c):
                        print("  round 1        " + fmt(c[:, 3] - c[:, 1]))
                        g = c[(c[:, 4] > c[:, 3]) & (c[:, 4] < c[:, 2])]
                        if len(g):
                            print("  group setup    " + fmt(g[:, 4] - g[:, 3]))
                            print("  group rounds   " + fmt(g[:, 2] - g[:, 4]))
                print("  drawn->exit    " + fmt(live[:, 5] - live[:, 2]))
        else:
            print("  entry->p1      " + fmt(sel[:, 1] - sel[:, 0]))
            print("  p1->p3 (step)  " + fmt(sel[:, 3] - sel[:, 1]))
            print("  p3->stores     " + fmt(sel[:, 4] - sel[:, 3]))
            print("  stores->exit   " + fmt(sel[:, 5] - sel[:, 4]))
    print(f"kernel span {(b[:3072, 5].max() - t0) * 10.0:.0f} ns")


if __name__ == "__main__":
    main()
