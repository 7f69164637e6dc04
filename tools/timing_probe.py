"""Per-wave phase timeline of one InvMgmt step (profiling only).

  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so \
      python tools/timing_probe.py [--n 65536] [--lostsales]

The TIMING build (csrc `make timing`) records s_memrealtime (100 MHz) per
wave at: 0 entry, 1 all step loads landed, 2 demand drawn, 3 dynamics + obs
tile done, 4 obs tile stores issued, 5 exit (all stores drained); probe 7 =
XCC_ID << 32 | HW_ID.  Prints the distribution of each phase over waves.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--lostsales", action="store_true")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--newsvendor", action="store_true")
    args = ap.parse_args()
    import invsim
    from invsim import _capi
    g = torch.Generator(device="cuda").manual_seed(1)
    if args.newsvendor:
        env = invsim.NewsvendorEnv(num_envs=args.n)
        env.reset(seed=0)
        acts = [torch.rand((args.n, 1), device=env.device, generator=g) * 400 for _ in range(args.steps)]
    else:
        cls = invsim.InvManagementLostSalesEnv if args.lostsales else invsim.InvManagementBacklogEnv
        env = cls(num_envs=args.n)
        env.reset(seed=0)
        hi = torch.as_tensor(env.single_action_space.high, device=env.device)
        acts = [torch.floor(torch.rand((args.n, env.action_dim), device=env.device, generator=g,
                                       dtype=torch.float64) * (hi + 1)).to(torch.int64) for _ in range(args.steps)]
    for a in acts:
        env.step(a)
    torch.cuda.synchronize()
    lib = _capi.lib()
    waves = min((args.n + 63) // 64, 8192)
    buf = np.zeros((8192, 8), dtype=np.uint64)
    fn = lib.invsim_debug_timing_nv if args.newsvendor else lib.invsim_debug_timing
    rc = fn(buf.ctypes.data_as(C.c_void_p), C.c_int64(buf.nbytes))
    assert rc == 0, rc
    b = buf[:waves].astype(np.int64)
    t0 = b[:, 0].min()
    ns = lambda x: (x * 10.0)
    print(f"waves {waves}; kernel span (first entry -> last exit) {ns(b[:, 5].max() - t0):.0f} ns")
    names = (["entry", "pre-demand", "demand", "step+tile", "stores issued", "exit"] if args.newsvendor else
             ["entry", "loads issued", "demand", "dynamics+tile", "stores issued", "exit"])
    print("phase               p0      p10     p50     p90     max   (ns)")
    print("entry offset     " + " ".join(f"{ns(v):7.0f}" for v in np.percentile(b[:, 0] - t0, [0, 10, 50, 90, 100])))
    for i in range(1, 6):
        d = b[:, i] - b[:, i - 1]
        print(f"{names[i - 1]:>6}->{names[i]:<10}" + " ".join(f"{ns(v):7.0f}" for v in np.percentile(d, [0, 10, 50, 90, 100])))
    if not args.newsvendor:
        for a_, b_, nm in ((2, 6, "demand->reward"), (6, 3, "reward->tile")):
            d = b[:, b_] - b[:, a_]
            print(f"{nm:<22}" + " ".join(f"{ns(v):7.0f}" for v in np.percentile(d, [0, 10, 50, 90, 100])))
    tot = b[:, 5] - b[:, 0]
    print("wave total       " + " ".join(f"{ns(v):7.0f}" for v in np.percentile(tot, [0, 10, 50, 90, 100])))
    hw = b[:, 7] & 0xFFFFFFFF
    xcc = b[:, 7] >> 32
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
    key = xcc * 1000 + se * 100 + sh * 20 + cu
    print("distinct XCC", len(np.unique(xcc)), "distinct (xcc,se,sh,cu)", len(np.unique(key)),
          "max waves per CU", np.bincount(np.unique(key, return_inverse=True)[1]).max(),
          "max waves per SIMD", np.bincount(np.unique(key * 4 + simd, return_inverse=True)[1]).max())
    # entry order by XCC: when does each XCC start / finish
    for x in np.unique(xcc):
        m = xcc == x
        print(f"  xcc {x}: waves {m.sum():4d} entry [{ns(b[m,0].min()-t0):6.0f},{ns(b[m,0].max()-t0):6.0f}] "
              f"exit max {ns(b[m,5].max()-t0):6.0f}")
    np.save(os.path.join(ROOT, "gpurun_out", f"timing_{'nv' if args.newsvendor else ('ls' if args.lostsales else 'bl')}_{args.n}.npy"), buf)


if __name__ == "__main__":
    main()
