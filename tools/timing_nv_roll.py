"""Per-wave timeline of the Newsvendor K=30 rollout (nv_roll_kernel, 4 waves
per 64-env workgroup; layout L0: PTRS wave, multiplication wave, dynamics
wave, obs wave; L1 names the roles of the lane-pair layout measured in
commit b4c9eaf: two PTRS pair waves, dynamics, obs with the multiplication
draws).  Profiling only; needs the TIMING build (csrc `make timing`):

  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/ablate/libinvsim_TIMING.so python tools/timing_nv_roll.py [L0|L1]

Probes (s_memrealtime, 100 MHz, lane 0 of every wave, row = workgroup * 4 +
wave): 0 entry, 1 ready (stream: state + tables loaded; dynamics: barrier 0
passed; obs: barrier 1 passed), 2-5 chunk c = 0..3 (stream: its draws done,
before the chunk's barrier; dynamics / obs: the chunk consumed, before the
next barrier), 6 exit (stores drained), 7 hardware ids (XCC, SE/CU/SIMD/wave
slot).  Also the accumulated barrier wait of every wave (g_tbar): the part of
its lifetime spent in the workgroup syncs, the rest is its own work.
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
    n, K = 65536, 30
    env = invsim.NewsvendorEnv(num_envs=n, copy=False)
    env.reset(seed=0)
    g = torch.Generator(device="cuda").manual_seed(1)
    acts = torch.rand((K, n, 1), device=env.device, generator=g) * 400
    for _ in range(4):
        env.rollout(acts)
    torch.cuda.synchronize()
    buf = np.zeros((8192, 8), dtype=np.uint64)
    rc = _capi.lib().invsim_debug_timing_nv(buf.ctypes.data_as(C.c_void_p), C.c_int64(buf.nbytes))
    assert rc == 0, rc
    layout = sys.argv[1] if len(sys.argv) > 1 else "L0"   # L0: the shipped 4-role kernel; L1: commit b4c9eaf's layout
    R = 4
    W = R * (n // 64)
    if layout == "L1":
        roles = ((0, "PTRS pairs A"), (1, "PTRS pairs B"), (2, "dynamics"), (3, "obs + mult"))
        trip_roles = ((0, "PTRS pairs A"), (1, "PTRS pairs B"), (3, "obs + mult"))
    else:
        roles = ((0, "PTRS stream"), (1, "mult stream"), (2, "dynamics"), (3, "obs"))
        trip_roles = ((0, "PTRS stream"), (1, "mult stream"))
    b = buf[:W].astype(np.int64)
    t0 = b[:, 0].min()
    pct = [0, 10, 50, 90, 100]
    fmt = lambda x: " ".join(f"{v * 10.0:8.0f}" for v in np.percentile(x, pct))  # noqa: E731
    print("ns percentiles        p0       p10      p50      p90      max")
    for role, name in roles:
        sel = b[role::R]
        print(f"-- {name}: {len(sel)} waves")
        print("  entry          " + fmt(sel[:, 0] - t0))
        print("  ready          " + fmt(sel[:, 1] - t0))
        prev = sel[:, 1]
        for c in range(4):
            print(f"  chunk {c} end    " + fmt(sel[:, 2 + c] - t0) + "   (+" + fmt(sel[:, 2 + c] - prev).strip() + ")")
            prev = sel[:, 2 + c]
        print("  exit           " + fmt(sel[:, 6] - t0))
    # per chunk: how long the dynamics wave waited at the barrier for its stream waves
    d, p, m = b[2::R], b[0::R], b[1::R]
    for c in range(3 if layout == "L0" else 0):
        ready = np.maximum(p[:, 3 + c], m[:, 3 + c])          # chunk c+1 drawn by the stream waves
        wait = np.maximum(0, ready - d[:, 2 + c])
        print(f"barrier {c + 1}: dynamics waits for the stream waves  " + fmt(wait))
    # SIMD sharing: waves per (XCC, SE, CU, SIMD)
    hw = buf[:W, 7]
    xcc = (hw >> 32) & 0xF
    hwid = hw & 0xFFFFFFFF
    simd = (hwid >> 4) & 0x3
    cu = (hwid >> 8) & 0xF
    sh = (hwid >> 12) & 0x1
    se = (hwid >> 13) & 0x7
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    _, cnt = np.unique(key, return_counts=True)
    print("waves per SIMD: " + " ".join(f"{k}:{v}" for k, v in zip(*np.unique(cnt, return_counts=True))))
    ptrs_key = key[0::R]
    same = np.mean([len(set(key[w * R:(w + 1) * R])) == 1 for w in range(W // R)])
    print("workgroups with all %d waves on one SIMD: %.1f %%" % (R, 100.0 * same))
    share = np.array([np.sum(ptrs_key == k) for k in ptrs_key])
    print("PTRS waves sharing their SIMD with another PTRS wave: %.1f %%" % (100.0 * np.mean(share > 1)))
    bar = np.zeros(8192, dtype=np.uint64)
    rc = _capi.lib().invsim_debug_timing_bar_nv(bar.ctypes.data_as(C.c_void_p), C.c_int64(bar.nbytes))
    assert rc == 0, rc
    bar = bar[:W].astype(np.int64)
    print("per role (last launch): lifetime = exit - entry, barrier wait, work = lifetime - wait")
    for role, name in roles:
        life = b[role::R, 6] - b[role::R, 0]
        wt = bar[role::R]
        print(f"  {name:12s} life {fmt(life)}\n  {'':12s} wait {fmt(wt)}\n  {'':12s} work {fmt(life - wt)}")
    trip = np.zeros(8192, dtype=np.uint32)
    if hasattr(_capi.lib(), "invsim_debug_timing_trip_nv"):
        rc = _capi.lib().invsim_debug_timing_trip_nv(trip.ctypes.data_as(C.c_void_p), C.c_int64(trip.nbytes))
        assert rc == 0, rc
        trip = trip[:W].astype(np.int64)
        print("loop trips per wave (PTRS: the per-chunk max over lanes, summed; mult: rounds) and work per trip")
        for role, name in trip_roles:
            tr = trip[role::R]
            life = b[role::R, 6] - b[role::R, 0]
            work = life - bar[role::R]
            ok = tr > 0
            print(f"  {name:12s} trips {fmt(tr / 10.0)}")
            print(f"  {'':12s} ns/trip {fmt(work[ok] / tr[ok])}")
    print(f"kernel span {(b[:, 6].max() - t0) * 10.0:.0f} ns")
    if layout == "L0":
        # the tail: the workgroups that end last, which role ends them, and how
        # many multiplication-branch envs (mu < 10) they hold after the launch
        ends = b[:, 6].reshape(-1, R)
        wg_end = ends.max(axis=1) - t0
        mu = env.params()[:, 4].cpu().numpy()[: (n // 64) * 64].reshape(-1, 64)
        nm = (mu < 10).sum(axis=1)
        order = np.argsort(wg_end)
        for label, sel in (("slowest 2 %", order[-len(order) // 50:]), ("median 50 %", order[len(order) // 4: 3 * len(order) // 4])):
            last = np.bincount(ends[sel].argmax(axis=1), minlength=R)
            print(f"  {label} of workgroups: end {np.percentile(wg_end[sel], 50) * 10.0:.0f} ns (p50); "
                  f"last role " + ", ".join(f"{name} {last[r]}" for r, name in roles) +
                  f"; mult envs p50 {np.percentile(nm[sel], 50):.0f} max {nm[sel].max()}")
            if len(trip) and trip.any():
                print(f"  {'':12s} PTRS trips p50 {np.percentile(trip[0::R][sel], 50):.1f}, "
                      f"mult rounds p50 {np.percentile(trip[1::R][sel], 50):.1f}")


if __name__ == "__main__":
    main()
