"""Fixed cost of bench.py's timed region at small K (the driver runs --steps 20).

Times, on the InvMgmt Backlog 65 536-env step, K back-to-back invsim_step
launches bracketed the way bench.py does (synchronize, t0, K launches,
synchronize), against variants of the closing wait, and the empty region.
Prints one line per variant: wall us per region, kernel-event us, K.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))

if "--spin" in sys.argv:
    # hipDeviceScheduleSpin (= 1) before the first context: host waits spin
    # instead of yielding / blocking on an interrupt
    import ctypes
    _hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", _hip.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)

import torch  # noqa: E402

import invsim  # noqa: E402
from invsim import _capi  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = invsim.InvManagementBacklogEnv(65536, device=dev, copy=False)
    env.reset(seed=0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    hi = torch.tensor([101.0, 201.0, 231.0], device=dev, dtype=torch.float64)
    acts = [torch.floor(torch.rand((65536, 3), device=dev, dtype=torch.float64, generator=g) * hi).to(torch.int64)
            for _ in range(16)]
    N, O = 65536, env.obs_dim
    obs = torch.empty((N, O), dtype=torch.int64, device=dev)
    rew = torch.empty(N, dtype=torch.float64, device=dev)
    te = torch.empty(N, dtype=torch.bool, device=dev)
    tr = torch.empty(N, dtype=torch.bool, device=dev)
    lib, h = env._lib, env._h
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    ptrs = [a.data_ptr() for a in acts]
    po, pr, pt, pu = obs.data_ptr(), rew.data_ptr(), te.data_ptr(), tr.data_ptr()
    hip = _capi.C.CDLL("libamdhip64.so")

    C = _capi.C
    raw0, raw1 = C.c_void_p(), C.c_void_p()
    hip.hipEventCreate(C.byref(raw0))
    hip.hipEventCreate(C.byref(raw1))
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    spv = C.c_void_p(sp)

    def region(K, wait):
        torch.cuda.synchronize(dev)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        if wait == "evpre":                  # the lazy event creation happens before the region
            e0.record(stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if wait == "rawev":
            hip.hipEventRecord(raw0, spv)
        elif wait != "noev":
            e0.record(stream)
        for i in range(K):
            lib.invsim_step(h, ptrs[i % 16], po, pr, pt, pu, None, sp)
        if wait == "rawev":
            hip.hipEventRecord(raw1, spv)
        elif wait != "noev":
            e1.record(stream)
        if wait in ("sync", "noev", "evpre", "rawev"):
            torch.cuda.synchronize(dev)
        elif wait == "evsync":                # bench.py --stop event
            e1.synchronize()
            el_ev = time.perf_counter() - t0
            torch.cuda.synchronize(dev)
            return el_ev * 1e6, e0.elapsed_time(e1) * 1e3
        elif wait == "spin":
            while not e1.query():
                pass
            torch.cuda.synchronize(dev)
        elif wait == "stream":
            hip.hipStreamSynchronize(_capi.C.c_void_p(sp))
            torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if wait == "rawev":
            ms = C.c_float()
            hip.hipEventElapsedTime(C.byref(ms), raw0, raw1)
            return el * 1e6, ms.value * 1e3
        return el * 1e6, (e0.elapsed_time(e1) * 1e3 if wait != "noev" else 0.0)

    for _ in range(50):
        region(20, "sync")
    for K in (0, 1, 20, 200):
        for wait in ("sync", "noev", "evpre", "rawev", "spin", "evsync"):
            w, k = zip(*[region(K, wait) for _ in range(15)])
            w, k = sorted(w), sorted(k)
            print(f"K={K:5d} wait={wait:6s} wall_us med={w[7]:9.1f} min={w[0]:9.1f}  "
                  f"events_us med={k[7]:9.1f}  per-step wall={w[7] / max(K, 1):7.2f} ev={k[7] / max(K, 1):7.2f}",
                  flush=True)


if __name__ == "__main__":
    main()
