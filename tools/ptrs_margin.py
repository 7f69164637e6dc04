"""PTRS log-acceptance statistics over >= 1e8 draws per sampler path (debug build).

  make -C or-gym-inventory_amd/csrc ptrs_stats
  INVSIM_LIB=or-gym-inventory_amd/invsim/_lib/debug/libinvsim_ptrs_stats.so \
      python tools/ptrs_margin.py > gpurun_out/ptrs_margin.json

For each path of tests/test_gpu_long_draws.py (same envs, seeds and actions)
it reports how many PTRS candidates reached the log test, how many of those
the f32 pre-test could not decide (f64 fallback), how many f32 decisions
disagreed with the f64 test (must be 0), and the smallest relative margin
|lhs - rhs| / (|log V| + |log(1/alpha)| + |log x| + |rhs|) over every test.
A 1-ulp difference between the device's OCML f64 log and glibc's (numpy's)
moves lhs by at most ~3 * 2^-53 relative to that sum, so a minimum margin far
above ~3e-16 means no decision could have gone the other way.
"""
import json
import os
import struct
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def stats(lib, clear):
    out = (np.zeros(5, np.uint64))
    rc = lib.invsim_debug_ptrs_stats(out.ctypes.data, 1 if clear else 0)
    if rc:
        raise RuntimeError("invsim_debug_ptrs_stats failed: not the PTRS-statistics build?")
    margin = struct.unpack("<d", struct.pack("<Q", int(out[2])))[0]
    return dict(log_tests=int(out[0]), f64_fallbacks=int(out[1]), min_rel_margin=margin,
                f32_disagreements=int(out[3]), decide_f32_undecided=int(out[4]))


def main():
    import invsim
    from invsim import _capi
    from invsim.topology import custom_graph, default_graph
    from test_gpu_long_draws import _gpu_run, _pool_f32, _pool_int
    assert "debug" in _capi.LIB_PATH, "set INVSIM_LIB to the ptrs_stats build"
    lib = _capi.lib()
    dev = torch.device("cuda:0")
    cases = []
    for cls, n, mode, mu, cyc in [("InvManagementBacklogEnv", 65536, "step", 20, 51),
                                  ("InvManagementBacklogEnv", 65536, "rollout", 20, 51),
                                  ("InvManagementLostSalesEnv", 32768, "rollout", 20, 102)]:
        cases.append((f"{cls} {n} {mode} mu={mu}", lambda cls=cls, n=n, mu=mu: getattr(invsim, cls)(
            n, device=dev, dist_param={"mu": mu}), _pool_int(np.random.default_rng(mu + n), 31, n, 3, 120),
            31 * cyc, mode, 1000 + mu, n * 30 * cyc))
    for mode in ("step", "rollout"):
        n = 65536
        pool = [p.reshape(n, 1) for p in _pool_f32(np.random.default_rng(200), 41, n, 1, 400.0)]
        cases.append((f"NewsvendorEnv {n} {mode} mu_max=200", lambda n=n: invsim.NewsvendorEnv(n, device=dev),
                      pool, 41 * 39, mode, 2200, n * 40 * 39))
    for graph, mode, cyc in [("default", "step", 102), ("default", "rollout", 102), ("custom", "rollout", 34)]:
        n = 32768
        g = default_graph() if graph == "default" else custom_graph()
        cases.append((f"NetInvMgmtBacklogEnv {graph} {n} {mode}",
                      lambda g=g, n=n: invsim.NetInvMgmtBacklogEnv(n, device=dev, graph=g),
                      lambda env, cyc=cyc, n=n: _pool_f32(np.random.default_rng(cyc), 31, n, env.action_dim, 150.0),
                      31 * cyc, mode, 3000 + cyc, n * 30 * cyc * (1 if graph == "default" else 3)))
    res = []
    tot = dict(log_tests=0, f64_fallbacks=0, f32_disagreements=0, decide_f32_undecided=0,
               min_rel_margin=float("inf"), draws=0)
    for name, mk, pool_np, T, mode, seed, draws in cases:
        env = mk()
        if callable(pool_np):
            pool_np = pool_np(env)
        pool = [torch.from_numpy(a).to(dev) for a in pool_np]
        env.reset(seed=seed)
        stats(lib, True)
        t0 = time.time()
        _gpu_run(env, pool, T, mode)
        torch.cuda.synchronize()
        s = stats(lib, True)
        s.update(path=name, draws=draws, seconds=round(time.time() - t0, 2))
        res.append(s)
        print(json.dumps(s), file=sys.stderr, flush=True)
        for k in ("log_tests", "f64_fallbacks", "f32_disagreements", "decide_f32_undecided", "draws"):
            tot[k] += s[k]
        tot["min_rel_margin"] = min(tot["min_rel_margin"], s["min_rel_margin"])
        env.close()
    print(json.dumps({"paths": res, "total": tot}))


if __name__ == "__main__":
    main()
