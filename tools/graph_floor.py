"""Per-launch floor of the step kernels, eager against HIP-graph replay
(VERDICT r03 item 4).  For each workload: 64 episode cycles of back-to-back
invsim_step calls (1 984 steps at 31 steps per cycle; Newsvendor 41) timed
with HIP events on the stream, issued eagerly (one ctypes call per step) and
as one captured graph replayed with one host call, so host submission is out
of the second figure.  Prints one JSON line per workload: µs per step for
both, and the empty-kernel floor from tools/dispatch_cost (graph mode) when
given its output file.

  python tools/graph_floor.py [--cycles 64] [--n-lostsales 32768]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))

import torch  # noqa: E402

import invsim  # noqa: E402
from invsim.graphs import StepGraph  # noqa: E402

CASES = [("invmgmt_lostsales", invsim.InvManagementLostSalesEnv, 32768),
         ("invmgmt_backlog", invsim.InvManagementBacklogEnv, 65536),
         ("net_backlog", invsim.NetInvMgmtBacklogEnv, 32768),
         ("newsvendor", invsim.NewsvendorEnv, 65536)]


def actions(env, gen, pool):
    N, A = env.num_envs, env.action_dim
    if env.act_dtype == torch.int64:
        return [torch.randint(0, 150, (N, A), device=env.device, generator=gen) for _ in range(pool)]
    return [torch.rand((N, A), device=env.device, generator=gen) * 150 for _ in range(pool)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name, cls, n in CASES:
        env = cls(n, device=dev, copy=False)
        env.reset(seed=0)
        gen = torch.Generator(device=dev).manual_seed(7)
        acts = actions(env, gen, 16)
        C = env._horizon() + 1
        steps = C * args.cycles
        N, O = env.num_envs, env.obs_dim
        obs = torch.empty((N, O), dtype=env.obs_dtype, device=dev)
        rew = torch.empty(N, dtype=torch.float64, device=dev)
        te = torch.empty(N, dtype=torch.bool, device=dev)
        tr = torch.empty(N, dtype=torch.bool, device=dev)
        lib, h = env._lib, env._h
        ptrs = [a.data_ptr() for a in acts]

        def loop():
            sp = torch._C._cuda_getCurrentRawStream(dev.index)
            for i in range(steps):
                rc = lib.invsim_step(h, ptrs[i % 16], obs.data_ptr(), rew.data_ptr(), te.data_ptr(),
                                     tr.data_ptr(), None, sp)
                if rc:
                    raise RuntimeError(invsim._capi.last_error(h))
        stream = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def timed(fn):
            best = 1e30
            for _ in range(args.reps):
                torch.cuda.synchronize(dev)
                e0.record(stream)
                fn()
                e1.record(stream)
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / steps)
            return best
        loop()
        eager = timed(loop)
        g = StepGraph(env, loop, warmup=1)
        graph = timed(g.replay)
        rec = {"workload": name, "envs": n, "steps": steps, "eager_us_per_step": eager,
               "graph_us_per_step": graph, "graph_gain_us": eager - graph}
        print(json.dumps(rec), flush=True)
        del g
        env.close()


if __name__ == "__main__":
    main()
