"""Step loop with a torch policy in it, eager against HIP-graph replay
(invsim.graphs.StepGraph): InvMgmt Backlog 65 536 envs and LostSales / Net
32 768 envs.  Each iteration is `a = policy(obs); obs, r, ... = env.step(a)`
plus a running return, i.e. the reference's evaluation loop
(benchmark_InvManagementBacklogEnv.py:389-440) batched.  Prints wall time per
env step and env-steps/s for: eager copy=True, eager copy=False, graph replay
(one replay = one episode cycle), and the raw invsim_step floor (no policy).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))

import torch  # noqa: E402

import invsim  # noqa: E402


def im_policy(o):        # base-stock-like: order up to a level from the obs (int64 [N, 3])
    return torch.clamp(60 - o[:, :3], min=0)


def net_policy(o):
    return torch.clamp(40.0 - o[:, :11], min=0.0)


CASES = {
    "invmgmt_backlog": (invsim.InvManagementBacklogEnv, 65536, im_policy),
    "invmgmt_lostsales": (invsim.InvManagementLostSalesEnv, 32768, im_policy),
    "net_backlog": (invsim.NetInvMgmtBacklogEnv, 32768, net_policy),
    # no policy ops: fixed actions, the env step alone (launch gaps, eager vs graph)
    "invmgmt_backlog_fixed": (invsim.InvManagementBacklogEnv, 65536, None),
}


def loop_fn(env, policy, obs, ret, steps):
    def fn():
        o = obs
        for _ in range(steps):
            o, r, te, tr, _ = env.step(policy(o))
            ret.add_(r)
        obs.copy_(o)
        return ret
    return fn


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    return t_enq, time.perf_counter() - t0


def main():
    dev = torch.device("cuda", 0)
    cycles = int(os.environ.get("CYCLES", "40"))
    out = {}
    for name, (cls, n, policy) in CASES.items():
        res = {}
        if policy is None:
            fixed = torch.randint(0, 150, (n, 3), device=dev, dtype=torch.int64)
            policy = lambda o, fixed=fixed: fixed  # noqa: E731
        for mode in ("eager_copy", "eager_nocopy", "graph"):
            env = cls(n, device=dev, copy=(mode == "eager_copy"))
            C = env._horizon() + 1
            obs = env.reset(seed=0)[0].clone()
            ret = torch.zeros(n, dtype=torch.float64, device=dev)
            fn = loop_fn(env, policy, obs, ret, C)
            if mode == "graph":
                g = env.capture(fn, warmup=2)
                run = g.replay
            else:
                for _ in range(2):
                    fn()
                run = fn
            run()
            t_enq, t_all = timed(run, cycles)
            steps = cycles * C
            res[mode] = {"us_per_step": t_all / steps * 1e6, "host_us_per_step": t_enq / steps * 1e6,
                         "env_steps_per_s": n * steps / t_all}
            env.close()
        out[name] = res
        print(name, json.dumps(res), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
