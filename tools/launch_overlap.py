"""Why a step kernel's rocprofv3 mean is above bench.py's HIP-event figure
(profiling aid, DESIGN §5 "Event time against rocprof time").

  python tools/launch_overlap.py [workload ...]

For each workload's per-step API (bench.py WORKLOADS, default batch sizes,
NEXT_STEP autoreset, random actions) it times the same invsim_step launches
three ways with HIP events on the launch stream:
  block     one event pair around 248 back-to-back launches (bench.py's way)
  paired    an event pair around EVERY launch, still back to back
  isolated  an event pair around every launch with a device synchronize
            between launches (each kernel starts on an idle GPU, as under
            kernel tracing, which gaps the launches); a ~40 us device-side
            sleep is queued before each pair so that the pair holds the kernel
            only, not the host's launch latency
and prints the means per launch (µs).  block ~ paired < isolated means that
consecutive launches overlap one's drain with the next one's dispatch ramp;
rocprofv3's per-dispatch durations are isolated-like.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))


def run(name, launches=248):
    import invsim
    from bench import WORKLOADS, make_actions
    wl = WORKLOADS[name]
    env = getattr(invsim, wl["cls"])(wl["n"], copy=False)
    env.reset(seed=0)
    gen = torch.Generator(device=env.device).manual_seed(7)
    acts = make_actions(env, 16, 0, gen)
    lib, h = env._lib, env._h
    N, O = env.num_envs, env.obs_dim
    obs = torch.empty((N, O), dtype=env.obs_dtype, device=env.device)
    rew = torch.empty(N, dtype=torch.float64, device=env.device)
    te = torch.empty(N, dtype=torch.bool, device=env.device)
    tr = torch.empty(N, dtype=torch.bool, device=env.device)
    s = torch.cuda.current_stream()
    sp = s.cuda_stream

    def one(i):
        rc = lib.invsim_step(h, acts[i % 16].data_ptr(), obs.data_ptr(), rew.data_ptr(), te.data_ptr(),
                             tr.data_ptr(), None, sp)
        assert rc == 0
    for i in range(64):
        one(i)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    for a, b in evs:
        a.record(s)
        b.record(s)
    torch.cuda.synchronize()
    out = {}
    # block
    a, b = evs[0]
    a.record(s)
    for i in range(launches):
        one(i)
    b.record(s)
    torch.cuda.synchronize()
    out["block"] = a.elapsed_time(b) * 1e3 / launches
    # paired, back to back
    for i in range(launches):
        evs[i][0].record(s)
        one(i)
        evs[i][1].record(s)
    torch.cuda.synchronize()
    out["paired"] = sum(x.elapsed_time(y) for x, y in evs) * 1e3 / launches
    # isolated
    for i in range(launches):
        torch.cuda._sleep(100000)
        evs[i][0].record(s)
        one(i)
        evs[i][1].record(s)
        torch.cuda.synchronize()
    out["isolated"] = sum(x.elapsed_time(y) for x, y in evs) * 1e3 / launches
    env.close()
    return out


def main():
    names = sys.argv[1:] or ["invmgmt_backlog", "invmgmt_lostsales", "newsvendor", "net_backlog"]
    print("workload              block µs  paired µs  isolated µs  isolated/block")
    for n in names:
        r = run(n)
        print(f"{n:20s} {r['block']:9.2f} {r['paired']:10.2f} {r['isolated']:12.2f} {r['isolated'] / r['block']:14.3f}",
              flush=True)


if __name__ == "__main__":
    main()
