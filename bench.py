"""Benchmark: vectorised env-steps/s of the invsim HIP hot path on MI355X.

Default workload (north_star target): InvManagementBacklogEnv, 4 stages,
65 536 envs per GPU, one `step` = one env.step() over the whole batch through
the C ABI (libinvsim `invsim_step`), actions pre-generated in HBM (a pool of
distinct batches cycled per step), outputs into preallocated device buffers,
NEXT_STEP autoreset (an episode boundary every 31 steps is part of the work).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--mode step|rollout]

Multi-GPU (one process per GPU, torchrun): each rank owns 65 536 envs with
global seeds rank*65536+i (weak scaling), no collective in the data path;
barrier + synchronize around the timed region, max time over ranks.  After
the timed region the per-rank episodic-return statistics are all-reduced over
RCCL (the only cross-GPU exchange the path has).  --strong splits the
workload's env count over the ranks instead (strong scaling).

Prints ONE JSON line (rank 0).  `roofline.achieved` = algorithmic bytes per
launch (SURVEY §8(d) B1 x N) / mean kernel time from HIP events on the stream
the kernel runs on.  `cpu_baseline` = the C oracle (a single-thread port of the
reference step, env loop OpenMP-parallel over up to 16 host cores; the
single-thread rate beside it) timed on this host on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "or-gym-inventory_amd"))

# algorithmic bytes per env-step: B1 for the per-step API,
# B_io + state/K for a fused K-step rollout
WORKLOADS = {
    "invmgmt_backlog": dict(cls="InvManagementBacklogEnv", n=65536, B_io=298, B_state=448,
                            B_state_rollout=880, dtype="int64",
                            desc="InvManagementBacklogEnv 4-echelon default, 65536 instances"),
    "invmgmt_lostsales": dict(cls="InvManagementLostSalesEnv", n=32768, B_io=298, B_state=384,
                              B_state_rollout=816, dtype="int64",
                              desc="InvManagementLostSalesEnv 4-echelon, 32768 instances per GPU"),
    "newsvendor": dict(cls="NewsvendorEnv", n=65536, B_io=54, B_state=136, B_state_rollout=136,
                       dtype="f32/f64", desc="NewsvendorEnv default, 65536 instances, Poisson demand"),
    "net_backlog": dict(cls="NetInvMgmtBacklogEnv", n=32768, B_io=326, B_state=720,
                        B_state_rollout=1136, dtype="f64",
                        desc="NetInvMgmtBacklogEnv default topology, 32768 instances"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--workload", default="invmgmt_backlog", choices=sorted(WORKLOADS))
    ap.add_argument("--mode", default="step", choices=["step", "rollout"])
    ap.add_argument("--rollout-k", type=int, default=30)
    ap.add_argument("--n-envs", type=int, default=0)
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the workload's env count is the GLOBAL batch, split over ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--pool", type=int, default=16, help="distinct action batches cycled")
    return ap.parse_args()


def make_actions(env, pool, K, gen):
    import torch
    N, A = env.num_envs, env.action_dim
    shape = (pool, K, N, A) if K else (pool, N, A)
    if env.act_dtype == torch.int64:
        hi = torch.as_tensor(env.single_action_space.high, device=env.device, dtype=torch.float64)
        u = torch.rand(shape, device=env.device, dtype=torch.float64, generator=gen)
        return torch.floor(u * (hi + 1)).to(torch.int64)
    hi = 400.0 if env.family == 1 else 200.0
    return torch.rand(shape, device=env.device, generator=gen) * hi


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_rate(pyoracle, wl, n, threads, seconds):
    """env-steps/s of the C oracle over whole episodes (resets included)."""
    import numpy as np
    pyoracle.set_threads(threads)
    rng = np.random.default_rng(0)
    if wl["cls"].startswith("InvManagement"):
        env = pyoracle.OracleInvMgmt(n, backlog=wl["cls"].endswith("BacklogEnv"))
        acts = [rng.integers(0, 231, size=(n, 3)).astype(np.int64) for _ in range(8)]
        T = 30
    elif wl["cls"] == "NewsvendorEnv":
        env = pyoracle.OracleNewsvendor(n)
        acts = [rng.uniform(0, 400, size=n).astype(np.float32) for _ in range(8)]
        T = 40
    else:
        env = pyoracle.OracleNet(n)
        acts = [rng.uniform(0, 200, size=(n, 11)).astype(np.float32) for _ in range(8)]
        T = 30
    env.seed(range(n))
    env.reset()
    steps = 0
    t0 = time.perf_counter()
    while True:
        for k in range(T):
            env.step(acts[k % 8])
        env.reset()
        steps += n * T
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    pyoracle.set_threads(1)
    return steps / el, steps // n, el


def cpu_baseline(wl, seconds):
    """C oracle (restatement of the reference step, env loop parallel over the
    host's cores with OpenMP) on this host; the single-thread rate beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))        # the box's CPU share per GPU is 16
    n1 = 8192
    nT = 32768 if wl["cls"].startswith("NetInvMgmt") else 65536
    v1, s1, e1 = _oracle_rate(pyoracle, wl, n1, 1, seconds / 2)
    vT, sT, eT = _oracle_rate(pyoracle, wl, nT, threads, seconds / 2)
    return dict(value=vT, unit="env-steps/s", cores=threads, kind="port",
                sample=f"{nT} envs x {sT} steps ({sT // (40 if wl['cls'] == 'NewsvendorEnv' else 30)} episodes "
                       f"incl. resets), oracle/oracle.c OpenMP {threads} threads, {eT:.1f} s",
                single_thread={"value": v1, "sample": f"{n1} envs x {s1} steps, 1 thread, {e1:.1f} s"},
                cpu_model=_cpu_model(), host_cpus_visible=cores)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL ("nccl") over xGMI; INVSIM_BENCH_BACKEND=gloo rehearses the multi-rank
    # path with several ranks on one GPU (RCCL refuses two ranks per device)
    backend = os.environ.get("INVSIM_BENCH_BACKEND", "nccl")
    if world > 1:
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import invsim
    wl = WORKLOADS[args.workload]
    n = args.n_envs or wl["n"]
    if args.strong:
        n = (n + world - 1) // world                      # this rank's share of the global batch
    env = getattr(invsim, wl["cls"])(n, device=dev, global_offset=rank * n, copy=False)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    K = args.rollout_k if args.mode == "rollout" else 0
    pool = max(1, args.pool if args.mode == "step" else 2)
    acts = make_actions(env, pool, K, gen)
    env.reset(seed=0)
    lib, h = env._lib, env._h
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    N, O = env.num_envs, env.obs_dim
    if args.mode == "step":
        obs = torch.empty((N, O), dtype=env.obs_dtype, device=dev)
        rew = torch.empty(N, dtype=torch.float64, device=dev)
        term = torch.empty(N, dtype=torch.bool, device=dev)
        trunc = torch.empty(N, dtype=torch.bool, device=dev)
        ptrs = [a.data_ptr() for a in acts]
        po, pr, pt, pu = obs.data_ptr(), rew.data_ptr(), term.data_ptr(), trunc.data_ptr()
        step_fn = lib.invsim_step

        def one(i):
            rc = step_fn(h, ptrs[i % pool], po, pr, pt, pu, None, sp)
            if rc:
                raise RuntimeError(invsim._capi.last_error(h))
        steps_per_call = 1
    else:
        obs = torch.empty((K, N, O), dtype=env.obs_dtype, device=dev)
        rew = torch.empty((K, N), dtype=torch.float64, device=dev)
        term = torch.empty((K, N), dtype=torch.bool, device=dev)
        trunc = torch.empty((K, N), dtype=torch.bool, device=dev)
        ptrs = [a.data_ptr() for a in acts]
        po, pr, pt, pu = obs.data_ptr(), rew.data_ptr(), term.data_ptr(), trunc.data_ptr()
        fn = lib.invsim_rollout

        def one(i):
            rc = fn(h, K, ptrs[i % pool], po, pr, pt, pu, sp)
            if rc:
                raise RuntimeError(invsim._capi.last_error(h))
        steps_per_call = K

    calls = max(1, args.steps // steps_per_call)
    warm = max(1, args.warmup // steps_per_call)
    # HIP events on the stream the kernels run on, around the timed region:
    # launches are back to back there, so (end - start) / calls is the mean
    # kernel duration (+ inter-kernel gaps, ~0 on a saturated queue).  torch
    # creates the HIP event at its first record: record both once here so the
    # creation stays out of the timed region (~10 us of wall time per region,
    # tools/sync_overhead.py)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for i in range(warm):
        one(i)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(calls):
        one(i)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # collectives on device tensors over RCCL; gloo (rehearsal) reduces host copies
    cdev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_steps = calls * steps_per_call  # env.step() calls over the batch
    env_steps = total_steps * N * world
    kern_ms_mean = ev0.elapsed_time(ev1) / calls

    # episodic-return statistics all-reduced across GPUs (RCCL): one short episode
    env2 = getattr(invsim, wl["cls"])(min(N, 4096), device=dev, global_offset=rank * N)
    env2.reset(seed=0)
    a2 = make_actions(env2, 1, 0, gen)[0]
    ret = torch.zeros(env2.num_envs, dtype=torch.float64, device=dev)
    while True:
        _, r, _, tr, _ = env2.step(a2)
        ret += r
        if bool(tr.all()):
            break
    stats = torch.stack([ret.sum(), (ret * ret).sum(),
                         torch.tensor(float(env2.num_envs), dtype=torch.float64, device=dev)])
    if world > 1:
        stats = stats.to(cdev)
        dist.all_reduce(stats)
    stats = stats.cpu().tolist()

    B = wl["B_io"] + (wl["B_state_rollout"] / K if K else wl["B_state"])
    achieved = B * N * steps_per_call / (kern_ms_mean * 1e-3) / 1e9
    traffic, traffic_src = None, None
    # the newest round's PMC summary (profiles/rNN/pmc_<workload>.json, tools/pmc_summary.py)
    import glob
    pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", f"pmc_{args.workload}.json")))
    pmc = pmcs[-1] if pmcs else ""
    if pmc and args.mode == "step" and N == wl["n"]:
        rec = json.load(open(pmc))
        traffic, traffic_src = rec["hbm_bytes_per_launch"], os.path.relpath(pmc, ROOT)
    out = {
        "metric": "env-steps/sec (batched) at 1/2/4/8 MI355X; % HBM roofline",
        "value": env_steps / el,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": total_steps,
        "warmup": warm * steps_per_call,
        "ms_per_step": el * 1e3 / total_steps,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": wl["dtype"],
        "data": "synthetic (pre-generated random actions in HBM, seeds 0..N-1 per global env index)",
        "config": {"workload": wl["desc"], "envs_per_gpu": N, "global_envs": N * world,
                   "mode": args.mode + (f" K={K}" if K else ""), "autoreset": "next_step",
                   "parallelism": f"dp{world} (env sharding, no data-path collective)",
                   "backend": backend if world > 1 else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, calibrated)",
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": B * N * steps_per_call,
                     "bytes_per_env_step": B, "kernel_ms_mean": kern_ms_mean,
                     "kernel_timing": "HIP events on the kernel stream around the timed region / launches"},
        "episode_stats": {"sum_return": stats[0], "sum_sq_return": stats[1], "episodes": stats[2]},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wl, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
