"""Benchmark: vectorised env-steps/s of the invsim HIP hot path on MI355X.

Default workload (north_star target): InvManagementBacklogEnv, 4 stages,
65 536 envs per GPU, one `step` = one env.step() over the whole batch through
the C ABI (libinvsim `invsim_step`), actions pre-generated in HBM (a pool of
distinct batches cycled per step), outputs into preallocated device buffers,
NEXT_STEP autoreset (an episode boundary every 31 steps is part of the work).
The step outputs land in a [128, N] slab that the HIP episode fold
(`invsim_episode_fold_groups`) reduces to episodic-return statistics every
128 steps inside the timed region (rollouts fold inside their kernels instead:
the episode sink, `invsim_set_episode_sink`); one all-reduce of the statistics
follows the region.  After the step region the same handle runs a timed region
of fused K=30 rollouts (`invsim_rollout`), reported under "rollout" in the
same line, and the step loop again as HIP-graph replays (one episode cycle per
replay), under "graph".  The default line then times BASELINE configs 2, 4
(per-GPU shard) and 5 the same way, under "configs".

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--mode step|rollout]

Multi-GPU (one process per GPU): under torch.distributed.run the ranks come
from the environment (WORLD_SIZE must equal --gpus); `bench.py --gpus N` run
directly starts the N ranks itself (torch.distributed.run child, before any
GPU call) and relays rank 0's line.  Each rank owns 65 536 envs with global
seeds rank*65536+i (weak scaling), no collective in the data path; barrier +
synchronize around the timed region, max time over ranks.  --strong splits
the workload's env count over the ranks instead (strong scaling).

Prints ONE JSON line (rank 0).  `roofline.frac` = frac_kernel: algorithmic
bytes per launch (SURVEY §8(d) B1 x N) / mean launch duration from HIP events
on the stream the kernel runs on; `frac_wall` beside it uses the wall-clock
`value` instead; `roofline.hbm_counter` is the physical rate: PMC counter
bytes per launch over the dominant kernel's rocprofv3 time (committed
profiles/rNN files).  `cpu_baseline` = the C oracle (a single-thread port of
the reference step, env loop OpenMP-parallel over up to 16 host cores; the
single-thread rate beside it) timed on this host on a bounded sample, with the
reference's own Python rate quoted from BASELINE.md beside it.
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
                            B_state_rollout=880, dtype="int64", agent=("BaseStockAgent", 1.0), B_act=24,
                            desc="InvManagementBacklogEnv 4-echelon default, 65536 instances"),
    "invmgmt_lostsales": dict(cls="InvManagementLostSalesEnv", n=32768, B_io=298, B_state=384,
                              B_state_rollout=816, dtype="int64", agent=("BaseStockAgent", 1.0), B_act=24,
                              desc="InvManagementLostSalesEnv 4-echelon, 32768 instances per GPU"),
    "newsvendor": dict(cls="NewsvendorEnv", n=65536, B_io=54, B_state=136, B_state_rollout=136,
                       dtype="f32/f64", agent=("OrderUpToHeuristicAgent", 1.0), B_act=4, desc="NewsvendorEnv default, 65536 instances, Poisson demand"),
    "net_backlog": dict(cls="NetInvMgmtBacklogEnv", n=32768, B_io=326, B_state=720,
                        B_state_rollout=1136, dtype="f64", agent=("ConstantOrderAgent", 0.1), B_act=44,
                        desc="NetInvMgmtBacklogEnv default topology, 32768 instances"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_ACHIEVABLE_GBS = 6300.0  # what a streaming kernel reaches (MI355X_MICROARCH.md, HBM section)
# The reference's own CPU step, measured in the survey container (BASELINE.md
# section 2: numpy/networkx, 8 independent processes on an 8-vCPU Intel Xeon KVM
# guest, constant actions, aggregate env-steps/s).  The reference cannot run on
# the GPU box, so this is quoted with its provenance, not re-timed.
REFERENCE_PYTHON = {
    "invmgmt_backlog": (200e3, "InvManagementBacklogEnv m=4"),
    "invmgmt_lostsales": (204e3, "InvManagementLostSalesEnv m=4"),
    "newsvendor": (561e3, "NewsvendorEnv L=5"),
    "net_backlog": (722.0, "NetInvMgmtBacklogEnv default graph"),
}
# profiles/rNN round whose committed rocprof / PMC files the line quotes (None:
# the newest round that has the file)
PROFILE_ROUND = None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--workload", default="invmgmt_backlog", choices=sorted(WORKLOADS))
    ap.add_argument("--mode", default="step", choices=["step", "rollout", "policy"],
                    help="policy: K-step rollouts with the workload's heuristic agent in the kernel "
                         "(invsim_rollout_policy; BaseStock / OrderUpTo / ConstantOrder)")
    ap.add_argument("--rollout-k", type=int, default=30)
    ap.add_argument("--n-envs", type=int, default=0)
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the workload's env count is the GLOBAL batch, split over ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fold", default="auto", choices=["auto", "sink", "side", "inline", "none"],
                    help="episodic-return statistics of the timed steps: sink = folded inside the step / "
                         "rollout kernels (invsim_set_episode_sink; auto picks it for InvMgmt, whose "
                         "kernels fold in-kernel), inline = a fold launch between blocks on the kernel "
                         "stream (auto for the other families), side = that fold on a side stream "
                         "(measured slower), none = off (A/B only: no episode_stats)")
    ap.add_argument("--stop", default="spin", choices=["event", "spin", "sync"],
                    help="end of the timed region: the kernel stream's last event completing, waited for "
                         "by polling hipEventQuery (spin, default: measured 1-2 %% higher on the 20-step "
                         "driver line than hipEventSynchronize, profiles/r06/stop_ab) or with "
                         "hipEventSynchronize (event), or "
                         "torch.cuda.synchronize returning (sync); the region is closed by "
                         "torch.cuda.synchronize either way")
    ap.add_argument("--no-graph-line", action="store_true",
                    help="step mode: skip the HIP-graph replay region reported under 'graph'")
    ap.add_argument("--no-rollout-line", action="store_true",
                    help="step mode: skip the K-step rollout region reported under 'rollout'")
    ap.add_argument("--no-config-lines", action="store_true",
                    help="default step run: skip the compact lines of the other BASELINE configs "
                         "(Newsvendor, the LostSales shard, NetInvMgmt) reported under 'configs'")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--pool", type=int, default=16, help="distinct action batches cycled")
    ap.add_argument("--demand-stream", default="numpy", choices=["numpy", "philox"],
                    help="numpy: the reference's PCG64 stream (parity, default); philox: the opt-in fast stream")
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


def _spawn_ranks(args):
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start N fresh rank
    processes with torch.distributed.run and relay rank 0's line.  Called
    before anything touches the GPU; the parent never execs."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return p.wait()


def _fold_rows(stats, rew, term, trunc, rows, sp):
    if rows:
        stats.update_block(rew[:rows], term[:rows], trunc[:rows], stream=sp)


def fold_mode(args, env, mode="step"):
    """--fold auto: K-step rollouts of InvMgmt fold inside the rollout kernels
    (the episode sink: the running return is read and written once per launch,
    16 B per env per K steps, and no second pass reads the outputs); single
    steps fold their output rows in one launch per block of steps (10 B per
    env-step of reward and flags, against the sink's 16 B of running return
    per env-step: measured 8.12 vs 8.51 us per step at 65 536 envs,
    profiles/r06/sink); the other families always fold per block (their kernels
    have no in-kernel fold, and the library would fold each launch's rows
    separately)."""
    import invsim
    if args.fold != "auto":
        return args.fold
    return "sink" if env.family == invsim._capi.INVSIM_INVMGMT and mode != "step" else "inline"


def _span(t0, t1, dev, dist):
    """The timed region across ranks: from the earliest rank's start to the
    latest rank's end.  time.perf_counter is CLOCK_MONOTONIC, one clock for
    every process of the node, so the ranks' stamps compare directly; the span
    includes the skew of the ranks' exits from the opening barrier (a max of
    per-rank durations would drop it)."""
    if not dist.is_initialized():
        return t1 - t0
    import torch
    cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([-t0, t1], dtype=torch.float64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[1].item()) + float(t[0].item())


def run_region(args, env, wl, mode, steps, warmup, world, dev, gen, dist):
    """Warm up, then time `steps` env.step()s of the whole batch (mode "step":
    one invsim_step each; "rollout": invsim_rollout launches of K steps;
    "policy": invsim_rollout_policy launches), with barrier + synchronize on
    both sides and the span over ranks.  The step outputs are written into
    [R, N] slabs; the episodic-return statistics come from the episode sink in
    the kernels (fold "sink") or from the HIP group fold
    (invsim_episode_fold_groups) of each slab on the kernel stream between
    blocks (fold "inline"; "side" is the measured-slower side-stream variant);
    they are all-reduced once after the region.  The clock stops when the
    kernel stream's last event completes (--stop spin / event) or at the
    return of torch.cuda.synchronize (--stop sync); torch.cuda.synchronize
    closes the region either way."""
    import torch
    import invsim
    from invsim.distributed import EpisodeStats
    lib, h = env._lib, env._h
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    N, O = env.num_envs, env.obs_dim
    K = args.rollout_k if mode in ("rollout", "policy") else 0
    pool = max(1, args.pool if mode == "step" else 2)
    acts = make_actions(env, pool, K, gen) if mode != "policy" else []
    ptrs = [a.data_ptr() for a in acts]
    # slab rows = steps per fold: 128 single steps, or 4 launches of K steps.  The
    # fold is a separate launch between blocks (17 us per 128 rows at 65 536
    # envs, measured), so blocks are long
    LPB = 4                                         # launches per block (rollout / policy)
    R = LPB * K if K else 128
    # two output slabs, alternating per block.  --fold inline (auto for steps) runs
    # each block's fold on the kernel stream after the block; --fold side runs it
    # on a side stream while the steps write the other slab (events order slab
    # reuse), measured slower because the fold then shares the CUs with the steps
    rew = torch.empty((2, R, N), dtype=torch.float64, device=dev)
    term = torch.empty((2, R, N), dtype=torch.bool, device=dev)
    trunc = torch.empty((2, R, N), dtype=torch.bool, device=dev)
    obs = torch.empty(((K or 1), N, O), dtype=env.obs_dtype, device=dev)
    po = obs.data_ptr()
    slab_ptrs = [(rew[b].data_ptr(), term[b].data_ptr(), trunc[b].data_ptr()) for b in range(2)]
    stats = EpisodeStats(N, dev)
    fm = fold_mode(args, env, mode)
    if fm == "sink":           # the step / rollout kernels fold their rows into `stats` themselves
        stats.attach(env)
    fstream = torch.cuda.Stream(dev)
    fsp = fstream.cuda_stream
    ev_out = [torch.cuda.Event() for _ in range(2)]     # slab written (kernel stream)
    ev_free = [torch.cuda.Event() for _ in range(2)]    # slab folded (side stream)
    for ev in ev_out + ev_free:
        ev.record(stream)
    if mode == "step":
        step_fn = lib.invsim_step
        calls_per_block = R

        def one(i, row, sl):
            pr, pt, pu = slab_ptrs[sl]
            rc = step_fn(h, ptrs[i % pool], po, pr + 8 * row * N, pt + row * N, pu + row * N, None, sp)
            if rc:
                raise RuntimeError(invsim._capi.last_error(h))
        steps_per_call = 1
    elif mode == "rollout":
        fn = lib.invsim_rollout
        calls_per_block = LPB

        def one(i, row, sl):
            pr, pt, pu = slab_ptrs[sl]
            rc = fn(h, K, ptrs[i % pool], po, pr + 8 * row * N, pt + row * N, pu + row * N, sp)
            if rc:
                raise RuntimeError(invsim._capi.last_error(h))
        steps_per_call = K
    else:
        # the workload's heuristic agent inside the kernel: no action input,
        # the evaluate_agent sums accumulated per env (invsim_rollout_policy)
        import ctypes
        cls_name, arg = wl["agent"]
        spec, keep = getattr(invsim.policies, cls_name)(arg).device_spec(env)
        md = ctypes.c_int32()
        lib.invsim_metrics_dim(h, ctypes.byref(md))
        metrics = torch.zeros((N, md.value), dtype=torch.float64, device=dev)
        fn = lib.invsim_rollout_policy
        calls_per_block = LPB

        def one(i, row, sl):
            pr, pt, pu = slab_ptrs[sl]
            rc = fn(h, K, ctypes.byref(spec), po, pr + 8 * row * N, pt + row * N, pu + row * N, None,
                    metrics.data_ptr(), sp)
            if rc:
                raise RuntimeError(invsim._capi.last_error(h))
        steps_per_call = K
    rows_per_call = steps_per_call

    calls = max(1, steps // steps_per_call)
    warm = max(1, warmup // steps_per_call)
    nblocks = (calls + calls_per_block - 1) // calls_per_block
    # HIP events on the kernel stream around each block of launches: sum of the
    # pairs / launches is the mean launch duration.  torch creates an event at
    # its first record: record every event once here, so creation stays out of
    # the timed region.
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nblocks)]
    for a, b in evs:
        a.record(stream)
        b.record(stream)
    end_ev = torch.cuda.Event()
    end_ev.record(stream)
    blk = [0]

    def region(n_calls, timed):
        for bi in range(0, n_calls, calls_per_block):
            nb = min(calls_per_block, n_calls - bi)
            sl = blk[0] & 1
            if fm == "side":
                stream.wait_event(ev_free[sl])          # this slab's previous fold is done
            if timed:
                evs[bi // calls_per_block][0].record(stream)
            for j in range(nb):
                one(bi + j, j * rows_per_call, sl)
            if timed:
                evs[bi // calls_per_block][1].record(stream)
            rows = nb * rows_per_call
            if fm == "side":
                ev_out[sl].record(stream)
                fstream.wait_event(ev_out[sl])
                _fold_rows(stats, rew[sl], term[sl], trunc[sl], rows, fsp)
                ev_free[sl].record(fstream)
            elif fm == "inline":
                _fold_rows(stats, rew[sl], term[sl], trunc[sl], rows, sp)
            blk[0] += 1

    region(warm, False)
    torch.cuda.synchronize(dev)
    stats.reset_acc()                  # count the episodes that finish in the timed region
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    region(calls, True)
    if args.stop in ("event", "spin"):
        # the end of the work is `stream`'s last event completing
        # (hipEventSynchronize, no device-wide drain); with --fold side the last
        # block's fold runs on fstream, so `stream` waits for it first
        if fm == "side":
            stream.wait_stream(fstream)
        end_ev.record(stream)
        if args.stop == "spin":
            while not end_ev.query():
                pass
        else:
            end_ev.synchronize()
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
    else:
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
    # the closing barrier brackets the region on every rank; each rank's clock
    # stops when its own work is done (not after the barrier's latency, which
    # is tens of us over RCCL against a ~0.2 ms driver-style region)
    if dist.is_initialized():
        dist.barrier()
    el = _span(t0, t1, dev, dist)
    ep = stats.allreduce()                                  # RCCL all-reduce of the timed batch's statistics
    ep["fold"] = fm
    stats.detach()
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / calls
    total_steps = calls * steps_per_call
    # the fast stream reads an 8-B key instead of the 32-B PCG64 state and writes no state back
    dB = -40 if env.demand_stream == "philox" else 0
    B = wl["B_io"] + ((wl["B_state_rollout"] + dB) / K if K else wl["B_state"] + dB)
    if mode == "policy":   # no action input; the per-env metric sums read and written once per launch
        B += -wl["B_act"] + 16 * metrics.shape[1] / K
    achieved = B * N * steps_per_call / (kern_ms * 1e-3) / 1e9
    achieved_wall = B * N * total_steps / el / 1e9
    return dict(el=el, calls=calls, warm=warm, steps_per_call=steps_per_call, total_steps=total_steps,
                N=N, K=K, B=B, kern_ms=kern_ms, achieved=achieved, achieved_wall=achieved_wall, ep=ep)


def run_graph_region(args, env, wl, steps, world, dev, gen, dist):
    """The step region as HIP-graph replays ("hipEvent around K
    launches (or a graph replay)"), reported beside the eager step line: one
    replay = Q whole episode cycles (Q <= 4, at most the requested steps'
    worth), Q * (periods + 1) invsim_step calls under NEXT_STEP (each writing
    its row of a [Q C, N] output slab) and one episode fold of the slab -- the
    eager region folds every 128 steps -- recorded once with
    invsim.graphs.StepGraph.  ceil(steps / (Q C)) replays, barrier +
    synchronize around them, max over ranks; one hipGraphLaunch per replay
    takes host submission out of the loop."""
    import torch
    import invsim
    from invsim.distributed import EpisodeStats
    from invsim.graphs import StepGraph
    lib, h = env._lib, env._h
    N, O = env.num_envs, env.obs_dim
    C1 = env._horizon() + 1
    Q = max(1, min(4, 128 // C1, -(-steps // C1)))   # cycles per replay
    # Newsvendor's demand lookahead flips its slot on step_limit - 1 launches of a
    # cycle: with an odd count a replay of Q cycles would not start where it was
    # recorded (invsim_capture_end refuses the capture), so Q is made even there
    if env.family == invsim._capi.INVSIM_NEWSVENDOR and (C1 - 2) % 2 and Q % 2:
        Q = Q + 1 if Q < 4 else Q - 1
    C = Q * C1
    pool = max(1, args.pool)
    acts = make_actions(env, pool, 0, gen)
    rew = torch.empty((C, N), dtype=torch.float64, device=dev)
    term = torch.empty((C, N), dtype=torch.bool, device=dev)
    trunc = torch.empty((C, N), dtype=torch.bool, device=dev)
    obs = torch.empty((N, O), dtype=env.obs_dtype, device=dev)
    stats = EpisodeStats(N, dev)
    sink = fold_mode(args, env) == "sink"
    if sink:                    # the captured step kernels fold into `stats` themselves
        stats.attach(env)

    def cycle():
        sp = torch._C._cuda_getCurrentRawStream(dev.index)
        for i in range(C):
            rc = lib.invsim_step(h, acts[i % pool].data_ptr(), obs.data_ptr(), rew[i].data_ptr(),
                                 term[i].data_ptr(), trunc[i].data_ptr(), None, sp)
            if rc:
                raise RuntimeError(invsim._capi.last_error(h))
        if not sink:
            stats.update_block(rew, term, trunc, stream=sp)
    g = StepGraph(env, cycle, warmup=1)
    reps = max(1, -(-steps // C))
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    e1.record(stream)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize(dev)
    stats.reset_acc()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps):
        g.replay()
    e1.record(stream)
    e1.synchronize()
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():                 # bracket; each rank's clock stopped at its own end (above)
        dist.barrier()
    el = _span(t0, t1, dev, dist)
    ep = stats.allreduce()
    stats.detach()
    total = reps * C
    return {"value": total * N * world / el, "unit": "env-steps/s", "steps": total, "replays": reps,
            "steps_per_replay": C, "ms_per_step": el * 1e3 / total,
            "event_ms_per_step": e0.elapsed_time(e1) / total,
            "cycles_per_replay": Q,
            "what": "invsim_step x Q (periods+1), with the episode sink in the step kernels or one episode fold "
                    "per replay, one HIP graph (StepGraph)",
            "episode_stats": dict(ep, fold="sink" if sink else "inline",
                                  source="the replays' own episode statistics, one all-reduce after the region")}


def _hbm_counter(traffic, traffic_src, rocprof):
    """The physical HBM rate of the dominant kernel: the PMC counter bytes per
    launch (FETCH_SIZE x2 + WRITE_SIZE, calibrated, tools/pmc_summary.py) over
    the same kernel's rocprofv3 mean duration, against the 8 TB/s peak and the
    ~6.3 TB/s a streaming kernel achieves.  Both figures come from committed
    profiles/rNN files of this workload and mode at this batch size."""
    if not traffic or not rocprof:
        return None
    ach = traffic / rocprof["dominant_ns"]
    return {"achieved": ach, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "frac_of_achievable": ach / HBM_ACHIEVABLE_GBS, "achievable": HBM_ACHIEVABLE_GBS,
            "bytes_per_launch": traffic, "dominant_ns": rocprof["dominant_ns"],
            "sources": [traffic_src, rocprof["source"]],
            "what": "counter HBM bytes per launch / rocprofv3 mean duration of the dominant kernel"}


def _roofline(r, traffic, traffic_src, rocprof=None, issue=None):
    out = {"bound": "hbm", "achieved": r["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": r["achieved"] / HBM_PEAK_GBS,
            "frac_kernel": r["achieved"] / HBM_PEAK_GBS,
            "frac_wall": r["achieved_wall"] / HBM_PEAK_GBS,
            "frac_is": "frac_kernel: algorithmic bytes per launch / mean launch duration (HIP events on the "
                       "kernel stream); frac_wall: value per GPU x bytes_per_env_step / peak (SURVEY 8(d))",
            "traffic": traffic,
            "traffic_unit": "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, calibrated)",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": r["B"] * r["N"] * r["steps_per_call"],
            "bytes_per_env_step": r["B"], "kernel_ms_mean": r["kern_ms"],
            "kernel_timing": "HIP events on the kernel stream around each block of launches / launches "
                             "(every env-step launch: the dominant kernel and the NEXT_STEP reset launches)"}
    if rocprof:
        rocprof["event_over_all_launches"] = r["kern_ms"] * 1e6 / rocprof["all_step_launches_ns"]
        out["rocprof"] = rocprof
    hc = _hbm_counter(traffic, traffic_src, rocprof)
    if hc:
        out["hbm_counter"] = hc
    if issue:
        out["issue"] = issue
    return out


# invsim kernels that run env steps (a launch of invsim_step / _rollout /
# _rollout_policy); the rest of a kernel-stats file is the episode fold, explicit
# reset / seed kernels and torch's own kernels
_STEP_KERNELS = ("_split_kernel", "_step1_kernel", "_step2_kernel", "_run_kernel", "_spec_kernel", "_roll",
                 "_commit_kernel")


def _newest(pattern):
    import glob
    rnd = PROFILE_ROUND or "r[0-9][0-9]"
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", rnd, pattern)))
    return fs[-1] if fs else None


def _rocprof(workload, mode, n_match, alg_bytes):
    """The newest round's rocprofv3 kernel stats of this workload and mode
    (profiles/rNN/<workload>_<mode>_kernel_stats.csv, the same bench command
    under --kernel-trace --stats): the dominant kernel's mean duration and the
    frac on it, and the mean over every env-step launch (the dominant kernel,
    the NEXT_STEP reset launch, lookahead commits), which is what the HIP-event
    figure averages."""
    import csv
    f = _newest(f"{workload}_{mode}_kernel_stats.csv")
    if not f or not n_match:
        return None
    rows = [r for r in csv.DictReader(open(f))
            if r["Name"].startswith(("void invsim::", "invsim::")) and any(k in r["Name"] for k in _STEP_KERNELS)]
    if not rows:
        return None
    dom = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    calls = sum(int(r["Calls"]) for r in rows)
    mean_all = sum(float(r["TotalDurationNs"]) for r in rows) / calls
    dom_ns = float(dom["AverageNs"])
    import re
    m = re.search(r"(\w+_kernel)", dom["Name"])
    return {"source": os.path.relpath(f, ROOT), "dominant_kernel": m.group(1) if m else dom["Name"][:80],
            "dominant_ns": dom_ns, "dominant_share_of_launches": int(dom["Calls"]) / calls,
            "frac_dominant": alg_bytes / dom_ns / HBM_PEAK_GBS,
            "all_step_launches_ns": mean_all, "frac_all_launches": alg_bytes / mean_all / HBM_PEAK_GBS}


def _issue(workload, mode, kern_ms, n_match):
    """Issue-rate roofline of the Newsvendor kernels, whose bound is the
    instruction stream, not HBM: VALU + SALU wave-instructions per
    launch (SQ_INSTS_VALU + SQ_INSTS_SALU, newest profiles/rNN/sq_newsvendor.json)
    over what 1 024 SIMDs issue in the launch's duration at the measured best
    SIMD issue interval (v_add_u32 with four waves: 2.2 cycles,
    profiles/r04/launch/valu_rates.txt) at 2.4 GHz."""
    if workload != "newsvendor" or mode not in ("step", "rollout") or not n_match:
        return None          # the SQ passes ran the default batch with the numpy stream only
    f = _newest("sq_newsvendor.json")
    if not f:
        return None
    rec = json.load(open(f)).get(mode)
    if not rec:
        return None
    c = rec["counters_mean_per_dispatch"]
    insts = c["SQ_INSTS_VALU"] + c["SQ_INSTS_SALU"]
    cap = 1024 * kern_ms * 1e-3 * 2.4e9 / 2.2
    return {"bound": "issue", "instructions_per_launch": insts, "achieved": insts / (kern_ms * 1e-3),
            "peak": 1024 * 2.4e9 / 2.2, "unit": "wave-instructions/s", "frac": insts / cap,
            "source": os.path.relpath(f, ROOT),
            "what": "VALU + SALU wave-instructions per launch (SQ) / (1024 SIMDs x launch cycles at 2.4 GHz / "
                    "2.2 cycles per instruction)"}


def _pmc(workload, mode, n_match):
    """The newest round's PMC summary for this workload and mode
    (profiles/rNN/pmc_<workload>[_rollout].json, tools/pmc_summary.py)."""
    suffix = {"step": "", "rollout": "_rollout", "policy": "_policy"}[mode]
    f = _newest(f"pmc_{workload}{suffix}.json")
    if not f or not n_match:
        return None, None
    rec = json.load(open(f))
    return rec["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)


def config_line(args, name, world, rank, dev, dist):
    """A compact line for another BASELINE config, timed in the same run the
    same way as the headline (eager step region, then the fused K-step rollout
    region): Newsvendor 65 536 (config 2), the per-GPU shard of InvMgmt
    LostSales 262 144 over 8 GPUs (config 4: 32 768 envs, global offset
    rank x 32 768) and NetInvMgmt Backlog 32 768 (config 5)."""
    import torch
    import invsim
    wl = WORKLOADS[name]
    n = wl["n"]
    env = getattr(invsim, wl["cls"])(n, device=dev, global_offset=rank * n, copy=False)
    gen = torch.Generator(device=dev)
    gen.manual_seed(4321 + rank)
    env.reset(seed=0)
    r = run_region(args, env, wl, "step", args.steps, args.warmup, world, dev, gen, dist)
    traffic, tsrc = _pmc(name, "step", True)
    roof = _roofline(r, traffic, tsrc, _rocprof(name, "step", True, r["B"] * n), _issue(name, "step", r["kern_ms"], True))
    C = env._horizon() + 1
    Kr = args.rollout_k
    unit = C * Kr
    rr = run_region(args, env, wl, "rollout", unit * max(1, -(-args.steps // unit)), 2 * Kr, world, dev, gen, dist)
    t2, s2 = _pmc(name, "rollout", True)
    roof2 = _roofline(rr, t2, s2, _rocprof(name, "rollout", True, rr["B"] * n * rr["K"]),
                      _issue(name, "rollout", rr["kern_ms"], True))

    def compact(x, ro):
        out = {"value": x["total_steps"] * n * world / x["el"], "ms_per_step": x["el"] * 1e3 / x["total_steps"],
               "steps": x["total_steps"], "bytes_per_env_step": x["B"], "frac": ro["frac_kernel"],
               "frac_wall": ro["frac_wall"]}
        if "rocprof" in ro:
            out["frac_rocprof"] = ro["rocprof"]["frac_dominant"]
            out["dominant_kernel"] = ro["rocprof"]["dominant_kernel"]
        if "hbm_counter" in ro:
            out["hbm_counter"] = {k: ro["hbm_counter"][k] for k in ("achieved", "frac", "frac_of_achievable")}
        if "issue" in ro:
            out["issue_frac"] = ro["issue"]["frac"]
        return out
    line = {"workload": wl["desc"], "envs_per_gpu": n, "global_envs": n * world, "dtype": wl["dtype"],
            "step": compact(r, roof), "rollout": dict(compact(rr, roof2), K=rr["K"])}
    del env
    return line


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL ("nccl") over xGMI, one rank per GPU; INVSIM_BENCH_BACKEND=gloo
    # rehearses the multi-rank path with several ranks on one GPU
    backend = os.environ.get("INVSIM_BENCH_BACKEND", "nccl")
    # a process group whenever torch.distributed.run started this process (also
    # a 1-rank one: it runs the same RCCL calls an 8-GPU node makes); none for a
    # plain `python bench.py`
    if "WORLD_SIZE" in os.environ:
        ndev = torch.cuda.device_count()
        if backend == "nccl":
            if local >= ndev:
                raise RuntimeError(f"bench.py: LOCAL_RANK {local} but only {ndev} GPUs visible (RCCL needs one GPU per rank)")
        else:
            local = local % ndev
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
    env = getattr(invsim, wl["cls"])(n, device=dev, global_offset=rank * n, copy=False,
                                     demand_stream=args.demand_stream)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    env.reset(seed=0)
    r = run_region(args, env, wl, args.mode, args.steps, args.warmup, world, dev, gen, dist)
    full = n == wl["n"] and not args.strong and args.demand_stream == "numpy"   # the PMC files are of that run
    traffic, traffic_src = _pmc(args.workload, args.mode, full)
    N = r["N"]
    out = {
        "metric": "env-steps/sec (batched) at 1/2/4/8 MI355X; % HBM roofline",
        "value": r["total_steps"] * N * world / r["el"],
        "unit": "env-steps/s",
        "n_gpus": world,
        "ranks": dist.get_world_size() if dist.is_initialized() else 1,
        "steps": r["total_steps"],
        "warmup": r["warm"] * r["steps_per_call"],
        "ms_per_step": r["el"] * 1e3 / r["total_steps"],
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": wl["dtype"],
        "data": "synthetic (pre-generated random actions in HBM, seeds 0..N-1 per global env index)",
        "config": {"workload": wl["desc"], "envs_per_gpu": N, "global_envs": N * world,
                   "mode": args.mode + (f" K={r['K']}" if r["K"] else "") +
                           (f" agent={wl['agent'][0]}({wl['agent'][1]})" if args.mode == "policy" else ""),
                   "autoreset": "next_step",
                   "parallelism": f"dp{world} (env sharding, no data-path collective)",
                   "backend": (backend if dist.is_initialized() else None), "demand_stream": args.demand_stream},
        "roofline": _roofline(r, traffic, traffic_src,
                              _rocprof(args.workload, args.mode, full, r["B"] * N * r["steps_per_call"]),
                              _issue(args.workload, args.mode, r["kern_ms"], full)),
        "episode_stats": dict(r["ep"], source="timed batch: the episode sink in the step kernels (fold 'sink') or "
                                              "the HIP episode fold of the timed steps' outputs (fold 'inline'), "
                                              "one all-reduce after the region"),
    }
    C = env._horizon() + 1                                  # steps per episode cycle (NEXT_STEP)
    if r["total_steps"] < C:
        out["episode_stats"]["note"] = (
            f"the timed window holds {r['total_steps']} steps, fewer than one episode cycle ({C} steps: "
            f"{C - 1} periods + the NEXT_STEP reset step), so no episode ends inside it; the rollout "
            f"region's episode_stats cover whole cycles")
    if args.mode == "step" and not args.no_rollout_line:
        # the fused K-step rollout of the same handle, timed the same way, over a
        # whole number of episode cycles (every env finishes the same number of
        # episodes whatever the phase it starts in)
        Kr = args.rollout_k
        unit = C * Kr
        rsteps = unit * max(1, -(-args.steps // unit))
        rr = run_region(args, env, wl, "rollout", rsteps, 2 * Kr, world, dev, gen, dist)
        t2, s2 = _pmc(args.workload, "rollout", full)
        out["rollout"] = {"value": rr["total_steps"] * N * world / rr["el"], "unit": "env-steps/s",
                          "steps": rr["total_steps"], "launches": rr["calls"], "K": rr["K"],
                          "ms_per_launch": rr["el"] * 1e3 / rr["calls"],
                          "roofline": _roofline(rr, t2, s2,
                                                _rocprof(args.workload, "rollout", full, rr["B"] * N * rr["K"]),
                                                _issue(args.workload, "rollout", rr["kern_ms"], full)),
                          "episode_stats": dict(rr["ep"], cycles=rr["total_steps"] // C,
                                                source="timed rollout batch: the episode sink in the rollout "
                                                       "kernels, or the HIP episode fold between launch "
                                                       "blocks; one all-reduce after the region")}
    if args.mode == "step" and not args.no_graph_line and args.demand_stream == "numpy":
        out["graph"] = run_graph_region(args, env, wl, args.steps, world, dev, gen, dist)
    if (args.mode == "step" and args.workload == "invmgmt_backlog" and not args.n_envs and not args.strong
            and args.demand_stream == "numpy" and not args.no_config_lines):
        out["configs"] = {k: config_line(args, k, world, rank, dev, dist)
                          for k in ("newsvendor", "invmgmt_lostsales", "net_backlog")}
        out["configs"]["note"] = ("BASELINE configs 2, 4 (the per-GPU shard of 262 144 envs over 8 GPUs) and 5, "
                                  "timed in this run like the headline: eager step region, then fused rollouts")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wl, args.cpu_seconds)
        rv, rwhat = REFERENCE_PYTHON[args.workload]
        out["cpu_baseline"]["reference_python"] = {
            "value": rv, "unit": "env-steps/s", "cores": 8,
            "what": f"the reference's own {rwhat} step (numpy/networkx), 8 independent processes, constant actions",
            "host": "Intel Xeon KVM guest, 8 vCPU (the survey container; the reference cannot run on the GPU box)",
            "source": "BASELINE.md section 2 (measured, not re-timed here)"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
