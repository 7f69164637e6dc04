"""bench.py contract on the GPU: one JSON line with the fields the driver and
the judge read, at N=1 and through the multi-rank path (torch.distributed.run,
2 ranks).  RCCL refuses two ranks on one device, so the 2-rank run rehearses
the launcher, sharding, barriers, max-over-ranks timing and the statistics
all-reduce over gloo (INVSIM_BENCH_BACKEND=gloo); on an 8-GPU node the same
code path runs over RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out):
    line = [x for x in out.strip().splitlines() if x.startswith("{")][-1]
    return json.loads(line)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _check_line(d, n_gpus, steps, warmup):
    assert d["metric"] == "env-steps/sec (batched) at 1/2/4/8 MI355X; % HBM roofline"
    assert d["unit"] == "env-steps/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == n_gpus and d["steps"] == steps and d["warmup"] == warmup
    assert d["value"] > 0 and d["ms_per_step"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] < 1.5
    assert r["achieved"] == pytest.approx(r["frac"] * r["peak"])
    assert d["config"]["global_envs"] == n_gpus * d["config"]["envs_per_gpu"]


def test_bench_single_gpu_line():
    p = subprocess.run([sys.executable, "bench.py", "--steps", "20", "--warmup", "5", "--cpu-seconds", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _last_json(p.stdout)
    _check_line(d, 1, 20, 5)
    assert d["ranks"] == 1
    assert d["config"]["envs_per_gpu"] == 65536
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    # the fused rollout region of the same handle rides along
    # over whole episode cycles (31 launches x 30 steps = 30 cycles of 31 steps),
    # so every env finishes exactly 30 episodes in its timed window
    ro = d["rollout"]
    assert ro["K"] == 30 and ro["steps"] == 930 and ro["value"] > 0
    assert 0 < ro["roofline"]["frac"] < 1.5
    rep = ro["episode_stats"]
    assert rep["episodes"] == 30 * 65536 and rep["cycles"] == 30
    assert rep["mean_return"] == rep["mean_return"] and rep["std_return"] > 0
    # timed steps 5..24: no episode ends (the line says why), every reward of the region is folded
    ep = d["episode_stats"]
    assert ep["episodes"] == 0 and ep["reward_sum"] != 0 and "no episode ends" in ep["note"]
    # the same step loop as graph replays: one 31-step cycle (+ fold) per replay
    # (at most the requested steps' worth of cycles per replay)
    gr = d["graph"]
    assert gr["steps"] == 31 and gr["replays"] == 1 and gr["cycles_per_replay"] == 1 and gr["value"] > 0
    assert gr["episode_stats"]["episodes"] == 65536


def test_bench_episode_stats_from_timed_batch():
    """steps 5..66 contain two truncations per env (periods 30, 61 of the
    31-call NEXT_STEP cycle): the fold counts exactly 2 N episodes."""
    p = subprocess.run([sys.executable, "bench.py", "--steps", "62", "--warmup", "5", "--no-cpu-baseline",
                        "--no-rollout-line", "--n-envs", "4096"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _last_json(p.stdout)
    assert d["episode_stats"]["episodes"] == 2 * 4096
    assert d["episode_stats"]["mean_return"] == d["episode_stats"]["mean_return"]   # not NaN


def test_bench_two_ranks_gloo_rehearsal():
    env = dict(os.environ, INVSIM_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--n-envs", "8192", "--no-rollout-line"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _last_json(p.stdout)
    _check_line(d, 2, 20, 5)
    assert d["config"]["backend"] == "gloo"
    assert "cpu_baseline" not in d                      # rank 0 at N=1 only
    assert d["ranks"] == 2


def _bench_spawned(extra, rollout=False):
    """plain `bench.py --gpus 2` (no torchrun around it): bench.py starts the ranks"""
    env = dict(os.environ, INVSIM_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--warmup", "5"] + ([] if rollout else ["--no-rollout-line"]) + extra
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    return _last_json(p.stdout)


def test_bench_gpus_flag_starts_ranks_weak():
    d = _bench_spawned(["--steps", "62", "--n-envs", "8192"])
    _check_line(d, 2, 62, 5)
    assert d["ranks"] == 2 and d["config"]["backend"] == "gloo" and d["scaling"] == "weak"
    assert d["config"]["envs_per_gpu"] == 8192 and d["config"]["global_envs"] == 2 * 8192
    # the statistics all-reduce summed both ranks' episodes of the timed batch
    assert d["episode_stats"]["episodes"] == 2 * 2 * 8192


def test_bench_gpus_flag_strong_net():
    """--strong (config 5: 32 768 Net envs split over the ranks).  The per-rank
    step is latency-bound at these sizes, so the line carries the
    modes that hold up beside the eager one: the fused K=30 rollout (the
    highest absolute rate) and the StepGraph replay, both over the same
    per-rank shard and timed the same way."""
    d = _bench_spawned(["--steps", "20", "--workload", "net_backlog", "--strong"], rollout=True)
    _check_line(d, 2, 20, 5)
    assert d["scaling"] == "strong" and d["ranks"] == 2
    assert d["config"]["envs_per_gpu"] == 16384 and d["config"]["global_envs"] == 32768
    ro, gr = d["rollout"], d["graph"]
    assert ro["K"] == 30 and ro["value"] > d["value"] and 0 < ro["roofline"]["frac"] < 1.5
    assert ro["episode_stats"]["episodes"] == ro["episode_stats"]["cycles"] * 32768
    assert gr["value"] > 0 and gr["steps"] % 31 == 0


@pytest.mark.parametrize("wl", ["invmgmt_backlog", "newsvendor", "net_backlog"])
def test_bench_policy_mode(wl):
    """--mode policy: K-step rollouts with the workload's heuristic agent in the kernel"""
    p = subprocess.run([sys.executable, "bench.py", "--workload", wl, "--mode", "policy", "--steps", "60",
                        "--warmup", "30", "--no-cpu-baseline", "--no-rollout-line"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _last_json(p.stdout)
    assert d["value"] > 0 and d["steps"] == 60 and "agent=" in d["config"]["mode"]
    assert d["episode_stats"]["reward_sum"] != 0
