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
    assert d["config"]["envs_per_gpu"] == 65536
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1


def test_bench_two_ranks_gloo_rehearsal():
    env = dict(os.environ, INVSIM_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--n-envs", "8192"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _last_json(p.stdout)
    _check_line(d, 2, 20, 5)
    assert d["config"]["backend"] == "gloo"
    assert "cpu_baseline" not in d                      # rank 0 at N=1 only
    # the statistics all-reduce summed both ranks' episodes
    assert d["episode_stats"]["episodes"] == 2 * 4096
