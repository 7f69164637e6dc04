"""CPU, world_size 2 over gloo: the multi-GPU path's host logic (contiguous
shards keyed by global env index, seeds seed+global_index, one all-reduce of
episodic-return statistics).  Each rank steps its shard with the CPU oracle
standing in for the GPU (test infrastructure only)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_shard_range_partitions():
    from invsim.distributed import shard_range
    for G in (1, 2, 3, 4, 8):
        for n in (0, 1, 7, 65536, 262144, 1000003):
            spans = [shard_range(n, r, G) for r in range(G)]
            assert sum(c for _, c in spans) == n
            assert all(spans[r][0] + spans[r][1] == spans[r + 1][0] for r in range(G - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_global, seed, out_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "or-gym-inventory_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import pyoracle
    from invsim.distributed import EpisodeStats, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, n = shard_range(n_global, rank, world)
    env = pyoracle.OracleInvMgmt(n, backlog=False)
    env.seed(range(seed + off, seed + off + n))
    env.reset()
    rng = np.random.default_rng(123)
    acts = rng.integers(0, 231, size=(30, n_global, 3))
    stats = EpisodeStats(n, torch.device("cpu"))
    obs_all = []
    for k in range(30):
        o, r, tr = env.step(acts[k, off:off + n])
        obs_all.append(o)
        stats.update(torch.from_numpy(r), torch.from_numpy(tr))
    res = stats.allreduce()
    np.save(os.path.join(out_dir, f"obs_{rank}.npy"), np.stack(obs_all))
    np.save(os.path.join(out_dir, f"stats_{rank}.npy"),
            np.array([res["episodes"], res["sum"], res["sum_sq"]]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shards_and_stats(tmp_path, oracle):
    n_global, seed, world = 1001, 500, 2
    mp.spawn(_worker, args=(world, _free_port(), n_global, seed, str(tmp_path)), nprocs=world,
             join=True)
    # single-process reference run over all envs
    env = oracle.OracleInvMgmt(n_global, backlog=False)
    env.seed(range(seed, seed + n_global))
    env.reset()
    rng = np.random.default_rng(123)
    acts = rng.integers(0, 231, size=(30, n_global, 3))
    ret = np.zeros(n_global)
    obs = []
    for k in range(30):
        o, r, tr = env.step(acts[k])
        obs.append(o)
        ret += r
    obs = np.stack(obs)
    from invsim.distributed import shard_range
    for r in range(world):
        off, n = shard_range(n_global, r, world)
        assert np.array_equal(np.load(tmp_path / f"obs_{r}.npy"), obs[:, off:off + n])
        st = np.load(tmp_path / f"stats_{r}.npy")
        assert st[0] == n_global
        assert st[1] == pytest.approx(ret.sum(), rel=1e-12)
        assert st[2] == pytest.approx((ret * ret).sum(), rel=1e-12)


def _span_worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r started at 10 + r and ended at 20 - 3 r: the span is from the
    # earliest start (10) to the latest end (20), not the longest duration (10)
    el = bench._span(10.0 + rank, 20.0 - 3 * rank, torch.device("cpu"), dist)
    np.save(os.path.join(out_dir, f"span_{rank}.npy"), np.array([el]))
    dist.destroy_process_group()


def test_gloo_world2_bench_span(tmp_path):
    """bench.py's multi-rank clock: earliest start to latest end
    over the ranks, on the node's shared monotonic clock."""
    mp.spawn(_span_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert np.load(tmp_path / f"span_{r}.npy")[0] == 10.0
