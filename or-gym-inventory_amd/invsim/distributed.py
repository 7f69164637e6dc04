"""Multi-GPU helpers: one process per GPU, envs sharded by global index.

The env path has no cross-env exchange, so sharding is pure data parallelism:
rank r of W owns global env indices ``[offset, offset + n)`` and seeds env i
with ``seed + offset + i`` (``global_offset`` of the VectorEnv), which makes
every env's trajectory identical for any W.  The only collective is the
episodic-return reduction the harness reports (mean / std / count of episode
returns, ``benchmark_InvManagementBacklogEnv.py:389-440``): ONE all-reduce of
three f64 per episode boundary over RCCL (torch.distributed "nccl" backend on
ROCm), latency-bound at 24 bytes.
"""
import torch
import torch.distributed as dist


def shard_range(global_envs, rank, world):
    """Contiguous, balanced shard of `global_envs` for `rank` -> (offset, count)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(int(global_envs), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


class EpisodeStats:
    """Accumulates per-env returns on device; folds finished episodes into
    [sum, sum of squares, count] and all-reduces them across ranks."""

    def __init__(self, num_envs, device):
        self.ret = torch.zeros(num_envs, dtype=torch.float64, device=device)
        self.acc = torch.zeros(3, dtype=torch.float64, device=device)

    def update(self, reward, done):
        """reward [N] f64, done [N] bool (terminated | truncated) of one step."""
        self.ret += reward
        d = done.to(torch.float64)
        r = self.ret * d
        self.acc += torch.stack([r.sum(), (r * r).sum(), d.sum()])
        self.ret *= (1.0 - d)

    def allreduce(self, group=None):
        out = self.acc.clone()
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        s, s2, n = out.tolist()
        mean = s / n if n else float("nan")
        var = max(s2 / n - mean * mean, 0.0) if n else float("nan")
        return {"episodes": n, "mean_return": mean, "std_return": var ** 0.5, "sum": s, "sum_sq": s2}
