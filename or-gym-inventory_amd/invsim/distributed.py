"""Multi-GPU helpers: one process per GPU, envs sharded by global index.

The env path has no cross-env exchange, so sharding is pure data parallelism:
rank r of W owns global env indices ``[offset, offset + n)`` and seeds env i
with ``seed + offset + i`` (``global_offset`` of the VectorEnv), which makes
every env's trajectory identical for any W.  The only collective is the
episodic-return reduction the harness reports (mean / std / count of episode
returns, ``benchmark_InvManagementBacklogEnv.py:389-440``): ONE all-reduce of
four f64 over RCCL (torch.distributed "nccl" backend on ROCm), latency-bound
at 32 bytes, after each rank sums its per-group partials.
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
    """Accumulates per-env returns; folds finished episodes into
    [sum, sum of squares, episodes, sum of all rewards] and all-reduces them
    across ranks.

    Device statistics are kept as per-64-env-group partials ``part``
    [ceil(N / 64), 4] (``acc`` is their column sum): either folded from output
    rows by the HIP kernel ``invsim_episode_fold_groups`` (``update_block``),
    or folded inside the step / rollout kernels themselves once the stats are
    attached to an env as its episode sink (``attach``, ``invsim_set_episode_sink``),
    which is the same arithmetic with no second pass over the outputs.  Host
    tensors (a CPU rehearsal stepping the oracle) are folded with the same
    arithmetic in torch into a single row: there is no device data to hand the
    kernel.
    """

    def __init__(self, num_envs, device):
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:      # "cuda" -> the current device, explicitly
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.num_envs = int(num_envs)
        self.ret = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        groups = (self.num_envs + 63) // 64 if dev.type == "cuda" else 1
        self.part = torch.zeros((max(groups, 1), 4), dtype=torch.float64, device=self.device)
        self._env = None

    @property
    def acc(self):
        """[sum of finished-episode returns, sum of their squares, episodes, sum of rewards]"""
        return self.part.sum(0)

    def reset_acc(self):
        """Forget the folded episodes; running returns carry on."""
        self.part.zero_()

    def attach(self, env):
        """Make these statistics `env`'s episode sink: every step / rollout of
        the env folds its rows here on the device (invsim_set_episode_sink)."""
        from . import _capi
        if self.device.type != "cuda" or env.device != self.device or env.num_envs != self.num_envs:
            raise ValueError("EpisodeStats.attach: a CUDA EpisodeStats of the env's device and size")
        _capi.check(_capi.lib().invsim_set_episode_sink(env._h, self.ret.data_ptr(), self.part.data_ptr()),
                    env._h, "invsim_set_episode_sink")
        self._env = env
        env._episode_sink = self           # the env's kernels write ret / part: keep them alive with it

    def detach(self):
        if self._env is not None:
            from . import _capi
            _capi.check(_capi.lib().invsim_set_episode_sink(self._env._h, None, None), self._env._h,
                        "invsim_set_episode_sink")
            self._env._episode_sink = None
            self._env = None

    def update(self, reward, done):
        """reward [N] f64, done [N] bool (terminated | truncated) of one step."""
        self.update_block(reward.reshape(1, -1), None, done.reshape(1, -1))

    def update_block(self, reward, terminated=None, truncated=None, stream=None):
        """reward [K, N] f64; terminated / truncated [K, N] bool (either may be
        None) of K consecutive steps."""
        K, N = reward.shape
        if N != self.num_envs:
            raise ValueError(f"EpisodeStats: {N} envs, expected {self.num_envs}")
        flags = [f for f in (terminated, truncated) if f is not None]
        if self.device.type == "cuda":
            from . import _capi
            for f in [reward] + flags:
                if f.device != self.device or not f.is_contiguous() or f.shape != (K, N):
                    raise ValueError("EpisodeStats: outputs must be contiguous [K, N] tensors on the stats device")
            if reward.dtype != torch.float64 or any(f.dtype not in (torch.bool, torch.uint8) for f in flags):
                raise TypeError("EpisodeStats: reward f64, flags bool/uint8")
            ptr = (lambda t: t.data_ptr() if t is not None else None)
            with torch.cuda.device(self.device):           # the launch goes to the stats' GPU
                if stream is None:
                    stream = torch._C._cuda_getCurrentRawStream(self.device.index)
                _capi.check(_capi.lib().invsim_episode_fold_groups(
                    reward.data_ptr(), ptr(terminated), ptr(truncated), K, N, self.ret.data_ptr(),
                    self.part.data_ptr(), stream), None, "invsim_episode_fold_groups")
            return
        done = torch.zeros((K, N), dtype=torch.bool)
        for f in flags:
            done |= f.to(torch.bool)
        for k in range(K):
            self.ret += reward[k]
            d = done[k].to(torch.float64)
            r = self.ret * d
            self.part[0] += torch.stack([r.sum(), (r * r).sum(), d.sum(), reward[k].sum()])
            self.ret *= (1.0 - d)

    def allreduce(self, group=None):
        out = self.acc.clone()
        if dist.is_available() and dist.is_initialized():
            if dist.get_backend(group) == "gloo" and out.is_cuda:
                out = out.cpu()
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        s, s2, n, tot = out.tolist()
        mean = s / n if n else float("nan")
        var = max(s2 / n - mean * mean, 0.0) if n else float("nan")
        return {"episodes": n, "mean_return": mean, "std_return": var ** 0.5, "sum": s, "sum_sq": s2,
                "reward_sum": tot}
