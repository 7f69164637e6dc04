"""Device-side heuristic agents and batched ``evaluate_agent``.

The reference's benchmark scripts drive one env per episode from Python:
``agent.get_action(obs, env)`` then ``env.step``, accumulating per-episode sums
(``evaluate_agent``).  Here the agent runs inside the step kernel
(``invsim_rollout_policy``): N episodes advance together with no host round
trip, and the per-env sums come back as one array.

Agents (restated from the reference, same names and constructor arguments):

* ``BaseStockAgent(safety_factor)``        benchmark_InvManagementBacklogEnv.py:142-198
  (and benchmark_InvManagementLostSalesEnv.py:137-165), InvMgmt envs
* ``ConstantOrderAgent(order_fraction)``   benchmark_NetInvMgmtBacklogEnv.py:119-135
  (and benchmark_NetInvMgmtLostSalesEnv.py:131-142), any env
* ``OrderUpToHeuristicAgent(safety_factor)`` benchmark_newsvendor.py:97-111, Newsvendor
* ``ClassicNewsvendorAgent(cr_method, safety_factor)`` benchmark_newsvendor.py:113-161,
  Newsvendor (scipy ``poisson.ppf`` restated on device, float32 loops included)
* ``sSPolicyAgent(s_quantile, S_buffer_factor)`` benchmark_newsvendor_sb3_rllib.py:363-371,
  Newsvendor (the module's last definition; ``s_quantile`` is unused there too)

``evaluate_agent(agent, env_cls, env_config, n_episodes, seed_offset)`` returns
the reference's summary columns (benchmark_InvManagementBacklogEnv.py:346-440,
benchmark_NetInvMgmtLostSalesEnv.py:241-312, benchmark_newsvendor.py:219-262):
episode i is env i seeded ``seed_offset + i``.
"""
import ctypes as C
import time

import numpy as np
import torch

from . import _capi


class _Agent:
    kind = None
    name = "agent"

    def device_spec(self, env):
        """(PolicySpec, keep-alive) for invsim_rollout_policy."""
        raise NotImplementedError


class BaseStockAgent(_Agent):
    """Independent base-stock level (L_i + 1) * mu * safety_factor per stage."""

    def __init__(self, safety_factor=1.0):
        self.name = f"BaseStock_SF={safety_factor:.1f}"
        self.safety_factor = safety_factor

    def device_spec(self, env):
        if env.family != _capi.INVSIM_INVMGMT:
            raise TypeError("BaseStockAgent needs an InvManagement env")
        mu = env.dist_param.get("mu", 10)       # the agent's own default (:156)
        return _capi.PolicySpec(_capi.POLICY_KINDS["base_stock"], 0, float(self.safety_factor), float(mu), None), None


class ConstantOrderAgent(_Agent):
    """order_fraction * action_space.high every step (inf bounds -> 1000)."""

    def __init__(self, order_fraction=0.1):
        self.name = f"ConstantOrder_{order_fraction * 100:.0f}%"
        self.order_fraction = order_fraction

    def action(self, env):
        sp = env.single_action_space
        high = np.array(sp.high, copy=True)
        high[high == np.inf] = 1000
        return (high * self.order_fraction).astype(sp.dtype)

    def device_spec(self, env):
        a = np.ascontiguousarray(self.action(env))
        return _capi.PolicySpec(_capi.POLICY_KINDS["constant"], 0, 0.0, 0.0, a.ctypes.data), a


class OrderUpToHeuristicAgent(_Agent):
    """Order up to mu * (lead_time + 1) * safety_factor over the pipeline."""

    def __init__(self, safety_factor=1.0):
        self.name = f"OrderUpTo_SF={safety_factor:.1f}"
        self.safety_factor = safety_factor

    def device_spec(self, env):
        if env.family != _capi.INVSIM_NEWSVENDOR:
            raise TypeError("OrderUpToHeuristicAgent needs a Newsvendor env")
        return _capi.PolicySpec(_capi.POLICY_KINDS["order_up_to"], 0, float(self.safety_factor), 0.0, None), None


class ClassicNewsvendorAgent(_Agent):
    """Order up to poisson.ppf(critical ratio, mu * (lead_time + 1) * sf) over
    the pipeline; cr_method 'k_vs_h' (k / (h + k), also any unknown method) or
    'profit_margin' ((p - c + k) / (p - c + k + h)), falling back to OrderUpTo
    without the safety factor when the ratio is undefined."""

    def __init__(self, cr_method="k_vs_h", safety_factor=1.0):
        self.name = f"ClassicNV_SF={safety_factor:.1f}_{cr_method}"
        self.cr_method = cr_method
        self.safety_factor = safety_factor

    def device_spec(self, env):
        if env.family != _capi.INVSIM_NEWSVENDOR:
            raise TypeError("ClassicNewsvendorAgent needs a Newsvendor env")
        variant = 1 if self.cr_method == "profit_margin" else 0
        return _capi.PolicySpec(_capi.POLICY_KINDS["classic_nv"], variant, float(self.safety_factor), 0.0,
                                None), None


class sSPolicyAgent(_Agent):
    """(s, S): s = poisson.ppf(clip(k / (h + k), 0.001, 0.999), mu * (lead_time + 1)),
    S = s * S_buffer_factor; order S - position when the position is below s."""

    def __init__(self, s_quantile=0.5, S_buffer_factor=1.2):
        self.name = f"sS_Policy(s={s_quantile:.2f},S={S_buffer_factor:.1f}s)"
        self.s_quantile = s_quantile
        self.S_buffer_factor = S_buffer_factor

    def device_spec(self, env):
        if env.family != _capi.INVSIM_NEWSVENDOR:
            raise TypeError("sSPolicyAgent needs a Newsvendor env")
        return _capi.PolicySpec(_capi.POLICY_KINDS["ss"], 0, float(self.S_buffer_factor), 0.0, None), None


def rollout_policy(env, agent, K, obs=False, rewards=True, actions=False, metrics=None):
    """K steps of every env of ``env`` under ``agent`` (in-kernel).  Returns a
    dict with the requested device tensors; ``metrics`` (float64 [N, M]) is
    accumulated in place when given."""
    spec, keep = agent.device_spec(env)
    N, dev = env.num_envs, env.device
    out = {}
    o = torch.empty((K, N, env.obs_dim), dtype=env.obs_dtype, device=dev) if obs else None
    if rewards:
        out["reward"] = torch.empty((K, N), dtype=torch.float64, device=dev)
        out["terminated"] = torch.empty((K, N), dtype=torch.bool, device=dev)
        out["truncated"] = torch.empty((K, N), dtype=torch.bool, device=dev)
    # the kernels record the agent's order of every stepped env; a NEXT_STEP
    # reset step (whose action the env ignores) keeps the 0 written here
    a = torch.zeros((K, N, env.action_dim), dtype=env.act_dtype, device=dev) if actions else None
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    _capi.check(env._lib.invsim_rollout_policy(
        env._h, int(K), C.byref(spec), p(o), p(out.get("reward")), p(out.get("terminated")),
        p(out.get("truncated")), p(a), p(metrics), env._stream()), env._h, "rollout_policy")
    del keep
    if obs:
        out["obs"] = o
    if actions:
        out["actions"] = a
    return out


def metrics_dim(env):
    d = C.c_int32()
    _capi.check(env._lib.invsim_metrics_dim(env._h, C.byref(d)), env._h, "metrics_dim")
    return d.value


def summarize(family, m, main_nodes=None):
    """Per-episode summary columns from the accumulated sums, with the
    reference's float expressions."""
    m = np.asarray(m, np.float64)
    rows = {"TotalReward": m[:, 0], "Steps": m[:, 1].astype(np.int64)}
    if family == _capi.INVSIM_INVMGMT:
        # benchmark_InvManagementBacklogEnv.py:412-415
        steps, dem, sales, stock, inv = m[:, 1], m[:, 2], m[:, 3], m[:, 4], m[:, 5]
        rows["AvgServiceLevel"] = np.array([s / max(1e-6, d) if d > 1e-6 else 1.0 for s, d in zip(sales, dem)])
        rows["TotalStockoutQty"] = stock
        rows["AvgEndingInv"] = np.array([i / n if n > 0 else 0 for i, n in zip(inv, steps)], np.float64)
    elif family == _capi.INVSIM_NETINVMGMT:
        # benchmark_NetInvMgmtLostSalesEnv.py:291-296: DataFrame sums / mean of column means
        steps, dem, sales, stock = m[:, 1], m[:, 2], m[:, 3], m[:, 4]
        X = m[:, 5:]
        rows["AvgServiceLevel"] = np.array([s / max(1e-6, d) if d > 1e-6 else 1.0 for s, d in zip(sales, dem)])
        rows["TotalStockoutQty"] = stock
        rows["AvgEndingInv"] = np.array([np.sum(x / n) / x.shape[0] if n > 0 else np.nan
                                         for x, n in zip(X, steps)])
    return rows


def _gather_rows(met, n_episodes, world, rank, group):
    """All ranks' per-episode metric rows, in global episode order (one
    all_gather of a padded [ceil(n / world), M] block; RCCL for device tensors
    with the nccl backend, host tensors with gloo)."""
    import torch.distributed as dist
    from .distributed import shard_range
    nmax = -(-n_episodes // world)
    dev = met.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    pad = torch.zeros((nmax, met.shape[1]), dtype=torch.float64, device=dev)
    pad[:met.shape[0]] = met.to(dev)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([parts[r][:shard_range(n_episodes, r, world)[1]] for r in range(world)]).cpu()


def evaluate_agent(agent, env_cls, env_config=None, n_episodes=100, seed_offset=0, device=None, group=None):
    """Batched evaluate_agent: episode i = env i seeded seed_offset + i, one
    full episode under ``agent`` in one kernel launch.  Returns a dict of
    per-episode columns (the reference's summary DataFrame columns).

    Under torch.distributed (one process per GPU) the episodes are sharded by
    global index over the ranks of ``group`` (rank r runs episodes
    [offset_r, offset_r + n_r), seeded by global index as above) and every
    rank gets all episodes' columns, gathered in one collective; Time is the
    slowest rank's time per episode."""
    import torch.distributed as dist
    from .distributed import shard_range
    on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if on else 1
    rank = dist.get_rank(group) if on else 0
    off, n_loc = shard_range(n_episodes, rank, world)
    env = env_cls(num_envs=max(n_loc, 1), device=device, autoreset_mode="disabled", global_offset=off,
                  **(env_config or {}))
    try:
        env.reset(seed=seed_offset)
        M = metrics_dim(env)
        met = torch.zeros((env.num_envs, M), dtype=torch.float64, device=env.device)
        torch.cuda.synchronize(env.device)
        t0 = time.perf_counter()
        rollout_policy(env, agent, env._horizon(), obs=False, rewards=False, metrics=met)
        torch.cuda.synchronize(env.device)
        dt = time.perf_counter() - t0
        met = met[:n_loc]
        family = env.family
        env_dev = env.device
    finally:
        env.close()
    if on:      # a 1-rank group too: the same collectives an N-GPU job runs
        met = _gather_rows(met, n_episodes, world, rank, group)
        # both collectives on the env's device (RCCL), or on the host (gloo)
        dev = env_dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dt = float(t.item())
    cols = summarize(family, met.cpu().numpy())
    n = n_episodes
    return {"Agent": [agent.name] * n, "Episode": np.arange(1, n + 1), **cols,
            "Time": np.full(n, dt / max(n, 1)), "Seed": seed_offset + np.arange(n), "Error": [None] * n}


def summary_table(results):
    """The reference's benchmark summary (process_and_report_results,
    benchmark_InvManagementBacklogEnv.py:474-516; the NetInvMgmt scripts'
    :333-353 are the same): per agent the mean / median / std / min / max
    episode reward, mean service level, stockout and ending inventory, time per
    episode, and episode counts, sorted by AvgReward.  ``results``: a list of
    evaluate_agent outputs.  Returns a pandas DataFrame indexed by Agent."""
    import pandas as pd
    raw = pd.concat([pd.DataFrame(r) for r in results], ignore_index=True)
    for c in ("AvgServiceLevel", "TotalStockoutQty", "AvgEndingInv"):
        if c not in raw:
            raw[c] = np.nan
    summary = raw.dropna(subset=["TotalReward"]).groupby("Agent").agg(
        AvgReward=("TotalReward", "mean"), MedianReward=("TotalReward", "median"),
        StdReward=("TotalReward", "std"), MinReward=("TotalReward", "min"), MaxReward=("TotalReward", "max"),
        AvgServiceLevel=("AvgServiceLevel", "mean"), AvgStockoutQty=("TotalStockoutQty", "mean"),
        AvgEndInv=("AvgEndingInv", "mean"), AvgTimePerEp=("Time", "mean"),
        SuccessfulEpisodes=("Episode", "count"))
    summary["TrainingTime(s)"] = 0.0                    # heuristic agents do not train
    summary["EpisodesAttempted"] = raw.groupby("Agent")["Episode"].count()
    summary["SuccessRate(%)"] = (summary["SuccessfulEpisodes"] / summary["EpisodesAttempted"]) * 100
    summary = summary.sort_values(by="AvgReward", ascending=False)
    return summary[["AvgReward", "MedianReward", "StdReward", "MinReward", "MaxReward", "AvgServiceLevel",
                    "AvgStockoutQty", "AvgEndInv", "AvgTimePerEp", "TrainingTime(s)", "SuccessfulEpisodes",
                    "EpisodesAttempted", "SuccessRate(%)"]]
