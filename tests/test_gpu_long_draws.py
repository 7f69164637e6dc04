"""Sampler parity at the survey's bar (SURVEY.md hard part 1: >= 1e8 draws per
sampler path): each case runs >= 1e8 demand draws through one kernel path of
the HIP engine and through the C oracle on the same seeds and actions, and
compares

* every env's final PCG64 state (state and increment, all streams): any PTRS
  accept/reject decision taken differently changes how many uniforms a draw
  consumes, and a multiplication-method draw consumes value + 1 uniforms;
* every env's sum of rewards over the whole run, added in step order on both
  sides (device: the HIP episode fold with no done flags; host: numpy), bit
  for bit: each step's reward depends on that step's demand.

Paths: the InvMgmt step lookahead (compacted second round) and the flat-loop
rollouts (2-role at 65 536 envs, 3-role at 32 768), for the PTRS table path
(mu = 20) and the multiplication method (mu = 8); Newsvendor's per-episode
rate on both branches (mu_max = 200: ~95 % PTRS; mu_max = 10: multiplication
only), step and rollout; NetInvMgmt's market draws, step lookahead and
3-role rollout, default and custom (3 markets) graphs.  NEXT_STEP autoreset
throughout, so resets (and Newsvendor's 5 reset uniforms) are in the streams.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

MIN_DRAWS = 100_000_000


def _threads():
    try:
        c = len(os.sched_getaffinity(0))
    except AttributeError:
        c = os.cpu_count() or 1
    return max(1, min(16, c))


def _gpu_run(env, pool, T, mode):
    """T calls under NEXT_STEP autoreset, call k with pool[k % P]; returns the
    per-env reward sums (device fold, step order) and the truncation count."""
    from invsim import _capi
    from invsim.distributed import EpisodeStats
    dev = env.device
    N, O, P = env.num_envs, env.obs_dim, len(pool)
    st = EpisodeStats(N, dev)
    sp = torch._C._cuda_getCurrentRawStream(dev.index)
    lib, h = env._lib, env._h
    ntr = torch.zeros((), dtype=torch.int64, device=dev)
    if mode == "step":
        rew = torch.empty((P, N), dtype=torch.float64, device=dev)
        term = torch.empty((P, N), dtype=torch.bool, device=dev)
        trunc = torch.empty((P, N), dtype=torch.bool, device=dev)
        obs = torch.empty((N, O), dtype=env.obs_dtype, device=dev)
        rows = 0
        for k in range(T):
            r = k % P
            _capi.check(lib.invsim_step(h, pool[r].data_ptr(), obs.data_ptr(), rew[r].data_ptr(),
                                        term[r].data_ptr(), trunc[r].data_ptr(), None, sp), h, "step")
            rows += 1
            if r == P - 1 or k == T - 1:
                st.update_block(rew[:rows], None, None)
                ntr += trunc[:rows, 0].sum()
                rows = 0
    else:
        assert T % P == 0
        acts = torch.stack(pool).contiguous()            # one launch = P steps, call k uses pool[k % P]
        obs = torch.empty((P, N, O), dtype=env.obs_dtype, device=dev)
        rew = torch.empty((P, N), dtype=torch.float64, device=dev)
        term = torch.empty((P, N), dtype=torch.bool, device=dev)
        trunc = torch.empty((P, N), dtype=torch.bool, device=dev)
        for _ in range(T // P):
            _capi.check(lib.invsim_rollout(h, P, acts.data_ptr(), obs.data_ptr(), rew.data_ptr(),
                                           term.data_ptr(), trunc.data_ptr(), sp), h, "rollout")
            st.update_block(rew, None, None)
            ntr += trunc[:, 0].sum()
    return st.ret.cpu().numpy(), int(ntr)


def _compare(env, orc, pool_np, T, mode, seed):
    dev = env.device
    pool = [torch.from_numpy(a).to(dev) for a in pool_np]
    env.reset(seed=seed)
    orc.seed(range(seed, seed + env.num_envs))
    orc.reset()
    ret_gpu, ntr_gpu = _gpu_run(env, pool, T, mode)
    rng_gpu = env.state_fields()["rng"].cpu().numpy().view(np.uint64).T
    import pyoracle
    pyoracle.set_threads(_threads())
    try:
        ret_orc, ntr_orc = orc.run_returns(pool_np, T)
    finally:
        pyoracle.set_threads(1)
    rng_orc = orc.rng_state()
    assert ntr_gpu == ntr_orc
    bad = np.nonzero((rng_gpu != rng_orc).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} streams end in a different PCG64 state (first env {bad[:5]})"
    eq = ret_gpu.view(np.int64) == ret_orc.view(np.int64)
    assert eq.all(), f"{(~eq).sum()} envs' reward sums differ (first {np.nonzero(~eq)[0][:5]})"


def _pool_int(rng, P, N, A, hi):
    return [rng.integers(0, hi, size=(N, A)).astype(np.int64) for _ in range(P)]


def _pool_f32(rng, P, N, A, hi):
    return [rng.uniform(0, hi, size=(N, A)).astype(np.float32) for _ in range(P)]


# (class, envs, mode, mu): InvMgmt T = 31 c calls -> 30 c draws per env
@pytest.mark.parametrize("cls,n,mode,mu,cycles", [
    ("InvManagementBacklogEnv", 65536, "step", 20, 51),       # im_split_kernel lookahead, PTRS table
    ("InvManagementBacklogEnv", 65536, "rollout", 20, 51),    # im_roll3 flat loop
    ("InvManagementLostSalesEnv", 32768, "rollout", 20, 102),  # im_roll3o flat loop
    ("InvManagementBacklogEnv", 65536, "step", 8, 51),        # multiplication method, lookahead
    ("InvManagementLostSalesEnv", 32768, "rollout", 8, 102),   # multiplication method, flat loop
])
def test_invmgmt_1e8_draws_vs_oracle(gpu, oracle, cls, n, mode, mu, cycles):
    import invsim
    env = getattr(invsim, cls)(n, device=gpu, dist_param={"mu": mu})
    orc = oracle.OracleInvMgmt(n, backlog=cls.endswith("BacklogEnv"), dist_param={"mu": mu})
    assert n * 30 * cycles >= MIN_DRAWS
    pool = _pool_int(np.random.default_rng(mu + n), 31, n, 3, 120)
    _compare(env, orc, pool, 31 * cycles, mode, 1000 + mu)


# Newsvendor: step_limit 40 -> 41-call cycles (the reset call draws 5 uniforms)
@pytest.mark.parametrize("mode", ["step", "rollout"])
@pytest.mark.parametrize("mu_max", [200.0, 10.0])
def test_newsvendor_1e8_draws_vs_oracle(gpu, oracle, mode, mu_max):
    import invsim
    n, cycles = 65536, 39
    env = invsim.NewsvendorEnv(n, device=gpu, mu_max=mu_max)
    orc = oracle.OracleNewsvendor(n, mu_max=mu_max)
    assert n * 40 * cycles >= MIN_DRAWS
    pool = _pool_f32(np.random.default_rng(int(mu_max)), 41, n, 1, 2 * mu_max)
    pool = [p.reshape(n, 1) for p in pool]
    _compare(env, orc, pool, 41 * cycles, mode, 2000 + int(mu_max))


@pytest.mark.parametrize("graph,mode,cycles", [("default", "step", 102), ("default", "rollout", 102),
                                               ("custom", "rollout", 34)])
def test_net_1e8_draws_vs_oracle(gpu, oracle, graph, mode, cycles):
    import invsim
    from invsim.topology import custom_graph, default_graph
    n = 32768
    g = default_graph() if graph == "default" else custom_graph()
    env = invsim.NetInvMgmtBacklogEnv(n, device=gpu, graph=g)
    orc = oracle.OracleNet(n, graph=g)
    markets = orc.topo["RL"]
    assert n * 30 * cycles * markets >= MIN_DRAWS
    pool = _pool_f32(np.random.default_rng(cycles), 31, n, env.action_dim, 150.0)
    _compare(env, orc, pool, 31 * cycles, mode, 3000 + cycles)
