"""CPU checks of bench.py's launcher contract and of the episodic-return fold's
host arithmetic (the HIP fold is checked in tests/test_gpu_episode_fold.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_world_size_mismatch():
    """under a launcher whose WORLD_SIZE differs from --gpus, bench.py exits
    non-zero before touching a GPU (no silent single-rank timing)"""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "8"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=1" in p.stderr


def _numpy_fold(rew, done, ret0):
    ret = ret0.copy()
    s = s2 = c = 0.0
    for k in range(rew.shape[0]):
        ret += rew[k]
        d = done[k]
        s += ret[d].sum()
        s2 += (ret[d] ** 2).sum()
        c += d.sum()
        ret[d] = 0.0
    return ret, np.array([s, s2, c, rew.sum()])


def test_episode_stats_block_fold_host():
    from invsim.distributed import EpisodeStats
    rng = np.random.default_rng(5)
    K, N = 37, 513
    st = EpisodeStats(N, "cpu")
    ret0 = np.zeros(N)
    acc = np.zeros(4)
    for _ in range(3):
        rew = rng.normal(size=(K, N)) * 100
        term = rng.random((K, N)) < 0.03
        trunc = rng.random((K, N)) < 0.05
        st.update_block(torch.from_numpy(rew), torch.from_numpy(term), torch.from_numpy(trunc))
        ret0, a = _numpy_fold(rew, term | trunc, ret0)
        acc += a
    assert np.allclose(st.ret.numpy(), ret0, rtol=1e-12, atol=1e-9)
    assert np.allclose(st.acc.numpy(), acc, rtol=1e-12)
    res = st.allreduce()
    assert res["episodes"] == acc[2] and res["reward_sum"] == pytest.approx(acc[3])


def test_roofline_rocprof_reconciliation_fields(monkeypatch):
    """the line's frac is reproduced from the committed
    rocprof kernel stats: the dominant kernel's mean and the mean over every
    env-step launch (what the HIP-event figure averages).  Pinned to the
    round-5 files: a later round's profiles do not move it."""
    import bench
    monkeypatch.setattr(bench, "PROFILE_ROUND", "r05")
    alg = 746 * 65536
    r = bench._rocprof("invmgmt_backlog", "step", True, alg)
    assert r is not None and r["source"] == "profiles/r05/invmgmt_backlog_step_kernel_stats.csv"
    assert r["dominant_kernel"] == "im_split_kernel"
    assert 0.9 < r["dominant_share_of_launches"] < 1.0          # the reset launch every 31 steps
    assert r["all_step_launches_ns"] < r["dominant_ns"]            # the reset launch is cheaper
    assert abs(r["frac_dominant"] - alg / r["dominant_ns"] / 8000.0) < 1e-12
    assert bench._rocprof("invmgmt_backlog", "step", False, alg) is None   # another batch size: no file applies
    i = bench._issue("newsvendor", "rollout", 0.06, True)
    assert i["bound"] == "issue" and 0 < i["frac"] < 1 and i["instructions_per_launch"] > 1e6
    assert bench._issue("newsvendor", "rollout", 0.06, False) is None     # not the SQ passes' batch
    assert bench._issue("invmgmt_backlog", "step", 0.009, True) is None


def test_hbm_counter_fraction(monkeypatch):
    """the physical HBM rate = counter bytes per launch /
    the dominant kernel's rocprof time; round 5's files give 4.53 TB/s (0.566)."""
    import bench
    monkeypatch.setattr(bench, "PROFILE_ROUND", "r05")
    traffic, src = bench._pmc("invmgmt_backlog", "step", True)
    rp = bench._rocprof("invmgmt_backlog", "step", True, 746 * 65536)
    hc = bench._hbm_counter(traffic, src, rp)
    assert hc["achieved"] == pytest.approx(41256485.86 / 9114.889764, rel=1e-6)
    assert hc["frac"] == pytest.approx(0.566, abs=1e-3)
    assert hc["frac_of_achievable"] == pytest.approx(hc["achieved"] / 6300.0)
    assert bench._hbm_counter(None, None, rp) is None and bench._hbm_counter(traffic, src, None) is None


def test_span_single_process():
    import bench

    class NoDist:
        @staticmethod
        def is_initialized():
            return False
    assert bench._span(1.0, 3.5, None, NoDist) == 2.5


def test_fold_mode_auto():
    """--fold auto: the in-kernel episode sink for InvMgmt rollouts (and policy
    rollouts), the block fold for single steps and for the other families
    (DESIGN §4 "Round 6: the episode sink")."""
    import types
    import bench
    from invsim import _capi

    def env(fam):
        return types.SimpleNamespace(family=fam)
    a = types.SimpleNamespace(fold="auto")
    assert bench.fold_mode(a, env(_capi.INVSIM_INVMGMT), "rollout") == "sink"
    assert bench.fold_mode(a, env(_capi.INVSIM_INVMGMT), "policy") == "sink"
    assert bench.fold_mode(a, env(_capi.INVSIM_INVMGMT), "step") == "inline"
    for fam in (_capi.INVSIM_NEWSVENDOR, _capi.INVSIM_NETINVMGMT):
        assert bench.fold_mode(a, env(fam), "rollout") == "inline"
    for f in ("sink", "side", "inline", "none"):
        assert bench.fold_mode(types.SimpleNamespace(fold=f), env(_capi.INVSIM_NEWSVENDOR), "step") == f


def test_episode_stats_host_partials():
    """host EpisodeStats: one partial row; acc is its column sum; reset_acc
    keeps the running returns"""
    from invsim.distributed import EpisodeStats
    st = EpisodeStats(5, "cpu")
    assert tuple(st.part.shape) == (1, 4)
    rew = torch.tensor([[1.0, 2.0, 3.0, 4.0, 5.0], [1.0, 1.0, 1.0, 1.0, 1.0]], dtype=torch.float64)
    done = torch.tensor([[False] * 5, [True, False, True, False, False]])
    st.update_block(rew, None, done)
    assert st.acc.tolist() == [2.0 + 4.0, 4.0 + 16.0, 2.0, 20.0]
    assert st.ret.tolist() == [0.0, 3.0, 0.0, 5.0, 6.0]
    st.reset_acc()
    assert st.acc.tolist() == [0.0] * 4 and st.ret.tolist() == [0.0, 3.0, 0.0, 5.0, 6.0]
