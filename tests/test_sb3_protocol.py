"""invsim.sb3.InvSimVecEnv against the SB3 2.x VecEnv base-class contract, on
CPU: stable_baselines3 is not installed here, so a stand-in base with SB3
2.x's constructor (num_envs, observation_space, action_space -> reset_infos,
_seeds, _options, render_mode via get_attr) is injected and the adapter
re-imported over a host-side fake batch.  Parity with real SB3 is unpinned
(SB3 absent); this pins that the adapter runs the base constructor and keeps
the attributes SB3 reads."""
import importlib
import sys
import types

import numpy as np


class _FakeSB3VecEnv:
    """Constructor of stable_baselines3 2.x common/vec_env/base_vec_env.VecEnv."""

    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space
        self.reset_infos = [{} for _ in range(num_envs)]
        self._seeds = [None for _ in range(num_envs)]
        self._options = [{} for _ in range(num_envs)]
        try:
            render_modes = self.get_attr("render_mode")
        except AttributeError:
            render_modes = [None for _ in range(num_envs)]
        self.render_mode = render_modes[0]
        self.base_init_ran = True


class _HostObs:
    def __init__(self, a):
        self.a = a

    def cpu(self):
        return self

    def numpy(self):
        return self.a


class _FakeBatch:
    """Host stand-in for an invsim VectorEnv (only what the adapter touches)."""

    def __init__(self, num_envs, device=None, autoreset_mode=None, **kw):
        assert autoreset_mode == "same_step"
        self.num_envs = num_envs
        self.device = "cpu"
        self.single_observation_space = "obs-space"
        self.single_action_space = "act-space"
        self.render_mode = None
        self.seen_seed = "unset"

    def reset(self, seed=None, options=None):
        self.seen_seed = seed
        return _HostObs(np.zeros((self.num_envs, 4), np.int64)), {"period": 0}

    def close(self):
        pass


def _reload_with(monkeypatch, base):
    mods = {}
    for name in ("stable_baselines3", "stable_baselines3.common", "stable_baselines3.common.vec_env",
                 "stable_baselines3.common.vec_env.base_vec_env"):
        mods[name] = types.ModuleType(name)
    mods["stable_baselines3.common.vec_env.base_vec_env"].VecEnv = base
    for name, mod in mods.items():
        monkeypatch.setitem(sys.modules, name, mod)
    import invsim.sb3 as sb3
    return importlib.reload(sb3)


def test_vecenv_runs_sb3_base_init(monkeypatch):
    sb3 = _reload_with(monkeypatch, _FakeSB3VecEnv)
    try:
        v = sb3.InvSimVecEnv(_FakeBatch, 5, seed=11)
        assert isinstance(v, _FakeSB3VecEnv) and v.base_init_ran
        assert v.num_envs == 5 and v.observation_space == "obs-space" and v.action_space == "act-space"
        assert v.reset_infos == [{}] * 5 and v._seeds == [None] * 5 and v._options == [{}] * 5
        v.set_options({"x": 1})
        assert v._options == [{"x": 1}] * 5
        assert v.seed(3) == [3, 4, 5, 6, 7] and v._seeds == [3, 4, 5, 6, 7]
        obs = v.reset()
        assert obs.shape == (5, 4) and v.venv.seen_seed == 3
        assert v.reset_infos == [{"period": 0}] * 5 and v._seeds == [None] * 5 and v._options == [{}] * 5
    finally:
        monkeypatch.undo()
        importlib.reload(sys.modules["invsim.sb3"])


def test_vecenv_without_sb3_keeps_same_attributes():
    import invsim.sb3 as sb3
    sb3 = importlib.reload(sb3)
    v = sb3.InvSimVecEnv(_FakeBatch, 3)
    assert v.reset_infos == [{}] * 3 and v._seeds == [None] * 3 and v._options == [{}] * 3
    v.reset()
    assert v.reset_infos == [{"period": 0}] * 3
