"""Stable-Baselines3 / RLlib adapters (SURVEY §8(b) callers, §8(f) row 4).

* :class:`InvSimVecEnv` — the SB3 ``VecEnv`` protocol over one invsim batch,
  replacing ``make_vec_env(EnvClass, n_envs)`` / ``DummyVecEnv([...])`` in the
  reference's ``benchmark_*_sb3_rllib.py`` scripts: numpy observations
  [n_envs, obs_dim], float32 rewards, ``dones`` = terminated | truncated, and
  SB3's immediate autoreset (the batch runs with SAME_STEP autoreset, the
  terminal observation in ``infos[i]["terminal_observation"]`` and
  ``infos[i]["TimeLimit.truncated"]``).  When stable_baselines3 is importable
  the class is a real ``VecEnv`` subclass; otherwise it duck-types the same
  methods (SB3 is not installed in this image).
* :func:`rllib_env_creator` — ``env_creator(env_config)`` for
  ``ray.tune.registry.register_env``: a single-env view (invsim.compat) with the
  reference's API; ``env_config`` holds the reference constructor kwargs plus
  an optional ``"env_class"`` name.

Env i of a batch seeded with ``seed`` uses ``seed + i`` (gymnasium SyncVectorEnv
and SB3's ``VecEnv.seed`` rule).
"""
import numpy as np
import torch

try:  # pragma: no cover - SB3 is absent in this image
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _SB3VecEnv
except Exception:  # noqa: BLE001
    _SB3VecEnv = object


class InvSimVecEnv(_SB3VecEnv):
    def __init__(self, env_cls, n_envs, env_config=None, device=None, seed=None):
        self.venv = env_cls(num_envs=n_envs, device=device, autoreset_mode="same_step", **(env_config or {}))
        if _SB3VecEnv is not object:   # SB3 2.x: sets reset_infos, _seeds, _options, render_mode
            super().__init__(n_envs, self.venv.single_observation_space, self.venv.single_action_space)
        self.num_envs = n_envs
        self.observation_space = self.venv.single_observation_space
        self.action_space = self.venv.single_action_space
        self.render_mode = None
        # SB3 2.x VecEnv state (also kept when SB3 is absent, so callers that
        # read them behave the same): per-env reset infos, pending seeds/options
        self.reset_infos = [{} for _ in range(n_envs)]
        self._seeds = [None for _ in range(n_envs)]
        self._options = [{} for _ in range(n_envs)]
        self._seed = seed
        self._actions = None
        self._obs = None

    # -- VecEnv protocol ------------------------------------------------------
    def reset(self):
        obs, info = self.venv.reset(seed=self._seed)
        self._seed = None
        self._seeds = [None for _ in range(self.num_envs)]
        self._options = [{} for _ in range(self.num_envs)]
        # SB3 2.x: one info dict per env, holding that env's own entries
        self.reset_infos = [{k: (v[i].cpu().numpy() if torch.is_tensor(v) else v) for k, v in info.items()}
                            for i in range(self.num_envs)]
        self._obs = obs
        return obs.cpu().numpy()

    def set_options(self, options=None):
        """SB3 2.x: options for the next reset (one dict, or one per env).  The
        reference envs ignore reset options, so they are only recorded."""
        if options is None:
            options = {}
        if isinstance(options, dict):
            options = [dict(options) for _ in range(self.num_envs)]
        self._options = list(options)

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        a = torch.as_tensor(np.asarray(self._actions), device=self.venv.device)
        obs, rew, te, tr, info = self.venv.step(a)
        dones = (te | tr).cpu().numpy()
        obs_np = obs.cpu().numpy()
        infos = [{} for _ in range(self.num_envs)]
        idx = np.nonzero(dones)[0]
        if len(idx):
            fobs = info["final_obs"].cpu().numpy()
            te_np, tr_np = te.cpu().numpy(), tr.cpu().numpy()
            for i in idx:
                infos[i]["terminal_observation"] = fobs[i]
                infos[i]["TimeLimit.truncated"] = bool(tr_np[i] and not te_np[i])
        return obs_np, rew.cpu().numpy().astype(np.float32), dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def seed(self, seed=None):
        self._seed = seed
        self._seeds = [None if seed is None else seed + i for i in range(self.num_envs)]
        return list(self._seeds)

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def get_attr(self, attr_name, indices=None):
        return [getattr(self.venv, attr_name) for _ in self._indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        raise NotImplementedError("invsim envs share one parameter set per batch; rebuild the VecEnv instead")

    def env_method(self, method_name, *args, indices=None, **kwargs):
        raise NotImplementedError("per-env methods are not available on a batched invsim env")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def get_images(self):
        return [None] * self.num_envs

    def render(self, mode=None):
        return None


def rllib_env_creator(env_config):
    """register_env("invsim", rllib_env_creator); env_config = reference kwargs
    plus "env_class" (default "InvManagementBacklogEnv")."""
    from .compat import make
    cfg = dict(env_config or {})
    cls = cfg.pop("env_class", "InvManagementBacklogEnv")
    return make(cls, **cfg)
