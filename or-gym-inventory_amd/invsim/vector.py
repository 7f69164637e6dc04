"""Gymnasium-style VectorEnv base over libinvsim (one handle = N envs on one GPU).

Mirrors ``gymnasium.vector.VectorEnv``: ``num_envs``, ``single_observation_space``,
``single_action_space``, ``observation_space``, ``action_space``,
``reset(seed=, options=)`` and ``step(actions)``, with torch tensors on the GPU
in and out.  Seeding follows ``gymnasium.vector.SyncVectorEnv`` /
SB3 ``DummyVecEnv``: ``reset(seed=s)`` seeds env i with ``s + i``
(``benchmark_InvManagementBacklogEnv.py:264``); a list seeds env i with
``seed[i]``; ``None`` draws fresh OS entropy the first time and afterwards
continues the streams (gymnasium ``Env.reset(seed=None)``).

Autoreset modes (``gymnasium.vector.AutoresetMode``):

* ``"next_step"`` (default, gymnasium >= 1.0): the step after an env is done
  resets it, ignoring its action, and returns the reset obs with reward 0.
* ``"same_step"`` (SB3 VecEnv): the done step returns the reset obs, the
  terminal obs is in ``info["final_obs"]`` (mask ``info["_final_obs"]``).
* ``"disabled"``: the caller resets; stepping an InvMgmt/NetInvMgmt env past
  its horizon raises IndexError as the reference does
  (``inventory_management.py:267``).

Demand stream (``demand_stream=``): ``"numpy"`` (default) draws from numpy's
PCG64 Generator stream, bit-exact with the reference on the same seeds;
``"philox"`` is the opt-in, non-parity fast stream (rocRAND Philox4x32-10,
counter-based: no per-env generator state per step; ``include/invsim.h``).
"""
import os

import numpy as np
import torch

from . import _capi
from .spaces import batch_box


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _to_device_index(device):
    if device is None:
        return torch.cuda.current_device()
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"invsim runs on a ROCm GPU (torch 'cuda' device), got {d}")
    return d.index if d.index is not None else torch.cuda.current_device()


def _seed_words(seeds):
    seeds = [int(s) for s in seeds]
    words = np.zeros((len(seeds), 4), np.uint32)
    nw = np.zeros(len(seeds), np.int32)
    for i, s in enumerate(seeds):
        if s < 0 or s >= 2**128:
            raise ValueError("seeds must be integers in [0, 2**128)")
        k = 0
        while True:
            words[i, k] = s & 0xFFFFFFFF
            k += 1
            s >>= 32
            if s == 0:
                break
        nw[i] = k
    return words, nw


class InvSimVectorEnv:
    """Base class; subclasses build the spec and the single-env spaces."""

    family = None
    metadata = {"autoreset_mode": "next_step"}
    obs_dtype = torch.float32
    act_dtype = torch.float32

    def __init__(self, num_envs, device=None, autoreset_mode="next_step", global_offset=0,
                 record_demand=False, record_info=False, copy=True, demand_stream="numpy"):
        if not torch.cuda.is_available():
            raise RuntimeError("invsim requires a ROCm GPU (torch.cuda.is_available() is False); "
                               "there is no CPU fallback")
        if autoreset_mode not in _capi.AUTORESET_MODES:
            raise ValueError(f"autoreset_mode must be one of {sorted(_capi.AUTORESET_MODES)}")
        self.num_envs = int(num_envs)
        self.global_offset = int(global_offset)
        self.device_index = _to_device_index(device)
        self.device = torch.device("cuda", self.device_index)
        self.autoreset_mode = autoreset_mode
        self.copy = bool(copy)
        self._lib = _capi.lib()
        self._h = None
        self._create()
        od, ad, dd, fam = (_capi.C.c_int32() for _ in range(4))
        _capi.check(self._lib.invsim_dims(self._h, _capi.C.byref(od), _capi.C.byref(ad),
                                          _capi.C.byref(dd), _capi.C.byref(fam)), self._h, "dims")
        self.obs_dim, self.action_dim, self.demand_dim = od.value, ad.value, dd.value
        self.observation_space = batch_box(self.single_observation_space, self.num_envs)
        self.action_space = batch_box(self.single_action_space, self.num_envs)
        self.set_demand_stream(demand_stream)
        self._seeded = False
        self._demand = None
        if record_demand:
            self._demand = torch.zeros((self.num_envs, self.demand_dim), dtype=torch.int64,
                                       device=self.device)
            _capi.check(self._lib.invsim_set_info_demand(self._h, self._demand.data_ptr()),
                        self._h, "set_info_demand")
        self._rec = None
        if record_info:
            d = _capi.C.c_int32()
            _capi.check(self._lib.invsim_info_record_dim(self._h, _capi.C.byref(d)), self._h, "info_record_dim")
            if d.value == 0:
                raise ValueError("record_info: this env family keeps no step record")
            rdt = torch.int64 if self.family == _capi.INVSIM_INVMGMT else torch.float64
            self._rec = torch.zeros((self.num_envs, d.value), dtype=rdt, device=self.device)
            _capi.check(self._lib.invsim_set_info_record(self._h, self._rec.data_ptr()), self._h, "set_info_record")
        self._out = None

    def _record_info(self, info):
        """Decode the per-step record into the reference's step-info names."""
        rec = self._rec.clone()
        if self.family == _capi.INVSIM_INVMGMT:
            m = (rec.shape[1] - 5) // 2
            info["sales"] = rec[:, :m]
            info["unfulfilled"] = rec[:, m:2 * m]
            f = rec[:, 2 * m:].view(torch.float64)
            for i, k in enumerate(("period_profit", "revenue", "procurement_cost", "holding_cost", "penalty_cost")):
                info[k] = f[:, i]
        elif self.family == _capi.INVSIM_NEWSVENDOR:
            # newsvendor.py:195-199; kinds: 0 Python float, 1 np.float32, 2 np.float64, 3 Python int
            kinds = rec[:, 4].to(torch.int64)
            for i, k in enumerate(("revenue", "purchase_cost", "holding_cost", "lost_sales_penalty")):
                info[k] = rec[:, i]
                info[k + "_kind"] = (kinds // (4 ** i)) % 4
        else:
            RL, J, E = len(self.retail_links), len(self.main_nodes), len(self.reorder_links)
            o = 0
            for k, w in (("sales", RL), ("unfulfilled", RL), ("inventory", J), ("replenishment", E),
                         ("pipeline", E), ("profit", J)):
                info[k] = rec[:, o:o + w]   # S[t], U[t+1] (retail links); X[t+1]; R[t], Y[t+1]; P[t]
                o += w
        return info

    # -- subclass hooks ------------------------------------------------------
    def _create(self):
        raise NotImplementedError

    def _horizon(self):
        raise NotImplementedError

    def _create_handle(self, fn, spec):
        h = _capi.C.c_void_p()
        rc = fn(_capi.C.byref(spec), self.num_envs, self.device_index,
                _capi.AUTORESET_MODES[self.autoreset_mode], _capi.C.byref(h))
        if rc != 0:
            raise _capi.InvsimError(f"invsim create failed ({rc}): {_capi.last_error(None)}")
        self._h = h

    # -- helpers --------------------------------------------------------------
    def _stream(self):
        # the raw hipStream_t of torch's current stream on this device (the
        # public torch.cuda.current_stream(dev).cuda_stream costs ~3 us a call)
        if _raw_stream is not None:
            return _raw_stream(self.device_index)
        return torch.cuda.current_stream(self.device).cuda_stream

    def _mask_ptr(self, mask):
        if mask is None:
            return None, None
        m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        if m.shape != (self.num_envs,):
            raise ValueError(f"reset_mask must have shape ({self.num_envs},)")
        return m, m.data_ptr()

    def _alloc(self, *shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    def _outputs(self):
        N, O = self.num_envs, self.obs_dim
        if self.copy or self._out is None:
            self._out = (self._alloc(N, O, dtype=self.obs_dtype),
                         self._alloc(N, dtype=torch.float64),
                         self._alloc(N, dtype=torch.bool),
                         self._alloc(N, dtype=torch.bool))
        return self._out

    def _actions(self, actions, lead_shape):
        a = actions
        if (type(a) is torch.Tensor and a.dtype == self.act_dtype and a.device == self.device
                and a.is_contiguous() and a.shape == tuple(lead_shape) + (self.action_dim,)):
            return a                                         # already in the kernel's layout
        a = torch.as_tensor(actions)
        shape = tuple(lead_shape) + (self.action_dim,)
        if a.shape != shape:
            if a.numel() == int(np.prod(shape)):
                a = a.reshape(shape)
            else:
                raise ValueError(f"actions must have shape {shape}, got {tuple(a.shape)}")
        return self._convert_actions(a.to(self.device)).contiguous()

    def _convert_actions(self, a):
        return a.to(self.act_dtype)

    # -- public API ------------------------------------------------------------
    def seed(self, seed=None):
        """Re-seed the env RNGs without resetting (gymnasium seeding.np_random)."""
        s = self._stream()
        if seed is None:
            ent = np.frombuffer(os.urandom(16 * self.num_envs), dtype=np.uint32).reshape(-1, 4)
            words = torch.from_numpy(ent.copy()).to(self.device)
            nw = torch.full((self.num_envs,), 4, dtype=torch.int32, device=self.device)
            _capi.check(self._lib.invsim_seed_words(self._h, words.data_ptr(), nw.data_ptr(), None, s),
                        self._h, "seed_words")
        elif isinstance(seed, (int, np.integer)):
            seed = int(seed)
            if seed < 0 or seed >= 2**128:
                raise ValueError("seed must be in [0, 2**128)")
            _capi.check(self._lib.invsim_seed_range(self._h, seed & (2**64 - 1), seed >> 64,
                                                    self.global_offset, None, s),
                        self._h, "seed_range")
        else:
            seeds = list(seed)
            if len(seeds) != self.num_envs:
                raise ValueError(f"expected {self.num_envs} seeds, got {len(seeds)}")
            w, nw = _seed_words(seeds)
            words = torch.from_numpy(w).to(self.device)
            nwt = torch.from_numpy(nw).to(self.device)
            _capi.check(self._lib.invsim_seed_words(self._h, words.data_ptr(), nwt.data_ptr(), None, s),
                        self._h, "seed_words")
        self._seeded = True

    def reset(self, *, seed=None, options=None):
        mask = (options or {}).get("reset_mask")
        if seed is not None or not self._seeded:
            if mask is not None and seed is not None:
                raise ValueError("seed together with reset_mask is not supported; seed first")
            self.seed(seed)
        m, mp = self._mask_ptr(mask)
        obs = self._alloc(self.num_envs, self.obs_dim, dtype=self.obs_dtype)
        _capi.check(self._lib.invsim_reset(self._h, mp, obs.data_ptr(), self._stream()), self._h, "reset")
        # with a reset_mask, rows of envs that were not reset are left unwritten in `obs`
        return obs, {}

    def step(self, actions):
        a = self._actions(actions, (self.num_envs,))
        obs, rew, term, trunc = self._outputs()
        fobs = None
        if self.autoreset_mode == "same_step":
            fobs = self._alloc(self.num_envs, self.obs_dim, dtype=self.obs_dtype)
        _capi.check(self._lib.invsim_step(self._h, a.data_ptr(), obs.data_ptr(), rew.data_ptr(),
                                          term.data_ptr(), trunc.data_ptr(),
                                          fobs.data_ptr() if fobs is not None else None,
                                          self._stream()), self._h, "step")
        info = {}
        if fobs is not None:
            info["final_obs"] = fobs
            info["_final_obs"] = trunc
        if self._demand is not None:
            info["demand"] = self._demand.clone() if self.demand_dim > 1 else self._demand[:, 0].clone()
        if self._rec is not None:
            self._record_info(info)
        return obs, rew, term, trunc, info

    def rollout(self, actions):
        """K consecutive steps in ONE kernel launch.  actions [K, N, A] ->
        obs [K, N, O], reward [K, N], terminated [K, N], truncated [K, N].
        Identical to K step() calls (next_step / disabled autoreset)."""
        a = torch.as_tensor(actions)
        K = int(a.shape[0])
        a = self._actions(a, (K, self.num_envs))
        N, O = self.num_envs, self.obs_dim
        obs = self._alloc(K, N, O, dtype=self.obs_dtype)
        rew = self._alloc(K, N, dtype=torch.float64)
        term = self._alloc(K, N, dtype=torch.bool)
        trunc = self._alloc(K, N, dtype=torch.bool)
        _capi.check(self._lib.invsim_rollout(self._h, K, a.data_ptr(), obs.data_ptr(), rew.data_ptr(),
                                             term.data_ptr(), trunc.data_ptr(), self._stream()),
                    self._h, "rollout")
        return obs, rew, term, trunc

    def rollout_policy(self, agent, K, obs=False, rewards=True, actions=False, metrics=None):
        """K steps with the agent's actions computed in the kernel (see
        invsim.policies); outputs optional, metrics [N, M] accumulated."""
        from .policies import rollout_policy
        return rollout_policy(self, agent, K, obs=obs, rewards=rewards, actions=actions, metrics=metrics)

    def status(self, clear=True):
        """Sticky device status word (synchronous): bit 0 = an env was stepped past its
        horizon with autoreset disabled after a masked reset (the step was not applied).
        step()/rollout() already check it in that mode and raise IndexError."""
        f = _capi.C.c_uint32()
        _capi.check(self._lib.invsim_status(self._h, _capi.C.byref(f), int(clear)), self._h, "status")
        return f.value

    def set_demand_stream(self, mode):
        """"numpy" (parity, default) or "philox" (fast, NOT the reference's draws)."""
        if mode not in _capi.DEMAND_STREAMS:
            raise ValueError(f"demand_stream must be one of {sorted(_capi.DEMAND_STREAMS)}")
        _capi.check(self._lib.invsim_set_demand_stream(self._h, _capi.DEMAND_STREAMS[mode]), self._h,
                    "set_demand_stream")

    @property
    def demand_stream(self):
        """The stream the handle draws demands from ("numpy" or "philox")."""
        m = _capi.C.c_int32()
        _capi.check(self._lib.invsim_demand_stream(self._h, _capi.C.byref(m)), self._h, "demand_stream")
        return {v: k for k, v in _capi.DEMAND_STREAMS.items()}[m.value]

    @property
    def kernel_variant(self):
        """0 = generic kernel; 1 / 2 = NetInvMgmt kernel specialised for the
        reference's default / custom supply network."""
        v = _capi.C.c_int32()
        _capi.check(self._lib.invsim_kernel_variant(self._h, _capi.C.byref(v)), self._h, "kernel_variant")
        return v.value

    def position(self):
        """Opaque token of the host-side position (lock-step period, lookahead
        slot) that picks each launch's kernel; see invsim.graphs."""
        p = _capi.C.c_int64()
        _capi.check(self._lib.invsim_position(self._h, _capi.C.byref(p)), self._h, "position")
        return p.value

    def capture(self, fn, warmup=1, pool=None):
        """Record fn() (a policy's torch ops + calls on this env) as one HIP
        graph: returns an invsim.graphs.StepGraph whose replay() reruns it."""
        from .graphs import StepGraph
        return StepGraph(self, fn, warmup=warmup, pool=pool)

    # -- state -----------------------------------------------------------------
    def state_bytes(self):
        b = _capi.C.c_int64()
        _capi.check(self._lib.invsim_state_bytes(self._h, _capi.C.byref(b)), self._h, "state_bytes")
        return b.value

    def get_state(self):
        """Checkpoint: the whole device state (RNG streams included) as a uint8 tensor."""
        buf = torch.empty(self.state_bytes(), dtype=torch.uint8, device=self.device)
        _capi.check(self._lib.invsim_get_state(self._h, buf.data_ptr(), self._stream()), self._h, "get_state")
        return buf

    def set_state(self, buf):
        buf = torch.as_tensor(buf, device=self.device).contiguous()
        if buf.dtype != torch.uint8 or buf.numel() != self.state_bytes():
            raise ValueError("state blob does not match this env's layout")
        _capi.check(self._lib.invsim_set_state(self._h, buf.data_ptr(), self._stream()), self._h, "set_state")
        self._seeded = True

    def state_fields(self, blob=None):
        """Decode a state blob into {name: tensor[rows, N]} views (debug / tests)."""
        blob = self.get_state() if blob is None else blob
        out = {}
        i = 0
        dt = {1: torch.uint8, 4: torch.int32, 8: torch.int64}
        while True:
            name = _capi.C.create_string_buffer(32)
            off, eb, rows, stride = _capi.C.c_int64(), _capi.C.c_int32(), _capi.C.c_int32(), _capi.C.c_int64()
            rc = self._lib.invsim_state_field(self._h, i, name, _capi.C.byref(off), _capi.C.byref(eb),
                                              _capi.C.byref(rows), _capi.C.byref(stride))
            if rc != 0:
                break
            r_, st_ = rows.value, stride.value
            if st_ > 0:     # [rows][stride]
                raw = blob[off.value: off.value + r_ * st_ * eb.value].view(dt[eb.value]).view(r_, st_)
                out[name.value.decode()] = raw[:, : self.num_envs] if st_ > 1 else raw
            elif st_ < 0:   # record layout [Npad][rows] -> [rows, N] view
                raw = blob[off.value: off.value + r_ * -st_ * eb.value].view(dt[eb.value]).view(-st_, r_)
                out[name.value.decode()] = raw[: self.num_envs].t()
            i += 1
        return out

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self._lib.invsim_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __repr__(self):
        return f"{type(self).__name__}(num_envs={self.num_envs}, device={self.device})"
