"""Multi-echelon inventory envs — vectorised, MI355X-native drop-ins for the
reference's ``inventory_management`` module (inventory_management.py:19-451).

``InvManagementMasterEnv`` / ``InvManagementBacklogEnv`` /
``InvManagementLostSalesEnv`` take the reference's constructor arguments
(``periods, I0, p, r, k, h, c, L, backlog, dist, dist_param, alpha, seed_int,
user_D, env_config``) plus the vector arguments (``num_envs, device,
autoreset_mode, global_offset, record_demand, copy``).  Observations and
actions are int64 like the reference's Box spaces; float actions are mapped
like ``np.maximum(action, 0).astype(np.int64)`` (:250).

The reference's dynamics are kept exactly, including its quirks: the supplier
stage is decremented by its OWN order (:300) so inventories may go negative,
and the observation window holds *requested* orders, left-aligned (:380-383).
"""
import numpy as np
import torch

from . import _capi
from .spaces import Box
from .vector import InvSimVectorEnv


class InvManagementMasterEnv(InvSimVectorEnv):
    family = _capi.INVSIM_INVMGMT
    obs_dtype = torch.int64
    act_dtype = torch.int64

    def __init__(self, num_envs=1, device=None, periods=30, I0=(100, 150, 200), p=20,
                 r=(15, 10, 7, 5), k=(0.10, 0.075, 0.05, 0.025), h=(0.15, 0.10, 0.05),
                 c=(100, 200, 230), L=(1, 5, 10), backlog=True, dist=1, dist_param=None,
                 alpha=0.97, seed_int=0, user_D=None, env_config=None, **vector_kwargs):
        # inventory_management.py:67-84 (+ env_config setattr overrides)
        self.periods, self.I0, self.p, self.r, self.k, self.h, self.c, self.L = \
            periods, I0, p, r, k, h, c, L
        self.backlog, self.dist = backlog, dist
        self.dist_param = dist_param if dist_param is not None else {"mu": 20}
        self.alpha, self.seed_int = alpha, seed_int
        self.user_D = user_D if user_D is not None else []
        for key, value in (env_config or {}).items():
            setattr(self, key, value)
        # :87-100 parameter processing
        self.init_inv = np.array(list(self.I0), dtype=np.int32)
        self.num_periods = int(self.periods)
        self.unit_price = np.append(self.p, self.r[:-1]).astype(np.float32)
        self.unit_cost = np.array(self.r, dtype=np.float32)
        self.demand_cost = np.array(self.k, dtype=np.float32)
        self.holding_cost = np.append(self.h, 0).astype(np.float32)
        self.supply_capacity = np.array(list(self.c), dtype=np.int64)
        self.lead_time = np.array(list(self.L), dtype=np.int64)
        self.discount = self.alpha
        self.user_D = np.array(list(self.user_D), dtype=np.int64)
        self.num_stages = len(self.init_inv) + 1
        m = self.num_stages
        self.lt_max = 0 if m <= 1 else int(self.lead_time.max())
        self._validate_inputs()
        # :111-128 spaces
        self.single_action_space = Box(low=np.zeros(m - 1, dtype=np.int64),
                                       high=self.supply_capacity.astype(np.int64), shape=(m - 1,),
                                       dtype=np.int64)
        self.pipeline_length = (m - 1) * (self.lt_max + 1)
        cap = self.supply_capacity.sum() * self.num_periods * 2
        low = -np.ones(self.pipeline_length, np.int64) * cap if self.backlog else \
            np.zeros(self.pipeline_length, np.int64)
        self.single_observation_space = Box(low=low, high=np.ones(self.pipeline_length, np.int64) * cap,
                                            shape=(self.pipeline_length,), dtype=np.int64)
        super().__init__(num_envs, device=device, **vector_kwargs)

    def _validate_inputs(self):
        """inventory_management.py:144-167 (AssertionError like the reference)."""
        m = self.num_stages
        assert np.all(self.init_inv >= 0), "Initial inventory cannot be negative"
        assert self.num_periods > 0, "Number of periods must be positive"
        assert np.all(self.unit_price >= 0), "Sales prices cannot be negative"
        assert np.all(self.unit_cost >= 0), "Procurement costs cannot be negative"
        assert np.all(self.demand_cost >= 0), "Unfulfilled demand costs cannot be negative"
        assert np.all(self.holding_cost >= 0), "Holding costs cannot be negative"
        assert np.all(self.supply_capacity > 0), "Supply capacities must be positive"
        assert np.all(self.lead_time >= 0), "Lead times cannot be negative"
        assert isinstance(self.backlog, bool), "Backlog parameter must be boolean"
        assert m >= 2, "Minimum number of stages is 2"
        assert len(self.unit_cost) == m, f"Length of r ({len(self.unit_cost)}) != num stages ({m})"
        assert len(self.demand_cost) == m, f"Length of k ({len(self.demand_cost)}) != num stages ({m})"
        assert len(self.holding_cost) == m, f"Length of h ({len(self.holding_cost)}) != num stages ({m})"
        assert len(self.supply_capacity) == m - 1, f"Length of c ({len(self.supply_capacity)}) != num stages - 1 ({m-1})"
        assert len(self.lead_time) == m - 1, f"Length of L ({len(self.lead_time)}) != num stages - 1 ({m-1})"
        assert self.dist in [1, 2, 3, 4, 5], "dist must be one of 1, 2, 3, 4, 5"
        if self.dist == 5:
            assert len(self.user_D) == self.num_periods, "User specified demand length != num periods"
        assert 0 < self.alpha <= 1, "alpha must be in the range (0, 1]"

    def _create(self):
        m = self.num_stages
        self._keep = dict(
            I0=np.ascontiguousarray(self.init_inv.astype(np.int64)),
            up=np.ascontiguousarray(self.unit_price), uc=np.ascontiguousarray(self.unit_cost),
            kc=np.ascontiguousarray(self.demand_cost), hc=np.ascontiguousarray(self.holding_cost),
            c=np.ascontiguousarray(self.supply_capacity), L=np.ascontiguousarray(self.lead_time),
            uD=np.ascontiguousarray(self.user_D if self.dist == 5 else np.zeros(1, np.int64)))
        k = self._keep
        dp = self.dist_param
        mu = float(dp["mu"]) if self.dist == 1 else 0.0
        # dist_param keys the reference's samplers read (:173-182); a missing key
        # raises KeyError here rather than at the first step
        dn = int(dp["n"]) if self.dist == 2 else 0
        dpp = float(dp["p"]) if self.dist in (2, 4) else 0.0
        lo, hi = (int(dp["low"]), int(dp["high"])) if self.dist == 3 else (0, 0)
        self._spec = _capi.InvMgmtSpec(
            m, self.num_periods, int(self.backlog), int(self.dist), mu, float(self.alpha),
            k["I0"].ctypes.data, k["up"].ctypes.data, k["uc"].ctypes.data, k["kc"].ctypes.data,
            k["hc"].ctypes.data, k["c"].ctypes.data, k["L"].ctypes.data,
            k["uD"].ctypes.data if self.dist == 5 else None, dn, dpp, lo, hi)
        self._create_handle(self._lib.invsim_create_invmgmt, self._spec)

    def _horizon(self):
        return self.num_periods

    def _convert_actions(self, a):
        # np.maximum(action, 0).astype(np.int64): float actions truncate toward zero (:250)
        if a.dtype.is_floating_point:
            a = torch.clamp(a, min=0)
        return a.to(torch.int64)

    def sample_action(self):
        """Uniform integer actions in [0, c] for every env (reference :402-404, batched)."""
        hi = torch.as_tensor(self.supply_capacity, device=self.device)
        u = torch.rand((self.num_envs, self.num_stages - 1), device=self.device, dtype=torch.float64)
        return torch.floor(u * (hi + 1).to(torch.float64)).to(torch.int64)


class InvManagementBacklogEnv(InvManagementMasterEnv):
    """inventory_management.py:429-434: backlog forced on."""

    def __init__(self, *args, **kwargs):
        kwargs["backlog"] = True
        super().__init__(*args, **kwargs)


class InvManagementLostSalesEnv(InvManagementMasterEnv):
    """inventory_management.py:436-451: backlog forced off, obs low bound 0."""

    def __init__(self, *args, **kwargs):
        kwargs["backlog"] = False
        super().__init__(*args, **kwargs)
        cap = self.supply_capacity.sum() * self.num_periods * 2
        self.single_observation_space = Box(low=np.zeros(self.pipeline_length, np.int64),
                                            high=np.ones(self.pipeline_length, np.int64) * cap,
                                            shape=(self.pipeline_length,), dtype=np.int64)
        from .spaces import batch_box
        self.observation_space = batch_box(self.single_observation_space, self.num_envs)
