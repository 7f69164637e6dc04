"""NewsvendorEnv — vectorised, MI355X-native drop-in for the reference's
``newsvendor.NewsvendorEnv`` (newsvendor.py:13-230).

Same constructor arguments and spaces as the reference; ``num_envs`` instances
step together in one HIP kernel.  Observation ``[p, c, h, k, mu, x_L..x_1]``
f32, action f32[1] (order quantity), reward f64 with the reference's NumPy-2
f32/f64 promotion reproduced bit for bit.
"""
import numpy as np
import torch

from . import _capi
from .spaces import Box
from .vector import InvSimVectorEnv


class NewsvendorEnv(InvSimVectorEnv):
    family = _capi.INVSIM_NEWSVENDOR
    obs_dtype = torch.float32
    act_dtype = torch.float32

    def __init__(self, num_envs=1, device=None, lead_time=5, max_inventory=4000,
                 max_order_quantity=2000, step_limit=40, p_max=100.0, h_max=5.0, k_max=10.0,
                 mu_max=200.0, gamma=1.0, **vector_kwargs):
        # newsvendor.py:65-88
        self.lead_time = max(0, int(lead_time))
        self.max_inventory = max_inventory
        self.max_order_quantity = max_order_quantity
        self.step_limit = int(step_limit)
        self.p_max, self.h_max, self.k_max, self.mu_max = p_max, h_max, k_max, mu_max
        self.gamma = gamma
        self.obs_dim_ref = self.lead_time + 5
        high = np.array([p_max, p_max, h_max, k_max, mu_max] + [max_order_quantity] * self.lead_time,
                        dtype=np.float32)
        self.single_observation_space = Box(low=np.zeros(self.obs_dim_ref, np.float32), high=high,
                                            dtype=np.float32)
        self.single_action_space = Box(low=np.array([0], np.float32),
                                       high=np.array([max_order_quantity], np.float32),
                                       dtype=np.float32)
        super().__init__(num_envs, device=device, **vector_kwargs)

    def _create(self):
        self._spec = _capi.NewsvendorSpec(int(self.lead_time), int(self.step_limit),
                                          float(self.max_inventory), float(self.max_order_quantity),
                                          float(self.p_max), float(self.h_max), float(self.k_max),
                                          float(self.mu_max), float(self.gamma))
        self._create_handle(self._lib.invsim_create_newsvendor, self._spec)

    def _horizon(self):
        return self.step_limit

    def params(self):
        """Per-env (price, cost, h, k, mu) as f64 [N, 5] (the reference's info fields)."""
        return self.state_fields()["params"].view(torch.float64).t().contiguous()
