"""Supply-network inventory envs — vectorised, MI355X-native drop-ins for the
reference's ``network_management`` module (network_management.py:26-770) and
its custom-topology variant (network_management_custom.py).

``NetInvMgmtMasterEnv`` / ``NetInvMgmtBacklogEnv`` / ``NetInvMgmtLostSalesEnv``
take ``graph, num_periods, backlog, alpha, seed_int, user_D, sample_path,
env_config`` plus the vector arguments.  ``graph=None`` is the reference's
default 9-node network; ``topology.custom_graph()`` is the custom one.
Actions are f32 per reorder link (rounded half-to-even, :449), observations
f32 ``[U[t] (retail links), X[t] (main nodes), fulfilled-order windows]``.

Reference behaviour kept on purpose: ``NetInvMgmtLostSalesEnv`` runs with
``backlog=True`` unless ``backlog=False`` is passed explicitly, because the
reference's ``__init__`` overwrites the subclass's env_config flag with the
``backlog`` argument (network_management.py:83-85 vs :755-761).
"""
import numpy as np
import torch

from . import _capi
from .spaces import Box, batch_box
from .topology import check_market_receivers, classify, compile_graph, default_graph, validate_inputs
from .vector import InvSimVectorEnv


class NetInvMgmtMasterEnv(InvSimVectorEnv):
    family = _capi.INVSIM_NETINVMGMT
    obs_dtype = torch.float32
    act_dtype = torch.float32

    def __init__(self, num_envs=1, device=None, graph=None, num_periods=30, backlog=True,
                 alpha=1.00, seed_int=0, user_D=None, sample_path=None, env_config=None,
                 **vector_kwargs):
        # network_management.py:67-85
        self.num_periods, self.backlog, self.alpha, self.seed_int = num_periods, backlog, alpha, seed_int
        self.user_D = dict(user_D) if user_D is not None else {}
        self.sample_path = dict(sample_path) if sample_path is not None else {}
        self.graph = graph.copy() if graph is not None else default_graph()
        if graph is None:                                 # :140-144 (the default graph only)
            self.user_D.setdefault((1, 0), np.zeros(self.num_periods))
            self.sample_path.setdefault((1, 0), False)
        cfg = dict(env_config) if env_config else {}
        cfg["backlog"] = self.backlog            # :84 — the argument wins over env_config
        for key, value in cfg.items():
            if key == "graph":
                self.graph = value.copy()
            else:
                setattr(self, key, value)
        # :149-163 -- market links carry their demand source on the graph
        for link, d in self.user_D.items():
            if link in self.graph.edges:
                self.graph.edges[link]["user_D"] = list(d) if not isinstance(d, (list, np.ndarray)) else d
                self.graph.edges[link]["sample_path"] = self.sample_path.get(link, False)
        for link in classify(self.graph)[7]:
            self.graph.edges[link].setdefault("user_D", np.zeros(self.num_periods))
            self.graph.edges[link].setdefault("sample_path", False)
        # :197-238 -- node / edge asserts, then the scalar ones
        validate_inputs(self.graph, self.num_periods, self.user_D, self.sample_path)
        assert isinstance(self.backlog, bool), "backlog must be boolean"
        assert 0 < self.alpha <= 1, "alpha must be in (0, 1]"
        assert self.num_periods > 0, "num_periods must be positive"
        self.topology = compile_graph(self.graph, self.num_periods, self.user_D, self.sample_path,
                                      validate=False)
        tp = self.topology
        self.main_nodes, self.reorder_links = tp.main_nodes, tp.reorder_links
        self.retail_links, self.network_links = tp.retail_links, tp.network_links
        self.market, self.rawmat, self.factory = tp.market, tp.rawmat, tp.factory
        self.distrib, self.retail = tp.distrib, tp.retail
        self.lead_times, self.lt_max = tp.lead_times, tp.lt_max
        self.pipeline_obs_length = sum(self.lead_times.values())
        self.obs_dim_ref = tp.obs_dim
        # :193-195, :270-298 spaces
        g = self.graph
        init_inv_max = max((g.nodes[j].get("I0", 0) for j in self.main_nodes), default=100)
        capacity_max = max((g.nodes[j].get("C", 0) for j in self.factory), default=100)
        self.order_cap_heuristic = init_inv_max + capacity_max * 5
        E = len(self.reorder_links)
        self.single_action_space = Box(low=np.zeros(E, np.float32),
                                       high=np.ones(E, np.float32) * self.order_cap_heuristic * 2,
                                       shape=(E,), dtype=np.float32)
        hi = self.order_cap_heuristic * self.num_periods * 2
        lo = 0.0 if not self.backlog else -hi
        obs_low = np.full(tp.obs_dim, lo, np.float32)
        obs_low[: len(self.retail_links)] = 0.0
        self.single_observation_space = Box(low=obs_low, high=np.full(tp.obs_dim, hi, np.float32),
                                            shape=(tp.obs_dim,), dtype=np.float32)
        super().__init__(num_envs, device=device, **vector_kwargs)

    def _create(self):
        self._spec = self.topology.spec(self.backlog, self.alpha)
        self._create_handle(self._lib.invsim_create_netinvmgmt, self._spec)

    def _horizon(self):
        return self.num_periods

    def reset(self, *, seed=None, options=None):
        # :301-306 -> :240-267: the reference re-binds the market samplers at every
        # reset; a lambda market must name this env (topology.check_market_receivers)
        check_market_receivers(self.graph, self.retail_links, self)
        return super().reset(seed=seed, options=options)

    def sample_action(self):
        hi = float(self.single_action_space.high[0]) if len(self.reorder_links) else 0.0
        return torch.rand((self.num_envs, len(self.reorder_links)), device=self.device) * hi


class NetInvMgmtBacklogEnv(NetInvMgmtMasterEnv):
    """network_management.py:747-753."""

    def __init__(self, *args, **kwargs):
        env_config = dict(kwargs.pop("env_config", None) or {})
        env_config["backlog"] = True
        super().__init__(*args, env_config=env_config, **kwargs)


class NetInvMgmtLostSalesEnv(NetInvMgmtMasterEnv):
    """network_management.py:755-770 (effective backlog = the ``backlog`` argument)."""

    def __init__(self, *args, **kwargs):
        env_config = dict(kwargs.pop("env_config", None) or {})
        env_config["backlog"] = False
        super().__init__(*args, env_config=env_config, **kwargs)
        low = self.single_observation_space.low.copy()
        low[: len(self.retail_links)] = 0.0
        self.single_observation_space = Box(low=low, high=self.single_observation_space.high,
                                            shape=(self.obs_dim_ref,), dtype=np.float32)
        self.observation_space = batch_box(self.single_observation_space, self.num_envs)
