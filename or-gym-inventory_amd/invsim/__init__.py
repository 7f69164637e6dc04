"""invsim — MI355X-native vectorised inventory-simulation engine.

Drop-in, batched replacements for the env classes of jacklu2016/or-gym-inventory,
running their ``step()``/``reset()`` as HIP kernels on gfx950 (libinvsim.so):

* :class:`NewsvendorEnv`                       (newsvendor.py)
* :class:`InvManagementMasterEnv`, :class:`InvManagementBacklogEnv`,
  :class:`InvManagementLostSalesEnv`            (inventory_management.py)
* :class:`NetInvMgmtMasterEnv`, :class:`NetInvMgmtBacklogEnv`,
  :class:`NetInvMgmtLostSalesEnv`               (network_management.py)

Env classes import torch; ``invsim._capi`` alone does not need a GPU.
"""
__version__ = "0.1.0"

_LAZY = {
    "NewsvendorEnv": "newsvendor",
    "InvManagementMasterEnv": "inventory_management",
    "InvManagementBacklogEnv": "inventory_management",
    "InvManagementLostSalesEnv": "inventory_management",
    "NetInvMgmtMasterEnv": "network_management",
    "NetInvMgmtBacklogEnv": "network_management",
    "NetInvMgmtLostSalesEnv": "network_management",
    "BaseStockAgent": "policies",
    "ConstantOrderAgent": "policies",
    "OrderUpToHeuristicAgent": "policies",
    "ClassicNewsvendorAgent": "policies",
    "sSPolicyAgent": "policies",
    "evaluate_agent": "policies",
    "rollout_policy": "policies",
    "StepGraph": "graphs",
}


_SUBMODULES = ("policies", "topology", "distributed", "spaces", "vector", "newsvendor",
               "inventory_management", "network_management", "graphs")


def __getattr__(name):
    import importlib
    if name in _LAZY:
        return getattr(importlib.import_module(f".{_LAZY[name]}", __name__), name)
    if name in _SUBMODULES:
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)


__all__ = list(_LAZY)
