"""ctypes binding of libinvsim.so (the C ABI in include/invsim.h).

The library is built in-tree (``or-gym-inventory_amd/csrc/Makefile`` ->
``invsim/_lib/libinvsim.so``).  There is no CPU fallback: if the library or a
GPU is missing, :func:`lib` raises.  torch is imported first so the library's
``libamdhip64.so.7`` dependency binds to the HIP runtime torch already loaded
(one runtime, shared streams and device pointers).
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# INVSIM_LIB: load another build of the same ABI (profiling ablations, tools/)
LIB_PATH = os.environ.get("INVSIM_LIB") or os.path.join(HERE, "_lib", "libinvsim.so")
CSRC = os.path.normpath(os.path.join(HERE, "..", "csrc"))

INVSIM_NEWSVENDOR, INVSIM_INVMGMT, INVSIM_NETINVMGMT = 1, 2, 3
AUTORESET_MODES = {"next_step": 0, "same_step": 1, "disabled": 2}

# every symbol include/invsim.h declares
EXPORTS = (
    "invsim_abi_version", "invsim_last_error", "invsim_create_newsvendor",
    "invsim_create_invmgmt", "invsim_create_netinvmgmt", "invsim_destroy", "invsim_dims",
    "invsim_set_autoreset", "invsim_seed_range", "invsim_seed_words", "invsim_reset",
    "invsim_step", "invsim_rollout", "invsim_status", "invsim_kernel_variant", "invsim_metrics_dim",
    "invsim_rollout_policy", "invsim_info_record_dim", "invsim_set_info_record", "invsim_set_info_demand",
    "invsim_state_bytes",
    "invsim_state_field", "invsim_get_state", "invsim_set_state", "invsim_episode_fold",
    "invsim_debug_ptrs_stats", "invsim_set_demand_stream", "invsim_demand_stream",
    "invsim_capture_begin", "invsim_capture_end", "invsim_position",
    "invsim_episode_fold_groups", "invsim_set_episode_sink",
)
ABI_VERSION = 4
DEMAND_STREAMS = {"numpy": 0, "philox": 1}


class NewsvendorSpec(C.Structure):
    _fields_ = [("lead_time", C.c_int32), ("step_limit", C.c_int32),
                ("max_inventory", C.c_double), ("max_order_quantity", C.c_double),
                ("p_max", C.c_double), ("h_max", C.c_double), ("k_max", C.c_double),
                ("mu_max", C.c_double), ("gamma", C.c_double)]


class InvMgmtSpec(C.Structure):
    _fields_ = [("num_stages", C.c_int32), ("periods", C.c_int32), ("backlog", C.c_int32),
                ("dist", C.c_int32), ("mu", C.c_double), ("alpha", C.c_double),
                ("I0", C.c_void_p), ("unit_price", C.c_void_p), ("unit_cost", C.c_void_p),
                ("demand_cost", C.c_void_p), ("holding_cost", C.c_void_p),
                ("supply_capacity", C.c_void_p), ("lead_time", C.c_void_p), ("user_D", C.c_void_p),
                ("dist_n", C.c_int64), ("dist_p", C.c_double), ("dist_low", C.c_int64), ("dist_high", C.c_int64)]


NET_TABLE_FIELDS = ("I0", "h", "C", "o", "v", "is_factory", "is_retail", "sup", "pur",
                    "sup_is_factory", "L", "lp", "lg", "rl_node", "rl_p", "rl_b", "rl_lam",
                    "rl_user", "user_D", "succ_ptr", "succ_kind", "succ_idx", "pred_ptr", "pred_idx",
                    "rl_dist", "rl_n", "rl_high", "rl_dp")


class NetInvMgmtSpec(C.Structure):
    _fields_ = [("n_main", C.c_int32), ("n_reorder", C.c_int32), ("n_retail", C.c_int32),
                ("num_periods", C.c_int32), ("backlog", C.c_int32), ("alpha", C.c_double)] + [
        (n, C.c_void_p) for n in NET_TABLE_FIELDS]


POLICY_KINDS = {"constant": 1, "base_stock": 2, "order_up_to": 3, "classic_nv": 4, "ss": 5}


class PolicySpec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("variant", C.c_int32), ("safety_factor", C.c_double),
                ("mu", C.c_double), ("constant", C.c_void_p)]


class InvsimError(RuntimeError):
    pass


_LIB = None


def _declare(lib):
    P, I32, I64, U64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    H = C.c_void_p
    sig = {
        "invsim_abi_version": ([], C.c_int),
        "invsim_last_error": ([H], C.c_char_p),
        "invsim_create_newsvendor": ([P, I64, I32, I32, P], C.c_int),
        "invsim_create_invmgmt": ([P, I64, I32, I32, P], C.c_int),
        "invsim_create_netinvmgmt": ([P, I64, I32, I32, P], C.c_int),
        "invsim_destroy": ([H], None),
        "invsim_dims": ([H, P, P, P, P], C.c_int),
        "invsim_set_autoreset": ([H, I32], C.c_int),
        "invsim_seed_range": ([H, U64, U64, I64, P, P], C.c_int),
        "invsim_seed_words": ([H, P, P, P, P], C.c_int),
        "invsim_reset": ([H, P, P, P], C.c_int),
        "invsim_step": ([H, P, P, P, P, P, P, P], C.c_int),
        "invsim_rollout": ([H, I32, P, P, P, P, P, P], C.c_int),
        "invsim_status": ([H, P, I32], C.c_int),
        "invsim_kernel_variant": ([H, P], C.c_int),
        "invsim_metrics_dim": ([H, P], C.c_int),
        "invsim_info_record_dim": ([H, P], C.c_int),
        "invsim_set_info_record": ([H, P], C.c_int),
        "invsim_rollout_policy": ([H, I32, P, P, P, P, P, P, P, P], C.c_int),
        "invsim_set_info_demand": ([H, P], C.c_int),
        "invsim_state_bytes": ([H, P], C.c_int),
        "invsim_state_field": ([H, I32, P, P, P, P, P], C.c_int),
        "invsim_get_state": ([H, P, P], C.c_int),
        "invsim_set_state": ([H, P, P], C.c_int),
        "invsim_episode_fold": ([P, P, P, I32, I64, P, P, P], C.c_int),
        "invsim_episode_fold_groups": ([P, P, P, I32, I64, P, P, P], C.c_int),
        "invsim_set_episode_sink": ([H, P, P], C.c_int),
        "invsim_debug_ptrs_stats": ([P, I32], C.c_int),
        "invsim_set_demand_stream": ([H, I32], C.c_int),
        "invsim_demand_stream": ([H, P], C.c_int),
        "invsim_capture_begin": ([H], C.c_int),
        "invsim_capture_end": ([H, P], C.c_int),
        "invsim_position": ([H, P], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res


def load_library(path=LIB_PATH):
    """Load libinvsim.so without requiring a GPU (symbol/ABI checks)."""
    if not os.path.exists(path):
        raise ImportError(
            f"libinvsim.so not found at {path}: build it with `make -C {CSRC}` "
            "(or __graft_entry__.build()); invsim has no CPU fallback")
    try:
        import torch  # noqa: F401  (bind to torch's HIP runtime, see module doc)
    except ImportError:
        pass
    lib = C.CDLL(path)
    _declare(lib)
    return lib


def lib():
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


def last_error(h=None):
    msg = lib().invsim_last_error(h)
    return msg.decode() if msg else ""


INVSIM_ERANGE = -34


def check(rc, h=None, what="invsim call"):
    if rc == INVSIM_ERANGE and "horizon" in last_error(h):
        raise IndexError(f"{what}: {last_error(h)}")
    if rc != 0:
        raise InvsimError(f"{what} failed ({rc}): {last_error(h)}")
    return rc
