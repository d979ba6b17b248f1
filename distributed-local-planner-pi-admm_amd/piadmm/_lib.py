"""ctypes binding of libpiadmm.so (include/piadmm.h).

There is no fallback: if the HIP library is missing or cannot be loaded,
``load()`` raises, and so does every solver entry point.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .config import PIADMMConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpiadmm.so")

c_i32, c_dbl = ctypes.c_int32, ctypes.c_double


class PiadmmConfigC(ctypes.Structure):
    """Byte-for-byte mirror of ``piadmm_config_t``."""
    _fields_ = [
        ("n_agents", c_i32), ("H", c_i32), ("max_outer", c_i32), ("dual_mode", c_i32),
        ("dt", c_dbl), ("L", c_dbl), ("dis_thres", c_dbl), ("beta", c_dbl), ("Pnorm", c_dbl),
        ("Pcost", c_dbl), ("rho", c_dbl), ("eps_pri", c_dbl), ("eps_dual", c_dbl),
        ("u_max", c_dbl), ("du_max", c_dbl),
        ("kP", c_dbl), ("kI", c_dbl), ("theta1", c_dbl), ("theta2", c_dbl), ("windup_sat", c_dbl),
        ("windup", c_i32), ("round_decimals", c_i32), ("collide_sq_thres", c_i32),
        ("alias_dual_residual", c_i32), ("pos_model", c_i32), ("term_dist_check", c_i32),
        ("fixed_iters", c_i32), ("max_inner", c_i32),
        ("admm_rho", c_dbl), ("admm_sigma", c_dbl), ("admm_alpha", c_dbl), ("qp_tol", c_dbl),
        ("polish_every", c_i32), ("device", c_i32),
        ("term_global", c_i32), ("warm_duals", c_i32), ("tighten", c_i32), ("precision", c_i32),
        ("tight_p", c_dbl), ("avg_delay", c_dbl), ("var_delay", c_dbl),
        ("rho_num", c_dbl), ("rho_min", c_dbl), ("rho_max", c_dbl), ("no_collision_gate", c_i32),
        ("pi_trad", c_i32), ("ki_adapt", c_i32), ("reserved1", c_i32), ("d_gain", c_dbl), ("dual_init", c_dbl),
    ]


def to_c(cfg: PIADMMConfig, n_agents: int, device: int = 0) -> PiadmmConfigC:
    c = PiadmmConfigC()
    for name, _ in PiadmmConfigC._fields_:
        if name == "n_agents":
            c.n_agents = int(n_agents)
        elif name == "device":
            c.device = int(device)
        else:
            setattr(c, name, getattr(cfg, name))
    return c


# (name, restype, argtypes) -- every symbol declared in include/piadmm.h
_P = ctypes.POINTER
_H = ctypes.c_void_p
_dp = _P(c_dbl)
_ip = _P(c_i32)
SYMBOLS = [
    ("piadmm_abi_version", c_i32, []),
    ("piadmm_build_info", ctypes.c_char_p, []),
    ("piadmm_device_count", c_i32, []),
    ("piadmm_config_size", c_i32, []),
    ("piadmm_create", c_i32, [_P(PiadmmConfigC), _P(_H)]),
    ("piadmm_destroy", c_i32, [_H]),
    ("piadmm_last_error", ctypes.c_char_p, [_H]),
    ("piadmm_set_scenario", c_i32, [_H, _dp, _dp, _dp, c_i32, _ip, c_i32]),
    ("piadmm_set_xt", c_i32, [_H, _dp]),
    ("piadmm_mpc_step", c_i32, [_H, c_i32, _dp, _dp, _dp, _ip, _ip]),
    ("piadmm_mpc_steps_async", c_i32, [_H, c_i32, c_i32]),
    ("piadmm_sync", c_i32, [_H]),
    ("piadmm_time_steps", c_i32, [_H, c_i32, c_i32, _P(ctypes.c_float)]),
    ("piadmm_get_state", c_i32, [_H, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _P(ctypes.c_uint8), _ip]),
    ("piadmm_outer_iter", c_i32, [_H, c_i32, c_i32, _ip]),
    ("piadmm_step_finish", c_i32, [_H, _dp, _dp]),
    ("piadmm_n_components", c_i32, [_H]),
    ("piadmm_steps_per_launch", c_i32, [_H]),
    ("piadmm_get_counters", c_i32, [_H, _P(ctypes.c_uint64)]),
    ("piadmm_reset_counters", c_i32, [_H]),
    ("piadmm_get_component_counters", c_i32, [_H, _P(ctypes.c_uint64), c_i32]),
    ("piadmm_debug_stamps", c_i32, [_H, _P(ctypes.c_uint64), c_i32]),
    ("piadmm_comm_unique_id", c_i32, [_P(ctypes.c_uint8)]),
    ("piadmm_comm_init", c_i32, [_H, _P(ctypes.c_uint8), c_i32, c_i32]),
    ("piadmm_global_resid", c_i32, [_H, _dp, _ip]),
    ("piadmm_set_scenario_shard", c_i32, [_H, _dp, _dp, _dp, c_i32, _ip, c_i32, _P(ctypes.c_uint8), _ip, c_i32,
                                          _P(ctypes.c_uint8)]),
    ("piadmm_set_allreduce", c_i32, [_H, ctypes.c_void_p, ctypes.c_void_p]),
    ("piadmm_candidate_pairs", c_i32, [_H, _dp, _dp, c_i32, _ip, c_i32, _ip, _P(ctypes.c_float)]),
    ("piadmm_set_tie_tolerance", c_i32, [_H, c_dbl]),
    ("piadmm_get_near_ties", c_i32, [_H, _P(ctypes.c_uint64), ctypes.c_void_p, c_i32, _ip]),
    ("piadmm_get_step_state", c_i32, [_H, _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
    ("piadmm_set_state", c_i32, [_H, _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
    ("piadmm_obca_create", c_i32, [c_i32, _P(_H)]),
    ("piadmm_obca_destroy", c_i32, [_H]),
    ("piadmm_obca_last_error", ctypes.c_char_p, [_H]),
    ("piadmm_obca_solve", c_i32, [_H, _dp, c_i32, _dp, _ip]),
    ("piadmm_obca_upload", c_i32, [_H, _dp, c_i32]),
    ("piadmm_obca_run", c_i32, [_H, c_i32]),
    ("piadmm_obca_time", c_i32, [_H, c_i32, _P(ctypes.c_float)]),
    ("piadmm_obca_download", c_i32, [_H, _dp, _ip, c_i32]),
    ("piadmm_obca_debug_stamps", c_i32, [_H, _P(ctypes.c_uint64), c_i32]),
]

# piadmm_near_tie_t (include/piadmm.h, ABI 6) as a NumPy record
TIE_KINDS = ("round_u", "round_uhat", "round_seed", "collide", "stop", "dist")
TIE_DTYPE = np.dtype([("step", np.int32), ("iter", np.int32), ("kind", np.int32), ("id", np.int32),
                      ("index", np.int32), ("reserved", np.int32), ("margin", np.float64)])
TIE_CAP = 4096

# piadmm_allreduce_fn: int32_t (*)(void* ctx, double* buf, int64_t n)
ALLREDUCE_FN = ctypes.CFUNCTYPE(c_i32, ctypes.c_void_p, _dp, ctypes.c_int64)

_lib = None


class PiadmmError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load libpiadmm.so (built by ``make`` / ``__graft_entry__.build()``); raise if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # PIADMM_LIB selects another build of the same library (e.g. the stamps build)
    p = path or os.environ.get("PIADMM_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise PiadmmError(f"HIP library not built: {p} (run `make -C distributed-local-planner-pi-admm_amd`)")
    lib = ctypes.CDLL(p)
    for name, res, args in SYMBOLS:
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.piadmm_config_size() != ctypes.sizeof(PiadmmConfigC):
        raise PiadmmError("piadmm_config_t layout mismatch between header and binding")
    if path is None:
        _lib = lib
    return lib


def unload():
    """dlclose libpiadmm.so once every handle is closed (bench.py's exit): its code object is then
    unregistered from the HIP runtime while the runtime -- and a profiler's tool library, when one
    is preloaded -- are still fully alive, instead of from the library destructors that run at
    process exit after the profiler has finalised (the round-5 exit fault)."""
    global _lib
    if _lib is None:
        return
    import _ctypes
    h = _lib._handle
    _lib = None
    _ctypes.dlclose(h)


def check(rc: int, handle=None):
    if rc != 0:
        msg = load().piadmm_last_error(handle)
        raise PiadmmError(f"libpiadmm error {rc}: {msg.decode() if msg else ''}")


def dptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def iptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_ip)
