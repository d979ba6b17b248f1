"""piadmm -- MI355X-native batched PI-ADMM consensus solver (host side).

The compute path is libpiadmm.so (HIP, gfx950) behind the C-ABI in
include/piadmm.h; this package is the Python host driver that mirrors the
reference's ``PI_ADMM_CASADI`` class and ``casadi/main.py`` loop.
"""
from .config import PIADMMConfig, PRESETS, casadi_default, matlab_pi  # noqa: F401
from .scenario import Scenario, intersection, tiled  # noqa: F401

__all__ = ["PIADMMConfig", "PRESETS", "casadi_default", "matlab_pi", "Scenario", "intersection",
           "tiled", "PI_ADMM_MI355X"]


def __getattr__(name):
    if name == "PI_ADMM_MI355X":
        from .solver import PI_ADMM_MI355X
        return PI_ADMM_MI355X
    raise AttributeError(name)
