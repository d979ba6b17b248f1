"""The C-ABI library: it loads, exports every symbol include/piadmm.h declares, and its
config struct matches the binding.  No kernels run here (no GPU in the build container)."""
import ctypes
import os
import re

import numpy as np
import pytest
from conftest import ROOT

from piadmm import _lib, config, scenario

HEADER = os.path.join(ROOT, "include", "piadmm.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|const char\*)\s+(piadmm_\w+)\s*\(", src, re.M)))


def test_library_is_built_for_gfx950():
    assert os.path.exists(_lib.LIB_PATH), "run make -C distributed-local-planner-pi-admm_amd"
    lib = _lib.load()
    info = lib.piadmm_build_info().decode()
    assert "gfx950" in info
    assert lib.piadmm_abi_version() == 7


def test_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 15
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    bound = {n for n, _, _ in _lib.SYMBOLS}
    assert set(names) <= bound, set(names) - bound


def test_config_struct_layout():
    lib = _lib.load()
    assert lib.piadmm_config_size() == ctypes.sizeof(_lib.PiadmmConfigC) == 312   # ABI 7
    c = _lib.to_c(config.matlab_pi(H=30), n_agents=256, device=3)
    assert (c.n_agents, c.H, c.device, c.dual_mode, c.windup) == (256, 30, 3, 1, 1)
    # every dataclass field the struct carries is mirrored
    fields = {f for f, _ in _lib.PiadmmConfigC._fields_} - {"n_agents", "device"}
    assert fields <= set(config.PIADMMConfig.__dataclass_fields__)


def test_loud_failure_without_library(tmp_path):
    with pytest.raises(_lib.PiadmmError):
        _lib.load(str(tmp_path / "missing.so"))


def test_create_fails_loudly_without_device():
    lib = _lib.load()
    if lib.piadmm_device_count() > 0:
        pytest.skip("a GPU is visible")
    c = _lib.to_c(config.casadi_default(H=10), n_agents=2)
    h = ctypes.c_void_p()
    rc = lib.piadmm_create(ctypes.byref(c), ctypes.byref(h))
    assert rc == -4 and not h.value
    assert b"no HIP device" in lib.piadmm_last_error(None)
    from piadmm.solver import PI_ADMM_MI355X
    with pytest.raises(_lib.PiadmmError):
        PI_ADMM_MI355X(config.casadi_default(H=10), scenario.intersection(10))


def test_near_tie_record_layout_matches_header():
    """piadmm_near_tie_t = 6 int32 + one double (32 bytes); kinds and capacity as in the header."""
    src = open(HEADER).read()
    assert _lib.TIE_DTYPE.itemsize == 32
    for k, name in enumerate(_lib.TIE_KINDS):
        assert re.search(rf"#define PIADMM_TIE_{name.upper()} {k}\b", src), name
    assert re.search(rf"#define PIADMM_TIE_CAP {_lib.TIE_CAP}\b", src)


def test_header_enums_match_python():
    src = open(HEADER).read()
    assert re.search(r"#define PIADMM_DUAL_PLAIN 0", src) and config.DUAL_PLAIN == 0
    assert re.search(r"#define PIADMM_DUAL_PI 1", src) and config.DUAL_PI == 1
    assert np.dtype(np.float64).itemsize == 8
