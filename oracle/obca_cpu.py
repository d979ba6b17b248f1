"""ctypes front end of the OBCA CPU baseline (oracle/obca_cpu.cpp -> oracle/libobca_cpu.so).

MEASUREMENT / TEST INFRASTRUCTURE ONLY (bench.py --obca cpu_baseline, tests/test_obca_cpu.py):
the SQP of oracle/obca_oracle.py in C++ -O3, OpenMP over the problems of a batch, same record /
output layout as the GPU path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libobca_cpu.so")
REC, OUT = 296, 224
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "-s", "libobca_cpu.so"], check=True)
        lib = ctypes.CDLL(LIB)
        lib.obca_cpu_solve.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.obca_cpu_solve.restype = ctypes.c_int
        _lib = lib
    return _lib


def solve(recs, threads=1):
    """(out n x 224, status n x 3) for a batch of records; wall seconds in the third slot."""
    recs = np.ascontiguousarray(recs, np.float64)
    n = recs.shape[0]
    out = np.zeros((n, OUT))
    ist = np.zeros((n, 3), np.int32)
    t0 = time.perf_counter()
    load().obca_cpu_solve(recs.ctypes.data, n, out.ctypes.data, ist.ctypes.data, int(threads))
    return out, ist, time.perf_counter() - t0
