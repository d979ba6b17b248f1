"""ctypes front end of the B-opt CPU baseline (oracle/piadmm_cpu.cpp -> oracle/libpiadmm_cpu.so).

MEASUREMENT / TEST INFRASTRUCTURE ONLY: bench.py's ``cpu_baseline`` leg and tests/ use it.  It
runs any scenario (the tiled intersection, the all-pairs crossings, any static candidate graph)
through the oracle's loop (oracle/piadmm_oracle.py, casadi/main.py:43-201) in C++ with OpenMP over
connected components and returns the same per-step records, so tests/test_cpu_bopt.py can hold it
to the NumPy oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libpiadmm_cpu.so")

_INT_FIELDS = ("H", "max_outer", "dual_mode", "windup", "round_decimals", "collide_sq_thres",
               "alias_dual_residual", "pos_model", "term_dist_check", "fixed_iters", "term_global", "tighten",
               "warm_duals", "no_collision_gate")
_DBL_FIELDS = ("dt", "L", "dis_thres", "beta", "Pnorm", "Pcost", "rho", "eps_pri", "eps_dual", "u_max",
               "du_max", "kI", "theta1", "theta2", "windup_sat", "tight_p", "avg_delay", "var_delay", "qp_tol")


class _Cfg(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int) for f in _INT_FIELDS] + [(f, ctypes.c_double) for f in _DBL_FIELDS]


_lib = None


def build() -> None:
    subprocess.run(["make", "-C", HERE, "-s", "libpiadmm_cpu.so"], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        lib.piadmm_cpu_cfg_size.restype = ctypes.c_int
        P = ctypes.c_void_p
        lib.piadmm_cpu_run_graph.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_int,
                                             P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P, P]
        lib.piadmm_cpu_run_graph.restype = ctypes.c_int
        lib.piadmm_cpu_set_tie_tol.argtypes = [ctypes.c_double]
        lib.piadmm_cpu_set_tie_tol.restype = None
        lib.piadmm_cpu_get_ties.argtypes = [P, P, P, ctypes.c_int]
        lib.piadmm_cpu_get_ties.restype = ctypes.c_int
        if lib.piadmm_cpu_cfg_size() != ctypes.sizeof(_Cfg):
            raise RuntimeError("libpiadmm_cpu.so config layout differs from oracle/cpu_bopt.py")
        _lib = lib
    return _lib


def _cfg(cfg) -> _Cfg:
    if cfg.dual_mode not in (0, 1):
        raise ValueError("the B-opt baseline covers dual modes 0/1 (not the global-PI law)")
    c = _Cfg()
    for f in _INT_FIELDS:
        setattr(c, f, int(getattr(cfg, f)))
    for f in _DBL_FIELDS:
        setattr(c, f, float(getattr(cfg, f)))
    return c


def is_tiled(scn) -> bool:
    N = scn.n_agents
    return N % 2 == 0 and scn.n_edges == N // 2 and np.array_equal(
        scn.edges, np.stack([np.arange(0, N, 2), np.arange(1, N, 2)], 1))


TIE_DTYPE = np.dtype([("step", np.int32), ("iter", np.int32), ("kind", np.int32), ("id", np.int32),
                      ("index", np.int32), ("reserved", np.int32), ("margin", np.float64)])
TIE_KINDS = ("round_u", "round_uhat", "round_seed", "collide", "stop", "dist")


def run(cfg, scn, n_steps: int, threads: int = 1, t0: int = 0, records: bool = True, tie_tol: float = 1e-9):
    """n_steps MPC steps of any scenario (candidate graph scn.edges).  Returns dict(seconds, xt
    (S,N,3), u (S,N,H), iters (S,C), resid (S,C,max_outer,2) NaN-padded, counters, ties); C =
    connected components in order of their first agent (the oracle's Scenario.components()).
    ties = (counts per kind, events): the near-tie log (include/piadmm.h piadmm_get_near_ties)."""
    lib = load()
    lib.piadmm_cpu_set_tie_tol(float(tie_tol))
    c = _cfg(cfg)
    N, H, MO = scn.n_agents, cfg.H, cfg.max_outer
    C = int(scn.components()[1])
    spd = np.ascontiguousarray(scn.spd, np.float64)
    xt0 = np.ascontiguousarray(scn.xt0, np.float64)
    ref = np.ascontiguousarray(scn.ref, np.float64)
    edges = np.ascontiguousarray(scn.edges, np.int32).reshape(-1)
    xt = np.zeros((n_steps, N, 3)) if records else None
    u = np.zeros((n_steps, N, H)) if records else None
    iters = np.zeros((n_steps, C), np.int32) if records else None
    resid = np.zeros((n_steps, C, MO, 2)) if records else None
    secs = ctypes.c_double(0.0)
    cnt = np.zeros(5, np.int64)
    ptr = (lambda a: a.ctypes.data if a is not None else None)
    rc = lib.piadmm_cpu_run_graph(ctypes.byref(c), N, spd.ctypes.data, xt0.ctypes.data, ref.ctypes.data,
                                  ref.shape[2], scn.n_edges, edges.ctypes.data if edges.size else None, t0, n_steps,
                                  threads, ptr(xt), ptr(u), ptr(iters), ptr(resid), ctypes.byref(secs),
                                  cnt.ctypes.data)
    if rc != C:
        raise RuntimeError(f"piadmm_cpu_run_graph failed ({rc})")
    tcnt = np.zeros(len(TIE_KINDS), np.int64)
    ev = np.zeros((4096, 6), np.int32)
    mg = np.zeros(4096)
    nt = lib.piadmm_cpu_get_ties(tcnt.ctypes.data, ev.ctypes.data, mg.ctypes.data, 4096)
    ties = np.zeros(nt, TIE_DTYPE)
    for k, f in enumerate(("step", "iter", "kind", "id", "index", "reserved")):
        ties[f] = ev[:nt, k]
    ties["margin"] = mg[:nt]
    return {"seconds": secs.value, "xt": xt, "u": u, "iters": iters, "resid": resid,
            "counters": dict(zip(("x_qps", "z_qps", "x_hits", "gi_steps", "inexact"), cnt.tolist())),
            "ties": (dict(zip(TIE_KINDS, tcnt.tolist())), ties)}


def time_baseline(cfg, n_tiles: int, budget_s: float, n_steps: int = 20, threads: int | None = None,
                  perturb: bool = True, scn=None, desc: str | None = None) -> dict:
    """Outer iterations per second of the job (bench.py's workload: by default n_tiles seeded tiles;
    ``scn``: any candidate graph), fixed outer iterations, on the host cores oracle.hostinfo
    reports: median and spread of repeats within ~budget_s."""
    import time
    from piadmm import scenario

    from oracle import hostinfo
    hi = hostinfo.host_cpu()
    threads = threads or hi["threads"]
    if scn is None:
        scn = scenario.tiled(n_tiles, cfg.H, n_steps=n_steps, perturb=perturb, seed=0)
    run(cfg, scn, 1, threads, records=False)            # warm-up (page-in, thread pool)
    times, t_end, cnt = [], time.perf_counter() + budget_s, None
    while len(times) < 5 or (time.perf_counter() < t_end and len(times) < 15):
        r = run(cfg, scn, n_steps, threads, records=False)
        times.append(r["seconds"])
        cnt = r["counters"]
        if time.perf_counter() > t_end and len(times) >= 1 and times[0] * 5 > budget_s:
            break
    ts = np.sort(np.asarray(times))
    med = float(np.median(ts))
    it_per_step = cfg.max_outer if cfg.fixed_iters else None
    value = n_steps * it_per_step / med if it_per_step else None
    job = desc or f"{n_tiles} tiles"
    return {"value": value, "unit": "outer_iters/s", "cores": threads, "kind": "port",
            "ms_per_step": 1e3 * med / n_steps,
            "spread": {"runs": len(ts), "min_ms_per_step": 1e3 * float(ts[0]) / n_steps,
                       "max_ms_per_step": 1e3 * float(ts[-1]) / n_steps,
                       "iqr_ms_per_step": 1e3 * float(np.percentile(ts, 75) - np.percentile(ts, 25)) / n_steps},
            "host": hi,
            "sample": f"B-opt: C++ -O3 (x86-64-v3) + OpenMP over components, "
                      f"{hostinfo.describe(hi) if threads == hi['threads'] else f'{threads} threads'} "
                      f"(oracle/piadmm_cpu.cpp: the GPU kernel's algorithm -- dual active set with bounded "
                      f"hinge multipliers, cached working-set factors -- exact answers, equal to the oracle, "
                      f"tests/test_cpu_bopt.py); the full job: {job} x MPC steps 0..{n_steps - 1} x "
                      f"{cfg.max_outer} outer iterations, median of {len(times)} runs ({med:.3f} s each, "
                      f"min {ts[0]:.3f} max {ts[-1]:.3f}); "
                      f"{cnt['x_qps']} x-QPs ({cnt['x_hits']} cached-set hits), {cnt['z_qps']} pair QPs, "
                      f"{cnt['inexact']} uncertified per run"}
