"""GPU near-tie log (piadmm_get_near_ties, include/piadmm.h ABI 6) against the oracle's
(oracle/piadmm_oracle.py TieLog), both kernels: the reference's discrete decisions -- rounding to 4
decimals (casadi/main.py:48-49,103,153), the collision test (:112-113), the stop test (:174),
MATLAB's distance check (ADMM_CVX_..._PI_antiwindup.m:202) -- logged with the same step, iteration,
kind, agent / pair / component and margin.  A wide tolerance makes events frequent; events whose
margin sits at the tolerance's edge (either side, by rounding) are not compared."""
import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import config, scenario

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Solver():
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    return PI_ADMM_MI355X


def _events(rows):
    return {tuple(int(v) for v in r[:5]): float(r[5]) for r in rows}


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("preset,tol", [("casadi_default", 3e-6), ("matlab_pi", 0.2)])
def test_gpu_near_ties_equal_the_oracles(Solver, monkeypatch, graph, preset, tol):
    cfg = config.PRESETS[preset](H=10)
    scn = scenario.tiled(2, 10, n_steps=26, seed=3)
    if graph:
        monkeypatch.setenv("PIADMM_GRAPH", "1")
    orc = O.Oracle(cfg, scn)
    orc.ties.tol = tol
    with Solver(cfg, scn) as s:
        s.set_tie_tolerance(tol)
        for _ in range(24):
            ro, rg = orc.mpc_step(), s.mpc_step()
            np.testing.assert_array_equal(rg.iters, ro.iters)
        counts, ev = s.near_ties()
    eo = {k: m for k, m in _events(orc.ties.events).items() if abs(abs(m) - tol) > 1e-6 * tol}
    eg = {}
    for r in ev:
        k = (int(r["step"]), int(r["iter"]), int(r["kind"]), int(r["id"]), int(r["index"]))
        if abs(abs(r["margin"]) - tol) > 1e-6 * tol:
            eg[k] = float(r["margin"])
    assert len(eo) > 0
    assert set(eo) == set(eg), (sorted(set(eo) ^ set(eg))[:10], len(eo), len(eg))
    for k in eo:
        assert abs(eo[k] - eg[k]) <= 1e-9 * max(1.0, abs(eo[k])), (k, eo[k], eg[k])
    assert sum(counts.values()) == len(ev)


def test_default_tolerance_and_reset(Solver):
    """The log is off by default (its kernel instantiation costs 3-10 %); at 1e-9 the golden
    2-vehicle run logs nothing; a wide tolerance logs; the log resets with the counters."""
    cfg = config.casadi_default(H=10)
    scn = scenario.intersection(10, n_steps=40)
    with Solver(cfg, scn) as s:
        s.set_tie_tolerance(1e-5)
        s.set_tie_tolerance(0.0)                 # off again: nothing is recorded
        for _ in range(3):
            s.mpc_step()
        counts, ev = s.near_ties()
        assert sum(counts.values()) == 0 and ev.size == 0
        s.set_tie_tolerance(1e-9)
        for _ in range(7):
            s.mpc_step()
        counts, ev = s.near_ties()
        assert sum(counts.values()) == 0 and ev.size == 0
        s.set_tie_tolerance(1e-5)
        for _ in range(5):
            s.mpc_step()
        counts, ev = s.near_ties()
        assert counts["round_u"] > 0 and ev.size == sum(counts.values())
        s.reset_counters()
        counts, ev = s.near_ties()
        assert sum(counts.values()) == 0 and ev.size == 0
