"""Near-tie logs of the CPU checkers (oracle TieLog, B-opt piadmm_cpu.cpp): the mirror of
piadmm_get_near_ties (include/piadmm.h).  The reference's loop takes discrete
decisions -- rounding to 4 decimals (casadi/main.py:48-49,103,153), the collision test
d^2 < dis_thres (:112-113), the stop test (:174), MATLAB's distance check -- and two exact
implementations can part only where one of them falls within rounding of its threshold.  The
oracle and B-opt must log the same decisions (with a tolerance wide enough for events to occur),
and the margins must be the arithmetic the kernels use."""
import numpy as np
import pytest

from oracle import cpu_bopt
from oracle import piadmm_oracle as O
from piadmm import config, scenario

KEY = ("step", "iter", "kind", "id", "index")


def oracle_events(orc):
    return {tuple(int(v) for v in e[:5]): e[5] for e in orc.ties.events}


def bopt_events(ties):
    return {tuple(int(e[k]) for k in KEY): float(e["margin"]) for e in ties}


def test_round_margins_are_the_kernels_arithmetic():
    """margin = x - (k + 1/2) 10^-4: zero exactly at a boundary, sign = side, |m| <= 5e-5."""
    x = np.array([0.12345, 0.12344999, -0.00005, 0.3, -0.52359])
    m = O.round_margins(x, 4)
    assert abs(m[0]) < 1e-15 and m[1] < 0 and abs(m[2]) < 1e-15
    assert np.all(np.abs(m) <= 5e-5 + 1e-15)
    # np.around and the boundary agree: values just off a boundary round away from it
    assert np.around(0.12345 + 1e-12, 4) == 0.1235 and np.around(0.12345 - 1e-12, 4) == 0.1234


@pytest.mark.parametrize("preset,tol", [("casadi_default", 3e-6), ("matlab_pi", 0.2)])
def test_oracle_and_bopt_log_the_same_near_ties(preset, tol):
    """casadi_default rounds (u, u_hat, seeds within 3e-6 of a boundary: ~6 % of the values);
    matlab_pi has no rounding but the collision, stop and distance tests (20 % relative)."""
    cfg = config.PRESETS[preset](H=10)
    scn = scenario.tiled(2, 10, n_steps=26, seed=3)
    orc = O.Oracle(cfg, scn)
    orc.ties.tol = tol
    for _ in range(24):
        orc.mpc_step()
    rc = cpu_bopt.run(cfg, scn, 24, threads=2, tie_tol=tol)
    eo, eb = oracle_events(orc), bopt_events(rc["ties"][1])
    assert len(eo) > 0
    # events whose margin sits at the tolerance edge may fall on either side (rounding): ignore them
    so = {k for k, m in eo.items() if abs(abs(m) - tol) > 1e-6 * tol}
    sb = {k for k, m in eb.items() if abs(abs(m) - tol) > 1e-6 * tol}
    assert so == sb, (sorted(so ^ sb)[:10], len(so), len(sb))
    for k in so:
        assert abs(eo[k] - eb[k]) <= 1e-9 * max(1.0, abs(eo[k])), (k, eo[k], eb[k])
    counts = rc["ties"][0]
    assert sum(counts.values()) == len(rc["ties"][1])
    if preset == "casadi_default":
        assert counts["round_u"] > 0 and counts["round_seed"] >= 0
    else:
        assert counts["round_u"] == 0 and counts["round_uhat"] == 0


def test_default_tolerance_logs_nothing_on_the_golden_run():
    """At the default 1e-9 the 2-vehicle reference run (casadi_default, H10, 40 steps) takes no
    decision within rounding of its threshold: its golden trajectory is robust."""
    cfg = config.casadi_default(H=10)
    scn = scenario.intersection(10, n_steps=40)
    orc = O.Oracle(cfg, scn)
    for _ in range(40):
        orc.mpc_step()
    assert orc.ties.events == []
