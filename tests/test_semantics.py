"""Oracle semantics of the ABI-2 rows: global termination (quirk B9), receding-horizon dual
warm start and delay tightening (row a13).  CPU only."""
import math

import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import config, scenario


def run(cfg, scn, n):
    o = O.Oracle(cfg, scn)
    return o, [o.mpc_step() for _ in range(n)]


def test_global_termination_single_pair_equals_per_component():
    """For the reference's two vehicles the global flag / termination IS the per-pair one."""
    scn = scenario.intersection(15)
    for preset in ("matlab_pi", "casadi_default"):
        _, a = run(config.PRESETS[preset](H=15), scn, 30)
        _, b = run(config.PRESETS[preset](H=15, term_global=1), scn, 30)
        for ra, rb in zip(a, b):
            np.testing.assert_array_equal(ra.iters, rb.iters)
            np.testing.assert_array_equal(ra.xt, rb.xt)
            np.testing.assert_allclose(np.array(ra.resid[0]).reshape(-1, 2), np.array(rb.global_resid).reshape(-1, 2))


def test_global_termination_couples_components():
    """Over several tiles every component runs the job's iteration count, the global history
    is the sum of the per-component ones, and a tile that stops early on its own runs on."""
    scn = scenario.tiled(3, 15, n_steps=30, seed=3)
    _, loc = run(config.casadi_default(H=15), scn, 12)
    _, glo = run(config.casadi_default(H=15, term_global=1), scn, 12)
    differs = False
    for rl, rg in zip(loc, glo):
        assert len(set(rg.iters.tolist())) == 1
        assert rg.iters[0] >= max(rl.iters)       # a global stop satisfies every local test
        n = int(rg.iters[0])
        summed = np.sum([np.array(r) for r in rg.resid], axis=0)
        if len(rg.global_resid):
            np.testing.assert_allclose(np.array(rg.global_resid), summed[:len(rg.global_resid)])
        differs |= bool(np.any(rl.iters != n))
    assert differs, "the scenario should contain a tile that stops before the others"


def test_global_fixed_iterations_equal_per_component_results():
    """With fixed_iters the termination scope cannot change any state."""
    scn = scenario.tiled(2, 12, n_steps=10, seed=1)
    _, a = run(config.matlab_pi(H=12, fixed_iters=1, max_outer=5), scn, 4)
    _, b = run(config.matlab_pi(H=12, fixed_iters=1, max_outer=5, term_global=1), scn, 4)
    for ra, rb in zip(a, b):
        np.testing.assert_array_equal(ra.xt, rb.xt)
        np.testing.assert_allclose(np.array(rb.global_resid), np.sum([np.array(r) for r in ra.resid], axis=0))


def test_shift_horizon_is_iterate_next_state():
    """decentralized/optimizer.py:337-344: concatenate(Z[:, 1:], Z[:, -1:]) along the horizon."""
    a = np.arange(2 * 3 * 5, dtype=float).reshape(2, 3, 5)
    np.testing.assert_array_equal(O.shift_horizon(a), np.concatenate((a[..., 1:], a[..., -1:]), axis=-1))


def test_warm_duals_carry_the_shifted_edge_state():
    scn = scenario.intersection(15)
    cfg_w = config.matlab_pi(H=15, warm_duals=1)
    o_c, cold = run(config.matlab_pi(H=15), scn, 14)
    o_w = O.Oracle(cfg_w, scn)
    warm = []
    for k in range(14):
        prev = None if o_w.edge_state is None else [x.copy() for x in o_w.edge_state]
        warm.append(o_w.mpc_step())
        if prev is None or not np.any(prev[1]):
            continue
        # a step whose pair never collides keeps the shifted duals untouched
        if warm[-1].iters[0] == 1:
            np.testing.assert_array_equal(warm[-1].lam, O.shift_horizon(prev[1]))
    np.testing.assert_array_equal(cold[0].xt, warm[0].xt)       # first step: nothing to carry
    assert any(not np.array_equal(c.xt, w.xt) for c, w in zip(cold, warm))


def test_delay_offset_restates_util_py():
    """compute_square_halfspaces_ca_prob (decentralized/util.py:81-96) written out by hand:
    delta = avg v (cos, sin) + sqrt(p / (1 - p)) ((var v cos)^2, (var v sin)^2)."""
    cfg = config.matlab_pi(tighten=1)
    v, th = 8.0, -math.pi / 2 + 0.3
    c, s = math.cos(th), math.sin(th)
    k = math.sqrt(0.95 / 0.05)
    want = [0.05 * v * c + k * (0.025 * v * c) ** 2, 0.05 * v * s + k * (0.025 * v * s) ** 2]
    np.testing.assert_allclose(O.delay_offset(cfg, np.array([1.0, 2.0, th]), v), want, rtol=1e-15)
    xt = np.array([[0.0, 0.0, 0.0], [0.0, 5.0, th]])
    d = O.safety_distance(cfg, xt, np.array([4.0, v]), 0, 1)
    assert d == pytest.approx(2.0 + math.hypot(*O.delay_offset(cfg, xt[0], 4.0)) + math.hypot(*want))
    assert O.safety_distance(config.matlab_pi(), xt, np.array([4.0, v]), 0, 1) == 2.0


def test_tightening_widens_the_collision_test():
    """A larger safety distance makes pairs collide at least as often, and changes the plan."""
    scn = scenario.intersection(15)
    _, base = run(config.matlab_pi(H=15), scn, 30)
    _, tight = run(config.matlab_pi(H=15, tighten=1, avg_delay=0.2, var_delay=0.1), scn, 30)
    n_base = sum(int(r.iters[0] > 1) for r in base)
    n_tight = sum(int(r.iters[0] > 1) for r in tight)
    assert n_tight >= n_base
    assert any(not np.array_equal(a.xt, b.xt) for a, b in zip(base, tight))
