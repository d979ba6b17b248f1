"""GPU parity of host stepping (piadmm_outer_iter / piadmm_step_finish, ABI 4) through the C-ABI:
the state of every single outer iteration inside an MPC step against the oracle's.

The reference's inner loop ``for i_iter in range(iter_num)`` (``casadi/main.py:78-181``) carries
pos_old, hat_pos_old and the duals from one iteration to the next; its PI anti-windup variant
(``matlab_old_files/ADMM_CVX_two_veh_intesection_PI_antiwindup.m:160-188``) also carries the
integral S and the back-calculation term D.  Here every iteration's pos_old, hat, lam, S, D from
``piadmm_get_state`` is held to the oracle's state after the same iteration (``Oracle.mpc_step``'s
``on_iter`` hook) at RTOL = ATOL = 1e-8, the stop flag must fire at the same iteration, and the
propagated state after ``piadmm_step_finish`` must equal the oracle's step record.
"""
import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import _lib, config, scenario

pytestmark = pytest.mark.gpu

TOL = 1e-8


@pytest.fixture(scope="module")
def Solver():
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    return PI_ADMM_MI355X


def close(a, b, what, it, scale=1.0):
    np.testing.assert_allclose(a, b, rtol=TOL, atol=TOL * scale, err_msg=f"{what} after outer iteration {it}")


def step_by_iterations(s, orc, t, check_sd=True):
    """Host-step MPC step t on the GPU and compare every iteration with the oracle's."""
    states = []
    rec = orc.mpc_step(on_iter=lambda it, st: states.append(st))
    for it, ost in enumerate(states):
        stop = s.outer_iter(it, t)
        g = s.state()
        close(g["pos_old"], ost["pos_old"], "pos_old", it)
        close(g["hat"], ost["hat"], "hat", it)
        close(g["lam"], ost["lam"], "lam", it)
        if check_sd:
            close(g["S"], ost["S"], "S", it)
            # D = lam_sat - lam_raw with lam_raw = S + K_P e: a difference of O(|S|) quantities, so
            # its absolute error scales with |S| (the integral grows over the step's iterations)
            close(g["D"], ost["D"], "D", it, scale=max(1.0, float(np.max(np.abs(ost["S"])))))
        assert stop == ost["stop"], f"stop flag at outer iteration {it}"
    xt, u = s.step_finish()
    np.testing.assert_allclose(xt, rec.xt, rtol=TOL, atol=TOL)
    np.testing.assert_allclose(u, rec.u, rtol=TOL, atol=TOL)
    return len(states), rec


@pytest.mark.parametrize("preset,term_global,fixed", [("matlab_pi", 0, 0), ("matlab_pi", 1, 0), ("matlab_pi", 1, 1),
                                                      ("casadi_default", 0, 0), ("casadi_default", 1, 1)])
def test_two_vehicle_iterations_match_oracle(Solver, preset, term_global, fixed):
    """The reference's two-vehicle intersection, iteration by iteration, through the steps where
    the vehicles interact (natural termination: 2-4 outer iterations per step from step 13 on;
    fixed: 12 outer iterations every step): PI + anti-windup (matlab_pi: S, D evolve, saturation
    at +-W with back-calculation) and the plain dual update (casadi_default: S = D = 0),
    per-component and global termination scopes."""
    H = 10
    cfg = config.PRESETS[preset](H=H, term_global=term_global, fixed_iters=fixed, max_outer=12 if fixed else 100)
    n_steps = 20 if fixed else 32
    scn = scenario.intersection(H, n_steps=n_steps + 2)
    orc = O.Oracle(cfg, scn)
    n_multi = 0
    saw_sd = False
    with Solver(cfg, scn) as s:
        for t in range(n_steps):
            n, rec = step_by_iterations(s, orc, t)
            n_multi += n > 1
            saw_sd |= bool(np.any(s.state()["S"] != 0.0))
    assert n_multi >= (n_steps if fixed else 15)      # steps with dual updates between iterations
    if preset == "matlab_pi":
        assert saw_sd                                 # the PI integral is exercised


def test_global_pi_iterations_match_oracle(Solver):
    """Global PI with adaptive rho and K_P (casadi_old_PI_ADMM/main.py:128-155, graph kernel):
    lam = S + K_P e, S += K_I e + 2 D, saturation over the pair, iteration by iteration -- through
    step 11, whose loop runs all 100 outer iterations."""
    H = 10
    cfg = config.casadi_old_pi(H=H)
    scn = scenario.intersection(H, n_steps=14)
    orc = O.Oracle(cfg, scn)
    n = []
    with Solver(cfg, scn) as s:
        for t in range(12):
            n.append(step_by_iterations(s, orc, t)[0])
    assert max(n) == cfg.max_outer


@pytest.mark.parametrize("preset,trad", [("matlab_adp_pi", 0), ("matlab_adp_pi", 1), ("casadi_old_pi", 1)])
def test_adaptive_gain_global_pi_iterations_match_oracle(Solver, preset, trad):
    """The adaptive-gain global PI (matlab_adp_pi: ADMM_CVX_two_veh_intesection_adp_PI_antiwindup1.m
    :121-147 -- K_I = 3 / d_min, K_P = min(5 / d_min, 3), the back-calculation added once, saturation
    +-50, hat = lam = 1e-4 at each step's start) and both scripts' trad branch (lam += rho e + D),
    iteration by iteration through the steps where the saturation engages and the loop runs long
    (H = 10: up to 100 outer iterations per step), on the graph kernel."""
    H = 10
    cfg = config.PRESETS[preset](H=H, pi_trad=trad)
    n_steps = 22
    scn = scenario.intersection(H, n_steps=n_steps + 2)
    orc = O.Oracle(cfg, scn)
    n, sat = [], False
    with Solver(cfg, scn) as s:
        for t in range(n_steps):
            n.append(step_by_iterations(s, orc, t, check_sd=not trad)[0])
            sat |= bool(np.any(np.abs(s.state()["lam"]) == cfg.windup_sat))
        rho = s.step_state()["rho_pi"]
    np.testing.assert_allclose(rho, orc.rho_pi, rtol=TOL, atol=TOL)
    assert max(n) >= 20                        # long loops: the PI law's dynamics are exercised
    if preset == "matlab_adp_pi" and not trad:
        assert sat                             # the saturation at +-50 engages


def test_per_component_stop_keeps_stopped_components(Solver):
    """Several components stopping at different iterations (term_global = 0): a component whose
    stop rule fired keeps its state while the others iterate on; the step's stop comes when the
    last one stops.  Fused kernel (tiles) and graph kernel (4-vehicle all-pairs crossings)."""
    H = 12
    cfg = config.matlab_pi(H=H)
    for scn, n_steps in ((scenario.tiled(4, H, n_steps=22, seed=7), 20),
                         (scenario.concat([scenario.crossing(4, H, n_steps=26, seed=k) for k in range(2)]), 24)):
        orc = O.Oracle(cfg, scn)
        ragged = 0
        with Solver(cfg, scn) as s:
            for t in range(n_steps):
                n, rec = step_by_iterations(s, orc, t)
                ragged += len(set(rec.iters.tolist())) > 1     # components stopped at different iterations
        assert ragged > 0


def test_host_stepping_equals_mpc_step(Solver):
    """Stepping a step iteration by iteration and finishing it gives the same trajectory as
    piadmm_mpc_step (the fused single launch), step after step."""
    H = 15
    cfg = config.matlab_pi(H=H)
    scn = scenario.tiled(3, H, n_steps=22, seed=3)
    with Solver(cfg, scn) as a, Solver(cfg, scn) as b:
        for t in range(20):
            ra = a.mpc_step(t)
            it = 0
            while True:
                stop = b.outer_iter(it, t)
                it += 1
                if stop or it == cfg.max_outer:
                    break
            xt, u = b.step_finish()
            np.testing.assert_allclose(xt, ra.xt, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(u, ra.u, rtol=1e-12, atol=1e-12)
            assert it == int(ra.iters.max())


def test_host_stepping_errors_are_loud(Solver):
    H = 10
    cfg = config.matlab_pi(H=H)
    scn = scenario.intersection(H, n_steps=6)
    with Solver(cfg, scn) as s:
        with pytest.raises(_lib.PiadmmError, match="out of order"):
            s.outer_iter(3, 0)
        s.outer_iter(0, 0)
        with pytest.raises(_lib.PiadmmError, match="out of order"):
            s.outer_iter(2, 0)
        with pytest.raises(_lib.PiadmmError, match="host-stepped"):
            s.mpc_step(0)
        s.step_finish()
        with pytest.raises(_lib.PiadmmError, match="no host-stepped"):
            s.step_finish()
        s.mpc_step(1)                                  # a normal step again
