"""The OBCA local subproblem oracle (oracle/obca_oracle.py) and the host-side record/bar_state
helpers (piadmm/obca.py), on CPU.

Pinned by executing the reference (tests/golden/ref_obca.npz, oracle/gen_ref_obca.py):
VehicleConfig + ref_traj_gen (veh_config.py:7-47), mid_state (optimizer.py:351-373),
iterate_next_state (optimizer.py:337-344).  The halfspace closed forms are held to the vertex
construction of util.py:12-68 and to compute_square_halfspaces_ca_prob (util.py:70-101), both
restated here from the reference's formulas (CasADi absent, so not executed).  The NLP's
derivatives are checked by finite differences, and the SQP's answers are certified as KKT points
of the NLP as written (optimizer.py:84-168).  Agreement with IPOPT itself is UNPINNED.
"""
import math
import os

import numpy as np
import pytest

from oracle import obca_oracle as O
from piadmm import obca

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_obca.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


def test_vehicle_config_and_references_match_the_reference(gold):
    cfg = gold["cfg"]
    assert (O.LENGTH, O.WIDTH, O.LF, O.LR, O.MAX_STEER, O.DT, O.T_PERIOD, O.MAX_ACC, O.MAX_V, O.MAX_STEER_RATE,
            O.AVG_DELAY, O.VAR_DELAY, O.DELAY_PROB) == tuple(cfg)
    for a, b in ((O.ref_traj_gen(), obca.ref_traj_gen()),):
        for v in range(2):
            np.testing.assert_array_equal(a[v], gold[f"ref{v}"])
            np.testing.assert_array_equal(b[v], gold[f"ref{v}"])


def test_mid_state_and_iterate_next_state_match_the_reference(gold):
    bar = obca.create_bar_state()
    for k in ("Z_bar", "A", "b", "lamb_bar", "lamb_ij", "local_x"):
        np.testing.assert_array_equal(bar[k], gold["mid_" + k])
    np.testing.assert_array_equal(O.mid_state_lamb_ij(), gold["mid_lamb_ij"])
    inp = {k: gold["in_" + k] for k in ("Z_bar", "A", "b", "lamb_bar", "lamb_ij", "local_x")}
    for f in (obca.iterate_next_state, O.iterate_next_state):
        out = f(inp)
        for k in inp:
            np.testing.assert_array_equal(out[k], gold["out_" + k])


def _vertices(st):
    """generate_vehicle_vertices (util.py:12-46, base_link=False), restated."""
    x, y, h = st[0], st[1], st[3]
    L, W = O.LENGTH, O.WIDTH
    vx = [x + L / 2 * math.cos(h) - W / 2 * math.sin(h), x + L / 2 * math.cos(h) + W / 2 * math.sin(h),
          x - L / 2 * math.cos(h) + W / 2 * math.sin(h), x - L / 2 * math.cos(h) - W / 2 * math.sin(h)]
    vy = [y + L / 2 * math.sin(h) + W / 2 * math.cos(h), y + L / 2 * math.sin(h) - W / 2 * math.cos(h),
          y - L / 2 * math.sin(h) - W / 2 * math.cos(h), y - L / 2 * math.sin(h) + W / 2 * math.cos(h)]
    return np.vstack((vx, vy)).T


def _halfspaces_from_vertices(P):
    """compute_square_halfspaces_ca (util.py:48-68), restated."""
    A, b = [], []
    for i in range(4):
        p1, p2 = P[i], P[(i + 1) % 4]
        a = np.array([p1[1] - p2[1], p2[0] - p1[0]])
        nrm = math.hypot(p2[1] - p1[1], p1[0] - p2[0])
        A.append(a / nrm)
        b.append((p2[0] * p1[1] - p2[1] * p1[0]) / nrm)
    return np.array(A), np.array(b)


def _halfspaces_prob(st):
    """compute_square_halfspaces_ca_prob (util.py:70-101), restated (prob = VehicleConfig.prob)."""
    x, y, v, h = st[0], st[1], st[2], st[3]
    d_avg = np.array([O.AVG_DELAY * v * math.cos(h), O.AVG_DELAY * v * math.sin(h)])
    d_var = np.array([(O.VAR_DELAY * v * math.cos(h)) ** 2, (O.VAR_DELAY * v * math.sin(h)) ** 2])
    R = np.array([[math.cos(h), -math.sin(h)], [math.sin(h), math.cos(h)]])
    A = np.vstack([R.T, -R.T])
    b0 = np.array([O.LENGTH / 2, O.WIDTH / 2, O.LENGTH / 2, O.WIDTH / 2])
    return A, b0 + A @ (np.array([x, y]) + d_avg + math.sqrt(O.DELAY_PROB / (1 - O.DELAY_PROB)) * d_var)


@pytest.mark.parametrize("seed", range(5))
def test_halfspace_closed_forms_equal_the_reference_constructions(seed):
    rng = np.random.default_rng(seed)
    st = np.array([rng.uniform(0, 100), rng.uniform(-5, 5), rng.uniform(0, 20), rng.uniform(-3, 3), 0.1])
    A0, b0 = _halfspaces_from_vertices(_vertices(st))
    for f in (O.halfspaces, obca.halfspaces):
        A, b = f(st, 0)
        np.testing.assert_allclose(A, A0, rtol=0, atol=1e-13)
        np.testing.assert_allclose(b, b0, rtol=1e-13, atol=1e-12)
        A, b = f(st, 1)
        Ap, bp = _halfspaces_prob(st)
        np.testing.assert_allclose(A, Ap, rtol=0, atol=1e-15)
        np.testing.assert_allclose(b, bp, rtol=1e-14, atol=1e-13)


def _fd(fun, x0, h=1e-6):
    v, g, H = fun(x0)
    G = np.zeros_like(g)
    HH = np.zeros_like(H)
    for i in range(len(x0)):
        e = np.zeros_like(x0)
        e[i] = h
        vp, gp, _ = fun(x0 + e)
        vm, gm, _ = fun(x0 - e)
        G[..., i] = (vp - vm) / (2 * h)
        HH[..., i] = (gp - gm) / (2 * h)
    return np.abs(G - g).max(), np.abs(HH - H).max()


@pytest.mark.parametrize("prob", [1, 0])
def test_constraint_and_dynamics_derivatives(prob):
    rng = np.random.default_rng(3 + prob)
    for _ in range(3):
        X = np.array([rng.uniform(0, 50), rng.uniform(-3, 3), rng.uniform(1, 20), rng.uniform(-1, 1),
                      rng.uniform(-0.5, 0.5)])
        Lt = rng.uniform(0, 1.5, 4)
        ct, wt = rng.normal(), rng.normal(size=2)
        e1, e2 = _fd(lambda z: O.ga_eval(z[:5], z[5:], ct, prob), np.concatenate([X, Lt]))
        assert e1 < 1e-7 and e2 < 1e-7
        e1, e2 = _fd(lambda z: O.gb_eval(z[:5], z[5:], wt, prob), np.concatenate([X, Lt]))
        assert e1 < 1e-7 and e2 < 1e-7
        A, b = O.halfspaces(X, prob)
        assert abs(O.ga_eval(X, Lt, ct, prob)[0] - (-(b @ Lt) - ct)) < 1e-12
        np.testing.assert_allclose(O.gb_eval(X, Lt, wt, prob)[0], A.T @ Lt + wt, atol=1e-14)
        U = rng.normal(size=2)
        e1, e2 = _fd(lambda z: (lambda r: (r[0], r[1], r[3] * O.DT))(O.dyn_eval(z, U)), X)
        assert e1 < 1e-7 and e2 < 1e-7


def test_record_layout_round_trip():
    rec = obca.overtaking_problem(9, 1, "perturbed", prob=0, seed=3)
    assert rec.shape == (obca.REC,) == (296,)
    d = obca.unpack(rec)
    rec2 = obca.pack(d["init"], d["ref"], d["A_o"], d["b_o"], d["lamb_ij_o"], d["lamb_bar"], d["Z_bar"], rho=d["rho"],
                     min_dis=d["min_dis"], max_x=d["max_x"], max_y=d["max_y"], r=d["r"], q=d["q"], prob=d["prob"],
                     max_iter=d["max_iter"])
    np.testing.assert_array_equal(rec, rec2)
    # the record local_record builds reads the OTHER vehicle's A, b, lamb_ij and this one's lamb_bar, Z_bar
    bar = obca.create_bar_state()
    rng = np.random.default_rng(0)
    for k in bar:
        bar[k] = rng.standard_normal(bar[k].shape)
    refs = obca.ref_traj_gen()
    d = obca.unpack(obca.local_record(bar, 0, 4, refs[0][4], refs))
    np.testing.assert_array_equal(d["A_o"], bar["A"][1])
    np.testing.assert_array_equal(d["lamb_ij_o"], bar["lamb_ij"][1])
    np.testing.assert_array_equal(d["Z_bar"], bar["Z_bar"][0])
    np.testing.assert_array_equal(d["ref"], refs[0][4:12])


def test_bar_state_update_exchanges_halfspaces():
    bar = obca.create_bar_state()
    refs = obca.ref_traj_gen()
    full = [np.concatenate([refs[v][1:8], np.ones((7, 4))], axis=1) for v in range(2)]
    out = obca.bar_state_update(bar, full, prob=1)
    for v in range(2):
        for t in range(7):
            A, b = O.halfspaces(refs[v][1 + t], 1)
            np.testing.assert_array_equal(out["A"][v, t], A)
            np.testing.assert_array_equal(out["b"][v, t], b)
    np.testing.assert_array_equal(out["lamb_ij"], bar["lamb_ij"])    # never updated (optimizer.py:220)


def _kkt(p, r):
    return O.kkt_residual(p, r.X, r.U, r.Lam, r.y_a, r.y_b, r.y_n, r.y_x, r.pi, r.y_u, r.y_l)


@pytest.mark.parametrize("t_step,veh,variant", [(0, 0, "initial"), (8, 0, "initial"), (12, 0, "consensus"),
                                                (14, 1, "perturbed"), (16, 0, "perturbed"), (33, 0, "initial")])
def test_sqp_converges_to_a_kkt_point_of_the_nlp(t_step, veh, variant):
    p, opt = O.from_record(obca.overtaking_problem(t_step, veh, variant))
    r = O.solve_local(p, opt)
    assert r.status == O.CONVERGED and r.iters <= 12
    k = _kkt(p, r)
    gscale = 1.0 + 2 * p.q * np.abs(r.X[1:] - p.ref[1:]).max()
    assert k["stat_x"] <= 1e-10 * gscale and k["stat_l"] <= 1e-10 * gscale and k["stat_u"] <= 1e-10 * gscale, k
    assert k["feas"] <= 1e-9 and k["comp"] <= 1e-9, k


def test_collision_constraint_binds_in_the_overtaking_window():
    """Between t_step 8 and 18 vehicle 0 is held off vehicle 1 by (5a): positive multipliers."""
    active = 0
    for ts in (8, 10, 12, 14, 16, 18):
        p, opt = O.from_record(obca.overtaking_problem(ts, 0, "initial"))
        r = O.solve_local(p, opt)
        assert r.status == O.CONVERGED
        active += int(np.any(r.y_a > 1.0))
    assert active >= 5


def test_reference_as_written_first_iterate_is_infeasible():
    """With the reference's initial bar_state (mid_state: A = b = 0), (5b) forces A(X_t)' Lambda_t = 0
    and (5a) reads -b0' Lambda >= min_dis > 0 with Lambda >= 0 -- infeasible for both vehicles."""
    for veh in (0, 1):
        p, opt = O.from_record(obca.as_written_problem(0, veh))
        r = O.solve_local(p, opt)
        assert r.status == O.QP_INFEASIBLE and r.iters == 1


def test_gi_qp_matches_a_reference_qp_solution():
    """The dense dual active set QP against scipy's SLSQP on random strictly convex QPs."""
    from scipy.optimize import minimize
    rng = np.random.default_rng(11)
    for _ in range(5):
        n, m = 8, 12
        Q = rng.normal(size=(n, n))
        H = Q @ Q.T + n * np.eye(n)
        g = rng.normal(size=n)
        C = rng.normal(size=(m, n))
        d = rng.normal(size=m) - 1.0
        x, _, u, st, _ = O.gi_qp(H, g, np.zeros((0, n)), np.zeros(0), C, d)
        assert st == 0
        res = minimize(lambda z: 0.5 * z @ H @ z + g @ z, np.zeros(n), jac=lambda z: H @ z + g,
                       constraints=[{"type": "ineq", "fun": lambda z: C @ z - d, "jac": lambda z: C}],
                       method="SLSQP", options={"ftol": 1e-14, "maxiter": 500})
        np.testing.assert_allclose(x, res.x, atol=1e-6)
        np.testing.assert_allclose(H @ x + g, C.T @ u, atol=1e-10)
        assert np.all(u >= 0) and np.all(C @ x - d >= -1e-10)
        assert np.abs(u * (C @ x - d)).max() < 1e-10
