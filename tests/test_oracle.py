"""The oracle (CPU restatement) against the reference's own numerics and golden fixtures.

Pinning chain ("Oracle and parity"):
  * rollouts: bit-exact against the reference's own ``dynamic_update_local`` /
    ``dynamic_update_edge`` numeric branches, executed on seeded inputs
    (tests/golden/ref_rollouts.npz, oracle/gen_ref_rollouts.py);
  * QP solutions: KKT certificates + an independent SciPy solve (the reference's
    OSQP answers do not exist anywhere: parity against reference outputs is unpinned);
  * loop semantics: regression against committed oracle runs + structural
    invariants (tiling, aliasing quirk B4, rounding B6, collision threshold B2).
"""
import ast
import os

import numpy as np
import pytest
from conftest import GOLD

from oracle import piadmm_oracle as O
from oracle import qp_exact
from piadmm import config, scenario


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


# ---------------------------------------------------------------- rollouts vs reference
def test_rollouts_bit_exact_vs_reference():
    d = load("ref_rollouts.npz")
    assert len(d["H"]) >= 10
    for c in range(len(d["H"])):
        H = int(d["H"][c])
        for i in range(2):
            xt, u, s = d["xt"][c][i], d["u"][c][i][:H], d["spd"][c][i]
            x, y, th = O.rollout_linear(xt, u, s, 0.1, 1.0)
            np.testing.assert_array_equal(x, d["loc_x"][c][i][:H + 1])
            np.testing.assert_array_equal(y, d["loc_y"][c][i][:H + 1])
            np.testing.assert_array_equal(th, d["loc_th"][c][i][:H + 1])
            x, y, th = O.rollout_nonlinear(xt, u, s, 0.1, 1.0)
            np.testing.assert_array_equal(x, d["edge_x"][c][i][:H + 1])
            np.testing.assert_array_equal(y, d["edge_y"][c][i][:H + 1])
            np.testing.assert_array_equal(th, d["edge_th"][c][i][:H + 1])


def test_affine_form_matches_reference_linear_rollout():
    """c + M u (the QP's dynamics) equals the reference's linearised rollout."""
    d = load("ref_rollouts.npz")
    for c in range(len(d["H"])):
        H = int(d["H"][c])
        for i in range(2):
            cc, M = O.rollout_affine(d["xt"][c][i], d["spd"][c][i], 0.1, 1.0, H)
            p = cc + M @ d["u"][c][i][:H]
            np.testing.assert_allclose(p[0], d["loc_x"][c][i][:H + 1], rtol=0, atol=1e-11)
            np.testing.assert_allclose(p[1], d["loc_y"][c][i][:H + 1], rtol=0, atol=1e-11)


# ---------------------------------------------------------------- QP solver
def _kkt_ok(P, q, A, l, u, x, y, tol=1e-8):
    st, inf, comp = qp_exact.kkt_residuals(P, q, A, l, u, x, y)
    sc = 1.0 + np.abs(q).max()
    return st <= tol * sc and inf <= tol and comp <= tol * sc


def test_xstep_qp_fixtures():
    d = load("qp_xstep.npz")
    for k in range(len(d["H"])):
        H = int(d["H"][k])
        m = 2 * H - 1
        P, q, A = d["P"][k][:H, :H], d["q"][k][:H], d["A"][k][:m, :H]
        lo, hi = d["l"][k][:m], d["u"][k][:m]
        x, y, _ = qp_exact.solve(P, q, A, lo, hi, np.zeros(H))
        assert _kkt_ok(P, q, A, lo, hi, x, y)
        np.testing.assert_allclose(x, d["x"][k][:H], rtol=0, atol=1e-10)


def test_pair_qp_fixtures():
    d = load("qp_pair.npz")
    H = int(d["H"])
    for k in range(d["P"].shape[0]):
        P, q, A, lo, hi = d["P"][k], d["q"][k], d["A"][k], d["l"][k], d["u"][k]
        x0 = np.zeros(3 * H)
        x0[2 * H:] = np.maximum(0.0, lo[-H:])
        x, y, _ = qp_exact.solve(P, q, A, lo, hi, x0)
        assert _kkt_ok(P, q, A, lo, hi, x, y)
        np.testing.assert_allclose(x[:2 * H], d["x"][k][:2 * H], rtol=0, atol=1e-9)


def test_qp_against_independent_scipy_solver():
    """An independent solver (SciPy SLSQP) agrees with the active-set oracle."""
    opt = pytest.importorskip("scipy.optimize")
    d = load("qp_xstep.npz")
    for k in (0, 4):
        H = int(d["H"][k])
        m = 2 * H - 1
        P, q, A = d["P"][k][:H, :H], d["q"][k][:H], d["A"][k][:m, :H]
        lo, hi = d["l"][k][:m], d["u"][k][:m]
        cons = [{"type": "ineq", "fun": lambda x, A=A, hi=hi: hi - A @ x, "jac": lambda x, A=A: -A},
                {"type": "ineq", "fun": lambda x, A=A, lo=lo: A @ x - lo, "jac": lambda x, A=A: A}]
        r = opt.minimize(lambda x: 0.5 * x @ P @ x + q @ x, np.zeros(H), jac=lambda x: P @ x + q,
                         constraints=cons, method="SLSQP", options={"ftol": 1e-14, "maxiter": 500})
        np.testing.assert_allclose(r.x, d["x"][k][:H], atol=2e-5)


def test_qp_rejects_infeasible_start():
    P = np.eye(2)
    with pytest.raises(qp_exact.QPError):
        qp_exact.solve(P, np.zeros(2), np.eye(2), -np.ones(2), np.ones(2), np.array([5.0, 0.0]))


def test_h40_crossing_step5_pair_qp_certifies():
    """The pair QP on which round 4's solver returned an infeasible, non-KKT answer without raising
    (the H = 40 four-vehicle crossing, step 5, iteration 0: 238 rows, 120 variables in slack form;
    it violated the steering box by 1.75 rad with complementarity 34 -- its ratio test skipped rows
    it judged dependent on the working set).  The null-space active set returns a certified answer:
    every row feasible, stationarity / dual signs / complementarity at 1e-9 relative, a saturated
    working set of 78 rows."""
    d = load("qp_pair_H40_crossing_step5.npz")
    P, q, A, lo, hi, x0 = d["P"], d["q"], d["A"], d["l"], d["u"], d["x0"]
    x, y, W = qp_exact.solve(P, q, A, lo, hi, x0)
    stat, infeas, comp = qp_exact.certify(P, q, A, lo, hi, x, y)
    assert max(stat, infeas, comp) <= 1e-12
    assert np.all(A @ x <= hi + 1e-12) and np.all(A @ x >= lo - 1e-12)
    assert np.max(np.abs(x[:80])) <= np.pi / 6 + 1e-12
    assert len(W) > 63                       # beyond one row per lane: the GPU's wide dual active set
    # the certificate rejects a perturbed answer (it is what solve() applies before returning)
    with pytest.raises(qp_exact.QPError):
        qp_exact.certify(P, q, A, lo, hi, x + 1e-6, y)
    with pytest.raises(qp_exact.QPError):
        qp_exact.certify(P, q, A, lo, hi, x, -y)


# ---------------------------------------------------------------- loop semantics
@pytest.mark.parametrize("name", ["casadi_default_H10", "casadi_default_H15", "matlab_pi_H10", "matlab_pi_H8"])
def test_oracle_runs_reproduce_fixtures(name):
    d = load(f"run_{name}.npz")
    cfg = config.PRESETS[str(d["preset"])](**ast.literal_eval(str(d["cfg_kw"])))   # fixture written by oracle/gen_golden.py
    scn = scenario.Scenario(spd=d["spd"], xt0=d["xt0"], ref=d["ref"], edges=d["edges"], n_steps=d["xt"].shape[0])
    orc = O.Oracle(cfg, scn)
    for s in range(d["xt"].shape[0]):
        r = orc.mpc_step()
        np.testing.assert_allclose(r.xt, d["xt"][s], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(r.u, d["u"][s], rtol=1e-10, atol=1e-10)
        np.testing.assert_array_equal(r.iters, d["iters"][s])


def test_tiles_reduce_to_the_two_vehicle_reference():
    """K unperturbed tiles give K copies of the 2-vehicle run (no coupling across tiles)."""
    cfg = config.matlab_pi(H=10)
    single = O.Oracle(cfg, scenario.intersection(10)).run(20)
    tiles = O.Oracle(cfg, scenario.tiled(3, 10, perturb=False)).run(20)
    for a, b in zip(single, tiles):
        for k in range(3):
            np.testing.assert_array_equal(b.xt[2 * k:2 * k + 2], a.xt)
            np.testing.assert_array_equal(b.iters[k], a.iters[0])


def test_alias_quirk_B4_zeroes_dual_residual_after_first_iteration():
    """casadi/main.py:63,180 aliases last_iter_hat_pos to hat_pos_old: s_k == 0 from iteration 2.

    matlab_pi H=10 keeps the pair active for several outer iterations around steps 28-31.
    """
    cfg = config.matlab_pi(H=10, fixed_iters=1, max_outer=6)
    alias = O.Oracle(cfg.replace(alias_dual_residual=1), scenario.intersection(10)).run(32)
    copy = O.Oracle(cfg, scenario.intersection(10)).run(32)
    active_later = 0
    for ra, rc in zip(alias, copy):
        for it in range(1, 6):
            assert ra.resid[0][it][1] == 0.0
            if rc.resid[0][it][0] > 0.0:          # the pair was active in that iteration
                active_later += 1
                assert rc.resid[0][it][1] > 0.0   # copied history: a real dual residual
    assert active_later > 0


def test_rounding_quirk_B6():
    r = O.Oracle(config.casadi_default(H=10), scenario.intersection(10)).run(3)[-1]
    np.testing.assert_array_equal(np.around(r.u * 1e4), r.u * 1e4)


def test_collision_threshold_quirk_B2():
    """Python compares squared distance with dis_thres (B2); MATLAB with dis_thres^2."""
    assert config.casadi_default().thr_collide == 2.0
    assert config.matlab_pi().thr_collide == 4.0


def test_pi_dual_update_matches_matlab_statement_order():
    """ADMM_CVX_..._PI_antiwindup.m:160-188 written out literally for one pair."""
    rng = np.random.default_rng(5)
    cfg = config.matlab_pi(H=6, windup_sat=1.5)
    H1 = 7
    p1, p2 = rng.normal(0, 2, (2, H1)), rng.normal(0, 2, (2, H1))
    hat = rng.normal(0, 2, (2, 2, H1))
    lam, S, D = rng.normal(0, 1, (2, 2, H1)), rng.normal(0, 1, (2, 2, H1)), rng.normal(0, 0.1, (2, 2, H1))
    dist = np.sqrt(np.sum((p1 - p2) ** 2, axis=0))
    # literal MATLAB
    kP = cfg.theta1 - cfg.theta2 / (1 + np.exp(-np.min(dist)))
    e1, e2 = p1 - hat[0], p2 - hat[1]
    S1 = S[0] + cfg.kI * e1 + D[0]
    S2 = S[1] + cfg.kI * e2 + D[1]
    l1, l2 = S1 + kP * e1, S2 + kP * e2
    exp_lam, exp_D = [], []
    for lv in (l1, l2):
        sat = np.minimum(cfg.windup_sat, np.maximum(lv, -cfg.windup_sat))
        exp_D.append(sat - lv if np.sum(lv != sat) > 0 else np.zeros_like(lv))
        exp_lam.append(sat)
    O.dual_update(cfg, p1, p2, hat, lam, S, D, dist)
    np.testing.assert_array_equal(lam[0], exp_lam[0])
    np.testing.assert_array_equal(lam[1], exp_lam[1])
    np.testing.assert_array_equal(D[0], exp_D[0])
    np.testing.assert_array_equal(D[1], exp_D[1])
    np.testing.assert_array_equal(S[0], S1)


def test_empty_candidate_graph_terminates_after_one_iteration():
    scn = scenario.intersection(10)
    scn.edges = np.zeros((0, 2), np.int32)
    r = O.Oracle(config.casadi_default(H=10), scn).mpc_step()
    assert list(r.iters) == [1, 1]


# ---------------------------------------------------------------------------------------------
# The casadi/main.py loop's own NumPy statements, executed (oracle/gen_ref_mainloop.py):
# the oracle's seeds, collision test, pair hat rollout, plain dual update, residual sums and
# propagation must reproduce them bit for bit.
def _mainloop_cases():
    d = np.load(os.path.join(GOLD, "ref_mainloop.npz"), allow_pickle=False)
    for k in range(int(d["n_cases"])):
        yield {name[len(f"c{k}_"):]: d[name] for name in d.files if name.startswith(f"c{k}_")}


def test_mainloop_statements_bit_exact():
    n = 0
    for c in _mainloop_cases():
        N, H = int(c["N"]), int(c["H"])
        cfg = config.casadi_default(H=H, rho=2.0)
        spd = c["spd"]
        # seeds, casadi/main.py:48-49
        scn = scenario.Scenario(spd=spd, xt0=c["xt"], ref=np.zeros((N, 2, H + 1)),
                                edges=np.zeros((0, 2), np.int32), n_steps=1)
        np.testing.assert_array_equal(O.Oracle(cfg, scn).seeds(), c["seeds"])
        # collision test over all pairs i < j, :110-113 (edge list in np.where order, :121)
        pos = c["pos_old"].reshape(N, 2, H + 1)
        hits = [(i, j) for i in range(N) for j in range(i + 1, N) if O.collides(cfg, pos[i], pos[j], cfg.dis_thres)]
        assert hits == list(zip(c["edge_row"].tolist(), c["edge_col"].tolist()))
        for i in range(N):
            for j in range(i + 1, N):
                assert float(O.collides(cfg, pos[i], pos[j], cfg.dis_thres)) == c["edge_mat"][i, j]
        # hat rollouts (:156-158) and plain dual updates (:161-162), edge by edge
        hat, lam, last = c["hat_in"].copy(), c["dual_in"].copy(), c["last_in"]
        for k, (v1, v2) in enumerate(hits):
            for d, v in enumerate((v1, v2)):
                hx, hy, _ = O.rollout_nonlinear(c["xt"][v], c["uh"][k][d], spd[v], cfg.dt, cfg.L)
                (hat[v1, v2] if d == 0 else hat[v2, v1])[:] = (hx, hy)
            hat_e = np.stack([hat[v1, v2], hat[v2, v1]])
            lam_e = np.stack([lam[v1, v2], lam[v2, v1]])
            O.dual_update(cfg, pos[v1], pos[v2], hat_e, lam_e, np.zeros_like(lam_e), np.zeros_like(lam_e), None)
            lam[v1, v2], lam[v2, v1] = lam_e
        np.testing.assert_array_equal(hat, c["hat_out"])
        np.testing.assert_array_equal(lam, c["dual_out"])
        # residual sums, :165-173 (edge-list order)
        rk = sk = 0.0
        for v1, v2 in hits:
            r, q = O.pair_residuals(cfg, pos[v1], hat[v1, v2], last[v1, v2])
            sk += q
            rk += r
        assert rk == c["error_rk"] and sk == c["error_sk"]
        # propagation, :185-192
        np.testing.assert_array_equal(O.propagate(cfg, c["xt"], c["primal_u"], spd), c["xt_next"])
        n += 1
    assert n == 20


def test_global_pi_law_matches_reference_statements():
    """The global PI law with adaptive rho and K_P and its residuals (oracle
    dual_update_global_pi / pair_residuals_global_pi) against casadi_old_PI_ADMM/main.py:128-155
    executed on seeded inputs over chained iterations (oracle/gen_ref_global_pi.py).  Pinned to
    rounding: the script forms dis_vec as diag(delta' delta) through a BLAS matmul, whose use of
    fused multiply-adds is platform-dependent (1 ulp in d_min, hence in K_P and rho)."""
    d = np.load(os.path.join(GOLD, "ref_global_pi.npz"))
    assert "casadi_old_PI_ADMM/main.py" in str(d["source"])
    n_sat = n_trad = 0
    for k in range(int(d["n_cases"])):
        H = int(d[f"c{k}_H"])
        xt = d[f"c{k}_xt"]
        trad = int(d[f"c{k}_trad"])
        cfg = config.casadi_old_pi(H=H, pi_trad=trad)
        n_trad += trad
        for j in range(int(d[f"c{k}_n"])):
            g = lambda n: d[f"c{k}_i{j}_{n}"]   # noqa: E731
            pos = g("pos_old").reshape(2, 2, H + 1)
            hat = g("hat").reshape(2, 2, H + 1).copy()
            S = g("S_in").reshape(2, 2, H + 1).copy()
            D = g("D_in").reshape(2, 2, H + 1).copy()
            lam = g("lam_in").reshape(2, 2, H + 1).copy()
            rho = np.array([float(g("rho_in"))])
            dchk = O.dual_update_global_pi(cfg, xt, np.array([4.0, 8.0]), g("primal_u"), 0, 1, pos, hat, lam, S, D, rho, 0)
            rk, sk = O.pair_residuals_global_pi(pos[0], pos[1], hat, g("last").reshape(2, 2, H + 1), rho[0])
            tol = dict(rtol=1e-14, atol=1e-14)
            np.testing.assert_allclose(lam.reshape(4, -1), g("dual_out"), **tol)
            np.testing.assert_allclose(S.reshape(4, -1), g("S_out"), **tol)
            np.testing.assert_allclose(D.reshape(4, -1), g("D_out"), **tol)
            np.testing.assert_allclose(rho[0], float(g("rho_out")), **tol)
            np.testing.assert_allclose(dchk, g("dis_vec")[1], **tol)
            np.testing.assert_allclose([rk, sk], [float(g("error_rk")), float(g("error_sk"))], **tol)
            n_sat += int(np.any(g("D_out") != 0))
    assert n_sat > 0          # the back-calculation branch is exercised
    assert n_trad > 0         # and the trad branch (lam += rho e + D)


@pytest.mark.parametrize("trad", [0, 1])
def test_adaptive_gain_law_equals_the_matlab_statements(trad):
    """The adaptive-gain global PI (matlab_adp_pi) against a line-by-line NumPy transliteration of
    ADMM_CVX_two_veh_intesection_adp_PI_antiwindup1.m:121-152 (MATLAB is absent: parity with the
    script's own execution is unpinned; this pins the oracle to its statements): K_I = 3 / dis_min,
    K_P = min(5 / dis_min, 3), rho = max(1, min(5, 4 / dis_min)), lam = sum_err + K_P e and
    sum_err += K_I e + diff_val (diff_val ONCE), or lam += rho e + diff_val (trad); saturation +-50
    with diff_val over the whole array; residuals over both vehicles, no factor 2."""
    rng = np.random.default_rng(7 + trad)
    H = 10
    cfg = config.matlab_adp_pi(H=H, pi_trad=trad)
    spd = np.array([4.0, 8.0])
    xt = np.array([[-10.0, 0.0, 0.0], [0.0, 20.0, -np.pi / 2]]) + rng.uniform(-1, 1, (2, 3)) * [4, 4, 0.2]
    # the script's state (2 vehicles: 4 x (H+1) arrays), carried over chained iterations
    sum_err, diff_val, rho_m = 0.0, 0.0, 1.0
    dual = 1e-4 * np.ones((4, H + 1))
    last = 1e-4 * np.ones((4, H + 1))
    # the oracle's pair state
    lam, S, D = dual.reshape(2, 2, H + 1).copy(), np.zeros((2, 2, H + 1)), np.zeros((2, 2, H + 1))
    rho = np.array([1.0])
    n_sat = 0
    for it in range(8):
        primal_u = np.round(rng.uniform(-np.pi / 6, np.pi / 6, size=(2, H)), 4)
        pos_old = rng.normal(0, 3, size=(4, H + 1))
        hat = pos_old + rng.normal(0, 6 if it % 2 else 25, size=(4, H + 1))
        # --- the MATLAB statements, :121-152
        xs, ys = zip(*[O.rollout_nonlinear(xt[v], primal_u[v], spd[v], 0.1, 1.0)[:2] for v in range(2)])
        pos_veh1, pos_veh2 = np.vstack((xs[0], ys[0])), np.vstack((xs[1], ys[1]))
        dis_vec = np.sqrt(np.diag((pos_veh1 - pos_veh2).T @ (pos_veh1 - pos_veh2)))
        dis_min = np.min(dis_vec)
        K_I = 3 / dis_min
        K_P = min(5 / dis_min, 3)
        rho_m = max(1, min(5, 4 / dis_min))
        if trad == 1:
            dual = dual + rho_m * (pos_old - hat) + diff_val
        else:
            dual = sum_err + K_P * (pos_old - hat)
            sum_err = sum_err + K_I * (pos_old - hat) + diff_val
        ori = dual
        dual = np.minimum(50, np.maximum(dual, -50))
        diff_val = (dual - ori) if np.sum(ori != dual) > 0 else 0
        error_sk = np.sqrt(np.sum((rho_m * (last - hat)) ** 2))
        error_rk = np.sqrt(np.sum((pos_old - hat) ** 2))
        # --- the oracle
        p3, h3 = pos_old.reshape(2, 2, H + 1), hat.reshape(2, 2, H + 1).copy()
        dchk = O.dual_update_global_pi(cfg, xt, spd, primal_u, 0, 1, p3, h3, lam, S, D, rho, 0)
        rk, sk = O.pair_residuals_global_pi(p3[0], p3[1], h3, last.reshape(2, 2, H + 1), rho[0])
        tol = dict(rtol=1e-13, atol=1e-12)
        np.testing.assert_allclose(lam.reshape(4, -1), dual, **tol)
        np.testing.assert_allclose(D.reshape(4, -1), np.broadcast_to(diff_val, (4, H + 1)), **tol)
        if trad == 0:
            np.testing.assert_allclose(S.reshape(4, -1), np.broadcast_to(sum_err, (4, H + 1)), **tol)
        np.testing.assert_allclose(rho[0], rho_m, **tol)
        np.testing.assert_allclose(dchk, dis_vec[1], **tol)
        np.testing.assert_allclose([rk, sk], [error_rk, error_sk], **tol)
        n_sat += int(np.any(np.broadcast_to(diff_val, (4, H + 1)) != 0))
        last = hat.copy()
    assert n_sat > 0
