"""GPU parity of the OBCA local subproblem: the batched SQP of
csrc/piadmm_obca.hip through the C-ABI (piadmm_obca_solve) against oracle/obca_oracle.py on the
two-vehicle overtaking scenario (decentralized_overtaking_ADMM.py:22-42; every MPC step 0..41,
both vehicles, three bar_state variants, both halfspace models).

Bar: same status; for converged problems X, U, Lambda within ATOL = 1e-7 (rel. 1e-9 of the state
scale) and the cost within RTOL = 1e-9; and the GPU answer, with the GPU's multipliers, is a KKT
point of the reference's NLP (optimizer.py:84-168) -- stationarity <= 1e-9 of the gradient
scale, feasibility and complementarity <= 1e-8.  Agreement with IPOPT is unpinned (CasADi absent).
"""
import numpy as np
import pytest

from oracle import obca_oracle as O
from piadmm import _lib, obca

pytestmark = pytest.mark.gpu

ATOL = 1e-7


@pytest.fixture(scope="module")
def batch():
    from piadmm.solver import device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    b = obca.OBCABatch(0)
    yield b
    b.close()


def _oracle(recs):
    out = []
    for rec in recs:
        p, opt = O.from_record(rec)
        out.append((p, O.solve_local(p, opt)))
    return out


def _check(recs, res, orc, kkt=True):
    n_conv = 0
    for k, (p, r) in enumerate(orc):
        assert res.status[k] == r.status, (k, res.status[k], r.status)
        if r.status != O.CONVERGED:
            continue
        n_conv += 1
        assert abs(int(res.iters[k]) - r.iters) <= 1, (k, res.iters[k], r.iters)
        np.testing.assert_allclose(res.X[k], r.X, rtol=1e-9, atol=ATOL, err_msg=f"X {k}")
        np.testing.assert_allclose(res.U[k], r.U, rtol=1e-9, atol=ATOL, err_msg=f"U {k}")
        np.testing.assert_allclose(res.Lam[k], r.Lam, rtol=1e-9, atol=ATOL, err_msg=f"Lambda {k}")
        assert abs(res.cost[k] - r.cost) <= 1e-9 * max(1.0, abs(r.cost)), (k, res.cost[k], r.cost)
        if kkt:
            kk = O.kkt_residual(p, res.X[k], res.U[k], res.Lam[k], res.y_a[k], res.y_b[k], res.y_n[k], res.y_x[k],
                                res.pi[k], res.y_u[k], res.y_l[k])
            gscale = 1.0 + 2 * p.q * np.abs(res.X[k][1:] - p.ref[1:]).max()
            assert max(kk["stat_x"], kk["stat_u"], kk["stat_l"]) <= 1e-9 * gscale, (k, kk)
            assert kk["feas"] <= 1e-8 and kk["comp"] <= 1e-8, (k, kk)
    return n_conv


@pytest.mark.parametrize("prob", [1, 0])
def test_gpu_equals_oracle_on_the_overtaking_scenario(batch, prob):
    recs = np.stack([obca.overtaking_problem(ts, v, var, prob=prob)
                     for ts in range(0, 42, 1 if prob else 3) for v in (0, 1)
                     for var in ("initial", "consensus", "perturbed")])
    res = batch.solve(recs)
    orc = _oracle(recs)
    n_conv = _check(recs, res, orc)
    assert n_conv >= 0.95 * len(recs)
    # the window where (5a) binds is covered
    assert np.sum(np.max(res.y_a, axis=1) > 1.0) >= 10


def test_reference_as_written_is_reported_infeasible(batch):
    recs = np.stack([obca.as_written_problem(ts, v) for ts in (0, 5) for v in (0, 1)])
    res = batch.solve(recs)
    assert np.all(res.status == obca_status("qp_infeasible"))
    assert np.all(res.iters == 1)


def obca_status(name):
    return {v: k for k, v in obca.STATUS.items()}[name]


def test_resident_batch_and_timing_equal_one_shot_solve(batch):
    recs = obca.scenario_batch(300, seed=2)
    a = batch.solve(recs)
    batch.upload(recs)
    ms = batch.time(3)
    assert ms > 0
    b = batch.download(len(recs))
    np.testing.assert_array_equal(a.raw, b.raw)
    np.testing.assert_array_equal(a.status, b.status)


def test_errors_are_reported_before_any_launch(batch):
    rec = obca.overtaking_problem(3, 0)
    bad = rec.copy()
    bad[283 + 6] = 2.0          # prob must be 0 / 1
    with pytest.raises(_lib.PiadmmError, match="bad parameters"):
        batch.solve(bad[None])
    bad = rec.copy()
    bad[283 + 7] = 0.0          # max_iter >= 1
    with pytest.raises(_lib.PiadmmError):
        batch.solve(bad[None])
    # the handle still works
    r = batch.solve(rec[None])
    assert r.status[0] == 0
