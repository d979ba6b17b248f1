"""The OBCA CPU baseline (oracle/obca_cpu.cpp, bench.py --obca cpu_baseline) computes what the
NumPy oracle computes: same status and iteration count, X / U / Lambda within 1e-8, on the
overtaking scenario set.  A baseline that solved an easier problem would not be a baseline."""
import numpy as np
import pytest

from oracle import obca_cpu
from oracle import obca_oracle as O
from piadmm import obca


@pytest.mark.parametrize("prob", [1, 0])
def test_cpu_baseline_equals_the_oracle(prob):
    recs = np.stack([obca.overtaking_problem(ts, v, var, prob=prob) for ts in range(0, 42, 4) for v in (0, 1)
                     for var in ("initial", "perturbed")])
    out, ist, _ = obca_cpu.solve(recs, threads=2)
    res = obca.OBCAResult(out, ist)
    for k, rec in enumerate(recs):
        p, opt = O.from_record(rec)
        r = O.solve_local(p, opt)
        assert res.status[k] == r.status and abs(int(res.iters[k]) - r.iters) <= 1, (k, res.status[k], r.status)
        if r.status == O.CONVERGED:
            np.testing.assert_allclose(res.X[k], r.X, rtol=1e-9, atol=1e-8)
            np.testing.assert_allclose(res.U[k], r.U, rtol=1e-9, atol=1e-8)
            np.testing.assert_allclose(res.Lam[k], r.Lam, rtol=1e-9, atol=1e-8)


def test_cpu_baseline_threads_do_not_change_results():
    recs = obca.scenario_batch(64, seed=1)
    a, ia, _ = obca_cpu.solve(recs, threads=1)
    b, ib, _ = obca_cpu.solve(recs, threads=4)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(ia, ib)
