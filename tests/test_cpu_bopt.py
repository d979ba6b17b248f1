"""The B-opt CPU baseline (oracle/piadmm_cpu.cpp, bench.py's cpu_baseline) computes what the
oracle computes: same outer-iteration counts, residual histories, controls and states (1e-8) over
MPC steps where the tile vehicles meet (pair QPs, hinge kinks, PI saturation).  A baseline that
solved an easier problem would not be a baseline."""
import numpy as np
import pytest

from oracle import cpu_bopt
from oracle import piadmm_oracle as O
from piadmm import config, scenario

CASES = [
    ("matlab_pi", 10, {}, 38),
    ("casadi_default", 10, {}, 38),
    ("matlab_pi", 15, {"term_global": 1}, 34),
    ("matlab_pi", 12, {"tighten": 1}, 36),
    ("casadi_default", 8, {"fixed_iters": 1, "max_outer": 20, "term_global": 1}, 40),
]


@pytest.mark.parametrize("preset,H,kw,n_steps", CASES, ids=[f"{p}-H{h}-{'-'.join(k) or 'natural'}" for p, h, k, _ in CASES])
def test_bopt_matches_oracle(preset, H, kw, n_steps):
    cfg = config.PRESETS[preset](H=H, **kw)
    scn = scenario.tiled(3, H, n_steps=n_steps, seed=5)
    r = cpu_bopt.run(cfg, scn, n_steps, threads=2)
    assert r["counters"]["inexact"] == 0
    orc = O.Oracle(cfg, scn)
    for st in range(n_steps):
        ro = orc.mpc_step()
        np.testing.assert_array_equal(ro.iters, r["iters"][st])
        np.testing.assert_allclose(r["u"][st], ro.u, rtol=0, atol=1e-8)
        np.testing.assert_allclose(r["xt"][st], ro.xt, rtol=1e-8, atol=1e-8)
        for k in range(3):
            res = np.array(ro.resid[k], np.float64).reshape(-1, 2)
            mine = r["resid"][st, k]
            np.testing.assert_allclose(mine[:len(res)], res, rtol=1e-8, atol=1e-8)
            assert np.all(np.isnan(mine[len(res):]))
    z_qps = r["counters"]["z_qps"]
    assert z_qps > 0          # the window covers the coupled steps


def test_bopt_threads_do_not_change_results():
    cfg = config.matlab_pi(H=12, term_global=1)
    scn = scenario.tiled(8, 12, n_steps=30, seed=9)
    a = cpu_bopt.run(cfg, scn, 30, threads=1)
    b = cpu_bopt.run(cfg, scn, 30, threads=4)
    for key in ("xt", "u", "iters"):
        np.testing.assert_array_equal(a[key], b[key])
    np.testing.assert_array_equal(np.nan_to_num(a["resid"], nan=-1), np.nan_to_num(b["resid"], nan=-1))


def test_bopt_rejects_what_it_does_not_cover():
    with pytest.raises(ValueError):
        cpu_bopt.run(config.casadi_old_pi(H=5), scenario.tiled(1, 5, n_steps=2), 1)


GRAPH_CASES = [
    ("crossings", "matlab_pi", 12, {}, 24),
    ("crossings", "matlab_pi", 12, {"term_global": 1}, 22),
    ("chains+pair", "casadi_default", 10, {"warm_duals": 1}, 26),
    ("crossings", "matlab_pi", 10, {"warm_duals": 1, "tighten": 1}, 22),
]


def graph_scenario(kind, H, n_steps):
    if kind == "crossings":
        return scenario.concat([scenario.crossing(4, H, n_steps=n_steps + 2, seed=k) for k in range(2)])
    return scenario.concat([scenario.crossing(4, H, n_steps=n_steps + 2, seed=3, pairs="chain"),
                            scenario.tiled(1, H, n_steps=n_steps + 2, seed=4),
                            scenario.crossing(3, H, n_steps=n_steps + 2, seed=5, pairs="chain")])


@pytest.mark.parametrize("kind,preset,H,kw,n_steps", GRAPH_CASES,
                         ids=[f"{k}-{p}-H{h}-{'-'.join(w) or 'natural'}" for k, p, h, w, _ in GRAPH_CASES])
def test_bopt_general_graph_matches_oracle(kind, preset, H, kw, n_steps):
    """Any candidate graph (4-vehicle all-pairs crossings: agents in three pairs each; chains next
    to a tile): the x-step's consensus sum over every candidate neighbour, pairs in index order,
    per-component or global stop -- equal to the oracle, step by step."""
    cfg = config.PRESETS[preset](H=H, **kw)
    scn = graph_scenario(kind, H, n_steps)
    r = cpu_bopt.run(cfg, scn, n_steps, threads=2)
    assert r["counters"]["inexact"] == 0
    orc = O.Oracle(cfg, scn)
    C = orc.n_comp
    assert r["iters"].shape == (n_steps, C)
    for st in range(n_steps):
        ro = orc.mpc_step()
        np.testing.assert_array_equal(ro.iters, r["iters"][st])
        np.testing.assert_allclose(r["u"][st], ro.u, rtol=0, atol=1e-8)
        np.testing.assert_allclose(r["xt"][st], ro.xt, rtol=1e-8, atol=1e-8)
        for k in range(C):
            res = np.array(ro.resid[k], np.float64).reshape(-1, 2)
            mine = r["resid"][st, k]
            np.testing.assert_allclose(mine[:len(res)], res, rtol=1e-8, atol=1e-8)
            assert np.all(np.isnan(mine[len(res):]))
    assert r["counters"]["z_qps"] > 0


@pytest.mark.parametrize("name", ["run_matlab_pi_H40_crossing4", "run_matlab_pi_H40_mixed"])
def test_bopt_matches_wide_working_set_golden_runs(name):
    """Saturated coupled pair QPs at H = 40 (working sets beyond 63 rows: the GPU's wide dual
    active set): B-opt (active sets of any size) equals the oracle's golden run
    (oracle/gen_golden_wide.py) over its 12 steps -- the same fixture the GPU test checks."""
    import os
    from oracle import gen_golden_wide as G
    path = os.path.join(os.path.dirname(__file__), "golden", name + ".npz")
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {path}: run oracle/gen_golden_wide.py")
    g = np.load(path)
    cfg, scn = G.make(name)
    K = int(g["n_steps"])
    r = cpu_bopt.run(cfg, scn, K, threads=2)
    assert r["counters"]["inexact"] == 0
    # every step at full tolerance (round 4's fixture was wrong from the crossing's step 5 on:
    # the oracle's QP solver returned an infeasible pair-QP answer there; oracle/qp_exact.py now
    # certifies every answer, tests/test_oracle.py::test_h40_crossing_step5_pair_qp_certifies)
    for st in range(K):
        np.testing.assert_array_equal(r["iters"][st], g["iters"][st])
        np.testing.assert_allclose(r["u"][st], g["u"][st], rtol=0, atol=1e-8)
        np.testing.assert_allclose(r["xt"][st], g["xt"][st], rtol=1e-8, atol=1e-8)
        for k in range(g["iters"].shape[1]):
            n = int(g["iters"][st][k])
            np.testing.assert_allclose(r["resid"][st, k][:n], g["resid"][st][k][:n], rtol=1e-8, atol=1e-8)


def test_oracle_reproduces_the_wide_golden_run_first_step():
    """The fixture is the oracle's: its first step (saturated pair QPs already) re-derived."""
    import os
    from oracle import gen_golden_wide as G
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", G.NAME + ".npz"))
    res = G.run(G.NAME, n_steps=1)
    np.testing.assert_array_equal(res["iters"][0], g["iters"][0])
    np.testing.assert_allclose(res["xt"][0], g["xt"][0], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(res["u"][0], g["u"][0], rtol=1e-10, atol=1e-10)
