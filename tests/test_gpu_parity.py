"""GPU parity: libpiadmm (HIP, gfx950) through the C-ABI vs the oracle and the golden fixtures.

Tolerance: the north-star contract is 1e-5 relative on states and controls.  Both
sides compute exact QP minimisers in fp64 (the GPU certifies each polished
solution by KKT), so these tests hold a tighter RTOL = 1e-8 and require the
discrete outcomes (outer-iteration counts, collision flags) to be identical.
At BASELINE sizes (256 and 1024 agents) parity is checked on sampled tiles
against the live oracle plus size-independent properties (tile independence,
permutation equivariance, certified solves).
"""
import ast
import os

import numpy as np
import pytest
from conftest import GOLD

from oracle import piadmm_oracle as O
from piadmm import _lib, config, scenario

pytestmark = pytest.mark.gpu

RTOL = 1e-8            # held (contract: 1e-5)
ATOL = 1e-8


@pytest.fixture(scope="module")
def Solver():
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    return PI_ADMM_MI355X


def close(a, b, rtol=RTOL, atol=ATOL):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def fixture_run(name):
    d = np.load(os.path.join(GOLD, f"run_{name}.npz"), allow_pickle=False)
    cfg = config.PRESETS[str(d["preset"])](**ast.literal_eval(str(d["cfg_kw"])))   # written by oracle/gen_golden.py
    scn = scenario.Scenario(spd=d["spd"], xt0=d["xt0"], ref=d["ref"], edges=d["edges"], n_steps=d["xt"].shape[0])
    return d, cfg, scn


@pytest.mark.parametrize("name", ["casadi_default_H10", "casadi_default_H15", "matlab_pi_H10", "matlab_pi_H8",
                                  "matlab_pi_H30_tiled3", "matlab_pi_H20_tiled2_fixed12"])
def test_gpu_matches_golden_runs(Solver, name):
    d, cfg, scn = fixture_run(name)
    with Solver(cfg, scn) as s:
        for k in range(d["xt"].shape[0]):
            r = s.mpc_step()
            np.testing.assert_array_equal(r.status, 0)
            np.testing.assert_array_equal(r.iters, d["iters"][k])
            close(r.xt, d["xt"][k])
            close(r.u, d["u"][k])
            n_it = int(d["iters"][k][0])
            close(np.nan_to_num(r.resid[0, :n_it]), np.nan_to_num(d["resid"][k, 0, :n_it]), rtol=1e-7, atol=1e-7)


def test_gpu_state_matches_oracle(Solver):
    """pos_old, hat, lam and the collision flag of the last iteration (piadmm_get_state)."""
    cfg = config.matlab_pi(H=12)
    scn = scenario.tiled(2, 12, n_steps=30, seed=4)
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s:
        for _ in range(24):
            ro = orc.mpc_step()
            s.mpc_step()
        st = s.state()
    close(st["pos_old"], ro.pos_old)
    close(st["hat"], ro.hat)
    close(st["lam"], ro.lam)
    np.testing.assert_array_equal(st["edge_active"].astype(bool), ro.edge_active)
    np.testing.assert_array_equal(st["iters"], ro.iters)


@pytest.mark.parametrize("H", [3, 5, 32, 33, 40, 41, 50])
def test_horizon_limits_match_oracle(Solver, H):
    """H <= 32: every matrix of a component in LDS; H > 32 ("big mode"): the agent and pair
    K_s^-1, G and X' in HBM / L2, the pair's K built in place with two columns per lane.  Odd H in
    big mode (33, 41): xrows(H) is odd, so the agent waves' LDS regions are rounded to even counts
    (piadmm_internal.h xreg) for the 16-byte row passes over S^-1."""
    cfg = config.matlab_pi(H=H)
    n = 12 if H <= 32 else 3          # the oracle's dense active set is slow at H > 32
    scn = scenario.tiled(2, H, n_steps=12, seed=H)
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s:
        for _ in range(n):
            ro, rg = orc.mpc_step(), s.mpc_step()
            np.testing.assert_array_equal(rg.status, 0)
            np.testing.assert_array_equal(rg.iters, ro.iters)
            close(rg.xt, ro.xt)
            close(rg.u, ro.u)


def test_largest_horizon_against_the_oracle(Solver):
    """H = 63 (the lane limit) against the oracle's golden run (oracle/gen_golden_wide.py
    run_matlab_pi_H63_tiled2: two seeded intersection tiles, 8 MPC steps, every oracle QP
    certified -- pair QPs of 189 variables in slack form, which round 4's oracle solver could
    not finish): states and controls at 1e-8, iteration counts and residual histories equal,
    every GPU QP certified, the plans inside the steering box and rate limits."""
    from oracle import gen_golden_wide as G
    g = np.load(os.path.join(GOLD, G.H63 + ".npz"))
    cfg, scn = G.make(G.H63)
    with Solver(cfg, scn) as s:
        for k in range(int(g["n_steps"])):
            r = s.mpc_step()
            np.testing.assert_array_equal(r.status, 0, err_msg=f"step {k}")
            np.testing.assert_array_equal(r.iters, g["iters"][k], err_msg=f"step {k}")
            close(r.xt, g["xt"][k])
            close(r.u, g["u"][k])
            for c in range(s.C):
                n = int(g["iters"][k][c])
                close(r.resid[c, :n], g["resid"][k][c][:n])
            assert np.all(np.abs(r.u) <= cfg.u_max + 1e-9)
            assert np.all(np.abs(np.diff(r.u, axis=1)) <= cfg.du_max + 1e-9)


def test_largest_horizon_tile_independent(Solver):
    """H = 63: two identical tiles stay bit-identical over 8 steps."""
    H = 63
    cfg = config.matlab_pi(H=H)
    scn = scenario.tiled(2, H, n_steps=12, perturb=False)
    with Solver(cfg, scn) as s:
        for _ in range(8):
            r = s.mpc_step()
            np.testing.assert_array_equal(r.status, 0)
            np.testing.assert_array_equal(r.xt[0:2], r.xt[2:4])
            np.testing.assert_array_equal(r.u[0:2], r.u[2:4])


def test_isolated_agents_and_pairs_mixed(Solver):
    """Components of one agent (no candidate pair) next to pairs; ragged component sizes."""
    base = scenario.tiled(3, 10, n_steps=20, seed=1)
    spd = np.concatenate([base.spd, [6.0]])
    xt0 = np.concatenate([base.xt0, [[3.0, -4.0, 0.3]]])
    ref = np.concatenate([base.ref, base.ref[:1]])
    edges = np.array([[0, 1], [4, 5]], np.int32)        # agents 2, 3 and 6 are alone
    scn = scenario.Scenario(spd=spd, xt0=xt0, ref=ref, edges=edges, n_steps=20)
    cfg = config.casadi_default(H=10)
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s:
        assert s.C == 5
        for _ in range(20):
            ro, rg = orc.mpc_step(), s.mpc_step()
            np.testing.assert_array_equal(rg.iters, ro.iters)
            close(rg.xt, ro.xt)


def test_bench_workload_sampled_tiles_match_oracle(Solver):
    """256 agents x H30 (the bench size): three sampled tiles against the live oracle."""
    cfg = config.matlab_pi(H=30)
    scn = scenario.tiled(128, 30, n_steps=4)
    orc = O.Oracle(cfg, scn)
    comps = [0, 57, 127]
    with Solver(cfg, scn) as s:
        for _ in range(3):
            ro = orc.mpc_step(components=comps)
            rg = s.mpc_step()
            np.testing.assert_array_equal(rg.status, 0)
            for c in comps:
                sl = slice(2 * c, 2 * c + 2)
                assert rg.iters[c] == ro.iters[c]
                close(rg.xt[sl], ro.xt[sl])
                close(rg.u[sl], ro.u[sl])


def test_degenerate_xstep_working_sets(Solver):
    """Bench tiles with hard QPs (oracle/gen_golden.py DEGENERATE): x-step QPs whose optimal
    working set is linearly dependent (two box rows and the three rate rows between them,
    one zero multiplier) -- the polish drops the dependent row and the one-step label update
    releases a wrong-signed row instead of flipping it -- and pair QPs with the hinge at its
    kink over the whole horizon (ADMM without the adaptive penalty).  All certified."""
    d = np.load(os.path.join(GOLD, "degenerate_xstep.npz"), allow_pickle=False)
    cfg = config.matlab_pi(H=30, fixed_iters=1, max_outer=int(d["outer"]))
    for k in range(len(d["tile"])):
        scn = scenario.Scenario(spd=d["spd"][k], xt0=d["xt0"][k], ref=d["ref"][k],
                                edges=np.array([[0, 1]], np.int32), n_steps=40)
        with Solver(cfg, scn) as s:
            s.set_xt(d["xt_t"][k])
            s.reset_counters()
            r = s.mpc_step(t=int(d["t"][k]))
            np.testing.assert_array_equal(r.status, 0)
            assert s.counters()["inexact"] == 0
            close(r.xt, d["xt_next"][k])
            close(r.u, d["u"][k])


def test_tiles_are_independent_at_1024_agents(Solver):
    """1024 agents x H30 (configs[3] size): identical tiles give bit-identical results,
    equal to the 2-vehicle run; every QP of the step is certified (status 0)."""
    cfg = config.matlab_pi(H=30, fixed_iters=1, max_outer=20)
    with Solver(cfg, scenario.tiled(512, 30, n_steps=3, perturb=False)) as s:
        rs = [s.mpc_step() for _ in range(3)]
    with Solver(cfg, scenario.intersection(30, n_steps=3)) as s1:
        r1 = [s1.mpc_step() for _ in range(3)]
    for a, b in zip(rs, r1):
        np.testing.assert_array_equal(a.status, 0)
        xt = a.xt.reshape(512, 2, 3)
        assert (xt == xt[0]).all()
        np.testing.assert_array_equal(xt[0], b.xt)
        np.testing.assert_array_equal(a.u.reshape(512, 2, -1)[7], b.u)


def test_permutation_equivariance_at_256_agents(Solver):
    """Reordering tiles reorders the results and nothing else."""
    cfg = config.matlab_pi(H=30, fixed_iters=1, max_outer=10)
    scn = scenario.tiled(128, 30, n_steps=2, seed=9)
    perm = np.random.default_rng(0).permutation(128)
    idx = np.stack([2 * perm, 2 * perm + 1], 1).reshape(-1)
    scn_p = scenario.Scenario(spd=scn.spd[idx], xt0=scn.xt0[idx], ref=scn.ref[idx], edges=scn.edges, n_steps=2)
    with Solver(cfg, scn) as s, Solver(cfg, scn_p) as sp:
        for _ in range(2):
            a, b = s.mpc_step(), sp.mpc_step()
            np.testing.assert_array_equal(b.xt, a.xt[idx])
            np.testing.assert_array_equal(b.iters, a.iters[perm])


def test_async_steps_equal_blocking_steps(Solver):
    cfg = config.matlab_pi(H=20)
    scn = scenario.tiled(8, 20, n_steps=10, seed=5)
    with Solver(cfg, scn) as s1, Solver(cfg, scn) as s2:
        for _ in range(6):
            r = s1.mpc_step()
        s2.steps_async(0, 6)
        s2.sync()
        np.testing.assert_array_equal(s2.state()["xt"], r.xt)
        cnt = s2.counters()
        assert cnt["x_qps"] >= 6 * 16 and cnt["inexact"] == 0


@pytest.mark.parametrize("H,fixed", [(30, 1), (40, 1), (12, 0)])
def test_persistent_launch_equals_single_steps(Solver, H, fixed):
    """Persistent multi-step launches (the bench's mode: fixed iterations under the global
    scope, chunks of steps_per_launch() steps) give bit-identical states, controls and the
    global residual history of the last step as one launch per MPC step."""
    n = 9
    cfg = config.matlab_pi(H=H, fixed_iters=fixed, max_outer=40, term_global=fixed)
    scn = scenario.tiled(16, H, n_steps=n + 1, perturb=True, seed=3)
    with Solver(cfg, scn) as s1, Solver(cfg, scn) as s2:
        assert s2.steps_per_launch() >= (n if fixed or not cfg.term_global else 1)
        for _ in range(n):
            r = s1.mpc_step()
        s2.steps_async(0, n)
        s2.sync()
        st = s2.state()
        np.testing.assert_array_equal(st["xt"], r.xt)
        np.testing.assert_array_equal(st["u"], r.u)
        if cfg.term_global:
            g1, i1 = s1.global_resid()
            g2, i2 = s2.global_resid()
            assert i1 == i2
            np.testing.assert_array_equal(g1, g2)
        assert s2.counters()["inexact"] == 0


@pytest.mark.parametrize("H", [20, 30, 40])
def test_pair_solvers_agree(Solver, H, monkeypatch):
    """The pair QP's dual active set (default) and its ADMM + PDAS fallback
    (PIADMM_PAIR_SOLVER=admm) certify the same minimiser: identical iteration counts and
    residual histories, states equal to 1e-10, and the oracle agrees with both."""
    cfg = config.matlab_pi(H=H)
    scn = scenario.tiled(12, H, n_steps=8, perturb=True, seed=11)
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s_gi:
        monkeypatch.setenv("PIADMM_PAIR_SOLVER", "admm")
        s_admm = Solver(cfg, scn)
        monkeypatch.delenv("PIADMM_PAIR_SOLVER")
        try:
            for _ in range(6):
                ro, r1, r2 = orc.mpc_step(), s_gi.mpc_step(), s_admm.mpc_step()
                np.testing.assert_array_equal(r1.iters, r2.iters)
                np.testing.assert_array_equal(r1.iters, ro.iters)
                np.testing.assert_allclose(r1.xt, r2.xt, rtol=1e-10, atol=1e-10)
                np.testing.assert_allclose(r1.xt, ro.xt, rtol=1e-8, atol=1e-8)
                np.testing.assert_allclose(r1.u, ro.u, rtol=0, atol=1e-8)
                assert np.all(r1.status == 0) and np.all(r2.status == 0)
            c1, c2 = s_gi.counters(), s_admm.counters()
            assert c1["z_qps"] == c2["z_qps"] > 0
            assert c1["admm_z"] == 0 and c2["admm_z"] > 0     # GI certified every pair QP
        finally:
            s_admm.close()


@pytest.mark.parametrize("H,alt", [(15, "pdas"), (30, "pdas"), (40, "pdas"), (30, "gi"), (40, "gi"),
                                   (30, "gi_warm"), (15, "gi_cold_all")])
def test_xstep_solvers_agree(Solver, H, alt, monkeypatch):
    """x-step working-set changes by the dual active set started cold at a step's first x-QP
    (default), from the shifted labels (gi_warm), after their reduced solve (gi), cold at every
    x-QP (gi_cold_all), or by one-step PDAS label moves + ADMM (pdas): the same certified
    minimisers, iteration counts and residual histories, and all match the oracle."""
    cfg = config.matlab_pi(H=H)
    scn = scenario.tiled(10, H, n_steps=8, perturb=True, seed=21)
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s_gi:
        monkeypatch.setenv("PIADMM_X_SOLVER", alt)
        s_pd = Solver(cfg, scn)
        monkeypatch.delenv("PIADMM_X_SOLVER")
        try:
            for _ in range(6):
                ro, r1, r2 = orc.mpc_step(), s_gi.mpc_step(), s_pd.mpc_step()
                np.testing.assert_array_equal(r1.iters, r2.iters)
                np.testing.assert_array_equal(r1.iters, ro.iters)
                np.testing.assert_allclose(r1.xt, r2.xt, rtol=1e-10, atol=1e-10)
                np.testing.assert_allclose(r1.u, ro.u, rtol=0, atol=1e-8)
                np.testing.assert_allclose(r1.xt, ro.xt, rtol=1e-8, atol=1e-8)
                assert np.all(r1.status == 0) and np.all(r2.status == 0)
            c1, c2 = s_gi.counters(), s_pd.counters()
            assert c1["x_qps"] == c2["x_qps"]
            if H <= 32 and alt == "pdas":      # LDS mode: the x-step's dual active set replaces ADMM
                assert c1["admm_x"] < c2["admm_x"]
        finally:
            s_pd.close()


def test_errors_are_loud(Solver):
    with pytest.raises(_lib.PiadmmError, match="H must be"):
        Solver(config.matlab_pi(H=64), scenario.tiled(1, 64, n_steps=1))
    bad = scenario.tiled(2, 10)
    bad.edges = np.array([[2, 0]], np.int32)
    with pytest.raises(_lib.PiadmmError, match="edge must satisfy"):
        Solver(config.matlab_pi(H=10), bad)
    dup = scenario.tiled(2, 10)
    dup.edges = np.array([[0, 1], [2, 3], [0, 1]], np.int32)     # the same pair twice
    with pytest.raises(_lib.PiadmmError, match="duplicate candidate pair"):
        Solver(config.matlab_pi(H=10), dup)
    with Solver(config.matlab_pi(H=10), scenario.intersection(10)) as s:
        with pytest.raises(_lib.PiadmmError, match="time index"):
            s.mpc_step(t=41)
