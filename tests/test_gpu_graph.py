"""GPU parity of graph mode (csrc/piadmm_graph.hip) through the C-ABI: candidate graphs beyond
disjoint two-vehicle pairs -- the reference's ``num_veh`` loop with every pair a candidate
(casadi/main.py:81,110-113; PI_ADMM_class.py:126-129), chains, several components of
different shapes, and the tiled benchmark forced onto the graph kernel (PIADMM_GRAPH=1),
which must agree with the fused kernel.  Tolerance as in test_gpu_parity.py (held 1e-8,
contract 1e-5), identical outer-iteration counts and residual histories."""
import os

import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import config, scenario

pytestmark = pytest.mark.gpu
RTOL = ATOL = 1e-8
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def Solver():
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    return PI_ADMM_MI355X


def close(a, b, rtol=RTOL, atol=ATOL):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def compare(Solver, cfg, scn, n_steps, setup=None):
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s:
        if setup:
            setup(s)
        assert s.C == orc.n_comp
        for k in range(n_steps):
            ro, rg = orc.mpc_step(), s.mpc_step()
            np.testing.assert_array_equal(rg.status, 0)
            np.testing.assert_array_equal(rg.iters, ro.iters, err_msg=f"step {k}")
            close(rg.xt, ro.xt)
            close(rg.u, ro.u)
            for c in range(s.C):
                n = len(ro.resid[c])
                if n:
                    close(rg.resid[c, :n], np.array(ro.resid[c]), rtol=1e-7, atol=1e-7)
                assert np.all(np.isnan(rg.resid[c, n:]))
            if cfg.term_global:
                n = len(ro.global_resid)
                assert rg.global_iters == int(ro.iters[0])
                if n:
                    close(rg.global_resid[:n], np.array(ro.global_resid), rtol=1e-7, atol=1e-7)
        st = s.state()
    close(st["pos_old"], ro.pos_old)
    close(st["hat"], ro.hat)
    close(st["lam"], ro.lam)
    np.testing.assert_array_equal(st["edge_active"].astype(bool), ro.edge_active)


@pytest.mark.parametrize("preset", ["matlab_pi", "casadi_default"])
@pytest.mark.parametrize("n", [3, 4])
def test_all_pairs_crossing(Solver, preset, n):
    """n vehicles, every pair a candidate: each agent's AL sum has n-1 terms, up to
    n(n-1)/2 pair QPs per outer iteration (matlab_pi at n = 4 includes a step that runs all
    100 outer iterations)."""
    compare(Solver, config.PRESETS[preset](H=15), scenario.crossing(n, 15, n_steps=30), 24)


def test_chain_graph(Solver):
    """Six vehicles, candidate pairs (k, k+1): interior agents in two pairs."""
    compare(Solver, config.matlab_pi(H=15), scenario.crossing(6, 15, n_steps=30, pairs="chain"), 24)


@pytest.mark.parametrize("H", [10, 30, 40])
def test_mixed_components_and_horizons(Solver, H):
    """Components of 4 (all pairs), 3 (chain), 2 and 1 agents side by side, per-component
    termination, 12 MPC steps; H = 40 takes the two-columns-per-lane pair K path (big mode) with
    two tiles of the intersection in place of the all-pairs crossing (that one is
    test_wide_working_sets_certify_against_the_oracle), and its 3-vehicle chain has a pair QP
    beyond 63 active rows at step 5 (the wide dual active set): against the oracle's golden run
    (oracle/gen_golden_wide.py -- the live oracle takes minutes at H = 40)."""
    if H > 32:
        from oracle import gen_golden_wide as G
        compare_golden(Solver, G.MIXED)
        return
    scn = scenario.concat([scenario.crossing(4, H, n_steps=14, seed=1), scenario.crossing(3, H, n_steps=14, pairs="chain"),
                           scenario.intersection(H, n_steps=14), scenario.crossing(1, H, n_steps=14)])
    compare(Solver, config.matlab_pi(H=H), scn, 12)


def test_wide_working_sets_certify_against_the_oracle(Solver):
    """Pair QPs whose dual active set needs more than 63 rows (the 4-vehicle all-pairs crossing at
    H = 40: both vehicles saturated, 78-79 active rows at some optima) are solved by the wide dual
    active set (two rows per lane, csrc/pd_qp.h gi_solve_wide) and certified: every QP status 0,
    no inexact QP, and the run equal to the NumPy oracle's golden run over 12 MPC steps
    (tests/golden/run_matlab_pi_H40_crossing4.npz, oracle/gen_golden_wide.py; step 7 runs all 100
    outer iterations), u and xt at 1e-8 on every step.  Before the wide solver these QPs were
    reported PIADMM_QP_INEXACT.  (Round 4 held only xt to 1e-4 from step 5 on: that fixture was
    wrong -- the oracle's QP solver returned an infeasible step-5 pair-QP answer without raising;
    oracle/qp_exact.py now certifies every answer it returns.)"""
    from oracle import gen_golden_wide as G
    compare_golden(Solver, G.NAME)


def compare_golden(Solver, name):
    """libpiadmm against a golden oracle run of oracle/gen_golden_wide.py (as compare()): every
    step at 1e-8, iteration counts and residual histories equal, the final pair state equal."""
    from oracle import gen_golden_wide as G
    g = np.load(os.path.join(GOLD, name + ".npz"))
    cfg, scn = G.make(name)
    K = int(g["n_steps"])
    with Solver(cfg, scn) as s:
        for k in range(K):
            r = s.mpc_step()
            np.testing.assert_array_equal(r.status, 0, err_msg=f"step {k}")
            np.testing.assert_array_equal(r.iters, g["iters"][k], err_msg=f"step {k}")
            close(r.xt, g["xt"][k])
            close(r.u, g["u"][k])
            for c in range(s.C):
                n = int(g["iters"][k][c])
                close(r.resid[c, :n], g["resid"][k][c][:n], rtol=1e-7, atol=1e-7)
        assert s.counters()["inexact"] == 0
        st = s.state()
    close(st["pos_old"], g["pos_old"])
    close(st["hat"], g["hat"])
    close(st["lam"], g["lam"])
    np.testing.assert_array_equal(st["edge_active"].astype(bool), g["edge_active"].astype(bool))


@pytest.mark.parametrize("warm", [0, 1])
@pytest.mark.parametrize("coop", [True, False])
def test_graph_global_termination(Solver, coop, warm, monkeypatch):
    """The reference's global flag / stop over all agents (term_global): in-kernel behind a grid
    barrier (cooperative launch) or host-decided (PIADMM_NO_COOP=1, one launch per iteration);
    with warm duals the step's final last_iter_hat carries over (copied only when continuing)."""
    scn = scenario.concat([scenario.crossing(4, 15, n_steps=20, seed=2), scenario.crossing(3, 15, n_steps=20, seed=3)])
    if not coop:
        monkeypatch.setenv("PIADMM_NO_COOP", "1")
    compare(Solver, config.matlab_pi(H=15, term_global=1, warm_duals=warm), scn, 14)


def test_graph_warm_duals_tightening_fixed(Solver):
    """a12 (receding-horizon dual shift) and a13 (delay tightening) on a 4-vehicle all-pairs
    crossing, and fixed iterations under the global scope."""
    compare(Solver, config.matlab_pi(H=15, warm_duals=1, tighten=1), scenario.crossing(4, 15, n_steps=24, seed=4), 16)
    compare(Solver, config.matlab_pi(H=12, fixed_iters=1, max_outer=8, term_global=1),
            scenario.crossing(4, 12, n_steps=12, seed=5), 6)


@pytest.mark.parametrize("H,fixed", [(12, 0), (30, 1), (40, 0)])
def test_graph_kernel_equals_fused_kernel_on_tiles(Solver, H, fixed, monkeypatch):
    """The tiled benchmark scenario forced onto the graph kernel gives the fused kernel's
    states, iteration counts and residual histories (to rounding: the two kernels contract
    multiply-adds differently)."""
    cfg = config.matlab_pi(H=H, fixed_iters=fixed, max_outer=30 if fixed else 100)
    scn = scenario.tiled(16, H, n_steps=10, seed=7)
    with Solver(cfg, scn) as s1:
        monkeypatch.setenv("PIADMM_GRAPH", "1")
        s2 = Solver(cfg, scn)
        monkeypatch.delenv("PIADMM_GRAPH")
        try:
            for _ in range(6):
                r1, r2 = s1.mpc_step(), s2.mpc_step()
                np.testing.assert_array_equal(r1.iters, r2.iters)
                close(r2.xt, r1.xt, rtol=1e-10, atol=1e-10)
                close(r2.u, r1.u, rtol=1e-10, atol=1e-10)
                np.testing.assert_allclose(r2.resid, r1.resid, rtol=1e-9, atol=1e-9)
                assert np.all(r2.status == 0)
            c1, c2 = s1.counters(), s2.counters()
            assert c1["x_qps"] == c2["x_qps"] and c1["z_qps"] == c2["z_qps"]
        finally:
            s2.close()


def test_all_pairs_tiles_at_256_agents(Solver):
    """64 copies of the 4-vehicle all-pairs crossing (256 agents, 384 candidate pairs, H = 30):
    sampled components against the oracle, every QP certified."""
    H = 30
    tiles = [scenario.crossing(4, H, n_steps=6, seed=k) for k in range(64)]
    scn = scenario.concat(tiles)
    cfg = config.matlab_pi(H=H)
    comps = [0, 31, 63]
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s:
        assert s.N == 256 and s.C == 64
        for _ in range(3):
            ro, rg = orc.mpc_step(components=comps), s.mpc_step()
            np.testing.assert_array_equal(rg.status, 0)
            for c in comps:
                sl = slice(4 * c, 4 * c + 4)
                assert rg.iters[c] == ro.iters[c]
                close(rg.xt[sl], ro.xt[sl])
                close(rg.u[sl], ro.u[sl])


@pytest.mark.parametrize("H,fixed,n", [(5, 0, 20), (15, 1, 6), (30, 1, 4)])
def test_global_pi_adaptive_rho(Solver, H, fixed, n):
    """The global PI law with adaptive rho and K_P (casadi_old_pi preset,
    casadi_old_PI_ADMM/main.py:133-155): every pair's penalty follows its minimum distance and
    enters the next x-steps (P = (2 Pnorm + sum_e rho_e) M'M + ...: the x-step and pair caches
    are rebuilt when it changes) and pair QPs; no collision gate; kept across MPC steps.  The
    script's own H = 5 with natural termination, and H = 15, 30 with 8 fixed iterations."""
    cfg = config.casadi_old_pi(H=H, fixed_iters=fixed, max_outer=8 if fixed else 100)
    compare(Solver, cfg, scenario.intersection(H, n_steps=n + 2), n)


def test_global_pi_on_a_crossing(Solver):
    """Three vehicles, every pair a candidate: each agent's P sums two adaptive penalties."""
    cfg = config.casadi_old_pi(H=12, fixed_iters=1, max_outer=6)
    compare(Solver, cfg, scenario.crossing(3, 12, n_steps=8, seed=2), 5)


@pytest.mark.parametrize("fixed", [0, 1])
def test_component_split_over_workgroups(Solver, monkeypatch, fixed):
    """A connected component larger than the workgroup block (term_global) spans several
    workgroups: blocks of 4 agents, the pairs dealt round-robin over the blocks, the X and Z
    phases as separate launches.  The job's residual sums run over the whole component in pair
    order (k_graph_partials, casadi/main.py:165-173), so a 24-vehicle chain (one component) equals
    the same job on one workgroup (PIADMM_GRAPH_BLOCK=0) to 1e-10 -- stop decisions included -- over
    all 24 steps (1 to 23 outer iterations, natural and fixed termination), and the oracle to 1e-8
    up to the first step with a logged near tie (none at the default 1e-9 here: all 24 steps)."""
    H = 12
    cfg = config.matlab_pi(H=H, term_global=1, fixed_iters=fixed, max_outer=30 if fixed else 100)
    scn = scenario.crossing(24, H, n_steps=26, seed=1, pairs="chain")
    s1 = Solver(cfg, scn)
    s1.set_tie_tolerance(1e-9)
    monkeypatch.setenv("PIADMM_GRAPH_BLOCK", "0")
    s2 = Solver(cfg, scn)
    monkeypatch.delenv("PIADMM_GRAPH_BLOCK")
    orc = O.Oracle(cfg, scn)
    tied = None                          # first step with a near tie (GPU or oracle)
    try:
        assert s1.C == 6 and s2.C == 1 and s1.steps_per_launch() == 1
        for k in range(24):
            r1, r2 = s1.mpc_step(), s2.mpc_step()
            assert np.all(r1.status == 0)
            assert r1.global_iters == r2.global_iters
            np.testing.assert_allclose(r1.xt, r2.xt, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
            np.testing.assert_allclose(r1.u, r2.u, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
            n = r1.global_iters
            np.testing.assert_array_equal(r1.global_resid[:n], r2.global_resid[:n])   # bit-identical sums
            if tied is None:
                ro = orc.mpc_step()
                if s1.near_ties()[1].size or orc.ties.events:
                    tied = k
                    continue
                assert r1.global_iters == int(ro.iters[0]), f"step {k}"
                close(r1.xt, ro.xt)
                close(r1.u, ro.u)
        assert tied is None, f"near tie at step {tied}: {s1.near_ties()}, {orc.ties.events[:3]}"
    finally:
        s1.close()
        s2.close()


def test_split_component_host_stepping(Solver):
    """Host stepping (piadmm_outer_iter, ABI 5) of a component split over workgroups: the step-init
    launch, then per iteration the X and Z launches and the pair-order partials; equal to
    mpc_step of the same job, iteration counts and residual histories included."""
    H = 12
    cfg = config.matlab_pi(H=H, term_global=1)
    scn = scenario.crossing(12, H, n_steps=8, seed=2, pairs="chain")
    with Solver(cfg, scn) as s1, Solver(cfg, scn) as s2:
        assert s1.C > 1
        for k in range(5):
            r1 = s1.mpc_step()
            it = 0
            while True:
                stop = s2.outer_iter(it)
                it += 1
                if stop or it == cfg.max_outer:
                    break
            xt, u = s2.step_finish()
            assert it == r1.global_iters, (k, it, r1.global_iters)
            np.testing.assert_array_equal(xt, r1.xt)
            np.testing.assert_array_equal(u, r1.u)


def test_large_connected_graph_split(Solver, monkeypatch):
    """256 agents in ONE connected chain at the bench horizon (H30, fixed 100 outer iterations,
    the bench's mode): 64 workgroups of 4 agents equal the single-workgroup job to 1e-10."""
    H = 30
    cfg = config.matlab_pi(H=H, term_global=1, fixed_iters=1)
    scn = scenario.crossing(256, H, n_steps=4, seed=2, pairs="chain")
    s1 = Solver(cfg, scn)
    monkeypatch.setenv("PIADMM_GRAPH_BLOCK", "0")
    s2 = Solver(cfg, scn)
    monkeypatch.delenv("PIADMM_GRAPH_BLOCK")
    try:
        assert s1.C == 64 and s2.C == 1
        for k in range(2):
            r1, r2 = s1.mpc_step(), s2.mpc_step()
            assert np.all(r1.status == 0)
            np.testing.assert_allclose(r1.xt, r2.xt, rtol=1e-10, atol=1e-10)
            np.testing.assert_allclose(r1.u, r2.u, rtol=1e-10, atol=1e-10)
            np.testing.assert_allclose(r1.global_resid, r2.global_resid, rtol=1e-9, atol=1e-12)
    finally:
        s1.close()
        s2.close()


def test_repeating_a_step_forgets_the_stored_active_sets(Solver):
    """a pair's stored dual active set (S^-1, Y columns, codes) is valid only for the
    MPC step that built it.  Solving the same t again (piadmm_mpc_step(h, t) twice: the second
    starts from the propagated state, another geometry) must not restore it; the library forgets
    the stored sets whenever a step does not continue the sequence (piadmm_capi.cpp
    continue_sequence).  The repeat must equal the same step on a fresh handle started from that
    state, with every QP certified."""
    cfg = config.matlab_pi(H=15)
    scn = scenario.concat([scenario.crossing(4, 15, n_steps=10, seed=2), scenario.crossing(3, 15, n_steps=10, seed=3)])
    with Solver(cfg, scn) as a:
        a.mpc_step(0)
        a.mpc_step(1)
        xt1 = a.xt.copy()
        rep = a.mpc_step(1)
        ca = a.counters()
    with Solver(cfg, scn) as b:
        b.set_xt(xt1)
        ref = b.mpc_step(1)
    np.testing.assert_array_equal(rep.status, 0)
    np.testing.assert_array_equal(ref.status, 0)
    np.testing.assert_array_equal(rep.iters, ref.iters)
    close(rep.xt, ref.xt)
    close(rep.u, ref.u)
    assert ca["inexact"] == 0
