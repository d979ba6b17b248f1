"""GPU parity of the ABI-2 modes through the C-ABI: global termination (stepped launches,
host decision from all-reduced partials), receding-horizon dual warm start (a12), delay
tightening (a13), and the RCCL communicator on a single rank.  Tolerances as in
test_gpu_parity.py (held 1e-8, contract 1e-5)."""
import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import config, scenario

pytestmark = pytest.mark.gpu
RTOL = ATOL = 1e-8


@pytest.fixture(scope="module")
def Solver():
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    return PI_ADMM_MI355X


def close(a, b):
    np.testing.assert_allclose(a, b, rtol=RTOL, atol=ATOL)


def compare(Solver, cfg, scn, n_steps, setup=None):
    orc = O.Oracle(cfg, scn)
    with Solver(cfg, scn) as s:
        if setup:
            setup(s)
        for _ in range(n_steps):
            ro, rg = orc.mpc_step(), s.mpc_step()
            np.testing.assert_array_equal(rg.status, 0)
            np.testing.assert_array_equal(rg.iters, ro.iters)
            close(rg.xt, ro.xt)
            close(rg.u, ro.u)
            for c in range(s.C):
                n = len(ro.resid[c])
                if n:
                    close(rg.resid[c, :n], np.array(ro.resid[c]))
                assert np.all(np.isnan(rg.resid[c, n:]))
            if cfg.term_global:
                n = len(ro.global_resid)
                assert rg.global_iters == int(ro.iters[0])
                if n:
                    close(rg.global_resid[:n], np.array(ro.global_resid))
                assert np.all(np.isnan(rg.global_resid[n:]))


@pytest.mark.parametrize("preset", ["casadi_default", "matlab_pi"])
def test_global_termination_matches_oracle(Solver, preset):
    compare(Solver, config.PRESETS[preset](H=15, term_global=1), scenario.tiled(3, 15, n_steps=30, seed=3), 14)


def test_global_termination_fixed_iterations(Solver):
    compare(Solver, config.matlab_pi(H=12, fixed_iters=1, max_outer=6, term_global=1),
            scenario.tiled(2, 12, n_steps=10, seed=1), 4)


def test_global_termination_without_any_collision(Solver):
    """No pair ever collides: the job stops at the first collision test (resid NaN)."""
    compare(Solver, config.matlab_pi(H=10, term_global=1), scenario.tiled(3, 10, n_steps=12, seed=3), 3)


def test_in_kernel_global_termination_equals_host_decision(Solver, monkeypatch):
    """Natural global termination on one rank runs the stop test in-kernel behind a grid
    barrier (cooperative launch, several MPC steps per launch); the host-decided path
    (PIADMM_NO_COOP=1: one launch per outer iteration) gives the same job."""
    cfg = config.matlab_pi(H=30, term_global=1)
    scn = scenario.tiled(24, 30, n_steps=12, perturb=True, seed=4)
    with Solver(cfg, scn) as s1:
        monkeypatch.setenv("PIADMM_NO_COOP", "1")
        s2 = Solver(cfg, scn)
        monkeypatch.delenv("PIADMM_NO_COOP")
        try:
            assert s1.steps_per_launch() > 1 and s2.steps_per_launch() == 1
            for _ in range(5):
                r1, r2 = s1.mpc_step(), s2.mpc_step()
                assert r1.global_iters == r2.global_iters
                np.testing.assert_array_equal(r1.iters, r2.iters)
                np.testing.assert_allclose(r1.global_resid, r2.global_resid, rtol=1e-12, atol=1e-12)
                np.testing.assert_allclose(r1.xt, r2.xt, rtol=1e-12, atol=1e-12)
            s1.steps_async(5, 4)
            s2.steps_async(5, 4)
            s1.sync()
            s2.sync()
            np.testing.assert_allclose(s1.state()["xt"], s2.state()["xt"], rtol=1e-12, atol=1e-12)
            assert s1.global_resid()[1] == s2.global_resid()[1]
        finally:
            s2.close()


@pytest.mark.parametrize("preset", ["casadi_default", "matlab_pi"])
def test_warm_duals_match_oracle(Solver, preset):
    compare(Solver, config.PRESETS[preset](H=15, warm_duals=1), scenario.tiled(2, 15, n_steps=30, seed=5), 20)


def test_tightening_matches_oracle(Solver):
    compare(Solver, config.matlab_pi(H=15, tighten=1, avg_delay=0.2, var_delay=0.1),
            scenario.tiled(2, 15, n_steps=30, seed=6), 20)


@pytest.mark.parametrize("coop", [True, False])
def test_all_modes_together_at_bench_horizon(Solver, coop, monkeypatch):
    """Global scope, warm duals and tightening at H = 30, the stop decided in-kernel (coop) or
    on the host (one launch per outer iteration): last_iter_hat is copied only when the job
    continues (casadi/main.py:180 after the stop test), which the warm duals carry over."""
    if not coop:
        monkeypatch.setenv("PIADMM_NO_COOP", "1")
    cfg = config.matlab_pi(H=30, term_global=1, warm_duals=1, tighten=1)
    compare(Solver, cfg, scenario.tiled(2, 30, n_steps=10, seed=8), 6)


def test_rccl_single_rank_communicator(Solver):
    """The RCCL path (ncclCommInitRank + one all-reduce per outer iteration) on one rank
    gives the same job as no communicator."""
    from piadmm.solver import comm_unique_id
    uid = comm_unique_id()
    assert len(uid) == 128
    compare(Solver, config.casadi_default(H=15, term_global=1), scenario.tiled(3, 15, n_steps=30, seed=3), 6,
            setup=lambda s: s.comm_init(uid, 1, 0))
    compare(Solver, config.matlab_pi(H=12, fixed_iters=1, max_outer=6, term_global=1),
            scenario.tiled(2, 12, n_steps=10, seed=1), 3, setup=lambda s: s.comm_init(comm_unique_id(), 1, 0))


@pytest.mark.parametrize("H,n", [(10, 12), (15, 8), (25, 6), (30, 6), (50, 3)])
def test_fp32_admm_matrices_keep_answers(Solver, H, n):
    """precision 1 (configs[4] study): the ADMM iterations read fp32 K_s^-1 images, the polish
    and its KKT certificate stay fp64 -- every QP certified, answers equal the oracle's.  Odd H
    (15, 25) checks the 8-byte alignment of the second wave's fp32 region in LDS mode."""
    compare(Solver, config.matlab_pi(H=H, precision=1, tighten=int(H == 50)),
            scenario.tiled(2, H, n_steps=12, seed=H + 1), n)


@pytest.mark.parametrize("kind", ["tiles", "crossings"])
def test_device_decided_termination_equals_host_decision(Solver, monkeypatch, kind):
    """Natural global termination without the in-kernel grid barrier (the path of every rank of
    a multi-GPU job; PIADMM_NO_COOP=1 takes it on one rank): the stop rules run on the device
    (k_decide after the all-reduced partials, chunks of iterations enqueued ahead, one host read
    per chunk) and give the same job as one host decision per outer iteration
    (PIADMM_HOST_DECIDE=1) -- steps of 1 to many outer iterations, fused and graph kernels."""
    H = 20
    cfg = config.matlab_pi(H=H, term_global=1)
    if kind == "tiles":
        scn = scenario.tiled(6, H, n_steps=24, perturb=True, seed=9)
    else:
        scn = scenario.concat([scenario.crossing(4, H, n_steps=24, seed=k) for k in range(3)])
    monkeypatch.setenv("PIADMM_NO_COOP", "1")
    s1 = Solver(cfg, scn)
    monkeypatch.setenv("PIADMM_HOST_DECIDE", "1")
    s2 = Solver(cfg, scn)
    monkeypatch.delenv("PIADMM_HOST_DECIDE")
    monkeypatch.delenv("PIADMM_NO_COOP")
    its = []
    try:
        for _ in range(22):
            r1, r2 = s1.mpc_step(), s2.mpc_step()
            assert r1.global_iters == r2.global_iters
            its.append(r1.global_iters)
            np.testing.assert_array_equal(r1.iters, r2.iters)
            np.testing.assert_allclose(r1.global_resid, r2.global_resid, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(r1.xt, r2.xt, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(r1.u, r2.u, rtol=1e-12, atol=1e-12)
        s1.steps_async(22, 2)
        s2.steps_async(22, 2)
        s1.sync()
        s2.sync()
        np.testing.assert_allclose(s1.state()["xt"], s2.state()["xt"], rtol=1e-12, atol=1e-12)
    finally:
        s1.close()
        s2.close()
    assert len(set(its)) > 1            # steps of different lengths: chunks shorter and longer than needed


@pytest.mark.parametrize("kind", ["fused_warm_duals", "graph_warm_duals", "global_pi"])
def test_checkpoint_resume_equals_uninterrupted_run(Solver, tmp_path, kind):
    """piadmm_get_step_state / piadmm_set_state + piadmm.io checkpoints: a run
    checkpointed mid-run (after the first collisions: xt and the carried pair state -- warm_duals'
    hat / lam / S / D / last_hat, the global-PI pair penalties, casadi_old_PI_ADMM/main.py:139) and
    resumed in a NEW handle equals the uninterrupted run over the remaining steps (to rounding: the
    QP solvers' warm starts are not part of the checkpoint, every answer is the certified minimiser)."""
    from piadmm import io
    if kind == "fused_warm_duals":
        cfg, scn, k1, k2 = config.matlab_pi(H=15, warm_duals=1), scenario.tiled(4, 15, n_steps=16, seed=2), 9, 14
    elif kind == "graph_warm_duals":
        cfg, scn, k1, k2 = config.matlab_pi(H=15, warm_duals=1), scenario.crossing(4, 15, n_steps=14, seed=4), 7, 12
    else:
        cfg, scn, k1, k2 = (config.casadi_old_pi(H=8, fixed_iters=1, max_outer=10), scenario.intersection(8, n_steps=22),
                            17, 20)
    with Solver(cfg, scn) as a:
        full = [a.mpc_step() for _ in range(k1)]
        path = io.save_checkpoint(str(tmp_path / "ckpt"), a.step_state(), cfg, scn)
        full += [a.mpc_step() for _ in range(k2 - k1)]
    st = io.load_checkpoint(path, cfg, scn)
    assert st["t"] == k1
    if kind != "global_pi":
        assert np.any(st["lam"] != 0.0)            # the carried duals are in the checkpoint
    else:
        assert np.any(st["rho_pi"] != cfg.rho)     # the adapted penalties are
    with Solver(cfg, scn) as b:
        b.set_state(st)
        for k in range(k1, k2):
            r = b.mpc_step()
            np.testing.assert_array_equal(r.iters, full[k].iters, err_msg=f"step {k}")
            np.testing.assert_allclose(r.xt, full[k].xt, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
            np.testing.assert_allclose(r.u, full[k].u, rtol=1e-10, atol=1e-10, err_msg=f"step {k}")
    with pytest.raises(ValueError, match="another configuration"):
        io.load_checkpoint(path, cfg.replace(rho=cfg.rho * 2))


def test_fp32_tables_config5_tolerance_study(Solver):
    """configs[4]'s fp32 tolerance study on the GPU (precision 2): 256 agents x H50 with delay
    tightening (decentralized/util.py:70-101), the x-step's parametric tables read in fp32 with one
    fp64 refinement step.  Sampled tiles against the oracle (fp64) over 4 MPC steps, and the whole job
    against the fp64 GPU run: max |du|, the relative dxt and the outer-iteration counts, held to the
    north-star contract 1e-5 (DESIGN.md section 6 reports the measured values)."""
    H = 50
    cfg64 = config.matlab_pi(H=H, tighten=1)
    cfg32 = cfg64.replace(precision=2)
    scn = scenario.tiled(128, H, n_steps=6)
    comps = [0, 63, 127]
    orc = O.Oracle(cfg64, scn)
    du_o = dx_o = du_g = dx_g = 0.0
    it_changes = 0
    with Solver(cfg32, scn) as s32, Solver(cfg64, scn) as s64:
        for _ in range(4):
            r32, r64, ro = s32.mpc_step(), s64.mpc_step(), orc.mpc_step(components=comps)
            assert np.all(r32.status == 0)
            it_changes += int(np.sum(r32.iters != r64.iters))
            du_g = max(du_g, float(np.max(np.abs(r32.u - r64.u))))
            dx_g = max(dx_g, float(np.max(np.abs(r32.xt - r64.xt) / (1.0 + np.abs(r64.xt)))))
            for c in comps:
                sl = slice(2 * c, 2 * c + 2)
                assert r32.iters[c] == ro.iters[c]
                du_o = max(du_o, float(np.max(np.abs(r32.u[sl] - ro.u[sl]))))
                dx_o = max(dx_o, float(np.max(np.abs(r32.xt[sl] - ro.xt[sl]) / (1.0 + np.abs(ro.xt[sl])))))
        c32 = s32.counters()
    print(f"precision 2 vs oracle: max|du| {du_o:.2e}, rel dxt {dx_o:.2e}; vs fp64 GPU: max|du| {du_g:.2e}, "
          f"rel dxt {dx_g:.2e}, iteration-count changes {it_changes}; counters {c32}")
    assert it_changes == 0
    assert max(du_o, dx_o, du_g, dx_g) <= 1e-5


@pytest.mark.parametrize("case", ["bench_fixed", "natural", "inexact", "big_fixed", "linear_fixed", "linear_natural"])
def test_speculative_loop_equals_plain_loop(Solver, monkeypatch, case):
    """The fused kernel's speculative loop shape (the agent waves solve iteration it+1's x-step
    while the pair wave rolls out, tests and decides iteration it; casadi/main.py:81-181) against
    the plain one (PIADMM_NO_SPEC=1): the same iteration counts, QP status and work counters, and
    states, controls and residual histories equal to rounding (1e-10: the two shapes are separately
    inlined copies of the same statements, whose floating-point contractions the compiler may
    schedule differently -- up to 1.4e-12 observed on the controls).  A speculation repeats a certified x-QP only; a
    discarded one gives its work and the warm ADMM state back and leaves no table the plain loop
    would not hold, so even uncertified (ADMM-capped) x-QPs see the plain loop's state.  Cases:
    the bench's tiles (matlab_pi 256 x H30 shape, fixed 100 outer iterations), natural
    per-component termination, and x-QPs forced uncertified (PIADMM_X_SOLVER=pdas with 3 ADMM
    iterations: INEXACT answers depend on the warm state, which the speculation must not touch), and
    the casadi_default preset's linearised position model (configs[1]'s 64 x H20 shape, fixed and
    natural)."""
    H = {"bench_fixed": 30, "big_fixed": 40, "linear_fixed": 20}.get(case, 15)
    kw = dict(H=H)
    if case in ("bench_fixed", "big_fixed", "linear_fixed"):
        kw.update(fixed_iters=1, term_global=1)
    if case == "linear_fixed":
        kw.update(max_outer=60)
    if case == "big_fixed":
        kw.update(max_outer=40)       # big mode (H > 32): the tables in HBM / L2, the lean repeat's global pass
    if case == "inexact":
        kw.update(max_inner=3, fixed_iters=1, max_outer=12)
        monkeypatch.setenv("PIADMM_X_SOLVER", "pdas")
    cfg = (config.casadi_default if case.startswith("linear") else config.matlab_pi)(**kw)
    assert cfg.pos_model == (config.POS_LINEAR if case.startswith("linear") else config.POS_NONLINEAR)
    n_tiles, n_steps = {"bench_fixed": (32, 6), "big_fixed": (16, 4), "linear_fixed": (32, 6)}.get(case, (16, 14))
    scn = scenario.tiled(n_tiles, H, n_steps=n_steps + 2, seed=5)
    runs = []
    for nospec in ("0", "1"):
        monkeypatch.setenv("PIADMM_NO_SPEC", nospec)
        with Solver(cfg, scn) as s:
            recs = [s.mpc_step() for _ in range(n_steps)]
            runs.append((recs, s.counters(), s.state()))
    (ra, ca, sa), (rb, cb, sb) = runs
    tol = dict(rtol=1e-10, atol=1e-10)
    for k, (a, b) in enumerate(zip(ra, rb)):
        for f in ("iters", "status"):
            np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f"{f} at step {k}")
        for f in ("xt", "u", "resid"):
            np.testing.assert_allclose(getattr(a, f), getattr(b, f), err_msg=f"{f} at step {k}", **tol)
    for f in ("pos_old", "hat", "lam", "S", "D"):
        np.testing.assert_allclose(sa[f], sb[f], err_msg=f, **tol)
    assert ca == cb
    if case == "inexact":
        assert ca["inexact"] > 0                 # the uncertified path is exercised
    else:
        assert ca["inexact"] == 0


@pytest.mark.parametrize("case", ["bench_fixed", "natural", "smoke_natural", "linear_natural", "smoke_job"])
def test_warm_helper_equals_pair_alone(Solver, monkeypatch, case):
    """The pair's warm build on two waves (the helper wave computes each stored row's P^-1 n, A y
    and its products with the earlier rows, pd_qp.h WarmPipe) against the pair wave alone
    (PIADMM_NO_HELPER=1): the helper hands over the values the pair wave would compute itself, so
    every output, residual history, iteration count and work counter is bit-identical.  Cases: the
    bench's tiles (fixed 100 iterations, the speculative shape's roller as the helper), natural
    global termination (the plain shape's fourth wave, cooperative launch), a small job under it,
    the linearised position model, and smoke()'s own job (per-component stop)."""
    H = {"bench_fixed": 30, "smoke_natural": 10, "linear_natural": 20, "smoke_job": 10}.get(case, 15)
    kw = dict(H=H)
    if case == "bench_fixed":
        kw.update(fixed_iters=1, term_global=1)
    elif case != "smoke_job":
        kw.update(term_global=1)
    cfg = (config.casadi_default if case == "linear_natural" else config.matlab_pi)(**kw)
    n_tiles, n_steps = {"bench_fixed": (32, 6), "smoke_natural": (2, 20), "smoke_job": (2, 30)}.get(case, (16, 12))
    if case == "smoke_job":   # __graft_entry__.smoke()'s job: per-component stop (the speculative shape)
        scn = scenario.tiled(2, 10, n_steps=30, seed=1)
    else:
        scn = scenario.tiled(n_tiles, H, n_steps=n_steps + 2, seed=7)
    runs = []
    for nh in ("0", "1"):
        monkeypatch.setenv("PIADMM_NO_HELPER", nh)
        with Solver(cfg, scn) as s:
            recs = [s.mpc_step() for _ in range(n_steps)]
            runs.append((recs, s.counters(), s.state()))
    (ra, ca, sa), (rb, cb, sb) = runs
    for k, (a, b) in enumerate(zip(ra, rb)):
        for f in ("iters", "status", "xt", "u"):
            np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f"{f} at step {k}")
        np.testing.assert_array_equal(np.nan_to_num(a.resid, nan=-1.0), np.nan_to_num(b.resid, nan=-1.0))
    for f in ("pos_old", "hat", "lam", "S", "D"):
        np.testing.assert_array_equal(sa[f], sb[f], err_msg=f)
    assert ca == cb
    assert ca["z_qps"] > 0
