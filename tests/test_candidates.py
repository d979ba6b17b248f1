"""Candidate-pair graph: the reach bound and the brute-force statement on
CPU; the GPU grid hash (piadmm_candidate_pairs) against it, bit for bit (integer pair sets)."""
import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import candidates, config


@pytest.mark.parametrize("preset,H", [("casadi_default", 15), ("matlab_pi", 30), ("casadi_default", 50)])
def test_reach_radius_bounds_every_rollout(preset, H):
    """Any admissible plan (|u| <= u_max) keeps the x-step positions within reach - d/2 of the
    start: the linearised (PI_ADMM_class.py:59-69) and the nonlinear (MATLAB) rollouts."""
    cfg = config.PRESETS[preset](H=H)
    rng = np.random.default_rng(3)
    dcol = cfg.dis_thres if cfg.collide_sq_thres else np.sqrt(cfg.dis_thres)
    for _ in range(200):
        s = rng.choice([2.0, 4.0, 8.0, 12.0])
        xt = np.array([rng.uniform(-50, 50), rng.uniform(-50, 50), rng.uniform(-np.pi, np.pi)])
        u = rng.choice([-1.0, 1.0], size=H) * cfg.u_max * rng.uniform(0.5, 1.0, size=H)
        if rng.random() < 0.5:
            u = np.full(H, cfg.u_max * rng.choice([-1.0, 1.0]))       # the extreme: steady full lock
        roll = O.rollout_linear if cfg.pos_model == 0 else O.rollout_nonlinear
        x, y, _ = roll(xt, u, s, cfg.dt, cfg.L)
        dmax = np.max(np.hypot(x - xt[0], y - xt[1]))
        r = candidates.reach_radii(cfg, np.array([s]))[0]
        assert dmax <= r - 0.5 * dcol + 1e-9


def test_bruteforce_statement_matches_kdtree():
    spatial = pytest.importorskip("scipy.spatial")
    rng = np.random.default_rng(5)
    xy = rng.uniform(0, 100, size=(3000, 2))
    r = np.full(3000, 1.3)
    ref = O.candidate_pairs(xy, r)
    kd = np.array(sorted(spatial.cKDTree(xy).query_pairs(2.6)), np.int32).reshape(-1, 2)
    assert ref.shape[0] > 1000
    np.testing.assert_array_equal(ref, kd)


def _cases():
    rng = np.random.default_rng(11)
    yield "clusters", np.concatenate([rng.normal(c, 3.0, size=(400, 2)) for c in rng.uniform(-200, 200, (12, 2))]), \
        rng.uniform(0.2, 2.5, 4800)
    yield "identical", np.zeros((300, 2)) + 7.0, np.zeros(300)                 # radius 0: identical points only
    yield "one_cell", rng.uniform(0, 1, (500, 2)), np.full(500, 5.0)           # every pair
    yield "huge_coords", rng.uniform(-1e12, 1e12, (200, 2)) + rng.uniform(0, 1, (200, 2)), np.full(200, 3e10)
    yield "lattice_ties", np.stack(np.meshgrid(np.arange(30.0), np.arange(30.0)), -1).reshape(-1, 2), np.full(900, 0.5)
    yield "single", np.zeros((1, 2)), np.ones(1)


@pytest.mark.gpu
def test_gpu_candidate_pairs_equal_bruteforce():
    """Integer pair lists equal bit for bit, incl. ties on the boundary (a unit lattice with
    r_i + r_j = 1 exactly), identical points, one crowded cell, 1e12 coordinates, n = 0 / 1, and
    a short output buffer (the total comes back, the caller retries)."""
    from piadmm.scenario import intersection
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    with PI_ADMM_MI355X(config.matlab_pi(H=10), intersection(10)) as s:
        for name, xy, r in _cases():
            got = candidates.candidate_pairs(s, xy, r)
            np.testing.assert_array_equal(got, O.candidate_pairs(xy, r), err_msg=name)
        assert candidates.candidate_pairs(s, np.zeros((0, 2)), np.zeros(0)).shape == (0, 2)


@pytest.mark.gpu
def test_gpu_candidate_pairs_million_agents():
    """1M agents at crowd density: sampled agents' partner lists against an exact scan of their
    neighbourhood (cKDTree superset, then the same fp64 test); the count and the order."""
    spatial = pytest.importorskip("scipy.spatial")
    from piadmm.scenario import intersection
    from piadmm.solver import PI_ADMM_MI355X
    rng = np.random.default_rng(2)
    n = 1 << 20
    xy = rng.uniform(0, 3000.0, size=(n, 2))
    r = rng.uniform(1.0, 3.0, n)
    with PI_ADMM_MI355X(config.matlab_pi(H=10), intersection(10)) as s:
        pairs, ms = candidates.candidate_pairs(s, xy, r, with_time=True)
    assert np.all(np.diff(pairs[:, 0]) >= 0) and np.all(pairs[:, 0] < pairs[:, 1])
    same = np.diff(pairs[:, 0]) == 0
    assert np.all(np.diff(pairs[:, 1])[same] > 0)
    tree = spatial.cKDTree(xy)
    starts = np.searchsorted(pairs[:, 0], np.arange(n))
    ends = np.searchsorted(pairs[:, 0], np.arange(n), side="right")
    for i in rng.choice(n, 300, replace=False):
        cand = np.array(sorted(j for j in tree.query_ball_point(xy[i], r[i] + 3.0 + 1e-6) if j > i), np.int64)
        if cand.size:
            dx, dy = xy[cand, 0] - xy[i, 0], xy[cand, 1] - xy[i, 1]
            cand = cand[dx * dx + dy * dy <= (r[i] + r[cand]) * (r[i] + r[cand])]
        np.testing.assert_array_equal(pairs[starts[i]:ends[i], 1], cand)
    print(f"\n1M agents: {pairs.shape[0]} candidate pairs in {ms:.3f} ms of device time")
    assert ms > 0


@pytest.mark.gpu
def test_dynamic_candidate_graph_planner_matches_oracle():
    """A receding-horizon planner on a dynamic candidate graph: every MPC step the graph is
    rebuilt on the GPU from the current states (reach discs) and the step runs on it; the
    oracle, given the same graph each step, follows the same trajectory."""
    from piadmm import scenario
    from piadmm.solver import PI_ADMM_MI355X
    H = 12
    cfg = config.matlab_pi(H=H)
    # two crossings 60 m apart: far-apart vehicles never become candidates of each other
    a, b = scenario.crossing(4, H, n_steps=14, seed=1), scenario.crossing(4, H, n_steps=14, seed=2)
    b.xt0[:, 0] += 60.0
    b.ref[:, 0, :] += 60.0
    scn = scenario.concat([a, b])
    with PI_ADMM_MI355X(cfg, scn) as s:
        xt = scn.xt0.copy()
        n_edges = []
        for k in range(10):
            r = candidates.reach_radii(cfg, scn.spd, xt[:, 2])
            edges = candidates.candidate_pairs(s, xt[:, :2], r)
            np.testing.assert_array_equal(edges, O.candidate_pairs(xt[:, :2], r))
            assert edges.shape[0] <= 12 and np.all((edges[:, 0] < 4) == (edges[:, 1] < 4))
            n_edges.append(edges.shape[0])
            s.set_candidate_graph(edges)
            rg = s.mpc_step(k)
            sub = scenario.Scenario(spd=scn.spd, xt0=xt, ref=scn.ref, edges=edges, n_steps=scn.n_steps)
            orc = O.Oracle(cfg, sub)
            orc.t = k
            ro = orc.mpc_step()
            assert np.all(rg.status == 0)
            np.testing.assert_array_equal(rg.iters, ro.iters)
            np.testing.assert_allclose(rg.xt, ro.xt, rtol=1e-8, atol=1e-8)
            xt = rg.xt
        assert n_edges[0] < max(n_edges) and max(n_edges) >= 4     # the graph grows as the vehicles close in
