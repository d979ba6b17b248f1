"""Host-side logic: presets vs the reference's parameter blocks, scenarios, sharding."""
import math

import numpy as np
import pytest

from piadmm import config, dist, scenario


def test_casadi_default_matches_reference_bunch():
    """casadi/PI_ADMM_class.py:15-28 and casadi/main.py (plain dual, no saturation)."""
    c = config.casadi_default()
    assert (c.dt, c.L, c.H, c.dis_thres, c.beta, c.Pnorm, c.Pcost, c.max_outer, c.rho, c.eps_pri, c.eps_dual) == \
        (0.1, 1.0, 15, 2.0, 10.0, 1.0, 1.0, 100, 2.0, 20.0, 1.0)
    assert c.dual_mode == config.DUAL_PLAIN and c.windup == 0
    assert c.round_decimals == 4 and c.alias_dual_residual == 1 and c.collide_sq_thres == 0
    assert c.u_max == math.pi / 6 and c.du_max == math.pi / 9          # nonlcon_function :173-180


def test_matlab_pi_matches_reference_block():
    """ADMM_CVX_two_veh_intesection_PI_antiwindup.m:6-25,43."""
    c = config.matlab_pi()
    assert (c.H, c.dis_thres, c.beta, c.Pnorm, c.Pcost, c.rho, c.eps_pri, c.eps_dual) == \
        (8, 2.0, 1000.0, 5.0, 1.0, 3.5, 0.1, 0.1)
    assert (c.kP, c.kI, c.theta1, c.theta2, c.windup_sat) == (0.0, 3.5, 5.0, 3.0, 30.0)
    assert c.dual_mode == config.DUAL_PI and c.windup == 1 and c.term_dist_check == 1
    assert config.matlab_pi(rho=2.0).kI == 2.0      # param.kI = param.rho


def test_intersection_matches_reference_scenario():
    """casadi/main.py:25, PI_ADMM_class.py:31-37."""
    s = scenario.intersection(15)
    np.testing.assert_array_equal(s.ref[0, 0], np.linspace(-10, 10, 50))
    np.testing.assert_array_equal(s.ref[1, 1], np.linspace(20, -20, 50))
    assert not s.ref[0, 1].any() and not s.ref[1, 0].any()
    np.testing.assert_array_equal(s.xt0, [[-10, 0, 0], [0, 20, -np.pi / 2]])
    np.testing.assert_array_equal(s.spd, [4, 8])
    assert s.n_steps == 35                                    # int(Nt/dt - num_ho)
    assert scenario.intersection(50).n_steps == 0            # quirk B13
    assert scenario.intersection(50, n_steps=10).ref.shape[2] == 60


def test_extended_reference_keeps_spacing():
    s = scenario.intersection(30, n_steps=40)
    d = np.diff(s.ref[0, 0])
    np.testing.assert_allclose(d, 20 / 49, rtol=1e-12)
    np.testing.assert_array_equal(s.ref[0, 0, :50], np.linspace(-10, 10, 50))


def test_tiled_scenario_and_graph():
    s = scenario.tiled(5, 20, perturb=True, seed=3)
    assert s.n_agents == 10 and s.n_edges == 5
    comp, nc = s.components()
    assert nc == 5 and list(comp) == [0, 0, 1, 1, 2, 2, 3, 3, 4, 4]
    ptr, nbr, eo, do = s.neighbours()
    assert list(ptr) == list(range(0, 11))
    assert list(nbr[:4]) == [1, 0, 3, 2] and list(do[:4]) == [0, 1, 0, 1]
    # seeded perturbations are reproducible and bounded
    s2 = scenario.tiled(5, 20, perturb=True, seed=3)
    np.testing.assert_array_equal(s.xt0, s2.xt0)
    base = scenario.tiled(5, 20, perturb=False)
    d = np.abs(s.xt0 - base.xt0)
    assert d[:, :2].max() <= 0.5 and d[:, 2].max() <= 0.05


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shards_cover_components_without_straddling(world):
    s = scenario.tiled(13, 10)
    seen = []
    for r in range(world):
        a0, a1 = dist.shard_bounds(s, r, world)
        sub = dist.shard(s, r, world)
        assert sub.n_agents == a1 - a0
        assert sub.n_edges == (a1 - a0) // 2
        np.testing.assert_array_equal(sub.xt0, s.xt0[a0:a1])
        seen.extend(range(a0, a1))
    assert seen == list(range(s.n_agents))


def test_shard_rejects_non_contiguous_component():
    s = scenario.tiled(2, 10)
    s.edges = np.array([[0, 3]], np.int32)     # a component that is not a contiguous agent range
    with pytest.raises(ValueError):
        dist.shard(s, 0, 2)
