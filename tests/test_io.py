"""Run records (piadmm.io): the reference driver's outputs as files.  CPU: recorder, npz/json
round trip, the reference's progress line and figure.  GPU: the CLI end to end."""
import os

import numpy as np
import pytest

from oracle import piadmm_oracle as O
from piadmm import config, io, scenario


def _oracle_record(n=6):
    cfg = config.casadi_default(H=10)
    orc = O.Oracle(cfg, scenario.intersection(10))
    rec = io.RunRecorder(meta={"preset": "casadi_default", "H": 10})
    for _ in range(n):
        r = orc.mpc_step()
        resid = np.full((orc.n_comp, cfg.max_outer, 2), np.nan)
        for c, rr in enumerate(r.resid):
            if rr:
                resid[c, :len(rr)] = rr
        rec.add(r.xt, r.u, r.iters, resid, r.lam)
    return rec.record(), cfg


def test_record_round_trip(tmp_path):
    run, _ = _oracle_record()
    npz, js = io.save_run(str(tmp_path / "run"), run)
    assert os.path.exists(npz) and os.path.exists(js)
    back = io.load_run(str(tmp_path / "run"))
    for f in ("x_vec", "theta_vec", "u_vec", "iter_his", "dual_max", "dual_min"):
        np.testing.assert_array_equal(getattr(back, f), getattr(run, f))
    np.testing.assert_array_equal(np.isnan(back.resid), np.isnan(run.resid))
    assert back.meta == {"preset": "casadi_default", "H": 10}
    assert run.x_vec.shape == (6, 2, 2) and run.u_vec.shape == (6, 2)


def test_step_line_is_the_reference_format():
    """casadi/main.py:193-196."""
    xt = np.array([[1.5, 0.0, 0.0], [0.0, 2.5, -1.0]])
    line = io.step_line(3, np.array([7]), 0.25, -0.5, 2.0, xt)
    want = ("t_step: {}, iter: {}, max dual: {}, min dual: {}, rho: {}, veh_x: {}, veh_y: {}"
            .format(4, 7, 0.25, -0.5, 2.0, xt[:, 0], xt[:, 1]))
    assert line == want


def test_plot_writes_the_trajectory_scatter(tmp_path):
    pytest.importorskip("matplotlib")
    run, _ = _oracle_record(4)
    p = io.plot_run(run, str(tmp_path / "traj.png"))
    assert os.path.getsize(p) > 1000


@pytest.mark.gpu
def test_cli_run_matches_oracle(tmp_path):
    from piadmm import run as cli
    from piadmm.solver import device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible")
    out = str(tmp_path / "cli")
    assert cli.main(["--preset", "casadi_default", "--H", "10", "--steps", "6", "--out", out,
                     "--plot", out + ".png", "--quiet"]) == 0
    got = io.load_run(out)
    want, _ = _oracle_record(6)
    np.testing.assert_allclose(got.x_vec, want.x_vec, rtol=1e-8, atol=1e-8)
    np.testing.assert_array_equal(got.iter_his, want.iter_his)
    assert os.path.getsize(out + ".png") > 1000


def test_checkpoint_round_trip(tmp_path):
    """save_checkpoint / load_checkpoint: xt, the carried pair state and the
    next time index through an .npz written and read without pickles; a checkpoint of another
    configuration is refused."""
    cfg = config.matlab_pi(H=8, warm_duals=1)
    scn = scenario.intersection(8, n_steps=6)
    orc = O.Oracle(cfg, scn)
    for _ in range(3):
        orc.mpc_step()
    hat, lam, S, D, last = orc.edge_state
    st = dict(xt=orc.xt, hat=hat, lam=lam, S=S, D=D, last_hat=last, rho_pi=orc.rho_pi, t=orc.t)
    path = io.save_checkpoint(str(tmp_path / "c"), st, cfg, scn)
    back = io.load_checkpoint(path, cfg, scn)
    assert back["t"] == 3
    for k in io.CHECKPOINT_KEYS:
        np.testing.assert_array_equal(back[k], np.asarray(st[k]))
    with pytest.raises(ValueError):
        io.load_checkpoint(path, cfg.replace(H=9))
    # another scenario with the same agent and pair counts but other pairs: refused
    other = scenario.crossing(3, 8, n_steps=6, pairs="chain")
    assert other.n_agents != scn.n_agents or not np.array_equal(other.edges, scn.edges)
    with pytest.raises(ValueError):
        io.load_checkpoint(path, cfg, other)
    # a checkpoint without a fingerprint is refused when the scenario is given
    bare = io.save_checkpoint(str(tmp_path / "bare"), st, cfg)
    with pytest.raises(ValueError):
        io.load_checkpoint(bare, cfg, scn)
    # non-finite pair state is refused
    bad = dict(st, lam=np.where(np.arange(lam.size).reshape(lam.shape) == 3, np.nan, lam))
    with pytest.raises(ValueError):
        io.load_checkpoint(io.save_checkpoint(str(tmp_path / "nan"), bad, cfg, scn), cfg, scn)
