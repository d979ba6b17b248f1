"""The sharded library in TWO PROCESSES on the one MI355X (the process model of
``bench.py --gpus N``): each process holds its own ``PI_ADMM_MI355X`` handle over its share of the
agents -- interleaved, so every candidate pair crosses the processes and every outer iteration
exchanges the boundary agents' positions and controls -- and the exchange all-reduce runs over a
gloo process group through ``piadmm_set_allreduce`` (RCCL refuses two ranks on one device; over
xGMI the same buffer goes to ``ncclAllReduce``).  The loops this replaces are the reference's
sequential ``for i_veh`` / edge loops (casadi/main.py:81,122).

Each rank's own agents must equal the unsharded job on one handle to 1e-12 (the exchange carries
exact values: one rank writes each slot, the others add zeros), with equal global iteration counts
and the job's residual history to 1e-9 (summation order).  The workers are child processes started
with subprocess (tests/_two_proc_worker.py); this process runs the unsharded job."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _two_proc_worker as W  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name", ["tiles_fixed", "crossing_natural"])
def test_two_processes_equal_the_unsharded_job(tmp_path, name):
    from piadmm.solver import PI_ADMM_MI355X, device_count
    if device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests need an MI355X")
    world, port = 2, _free_port()
    outs = [str(tmp_path / f"rank{r}.npz") for r in range(world)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_two_proc_worker.py"), name, str(r), str(world),
                               str(port), outs[r]], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=240)
            logs.append(o.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    cfg, scn, n_steps = W.case(name)
    with PI_ADMM_MI355X(cfg, scn) as s:
        ref = [s.mpc_step() for _ in range(n_steps)]
    seen = np.zeros(scn.n_agents, bool)
    for r in range(world):
        d = np.load(outs[r], allow_pickle=False)
        a = d["agents"]
        assert int(d["n_slots"]) > 0               # pairs cross the processes: a real exchange
        seen[a] = True
        for k in range(n_steps):
            np.testing.assert_array_equal(d["status"][k], 0)
            np.testing.assert_array_equal(ref[k].status, 0)
            np.testing.assert_allclose(d["xt"][k], ref[k].xt[a], rtol=1e-12, atol=1e-12, err_msg=f"rank {r} step {k}")
            np.testing.assert_allclose(d["u"][k], ref[k].u[a], rtol=1e-12, atol=1e-12, err_msg=f"rank {r} step {k}")
            assert int(d["global_iters"][k]) == ref[k].global_iters
            n = ref[k].global_iters
            np.testing.assert_allclose(d["global_resid"][k][:n], np.nan_to_num(ref[k].global_resid[:n], nan=-1.0),
                                       rtol=1e-9, atol=1e-12)
    assert seen.all()
