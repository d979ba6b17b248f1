"""Diagnostic: the host-decided global-termination path with a host all-reduce transport, in one
process (fixed run, close, natural run -- bench.py's sequence for N > 1 ranks)."""
import sys

sys.path[:0] = ['.', 'distributed-local-planner-pi-admm_amd']
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 128
for fixed in (1, 0):
    cfg = config.matlab_pi(H=30, max_outer=100, fixed_iters=fixed, term_global=1)
    scn = scenario.tiled(tiles, 30, n_steps=6, perturb=True, seed=0)
    with PI_ADMM_MI355X(cfg, scn, device=0) as s:
        s.set_allreduce(lambda b: None)
        try:
            s.steps_async(0, 2)
            s.sync()
            s.set_xt(scn.xt0)
            s.steps_async(0, 3)
            s.sync()
            print("fixed" if fixed else "natural", "ok", s.state()["xt"][:2].ravel()[:3], flush=True)
        except Exception as e:          # noqa: BLE001
            print("fixed" if fixed else "natural", "FAIL", e, flush=True)
