"""Development diagnostic (not shipped): per-iteration cost of the graph kernel against the fused
kernel on the tiled bench workload (PIADMM_GRAPH=1), and of the coupling-heavy crossing workload."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402


def timeit(cfg, scn, steps, graph=False):
    if graph:
        os.environ["PIADMM_GRAPH"] = "1"
    s = PI_ADMM_MI355X(cfg, scn)
    os.environ.pop("PIADMM_GRAPH", None)
    s.steps_async(0, 2)
    s.sync()
    s.set_xt(scn.xt0)
    s.reset_counters()
    ms = s.time_steps(0, steps)
    c = s.counters()
    s.close()
    return ms / steps, c


H = 30
steps = 4
for M in (100, 10):
    cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=M, term_global=1)
    scn = scenario.tiled(128, H, n_steps=steps + 2)
    for g in (False, True):
        ms, c = timeit(cfg, scn, steps, g)
        print(f"tiles M={M} graph={g}: {ms:.3f} ms/step  {1e3 * ms / M:.1f} us/iter  {c}", flush=True)
    scn = scenario.concat([scenario.crossing(4, H, n_steps=steps + 2, seed=k) for k in range(64)])
    ms, c = timeit(cfg, scn, steps, True)
    print(f"crossing M={M}: {ms:.3f} ms/step  {1e3 * ms / M:.1f} us/iter  {c}", flush=True)
    scn = scenario.concat([scenario.crossing(4, H, n_steps=steps + 2, seed=k, pairs="chain") for k in range(64)])
    ms, c = timeit(cfg, scn, steps, True)
    print(f"chain4 M={M}: {ms:.3f} ms/step  {1e3 * ms / M:.1f} us/iter  {c}", flush=True)
