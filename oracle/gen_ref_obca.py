"""Generate tests/golden/ref_obca.npz by executing the reference's OWN OBCA-path helpers.

TEST INFRASTRUCTURE (fixture generator; run in the build container, never on the GPU box).

`Distributed_planner/decentralized/optimizer.py` imports casadi at module level (absent here,
SURVEY 8c, an ordinary ModuleNotFoundError), so the module is not imported.  This script parses
it with `ast` and executes, unchanged, the pieces that need only NumPy:
  * OBCAOptimizer.iterate_next_state (:337-344)  -- the receding-horizon shift of bar_state;
  * OBCAOptimizer.mid_state (:351-373)           -- the initial bar_state, incl. the hard-coded
                                                    lamb_ij;
and imports `decentralized/veh_config.py` by file path (math + numpy only) for
VehicleConfig() and ref_traj_gen (:30-47).  Nothing from CasADi is stubbed.

Usage: python oracle/gen_ref_obca.py [/root/reference]
"""
from __future__ import annotations

import ast
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "ref_obca.npz")


def load(ref_root):
    base = os.path.join(ref_root, "Distributed_planner", "decentralized")
    spec = importlib.util.spec_from_file_location("ref_veh_config", os.path.join(base, "veh_config.py"))
    vc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(vc)
    path = os.path.join(base, "optimizer.py")
    tree = ast.parse(open(path).read(), filename=path)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "OBCAOptimizer")
    fn = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "iterate_next_state")
    ms = next(n for n in cls.body if isinstance(n, ast.ClassDef) and n.name == "mid_state")
    ns = {"np": np}
    exec(compile(ast.Module(body=[fn, ms], type_ignores=[]), path, "exec"), ns)
    return vc, ns["iterate_next_state"], ns["mid_state"]


def main(ref_root="/root/reference"):
    vc, iterate_next_state, mid_state = load(ref_root)
    cfg = vc.VehicleConfig()
    refs = cfg.ref_traj_gen()
    outer = types.SimpleNamespace(num_veh=2, N_horz=8, n_states=5, n_loc_lambda=4, n_dual_variable=4)
    m0 = mid_state(outer)
    rng = np.random.default_rng(20241017)
    bar = types.SimpleNamespace(
        Z_bar=rng.standard_normal((2, 7, 9)), A=rng.standard_normal((2, 7, 4, 2)), b=rng.standard_normal((2, 7, 4)),
        lamb_bar=rng.standard_normal((2, 7, 9)), lamb_ij=rng.standard_normal((2, 7, 4)),
        local_x=rng.standard_normal((2, 7, 5)))
    inp = {k: getattr(bar, k).copy() for k in ("Z_bar", "A", "b", "lamb_bar", "lamb_ij", "local_x")}
    nxt = iterate_next_state(None, bar)
    rec = dict(ref0=refs[0], ref1=refs[1],
               cfg=np.array([cfg.length, cfg.width, cfg.lf, cfg.lr, cfg.max_front_wheel_angle, cfg.dt, cfg.T,
                             cfg.max_acc, cfg.max_v, cfg.max_steer_rate, cfg.avg_delay, cfg.var_delay, cfg.prob]),
               mid_Z_bar=m0.Z_bar, mid_A=m0.A, mid_b=m0.b, mid_lamb_bar=m0.lamb_bar, mid_lamb_ij=m0.lamb_ij,
               mid_local_x=m0.local_x)
    for k, v in inp.items():
        rec["in_" + k] = v
        rec["out_" + k] = getattr(nxt, k)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **rec, source=np.array(
        "decentralized/veh_config.py:7-47 (imported), decentralized/optimizer.py:337-373 (executed)"))
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main(*sys.argv[1:])
