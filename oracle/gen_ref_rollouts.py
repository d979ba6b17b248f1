"""Generate tests/golden/ref_rollouts.npz by executing the reference's OWN numeric rollouts.

TEST INFRASTRUCTURE (fixture generator; run in the build container, never on the GPU box).

The reference module ``casadi/PI_ADMM_class.py`` cannot be imported here: it
imports ``bunch`` and ``casadi`` at module level and neither is installed
(an ordinary ModuleNotFoundError).  Its two numeric rollout
functions, ``dynamic_update_local`` (:45-70) and ``dynamic_update_edge`` (:77-105),
need only NumPy when called with ``if_SX=0``.  This script parses the
reference source with ``ast``, takes exactly those two function definitions
unchanged, and runs them on seeded inputs with a plain parameter namespace in
place of the ``Bunch`` the reference's constructor would build.  Nothing from
CasADi is stubbed: the ``if_SX=1`` branches are never executed.

The inputs and the reference's outputs are written as data to
tests/golden/ref_rollouts.npz; tests/test_oracle.py checks
oracle.piadmm_oracle.rollout_linear / rollout_nonlinear against them.

Usage: python oracle/gen_ref_rollouts.py [/root/reference]
"""
from __future__ import annotations

import ast
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "ref_rollouts.npz")


def load_reference_rollouts(ref_root: str):
    path = os.path.join(ref_root, "casadi", "PI_ADMM_class.py")
    src = open(path).read()
    tree = ast.parse(src, filename=path)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "PI_ADMM_CASADI")
    wanted = {"dynamic_update_local", "dynamic_update_edge"}
    fns = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in wanted]
    assert {f.name for f in fns} == wanted, "reference functions not found"
    mod = ast.Module(body=fns, type_ignores=[])
    ns = {"np": np, "ca": None}   # ca is only touched by the if_SX=1 branches (never run here)
    exec(compile(mod, path, "exec"), ns)
    return ns["dynamic_update_local"], ns["dynamic_update_edge"]


def main(ref_root: str = "/root/reference"):
    dul, due = load_reference_rollouts(ref_root)
    rng = np.random.default_rng(20240601)
    rec = {k: [] for k in ("H", "xt", "u", "spd", "loc_x", "loc_y", "loc_th", "edge_x", "edge_y", "edge_th")}
    cases = []
    for H in (8, 10, 15, 20, 30):
        for rep in range(4):
            cases.append(H)
    for H in cases:
        # reference parameters (PI_ADMM_class.py:15-28) with num_ho = H, two vehicles
        param = types.SimpleNamespace(dt=0.1, L=1, num_ho=H, num_veh=2, spd=np.array([4, 8]))
        obj = types.SimpleNamespace(param=param)
        xt = np.array([[-10, 0, 0], [0, 20, -np.pi / 2]], dtype=np.float64)
        xt = xt + rng.uniform(-1, 1, size=(2, 3)) * np.array([2.0, 2.0, 0.5])
        u = np.round(rng.uniform(-np.pi / 6, np.pi / 6, size=(2, H)), 4)
        lx, ly, lth = [], [], []
        for i in range(2):
            x, y, th = dul(obj, xt[i], u[i].reshape(1, H), i, 0)   # numeric branch: u[0][k]
            lx.append(x)
            ly.append(y)
            lth.append(th)
        ex, ey, eth = due(obj, xt, u, 0)
        rec["H"].append(H)
        rec["xt"].append(xt)
        rec["u"].append(np.pad(u, ((0, 0), (0, 30 - H))))
        rec["spd"].append(param.spd.astype(np.float64))
        pad = lambda a: np.pad(np.asarray(a, np.float64), ((0, 0), (0, 31 - (H + 1))))  # noqa: E731
        rec["loc_x"].append(pad(lx))
        rec["loc_y"].append(pad(ly))
        rec["loc_th"].append(pad(lth))
        rec["edge_x"].append(pad(ex))
        rec["edge_y"].append(pad(ey))
        rec["edge_th"].append(pad(eth))
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **{k: np.asarray(v) for k, v in rec.items()},
                        source=np.array("casadi/PI_ADMM_class.py:45-105 (numeric branches, executed)"))
    print(f"wrote {OUT} ({len(cases)} cases)")


if __name__ == "__main__":
    main(*sys.argv[1:])
