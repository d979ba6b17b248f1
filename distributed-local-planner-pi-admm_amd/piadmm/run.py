"""Command-line MPC run on the GPU: the counterpart of running ``casadi/main.py``.

  python -m piadmm.run --preset casadi_default --H 15 [--tiles 1] [--steps 35]
                       [--out run] [--plot run.png] [--quiet]

Prints the reference's per-step line (``casadi/main.py:193-196``), writes the run record
(``piadmm.io.save_run``: ``run.npz`` + ``run.json``) and, with ``--plot``, the reference's
trajectory scatter (``casadi/main.py:206-220``).  Needs an MI355X; there is no CPU fallback.
"""
from __future__ import annotations

import argparse
import sys

from . import config, io, scenario


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m piadmm.run")
    ap.add_argument("--preset", choices=sorted(config.PRESETS), default="casadi_default")
    ap.add_argument("--H", type=int, default=15)
    ap.add_argument("--tiles", type=int, default=1, help="copies of the two-vehicle intersection")
    ap.add_argument("--steps", type=int, default=None, help="MPC steps (default: the reference's Nt/dt - H)")
    ap.add_argument("--term-global", type=int, default=1)
    ap.add_argument("--warm-duals", type=int, default=0)
    ap.add_argument("--tighten", type=int, default=0)
    ap.add_argument("--out", default=None, help="write <out>.npz and <out>.json")
    ap.add_argument("--plot", default=None, help="write the trajectory scatter to this PNG")
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args(argv)

    from .solver import PI_ADMM_MI355X
    cfg = config.PRESETS[args.preset](H=args.H, term_global=args.term_global, warm_duals=args.warm_duals,
                                     tighten=args.tighten)
    scn = (scenario.intersection(args.H, args.steps) if args.tiles == 1
           else scenario.tiled(args.tiles, args.H, n_steps=args.steps))
    n = scn.n_steps if args.steps is None else args.steps
    rec = io.RunRecorder(meta={"preset": args.preset, "H": args.H, "tiles": args.tiles, "steps": n,
                               "term_global": args.term_global, "warm_duals": args.warm_duals,
                               "tighten": args.tighten})
    with PI_ADMM_MI355X(cfg, scn) as s:
        for k in range(n):
            r = s.mpc_step()
            lam = s.state()["lam"]
            rec.add(r.xt, r.u, r.iters, r.resid, lam)
            if not args.quiet:
                print(io.step_line(k, r.iters, float(lam.max()) if lam.size else 0.0,
                                   float(lam.min()) if lam.size else 0.0, cfg.rho, r.xt), flush=True)
    run = rec.record()
    if args.out:
        npz, js = io.save_run(args.out, run)
        print(f"wrote {npz}, {js}")
    if args.plot:
        print(f"wrote {io.plot_run(run, args.plot)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
