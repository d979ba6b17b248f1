"""All-cores CPU baseline for bench.py: the NumPy oracle over a process pool.

TEST / MEASUREMENT INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` leg).  The reference loop
(casadi/main.py:43-201) is sequential Python with one CasADi/OSQP solve per QP and cannot run
here; its restatement, oracle/piadmm_oracle.py, solves each QP exactly with a
dense active set.  Components (tiles) are independent under per-component termination, so the
oracle parallelises over them without changing a number: worker w runs tiles w, w + P, ...,
each through MPC steps 0 .. n_steps-1 (the fixed-iteration bench mode), one process per host
core with BLAS pinned to one thread.  Throughput = the workers' tile-iterations per second of
compute (each over its own busy time) summed over the pool, divided by the job's tile count =
outer iterations per second of the whole job.

The pool must start before the calling process touches the GPU (bench.py runs it first): the
workers are started with the "spawn" method, i.e. fresh interpreters.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time

import numpy as np


def _worker(args):
    cfg, n_tiles, H, n_steps, tile_ids, deadline = args
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=1):
        from oracle import piadmm_oracle as O
        from piadmm import scenario
        done_iters = 0
        busy = 0.0
        tiles_done = 0
        for k in tile_ids:
            if time.time() > deadline:
                break
            scn = scenario.tiled(n_tiles, H, n_steps=n_steps)
            sub = scenario.Scenario(spd=scn.spd[2 * k:2 * k + 2], xt0=scn.xt0[2 * k:2 * k + 2],
                                    ref=scn.ref[2 * k:2 * k + 2], edges=np.array([[0, 1]], np.int32),
                                    n_steps=scn.n_steps)
            orc = O.Oracle(cfg, sub)
            t0 = time.perf_counter()
            for _ in range(n_steps):
                r = orc.mpc_step()
                done_iters += int(r.iters[0])
            busy += time.perf_counter() - t0
            tiles_done += 1
        return done_iters, busy, tiles_done


def time_baseline(cfg, n_tiles: int, budget_s: float, n_steps: int = 5, workers: int | None = None) -> dict:
    """Outer iterations per second of the n_tiles-tile job on all host cores (bounded sample)."""
    from oracle import hostinfo
    hi = hostinfo.host_cpu()
    workers = workers or hi["threads"]
    ctx = mp.get_context("spawn")
    deadline = time.time() + budget_s
    jobs = [(cfg, n_tiles, cfg.H, n_steps, list(range(w, n_tiles, workers)), deadline) for w in range(workers)]
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_worker, jobs)
    wall = time.perf_counter() - t0
    iters = sum(r[0] for r in res)
    tiles = sum(r[2] for r in res)
    busy = sum(r[1] for r in res)
    # per-worker rates summed: each worker's own compute time (its interpreter start-up excluded)
    tile_iter_s = sum(r[0] / r[1] for r in res if r[1] > 0)
    return {"value": tile_iter_s / n_tiles, "unit": "outer_iters/s", "cores": workers, "kind": "port",
            "sample": f"NumPy oracle (oracle/piadmm_oracle.py: exact active-set QPs, one QP at a time like "
                      f"casadi/main.py) on a pool of {workers} processes x 1 BLAS thread, {tiles} of {n_tiles} "
                      f"tiles x MPC steps 0..{n_steps - 1} x {cfg.max_outer} outer iterations (fixed) in "
                      f"{wall:.1f} s wall ({busy:.0f} core-s of compute); job rate = sum of the workers' tile-iterations/s "
                      f"/ {n_tiles}; {hostinfo.describe(hi)}", "host": hi}
