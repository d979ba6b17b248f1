#!/usr/bin/env python3
"""Benchmark: PI-ADMM outer iterations/s at 256 agents x H=30 per GPU (BASELINE.json configs[2]).

One "step" = one MPC step of the full PI anti-windup loop (matlab_pi preset:
x-step QPs of all agents, collision graph, pair z-step QPs, PI + back-calculation
dual update, residuals) run for a fixed ``max_outer`` = 100 outer iterations
(termination disabled), plus propagation.  Inputs (scenario,
states) are resident in HBM before the timed region; the library's MPC loop
never returns to the host inside it.

  python bench.py [--gpus N --steps K --warmup W]

The job runs with the reference's global termination scope (term_global, quirk B9):
all agents of all ranks form one ADMM job whose residual history (rk, sk summed over
every pair) is the reference's.  With fixed iterations that is one fused launch per
MPC step plus one RCCL all-reduce of the 2 x 100 residual partials over xGMI.

N>1: launched by torch.distributed.run, one process per GPU; each rank owns its
own 128 intersection tiles (256 agents), so per-GPU work is fixed ("weak").
Components never straddle ranks; the ranks join one RCCL communicator (the unique
id travels over torch.distributed's gloo group, which is otherwise only the
harness's barrier and max-over-ranks timer).

--natural: natural termination instead, reported as its own line: on one rank the stop
test runs in-kernel behind a grid barrier (cooperative launch, several steps per launch);
across ranks one launch + one RCCL all-reduce of the termination partials per outer
iteration, host decision.

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"))

import numpy as np  # noqa: E402

from piadmm import _lib, config, scenario  # noqa: E402

N_TILES = 128          # 256 agents
H = 30
MAX_OUTER = 100
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def algorithmic_bytes(cnt: dict, H: int) -> float:
    """Bytes the path must move per SURVEY.md 8(d), from the device work counters.

    x-step QP (per agent per outer iteration): reads xt(3) + spd(1) + ref 2(H+1)
      + per neighbour hat 2(H+1) + lam 2(H+1); writes u (H) + pos_old 2(H+1)
      = 282 doubles at H=30 (deg 1).
    z-step (per active pair per outer iteration): reads p_i, p_j 4(H+1) + lam pair
      4(H+1) + xt 6 + seeds 4; writes hat pair 4(H+1) + lam, S, D pair 12(H+1)
      = 754 doubles at H=30.
    """
    H1 = H + 1
    x_doubles = 3 + 1 + 2 * H1 + (2 * H1 + 2 * H1) + H + 2 * H1
    z_doubles = 4 * H1 + 4 * H1 + 6 + 4 + 4 * H1 + 12 * H1
    b = 8.0 * (cnt["x_qps"] * x_doubles + cnt["z_qps"] * z_doubles)
    if H > 32:
        # big mode: the polish tables G (H^2+H) and X' (<= H1 x H) of each x-step QP
        # and the pair's K_s^-1 (4H^2) per pair ADMM iteration stream from L2 / HBM
        b += 8.0 * (cnt["x_qps"] * (H * H + H + H1 * H) + cnt["admm_z"] * 4 * H * H)
    return b


def latest_traffic(workload: str):
    """HBM bytes per launch from the newest committed PMC summary (profiles/traffic_<tag>.json,
    tags sort by round: r01 < r01b < r01c ...) for this workload, else None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json")), reverse=True):
        try:
            with open(path) as f:
                tj = json.load(f)
        except (OSError, ValueError):
            continue
        if tj.get("workload") == workload and tj.get("hbm_bytes_per_step"):
            return tj["hbm_bytes_per_step"]
    return None


def cpu_baseline(n_tiles: int, budget_s: float, H: int = H, tighten: int = 0) -> dict:
    """Time the NumPy oracle (the reference's loop structure, one QP at a time) on a bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import piadmm_oracle as O
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:      # pragma: no cover
        threadpool_limits = None
    cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=MAX_OUTER, tighten=tighten)
    scn = scenario.tiled(N_TILES, H, n_steps=4)
    done_tiles = 0
    t_used = 0.0
    limit = threadpool_limits(limits=1) if threadpool_limits else None   # one core
    try:
        orc = O.Oracle(cfg, scn)
        for c in range(min(n_tiles, orc.n_comp)):
            orc.xt = scn.xt0.copy()
            orc.t = 0
            t0 = time.perf_counter()
            orc.mpc_step(components=[c])
            t_used += time.perf_counter() - t0
            done_tiles += 1
            if t_used > budget_s:
                break
    finally:
        if limit is not None:
            limit.restore_original_limits()
    per_tile_iter = t_used / (done_tiles * MAX_OUTER)
    it_s = 1.0 / (per_tile_iter * N_TILES)
    return {"value": it_s, "unit": "outer_iters/s", "cores": 1, "kind": "port",
            "sample": f"NumPy oracle (oracle/piadmm_oracle.py, exact active-set QPs, one QP at a time "
                      f"like casadi/main.py), MPC step t=0 of {done_tiles} of {N_TILES} tiles x "
                      f"{MAX_OUTER} outer iterations, {t_used:.1f} s, scaled linearly to 128 tiles; "
                      f"host {platform.processor() or platform.machine()}, {os.cpu_count()} cpus visible"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    # default warmup = default steps: the warmup launch and the timed launch of k_mpc_step have
    # the same size, so rocprofv3's per-kernel average over the run compares with avg_launch_ms
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle timing (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--natural", action="store_true", help="natural (global) termination, not the headline")
    ap.add_argument("--config5", action="store_true",
                    help="BASELINE configs[4]: H=50 with delay tightening (not the headline)")
    args = ap.parse_args()
    H = 50 if args.config5 else globals()["H"]
    tighten = 1 if args.config5 else 0

    lib = _lib.load()                       # HIP runtime loaded before torch (same SONAME)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from piadmm.solver import PI_ADMM_MI355X
    K, W = args.steps, args.warmup
    n_steps = max(K, W, 1)
    cfg = config.matlab_pi(H=H, fixed_iters=0 if args.natural else 1, max_outer=MAX_OUTER, term_global=1,
                           tighten=tighten)
    scn = scenario.tiled(N_TILES, H, n_steps=n_steps, perturb=True, seed=1000 * rank)
    solver = PI_ADMM_MI355X(cfg, scn, device=local_rank)
    if dist is not None:
        from piadmm import dist as pdist

        def bcast(b):
            obj = [b]
            dist.broadcast_object_list(obj, src=0)
            return obj[0]
        pdist.attach_rccl(solver, rank, world, bcast)

    # warmup: W steps from t=0, then reset the state so the timed steps repeat t=0..K-1
    if W > 0:
        solver.steps_async(0, W)
        solver.sync()
    solver.set_xt(scn.xt0)
    solver.reset_counters()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    solver.sync()
    t0 = time.perf_counter()
    ev_ms = solver.time_steps(0, K)          # hipEvents on the library's stream around the K launches
    solver.sync()
    wall = time.perf_counter() - t0
    barrier()
    cnt = solver.counters()
    if dist is not None:
        import torch
        tt = torch.tensor([wall, ev_ms], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, ev_ms = float(tt[0]), float(tt[1])

    outer_total = world * cnt["outer_iters"] / max(solver.C, 1)      # job iterations x ranks
    value = outer_total / wall
    # k_mpc_step launches in the timed region: one persistent launch per steps_per_launch()
    # MPC steps (fixed iterations; natural global termination on one rank, where the stop
    # test runs in-kernel behind a grid barrier), or -- natural termination across ranks --
    # one per outer iteration plus one per step (each launch's share of the time taken equal)
    spl = solver.steps_per_launch()
    n_launch = -(-K // spl) if spl > 1 else int(cnt["outer_iters"] / max(solver.C, 1)) + K
    avg_launch_s = (ev_ms / 1e3) / n_launch
    bytes_launch = algorithmic_bytes(cnt, H) / n_launch
    achieved = bytes_launch / avg_launch_s / 1e9

    traffic_step = latest_traffic(f"tiled{N_TILES}_H{H}_matlab_pi_fixed{MAX_OUTER}") if not args.natural else None
    traffic = traffic_step * K / n_launch if traffic_step else None

    line = {
        "metric": "PI-ADMM outer iterations/sec (and ms/MPC step) at N_agents×H; 1/2/4/8 GPU",
        "value": value,
        "unit": "outer_iters/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": wall / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: 128 seeded tiles of the reference 2-vehicle intersection per GPU",
        "config": {
            "workload": f"256 agents x H{H} per GPU (128 tiles), matlab_pi preset (PI anti-windup), "
                        + ("delay tightening p=0.95 (configs[4]), " if tighten else "")
                        + (f"global natural termination (max {MAX_OUTER} outer iterations)" if args.natural else
                           f"{MAX_OUTER} outer iterations per MPC step (fixed), global residual history"),
            "agents_per_gpu": 2 * N_TILES, "horizon": H,
            "outer_iters_per_step": outer_total / world / K,
            "parallelism": f"components sharded over {world} GPU(s); " + (
                ("one RCCL all-reduce of the termination partials per outer iteration" if world > 1 else
                 "stop test in-kernel behind a grid barrier (cooperative launch)") if args.natural else
                "one RCCL all-reduce of the residual history per MPC step") + (" (single rank: none)" if world == 1 else ""),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
            "kernel": "pd::k_mpc_step", "avg_launch_ms": avg_launch_s * 1e3,
            "steps_per_launch": spl, "launches": n_launch,
            "algorithmic_bytes_per_launch": bytes_launch,
            "note": "latency-bound: one dependent ADMM/PDAS chain per wave; see DESIGN.md",
        },
        "inner": {
            "x_qps_per_step": cnt["x_qps"] / K, "z_qps_per_step": cnt["z_qps"] / K,
            "admm_iters_per_xqp": cnt["admm_x"] / max(cnt["x_qps"], 1),
            "admm_iters_per_zqp": cnt["admm_z"] / max(cnt["z_qps"], 1),
            "pdas_solves_per_xqp": cnt["pdas_x"] / max(cnt["x_qps"], 1),
            "pdas_solves_per_zqp": cnt["pdas_z"] / max(cnt["z_qps"], 1),
            "inexact_qps": cnt["inexact"],
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(N_TILES, args.cpu_budget, H, tighten)
        line["speedup_vs_cpu_baseline"] = value / line["cpu_baseline"]["value"]
    solver.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    del lib


if __name__ == "__main__":
    main()
