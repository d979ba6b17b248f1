#!/usr/bin/env python3
"""Benchmark: PI-ADMM outer iterations/s and ms per MPC step (BASELINE.json metric).

Workloads (BASELINE.json configs; synthetic seeded tiles of the reference's two-vehicle
intersection, inputs resident in HBM before the timed region):

  default      configs[2]: 256 agents x H30 per GPU, matlab_pi preset (PI anti-windup), the
               reference's global termination scope, FIXED 100 outer iterations per MPC step
                -- the headline ``value`` -- plus, in the same line, the same
               workload under NATURAL global termination (``natural``: the latency a planner
               sees per MPC step)
  --config2    configs[1]: 64 agents x H20, casadi_default, fixed 200 outer iterations (C2)
  --config5    configs[4]: 256 agents x H50 with delay tightening
  --strong     configs[3]: 1024 agents x H30 in total, sharded over the N ranks (strong scaling);
               --split interleaved puts the two agents of every tile on different ranks (SURVEY.md
               8d C4 "adversarial": every pair crosses ranks, one all-reduce of the boundary
               exchange buffer per outer iteration)
  --crossing   coupling-heavy: 64 four-vehicle all-pairs crossings (256 agents, 384 candidate
               pairs, H30) on the graph kernel -- pairs stay active for many outer iterations
  --chain      one connected 1024-agent chain (one component split over workgroups)
  --obca       the OBCA local subproblem: 4096 local NLPs of the overtaking
               scenario per GPU, batched SQP, local NLP solves/s

One "step" = one MPC step of the full loop (x-step QPs of all agents, collision graph, pair
z-step QPs, PI + back-calculation dual update, residuals) plus propagation; the library's MPC
loop never returns to the host inside the timed region.

  python bench.py [--gpus N --steps K --warmup W] [--config2 | --config5 | --strong [--split interleaved] | --crossing] [--natural]

N > 1: one process per GPU (torch.distributed.run).  Run directly with --gpus N and no
WORLD_SIZE in the environment, this script starts ``torch.distributed.run --nproc-per-node N``
as a child process before anything touches the GPU and relays its output.  Each rank owns
whole components; the ranks join one RCCL communicator (the unique id travels over the gloo
group, which otherwise only carries the harness's barrier and max-over-ranks timer).

Prints ONE JSON line (rank 0) with roofline, latency and cpu_baseline objects.
"""
from __future__ import annotations

import argparse
import dataclasses
import glob
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"))

PEAK_HBM_GBS = 8000.0       # MI355X HBM3E (MI355X_MICROARCH.md)
PEAK_FP64_TFLOPS = 78.6     # MI355X fp64 vector (256 CU x 4 SIMD x 16 lanes x 2 x 2.4 GHz)
CLOCK_GHZ = 2.4             # max shader clock (MI355X_MICROARCH.md)
METRIC = "PI-ADMM outer iterations/sec (and ms/MPC step) at N_agents×H; 1/2/4/8 GPU"

WORKLOADS = {
    # name: (tiles per GPU or total, H, preset, max_outer, tighten, scaling)
    "c3": dict(tiles=128, H=30, preset="matlab_pi", max_outer=100, tighten=0, scaling="weak",
               desc="256 agents x H30 per GPU (128 tiles), matlab_pi preset (PI anti-windup)"),
    "c2": dict(tiles=32, H=20, preset="casadi_default", max_outer=200, tighten=0, scaling="weak",
               desc="64 agents x H20 per GPU (32 tiles), casadi_default preset (plain dual)"),
    "c5": dict(tiles=128, H=50, preset="matlab_pi", max_outer=100, tighten=1, scaling="weak",
               desc="256 agents x H50 per GPU (128 tiles), matlab_pi + delay tightening p=0.95"),
    "c4": dict(tiles=512, H=30, preset="matlab_pi", max_outer=100, tighten=0, scaling="strong",
               desc="1024 agents x H30 in total (512 tiles) sharded over the GPUs, matlab_pi preset"),
    "x4": dict(tiles=64, H=30, preset="matlab_pi", max_outer=100, tighten=0, scaling="weak", kind="crossing",
               desc="256 agents x H30 per GPU (64 four-vehicle all-pairs crossings, 384 candidate pairs), "
                    "matlab_pi preset"),
    "ch": dict(tiles=1024, H=30, preset="matlab_pi", max_outer=100, tighten=0, scaling="weak", kind="chain",
               desc="1024 agents x H30 per GPU in ONE connected chain (1023 candidate pairs; the component spans "
                    "256 workgroups of 4 agents), matlab_pi preset"),
}


def spawn_ranks(n: int) -> int:
    """Start torch.distributed.run with n ranks as a child process (before any HIP call)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # relay rank 0's JSON line on stdout; everything else the ranks print (gloo connection
    # notices, launcher messages) goes to stderr, so stdout stays ONE JSON line
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return p.wait()


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
    return 8.0 * (cnt["x_qps"] * x_doubles + cnt["z_qps"] * z_doubles)


def l2_table_bytes(cnt: dict, H: int) -> float:
    """Big mode (H > 32): the x-step polish tables G (H^2 + H) and X' (<= H1 x H)
    re-read by every x-step QP and the pair's K_s^-1 (4H^2) per pair ADMM iteration.  They are
    per-scenario state (256 agents x ~40 KB at H = 50: ~10 MB) that stays resident in L2 / MALL, so
    they are reported beside the roofline as L2 reads, not counted as HBM bytes (the PMC traffic
    says what reached HBM)."""
    if H <= 32:
        return 0.0
    H1 = H + 1
    return 8.0 * (cnt["x_qps"] * (H * H + H + H1 * H) + cnt["admm_z"] * 4 * H * H)


def latest_profile(kind: str, workload: str):
    """Newest committed profile summary profiles/<kind>_r*.json for this workload (tags sort by
    round: r01 < r01b < ... < r02 < r02b), else None."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"{kind}_r*.json")), reverse=True):
        try:
            with open(path) as f:
                tj = json.load(f)
        except (OSError, ValueError):
            continue
        if tj.get("workload") == workload:
            tj["_file"] = os.path.relpath(path, ROOT)
            return tj
    return None


def make_scenario(wl: dict, n_steps: int, rank: int = 0):
    """The workload's scenario on one rank (weak scaling: a seeded block per rank)."""
    from piadmm import scenario
    if wl.get("kind") == "crossing":
        return scenario.concat([scenario.crossing(4, wl["H"], n_steps=n_steps, seed=1000 * rank + k)
                                for k in range(wl["tiles"])])
    if wl.get("kind") == "chain":
        return scenario.crossing(wl["tiles"], wl["H"], n_steps=n_steps, seed=1000 * rank + 1, pairs="chain")
    return scenario.tiled(wl["tiles"], wl["H"], n_steps=n_steps, perturb=True, seed=1000 * rank)


def cpu_baseline(wl: dict, budget_s: float, K: int) -> dict:
    """The CPU baselines on this host, timed BEFORE anything touches the GPU.

    Primary (B-opt): oracle/piadmm_cpu.cpp -- C++ -O3 + OpenMP over tiles on
    min(16, host) threads, the GPU kernel's algorithm with exact answers equal to the oracle's
    (tests/test_cpu_bopt.py) -- on the same job as the GPU (same seeded tiles, steps 0..K-1, fixed
    iterations; its natural-termination ms per step next to it).  Second (``numpy_oracle``): the
    NumPy oracle over a process pool (oracle/cpu_parallel.py), the stand-in for the reference's
    one-QP-at-a-time Python loop (B-ref, which cannot run here: CasADi / OSQP are absent)."""
    sys.path.insert(0, ROOT)
    from piadmm import config
    n_tiles, H = wl["tiles"], wl["H"]
    cfg = config.PRESETS[wl["preset"]](H=H, fixed_iters=1, max_outer=wl["max_outer"], tighten=wl["tighten"],
                                        term_global=1)
    kind = wl.get("kind", "tiles")
    K = wl.get("cpu_steps", K)      # a bounded sample of the job's steps (the chain: all of the timed
                                    # steps -- later steps are harder, so a 2-step sample flattered the CPU)
    bopt = pool = None
    try:
        from oracle import cpu_bopt
        scn = make_scenario(wl, K)
        desc = {"crossing": f"{n_tiles} four-vehicle crossings", "chain": f"one {n_tiles}-agent chain"}.get(kind)
        bopt = cpu_bopt.time_baseline(cfg, n_tiles, (0.6 if kind == "tiles" else 1.0) * budget_s, n_steps=K, scn=scn,
                                      desc=desc)
        r = cpu_bopt.run(cfg.replace(fixed_iters=0), scn, K, bopt["cores"])
        bopt["natural_ms_per_step"] = 1e3 * r["seconds"] / K
        bopt["natural_outer_iters_per_step"] = float(r["iters"][:, 0].mean())
    except Exception as e:          # noqa: BLE001 -- report the NumPy pool alone
        print(f"bench.py: B-opt CPU baseline failed ({e})", file=sys.stderr)
    if kind == "tiles":             # the NumPy pool parallelises over two-vehicle tiles
        try:
            from oracle import cpu_parallel
            pool = cpu_parallel.time_baseline(cfg, n_tiles, 0.4 * budget_s)
        except Exception as e:          # noqa: BLE001
            print(f"bench.py: NumPy oracle pool failed ({e})", file=sys.stderr)
    if bopt is None:
        return pool
    if pool is not None:
        bopt["numpy_oracle"] = {k: pool[k] for k in ("value", "unit", "cores", "kind", "sample")}
    return bopt


def run(wl: dict, natural: bool, K: int, W: int, rank: int, world: int, local_rank: int, dist, split="components",
        share: int = 0, precision: int = 0, cold: bool = False):
    """Time K MPC steps of workload wl on this rank; returns (metrics, counters, solver info).
    share > 1 (strong scaling, one process): rank 0's share of a share-rank job alone on this GPU --
    its agents (and, interleaved, its ghosts), every collective a no-op (SURVEY.md 8e readiness)."""
    import numpy as np
    from piadmm import config, scenario
    from piadmm import dist as pdist
    from piadmm.solver import PI_ADMM_MI355X
    H, M = wl["H"], wl["max_outer"]
    cfg = config.PRESETS[wl["preset"]](H=H, fixed_iters=0 if natural else 1, max_outer=M, term_global=1,
                                       tighten=wl["tighten"], precision=precision)
    n_steps = max(K, W, 1)
    shard = None
    if wl["scaling"] == "strong":
        full = scenario.tiled(wl["tiles"], H, n_steps=n_steps, perturb=True, seed=0)
        srank, sworld = (0, share) if share > 1 else (rank, world)
        if split == "interleaved":
            shard = pdist.shard_graph(full, srank, sworld, pdist.owners_interleaved(full.n_agents, sworld))
            scn = shard.scn
            n_own = int(shard.owned.sum())
            if share > 1:
                # one rank alone: no other rank fills the ghosts' exchange slots, so the share
                # solves its ghosts' x-steps itself, on the component's second wave (a tile's two
                # agents run on its two waves at once) -- the pair QPs see the positions the
                # owners would send; the exchange stays (X, device copy, Z + X per iteration)
                shard = dataclasses.replace(shard, owned=np.ones_like(shard.owned))
        else:
            scn = pdist.shard(full, srank, sworld)
    else:
        scn = make_scenario(wl, n_steps, rank)
    from piadmm.solver import device_count
    if share > 1:
        # a rank of a multi-rank job decides the natural stop on the device after an all-reduce
        # per outer iteration (devstop_step), never in a single-rank cooperative launch
        os.environ["PIADMM_NO_COOP"] = "1"
    solver = PI_ADMM_MI355X(cfg, scn, device=local_rank % max(device_count(), 1), shard=shard)
    try:
        if dist is not None and os.environ.get("PIADMM_BENCH_TRANSPORT") == "host":
            # rehearsal transport (several ranks sharing one GPU, where RCCL refuses duplicate
            # devices): the library's host all-reduce callback over the gloo group
            import torch

            def host_allreduce(buf):
                t = torch.from_numpy(buf.copy())
                dist.all_reduce(t)
                buf[:] = t.numpy()
            solver.set_allreduce(host_allreduce)
        elif dist is not None:
            def bcast(b):
                obj = [b]
                dist.broadcast_object_list(obj, src=0)
                return obj[0]
            pdist.attach_rccl(solver, rank, world, bcast)
        # warmup: W steps from t=0 (per-scenario setup caches are built here), then the state is
        # reset (xt0, warm labels, ADMM penalties) so the timed steps replay t = 0 .. K-1
        if W > 0:
            solver.steps_async(0, W)
            solver.sync()
        solver.set_xt(scn.xt0)
        solver.reset_counters()
        if dist is not None:
            dist.barrier()
        solver.sync()
        t0 = time.perf_counter()
        ev_ms = solver.time_steps(0, K)        # hipEvents on the library's stream around the launches
        solver.sync()
        wall = time.perf_counter() - t0
        if dist is not None:
            dist.barrier()
        cnt = solver.counters()
        spl, C = solver.steps_per_launch(), max(solver.C, 1)
        N = n_own if shard is not None else solver.N
        # pairs across ranks (an X and a Z launch per outer iteration), or one component split over
        # workgroups (the same two launches, no exchange)
        xchg = (shard is not None and shard.n_slots > 0) or wl.get("kind") == "chain"
    finally:
        solver.close()
    # the cold first step: MPC step 0 on a FRESH handle, its per-scenario caches (the agents' P^-1,
    # K_s^-1 and scaling, the pairs' speed-only polish tables) built inside the timed launch -- the
    # timed steps above replay t = 0 .. K-1 after the warmup built them, while B-opt builds its own
    # inside every timed run (oracle/cpu_bopt.py).  hipEvents around that one launch.
    cold_ms = None
    if cold and dist is None and not share:
        with PI_ADMM_MI355X(cfg, scn, device=local_rank % max(device_count(), 1), shard=shard) as fresh:
            cold_ms = fresh.time_steps(0, 1)
    if dist is not None:
        import torch
        tt = torch.tensor([wall, ev_ms], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, ev_ms = float(tt[0]), float(tt[1])
    job_iters = cnt["outer_iters"] / C                  # iterations of the job (every component runs them)
    # step-kernel launches in the timed region: one persistent launch per steps_per_launch() steps,
    # or (natural termination across ranks) one per outer iteration plus one per step, or (pairs
    # across ranks) an X and a Z launch per outer iteration plus one per step
    if xchg and shard is not None and not natural:
        # fixed iterations of a sharded job: X(0), a fused Z(it) + X(it+1) launch per iteration,
        # Z(M-1), the step's last launch (piadmm_capi.cpp run_steps_phases)
        n_launch = K * (M + 1) + K
    elif xchg:
        n_launch = 2 * int(job_iters) + K
    else:
        n_launch = -(-K // spl) if spl > 1 else int(job_iters) + K
    graph = xchg or wl.get("kind") in ("crossing", "chain")
    return dict(wall=wall, ev_ms=ev_ms, job_iters=job_iters, n_launch=n_launch, spl=spl, N=N, C=C, xchg=xchg,
                kernel="pd::k_graph_step" if graph else "pd::k_mpc_step", cold_ms=cold_ms), cnt


def _obca_chunk(recs):
    """worker: the NumPy SQP oracle on a chunk of records (CPU baseline of --obca)."""
    sys.path.insert(0, ROOT)
    from oracle import obca_oracle as O
    n_conv = 0
    for rec in recs:
        p, opt = O.from_record(rec)
        n_conv += int(O.solve_local(p, opt).status == O.CONVERGED)
    return len(recs), n_conv


def obca_cpu_baseline(recs, budget_s: float) -> dict:
    """CPU baselines of --obca on the host cores, run before the GPU is touched.  Primary
    (B-opt analogue): oracle/obca_cpu.cpp -- the SQP in C++ -O3, OpenMP over the problems,
    equal to the NumPy oracle (tests/test_obca_cpu.py) -- on the WHOLE batch, best of repeats
    within the budget.  Second (``numpy_oracle``): the NumPy oracle over a process pool on a
    bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import hostinfo
    hi = hostinfo.host_cpu()
    cores = max(1, min(16, hi["threads"]))
    prim = None
    try:
        from oracle import obca_cpu
        best, reps, t_end = None, 0, time.perf_counter() + 0.6 * budget_s
        while reps < 2 or (time.perf_counter() < t_end and reps < 20):
            _, ist, dt = obca_cpu.solve(recs, cores)
            best = dt if best is None else min(best, dt)
            reps += 1
        prim = {"value": len(recs) / best, "unit": "local_nlp_solves/s", "cores": cores, "kind": "port",
                "sample": f"the whole batch ({len(recs)} problems), oracle/obca_cpu.cpp (C++ -O3 -march=x86-64-v3, "
                          f"OpenMP over problems), best of {reps}",
                "host": hostinfo.describe(hi), "converged": int((ist[:, 0] == 0).sum())}
    except Exception as e:      # noqa: BLE001
        print(f"bench.py: OBCA C++ baseline failed ({e})", file=sys.stderr)
    pool = _obca_numpy_pool(recs, 0.4 * budget_s, cores, hi)
    if prim is None:
        return pool
    prim["numpy_oracle"] = pool
    return prim


def _obca_numpy_pool(recs, budget_s, cores, hi):
    import multiprocessing as mp
    from oracle import hostinfo
    # calibrate: one worker's rate on a few problems, then a sample sized for ~budget_s
    t0 = time.perf_counter()
    _obca_chunk(recs[:8])
    per = (time.perf_counter() - t0) / 8
    n = int(min(len(recs), max(cores * 4, budget_s * cores / max(per, 1e-6))))
    sample = recs[:n]
    chunks = [sample[i::cores] for i in range(cores)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(cores) as pool:
        t0 = time.perf_counter()
        res = pool.map(_obca_chunk, chunks)
        dt = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    return {"value": done / dt, "unit": "local_nlp_solves/s", "cores": cores, "kind": "port",
            "sample": f"first {done} problems of the batch (SQP oracle, NumPy fp64) over a {cores}-process pool, "
                      f"{dt:.1f} s", "host": hostinfo.describe(hi),
            "converged": sum(r[1] for r in res)}


def main_obca(args, world, rank, local_rank):
    """--obca: the OBCA local subproblem, a batch of local NLPs of the
    two-vehicle overtaking scenario per GPU; one step = one batched SQP launch over the batch."""
    from piadmm import obca
    n = args.obca_batch
    recs = obca.scenario_batch(n, seed=rank)
    cpu = obca_cpu_baseline(recs, args.cpu_budget) if (rank == 0 and world == 1 and not args.no_cpu) else None
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from piadmm.solver import device_count
    b = obca.OBCABatch(local_rank % max(device_count(), 1))
    try:
        b.upload(recs)
        if args.warmup > 0:
            b.time(args.warmup)
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        ev_ms = b.time(args.steps)           # hipEvents around the K launches on the handle's stream
        wall = time.perf_counter() - t0
        if dist is not None:
            dist.barrier()
        res = b.download(n)
    finally:
        b.close()
    if dist is not None:
        import torch
        tt = torch.tensor([wall, ev_ms], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, ev_ms = float(tt[0]), float(tt[1])
    K = args.steps
    value = n * K * world / wall
    bytes_launch = n * (obca.REC * 8 + obca.OUT * 8 + 12)
    achieved = bytes_launch / (ev_ms / 1e3) / 1e9
    traffic = latest_profile("traffic", f"obca{n}")     # PMC bytes per launch (tools/profile_line.sh)
    line = {
        "metric": "OBCA local NLP solves/s (batched SQP, two-vehicle overtaking, N_horz 8)",
        "value": value, "unit": "local_nlp_solves/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
        "ms_per_step": wall / K * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: local problems of the reference's two-vehicle overtaking scenario (every MPC step, "
                "both vehicles, three bar_state variants; piadmm.obca.scenario_batch)",
        "config": {"workload": f"{n} OBCA local NLPs per GPU (82 variables, 35 dynamics equalities, 7 x (5a, 5b, "
                               f"norm)), one wavefront each, one launch per step",
                   "problems_per_gpu": n, "converged": int((res.status == 0).sum()),
                   "sqp_iters_mean": float(res.iters.mean()), "qp_steps_mean": float(res.qp_steps.mean()),
                   "parallelism": f"independent problems per GPU ({world} GPU(s)), no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS,
                     "traffic": traffic["hbm_bytes_per_step"] if traffic else None,
                     "traffic_source": traffic["_file"] if traffic else None, "kernel": "obca::k_obca_sqp",
                     "avg_launch_ms": ev_ms, "algorithmic_bytes_per_launch": bytes_launch,
                     "note": "latency bound: 520 doubles of HBM traffic per problem, the SQP state stays in LDS; "
                             "see DESIGN.md section 9"},
        "cpu_baseline": cpu,
    }
    if cpu is not None:
        line["speedup_vs_cpu_baseline"] = value / cpu["value"]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU-baseline timing (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-natural", action="store_true", help="skip the natural-termination co-headline")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold first step (a fresh handle's step 0)")
    ap.add_argument("--natural", action="store_true", help="natural termination as the headline itself")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--config2", action="store_true", help="BASELINE configs[1]: 64 agents x H20")
    g.add_argument("--config5", action="store_true", help="BASELINE configs[4]: H=50 with delay tightening")
    g.add_argument("--strong", action="store_true", help="BASELINE configs[3]: 1024 agents sharded over N GPUs")
    g.add_argument("--crossing", action="store_true", help="coupling-heavy: 64 four-vehicle all-pairs crossings")
    g.add_argument("--chain", action="store_true", help="one connected 1024-agent chain (component over workgroups)")
    g.add_argument("--obca", action="store_true", help="OBCA local subproblem: a batch of local NLPs (SQP)")
    ap.add_argument("--obca-batch", type=int, default=4096, help="--obca: local problems per GPU")
    ap.add_argument("--split", choices=("components", "interleaved"), default="components",
                    help="--strong: whole tiles per rank, or every tile across two ranks (boundary exchange)")
    ap.add_argument("--precision", type=int, default=0, choices=(0, 1, 2),
                    help="piadmm_config_t.precision: 2 = the x-step tables read in fp32 + one fp64 refinement "
                         "(where they live in HBM: --config5's H = 50), the configs[4] fp32 study")
    ap.add_argument("--share", type=int, default=0,
                    help="--strong on one GPU: time rank 0's share of a SHARE-rank job alone, collectives as "
                         "no-ops (interleaved: the exchange is a device copy, ghosts read zeros) -- the "
                         "per-rank compute of the strong-scaling model, DESIGN.md section 7")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:
        if args.gpus > 1:          # direct call: become the launcher, before any HIP call
            sys.exit(spawn_ranks(args.gpus))
        world = 1
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.obca:
        return main_obca(args, world, rank, local_rank)
    key = ("c2" if args.config2 else "c5" if args.config5 else "c4" if args.strong else "x4" if args.crossing
           else "ch" if args.chain else "c3")
    wl = WORKLOADS[key]
    # the CPU baseline first, on the host cores, before this process touches the GPU (its worker
    # pool is started with the spawn method)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(wl, args.cpu_budget, args.steps)

    from piadmm import _lib
    lib = _lib.load()                       # HIP runtime loaded before torch (same SONAME)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

    H, M = wl["H"], wl["max_outer"]
    K, W = args.steps, args.warmup
    if args.share and (not args.strong or world != 1):
        raise SystemExit("bench.py: --share needs --strong on one GPU")
    m, cnt = run(wl, args.natural, K, W, rank, world, local_rank, dist, args.split, args.share, args.precision,
                 cold=not args.no_cold)

    # value = units all ranks processed / the max-over-ranks wall time.  Weak scaling: one unit =
    # one outer iteration of a rank's (256-agent) block, so all ranks processed world x job
    # iterations; strong scaling: the unit is an outer iteration of the whole 1024-agent job.
    units = m["job_iters"] * (world if wl["scaling"] == "weak" else 1)
    if args.share:
        # one rank's share alone: its iterations are the job's (every rank runs them), but only
        # 1/share of the job's agents -- the rate is the share's, not a scaling claim
        wl = dict(wl, desc=wl["desc"] + f"; rank 0's SHARE of a {args.share}-rank job alone on one GPU "
                                        f"({args.split}), collectives as no-ops")
    value = units / m["wall"]
    agents_job = m["N"] * world if wl["scaling"] == "weak" else 2 * wl["tiles"]
    avg_launch_s = (m["ev_ms"] / 1e3) / m["n_launch"]
    bytes_launch = algorithmic_bytes(cnt, H) / m["n_launch"]
    achieved = bytes_launch / avg_launch_s / 1e9
    wname = f"{ {'crossing': 'crossing4x', 'chain': 'chain'}.get(wl.get('kind'), 'tiled')}{wl['tiles']}_H{H}_{wl['preset']}_fixed{M}" + (
        "_tight" if wl["tighten"] else "")
    traffic = latest_profile("traffic", wname) if not args.natural else None
    traffic_launch = traffic["hbm_bytes_per_step"] * K / m["n_launch"] if traffic else None
    sq = latest_profile("sq", wname) if not args.natural else None

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "outer_iters/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": m["wall"] / K * 1e3,
        "higher_is_better": True,
        "scaling": wl["scaling"],
        "vs_baseline": None,
        "dtype": "f64" if args.precision != 2 else "f64 (x-step tables read as f32, one f64 refinement)",
        "data": (f"synthetic: seeded four-vehicle all-pairs crossings (lanes 0, 1 = the reference's 2-vehicle "
                 f"intersection; {agents_job} agents in the job)" if wl.get("kind") == "crossing" else
                 f"synthetic: one seeded {agents_job}-vehicle chain on the crossing's lanes (candidate pairs (k, k+1))"
                 if wl.get("kind") == "chain" else
                 f"synthetic: seeded tiles of the reference 2-vehicle intersection ({agents_job} agents in the job)"),
        "config": {
            "workload": wl["desc"] + ", " + (
                f"global natural termination (max {M} outer iterations)" if args.natural else
                f"{M} outer iterations per MPC step (fixed), global residual history"),
            "agents_per_gpu": m["N"], "agents_total": agents_job, "horizon": H,
            "outer_iters_per_step": m["job_iters"] / K,
            "job_outer_iters_per_s": m["job_iters"] / m["wall"],
            "agent_qps_per_s": cnt["x_qps"] * world / m["wall"],
            "transport": ("host all-reduce over gloo (rehearsal)" if os.environ.get("PIADMM_BENCH_TRANSPORT") == "host"
                          else "RCCL") if world > 1 else None,
            "parallelism": (f"agents sharded over {world} GPU(s), every tile across two ranks: one all-reduce of "
                            f"the boundary exchange buffer per outer iteration + " if m["xchg"] else
                            f"components sharded over {world} GPU(s); ") + (
                ("one RCCL all-reduce of the termination partials per outer iteration" if world > 1 else
                 "stop test in-kernel behind a grid barrier (cooperative launch)") if args.natural else
                "one RCCL all-reduce of the residual history per persistent launch") + (
                " (single rank: none)" if world == 1 else ""),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBS, "traffic": traffic_launch,
            "kernel": m["kernel"], "avg_launch_ms": avg_launch_s * 1e3,
            "steps_per_launch": m["spl"], "launches": m["n_launch"],
            "algorithmic_bytes_per_launch": bytes_launch,
            "l2_table_bytes_per_launch": l2_table_bytes(cnt, H) / m["n_launch"],
            "traffic_source": traffic["_file"] if traffic else None,
            "note": "not bandwidth-bound: the algorithmic bytes stay in LDS; see latency and DESIGN.md §5",
        },
        "inner": {
            "x_qps_per_step": cnt["x_qps"] / K, "z_qps_per_step": cnt["z_qps"] / K,
            "z_qps_per_outer_iter": cnt["z_qps"] / max(m["job_iters"], 1),
            "admm_iters_per_xqp": cnt["admm_x"] / max(cnt["x_qps"], 1),
            "admm_iters_per_zqp": cnt["admm_z"] / max(cnt["z_qps"], 1),
            "pdas_solves_per_xqp": cnt["pdas_x"] / max(cnt["x_qps"], 1),
            "pdas_solves_per_zqp": cnt["pdas_z"] / max(cnt["z_qps"], 1),
            "inexact_qps": cnt["inexact"],
        },
        "latency": None,
        "fp64": None,
        "cpu_baseline": None,
    }
    if m["cold_ms"] is not None:
        line["cold_first_step"] = {
            "ms": m["cold_ms"],
            "note": "MPC step 0 on a fresh handle, per-scenario caches (P^-1, K_s^-1, pair polish tables) built "
                    "inside (hipEvents); ms_per_step replays t = 0.. after the warmup built them, as a planner "
                    "re-solving one scenario does -- B-opt builds its caches inside every timed run"}
    # latency model: the kernel runs one dependent QP chain per wave; cycles per wave per outer
    # iteration from this run's launch time, against the issue bound from the committed SQ counters
    # (VALU wave-instructions x 4 cycles: a wave64 fp64 VALU op occupies a 16-lane SIMD 4 cycles)
    cyc_iter = avg_launch_s * m["n_launch"] * CLOCK_GHZ * 1e9 / max(m["job_iters"], 1)
    lat = {"cycles_per_outer_iter_per_wave": cyc_iter, "clock_ghz_assumed": CLOCK_GHZ}
    if sq:
        lat.update({k: sq[k] for k in ("valu_insts_per_wave_iter", "lds_insts_per_wave_iter",
                                       "salu_insts_per_wave_iter", "wave_cycles_per_wave_iter") if k in sq})
        if "valu_insts_per_wave_iter" in sq:
            bound = 4.0 * sq["valu_insts_per_wave_iter"]
            lat["issue_bound_cycles"] = bound
            lat["frac"] = bound / cyc_iter
            if sq.get("waves", 0) > 2 * m["C"]:
                # three waves per component (two agent waves + the pair wave, which mostly waits at
                # the barriers): the VALU work is the agent waves', so their issue bound is 3/2 of
                # the average over all waves
                nw = sq["waves"] / max(m["C"], 1)
                lat["waves_per_component"] = nw
                lat["issue_bound_cycles_agent_wave"] = bound * nw / 2.0
                lat["frac_agent_wave"] = bound * nw / 2.0 / cyc_iter
        lat["source"] = sq["_file"]
        if "fp64_flops_per_step" in sq:
            gf = sq["fp64_flops_per_step"] * K / (m["ev_ms"] / 1e3) / 1e9
            line["fp64"] = {"gflops": gf, "peak_tflops": PEAK_FP64_TFLOPS, "frac": gf / (PEAK_FP64_TFLOPS * 1e3),
                            "source": sq["_file"] + " (SQ_INSTS_VALU_{ADD,MUL,FMA}_F64 x 64 lanes; FMA = 2)"}
    line["latency"] = lat

    if not args.natural and not args.no_natural:
        mn, cn = run(wl, True, K, W, rank, world, local_rank, dist, args.split, args.share, args.precision)
        line["natural"] = {
            "ms_per_step": mn["wall"] / K * 1e3,
            "outer_iters_per_step": mn["job_iters"] / K,
            "outer_iters_per_s": mn["job_iters"] * (world if wl["scaling"] == "weak" else 1) / mn["wall"],
            "z_qps_per_outer_iter": cn["z_qps"] / max(mn["job_iters"], 1),
            "steps_per_launch": mn["spl"],
            "note": "same workload, the reference's stop test on (casadi/main.py:174-178): the per-step latency",
        }
    if cpu is not None:
        line["cpu_baseline"] = cpu
        line["speedup_vs_cpu_baseline"] = value / cpu["value"]
        if "natural" in line and cpu.get("natural_ms_per_step"):
            line["natural"]["speedup_vs_cpu_baseline"] = cpu["natural_ms_per_step"] / line["natural"]["ms_per_step"]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    del lib
    if os.environ.get("PIADMM_BENCH_UNLOAD") == "1":
        _lib.unload()
    if os.environ.get("PIADMM_BENCH_RESET") == "1":
        # diagnostic (the exit fault under rocprofv3 after a cooperative launch):
        # tear the device's HIP state down while the profiler is still attached
        import ctypes
        ctypes.CDLL("libamdhip64.so").hipDeviceReset()
    if os.environ.get("PIADMM_BENCH_MAPS"):
        # diagnostic: the process's mappings at exit (which libraries the exit handlers run in)
        with open("/proc/self/maps") as f, open(os.environ["PIADMM_BENCH_MAPS"], "w") as g:
            g.write(f.read())


if __name__ == "__main__":
    main()
