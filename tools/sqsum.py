"""Sum the SQ counters of tools/sqpmc.sh over the TIMED pd::k_mpc_step dispatch of bench.py
(--no-natural: the warmup launch, then the timed launch = the last dispatch), per wave and per
outer iteration, and write profiles/sq_<tag>.json for bench.py's latency / fp64 objects.

usage: python tools/sqsum.py <gpurun_out/sq_tag> <tag> [steps=20] [outer=100] [waves=256]
SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles (x4 = cycles); SQ_INSTS_* count wave
instructions; fp64 flops = 64 lanes x (ADD + MUL + TRANS + 2 FMA) wave instructions (all lanes
counted, masked-off lanes included: an upper bound on useful flops)."""
import collections
import csv
import glob
import json
import os
import sys

out, tag = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
outer = int(sys.argv[4]) if len(sys.argv) > 4 else 100
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tot = collections.OrderedDict()
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_mpc_step" in r.get("Kernel_Name", ""):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if per:
        tot.update(per[max(per)])
waves = tot.get("SQ_WAVES") or 256.0
iters = float(steps * outer)
for k, v in tot.items():
    print(f"{k:24s} {v:16.0f}   per wave {v / waves:12.1f}   per wave-iteration {v / waves / iters:10.2f}")
res = {"workload": "tiled128_H30_matlab_pi_fixed100", "kernel": "pd::k_mpc_step", "steps": steps,
       "outer_per_step": outer, "waves": waves, "raw": tot}
pw = lambda k: tot[k] / waves / iters   # noqa: E731
if "SQ_INSTS_VALU" in tot:
    res["valu_insts_per_wave_iter"] = pw("SQ_INSTS_VALU")
if "SQ_INSTS_LDS" in tot:
    res["lds_insts_per_wave_iter"] = pw("SQ_INSTS_LDS")
if "SQ_INSTS_SALU" in tot:
    res["salu_insts_per_wave_iter"] = pw("SQ_INSTS_SALU")
if "SQ_WAVE_CYCLES" in tot:
    res["wave_cycles_per_wave_iter"] = 4.0 * pw("SQ_WAVE_CYCLES")
f64 = [tot.get(k) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64")]
if "SQ_INSTS_VALU_FMA_F64" in tot:
    wi = sum(v for v in f64 if v) + 2.0 * tot["SQ_INSTS_VALU_FMA_F64"]
    res["fp64_flops_per_step"] = 64.0 * wi / steps
json.dump(res, open(os.path.join(ROOT, "profiles", f"sq_{tag}.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "raw"}))
