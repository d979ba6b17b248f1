"""Summarise the rocprofv3 passes of tools/profile.sh into profiles/ (kernel stats + HBM traffic).

traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes for pd::k_mpc_step, using
MI355X_MICROARCH.md's gfx950 correction (FETCH_SIZE reads 1/2 of the bytes of wide
streaming reads; this kernel's 8-byte scattered reads are uncalibrated, so the raw values
are kept next to the corrected one).
"""
import csv
import glob
import json
import os
import shutil
import sys

out, tag = sys.argv[1], sys.argv[2]
steps_per_launch = int(sys.argv[3]) if len(sys.argv) > 3 else 20   # bench.py default: the timed 20-step launch
# optional (tools/profile_line.sh, every bench line): the workload name bench.py looks the file up by,
# a kernel-name substring, and the MPC steps the profiled run executed (warmup + timed): the counters
# are then summed over EVERY dispatch of the matching kernels and divided by those steps
WNAME = sys.argv[4] if len(sys.argv) > 4 else "tiled128_H30_matlab_pi_fixed100"
KSUB = sys.argv[5] if len(sys.argv) > 5 else None
STEPS_TOTAL = int(sys.argv[6]) if len(sys.argv) > 6 else None
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)


def rows(pattern):
    fs = glob.glob(os.path.join(out, pattern), recursive=True)
    if not fs:
        return []
    with open(fs[0]) as f:
        return list(csv.DictReader(f))


stats = glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(prof, f"kernel_stats_{tag}.csv"))


def pmc(name):
    """The counter summed over the timed launch (the last k_mpc_step dispatch: bench.py
    --no-natural runs the warmup launch, then the timed one) -- or, with KSUB, over every dispatch
    of the kernels whose name contains KSUB."""
    per = {}
    for r in rows(os.path.join(name.lower().split("_")[0], "**", "*counter_collection.csv")):
        if (KSUB or "k_mpc_step") in r.get("Kernel_Name", "") and r.get("Counter_Name") == name:
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    if KSUB:
        return [sum(per.values())] if per else []
    return [per[max(per)]] if per else []


fetch = pmc("FETCH_SIZE")
write = pmc("WRITE_SIZE")
res = {"workload": WNAME, "kernel": "pd::" + KSUB + "*" if KSUB else "pd::k_mpc_step",
       "launches_fetch": len(fetch), "launches_write": len(write)}
if fetch and write and KSUB:
    f, w = fetch[0], write[0]
    res.update(fetch_size_kb_raw=f, write_size_kb_raw=w, steps_total=STEPS_TOTAL,
               hbm_bytes_per_step=(2.0 * f + w) * 1024.0 / STEPS_TOTAL,
               note="traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE 1/2 correction), summed over "
                    "every dispatch of the kernels in the profiled run and divided by its MPC steps (warmup + timed)")
elif fetch and write:
    f = sum(fetch) / len(fetch)
    w = sum(write) / len(write)
    res.update(fetch_size_kb_raw=f, write_size_kb_raw=w,
               hbm_bytes_per_launch=(2.0 * f + w) * 1024.0, steps_per_launch=steps_per_launch,
               hbm_bytes_per_step=(2.0 * f + w) * 1024.0 / steps_per_launch,
               note="traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE 1/2 correction)")
json.dump(res, open(os.path.join(prof, f"traffic_{tag}.json"), "w"), indent=1)
print(json.dumps(res))
