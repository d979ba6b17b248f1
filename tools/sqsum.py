"""Sum the SQ counters of tools/sqpmc.sh over pd::k_mpc_step dispatches (the timed launch only:
the last dispatch), per wave and per outer iteration (bench: 128 components x 2 waves, 10 steps x
100 outer iterations per launch).  SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles."""
import collections
import csv
import glob
import os
import sys

out = sys.argv[1]
tot = collections.OrderedDict()
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_mpc_step" in r.get("Kernel_Name", ""):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if per:
        last = per[max(per)]
        tot.update(last)
waves = tot.get("SQ_WAVES", 256.0) or 256.0
iters = 1000.0
for k, v in tot.items():
    print(f"{k:24s} {v:16.0f}   per wave {v / waves:12.1f}   per wave-iteration {v / waves / iters:10.2f}")
