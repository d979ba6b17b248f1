"""Sum the instruction-cache counters of k_mpc_step per run (tools/icache.sh output)."""
import csv, glob, os, sys, collections
base = sys.argv[1]
for run in ("nat", "fix"):
    files = glob.glob(os.path.join(base, run, "**", "*counter_collection.csv"), recursive=True)
    tot = collections.Counter()
    nd = collections.Counter()
    for f in files:
        for r in csv.DictReader(open(f)):
            if "k_mpc_step" not in r.get("Kernel_Name", ""):
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            nd[r["Dispatch_Id"]] += 1
    print(run, "dispatches", len(nd), {k: f"{v:.4g}" for k, v in sorted(tot.items())})
    if tot.get("SQC_ICACHE_REQ"):
        print(f"  icache miss rate {tot['SQC_ICACHE_MISSES'] / tot['SQC_ICACHE_REQ']:.4f}, "
              f"wait-inst share of wave cycles {4 * tot['SQ_WAIT_INST_ANY'] / max(tot['SQ_WAVE_CYCLES'], 1):.3f}")
