"""Development diagnostic (not shipped): aggregate a rocprofv3 PC-sampling CSV (tools/pcsample.sh)
per instruction address and print the hottest instructions with their share, plus a histogram by
opcode.  Usage: python tools/pcmap.py gpurun_out/pc_<tag>/raw [top]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 60
files = [f for f in glob.glob(os.path.join(root, "**", "*.csv"), recursive=True) if "pc_sampling" in os.path.basename(f)]
if not files:
    print("no pc_sampling csv under", root, ":", glob.glob(os.path.join(root, "**", "*.csv"), recursive=True))
    sys.exit(1)
for f in files:
    with open(f) as fh:
        rd = csv.DictReader(fh)
        cols = rd.fieldnames
        print(f, cols)
        key_off = next((c for c in cols if "offset" in c.lower()), None)
        key_ins = next((c for c in cols if c.lower() in ("instruction", "inst", "instruction_text")), None)
        key_cmt = next((c for c in cols if "comment" in c.lower()), None)
        cnt = collections.Counter()
        txt = {}
        op = collections.Counter()
        n = 0
        for r in rd:
            k = r.get(key_off, "") if key_off else ""
            cnt[k] += 1
            ins = r.get(key_ins, "") if key_ins else ""
            txt[k] = (ins, r.get(key_cmt, "") if key_cmt else "")
            op[ins.split()[0] if ins else "?"] += 1
            n += 1
    print(f"{n} samples")
    for k, c in cnt.most_common(top):
        ins, cm = txt[k]
        print(f"{100 * c / n:6.2f}%  {k:>10}  {ins:60s} {cm[:80]}")
    print("by opcode:")
    for o, c in op.most_common(40):
        print(f"{100 * c / n:6.2f}%  {o}")
