#!/bin/bash
# Round evidence, part 2 (GPU box, repo root): every other bench.py line with its CPU baseline.
set -e
TAG=${1:?tag}
OUT=gpurun_out/ev_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
for W in config2 config5 strong crossing chain obca; do
  timeout -k 10 300 python3 -u bench.py --$W > $OUT/bench_$W.json 2> $OUT/bench_$W.err
  python3 -c "import json; d=json.loads(open('$OUT/bench_$W.json').read().strip().splitlines()[-1]); print('$W', d['ms_per_step'], (d.get('natural') or {}).get('ms_per_step'), (d.get('cpu_baseline') or {}).get('value'))"
done
echo EVIDENCE_B_DONE
