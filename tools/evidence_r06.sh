#!/bin/bash
# Round-6 bench lines, each with its CPU baseline (B-opt on the box's host cores), on the final tree
# (run on the GPU box from the repo root).  Every step has its own time limit; stops at the first failure.
set -o pipefail
OUT=gpurun_out/ev_${1:-r06}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err || exit 1
for W in config2 config5 strong crossing chain obca; do
  timeout -k 10 400 python3 -u bench.py --$W > $OUT/bench_$W.json 2> $OUT/bench_$W.err || exit 1
  echo "$W done"
done
echo EVIDENCE_DONE
