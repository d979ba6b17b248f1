#!/bin/bash
# bench.py lines on the GPU box (each under its own limit; stops at the first failure):
#   bash tools/gpu_bench.sh <tag> [line ...]    lines: headline config2 config5 crossing chain obca strong
set -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for W in "${@:-headline}"; do
  if [ "$W" = headline ]; then ARGS=""; else ARGS="--$W"; fi
  timeout -k 10 400 python3 -u bench.py $ARGS > $O/bench_$W.json 2> $O/bench_$W.err || { tail -20 $O/bench_$W.err; exit 1; }
  cat $O/bench_$W.json
done
echo ${TAG}_DONE
