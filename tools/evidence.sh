#!/bin/bash
# One GPU call's worth of round evidence (run on the GPU box from the repo root):
#   profile.sh <tag>      kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes (bench.py headline)
#   stamps                per-phase cycles of the fused kernel (diagnostic build) and the graph kernel
#   bench lines           every workload of bench.py with its CPU baseline
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:-r03}
OUT=gpurun_out/ev_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 bash tools/profile.sh $TAG > $OUT/profile.log 2>&1
timeout -k 10 120 python3 tools/stamps.py 128 30 4 > $OUT/stamps_fixed.log 2>&1
timeout -k 10 120 python3 tools/stamps.py 1 30 4 > $OUT/stamps_fixed_1tile.log 2>&1
timeout -k 10 180 python3 tools/graph_stamps.py 64 30 2 fixed all > $OUT/graph_stamps_x64.log 2>&1
for W in config2 config5 crossing chain obca; do
  timeout -k 10 300 python3 bench.py --$W > $OUT/bench_$W.json 2> $OUT/bench_$W.err
done
timeout -k 10 300 python3 bench.py --strong > $OUT/bench_strong.json 2> $OUT/bench_strong.err
echo EVIDENCE_DONE
