#!/bin/bash
# GPU-call bundle: headline bench (no CPU leg), the SQ counter passes, the 4-rank rehearsal of
# natural global termination (host transport, one GPU) and, last, PC sampling of the fused kernel.
# Every step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:-r03}
OUT=gpurun_out/b_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 bash tools/sqpmc.sh $TAG > $OUT/sq.log 2>&1
PIADMM_BENCH_TRANSPORT=host timeout -k 10 300 python3 bench.py --gpus 4 --natural --no-cpu --steps 10 --warmup 2 > $OUT/reh_g4_natural.json 2> $OUT/reh_g4_natural.err
timeout -k 10 300 python3 bench.py --natural --no-cpu --steps 10 --warmup 2 > $OUT/g1_natural.json 2> $OUT/g1_natural.err
timeout -k 10 240 bash tools/pcsample.sh $TAG > $OUT/pc.log 2>&1
echo BUNDLE_DONE
