#!/bin/bash
# SQ instruction-mix / stall passes for bench.py's kernel (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run (<= 8 SQ counters); the script stops at the first failure.
set -e
TAG=${1:-r01}
OUT=gpurun_out/sq_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--no-cpu"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/p$i -o bench --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  i=$((i+1))
done
python3 tools/sqsum.py $OUT > $OUT/summary.txt 2>&1
echo SQ_DONE
