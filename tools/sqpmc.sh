#!/bin/bash
# SQ instruction-mix / stall / fp64 passes for bench.py's dominant kernel (run on the GPU box from
# the repo root).  Each pass is its own rocprofv3 run (<= 8 SQ counters); the script stops at the
# first failure.  tools/sqsum.py writes profiles/sq_<tag>.json (read by bench.py).
set -e
TAG=${1:-r02}
OUT=gpurun_out/sq_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--no-cpu --no-natural --no-cold --warmup 20"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/p$i -o bench --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  i=$((i+1))
done
python3 tools/sqsum.py $OUT $TAG > $OUT/summary.txt 2>&1
echo SQ_DONE
