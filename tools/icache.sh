#!/bin/bash
# Instruction-cache counters of k_mpc_step (GPU box, repo root): one PMC pass each for the
# natural and the fixed headline, then tools/icache_sum.py.   bash tools/icache.sh <tag>
set -e
O=gpurun_out/ic_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
C="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $C -d $O/nat -o bench --output-format csv -- python3 bench.py --no-cpu --natural --steps 10 --warmup 10 > $O/nat.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc $C -d $O/fix -o bench --output-format csv -- python3 bench.py --no-cpu --no-natural --steps 10 --warmup 10 > $O/fix.log 2>&1
python3 tools/icache_sum.py $O
echo ICACHE_DONE
