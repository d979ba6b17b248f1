#!/bin/bash
# PC sampling (rocprofv3 beta, host trap) of bench.py's fused kernel: where the waves spend their
# time, per instruction.  Run on the GPU box from the repo root; tools/pcmap.py reads the result.
#   bash tools/pcsample.sh <tag> [bench args...]
# PIADMM_LIB may select the line-table build (make lines) so that the samples map to source lines.
set -e
TAG=${1:-r05}
shift || true
OUT=gpurun_out/pc_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
  --pc-sampling-unit time --pc-sampling-interval 1 -d $OUT/raw -o pc --output-format csv \
  -- python3 bench.py --no-cpu --steps 10 --warmup 2 "$@" > $OUT/run.log 2>&1
echo PC_DONE
