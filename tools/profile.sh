#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box from the repo root).
#   1. kernel trace + stats           -> gpurun_out/prof_<tag>/trace
#   2. PMC FETCH_SIZE (own pass)      -> gpurun_out/prof_<tag>/fetch
#   3. PMC WRITE_SIZE (own pass)      -> gpurun_out/prof_<tag>/write
# Each step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:-r02}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--no-cpu --no-natural --no-cold --warmup 20"   # a 20-step warmup launch, then the 20-step timed launch (equal launches)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/traffic.py $OUT $TAG 20 > $OUT/traffic.log 2>&1
echo PROFILE_DONE
