#!/bin/bash
# rocprofv3 HBM traffic of one bench line (run on the GPU box from the repo root):
#   bash tools/profile_line.sh <tag> <workload-name> <kernel-substring> <bench args...>
# Two PMC passes of their own (FETCH_SIZE, WRITE_SIZE; no tracing domains), each under its own time
# limit; tools/traffic.py sums the counters over every dispatch of the kernels and divides by the
# MPC steps the run executed (warmup + timed: --warmup and --steps below), writing
# profiles/traffic_<tag>.json for bench.py's latest_profile() lookup.  Stops at the first failure.
set -e
TAG=$1; WNAME=$2; KSUB=$3; shift 3
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--no-cpu --no-natural --no-cold --warmup 5 --steps 10 $*"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/traffic.py $OUT $TAG 0 $WNAME $KSUB 15 > $OUT/traffic.log 2>&1
cat $OUT/traffic.log
echo PROFILE_LINE_DONE
