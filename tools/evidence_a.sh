#!/bin/bash
# Round evidence, part 1 (GPU box, repo root): the headline bench line as the driver runs it (CPU
# leg included), then profile.sh <tag> (kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes) and
# the fused kernel's phase stamps.  Each GPU step has its own time limit; stops at the first failure.
set -e
TAG=${1:?tag}
OUT=gpurun_out/ev_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $OUT/bench_headline.json 2> $OUT/bench_headline.err
timeout -k 10 600 bash tools/profile.sh $TAG > $OUT/profile.log 2>&1
timeout -k 10 150 python3 tools/stamps.py 128 30 4 > $OUT/stamps_fixed.log 2>&1
timeout -k 10 150 python3 tools/stamps.py 128 30 4 natural > $OUT/stamps_natural.log 2>&1
echo EVIDENCE_A_DONE
