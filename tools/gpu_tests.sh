#!/bin/bash
# GPU test run (on the GPU box, from the repo root): pytest -m gpu [on the given test files / -k
# expression], then smoke() and the headline bench, each under its own time limit; the script
# stops at the first failure.
#   bash tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" \
  > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
echo ${TAG}_DONE
