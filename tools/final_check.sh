#!/bin/bash
# Round-end check on the GPU box (from the repo root): the GPU test suite, smoke() and the default
# bench line, each under its own time limit; stops at the first failure.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-250
