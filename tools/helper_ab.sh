#!/bin/bash
# A/B of the pair's warm build on two waves (the helper wave, pd_qp.h WarmPipe) against the pair
# wave alone (PIADMM_NO_HELPER=1): targeted GPU tests first, then the headline and configs[1]
# lines both ways.  Each step under its own time limit; stops at the first failure.
set -o pipefail
O=gpurun_out/helper_ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_modes.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for nh in 0 1; do
  for w in headline config2; do
    case $w in headline) a="";; *) a="--$w";; esac
    PIADMM_NO_HELPER=$nh timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold $a > $O/${w}_nh$nh.json 2> $O/${w}_nh$nh.err || { tail -5 $O/${w}_nh$nh.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${w}_nh$nh.json').read().strip().splitlines()[-1]); print('$w no_helper=$nh', d['ms_per_step'], d['natural']['ms_per_step'])"
  done
done
