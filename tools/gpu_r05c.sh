set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_modes.py tests/test_gpu_parity.py -k "speculative or gpu_parity" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench_headline.json 2> $O/bench_headline.err || exit 1
cat $O/bench_headline.json
echo R05C_DONE
