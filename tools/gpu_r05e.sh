set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_modes.py -k "speculative" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench_headline.json 2> $O/bench_headline.err || exit 1
cat $O/bench_headline.json
export PIADMM_LIB=$PWD/distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_lines.so
timeout -k 10 300 bash tools/pcsample.sh r05e_fixed --no-natural || exit 1
timeout -k 10 300 bash tools/pcsample.sh r05e_natural --natural || exit 1
echo R05E_DONE
