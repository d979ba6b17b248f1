set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ties.py tests/test_gpu_modes.py -k "ties or speculative" > $O/ties.log 2>&1 || { tail -40 $O/ties.log; exit 1; }
tail -3 $O/ties.log
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
