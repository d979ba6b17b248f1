set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1150 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
