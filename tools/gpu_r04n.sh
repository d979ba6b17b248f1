# r04n: round-4 evidence, part 1 -- the driver-equivalent headline bench (CPU leg included), the
# rocprofv3 kernel trace / stats and FETCH_SIZE / WRITE_SIZE passes of it, smoke() and the full
# GPU test suite.  Each step has its own time limit; the script stops at the first failure.
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 600 bash tools/profile.sh r04 > $O/profile.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo R04N_DONE
