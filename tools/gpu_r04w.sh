# r04w: the final round-4 tree -- full GPU suite, smoke, the driver-equivalent headline bench,
# and the OBCA phase stamps (where its time goes, for the next round).
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
PIADMM_LIB=distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_stamps.so timeout -k 10 200 python3 tools/obca_stamps.py > $O/obca_stamps.log 2>&1 || exit 1
echo R04W_DONE
