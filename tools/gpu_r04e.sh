# r04e: gi_solve as a called (non-inlined) function, measured against the inlined build.
set -o pipefail
mkdir -p gpurun_out/r04e
V=distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_gino.so
PIADMM_LIB=$V timeout -k 10 200 python3 bench.py --no-cpu > gpurun_out/r04e/h_gino.json 2> gpurun_out/r04e/h_gino.err && \
PIADMM_LIB=$V timeout -k 10 300 python3 bench.py --crossing --no-cpu > gpurun_out/r04e/x4_gino.json 2> gpurun_out/r04e/x4_gino.err && \
PIADMM_LIB=$V timeout -k 10 300 python3 bench.py --chain --no-cpu > gpurun_out/r04e/chain_gino.json 2> gpurun_out/r04e/chain_gino.err && \
PIADMM_LIB=$V timeout -k 10 200 python3 bench.py --config2 --no-cpu > gpurun_out/r04e/c2_gino.json 2> gpurun_out/r04e/c2_gino.err && \
timeout -k 10 200 python3 bench.py --config2 --no-cpu > gpurun_out/r04e/c2.json 2> gpurun_out/r04e/c2.err && \
PIADMM_LIB=$V timeout -k 10 300 python3 tools/graph_iter_profile.py 1 3 > gpurun_out/r04e/x1_gino.log 2>&1
echo R04E_DONE
