set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 300 python3 tools/graph_iter_profile.py 64 3 > gpurun_out/r04d/x64.log 2>&1 && \
timeout -k 10 300 python3 tools/graph_iter_profile.py 1 3 > gpurun_out/r04d/x1.log 2>&1 && \
PIADMM_PAIR_SOLVER=admm timeout -k 10 300 python3 tools/graph_iter_profile.py 1 2 > gpurun_out/r04d/x1_admm.log 2>&1
echo R04D_DONE
