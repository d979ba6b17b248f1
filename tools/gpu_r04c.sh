# r04c: tests of the touched paths, headline bench, crossing split experiments, chain.
set -o pipefail
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_gpu_ties.py tests/test_gpu_graph.py tests/test_gpu_outer_iter.py tests/test_gpu_shard.py "tests/test_gpu_modes.py" > gpurun_out/r04c/tests1.log 2>&1 && \
timeout -k 10 200 python3 bench.py --no-cpu > gpurun_out/r04c/h.json 2> gpurun_out/r04c/h.err && \
timeout -k 10 300 python3 bench.py --crossing --no-cpu > gpurun_out/r04c/x4.json 2> gpurun_out/r04c/x4.err && \
PIADMM_GRAPH_BLOCK=1 timeout -k 10 300 python3 bench.py --crossing --no-cpu > gpurun_out/r04c/x4_b1.json 2> gpurun_out/r04c/x4_b1.err && \
PIADMM_GRAPH_BLOCK=2 timeout -k 10 300 python3 bench.py --crossing --no-cpu > gpurun_out/r04c/x4_b2.json 2> gpurun_out/r04c/x4_b2.err && \
timeout -k 10 300 python3 bench.py --chain --no-cpu > gpurun_out/r04c/chain.json 2> gpurun_out/r04c/chain.err && \
timeout -k 10 600 $T "tests/test_gpu_configs.py::test_gpu_equals_bopt_on_the_crossing_workload" -s > gpurun_out/r04c/tests2.log 2>&1
echo R04C_DONE
