set -o pipefail
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ties.py tests/test_gpu_graph.py::test_component_split_over_workgroups tests/test_gpu_graph.py::test_split_component_host_stepping "tests/test_gpu_modes.py::test_checkpoint_resume_equals_uninterrupted_run" tests/test_gpu_parity.py -s > gpurun_out/r04a/tests1.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err && \
PIADMM_NO_ROLLER=1 timeout -k 10 300 python -u bench.py > gpurun_out/r04a/bench_noroll.json 2> gpurun_out/r04a/bench_noroll.err && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu "tests/test_gpu_configs.py::test_gpu_equals_bopt_on_the_crossing_workload" -s > gpurun_out/r04a/tests2.log 2>&1
