set -o pipefail
mkdir -p gpurun_out/r04f
T="python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu"
timeout -k 10 600 $T "tests/test_gpu_modes.py::test_fp32_tables_config5_tolerance_study" "tests/test_gpu_modes.py::test_fp32_admm_matrices_keep_answers" "tests/test_gpu_configs.py::test_config5_256_agents_H50_tightening_sampled_tiles" -s > gpurun_out/r04f/tests.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config5 --no-cpu > gpurun_out/r04f/c5.json 2> gpurun_out/r04f/c5.err && \
timeout -k 10 300 python3 bench.py --config5 --no-cpu --precision 2 > gpurun_out/r04f/c5_p2.json 2> gpurun_out/r04f/c5_p2.err
echo R04F_DONE
