set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_ab.sh r06a_ab 2 libpiadmm.so libpiadmm_xrep.so || exit 1
PIADMM_EVIDENCE_DIR=$O timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests/test_gpu_two_process.py "tests/test_gpu_parity.py::test_horizon_limits_match_oracle" "tests/test_gpu_configs.py::test_gpu_equals_bopt_on_the_crossing_workload" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -15 $O/tests.log
