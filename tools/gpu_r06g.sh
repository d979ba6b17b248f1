set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
L=distributed-local-planner-pi-admm_amd/piadmm
timeout -k 10 600 python3 -u tools/iter_slope.py $L/libpiadmm.so $L/libpiadmm_base.so > $O/slope.log 2>&1 || { cat $O/slope.log; exit 1; }
cat $O/slope.log
bash tools/gpu_ab.sh r06g_ab 1 libpiadmm.so || exit 1
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_modes.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_outer_iter.py tests/test_gpu_ties.py -k "not crossing" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -5 $O/tests.log
