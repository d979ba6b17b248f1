set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
L=distributed-local-planner-pi-admm_amd/piadmm
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_modes.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_outer_iter.py -k "not crossing" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for lib in libpiadmm_base.so libpiadmm.so; do
PIADMM_LIB=$PWD/$L/$lib timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold > $O/c3_$lib.json 2> $O/c3.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c3_$lib.json').read().strip().splitlines()[-1]); print('headline $lib', d['ms_per_step'], d['natural']['ms_per_step'])"
done
timeout -k 10 600 python3 -u tools/iter_slope.py $L/libpiadmm.so > $O/slope.log 2>&1 || { cat $O/slope.log; exit 1; }
cat $O/slope.log
