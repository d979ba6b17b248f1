set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
L=distributed-local-planner-pi-admm_amd/piadmm
for k in 1 2; do
for lib in libpiadmm_base.so libpiadmm.so; do
PIADMM_LIB=$PWD/$L/$lib timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold > $O/c3_${lib}_$k.json 2> $O/c3.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c3_${lib}_$k.json').read().strip().splitlines()[-1]); print('headline $lib', d['ms_per_step'], d['natural']['ms_per_step'], d['natural']['outer_iters_per_step'])"
done
done
PIADMM_LIB=$PWD/$L/libpiadmm.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold --config2 > $O/c2.json 2> $O/c2.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('config2', d['ms_per_step'], d['natural']['ms_per_step'])"
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_modes.py tests/test_gpu_configs.py tests/test_gpu_outer_iter.py -k "not crossing" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
