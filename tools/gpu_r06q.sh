set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
export TMPDIR=/tmp
L=distributed-local-planner-pi-admm_amd/piadmm
for lib in libpiadmm_base.so libpiadmm.so; do
PIADMM_LIB=$PWD/$L/$lib timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold --config5 > $O/c5_$lib.json 2> $O/c5.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c5_$lib.json').read().strip().splitlines()[-1]); print('config5 $lib', d['ms_per_step'], d['natural']['ms_per_step'])"
done
PIADMM_LIB=$PWD/$L/libpiadmm.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold > $O/c3.json 2> $O/c3.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); print('headline', d['ms_per_step'], d['natural']['ms_per_step'])"
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_modes.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "not crossing" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
