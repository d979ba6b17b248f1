# one-off: the OBCA solo-launch variant (libpiadmm_solo.so) probed and tested, and the repeated-step test
set -o pipefail
O=gpurun_out/solo
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_solo.so
PIADMM_LIB=$L timeout -k 10 300 python3 -u tools/obca_probe.py > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
PIADMM_LIB=$L timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_obca.py > $O/obca_tests.log 2>&1 || { tail -20 $O/obca_tests.log; exit 1; }
tail -1 $O/obca_tests.log
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_graph.py -k repeating > $O/repeat_test.log 2>&1 || { tail -20 $O/repeat_test.log; exit 1; }
tail -1 $O/repeat_test.log
PIADMM_LIB=$L timeout -k 10 300 python3 -u bench.py --obca --no-cpu > $O/bench_obca_solo.json 2> $O/b.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_obca_solo.json').read().strip().splitlines()[-1]); print('obca solo', d['ms_per_step'], d['value'])"
echo SOLO_DONE
