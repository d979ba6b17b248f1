# Big-mode (H > 32) check + A/B (GPU box): configs[4] line per library, then the GPU tests that
# run big-mode jobs (H = 33..63 parity, wide working sets, configs[4] against B-opt).
#   bash tools/gpu_big_ab.sh <tag> <lib> [<lib> ...]
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p $O
export TMPDIR=/tmp
for L in "$@"; do
  PIADMM_LIB=$PWD/distributed-local-planner-pi-admm_amd/piadmm/$L timeout -k 10 300 python3 -u bench.py --config5 --no-cpu \
    > $O/b_c5_$L.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_c5_$L.json').read().strip().splitlines()[-1]); print('$L c5', round(d['ms_per_step'], 4), round(d['natural']['ms_per_step'], 4))"
done
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_configs.py > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo BIG_AB_DONE
