# Graph-kernel check + A/B (on the GPU box): the graph GPU tests on the product library, then the
# crossing and chain bench lines for each library named (default: the product library).
#   bash tools/gpu_graph_ab.sh <tag> [<lib> ...]
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_graph.py tests/test_gpu_configs.py tests/test_gpu_shard.py > $O/graph_tests.log 2>&1 \
  || { tail -30 $O/graph_tests.log; exit 1; }
tail -2 $O/graph_tests.log
for L in "${@:-libpiadmm.so}"; do
  for W in crossing chain; do
    PIADMM_LIB=$PWD/distributed-local-planner-pi-admm_amd/piadmm/$L timeout -k 10 300 python3 -u bench.py --$W --no-cpu \
      > $O/b_${W}_$L.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${W}_$L.json').read().strip().splitlines()[-1]); print('$L $W', round(d['ms_per_step'], 3), round((d.get('natural') or {}).get('ms_per_step', 0), 3))"
  done
done
echo GRAPH_AB_DONE
