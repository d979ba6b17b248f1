# r04ab: the final round-4 tree -- smoke, the full GPU suite, the headline and the graph-kernel
# lines with their CPU baselines.
set -o pipefail
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
for W in crossing chain config5; do
  timeout -k 10 300 python3 bench.py --$W > $O/bench_$W.json 2> $O/bench_$W.err || exit 1
done
echo R04AB_DONE
