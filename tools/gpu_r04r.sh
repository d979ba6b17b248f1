# r04r: A/B of skipping the pair's warm-label reduced solve when this step's dual active set is
# restorable (PIADMM_PAIR_SNAP_FIRST=1), crossings and chain, plus the graph tests with it on.
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
B="python3 bench.py --no-cpu"
timeout -k 10 300 $B --crossing > $O/x4.json 2> $O/x4.err || exit 1
PIADMM_PAIR_SNAP_FIRST=1 timeout -k 10 300 $B --crossing > $O/x4_first.json 2> $O/x4_first.err || exit 1
timeout -k 10 300 $B --chain > $O/chain.json 2> $O/chain.err || exit 1
PIADMM_PAIR_SNAP_FIRST=1 timeout -k 10 300 $B --chain > $O/chain_first.json 2> $O/chain_first.err || exit 1
PIADMM_PAIR_SNAP_FIRST=1 timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_graph.py > $O/tests_first.log 2>&1 || exit 1
echo R04R_DONE
