# r04aa: the pair snapshot restores the hinge regimes too -- graph / crossing / shard tests, the
# chain and crossing lines, the chain's stamps.
set -o pipefail
O=gpurun_out/r04aa
mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_graph.py tests/test_gpu_configs.py tests/test_gpu_shard.py -k "not capacity" > $O/tests.log 2>&1 || exit 1
B="python3 bench.py --no-cpu"
timeout -k 10 300 $B --chain > $O/chain.json 2> $O/chain.err || exit 1
timeout -k 10 300 $B --crossing > $O/x4.json 2> $O/x4.err || exit 1
echo R04AA_DONE
