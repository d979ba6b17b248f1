# r04q: graph-kernel pairs restore their last dual active set (S^-1, Y) within an MPC step --
# graph / shard / crossing parity tests, then the crossing and chain lines with and without it.
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_configs.py tests/test_gpu_shard.py -k "crossing or sharded or adversarial or config3" > $O/tests.log 2>&1 || exit 1
B="python3 bench.py --no-cpu"
timeout -k 10 300 $B --crossing > $O/x4.json 2> $O/x4.err || exit 1
PIADMM_PAIR_SNAP=0 timeout -k 10 300 $B --crossing > $O/x4_nosnap.json 2> $O/x4_nosnap.err || exit 1
timeout -k 10 300 $B --chain > $O/chain.json 2> $O/chain.err || exit 1
PIADMM_PAIR_SNAP=0 timeout -k 10 300 $B --chain > $O/chain_nosnap.json 2> $O/chain_nosnap.err || exit 1
echo R04Q_DONE
