# r04j: a sharded job's fixed iterations with one launch between two exchanges (Z(it) + X(it+1)):
# the shard / graph parity tests, then interleaved shares with and without the fused launch.
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
B="python3 bench.py --no-cpu --no-natural --strong"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_graph.py > $O/tests.log 2>&1 && \
timeout -k 10 300 $B --share 8 --split interleaved > $O/s8_inter.json 2> $O/s8_inter.err && \
PIADMM_NO_ZX=1 timeout -k 10 300 $B --share 8 --split interleaved > $O/s8_inter_nozx.json 2> $O/s8_inter_nozx.err && \
timeout -k 10 300 $B --share 2 --split interleaved > $O/s2_inter.json 2> $O/s2_inter.err && \
timeout -k 10 300 $B --share 4 --split interleaved > $O/s4_inter.json 2> $O/s4_inter.err && \
echo R04J_DONE
