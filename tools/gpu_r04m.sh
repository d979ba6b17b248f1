# r04m: the wide dual active set (pair working sets beyond 63 rows) -- graph and big-mode parity
# tests -- then the strong-scaling shares (contiguous / interleaved with locally solved ghosts,
# natural via the device-decided path) and the configs[4] (H = 50, big mode) bench.
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_graph.py -k "wide or mixed or global_termination" > $O/tests_wide.log 2>&1 || exit 1
timeout -k 10 600 $T tests/test_gpu_parity.py -k "horizon or largest or pair_solvers" > $O/tests_big.log 2>&1 || exit 1
B="python3 bench.py --strong --no-cpu"
timeout -k 10 200 $B > $O/s1.json 2> $O/s1.err || exit 1
for n in 2 4 8; do
  timeout -k 10 200 $B --share $n > $O/s${n}_contig.json 2> $O/s${n}_contig.err || exit 1
  timeout -k 10 300 $B --share $n --split interleaved > $O/s${n}_inter.json 2> $O/s${n}_inter.err || exit 1
done
timeout -k 10 300 python3 bench.py --config5 --no-cpu > $O/c5.json 2> $O/c5.err || exit 1
echo R04M_DONE
