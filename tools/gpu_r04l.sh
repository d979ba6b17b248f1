# r04l: strong-scaling readiness (configs[3]), one rank's share of an N-rank job alone
# on this GPU: contiguous and interleaved splits, N = 2, 4, 8, fixed and natural (the natural stop
# decided on the device after each iteration, as across ranks); interleaved shares solve their
# ghosts' x-steps on the tile's second wave and run the fused Z + X launch between exchanges.
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
B="python3 bench.py --strong --no-cpu"
timeout -k 10 200 $B > $O/s1.json 2> $O/s1.err || exit 1
for n in 2 4 8; do
  timeout -k 10 200 $B --share $n > $O/s${n}_contig.json 2> $O/s${n}_contig.err || exit 1
  timeout -k 10 300 $B --share $n --split interleaved > $O/s${n}_inter.json 2> $O/s${n}_inter.err || exit 1
done
echo R04L_DONE
