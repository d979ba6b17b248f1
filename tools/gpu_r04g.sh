# r04g: strong-scaling readiness (configs[3]): one rank's share of an N-rank job alone on
# this GPU (collectives as no-ops), contiguous and interleaved splits, N = 1, 2, 4, 8.
set -o pipefail
mkdir -p gpurun_out/r04g
B="python3 bench.py --strong --no-cpu"
timeout -k 10 200 $B > gpurun_out/r04g/s1.json 2> gpurun_out/r04g/s1.err && \
for n in 2 4 8; do
  timeout -k 10 200 $B --share $n > gpurun_out/r04g/s${n}_contig.json 2> gpurun_out/r04g/s${n}_contig.err || exit 1
  timeout -k 10 300 $B --share $n --split interleaved > gpurun_out/r04g/s${n}_inter.json 2> gpurun_out/r04g/s${n}_inter.err || exit 1
done
echo R04G_DONE
