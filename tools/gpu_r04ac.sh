# r04ac: strong-scaling shares (configs[3]) on the final round-4 tree, as r04m
set -o pipefail
O=gpurun_out/r04ac
mkdir -p $O
B="python3 bench.py --strong --no-cpu"
timeout -k 10 200 $B > $O/s1.json 2> $O/s1.err || exit 1
for n in 2 4 8; do
  timeout -k 10 200 $B --share $n > $O/s${n}_contig.json 2> $O/s${n}_contig.err || exit 1
  timeout -k 10 300 $B --share $n --split interleaved > $O/s${n}_inter.json 2> $O/s${n}_inter.err || exit 1
done
echo R04AC_DONE
