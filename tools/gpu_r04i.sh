# r04i: the split / exchange paths after the copy kernel and the cached LDS attribute: interleaved
# strong-scaling shares (2, 8 ranks) and the 1024-agent chain (a component split over workgroups).
set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
B="python3 bench.py --no-cpu"
timeout -k 10 300 $B --strong --share 8 --split interleaved > $O/s8_inter.json 2> $O/s8_inter.err && \
timeout -k 10 300 $B --strong --share 2 --split interleaved > $O/s2_inter.json 2> $O/s2_inter.err && \
timeout -k 10 300 $B --chain --steps 5 --warmup 1 > $O/chain.json 2> $O/chain.err && \
echo R04I_DONE
