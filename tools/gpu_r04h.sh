# r04h: where an interleaved strong-scaling share spends its time: a kernel trace of
# rank 0's share of an 8-rank interleaved job, and the same tiles on the graph kernel unsplit.
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --strong --no-cpu"
PIADMM_GRAPH=1 timeout -k 10 200 $B --share 8 > $O/s8_graph_contig.json 2> $O/s8_graph_contig.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o tr --output-format csv -- python3 bench.py --strong --no-cpu --share 8 --split interleaved --steps 3 --warmup 1 > $O/trace.log 2>&1 && \
echo R04H_DONE
