# r04k: kernel trace of rank 0's share of an 8-rank interleaved job over 20 fixed steps
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o tr --output-format csv -- python3 bench.py --strong --no-cpu --no-natural --share 8 --split interleaved --steps 20 --warmup 1 > $O/trace.log 2>&1 && \
echo R04K_DONE
