# r04o: round-4 evidence, part 2 -- phase stamps (fused kernel fixed / natural, graph kernel on the
# 64 crossings) and every other bench.py line with its CPU baseline.
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 120 python3 tools/stamps.py 128 30 4 > $O/stamps_fixed.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/stamps.py 128 30 20 natural > $O/stamps_natural.log 2>&1 || exit 1
timeout -k 10 180 python3 tools/graph_stamps.py 64 30 2 fixed all > $O/graph_stamps_x64.log 2>&1 || exit 1
for W in config2 config5 crossing chain obca strong; do
  timeout -k 10 300 python3 bench.py --$W > $O/bench_$W.json 2> $O/bench_$W.err || exit 1
done
echo R04O_DONE
