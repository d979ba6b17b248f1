set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/stamps.py 128 30 4 > $O/stamps_fixed.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/stamps.py 128 30 10 natural > $O/stamps_natural.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py > $O/bench_headline.json 2> $O/bench_headline.err || exit 1
echo R05B_DONE
