set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_modes.py -k "speculative" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for k in 1 2; do
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench_headline_$k.json 2> $O/bench_headline.err || exit 1
python3 -c "import json,sys; d=json.loads(open('$O/bench_headline_$k.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['natural']['ms_per_step'])"
done
echo R05G_DONE
