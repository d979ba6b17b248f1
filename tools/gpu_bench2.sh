set -o pipefail
O=gpurun_out/${1:-bench2}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench_headline_$k.json 2> $O/bench_headline.err || exit 1
python3 -c "import json,sys; d=json.loads(open('$O/bench_headline_$k.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['natural']['ms_per_step'])"
done
echo BENCH2_DONE
