set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_modes.py -k "speculative" > $O/spec.log 2>&1 || { tail -40 $O/spec.log; exit 1; }
tail -3 $O/spec.log
timeout -k 10 300 python3 -u bench.py --no-cold --config2 > $O/c2.json 2> $O/c2.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('config2', d['ms_per_step'], d['natural']['ms_per_step'], d.get('speedup_vs_cpu_baseline'), d['natural'].get('speedup_vs_cpu_baseline'))"
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
