set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
for w in crossing chain headline; do
  case $w in headline) a="";; *) a="--$w";; esac
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold $a > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'], d['natural']['ms_per_step'])"
done
timeout -k 10 1200 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
