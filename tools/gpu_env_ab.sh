# A/B of run-time variants (GPU box): bash tools/gpu_env_ab.sh <tag> <rounds> "<ENV=VAL ...>" ...
# ("-" = no variables); one headline bench per variant and round, fixed and natural ms per step.
set -o pipefail
O=gpurun_out/$1
R=$2
shift 2
mkdir -p $O
export TMPDIR=/tmp
for k in $(seq 1 $R); do
  i=0
  for V in "$@"; do
    i=$((i + 1))
    if [ "$V" = "-" ]; then E=""; else E="$V"; fi
    env $E timeout -k 10 300 python3 -u bench.py --no-cpu > $O/b_${i}_$k.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${i}_$k.json').read().strip().splitlines()[-1]); print('$V', round(d['ms_per_step'], 4), round(d['natural']['ms_per_step'], 4))"
  done
done
echo ENV_AB_DONE
