# A/B of two builds of the library on one box: bash tools/gpu_ab.sh <tag> <libA> <libB> [rounds]
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
R=${4:-2}
for k in $(seq 1 $R); do
for L in $2 $3; do
PIADMM_LIB=$PWD/distributed-local-planner-pi-admm_amd/piadmm/$L timeout -k 10 300 python3 -u bench.py --no-cpu > $O/b_${L}_$k.json 2> $O/b.err || exit 1
python3 -c "import json,sys; d=json.loads(open('$O/b_${L}_$k.json').read().strip().splitlines()[-1]); print('$L', d['ms_per_step'], d['natural']['ms_per_step'])"
done
done
echo AB_DONE
