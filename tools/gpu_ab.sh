# A/B of builds of the library on one box: bash tools/gpu_ab.sh <tag> <rounds> <lib> [<lib> ...]
set -o pipefail
O=gpurun_out/$1
R=$2
shift 2
mkdir -p $O
export TMPDIR=/tmp
for k in $(seq 1 $R); do
for L in "$@"; do
PIADMM_LIB=$PWD/distributed-local-planner-pi-admm_amd/piadmm/$L timeout -k 10 300 python3 -u bench.py --no-cpu > $O/b_${L}_$k.json 2> $O/b.err || exit 1
python3 -c "import json,sys; d=json.loads(open('$O/b_${L}_$k.json').read().strip().splitlines()[-1]); print('$L', d['ms_per_step'], d['natural']['ms_per_step'])"
done
done
echo AB_DONE
