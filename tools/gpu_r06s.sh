set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
for ns in 0 2; do
PIADMM_NO_SPEC=$ns timeout -k 10 300 python3 -u bench.py --no-cpu --no-cold --config2 > $O/c2_$ns.json 2> $O/c2_$ns.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c2_$ns.json').read().strip().splitlines()[-1]); print('config2 ns=$ns', d['ms_per_step'], d['natural']['ms_per_step'])"
PIADMM_NO_SPEC=$ns PIADMM_SLOPE_JOB=casadi_default,20,32 timeout -k 10 300 python3 -u tools/iter_slope.py > $O/slope_c2_$ns.log 2>&1 || { cat $O/slope_c2_$ns.log; exit 1; }
cat $O/slope_c2_$ns.log
done
