set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
export TMPDIR=/tmp
PIADMM_SLOPE_JOB=casadi_default,20,32 timeout -k 10 300 python3 -u tools/iter_slope.py > $O/slope_c2.log 2>&1 || { cat $O/slope_c2.log; exit 1; }
cat $O/slope_c2.log
bash tools/profile_line.sh r06_ob obca4096 k_obca --obca
