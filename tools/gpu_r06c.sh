set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
L=distributed-local-planner-pi-admm_amd/piadmm
timeout -k 10 600 python3 -u tools/iter_slope.py $L/libpiadmm_base.so $L/libpiadmm_xrep.so $L/libpiadmm_prep.so > $O/slope.log 2>&1 || { cat $O/slope.log; exit 1; }
cat $O/slope.log
