set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
L=distributed-local-planner-pi-admm_amd/piadmm
timeout -k 10 120 tools/xhit_ubench > $O/xhit.log 2>&1 || exit 1
cat $O/xhit.log
timeout -k 10 600 python3 -u tools/iter_slope.py $L/libpiadmm.so $L/libpiadmm_base.so > $O/slope.log 2>&1 || { cat $O/slope.log; exit 1; }
cat $O/slope.log
# the round-5 exit fault: a --pmc pass of the natural bench (last: a fault ends the call here)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_nat -o bench --output-format csv -- python3 bench.py --no-cpu --natural --steps 10 --warmup 10 > $O/pmc_nat.log 2>&1
echo "pmc_nat rc=$?"
tail -5 $O/pmc_nat.log
