set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/xhit_ubench > $O/xhit.log 2>&1 || exit 1
grep -E "replica|barriers|xhit_repeat" $O/xhit.log
# the round-5 exit fault with the library unloaded before exit (last: a fault ends the call here)
PIADMM_BENCH_UNLOAD=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_nat -o bench --output-format csv -- python3 bench.py --no-cpu --natural --steps 10 --warmup 10 > $O/pmc_nat.log 2>&1
echo "pmc_nat_unload rc=$?"
tail -4 $O/pmc_nat.log
