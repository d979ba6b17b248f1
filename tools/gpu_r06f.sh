set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
# the round-5 exit fault: which launch path and counter pass it needs
PIADMM_NO_COOP=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_nat_nocoop -o bench --output-format csv -- python3 bench.py --no-cpu --natural --steps 10 --warmup 10 > $O/pmc_nat_nocoop.log 2>&1
echo "pmc natural, no cooperative launch: rc=$?"
[ -s $O/pmc_nat_nocoop/bench_counter_collection.csv ] || true
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace_nat -o bench --output-format csv -- python3 bench.py --no-cpu --natural --steps 10 --warmup 10 > $O/trace_nat.log 2>&1
echo "kernel-trace natural (cooperative): rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fix -o bench --output-format csv -- python3 bench.py --no-cpu --no-natural --steps 10 --warmup 10 > $O/pmc_fix.log 2>&1
echo "pmc fixed: rc=$?"
PIADMM_BENCH_MAPS=$O/maps.txt timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_nat -o bench --output-format csv -- python3 bench.py --no-cpu --natural --steps 10 --warmup 10 > $O/pmc_nat.log 2>&1
echo "pmc natural (cooperative), maps: rc=$?"
