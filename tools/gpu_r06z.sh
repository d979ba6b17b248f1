# the exit fault under rocprofv3 on the flag-barrier tree: natural bench (cooperative launch), PMC pass
# and kernel-trace pass; each run's exit status recorded, nothing run after a failing GPU step
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o bench --output-format csv -- python3 bench.py --no-cpu --no-cold --natural --warmup 5 --steps 10 > $O/pmc_nat.log 2>&1
rc=$?; echo "pmc natural exit $rc"
[ $rc -eq 0 ] || exit 0
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py --no-cpu --no-cold --natural --warmup 5 --steps 10 > $O/trace_nat.log 2>&1
rc=$?; echo "kernel-trace natural exit $rc"
