# r04x: kernel trace of the 1024-agent chain (a component split over 256 workgroups; fixed
# iterations): the X / Z / partials launch durations per outer iteration, steps 0..4 and 15..19.
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o tr --output-format csv -- python3 bench.py --chain --no-cpu --no-natural --steps 20 --warmup 1 > $O/trace.log 2>&1 || exit 1
echo R04X_DONE
