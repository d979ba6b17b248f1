# Graph-kernel investigation (r04): per-launch kernel durations of the chain (X / Z launches) and of
# the crossing under host-stepped natural termination (one launch per outer iteration).
set -o pipefail
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04b/chain -o chain --output-format csv -- python3 bench.py --chain --no-cpu --no-natural --steps 2 --warmup 0 > gpurun_out/r04b/chain.log 2>&1 && \
PIADMM_NO_COOP=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04b/x4n -o x4n --output-format csv -- python3 bench.py --crossing --natural --no-cpu --steps 3 --warmup 0 > gpurun_out/r04b/x4n.log 2>&1 && \
timeout -k 10 300 python3 bench.py --crossing --no-cpu --steps 20 --warmup 5 > gpurun_out/r04b/x4.json 2> gpurun_out/r04b/x4.err && \
timeout -k 10 300 python3 bench.py --chain --no-cpu --steps 20 --warmup 5 > gpurun_out/r04b/chain.json 2> gpurun_out/r04b/chain.err
echo R04B_DONE
