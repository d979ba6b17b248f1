# r04 experiments: price of the near-tie log (a -DPIADMM_NO_TIES build) with and without the roller
# wave; graph-kernel per-launch durations (chain X / Z launches, crossing one launch per iteration).
set -o pipefail
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
NT=distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_noties.so
B="python3 bench.py --no-cpu"
timeout -k 10 200 $B > gpurun_out/r04b/h_ties_roll.json 2>/dev/null && \
PIADMM_LIB=$NT timeout -k 10 200 $B > gpurun_out/r04b/h_noties_roll.json 2>/dev/null && \
PIADMM_NO_ROLLER=1 PIADMM_LIB=$NT timeout -k 10 200 $B > gpurun_out/r04b/h_noties_noroll.json 2>/dev/null && \
timeout -k 10 200 $B --config2 > gpurun_out/r04b/c2_ties.json 2>/dev/null && \
PIADMM_LIB=$NT timeout -k 10 200 $B --config2 > gpurun_out/r04b/c2_noties.json 2>/dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04b/chain -o chain --output-format csv -- python3 bench.py --chain --no-cpu --no-natural --steps 2 --warmup 0 > gpurun_out/r04b/chain.log 2>&1 && \
PIADMM_NO_COOP=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r04b/x4n -o x4n --output-format csv -- python3 bench.py --crossing --natural --no-cpu --steps 3 --warmup 0 > gpurun_out/r04b/x4n.log 2>&1
echo R04B_DONE
