# r04v: the in-kernel global stop's grid barrier as one arrival counter (relaxed poll + one acquire)
# in place of cooperative_groups' grid sync -- the coop / natural-termination parity tests, then
# the natural lines (headline, configs[3] on one GPU, crossings).
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_modes.py tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_outer_iter.py -k "global or termination or coop or natural or golden or persistent or async" > $O/tests.log 2>&1 || exit 1
B="python3 bench.py --no-cpu"
timeout -k 10 300 $B > $O/h.json 2> $O/h.err || exit 1
timeout -k 10 300 $B --strong > $O/strong.json 2> $O/strong.err || exit 1
timeout -k 10 300 $B --config2 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 $B --crossing > $O/x4.json 2> $O/x4.err || exit 1
echo R04V_DONE
