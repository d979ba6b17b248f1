# r04p: OBCA with the linearisation blocks in HBM (LDS 48.3 -> 39.0 KB per problem: four problems
# per CU) -- its GPU parity tests, then the --obca bench line (CPU baselines included), then the
# evidence part 2 (stamps, the other bench lines).
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_obca.py > $O/tests_obca.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --obca > $O/bench_obca.json 2> $O/bench_obca.err || exit 1
bash tools/gpu_r04o.sh || exit 1
echo R04P_DONE
