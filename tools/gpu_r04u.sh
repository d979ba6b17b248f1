# r04u: A/B of 16-row batches in the dual active set's LDS passes (SINV_U = 16, the variant library
# libpiadmm_sinv16.so) against the default 8: headline, configs[4], crossings, chain.
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
V=distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_sinv16.so
B="python3 bench.py --no-cpu"
for W in "" "--config5" "--crossing" "--chain"; do
  n=$(echo "${W:-h}" | tr -d -)
  timeout -k 10 300 $B $W > $O/${n}_8.json 2> $O/${n}_8.err || exit 1
  PIADMM_LIB=$V timeout -k 10 300 $B $W > $O/${n}_16.json 2> $O/${n}_16.err || exit 1
done
echo R04U_DONE
