# r04ad: A/B of more warm-label reduced solves before a graph pair QP's dual active set
# (PIADMM_PAIR_PDAS = 1 default, 3, 6): chain and crossings.
set -o pipefail
O=gpurun_out/r04ad
mkdir -p $O
B="python3 bench.py --no-cpu"
for P in 1 3 6; do
  PIADMM_PAIR_PDAS=$P timeout -k 10 300 $B --chain > $O/chain_$P.json 2> $O/chain_$P.err || exit 1
  PIADMM_PAIR_PDAS=$P timeout -k 10 300 $B --crossing > $O/x4_$P.json 2> $O/x4_$P.err || exit 1
done
echo R04AD_DONE
