# r04y: per-iteration profile of the chain's last steps (what makes its Z launches slow)
set -o pipefail
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 500 python3 -u tools/chain_iter_profile.py 17 3 > $O/chain_iter.log 2>&1 || exit 1
echo R04Y_DONE
