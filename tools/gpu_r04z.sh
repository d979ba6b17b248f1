# r04z: phase stamps of the chain's last steps (diagnostic stamps build)
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 400 python3 -u tools/chain_stamps.py 17 3 > $O/chain_stamps.log 2>&1 || exit 1
echo R04Z_DONE
