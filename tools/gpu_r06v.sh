set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/gbar_ubench > $O/gbar.log 2>&1 || { cat $O/gbar.log; exit 1; }
cat $O/gbar.log
timeout -k 10 300 python3 -u tools/graph_stamps.py 64 30 2 fixed > $O/graph_fixed.log 2>&1 || { tail -20 $O/graph_fixed.log; exit 1; }
head -3 $O/graph_fixed.log
timeout -k 10 300 python3 -u tools/graph_stamps.py 64 30 2 natural > $O/graph_natural.log 2>&1 || { tail -20 $O/graph_natural.log; exit 1; }
head -3 $O/graph_natural.log
timeout -k 10 300 python3 -u tools/stamps.py 128 30 8 natural 2 > $O/stamps_natural.log 2>&1 || { tail -20 $O/stamps_natural.log; exit 1; }
head -3 $O/stamps_natural.log
