set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/stamps.py 128 30 8 natural 4 > $O/stamps_natural.log 2>&1 || { tail -20 $O/stamps_natural.log; exit 1; }
timeout -k 10 300 python3 -u tools/stamps.py 128 30 4 fixed 2 > $O/stamps_fixed.log 2>&1 || { tail -20 $O/stamps_fixed.log; exit 1; }
tail -40 $O/stamps_natural.log
