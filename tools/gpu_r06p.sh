set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/distributed-local-planner-pi-admm_amd/piadmm
PIADMM_LIB=$L/libpiadmm_stamps_wb.so timeout -k 10 300 python3 -u tools/stamps.py 128 30 8 natural 4 > $O/stamps_natural_wb.log 2>&1 || { tail -20 $O/stamps_natural_wb.log; exit 1; }
sed -n '/per wave, mean/,$p' $O/stamps_natural_wb.log | head -40
head -1 $O/stamps_natural_wb.log | cut -c1-250
