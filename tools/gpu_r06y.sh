set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
export TMPDIR=/tmp
PIADMM_STAMPS_PRESET=casadi_default timeout -k 10 300 python3 -u tools/stamps.py 32 20 16 natural 2 > $O/stamps_c2_natural.log 2>&1 || { tail -20 $O/stamps_c2_natural.log; exit 1; }
head -2 $O/stamps_c2_natural.log
bash tools/profile_line.sh r06_c2 tiled32_H20_casadi_default_fixed200 k_mpc_step --config2
