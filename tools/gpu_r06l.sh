# PMC traffic of every other bench line (tools/profile_line.sh)
set -o pipefail
R=${1:-r06}
bash tools/profile_line.sh ${R}_c5 tiled128_H50_matlab_pi_fixed100_tight k_mpc_step --config5 || exit 1
bash tools/profile_line.sh ${R}_c2 tiled32_H20_casadi_default_fixed200 k_mpc_step --config2 || exit 1
bash tools/profile_line.sh ${R}_c4 tiled512_H30_matlab_pi_fixed100 k_mpc_step --strong || exit 1
bash tools/profile_line.sh ${R}_x4 crossing4x64_H30_matlab_pi_fixed100 k_graph --crossing || exit 1
bash tools/profile_line.sh ${R}_ch chain1024_H30_matlab_pi_fixed100 k_graph --chain || exit 1
