# r04t: SQ counter passes (instruction mix, stalls, fp64) of the final headline kernel
set -o pipefail
timeout -k 10 900 bash tools/sqpmc.sh r04 > gpurun_out/sq_r04.log 2>&1 || exit 1
echo R04T_DONE
