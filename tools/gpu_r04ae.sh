# r04ae: rocprofv3 kernel trace + stats and FETCH_SIZE / WRITE_SIZE passes of the final tree's headline
set -o pipefail
timeout -k 10 600 bash tools/profile.sh r04final > gpurun_out/prof_r04final.log 2>&1 || exit 1
echo R04AE_DONE
