# evidence of the current kernel: headline kernel trace + PMC traffic, SQ counters
set -o pipefail
TAG=${1:-r06a}
bash tools/profile.sh $TAG || exit 1
tail -3 gpurun_out/prof_$TAG/traffic.log
bash tools/sqpmc.sh $TAG || exit 1
cat gpurun_out/sq_$TAG/summary.txt | tail -20
