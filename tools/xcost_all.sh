set -e
for v in ${VARIANTS:-"" noxqp noroll nopair}; do
  if [ -n "$v" ]; then export PIADMM_LIB=$PWD/distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_$v.so; fi
  echo "== ${v:-full}"
  timeout -k 10 120 python3 tools/xcost.py
done
