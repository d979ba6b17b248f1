#!/bin/bash
# N-rank rehearsal of bench.py on the one GPU (run on the GPU box from the repo root): the library's
# host all-reduce transport over gloo (RCCL refuses two ranks on one device), N ranks sharing the
# device -- a path check of `bench.py --gpus N`, not a scaling number.  Stops at the first failure.
set -o pipefail
O=gpurun_out/rehearse
mkdir -p $O
export TMPDIR=/tmp
for N in 2 4; do
  for extra in "" "--natural"; do
    tag=n$N${extra:+_natural}
    PIADMM_BENCH_TRANSPORT=host timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus $N --steps 10 --warmup 3 --no-cpu --no-cold $extra > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['n_gpus'], d['ms_per_step'], d['value'])"
  done
done
