#!/bin/bash
# bench.py's N > 1 path on a one-GPU box: N ranks (torch.distributed.run, 127.0.0.1) all on cuda:0,
# gloo collectives instead of RCCL (MZBA_DIST_REHEARSAL=1): target-net broadcast, record gather to
# rank 0, barriers and the max-over-ranks timing. usage (repo root on the box): bash tools/gpu_dist_rehearsal.sh TAG
set -euo pipefail
export TMPDIR=/tmp MZBA_DIST_REHEARSAL=1
O=gpurun_out/$1
mkdir -p $O
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N --envs 512 --steps 20 --warmup 2 > $O/bench_n$N.json 2> $O/bench_n$N.err
  cat $O/bench_n$N.json
done
