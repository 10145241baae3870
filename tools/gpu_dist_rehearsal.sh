#!/bin/bash
# bench.py's N > 1 path on a one-GPU box: N ranks (torch.distributed.run, 127.0.0.1) all on cuda:0, gloo
# collectives instead of RCCL (MZBA_DIST_REHEARSAL=1): target-net broadcast, record gather to rank 0, barriers
# and the max-over-ranks timing (tools/gpu_run.sh 'rehearse' steps).
# usage (repo root on the box): bash tools/gpu_dist_rehearsal.sh TAG [ENVS_PER_RANK]
set -euo pipefail
E=${2:-512}
exec bash tools/gpu_run.sh $1 "rehearse:2:$E:--steps 20 --warmup 2" "rehearse:4:$E:--steps 20 --warmup 2"
