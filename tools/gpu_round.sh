#!/bin/bash
# One gpurun call: GPU parity tests, smoke, the headline bench (north_star 4096 x 50) and config 2 (1024 x 50),
# kernel-trace stats, and the HBM-traffic PMC passes on the dominant kernel (tools/gpu_run.sh steps).
# usage (from the repo root on the box): bash tools/gpu_round.sh TAG [skip-tests]
set -euo pipefail
TAG=${1:-run}
pre=(tests smoke)
[ "${2:-}" = "skip-tests" ] && pre=()
exec bash tools/gpu_run.sh $TAG "${pre[@]}" "bench:bench" \
  "bench:bench_1024:--envs 1024 --steps 10 --warmup 3 --no-cpu --no-parity" \
  "prof:4096:--steps 4 --warmup 2 --no-cpu --no-parity" pmc:4096 pmc:1024
