#!/bin/bash
# One gpurun call: every BASELINE config on the current tree (one MI355X), JSON lines under gpurun_out/TAG/
# (tools/gpu_run.sh steps; config 4 = the headline per GPU, its 8-way partition in tests/test_gpu_configs.py).
# usage (repo root on the box): bash tools/gpu_configs.sh TAG
set -euo pipefail
exec bash tools/gpu_run.sh $1 \
  "bench:config1_env_64:--workload env --envs 64 --height 16 --width 20 --hist 32 --steps 200 --warmup 20" \
  "bench:config2_1024x50:--envs 1024 --steps 10 --warmup 3" \
  "bench:config3_env_84x84_4096:--workload env --envs 4096 --height 84 --width 84 --hist 4 --steps 200 --warmup 5" \
  "bench:config3_acting_84x84_4096x50:--envs 4096 --height 84 --width 84 --hist 4 --steps 2 --warmup 1 --no-cpu" \
  "bench:config5_4096x200_fp16dyn:--envs 4096 --sims 200 --dyn-dtype fp16 --steps 3 --warmup 1 --no-cpu" \
  "bench:config5_4096x200_bf16:--envs 4096 --sims 200 --steps 3 --warmup 1 --no-cpu"
