#!/bin/bash
# One gpurun call: every BASELINE config on the current tree (one MI355X). JSON lines under
# gpurun_out/TAG/. Any failure ends it.
# usage (repo root on the box): bash tools/gpu_configs.sh TAG
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python bench.py --workload env --envs 64 --height 16 --width 20 --hist 32 --steps 200 --warmup 20 > $O/config1_env_64.json 2> $O/c1.err
timeout -k 10 300 python bench.py --envs 1024 --steps 10 --warmup 3 > $O/config2_1024x50.json 2> $O/c2.err
timeout -k 10 200 python bench.py --workload env --envs 4096 --height 84 --width 84 --hist 4 --steps 200 --warmup 5 > $O/config3_env_84x84_4096.json 2> $O/c3e.err
timeout -k 10 400 python bench.py --envs 4096 --height 84 --width 84 --hist 4 --steps 2 --warmup 1 --no-cpu > $O/config3_acting_84x84_4096x50.json 2> $O/c3a.err
timeout -k 10 400 python bench.py --envs 4096 --sims 200 --dyn-dtype fp16 --steps 3 --warmup 1 --no-cpu > $O/config5_4096x200_fp16dyn.json 2> $O/c5.err
timeout -k 10 400 python bench.py --envs 4096 --sims 200 --steps 3 --warmup 1 --no-cpu > $O/config5_4096x200_bf16.json 2> $O/c5b.err
for f in $O/config*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value'],1), d['unit'], d.get('roofline',{}).get('frac'))"; done
echo configs done
