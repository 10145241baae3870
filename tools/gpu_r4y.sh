#!/bin/bash
# conv_halo two-block staging (Cin 256 past W = 30) + Cin/Cout 128: parity, then config 3 (the round-4 A/B against
# conv_big / conv_igemm used a temporary pack-time switch: profiles/r04/c3_halo_2blk/, ex20 = before)
set -o pipefail
O=gpurun_out/r4y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "halo" > $O/pytest_halo.log 2>&1 || { tail -30 $O/pytest_halo.log; exit 1; }
grep -E "max err|passed|failed" $O/pytest_halo.log
for i in 1 2; do
  for v in 1; do
    timeout -k 10 300 python bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 2 --warmup 1 > $O/c3_ex$v.$i.json 2> $O/c3_ex$v.$i.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/c3_ex$v.$i.json').read().strip().splitlines()[-1]); print('ex2=$v', d['value'], d['ms_per_step'])"
  done
done
