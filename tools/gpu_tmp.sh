# one-quad tower (config 2, NQ = 1): the one-pass column-major loop with a 6 / 12-entry ring
# (TOWER_Q1_ALL, libmzba_q6.so / libmzba_q12.so) vs the two-pass default (libmzba.so); parity tests on q12
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/q1
mkdir -p $O
M=$PWD/muzero-breakout_amd/mzba
MZBA_LIB=$M/libmzba_q12.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "tower_matches_conv_chain or fused_bf16_steps_vs_torch or fused_steps_match_unfused or fp16_dynamics or tree_step_fused" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_tower.sh $O/conv libmzba.so libmzba_q6.so libmzba_q12.so
for B in 1024; do
  for lib in libmzba.so libmzba_q6.so libmzba_q12.so libmzba.so libmzba_q6.so libmzba_q12.so; do
    MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --envs $B --steps 8 --warmup 2 --no-cpu > $O/bench_${B}_$lib.json 2> $O/bench_${B}_$lib.err
    python3 -c "import json; d=json.load(open('$O/bench_${B}_$lib.json')); print($B, '$lib', round(d['value'],1), round(d['roofline']['frac'],4), round(d['whole_step_mfma_frac'],4))"
  done
done
echo "q1 done"
