# merged dx = -1 / +1 tower k loop: tower parity tests, then A/B against the previous build
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/dpm
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "tower_matches_conv_chain or fused_bf16_steps_vs_torch or fused_steps_match_unfused or rep_tail or fp16_dynamics or full_size_bf16 or tree_step_fused" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export MZBA_LIB_PARTIAL=1
M=$PWD/muzero-breakout_amd/mzba
bash tools/ab_tower.sh $O/conv libmzba_base.so libmzba.so
for B in 4096 1024; do
  for lib in libmzba_base.so libmzba.so libmzba_base.so libmzba.so; do
    MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --envs $B --steps 6 --warmup 2 --no-cpu > $O/bench_${B}_$lib.json 2> $O/bench_${B}_$lib.err
    python3 -c "import json; d=json.load(open('$O/bench_${B}_$lib.json')); print($B, '$lib', round(d['value'],1), round(d['roofline']['frac'],4), round(d['whole_step_mfma_frac'],4))"
  done
done
echo "dpm done"
