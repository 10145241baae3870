# one-pass tower loop column-tile major with a 6-entry ring (TOWER_DALL_CT=1, libmzba_ct.so) vs the
# default build (libmzba.so): tower parity tests on the variant, isolated tower and headline A/B, stamps
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/ct
mkdir -p $O
M=$PWD/muzero-breakout_amd/mzba
MZBA_LIB=$M/libmzba_ct.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "tower_matches_conv_chain or fused_bf16_steps_vs_torch or fused_steps_match_unfused or rep_tail or fp16_dynamics or full_size_bf16 or tree_step_fused" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_tower.sh $O/conv libmzba.so libmzba_ct.so
for B in 4096; do
  for lib in libmzba.so libmzba_ct.so libmzba.so libmzba_ct.so; do
    MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --envs $B --steps 6 --warmup 2 --no-cpu > $O/bench_${B}_$lib.json 2> $O/bench_${B}_$lib.err
    python3 -c "import json; d=json.load(open('$O/bench_${B}_$lib.json')); print($B, '$lib', round(d['value'],1), round(d['roofline']['frac'],4), round(d['whole_step_mfma_frac'],4))"
  done
done
TSTAMP_LIB=libmzba_tstamp_ct.so timeout -k 10 120 python tools/stamp_tower.py 4096 14 $O/stamps_ct.json > $O/stamps_log.txt 2>&1 || { tail $O/stamps_log.txt; exit 1; }
python3 -c "import json; d=json.load(open('$O/stamps_ct.json')); print(d['launch_us'], d['clock_ghz'], d['cycles_per_conv'], d['mfma_frac_in_conv'], d['phase_cycles'])"
echo "ct done"
