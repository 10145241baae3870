# band kernel one-pass k loop (default build, libmzba.so) vs the three per-shift loops
# (BAND_ONEPASS=0, libmzba_base.so): band / representation parity tests, isolated band convs, headline
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/band1
mkdir -p $O
M=$PWD/muzero-breakout_amd/mzba
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "band or rep_tail or nets_bf16 or full_size_bf16 or fused_bf16_steps_vs_torch" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export MZBA_LIB_PARTIAL=1
for i in 1 2; do
  for lib in libmzba_base.so libmzba.so; do
    MZBA_LIB=$M/$lib timeout -k 10 120 python tools/bench_band_xt.py 4096 > $O/band_${lib}_$i.log 2>&1
    echo "== $lib $i"; cat $O/band_${lib}_$i.log
  done
done
for lib in libmzba_base.so libmzba.so libmzba_base.so libmzba.so; do
  MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --envs 4096 --steps 6 --warmup 2 --no-cpu > $O/bench_$lib.json 2> $O/bench_$lib.err
  python3 -c "import json; d=json.load(open('$O/bench_$lib.json')); print('$lib', round(d['value'],1), round(d['roofline']['frac'],4), round(d['whole_step_mfma_frac'],4))"
done
echo "band1 done"
