# A/B of two library builds on one box (headline acting bench, interleaved) after the whole GPU suite
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_agpr
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for i in 1 2; do
  for lib in libmzba_prev.so libmzba.so; do
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu > $O/bench_${lib}_$i.json 2> $O/bench_${lib}_$i.err
    python3 -c "import json,sys; d=json.load(open('$O/bench_${lib}_$i.json')); print('$lib', $i, round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
  done
done
