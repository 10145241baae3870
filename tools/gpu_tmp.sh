# A/B of two library builds on one box: the headline acting bench, interleaved, and the band tests
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_heads
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or tower or fp16 or acting or episode or smoke" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for i in 1 2; do
  for lib in libmzba_towerold.so libmzba.so; do
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu > $O/bench_${lib}_$i.json 2> $O/bench_${lib}_$i.err
    python3 -c "import json,sys; d=json.load(open('$O/bench_${lib}_$i.json')); print('$lib', $i, round(d['value'],1), round(d['ms_per_step'],2), round(d['roofline']['frac'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu > $O/prof.log 2>&1
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats_4096.csv
rm -rf $O/prof
head -12 $O/kernel_stats_4096.csv
