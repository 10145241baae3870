# tower8: one-pass k loop at NQ = 2 (ring 3), two passes at NQ = 1: full GPU suite + smoke, then A/B
# against the previous commit's build (libmzba_base.so)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/mix
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
export MZBA_LIB_PARTIAL=1
M=$PWD/muzero-breakout_amd/mzba
bash tools/ab_tower.sh $O/conv libmzba_base.so libmzba.so
for B in 4096 1024; do
  for lib in libmzba_base.so libmzba.so libmzba_base.so libmzba.so; do
    MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --envs $B --steps 6 --warmup 2 --no-cpu > $O/bench_${B}_$lib.json 2> $O/bench_${B}_$lib.err
    python3 -c "import json; d=json.load(open('$O/bench_${B}_$lib.json')); print($B, '$lib', round(d['value'],1), round(d['roofline']['frac'],4), round(d['whole_step_mfma_frac'],4))"
  done
done
echo "mix done"
