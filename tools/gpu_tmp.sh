set -o pipefail
O=gpurun_out/r3e; mkdir -p $O
M=$PWD/muzero-breakout_amd/mzba
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1; grep "^seed" $O/pytest.log
for i in 1 2; do for lib in libmzba_b128.so libmzba.so; do
  MZBA_LIB=$M/$lib timeout -k 10 120 python tools/ab_band128.py >> $O/band_ab.jsonl 2>/dev/null
  MZBA_LIB=$M/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --no-parity > $O/bench_${lib}_$i.json 2>/dev/null
done; done
cat $O/band_ab.jsonl; for f in $O/bench_*.json; do echo $f; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'])"; done
for x in 5 10; do BSTAMP_LIB=libmzba_bstamp.so timeout -k 10 120 python tools/stamp_band.py 4096 $x $O/band_stamps_xt$x.json > /dev/null 2>&1; done
for e in 0 1 0 1; do STAMP_ELEM=$e timeout -k 10 120 python tools/stamp_tower.py 4096 14 >> $O/tower_stamps_elem.jsonl 2>/dev/null; done
python -c "
import json
for x in (5,10):
    for r in json.load(open('$O/band_stamps_xt%d.json'%x)): print(x, r['cin'], r['cout'], round(r['launch_us']), round(r['frac_of_2500'],3), round(r['clock_ghz'],2), {k: round(v) for k,v in r['median_cycles'].items()}, round(r['k_loop_mfma_frac'],3))
for l in open('$O/tower_stamps_elem.jsonl'):
    r=json.loads(l); print(r['elem'], round(r['launch_us']), round(r['clock_ghz'],3), round(r['cycles_per_conv']), {k: round(v) for k,v in r['phase_cycles'].items()})
"
