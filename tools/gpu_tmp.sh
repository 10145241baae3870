set -o pipefail
O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "band or rep_tail or nets_f32 or nets_bf16" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 200 python tools/ab_rep.py 4096 > $O/ab_rep.json 2>$O/ab_rep.err && cat $O/ab_rep.json
for x in 0 5; do BSTAMP_LIB=libmzba_bstamp.so timeout -k 10 120 python tools/stamp_band.py 4096 $x $O/band_stamps_xt$x.json > /dev/null 2>&1; done
python -c "
import json
for x in (0,5):
    for r in json.load(open('$O/band_stamps_xt%d.json'%x)): print(x, r['cin'], r['cout'], round(r['launch_us']), round(r['frac_of_2500'],3), round(r['clock_ghz'],2), {k: round(v) for k,v in r['median_cycles'].items()}, round(r['k_loop_mfma_frac'],3))
"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-parity > $O/bench.json 2>/dev/null; python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'])"
