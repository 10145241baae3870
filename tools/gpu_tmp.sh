# confirmation on the committed tree: GPU suite, smoke, default bench
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.load(open('$O/bench.json')); print(round(d['value'],1), round(d['roofline']['frac'],4), round(d['whole_step_mfma_frac'],4), d['cpu_baseline']['value'])"
echo "final2 done"
