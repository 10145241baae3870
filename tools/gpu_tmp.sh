set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "band" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 200 python tools/bench_band_xt.py 4096 > $O/band_xt.log 2>&1
python3 -c "
import json
for l in open('$O/band_xt.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['xt'], d['Cin'], d['Cout'], round(d['us'],1), round(d['tflops'],1))"
