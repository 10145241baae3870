#!/bin/bash
# Round-4 GPU call: the GPU test suite, then a same-box A/B of the previous library (libmzba_base.so) against
# the working tree's libmzba.so on the headline bench (alternated twice), then the SQ counter passes of the
# dominant kernel for the new library. Every GPU step has its own time limit; any failure ends the script.
# usage (repo root on the box): bash tools/gpu_r4.sh TAG [skip-tests]
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
    > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
  tail -3 $O/pytest.txt
fi
for i in 1 2; do
  for lib in libmzba_base.so libmzba.so; do
    MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --no-cpu --no-parity --steps 8 --warmup 2 > $O/bench_${lib}_$i.json 2> $O/bench_${lib}_$i.err
    python3 -c "import json; d=json.load(open('$O/bench_${lib}_$i.json')); r=d['roofline']; print('$lib', round(d['value'],1), round(r['avg_launch_ms'],4), round(r['frac'],4))"
  done
done
bash tools/pmc_towerp_sq.sh $1/sq_new
python3 tools/sq_record.py $O/sq_new/sq1.json $O/sq_new/sq2.json 4096 towerp_kernel gpurun_out/$1/sq_new $O/tower_sq_counters.json
echo r4 done
