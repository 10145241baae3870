set -euo pipefail
export TMPDIR=/tmp MZBA_LIB_PARTIAL=1
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_learner.log 2>&1
tail -2 $O/pytest_learner.log
for lib in libmzba_base.so libmzba.so; do
  MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 400 python bench.py --workload learner --steps 10 --warmup 3 > $O/learner_$lib.json 2> $O/learner_$lib.err
  python3 -c "import json,sys; d=json.load(open('$O/learner_$lib.json')); print('$lib', round(d['value']), d['unit'], round(d['ms_per_step'],2))"
done
