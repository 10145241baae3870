# round run after the band kernel's one pass for every conv (profiles/r02/r2m) + learner bench
set -euo pipefail
export TMPDIR=/tmp
bash tools/gpu_round.sh r2m
O=gpurun_out/r2m
timeout -k 10 300 python bench.py --workload learner > $O/learner_bench.json 2> $O/learner_bench.err
python3 -c "import json; d=json.load(open('$O/learner_bench.json')); print('learner', round(d['value'],1), round(d['ms_per_step'],2))"
echo "r2m done"
