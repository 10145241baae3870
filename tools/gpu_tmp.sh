# round run on the round's last tree (profiles/r02/r2l): GPU suite, smoke, headline + config 2, kernel
# stats, tower PMC traffic; then the learner bench and the tower phase stamps
set -euo pipefail
export TMPDIR=/tmp
bash tools/gpu_round.sh r2l
O=gpurun_out/r2l
timeout -k 10 300 python bench.py --workload learner > $O/learner_bench.json 2> $O/learner_bench.err
cat $O/learner_bench.json
timeout -k 10 120 python tools/stamp_tower.py 4096 14 $O/stamps_4096.json > $O/stamps_log.txt 2>&1 || { tail $O/stamps_log.txt; exit 1; }
python3 -c "import json; d=json.load(open('$O/stamps_4096.json')); print(d['launch_us'], d['clock_ghz'], d['cycles_per_conv'], d['mfma_frac_in_conv'])"
echo "r2l done"
