# round run on the one-pass column-major tower (profiles/r02/r2k) + tower8 phase stamps at B = 4096
set -euo pipefail
export TMPDIR=/tmp
bash tools/gpu_round.sh r2k
O=gpurun_out/r2k
timeout -k 10 120 python tools/stamp_tower.py 4096 14 $O/stamps_4096.json > $O/stamps_log.txt 2>&1 || { tail $O/stamps_log.txt; exit 1; }
python3 -c "import json; d=json.load(open('$O/stamps_4096.json')); print(d['launch_us'], d['clock_ghz'], d['cycles_per_conv'], d['mfma_frac_in_conv'], d['phase_cycles'])"
echo "r2k done"
