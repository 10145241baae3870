# tower8 launch timeline from the phase-stamp build (isolated tower, B = 4096 and 2048)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/timeline
mkdir -p $O
for B in 4096; do
  timeout -k 10 120 python tools/stamp_tower.py $B 14 $O/stamps_$B.json > $O/log_$B.txt 2>&1
  python3 -c "import json; d=json.load(open('$O/stamps_$B.json')); print($B, d['launch_us'], d['kernel_cycles_per_wg'], round(d['clock_ghz'],3), d['timeline_us'])"
done
