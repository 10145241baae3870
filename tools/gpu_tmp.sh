# tower8 k-step schedule variants: phase stamps of the isolated tower (diagnostic builds), interleaved
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/sched
mkdir -p $O
for i in 1 2; do
  for lib in libmzba_tstamp.so libmzba_tstamp_s1.so libmzba_tstamp_s2.so; do
    TSTAMP_LIB=$lib timeout -k 10 120 python tools/stamp_tower.py 4096 14 $O/stamps_${lib}_$i.json > $O/log_${lib}_$i.txt 2>&1
    python3 -c "import json; d=json.load(open('$O/stamps_${lib}_$i.json')); print('$lib', $i, d['launch_us'], d['cycles_per_conv'], round(d['clock_ghz'],3), d['phase_cycles'])"
  done
done
