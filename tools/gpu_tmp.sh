set -o pipefail
O=gpurun_out/r3m; mkdir -p $O
for i in 1 2; do for lib in libmzba_tstamp.so libmzba_tstamp_ab5.so libmzba_tstamp_ab6.so; do
  TSTAMP_LIB=$lib timeout -k 10 120 python tools/stamp_tower.py 4096 14 > $O/st_${lib}_$i.json 2>>$O/err.txt || exit 1
  python -c "
import json; r=json.load(open('$O/st_${lib}_$i.json'))
print('$lib', round(r['launch_us']), round(r['clock_ghz'],3), round(r['cycles_per_conv']), {k: round(v) for k,v in r['phase_cycles'].items()})"
done; done
