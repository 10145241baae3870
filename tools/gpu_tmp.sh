set -o pipefail
O=gpurun_out/r3h; mkdir -p $O
M=$PWD/muzero-breakout_amd/mzba
for i in 1 2; do for lib in libmzba.so libmzba_skew4.so libmzba_skew8.so libmzba_skew16.so; do
  echo -n "$lib " >> $O/ab.txt
  MZBA_LIB=$M/$lib timeout -k 10 200 python tools/ab_rep.py 4096 >> $O/ab.txt 2>>$O/ab.err || exit 1
done; done
cat $O/ab.txt | python -c "
import sys, json
for l in sys.stdin:
    lib, j = l.split(' ', 1); d = json.loads(j)
    print(lib, [round(x,3) for x in d['representation_ms_band_res_True']], round(d['block256']['band_res_us']), round(d['block256']['two_band_us']), round(d['block128']['band_res_us']), round(d['block128']['two_band_us']))
"
