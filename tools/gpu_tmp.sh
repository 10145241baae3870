# band kernel width A/B (10 vs 5 output columns per workgroup) after the staging batch fix
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/band_xt2
mkdir -p $O
for i in 1 2; do timeout -k 10 200 python tools/bench_band_xt.py 4096 >> $O/band_xt.jsonl 2> $O/err.txt; done
cat $O/band_xt.jsonl | cut -c1-200
