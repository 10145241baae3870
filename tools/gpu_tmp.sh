set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
for v in 1 3; do
  timeout -k 10 300 python bench.py --envs 1024 --steps 10 --warmup 2 --no-cpu --tower-variant $v > $O/bench1024_v${v}_${i}.json 2> $O/bench_v$v.err
  python3 -c "import json,sys; d=json.load(open('$O/bench1024_v${v}_${i}.json')); print('v$v', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],4))"
done
done
