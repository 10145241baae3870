# A/B one box: learner bench with an environment flag 0 vs 1 (usage: bash tools/ab_env_flag.sh <outdir> <VAR>)
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-abf}
V=$2
mkdir -p $O
for i in 1 2; do
  for f in 0 1; do
    env $V=$f timeout -k 10 200 python bench.py --workload learner --steps 20 --warmup 5 --no-cpu > $O/${V}_${f}_$i.json 2> $O/err_$f.log
  done
done
