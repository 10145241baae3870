# A/B one box: learner bench from ab_old/ (previous commit's Python, same libmzba.so) vs the tree
# usage on the box: bash tools/ab_learner_py.sh <outdir>
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-abl}
mkdir -p $O
LIBP=$PWD/muzero-breakout_amd/mzba/libmzba.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner.py > $O/pytest.log 2>&1
for i in 1 2; do
  (cd ab_old && MZBA_LIB=$LIBP timeout -k 10 200 python bench.py --workload learner --steps 20 --warmup 5 --no-cpu > $O/old_$i.json 2> $O/old.err)
  timeout -k 10 200 python bench.py --workload learner --steps 20 --warmup 5 --no-cpu > $O/new_$i.json 2> $O/new.err
done
