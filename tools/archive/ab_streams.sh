# A/B one box: learner streams=1 vs 2, graph and eager (usage: bash tools/ab_streams.sh <outdir>)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-st}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner.py -k "side_stream or graph_replay" > $O/pytest.log 2>&1
for i in 1 2; do
  for st in 1 2; do
    timeout -k 10 200 python bench.py --workload learner --steps 20 --warmup 5 --no-cpu --learner-streams $st > $O/graph_s${st}_$i.json 2> $O/graph_s${st}.err
    timeout -k 10 200 python bench.py --workload learner --steps 20 --warmup 5 --no-cpu --no-graph --learner-streams $st > $O/eager_s${st}_$i.json 2> $O/eager_s${st}.err
  done
done
