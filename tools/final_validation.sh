# final-tree validation: GPU tests, smoke, headline and learner bench lines, rocprof stats of the learner
set -e
D=gpurun_out/r6x; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 200 python bench.py --steps 8 --warmup 2 > $D/headline.json
timeout -k 10 200 python bench.py --workload learner --dtype bf16 --steps 10 --warmup 3 > $D/learner_bf16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_learner -o run -- python3 bench.py --workload learner --dtype bf16 --steps 6 --warmup 2 --no-cpu > $D/prof_learner.out 2>&1
