#!/bin/bash
# One gpurun call: GPU parity tests, smoke, the headline bench (north_star 4096 x 50) and config 2
# (1024 x 50), kernel-trace stats, and PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) on the
# dominant kernel inside the bench. Any failing or timed-out step ends the script (set -e).
# usage (from the repo root on the box): bash tools/gpu_round.sh TAG [skip-tests]
set -euo pipefail
TAG=${1:-run}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  tail -2 $O/pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 300 python bench.py --envs 1024 --steps 10 --warmup 3 --no-cpu --no-parity > $O/bench_1024.json 2> $O/bench_1024.err
cat $O/bench_1024.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu --no-parity > $O/prof.log 2>&1
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats_4096.csv
rm -rf $O/prof
for B in 4096 1024; do
  K=$(python3 -c "import sys; sys.path.insert(0,'muzero-breakout_amd'); from mzba import _lib as L; print({2: 'tower8_kernel<0, 2>', 3: 'tower8_kernel<0, 1>', 4: 'towerp_kernel'}.get(L.lib().mzba_tower_plan($B), 'tower_kernel<0>'))")
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 bench.py --envs $B --steps 1 --warmup 1 --no-graph --no-cpu --no-parity > $O/pmc_f_$B.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 bench.py --envs $B --steps 1 --warmup 1 --no-graph --no-cpu --no-parity > $O/pmc_w_$B.log 2>&1
  python3 tools/pmc_tower_bench.py $O/pmc_fetch $O/pmc_write $B "$K" $O/tower_hbm_traffic.json
  rm -rf $O/pmc_fetch $O/pmc_write
done
echo "round script done"
