#!/bin/bash
# One gpurun call: GPU parity tests, bench, kernel-trace stats, PMC passes on the dominant kernel.
# usage (from the repo root on the box): bash tools/gpu_round.sh TAG
set -e
TAG=${1:-run}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 && echo "pytest ok"
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err && echo "bench ok"
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof.log 2>&1 && echo "prof ok"
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats.csv
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/pmc_f.log 2>&1 && echo "pmc fetch ok"
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/pmc_w.log 2>&1 && echo "pmc write ok"
python3 tools/pmc_summarize.py $O/pmc_fetch $O/pmc_write 1024 $O/tower_hbm_traffic.json tower 14
rm -rf $O/pmc_fetch $O/pmc_write
