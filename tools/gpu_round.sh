#!/bin/bash
# One gpurun call: GPU parity tests, bench, kernel-trace stats, PMC passes on the dominant kernel.
# usage (from the repo root on the box): bash tools/gpu_round.sh TAG
set -e
TAG=${1:-run}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo "pytest ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok"
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err && echo "bench ok"
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $O/prof.log 2>&1 && echo "prof ok"
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats.csv
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/pmc_f.log 2>&1 && echo "pmc fetch ok"
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/pmc_w.log 2>&1 && echo "pmc write ok"
python3 tools/pmc_summarize.py $O/pmc_fetch $O/pmc_write 1024 $O/tower_hbm_traffic.json tower 14
rm -rf $O/pmc_fetch $O/pmc_write
# HBM traffic of the env render kernel (config 3 geometry)
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/env_fetch -o run -- python3 bench.py --workload env --envs 4096 --height 84 --width 84 --hist 4 --steps 30 --warmup 5 --no-cpu > $O/env_f.log 2>&1 && echo "env fetch ok"
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/env_write -o run -- python3 bench.py --workload env --envs 4096 --height 84 --width 84 --hist 4 --steps 30 --warmup 5 --no-cpu > $O/env_w.log 2>&1 && echo "env write ok"
python3 - "$O" <<'PY'
import sys, json, statistics
sys.path.insert(0, "tools")
from rocpd_report import counter_values
o = sys.argv[1]
f = counter_values(o + "/env_fetch", "FETCH_SIZE", "env_step_compact_kernel")
w = counter_values(o + "/env_write", "WRITE_SIZE", "env_step_compact_kernel")
res = {"kernel": "env_step_compact_kernel", "envs": 4096, "H": 84, "W": 84,
       "fetch_bytes": statistics.median(f[10:]) * 1024 * 2 if f else None,
       "write_bytes": statistics.median(w[10:]) * 1024 if w else None, "algorithmic_bytes": 4096 * 7104,
       "n_samples": [len(f), len(w)], "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, median of launches 11..35, FETCH x2"}
json.dump(res, open(o + "/env_hbm_traffic.json", "w"), indent=1)
print(json.dumps(res))
PY
rm -rf $O/env_fetch $O/env_write
