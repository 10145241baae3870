#!/bin/bash
# One gpurun call for the env render kernel (config 3 geometry): GPU tests, env bench,
# kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes (separate runs).
# usage (repo root on the box): bash tools/gpu_env.sh TAG [pytest -k expr]
set -e
TAG=${1:-env}
K=${2:-}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
fi
tail -2 $O/pytest.log
EB="bench.py --workload env --envs 4096 --height 84 --width 84 --hist 4 --steps 200 --warmup 5"
timeout -k 10 200 python $EB > $O/env_bench.json 2> $O/env_bench.err
cat $O/env_bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/env_prof -o run -- python3 $EB --no-cpu > $O/env_prof.log 2>&1
python3 tools/rocpd_report.py stats $O/env_prof $O/env_kernel_stats.csv
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/env_fetch -o run -- python3 $EB --no-cpu > $O/env_f.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/env_write -o run -- python3 $EB --no-cpu > $O/env_w.log 2>&1
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
