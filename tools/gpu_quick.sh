#!/bin/bash
# One gpurun call: GPU parity tests, smoke, the headline bench. Any failing step ends the script.
# usage (repo root on the box): bash tools/gpu_quick.sh TAG [pytest -k expression]
set -euo pipefail
TAG=${1:-quick}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
fi
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
