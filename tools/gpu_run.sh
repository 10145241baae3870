#!/bin/bash
# The one parametrised GPU launcher (replaces round 4's one-off gpu_r4*.sh scripts). Every step runs under
# its own time limit; the first failing step ends the call (set -e: no GPU step runs after a fault, abort or
# time-out). Every command is appended to $O/commands.txt before it runs, so every record under $O names the
# command it came from.
# usage (repo root on the box): bash tools/gpu_run.sh TAG STEP [STEP ...]
#   tests[:PYTEST_K]          pytest -m gpu [-k PYTEST_K]                    -> pytest.log
#   smoke                     __graft_entry__.smoke()                          -> smoke.log
#   bench:NAME[:ARGS]         python bench.py ARGS                            -> NAME.json (one JSON line)
#   prof:NAME[:ARGS]          rocprofv3 --kernel-trace --stats of bench.py     -> NAME_kernel_stats.csv
#   pmc:B                     FETCH_SIZE / WRITE_SIZE passes (separate runs) of the tower kernel at B envs
#                                                                              -> tower_hbm_traffic.json
#   sq:NAME:KERNELS[:ARGS]    two SQ counter passes of bench.py ARGS; KERNELS = comma-separated rocprof name
#                             substrings (e.g. "towerp_kernel<0>,towerp_kernel<1>") -> NAME/sq{1,2}_<k>.json
#   pmck:NAME:KERNEL:ENVS:H:W:ARGS  FETCH_SIZE / WRITE_SIZE / two SQ passes of one conv kernel over bench.py ARGS
#                                                                              -> NAME.json, conv_counters.json
#   rehearse:N:ENVS[:ARGS]    bench.py's N > 1 path: N ranks on cuda:0 over gloo (MZBA_DIST_REHEARSAL=1)
#                                                                              -> rehearse_nN.json
#   selflaunch:N:ENVS[:ARGS]  plain `bench.py --gpus N` (it starts its N ranks itself), ranks on cuda:0 over gloo
#                                                                              -> selflaunch_nN.json
#   py:NAME:SECONDS:CMD       any python tool (CMD = script + args)           -> NAME.log
set -euo pipefail
TAG=$1
shift
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
log() { echo "$*" >> $O/commands.txt; }
kname_py="import sys; sys.path.insert(0,'muzero-breakout_amd'); from mzba import _lib as L"

for step in "$@"; do
  IFS=: read -r kind name rest <<< "$step"
  case $kind in
    tests)
      k=()
      [ -n "${name:-}" ] && k=(-k "$name")
      cmd=(timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${k[@]}")
      log "${cmd[*]} > $O/pytest.log"
      "${cmd[@]}" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
      tail -2 $O/pytest.log ;;
    smoke)
      log "python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      log "python bench.py ${rest:-} > $O/$name.json"
      timeout -k 10 600 python bench.py ${rest:-} > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
      python3 tools/bench_summary.py $O/$name.json ;;
    prof)
      log "rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run -- python3 bench.py ${rest:-}"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run -- python3 bench.py ${rest:-} \
        > $O/prof_$name.log 2>&1 || { tail -20 $O/prof_$name.log; exit 1; }
      python3 tools/rocpd_report.py stats $O/prof_$name $O/${name}_kernel_stats.csv
      rm -rf $O/prof_$name ;;
    pmc)
      B=$name
      K=$(python3 -c "$kname_py; print({2: 'tower8_kernel<0, 2>', 3: 'tower8_kernel<0, 1>', 4: 'towerp_kernel<0>'}.get(L.lib().mzba_tower_plan($B), 'tower_kernel<0>'))")
      for c in FETCH_SIZE WRITE_SIZE; do
        log "rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o run -- python3 bench.py --envs $B --steps 1 --warmup 1 --no-graph --no-cpu --no-parity"
        timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o run -- python3 bench.py --envs $B --steps 1 \
          --warmup 1 --no-graph --no-cpu --no-parity > $O/pmc_${c}_$B.log 2>&1
      done
      python3 tools/pmc_tower_bench.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $B "$K" $O/tower_hbm_traffic.json
      rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE ;;
    sq)
      IFS=: read -r kernels args <<< "$rest"
      args=${args:-"--steps 1 --warmup 1 --no-graph --no-cpu --no-parity"}
      mkdir -p $O/$name
      p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
      p2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
      for pass in 1 2; do
        [ $pass = 1 ] && ctr=$p1 || ctr=$p2
        log "rocprofv3 --pmc $ctr --kernel-trace -d $O/$name/sq$pass -o run -- python3 bench.py $args"
        timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d $O/$name/sq$pass -o run -- python3 bench.py $args \
          > $O/$name/sq$pass.log 2>&1
        IFS=, read -ra ks <<< "$kernels"
        for k in "${ks[@]}"; do
          python3 tools/pmc_sq.py $O/$name/sq$pass "$k" "$O/$name/sq${pass}_$(echo "$k" | tr -c 'A-Za-z0-9_\n' '_').json" > /dev/null
        done
        rm -rf $O/$name/sq$pass
      done
      read -r envs sims dyn <<< "$(BENCH_ARGS="$args" python3 -c "import os, sys; sys.argv = ['bench.py'] + os.environ['BENCH_ARGS'].split(); import bench; a = bench.parse(); print(a.envs, a.sims, a.dyn_dtype)")"
      for k in "${ks[@]}"; do
        kk=$(echo "$k" | tr -c 'A-Za-z0-9_\n' '_')
        python3 tools/sq_record.py $O/$name/sq1_$kk.json $O/$name/sq2_$kk.json $envs "$k" "gpurun_out/$TAG/$name" \
          $O/tower_sq_counters.json $sims $dyn
      done
      echo "sq $name done: $kernels" ;;
    pmck)
      # pmck:NAME:KERNEL:ENVS:H:W:ARGS — HBM bytes + SQ figures of one conv kernel over bench.py ARGS (four --pmc passes
      # of their own) -> NAME.json (and merged into $O/conv_counters.json)
      IFS=: read -r kname envs hh ww args <<< "$rest"
      mkdir -p $O/$name
      i=0
      for ctr in "FETCH_SIZE" "WRITE_SIZE" \
                 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                 "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
        sub=(fetch write sq1 sq2); sub=${sub[$i]}; i=$((i + 1))
        log "rocprofv3 --pmc $ctr --kernel-trace -d $O/$name/$sub -o run -- python3 bench.py $args"
        timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d $O/$name/$sub -o run -- python3 bench.py $args \
          > $O/$name/$sub.log 2>&1
      done
      python3 tools/pmc_conv_summary.py $O/$name "$kname" $envs $hh $ww $O/conv_counters.json > $O/$name.json
      rm -rf $O/$name/fetch $O/$name/write $O/$name/sq1 $O/$name/sq2
      cat $O/$name.json ;;
    rehearse)
      N=$name
      IFS=: read -r envs args <<< "$rest"
      log "MZBA_DIST_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --envs $envs ${args:-}"
      MZBA_DIST_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
        --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --envs $envs ${args:-} \
        > $O/rehearse_n$N.json 2> $O/rehearse_n$N.err || { tail -30 $O/rehearse_n$N.err; exit 1; }
      python3 tools/bench_summary.py $O/rehearse_n$N.json ;;
    selflaunch)
      # plain `bench.py --gpus N` (no torchrun around it): bench.py starts its own N ranks (all on cuda:0, gloo)
      N=$name
      IFS=: read -r envs args <<< "$rest"
      log "MZBA_DIST_REHEARSAL=1 python bench.py --gpus $N --envs $envs ${args:-} > $O/selflaunch_n$N.json"
      MZBA_DIST_REHEARSAL=1 timeout -k 10 600 python bench.py --gpus $N --envs $envs ${args:-} \
        > $O/selflaunch_n$N.json 2> $O/selflaunch_n$N.err || { tail -30 $O/selflaunch_n$N.err; exit 1; }
      python3 tools/bench_summary.py $O/selflaunch_n$N.json ;;
    py)
      IFS=: read -r secs cmd <<< "$rest"
      log "python $cmd > $O/$name.log"
      timeout -k 10 $secs python $cmd > $O/$name.log 2>&1 || { tail -30 $O/$name.log; exit 1; }
      tail -5 $O/$name.log ;;
    *)
      echo "unknown step $step" >&2
      exit 2 ;;
  esac
done
echo "gpu_run $TAG done"
