#!/bin/bash
# Same-box A/B of the trunk k-loop schedule: the shipped library vs libmzba_rfN.so (make rf-prod),
# representation timing at B = 4096 (tools/ab_reptrunk.py), alternated twice.
set -euo pipefail
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in base $2; do
    lib=muzero-breakout_amd/mzba/libmzba.so
    [ "$v" != base ] && lib=muzero-breakout_amd/mzba/libmzba_rf$v.so
    MZBA_LIB=$PWD/$lib timeout -k 10 200 python tools/ab_reptrunk.py > $O/rep_$v.$i.json 2> $O/rep_$v.$i.err
    python3 -c "import json; d=json.load(open('$O/rep_$v.$i.json')); print('$v', d['representation_ms_rep_trunk_True'])"
  done
done
