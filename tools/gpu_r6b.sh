#!/bin/bash
# Round 6: GPU suite after the update-launch change, its per-item stamps, A/B of the headline
# legs against the HEAD-before library (libinf_hip_base.so), and chain4's SQ counter pass.
set -o pipefail
O=gpurun_out/${1:-r6b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
BASE="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_base.so INF_ALLOW_STALE_LIB=1"
timeout -k 10 120 python3 tools/update_items.py > $O/upd_new.log 2>&1 || exit 1
env $BASE timeout -k 10 120 python3 tools/update_items.py > $O/upd_base.log 2>&1 || exit 1
grep "update stage" $O/upd_new.log $O/upd_base.log
grep -A6 "trial 2" $O/upd_new.log
H="--steps 200 --warmup 8 --no-render --no-cpu-baseline --no-config-d --extra-batches= --only none"
A="--k 64 --layers 4 --hidden 128 --skip 2 --verts 20000"
R="--k 1023 --layers 6 --hidden 128 --skip 3 --loss L1"
for r in 1 2; do
 for lib in new base; do
  for cfg in B A R; do
    case $cfg in A) X=$A;; R) X=$R;; B) X="";; esac
    if [ $lib = base ]; then E=$BASE; else E=""; fi
    env $E timeout -k 10 120 python3 bench.py $H $X > $O/ab_${cfg}_${lib}_$r.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/ab_${cfg}_${lib}_$r.log') if l.startswith('{')][-1]); print('$cfg $lib $r', round(d['ms_per_step']*1e3,2), {k: round(v['ms']*1e3,2) for k,v in d['stages'].items()})"
  done
 done
done
bash scratch/pmc4.sh ${1:-r6b}/pmc4 > $O/pmc4.log 2>&1; tail -30 $O/pmc4.log
