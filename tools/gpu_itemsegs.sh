#!/bin/bash
# The update launch with each item's segment copy loaded beside the item (AdamArgs::item_segs):
# GPU suite, the headline A/B against the library before it (libinf_hip_base.so), and the
# update's per-item stamps in the step.
set -o pipefail
O=gpurun_out/${1:-itemsegs}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_base.sh ${1:-itemsegs}/ab || exit 1
UPD_STEP=1 timeout -k 10 120 python3 tools/update_items.py > $O/update_items_step.log 2>&1 || exit 1
tail -8 $O/update_items_step.log
