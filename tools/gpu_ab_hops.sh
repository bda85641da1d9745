#!/bin/bash
# A/B of the config-B step (tools/hops_gain.py variants) between the tree's library and
# libinf_hip_$1.so, alternated twice
set -o pipefail
O=gpurun_out/${2:-abh}
mkdir -p $O
for r in 1 2; do
  for lib in new $1; do
    if [ $lib = new ]; then E=""; else E="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$lib.so INF_ALLOW_STALE_LIB=1"; fi
    env $E timeout -k 10 200 python3 tools/hops_gain.py > $O/${lib}_$r.log 2>&1 || { cat $O/${lib}_$r.log; exit 1; }
    echo "$lib $r: $(tail -1 $O/${lib}_$r.log)"
  done
done
