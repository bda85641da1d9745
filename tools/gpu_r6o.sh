#!/bin/bash
# Round 6: zg.hip's two-phase schedule -- bitwise the round-start zg (step fingerprints under
# both libraries), its parity tests, and config D's step against the round-start library.
set -o pipefail
O=gpurun_out/${1:-r6o}
mkdir -p $O
BASE="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_base.so INF_ALLOW_STALE_LIB=1"
for args in "4096 4096" "1024 4096" "4096 2048"; do
  timeout -k 10 120 python3 tools/step_hash.py $args > $O/hash_new.log 2>&1 || { cat $O/hash_new.log; exit 1; }
  env $BASE timeout -k 10 120 python3 tools/step_hash.py $args > $O/hash_base.log 2>&1 || exit 1
  echo "new  $(tail -1 $O/hash_new.log)"; echo "base $(tail -1 $O/hash_base.log)"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_config_d_adam.py tests/test_gpu_kernels.py -k "zg or chunked or config_d" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then E=$BASE; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --only configD --no-render --no-cpu-baseline --extra-batches= > $O/d_${lib}_$r.log 2>&1 || exit 1
    grep '^{' $O/d_${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config_D']; print('$lib $r D', round(c['ms_per_step']*1e3,2), {k: round(v['ms']*1e3,2) for k,v in c['stages'].items()})"
  done
done
