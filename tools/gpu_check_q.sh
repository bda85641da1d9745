set -o pipefail
for l in "" v1 v2 v4; do
  if [ -n "$l" ]; then export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$l.so; else unset INF_LIB; fi
  echo "== lib ${l:-default}"
  PROJ=1 timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids | sed -n '2p;4p' || exit 1
done
export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_v2.so
timeout -k 10 200 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 150 --timeout-method thread 2>&1 | tail -2
