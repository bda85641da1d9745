set -o pipefail
for l in "" r1 r4; do
  if [ -n "$l" ]; then export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$l.so; else unset INF_LIB; fi
  echo "== lib ${l:-default}"
  timeout -k 10 100 python tools/chain3_timing.py 2>&1 | grep -v amdgpu.ids | sed -n '1,4p;6p;10p' || exit 1
done
export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_r1.so
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread 2>&1 | tail -2
