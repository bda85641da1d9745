set -o pipefail
for v in "" d6b1 d4b1; do
  if [ -n "$v" ]; then export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$v.so; else unset INF_LIB; fi
  echo "== variant ${v:-default}"
  PROJ=1 INF_PROJECT_GEMM=own timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids | tail -5 || exit 1
done
unset INF_LIB
echo "== hipBLASLt projection"
timeout -k 10 90 python -u tools/blaslt_check.py 2>&1 | grep -v amdgpu.ids
