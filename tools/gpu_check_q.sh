set -o pipefail
for v in "" idle d6; do
  if [ -n "$v" ]; then export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$v.so; else unset INF_LIB; fi
  echo "== variant ${v:-default}"
  PROJ=1 timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids | tail -5 || exit 1
done
