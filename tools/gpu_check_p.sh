set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02p_t.log 2>&1; rc=$?; echo rc=$rc; tail -2 gpurun_out/r02p_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 90 python -u tools/blaslt_check.py 2>&1 | grep -v amdgpu.ids
