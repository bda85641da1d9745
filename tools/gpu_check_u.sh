set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_render.py tests/test_gpu_large.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02u_t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/r02u_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids | head -2 && PROJ=1 timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids | head -3 && \
timeout -k 10 300 python bench.py --steps 100 --only render --no-cpu-baseline > gpurun_out/r02u_b.log 2>&1; rc=$?; echo bench rc=$rc; python tools/show_bench.py gpurun_out/r02u_b.log | cut -c1-250 | head -4; exit $rc
