set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r02p_t.log 2>&1; rc=$?; echo rc=$rc; tail -15 gpurun_out/r02p_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids && PROJ=1 timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids && \
timeout -k 10 200 python bench.py --steps 50 --only render --no-cpu-baseline > gpurun_out/r02p_b.log 2>&1; rc=$?; python tools/show_bench.py gpurun_out/r02p_b.log | grep -i render | cut -c1-900; exit $rc
