set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02v_t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/r02v_t.log
[ $rc -eq 0 ] || exit $rc
PROJ=1 timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids | head -4 && \
timeout -k 10 300 python bench.py --steps 20 --only render --no-cpu-baseline > gpurun_out/r02v_b.log 2>&1; rc=$?; echo bench rc=$rc; python tools/show_bench.py gpurun_out/r02v_b.log | grep render | cut -c1-250; exit $rc
