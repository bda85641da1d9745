set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prefetch.py tests/test_gpu_trainer_state.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c3_t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/c3_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/chain3_timing.py 2>&1 | grep -v amdgpu.ids | grep -E "stage|fwd6" && \
timeout -k 10 200 python bench.py --steps 200 --only none --no-cpu-baseline > gpurun_out/c3_b.log 2>&1 && python tools/show_bench.py gpurun_out/c3_b.log | head -2
