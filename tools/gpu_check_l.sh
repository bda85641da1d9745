timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py tests/test_gpu_render.py tests/test_gpu_frontends.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02l_t.log 2>&1; rc=$?; echo rc=$rc; tail -3 gpurun_out/r02l_t.log
if [ $rc -eq 0 ]; then
  timeout -k 10 100 python tools/chain3_timing.py 2>&1 | grep -v amdgpu.ids | head -3
  timeout -k 10 100 python tools/rchain_timing.py 2>&1 | grep -v amdgpu.ids | head -3
  timeout -k 10 200 python bench.py --steps 200 --only configD,render --no-cpu-baseline > gpurun_out/r02l_b.log 2>&1
  python tools/show_bench.py gpurun_out/r02l_b.log
fi
