timeout -k 10 300 python -u -m pytest tests/test_gpu_prefetch.py tests/test_gpu_kernels.py tests/test_gpu_dp.py tests/test_gpu_host.py tests/test_gpu_trainer_state.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r02m_t.log 2>&1; rc=$?; echo rc=$rc; tail -15 gpurun_out/r02m_t.log
if [ $rc -eq 0 ]; then
  for pf in 1 0; do
    INF_PREFETCH=$pf timeout -k 10 200 python bench.py --steps 200 --only configD --no-cpu-baseline > gpurun_out/r02m_b$pf.log 2>&1; echo pf=$pf rc=$?
    python tools/show_bench.py gpurun_out/r02m_b$pf.log | head -3
  done
fi
