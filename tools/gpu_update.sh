set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_trainer_state.py tests/test_gpu_prefetch.py tests/test_gpu_host.py -x -q --timeout 200 --timeout-method thread > gpurun_out/upd_t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/upd_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --only none --no-cpu-baseline > gpurun_out/upd_a.log 2>&1 && python tools/show_bench.py gpurun_out/upd_a.log | head -2 && \
INF_UPDATE_PAIRS=0 timeout -k 10 200 python bench.py --steps 200 --only none --no-cpu-baseline > gpurun_out/upd_b.log 2>&1 && python tools/show_bench.py gpurun_out/upd_b.log | head -2
