set -e
bash tools/gpu_run_steps.sh \
 "b12_tests|600|python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_shard.py tests/test_gpu_dp.py" \
 "b12_sweep|400|bash tools/gpu_r4_envsweep.sh - INF_LGEMM_KS=1" \
 "b12_lgb|120|python tools/lgemm_blocks.py"
