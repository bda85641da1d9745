set -e
bash tools/gpu_run_steps.sh \
 "b9_tests|500|python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_shard.py -k 'adam or fused or shard or dp_step or golden'" \
 "b9_sweep|300|bash tools/gpu_r4_envsweep.sh -"
