set -e
bash tools/gpu_run_steps.sh \
 "b15_big_test|400|python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k 'bf16_chain3_matches_bf16_oracle'" \
 "b15_big_bench|300|INF_BIG_LAYERED=1 python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536"
