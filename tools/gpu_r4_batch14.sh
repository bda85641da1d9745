set -e
bash tools/gpu_run_steps.sh \
 "b14_tests|600|python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_bf16x3.py tests/test_gpu_chainf.py" \
 "b14_x3|200|python bench.py --mode bf16x3 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''" \
 "b14_x3_ks1|200|INF_LGEMM_KS=1 python bench.py --mode bf16x3 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''"
