set -e
bash tools/gpu_run_steps.sh \
 "b7_x3_def|200|python bench.py --mode bf16x3 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''" \
 "b7_x3_s4|200|INF_DW_SPLITS=4 python bench.py --mode bf16x3 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''" \
 "b7_x3_bm32|200|INF_SPLIT_LGEMM_BM=32 python bench.py --mode bf16x3 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''"
