set -e
bash tools/gpu_run_steps.sh \
 "b3_tests|600|python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k 'lgf or fused_update or golden or dp_step' tests/test_gpu_shard.py tests/test_gpu_dp.py" \
 "b3_dp1|500|INF_BENCH_DP=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 50 --warmup 10 --only strong --no-cpu-baseline --extra-batches ''" \
 "b3_D_slab|300|python bench.py --steps 30 --warmup 10 --only configD --no-cpu-baseline --extra-batches ''" \
 "b3_D_lgf|300|INF_LGF=1 python bench.py --steps 30 --warmup 10 --only configD --no-cpu-baseline --extra-batches ''" \
 "b3_cfg_slab|300|python bench.py --steps 30 --warmup 10 --only configs --no-cpu-baseline --extra-batches ''" \
 "b3_cfg_lgf|300|INF_LGF=1 python bench.py --steps 30 --warmup 10 --only configs --no-cpu-baseline --extra-batches ''"
