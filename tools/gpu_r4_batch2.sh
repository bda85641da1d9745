set -e
GT0="INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_gt0.so INF_ALLOW_STALE_LIB=1"
bash tools/gpu_run_steps.sh \
 "b2_tests|500|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k 'lgf or fused_update or golden or dp_step' tests/test_gpu_shard.py" \
 "b2_lgb_new|120|LGB_STEP=1 python tools/lgemm_blocks.py" \
 "b2_lgb_gt0|120|LGB_STEP=1 $GT0 python tools/lgemm_blocks.py" \
 "b2_sweep|500|bash tools/gpu_r4_envsweep.sh - INF_NO_LGF=1 '$GT0'" \
 "b2_dp1|400|INF_BENCH_DP=1 python bench.py --steps 50 --warmup 10 --only strong --no-cpu-baseline --extra-batches ''"
