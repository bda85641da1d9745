set -e
bash tools/gpu_run_steps.sh \
 "lgfdbg|200|python tools/lgf_debug.py" \
 "r4_lgf_tests|400|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k 'lgf or fused_update or golden' tests/test_gpu_bf16x3.py tests/test_gpu_chainf.py" \
 "r4_lgf_sweep|400|bash tools/gpu_r4_envsweep.sh - INF_NO_LGF=1" \
 "r4_x3_bench|200|python bench.py --mode bf16x3 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''" \
 "r4_strong|300|python bench.py --steps 50 --warmup 10 --only strong --no-cpu-baseline --extra-batches ''"
bash tools/gpu_run_steps.sh \
 "r4_large_def|300|python bench.py --steps 20 --warmup 5 --only large --no-cpu-baseline --extra-batches 65536" \
 "r4_large_nr2|300|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_nr2.so INF_ALLOW_STALE_LIB=1 python bench.py --steps 20 --warmup 5 --only large --no-cpu-baseline --extra-batches 65536" \
 "r4_large_nr2_test|300|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_nr2.so INF_ALLOW_STALE_LIB=1 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k 'bf16_chain3_matches_bf16_oracle'"
