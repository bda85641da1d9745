set -e
bash tools/gpu_run_steps.sh \
 "b11_D_def|300|python bench.py --steps 30 --warmup 10 --only configD --no-cpu-baseline --extra-batches ''" \
 "b11_D_kc2048|300|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_kc2048.so INF_ALLOW_STALE_LIB=1 python bench.py --steps 30 --warmup 10 --only configD --no-cpu-baseline --extra-batches ''" \
 "b11_D_def2|300|python bench.py --steps 30 --warmup 10 --only configD --no-cpu-baseline --extra-batches ''" \
 "b11_D_kc2048b|300|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_kc2048.so INF_ALLOW_STALE_LIB=1 python bench.py --steps 30 --warmup 10 --only configD --no-cpu-baseline --extra-batches ''"
bash tools/gpu_run_steps.sh \
 "b11_lg_sweep|600|bash tools/gpu_r4_envsweep.sh - 'INF_LGEMM_BM=128 INF_DW_SPLITS=4' 'INF_LGEMM_BM=128' 'INF_DW_SPLITS=4'"
