set -e
bash tools/gpu_run_steps.sh \
 "b10_def|200|python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536" \
 "b10_kc512|200|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_kc512.so INF_ALLOW_STALE_LIB=1 python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536" \
 "b10_kc512g2|200|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_kc512g2.so INF_ALLOW_STALE_LIB=1 python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536" \
 "b10_kc512_test|300|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_kc512.so INF_ALLOW_STALE_LIB=1 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k 'bf16_chain3_matches_bf16_oracle'"
