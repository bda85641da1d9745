set -e
bash tools/gpu_run_steps.sh \
 "b13_sweep|600|bash tools/gpu_r4_envsweep.sh - 'INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_r4d4.so INF_ALLOW_STALE_LIB=1' 'INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_r2d2.so INF_ALLOW_STALE_LIB=1' INF_LGEMM_KS=1" \
 "b13_lgb|120|python tools/lgemm_blocks.py" \
 "b13_lgb_r2d2|120|INF_LIB=intrinsic-neural-fields_amd/inf_hip/libinf_hip_r2d2.so INF_ALLOW_STALE_LIB=1 python tools/lgemm_blocks.py"
