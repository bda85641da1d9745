set -e
bash tools/gpu_run_steps.sh \
 "b5_sweep|600|bash tools/gpu_r4_envsweep.sh - 'INF_FGEMM_NARROW=1 INF_DW_SPLITS=8' 'INF_FGEMM_NARROW=1 INF_DW_SPLITS=16' 'INF_FGEMM_NARROW=1 INF_DW_SPLITS=4'"
