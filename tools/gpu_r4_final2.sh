set -e
bash tools/gpu_r4_final.sh
bash tools/gpu_run_steps.sh "sq_large|700|bash tools/gpu_r4_sq_large.sh"
