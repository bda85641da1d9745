# Round-4 closing run: the whole GPU suite + smoke, the rocprofv3 kernel trace and the two
# PMC passes of the headline command (tools/profile.sh), then the driver's own bench command.
set -e
export TMPDIR=/tmp
bash tools/gpu_run_steps.sh \
 "final_suite|1100|bash tools/gpu_r4_suite.sh" \
 "final_prof|900|PROF_TAG=bf16_B4096 bash tools/profile.sh r04 --steps 40 --warmup 10 --only none --no-cpu-baseline --extra-batches ''" \
 "final_bench|600|python3 bench.py --gpus 1 --steps 20 --warmup 5"
