set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_run_steps.sh \
 "b8_large_layered|300|INF_NO_CHAIN=1 python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536" \
 "b8_prof_layered|300|INF_NO_CHAIN=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lay -o lay -- python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536" \
 "b8_prof_wide|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wide -o wide -- python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536"
