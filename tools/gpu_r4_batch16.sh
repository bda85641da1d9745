set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_run_steps.sh \
 "b16_prof_big|300|INF_BIG_LAYERED=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_big -o big -- python bench.py --steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536"
