set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_run_steps.sh \
 "b4_prof_x3|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x3 -o x3 -- python bench.py --mode bf16x3 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''" \
 "b4_b512|200|python bench.py --batch 512 --steps 100 --warmup 20 --only none --no-cpu-baseline --extra-batches ''" \
 "b4_b1024|200|python bench.py --batch 1024 --steps 100 --warmup 20 --only none --no-cpu-baseline --extra-batches ''" \
 "b4_prof_512|300|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_512 -o b512 -- python bench.py --batch 512 --steps 50 --warmup 10 --only none --no-cpu-baseline --extra-batches ''"
