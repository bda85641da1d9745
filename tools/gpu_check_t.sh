set -o pipefail
timeout -k 10 300 python bench.py --steps 20 --only render --no-cpu-baseline > gpurun_out/r02t_b.log 2>&1; rc=$?; echo rc=$rc; tail -3 gpurun_out/r02t_b.log | cut -c1-300; exit $rc
