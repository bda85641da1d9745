set -o pipefail
timeout -k 10 200 python bench.py --steps 200 --only none --no-cpu-baseline > gpurun_out/fu_a.log 2>&1 && python tools/show_bench.py gpurun_out/fu_a.log | head -2 && \
INF_FUSED_UPDATE=1 timeout -k 10 200 python bench.py --steps 200 --only none --no-cpu-baseline > gpurun_out/fu_b.log 2>&1 && python tools/show_bench.py gpurun_out/fu_b.log | head -2
