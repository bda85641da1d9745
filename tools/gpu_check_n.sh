timeout -k 10 300 python -u -m pytest tests/test_gpu_prefetch.py tests/test_gpu_dp.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r02n_t.log 2>&1; rc=$?; echo rc=$rc; tail -3 gpurun_out/r02n_t.log
if [ $rc -eq 0 ]; then
  timeout -k 10 200 python bench.py --steps 200 --only none --no-cpu-baseline > gpurun_out/r02n_single.log 2>&1; echo single rc=$?
  python tools/show_bench.py gpurun_out/r02n_single.log | head -2
  for pf in 1 0; do
    INF_BENCH_DP=1 INF_PREFETCH=$pf timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 200 --only none --no-cpu-baseline > gpurun_out/r02n_dp$pf.log 2>&1; echo dp pf=$pf rc=$?
    python tools/show_bench.py gpurun_out/r02n_dp$pf.log | head -2
  done
fi
