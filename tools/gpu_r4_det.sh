set -o pipefail
T="timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for i in 1 2; do $T tests/test_gpu_dp.py -k "two_ranks_one_gpu_gloo and fp32" -s > gpurun_out/r4_det_cur$i.log 2>&1; done
(cd tmp_r3 && $T tests/test_gpu_dp.py -k "two_ranks_one_gpu_gloo and fp32" -s > ../gpurun_out/r4_det_r3.log 2>&1)
$T tests/test_gpu_dp.py tests/test_gpu_shard.py -k "shard" -s > gpurun_out/r4_shard3.log 2>&1
