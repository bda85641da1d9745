set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -v -s --timeout 250 --timeout-method thread -k g12 > gpurun_out/g12.log 2>&1; rc=$?; echo rc=$rc; grep -n "{'fp32'\|passed\|failed\|Error" gpurun_out/g12.log | head; exit $rc
