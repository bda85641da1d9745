set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/full_t.log 2>&1; rc=$?; echo tests rc=$rc; tail -4 gpurun_out/full_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/full_b.log 2>&1; rc=$?; echo bench rc=$rc; tail -c 600 gpurun_out/full_b.log; exit $rc
