set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -v --timeout 200 --timeout-method thread -k "schedules or small_models" > gpurun_out/r02s_t.log 2>&1; rc=$?; echo rc=$rc; tail -12 gpurun_out/r02s_t.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
PROJ=1 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmc_rproj -o run --output-format csv -- python3 tools/rchain_timing.py > gpurun_out/pmc_rproj.log 2>&1; echo pmc rc=$?
