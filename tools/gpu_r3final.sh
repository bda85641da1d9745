#!/bin/bash
# Round 3 final checkpoint: whole GPU suite, smoke, the full bench line, the step's kernel
# trace and the 65,536-ray kernel stats (logs under gpurun_out/)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/fin_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/fin_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/fin_smoke.log 2>&1 || exit 1
timeout -k 10 700 python bench.py > $O/fin_bench.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fin_step -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --only none --no-cpu-baseline --extra-batches "" > $O/fin_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fin_65k -o run --output-format csv -- python3 bench.py --batch 65536 --steps 16 --warmup 4 --extra-batches "" --only none --no-cpu-baseline > $O/fin_65k.log 2>&1
