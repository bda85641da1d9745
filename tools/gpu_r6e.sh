#!/bin/bash
# Round 6: the rest of the GPU suite (-s), the k-tiled projection experiment, and the render
# launch on random vs pixel-coherent hit distributions (kernel trace + PMC traffic + SQ).
set -o pipefail
O=gpurun_out/${1:-r6e}
mkdir -p $O
export TMPDIR=/tmp
T="tests/test_gpu_kernels.py tests/test_gpu_large.py tests/test_gpu_lazy_shadow.py tests/test_gpu_metrics.py tests/test_gpu_prefetch.py tests/test_gpu_raycast.py tests/test_gpu_render.py tests/test_gpu_shard.py tests/test_gpu_trainer_state.py tests/test_gpu_viewdep.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^(D |4096 |1024 )" $O/tests.log | cut -c1-700
[ $rc -eq 0 ] || exit $rc
VAR="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_ptabt.so INF_ALLOW_STALE_LIB=1"
for r in 1 2; do
  timeout -k 10 120 python3 tools/ptab_tiled_exp.py rowmajor >> $O/ptab.log 2>&1 || exit 1
  env $VAR timeout -k 10 120 python3 tools/ptab_tiled_exp.py tiled >> $O/ptab.log 2>&1 || exit 1
done
grep -E "rowmajor|tiled" $O/ptab.log
for kind in random coherent; do
  timeout -k 10 120 python3 tools/render_ids.py $kind 10 > $O/render_$kind.log 2>&1 || exit 1
  cat $O/render_$kind.log | tail -1
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/tr_$kind -o run --output-format csv -- python3 tools/render_ids.py $kind 10 > $O/tr_$kind.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch_$kind -o run --output-format csv -- python3 tools/render_ids.py $kind 3 > $O/fetch_$kind.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write_$kind -o run --output-format csv -- python3 tools/render_ids.py $kind 3 > $O/write_$kind.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq_$kind -o run --output-format csv -- python3 tools/render_ids.py $kind 3 > $O/sq_$kind.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum -d $O/hit_$kind -o run --output-format csv -- python3 tools/render_ids.py $kind 3 > $O/hit_$kind.log 2>&1 || echo "hit pass failed (counter names)"
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for kind in ("random", "coherent"):
    for tag in ("fetch", "write", "sq", "hit"):
        fs = glob.glob(f"{O}/{tag}_{kind}/**/*counter_collection.csv", recursive=True)
        if not fs:
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(fs[0])):
            if "rprojw" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(kind, tag, {c: round(sum(v) / len(v)) for c, v in agg.items()})
    fs = glob.glob(f"{O}/tr_{kind}/**/*kernel_stats.csv", recursive=True)
    for r in csv.DictReader(open(fs[0])):
        if "rprojw" in r["Name"]:
            print(kind, "rprojw avg us", float(r["AverageNs"]) / 1e3, "calls", r["Calls"])
PY
