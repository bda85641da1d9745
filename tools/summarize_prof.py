"""Summarise rocprofv3 outputs of tools/profile.sh into one JSON document.

* per kernel: calls, average / total duration (kernel-trace stats);
* per kernel: average FETCH_SIZE and WRITE_SIZE per dispatch, in bytes.  rocprofv3 reports
  both in KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide coalesced read
  (MI355X_MICROARCH.md, HBM section), so the HBM read estimate is 2 x FETCH_SIZE.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    if "chain3_kernel" in name and ("Lb0ELb1E" in name or "false, true>" in name or "false, true, 1," in name):
        return "chain3_kernel<chunked>"
    if name.startswith("Cijk_"):  # hipBLASLt's kernels (the projection GEMM)
        return "hipblaslt_gemm"
    for key in ("zg_kernel", "gather_rows_kernel", "proj_gemm_kernel", "fgemm_kernel", "chainf_kernel", "rprojw_kernel", "rproj_kernel", "rchain_kernel", "chain3_kernel", "lgemm_kernel", "prefetch_advance_kernel", "chain_kernel", "gemm_nt_kernel", "gather_kernel", "update_kernel", "head_fwd_kernel",
                "head_bwd_kernel", "pack_kernel", "ctrl_advance_kernel"):
        if key in name:
            tail = ""
            if key == "gemm_nt_kernel":
                tail = "<128x128>" if ("128ELi128" in name or "128, 128" in name) else "<64x64>"
                tail = ("<bf16," if ("DF16b" in name or "bf16" in name.lower()) else "<f32,") + tail[1:] if tail else tail
            if key == "chain_kernel":
                for t in ("256, 64, 64", "256, 128, 32", "128, 64, 64", "128, 128, 32", "Li256ELi64", "Li256ELi128",
                          "Li128ELi64", "Li128ELi128"):
                    if t in name:
                        tail = "<" + t.replace("Li", "").replace("E", ",") + ">"
                        break
            return key + tail
    return name[:60]


def stats(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True) or \
        glob.glob(os.path.join(d, "*kernel_stats.csv"))
    out = {}
    if not f:
        return out
    for r in csv.DictReader(open(f[0])):
        k = short(r["Name"])
        e = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
        e["calls"] += int(r["Calls"])
        e["total_ns"] += float(r["TotalDurationNs"])
    for e in out.values():
        e["avg_us"] = e["total_ns"] / max(e["calls"], 1) / 1e3
    return out


def counters(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    if not files:
        return {}
    for r in csv.DictReader(open(files[0])):
        if r.get("Counter_Name") != counter:
            continue
        acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) * 1024.0 for k, v in acc.items()}  # KiB -> bytes per dispatch


# bench.py stage -> kernel, for the per-launch traffic table bench.py reads
STAGE_KERNEL = {"chain3": "chain3_kernel", "dw_gemm": "lgemm_kernel", "update": "update_kernel",
                "rchain": "rchain_kernel", "chain3_chunked": "chain3_kernel<chunked>",
                "rproj": "rproj_kernel", "rprojw": "rprojw_kernel", "project_gemm": "proj_gemm_kernel"}


def main(root, tag=None):
    tdir = os.path.join(root, "trace")
    res = {"kernels": stats(tdir if os.path.isdir(tdir) else root)}
    fetch = counters(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(root, "write"), "WRITE_SIZE")
    for k, e in res["kernels"].items():
        if k in fetch:
            e["fetch_size_bytes"] = fetch[k]
            e["hbm_read_est_bytes"] = 2.0 * fetch[k]
        if k in write:
            e["write_size_bytes"] = write[k]
        if k in fetch and k in write:
            e["traffic_bytes"] = 2.0 * fetch[k] + write[k]
    if tag:  # e.g. bf16_B4096: {"chain3_bf16_B4096": bytes per launch, ...}
        res["bench_traffic"] = {f"{st}_{tag}": res["kernels"][k]["traffic_bytes"]
                                for st, k in STAGE_KERNEL.items()
                                if "traffic_bytes" in res["kernels"].get(k, {})}
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
