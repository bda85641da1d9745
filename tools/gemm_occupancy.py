"""Layered GEMMs of the fp32 / bf16x3 parity modes at config B (4096 rays): does placing
ONE workgroup per CU (reserving more LDS, INF_GEMM_LDS) change a hidden layer's forward
GEMM, the skip layer's and the dW GEMM?  Interleaved rounds in one process."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from inf_hip import STAGE_DW_GEMM, STAGE_FWD_GEMM  # noqa: E402

args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
sys.argv = [sys.argv[0]]
args = bench.parse()
res = {}
for mode in ("fp32", "bf16x3"):
    args.mode = mode
    tr = bench.Trainer(args, torch.device("cuda", 0), 4096, 0, 1, nb=8)
    tr.step_eager()
    torch.cuda.synchronize()
    for r in range(3):
        for lds in ("0", "90000", "150000"):
            os.environ["INF_GEMM_LDS"] = lds
            for name, st, layer in (("fwd_l1", STAGE_FWD_GEMM, 1), ("fwd_l4_skip", STAGE_FWD_GEMM, 4),
                                    ("dw", STAGE_DW_GEMM, 0)):
                ms, fl, _ = bench.time_stage(tr.plan, st, reps=10, layer=layer)
                res.setdefault((mode, lds, name), []).append(ms)
    del tr
    torch.cuda.empty_cache()
for (mode, lds, name), v in sorted(res.items()):
    print(f"{mode:7s} lds={lds:>6s} {name:12s} median {sorted(v)[len(v) // 2] * 1e3:8.2f} us  all {[round(x * 1e3, 2) for x in v]}",
          flush=True)
