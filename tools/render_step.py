"""Runs only bench.py's render-slice line (for rocprofv3 kernel traces)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

args = bench.parse()
print(json.dumps(bench.render_bench(args, torch.device("cuda", 0))))
