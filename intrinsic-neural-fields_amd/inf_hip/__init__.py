"""ctypes binding of libinf_hip.so (C ABI declared in include/inf_hip.h).

The library is built in-tree (``make -C intrinsic-neural-fields_amd/csrc`` or
``__graft_entry__.build()``).  There is no fallback: importing this module without the
library raises, and every entry point raises ``RuntimeError`` with the library's own
message on a non-zero status.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("INF_LIB") or os.path.join(_HERE, "libinf_hip.so")

# ---- constants (inf_hip.h) ---------------------------------------------------------
INF_OK = 0
DTYPE_F32, DTYPE_BF16, DTYPE_I32, DTYPE_I64 = 0, 1, 2, 3
MODE_FP32, MODE_BF16, MODE_BF16X3 = 0, 1, 2
LOSS_L2, LOSS_L1, LOSS_CAUCHY = 0, 1, 2
LOSS_CODES = {"L2": LOSS_L2, "L1": LOSS_L1, "cauchy": LOSS_CAUCHY}
MODE_CODES = {"fp32": MODE_FP32, "bf16": MODE_BF16, "bf16x3": MODE_BF16X3}
STAGE_GATHER, STAGE_FWD_GEMM, STAGE_DW_GEMM, STAGE_UPDATE, STAGE_CHAIN = 0, 1, 2, 3, 4
STEP_ADAM, STEP_ADVANCE, STEP_XSLOT0, STEP_XSLOT1, STEP_PART1, STEP_PART2, STEP_SHARD = 1, 2, 4, 8, 16, 32, 64  # inf_train_step
ENC_NONE, ENC_XYZ, ENC_RFF, ENC_FF, ENC_PROJECTED = 0, 1, 2, 3, 4
ENC_CODES = {"xyz": ENC_XYZ, "rff": ENC_RFF, "ff": ENC_FF}

c_void_p, c_int, c_int32, c_int64, c_float, c_double = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int32,
                                                        ctypes.c_int64, ctypes.c_float, ctypes.c_double)


class MlpDesc(ctypes.Structure):
    _fields_ = [("in_dim", c_int32), ("hidden", c_int32), ("num_layers", c_int32), ("skip", c_int32),
                ("out_dim", c_int32), ("mode", c_int32), ("loss", c_int32)]


class PlanInfo(ctypes.Structure):
    _fields_ = [("num_params", c_int64), ("num_segments", c_int32), ("in_pad", c_int32),
                ("max_batch_pad", c_int32), ("dw_splits", c_int32), ("shadow_bytes", c_int64),
                ("workspace_bytes", c_int64), ("table_ld", c_int64)]


class Batch(ctypes.Structure):
    _fields_ = [("table", c_void_p), ("table_dtype", c_int32), ("num_vertices", c_int64),
                ("vids", c_void_p), ("vid_dtype", c_int32), ("bary", c_void_p), ("rgb", c_void_p),
                ("ray_idx", c_void_p), ("idx_dtype", c_int32), ("idx_offset", c_int64),
                ("offset_from_ctrl", c_int32), ("features", c_void_p), ("ld_features", c_int64),
                ("batch", c_int32), ("loss_count", c_int64), ("loss", c_int32), ("num_rays", c_int64),
                ("encoding", c_int32), ("enc_k", c_int32), ("enc_proj", c_void_p), ("enc_include_input", c_int32),
                ("num_source_rays", c_int64)]


class Ctrl(ctypes.Structure):
    _fields_ = [("step", c_int32), ("batch_index", c_int32), ("prefetch_index", c_int32), ("reserved", c_int32),
                ("lr", c_double), ("loss_sum", c_double), ("sse_sum", c_double), ("epoch_loss", c_double),
                ("epoch_sse", c_double)]


CTRL_BYTES = ctypes.sizeof(Ctrl)
assert CTRL_BYTES == 56

_SIGNATURES = {
    "inf_last_error": (ctypes.c_char_p, []),
    "inf_abi_version": (c_int, []),
    "inf_build_id": (ctypes.c_char_p, []),
    "inf_gather": (c_int, [c_void_p, c_int, c_int64, c_int, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_int,
                           c_int64, c_int, c_int64, c_void_p, c_int, c_int64, c_int, c_void_p, c_int64, c_void_p]),
    "inf_encode": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int64, c_int, c_int64,
                           c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int64, c_int, c_void_p]),
    "inf_encoded_dim": (c_int, [c_int, c_int, c_int]),
    "inf_ssim_workspace_bytes": (c_int64, [c_int, c_int, c_int]),
    "inf_ssim": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.c_double, c_void_p, c_void_p, c_void_p]),
    "inf_masked_sse_workspace_bytes": (c_int64, []),
    "inf_compact_faces": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p]),
    "inf_uv_raster": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, ctypes.c_double, c_void_p, c_void_p,
                              c_void_p, c_void_p]),
    "inf_dense_gemm": (c_int, [c_int, c_int, c_int, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64,
                               c_void_p, c_int, c_float, c_void_p, c_int64, c_void_p]),
    "inf_dense_act_bwd": (c_int, [c_int64, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "inf_colsum": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    "inf_view_angle": (c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "inf_adam_dense": (c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_double, c_double, c_double,
                               c_double, c_void_p]),
    "inf_ff_encode": (c_int, [c_int64, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_void_p]),
    "inf_uv_fill_holes": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "inf_masked_sse": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "inf_plan_create": (c_int, [ctypes.POINTER(MlpDesc), c_int, ctypes.POINTER(c_void_p)]),
    "inf_plan_destroy": (None, [c_void_p]),
    "inf_plan_get_info": (c_int, [c_void_p, ctypes.POINTER(PlanInfo)]),
    "inf_plan_param_layout": (c_int, [c_void_p, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64), c_int]),
    "inf_plan_bind": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "inf_plan_set_adam": (c_int, [c_void_p, c_double, c_double, c_double]),
    "inf_sync_shadow": (c_int, [c_void_p, c_void_p]),
    "inf_forward": (c_int, [c_void_p, ctypes.POINTER(Batch), c_void_p, c_int, c_void_p]),
    "inf_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "inf_train_step": (c_int, [c_void_p, ctypes.POINTER(Batch), c_void_p, c_int, c_void_p]),
    "inf_adam": (c_int, [c_void_p, c_int, c_double, c_void_p]),
    "inf_adam_ex": (c_int, [c_void_p, c_int, c_double, c_int, c_void_p]),
    "inf_render": (c_int, [c_void_p, ctypes.POINTER(Batch), c_void_p, c_void_p, c_void_p, c_void_p]),
    "inf_projected_rows": (c_int64, [c_int64]),
    "inf_project_table": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "inf_ctrl_advance": (c_int, [c_void_p, c_void_p]),
    "inf_plan_last_step_path": (c_int, [c_void_p]),
    "inf_plan_grad_split": (c_int64, [c_void_p]),
    "inf_plan_last_part1_bucketed": (c_int, [c_void_p]),
    "inf_plan_last_step_fused_update": (c_int, [c_void_p]),
    "inf_debug_buffer": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "inf_plan_shard": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "inf_plan_bind_shard": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "inf_plan_can_shard": (c_int, [c_void_p, c_void_p]),
    "inf_adam_shard": (c_int, [c_void_p, c_int, c_void_p]),
    "inf_shard_scatter": (c_int, [c_void_p, c_void_p]),
    "inf_shard_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "inf_shard_unpack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "inf_plan_weight_generation": (c_int64, [c_void_p]),
    "inf_prefetch_batch": (c_int, [c_void_p, ctypes.POINTER(Batch), c_int, c_void_p]),
    "inf_debug_ranges": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "inf_debug_timing": (c_int, [c_void_p, c_void_p, c_int]),
    "inf_debug_block_times": (c_int, [c_void_p, c_void_p]),
    "inf_bvh_create": (c_int, [c_void_p, ctypes.c_int64, c_void_p, ctypes.c_int64, ctypes.POINTER(c_void_p)]),
    "inf_bvh_destroy": (None, [c_void_p]),
    "inf_bvh_info": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32),
                             ctypes.POINTER(ctypes.c_int32)]),
    "inf_raycast": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, ctypes.c_int64, c_void_p,
                            c_void_p, c_void_p, c_void_p]),
    "inf_raycast_rays": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_int64, c_void_p, c_void_p, c_void_p]),
    "inf_compact_hits": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_int64, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p]),
    "inf_run_stage": (c_int, [c_void_p, ctypes.POINTER(Batch), c_int, c_int, ctypes.POINTER(c_double),
                              ctypes.POINTER(c_double), c_void_p]),
}

EXPORTED = tuple(_SIGNATURES)


def _load():
    # PyTorch ships its own HIP runtime (same soname, libamdhip64.so.7).  Load it first so
    # the library binds to the runtime that owns torch's device allocations and streams;
    # loading ours first would put two HIP runtimes in the process.
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP library first (make -C intrinsic-neural-fields_amd/csrc "
            "or python -c 'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _check_provenance(lib)
    return lib


CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
BUILD_ID = None       # inf_build_id() of the loaded library
BUILD_VERIFIED = None  # True: recomputed from the sources beside it; None: sources absent


def source_hash(files, base=CSRC, flags=None) -> str:
    import hashlib
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(base, f), "rb") as fh:
            h.update(fh.read())
    if flags is not None:
        h.update(flags.encode())
    return h.hexdigest()[:16]


def parse_build_id(build_id: str):
    """inf_build_id() = "<hash> <files...> -- <compile flags>" -> (hash, files, flags)."""
    head, _, flags = build_id.partition(" -- ")
    want, *files = head.split()
    return want, files, flags.strip()


def _check_provenance(lib):
    """The library must have been linked from the sources next to it, with the plain
    compile flags (csrc/Makefile hashes the source bytes and the flags into inf_build_id): a
    stale or foreign libinf_hip.so, or a variant build (-D... diagnostics such as
    C3_STREAM_ONLY, which compute garbage), raises here instead of running other kernels
    than the tree's.  INF_ALLOW_STALE_LIB=1 skips the refusal (tuning experiments)."""
    global BUILD_ID, BUILD_VERIFIED
    BUILD_ID = lib.inf_build_id().decode()
    want, files, flags = parse_build_id(BUILD_ID)
    if not files or not all(os.path.exists(os.path.join(CSRC, f)) for f in files):
        BUILD_VERIFIED = None
        return
    got = source_hash(files, flags=flags)
    variant = any(t.startswith("-D") for t in flags.split())
    BUILD_VERIFIED = got == want and not variant
    if not BUILD_VERIFIED and os.environ.get("INF_ALLOW_STALE_LIB", "0") == "0":
        why = f"with variant flags ({flags})" if got == want else f"from other sources (build id {want}, sources hash {got})"
        raise ImportError(f"{LIB_PATH} was built {why}: rebuild it (make -C intrinsic-neural-fields_amd/csrc)")


lib = _load()


def check(rc: int, what: str = "") -> None:
    if rc != INF_OK:
        msg = lib.inf_last_error().decode(errors="replace")
        raise RuntimeError(f"inf_hip {what} failed ({rc}): {msg}")
