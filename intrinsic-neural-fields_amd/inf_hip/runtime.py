"""Torch-facing runtime over the C ABI: device buffers, packed tables, plans.

PyTorch is plumbing here: it allocates device memory and provides the current HIP
stream; all arithmetic of the hot path runs in libinf_hip.so.  Every function refuses
CPU tensors (there is no CPU fallback of the product path).
"""
from __future__ import annotations

import ctypes

import torch

from . import (CTRL_BYTES, Ctrl, ENC_CODES, ENC_NONE, ENC_PROJECTED, DTYPE_BF16, DTYPE_F32, DTYPE_I32, DTYPE_I64, INF_OK, LOSS_CODES, MODE_BF16,
               MODE_CODES, Batch, STEP_ADAM, STEP_ADVANCE, STEP_PART1, STEP_PART2, STEP_SHARD, STEP_XSLOT0, STEP_XSLOT1, MlpDesc, PlanInfo,
               c_int64, c_void_p,
               check, lib)

_TORCH_DTYPE = {DTYPE_F32: torch.float32, DTYPE_BF16: torch.bfloat16}
_CODE = {torch.float32: DTYPE_F32, torch.bfloat16: DTYPE_BF16, torch.int32: DTYPE_I32, torch.int64: DTYPE_I64}


def require_hip(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("intrinsic-neural-fields_amd runs its hot path on MI355X (HIP) devices only; "
                               f"got a tensor on {t.device}. There is no CPU fallback.")


def stream_handle() -> c_void_p:
    return c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> c_void_p | None:
    return None if t is None else c_void_p(t.data_ptr())


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _CODE[t.dtype]
    except KeyError:
        raise RuntimeError(f"unsupported dtype {t.dtype}") from None


# ---------------------------------------------------------------------------------
# Gather (mesh.py:313-324)
# ---------------------------------------------------------------------------------

def gather(E: torch.Tensor, vids: torch.Tensor, bary: torch.Tensor, ray_idx: torch.Tensor | None = None,
           offset: int = 0, batch: int | None = None, out_dtype: torch.dtype = torch.float32,
           k: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """F[b] = sum_i bary[r, i] * E[vids[r, i]] with r = ray_idx[offset + b] (or offset + b).
    E: [V, ld] fp32/bf16 (first k columns used); vids [N, 3] int32/int64; bary [N, 3] fp32."""
    require_hip(E, vids, bary, ray_idx)
    if E.dim() != 2 or E.stride(1) != 1:
        raise ValueError("E must be a row-major [V, k] matrix")
    if vids.dim() != 2 or vids.shape[1] != 3 or not vids.is_contiguous():
        raise ValueError("vertex ids must be a contiguous [N, 3] tensor")
    if bary.shape != vids.shape or bary.dtype != torch.float32 or not bary.is_contiguous():
        raise ValueError("barycentric coordinates must be a contiguous fp32 [N, 3] tensor")
    k = E.shape[1] if k is None else k
    n_rows = ray_idx.shape[0] if ray_idx is not None else vids.shape[0]
    batch = n_rows - offset if batch is None else batch
    if batch < 0 or offset + batch > n_rows:
        raise ValueError("batch out of range")
    if out is None:
        out = torch.empty((batch, k), dtype=out_dtype, device=E.device)
    if batch == 0:
        return out
    check(lib.inf_gather(ptr(E), dtype_code(E), E.shape[0], k, E.stride(0), ptr(vids), dtype_code(vids), ptr(bary),
                         ptr(ray_idx), dtype_code(ray_idx) if ray_idx is not None else DTYPE_I64, offset, batch,
                         vids.shape[0], ptr(out), dtype_code(out), out.stride(0), out.shape[0], None, 0, stream_handle()), "gather")
    return out


class Encoding:
    """An input front-end (model.py:33-40): 'xyz', 'rff' (proj = the RFF matrix B [3, k],
    layers.py:28-31) or 'ff' (proj = the frequency bands [k], layers.py:11-18)."""

    def __init__(self, kind: str, k: int = 0, proj: torch.Tensor | None = None, include_input: bool = True):
        if kind not in ENC_CODES:
            raise ValueError(f"unknown encoding {kind!r}")
        self.kind, self.code = kind, ENC_CODES[kind]
        self.k = int(k) if kind != "xyz" else 0
        self.include_input = bool(include_input) if kind != "xyz" else False
        if kind != "xyz":
            require_hip(proj)
            want = (3, self.k) if kind == "rff" else (self.k,)
            if proj is None or tuple(proj.shape) != want or proj.dtype != torch.float32 or not proj.is_contiguous():
                raise ValueError(f"{kind} encoding needs a contiguous fp32 {list(want)} tensor")
        self.proj = proj
        self.dim = int(lib.inf_encoded_dim(self.code, self.k, int(self.include_input)))
        if self.dim <= 0:
            raise ValueError("bad encoding parameters")


def encode(enc: Encoding, points: torch.Tensor, vids: torch.Tensor | None = None, bary: torch.Tensor | None = None,
           ray_idx: torch.Tensor | None = None, offset: int = 0, batch: int | None = None) -> torch.Tensor:
    """Encoded features [B, enc.dim] fp32.  With vids/bary: points is the V x 3 vertex
    table and rays are interpolated first (ray_dataloader.py:134-136); without: points
    are the rays' positions (layers.py:21-39 applied to batch["xyz"])."""
    require_hip(points, vids, bary, ray_idx)
    if points.dim() != 2 or points.shape[1] != 3 or points.dtype != torch.float32 or not points.is_contiguous():
        raise ValueError("positions must be a contiguous fp32 [N, 3] tensor")
    if vids is not None:
        if vids.dim() != 2 or vids.shape[1] != 3 or not vids.is_contiguous():
            raise ValueError("vertex ids must be a contiguous [N, 3] tensor")
        if bary is None or bary.shape != vids.shape or bary.dtype != torch.float32 or not bary.is_contiguous():
            raise ValueError("barycentric coordinates must be a contiguous fp32 [N, 3] tensor")
        n_rows = ray_idx.shape[0] if ray_idx is not None else vids.shape[0]
    else:
        n_rows = ray_idx.shape[0] if ray_idx is not None else points.shape[0]
    batch = n_rows - offset if batch is None else batch
    if batch < 0 or offset + batch > n_rows:
        raise ValueError("batch out of range")
    out = torch.empty((batch, enc.dim), dtype=torch.float32, device=points.device)
    if batch == 0:
        return out
    check(lib.inf_encode(ptr(points), points.shape[0], ptr(vids), dtype_code(vids) if vids is not None else DTYPE_I32,
                         ptr(bary), ptr(ray_idx), dtype_code(ray_idx) if ray_idx is not None else DTYPE_I64, offset,
                         batch, vids.shape[0] if vids is not None else points.shape[0], enc.code, enc.k, ptr(enc.proj), int(enc.include_input), ptr(out), DTYPE_F32,
                         out.stride(0), out.shape[0], stream_handle()), "encode")
    return out


def ssim(fake: torch.Tensor, real: torch.Tensor, data_range: float = 2.0) -> float:
    """Mean SSIM over channels of two fp32 [H, W, C] device images (csrc/metrics.hip)."""
    require_hip(fake, real)
    if fake.shape != real.shape or fake.dim() != 3:
        raise ValueError("images must be [H, W, C] of the same shape")
    a = fake.to(torch.float32).contiguous()
    b = real.to(torch.float32).contiguous()
    H, W, C = a.shape
    ws = int(lib.inf_ssim_workspace_bytes(H, W, C))
    if ws < 0:
        raise ValueError("ssim needs images of at least 7 x 7 with 1..4 channels")
    work = torch.empty(max(ws, 8), dtype=torch.uint8, device=a.device)
    out = torch.empty(C, dtype=torch.float64, device=a.device)
    check(lib.inf_ssim(ptr(a), ptr(b), H, W, C, float(data_range), ptr(work), ptr(out), stream_handle()), "ssim")
    return float(out.mean().item())


def masked_sse(fake: torch.Tensor, real: torch.Tensor, mask: torch.Tensor | None = None):
    """(sum of squared differences over the masked pixels, pixel count) of [.., C] images."""
    require_hip(fake, real, mask)
    a = fake.to(torch.float32).contiguous()
    b = real.to(torch.float32).contiguous()
    C = a.shape[-1]
    n = a.numel() // C
    m = None
    if mask is not None:
        if mask.numel() != n:
            raise ValueError("mask must have one entry per pixel")
        m = mask.reshape(-1).to(torch.uint8).contiguous()
    work = torch.empty(int(lib.inf_masked_sse_workspace_bytes()), dtype=torch.uint8, device=a.device)
    out = torch.empty(2, dtype=torch.float64, device=a.device)
    check(lib.inf_masked_sse(ptr(a), ptr(b), ptr(m), n, C, ptr(work), ptr(out), stream_handle()), "masked_sse")
    s, c = out.tolist()
    return s, int(c)


def uv_raster(uv_px: torch.Tensor, faces: torch.Tensor, H: int, W: int, min_area: float = 1e-4):
    """Texel -> UV triangle + barycentrics (csrc/bake.hip): (texel_face [H*W] int32, -1 =
    none; texel_bary [H*W, 3] f32).  uv_px [Nv, 2] f64 texel coordinates, faces [F, 3]."""
    require_hip(uv_px, faces)
    uv = uv_px.to(torch.float64).contiguous()
    f = faces.to(torch.int32).contiguous()
    dev = uv.device
    keys = torch.empty(H * W, dtype=torch.int64, device=dev)
    tf = torch.empty(H * W, dtype=torch.int32, device=dev)
    tb = torch.empty((H * W, 3), dtype=torch.float32, device=dev)
    check(lib.inf_uv_raster(ptr(uv), uv.shape[0], ptr(f), f.shape[0], int(H), int(W), float(min_area), ptr(keys),
                            ptr(tf), ptr(tb), stream_handle()), "uv_raster")
    return tf, tb


def compact_faces(faces: torch.Tensor, face: torch.Tensor, bary: torch.Tensor):
    """Hit lists (vids [M, 3] int64 from `faces`, bary [M, 3], index [M], face [M]) of the
    entries with face >= 0, in order."""
    require_hip(faces, face, bary)
    fa = faces.to(torch.int32).contiguous()
    n = face.shape[0]
    dev = face.device
    scratch = torch.empty(max((n + 255) // 256, 1), dtype=torch.int32, device=dev)
    count = torch.zeros(1, dtype=torch.int64, device=dev)
    vids = torch.empty((n, 3), dtype=torch.int64, device=dev)
    ob = torch.empty((n, 3), dtype=torch.float32, device=dev)
    idx = torch.empty(n, dtype=torch.int64, device=dev)
    fc = torch.empty(n, dtype=torch.int64, device=dev)
    check(lib.inf_compact_faces(ptr(fa), ptr(face), ptr(bary.contiguous()), n, ptr(scratch), ptr(count), ptr(vids),
                                ptr(ob), ptr(idx), ptr(fc), stream_handle()), "compact_faces")
    m = int(count.item())
    return vids[:m], ob[:m], idx[:m], fc[:m]


def uv_fill_holes(img: torch.Tensor):
    """uv_fill_holes + 8-bit quantisation of an [H, W, 3] texture: (uint8, filled f32)."""
    require_hip(img)
    a = img.to(torch.float32).contiguous()
    H, W, C = a.shape
    if C != 3:
        raise ValueError("texture must be [H, W, 3]")
    u8 = torch.empty((H, W, 3), dtype=torch.uint8, device=a.device)
    f = torch.empty((H, W, 3), dtype=torch.float32, device=a.device)
    check(lib.inf_uv_fill_holes(ptr(a), H, W, ptr(u8), ptr(f), stream_handle()), "uv_fill_holes")
    return u8, f


def pack_table(E: torch.Tensor, k_pad: int, dtype: torch.dtype) -> torch.Tensor:
    """Device copy of the V x k table with zero columns up to k_pad (the GEMM tile),
    in the GEMM dtype (mesh.py:53-108 produces E; this is the upload of it)."""
    V, k = E.shape
    T = torch.zeros((V, k_pad), dtype=dtype, device=E.device)
    T[:, :k] = E
    return T


# ---------------------------------------------------------------------------------
# Plan
# ---------------------------------------------------------------------------------

class Plan:
    """One TextureField architecture bound to a flat parameter arena on one device."""

    def __init__(self, in_dim: int, hidden: int, num_layers: int, skip: int, mode: str, loss: str,
                 max_batch: int, params: torch.Tensor, grads: torch.Tensor | None = None,
                 exp_avg: torch.Tensor | None = None, exp_avg_sq: torch.Tensor | None = None):
        require_hip(params)
        self.device = params.device
        self.mode = mode
        self.mode_code = MODE_CODES[mode]
        self.loss = loss
        self.desc = MlpDesc(in_dim, hidden, num_layers, skip, 3, self.mode_code, LOSS_CODES[loss])
        handle = c_void_p()
        check(lib.inf_plan_create(ctypes.byref(self.desc), int(max_batch), ctypes.byref(handle)), "plan_create")
        self.handle = handle
        self.info = PlanInfo()
        check(lib.inf_plan_get_info(self.handle, ctypes.byref(self.info)), "plan_get_info")
        n = self.info.num_segments
        offs, nums = (c_int64 * n)(), (c_int64 * n)()
        check(lib.inf_plan_param_layout(self.handle, offs, nums, n), "param_layout")
        self.offsets = list(offs)
        self.numels = list(nums)
        self.max_batch = int(max_batch)
        self.in_pad = self.info.in_pad
        self.gemm_dtype = torch.bfloat16 if self.mode_code == MODE_BF16 else torch.float32
        if params.numel() != self.info.num_params:
            raise ValueError(f"parameter arena has {params.numel()} floats, plan needs {self.info.num_params}")
        with torch.cuda.device(self.device):
            self.shadow = torch.empty(max(self.info.shadow_bytes, 256), dtype=torch.uint8, device=self.device)
            self.workspace = torch.empty(max(self.info.workspace_bytes, 256), dtype=torch.uint8, device=self.device)
            self.ctrl = torch.zeros(CTRL_BYTES, dtype=torch.uint8, device=self.device)
        for t in (self.shadow, self.workspace):
            assert t.data_ptr() % 256 == 0
        self.params = params
        self.encoding: Encoding | None = None  # the model's front-end (set by TextureField)
        self.bind(grads, exp_avg, exp_avg_sq)

    def bind(self, grads=None, exp_avg=None, exp_avg_sq=None):
        for t in (grads, exp_avg, exp_avg_sq):
            if t is not None and (t.numel() != self.info.num_params or t.device != self.device):
                raise ValueError("optimizer arenas must match the parameter arena")
        self.grads, self.exp_avg, self.exp_avg_sq = grads, exp_avg, exp_avg_sq
        # inf_plan_bind resets the C side's shard layout and buffers: forget ours with it, so
        # a sharded step after a rebind re-shards (dp._ensure_shard) instead of failing
        self.shard_world = self.shard_rank = 0
        self.grad_staging = self.grad_chunk = self.weight_staging = None
        with torch.cuda.device(self.device):
            check(lib.inf_plan_bind(self.handle, ptr(self.params), ptr(grads), ptr(exp_avg), ptr(exp_avg_sq),
                                    ptr(self.shadow), ptr(self.workspace), ptr(self.ctrl)), "plan_bind")
            self.sync_shadow()

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and lib is not None:
            try:
                lib.inf_plan_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None

    # ---- ctrl block -------------------------------------------------------------
    @property
    def ctrl_i32(self):
        return self.ctrl.view(torch.int32)

    @property
    def ctrl_f32(self):
        return self.ctrl.view(torch.float32)

    @property
    def ctrl_f64(self):
        return self.ctrl.view(torch.float64)

    def set_lr(self, lr: float):
        self.ctrl_f64[Ctrl.lr.offset // 8].fill_(float(lr))

    def set_step(self, step: int):
        self.ctrl_i32[Ctrl.step.offset // 4].fill_(int(step))

    def set_batch_index(self, i: int):
        self.ctrl_i32[Ctrl.batch_index.offset // 4].fill_(int(i))

    def set_prefetch_index(self, i: int):
        self.ctrl_i32[Ctrl.prefetch_index.offset // 4].fill_(int(i))

    def reset_epoch_sums(self):
        self.ctrl_f64[Ctrl.epoch_loss.offset // 8:Ctrl.epoch_sse.offset // 8 + 1].zero_()

    def read_ctrl(self) -> dict:
        raw = bytes(self.ctrl.cpu().numpy().tobytes())
        c = Ctrl.from_buffer_copy(raw)
        return {f: getattr(c, f) for f, _ in Ctrl._fields_}

    # ---- calls ------------------------------------------------------------------
    def sync_shadow(self):
        check(lib.inf_sync_shadow(self.handle, stream_handle()), "sync_shadow")

    def set_adam(self, beta1: float, beta2: float, eps: float):
        check(lib.inf_plan_set_adam(self.handle, beta1, beta2, eps), "set_adam")

    def make_batch(self, *, features=None, rgb=None, source=None, ray_idx=None, offset=0, batch=None, loss_count=0,
                   offset_from_ctrl=False, loss=None, xyz=None, projected=None) -> Batch:
        """Rays of a RaySource (gathered, or interpolated + encoded under self.encoding),
        given positions `xyz` [B, 3] (encoded), or given features [B, in_dim].
        projected: the source table's project_table() output (forward-only batches)."""
        b = Batch()
        b.encoding = ENC_NONE
        enc = self.encoding
        if enc is not None and features is None:
            if enc.dim != self.desc.in_dim:
                raise ValueError(f"encoding width {enc.dim} does not match the model's in_dim {self.desc.in_dim}")
            b.encoding, b.enc_k, b.enc_include_input = enc.code, enc.k, int(enc.include_input)
            b.enc_proj = enc.proj.data_ptr() if enc.proj is not None else None
        if xyz is not None:
            if enc is None:
                raise ValueError("positions given to a model without an xyz/ff/rff front-end")
            require_hip(xyz)
            if xyz.dim() != 2 or xyz.shape[1] != 3 or xyz.dtype != torch.float32 or not xyz.is_contiguous():
                raise ValueError("positions must be a contiguous fp32 [B, 3] tensor")
            b.table = xyz.data_ptr()
            b.table_dtype = DTYPE_F32
            b.num_vertices = xyz.shape[0]
            b.vids = None
            b.batch = xyz.shape[0] if batch is None else int(batch)
            b.num_rays = xyz.shape[0]
            b.num_source_rays = xyz.shape[0]
        elif features is not None:
            require_hip(features)
            if features.dtype != torch.float32 or features.dim() != 2 or features.stride(1) != 1:
                raise ValueError("features must be a row-major fp32 [B, k] tensor")
            if features.shape[1] != self.desc.in_dim:
                raise ValueError(f"features have {features.shape[1]} columns, model expects {self.desc.in_dim}")
            b.features = features.data_ptr()
            b.ld_features = features.stride(0)
            b.batch = features.shape[0] if batch is None else batch
            if rgb is not None:
                require_hip(rgb)
                if rgb.dtype != torch.float32 or not rgb.is_contiguous() or rgb.shape != (b.batch, 3):
                    raise ValueError("targets must be a contiguous fp32 [B, 3] tensor")
                b.rgb = rgb.data_ptr()
        else:
            src = source
            T = src.table_for(self)
            b.table = T.data_ptr()
            b.table_dtype = dtype_code(T)
            b.num_vertices = T.shape[0]
            b.vids = src.vids32.data_ptr()
            b.vid_dtype = DTYPE_I32
            b.bary = src.bary.data_ptr()
            b.rgb = src.rgbs.data_ptr() if src.rgbs is not None else None
            # rows the permutation may name: an entry outside them reads as a zero row
            b.num_source_rays = src.vids32.shape[0]
            if ray_idx is not None:
                b.ray_idx = ray_idx.data_ptr()
                b.idx_dtype = dtype_code(ray_idx)
                b.num_rays = ray_idx.numel()  # the kernels never read past the permutation
            else:
                b.num_rays = src.vids32.shape[0]
            if projected is not None:
                if projected.dtype != torch.bfloat16 or projected.shape[1] != 2 * self.desc.hidden or \
                        projected.shape[0] < T.shape[0]:
                    raise ValueError("projected table does not match this plan / source")
                b.table = projected.data_ptr()
                b.encoding = ENC_PROJECTED
            b.idx_offset = int(offset)
            b.offset_from_ctrl = 1 if offset_from_ctrl else 0
            b.batch = int(batch)
        b.loss_count = int(loss_count)
        b.loss = -1 if loss is None else LOSS_CODES[loss]
        # the struct holds raw device pointers: keep their tensors alive with it (a
        # temporary ray_idx would otherwise return to the caching allocator)
        b._refs = (features, rgb, source, ray_idx, xyz, projected, enc)
        if b.batch < 1 or (b.batch > self.max_batch and b.encoding != ENC_PROJECTED):
            raise ValueError(f"batch of {b.batch} rays outside this plan's range 1..{self.max_batch}")
        return b

    def forward(self, b: Batch, pred: torch.Tensor, save: bool):
        check(lib.inf_forward(self.handle, ctypes.byref(b), ptr(pred), 1 if save else 0, stream_handle()), "forward")

    def backward(self, dpred: torch.Tensor, grads: torch.Tensor):
        check(lib.inf_backward(self.handle, ptr(dpred), ptr(grads), stream_handle()), "backward")

    def train_step(self, b: Batch, pred: torch.Tensor | None, apply_adam: bool, advance: bool = False,
                   xslot: int | None = None, part: int | None = None, shard: bool = False):
        """inf_train_step; advance=True also moves ctrl.batch_index on (graph-replayed epochs);
        xslot: the batch's features were gathered into that pre-gather slot (prefetch);
        part 1 / 2: the bucketed halves of a gradient-only step (grad_split());
        shard: the reduced local gradient into grad_staging (the sharded step, shard())."""
        flags = (STEP_ADAM if apply_adam else 0) | (STEP_ADVANCE if advance else 0) | (STEP_SHARD if shard else 0)
        if xslot is not None:
            flags |= STEP_XSLOT0 if xslot == 0 else STEP_XSLOT1
        if part is not None:
            flags |= STEP_PART1 if part == 1 else STEP_PART2
        check(lib.inf_train_step(self.handle, ctypes.byref(b), ptr(pred), flags, stream_handle()), "train_step")

    def prefetch(self, b: Batch, slot: int) -> bool:
        """inf_prefetch_batch: gather the batch's features into pre-gather slot 0 / 1 on the
        current stream.  False (nothing launched) when its step does not run the fused chain."""
        rc = lib.inf_prefetch_batch(self.handle, ctypes.byref(b), int(slot), stream_handle())
        if rc == INF_OK:
            return True
        if rc == -4:  # INF_ERR_STATE: not a fused-chain batch
            return False
        check(rc, "prefetch_batch")

    def adam(self, step: int = 0, lr: float = 0.0, advance: bool = False):
        """inf_adam; advance=True also moves ctrl.batch_index on in the same launch
        (inf_adam_ex with INF_STEP_ADVANCE: the data-parallel step's tail)."""
        check(lib.inf_adam_ex(self.handle, int(step), float(lr), STEP_ADVANCE if advance else 0, stream_handle()),
              "adam")

    # ---- sharded optimizer step (data parallel; include/inf_hip.h) -----------------
    def shard(self, world: int, rank: int):
        """inf_plan_shard + inf_plan_bind_shard: the item-major staging layout of `world` ranks.
        Allocates grad_staging [world * shard_g] f32 (the reduce-scatter input), grad_chunk
        [shard_g] f32 (its output), weight_staging [world * shard_w] bytes (the all-gather
        buffer; weight_chunk() is this rank's part).  At world 1 the chunks alias the staging,
        so the collectives vanish."""
        g, w = c_int64(), c_int64()
        check(lib.inf_plan_shard(self.handle, int(world), int(rank), ctypes.byref(g), ctypes.byref(w)), "plan_shard")
        self.shard_world, self.shard_rank = int(world), int(rank)
        self.shard_g, self.shard_w = int(g.value), int(w.value)
        with torch.cuda.device(self.device):
            self.grad_staging = torch.zeros(world * self.shard_g, dtype=torch.float32, device=self.device)
            self.grad_chunk = self.grad_staging if world == 1 else torch.zeros(self.shard_g, dtype=torch.float32,
                                                                                device=self.device)
            self.weight_staging = torch.zeros(world * self.shard_w, dtype=torch.uint8, device=self.device)
            check(lib.inf_plan_bind_shard(self.handle, ptr(self.grad_staging), ptr(self.grad_chunk),
                                          ptr(self.weight_staging)), "plan_bind_shard")
        return self.shard_g, self.shard_w

    def debug_buffer(self, which: int) -> torch.Tensor:
        """inf_debug_buffer: a uint8 copy of a plan buffer (which 0 = the X^T images of the
        last fused step, 1 + i / 101 + i = segment i's forward / backward weight image; empty
        when it has none).  Diagnostics only."""
        n = c_int64(0)
        check(lib.inf_debug_buffer(self.handle, int(which), None, ctypes.byref(n), stream_handle()), "debug_buffer")
        out = torch.empty(max(n.value, 0), dtype=torch.uint8, device=self.device)
        if n.value:
            check(lib.inf_debug_buffer(self.handle, int(which), ptr(out), ctypes.byref(n), stream_handle()),
                  "debug_buffer")
        return out

    def can_shard(self, b: Batch) -> bool:
        """inf_plan_can_shard: this batch's step takes a fused chain, so it can run sharded."""
        return bool(lib.inf_plan_can_shard(self.handle, ctypes.byref(b)))

    def weight_chunk(self) -> torch.Tensor:
        r, n = self.shard_rank, self.shard_w
        return self.weight_staging[r * n:(r + 1) * n]

    def adam_shard(self, advance: bool = False):
        """inf_adam_shard: Adam on this rank's items from grad_chunk, new weights into weight_chunk()."""
        check(lib.inf_adam_shard(self.handle, STEP_ADVANCE if advance else 0, stream_handle()), "adam_shard")

    def shard_scatter(self):
        """inf_shard_scatter: every weight image and fp32 vector parameter from weight_staging."""
        check(lib.inf_shard_scatter(self.handle, stream_handle()), "shard_scatter")

    def shard_pack(self, arena: torch.Tensor):
        """inf_shard_pack: this rank's items of `arena` (params / exp_avg / exp_avg_sq) -> grad_chunk."""
        check(lib.inf_shard_pack(self.handle, ptr(arena), ptr(self.grad_chunk), stream_handle()), "shard_pack")

    def shard_unpack(self, arena: torch.Tensor):
        """inf_shard_unpack: every item of grad_staging -> `arena`."""
        check(lib.inf_shard_unpack(self.handle, ptr(self.grad_staging), ptr(arena), stream_handle()), "shard_unpack")

    def render(self, b: Batch, hit: torch.Tensor, pixel_map: torch.Tensor | None, img: torch.Tensor):
        check(lib.inf_render(self.handle, ctypes.byref(b), ptr(hit), ptr(pixel_map), ptr(img), stream_handle()),
              "render")

    def can_project(self) -> bool:
        """project_table() applies: bf16 eigenfunction plans with the input skip layer."""
        d = self.desc
        return self.encoding is None and self.gemm_dtype == torch.bfloat16 and 0 <= d.skip < d.num_layers - 1

    def project_table(self, T: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """inf_project_table: rows (W_0 E[v], W_y E[v]) of a packed bf16 table T [V, in_pad]
        under the current weights, bf16 [inf_projected_rows(V), 2H]."""
        require_hip(T)
        if T.dtype != torch.bfloat16 or T.dim() != 2 or T.shape[1] != self.in_pad or not T.is_contiguous():
            raise ValueError("project_table reads the packed bf16 [V, in_pad] table")
        rows = int(lib.inf_projected_rows(T.shape[0]))
        if out is None:
            out = torch.empty((rows, 2 * self.desc.hidden), dtype=torch.bfloat16, device=T.device)
        check(lib.inf_project_table(self.handle, ptr(T), T.shape[0], ptr(out), stream_handle()), "project_table")
        return out

    def run_stage(self, stage: int, layer: int = 0, b: Batch | None = None):
        """Re-launch one stage of the last saved step; returns (flops, bytes) per launch."""
        f, by = ctypes.c_double(), ctypes.c_double()
        check(lib.inf_run_stage(self.handle, ctypes.byref(b) if b is not None else None, int(stage), int(layer),
                                ctypes.byref(f), ctypes.byref(by), stream_handle()), "run_stage")
        return f.value, by.value

    def last_step_path(self) -> str:
        """Kernel path of the last train_step: 'layered', 'chain', 'chain3', 'chain3_chunked',
        'chain3_wide' (64-ray tiles), 'chain3_zg' (chain3 after the gather + input-layer GEMM
        launch, zg.hip: the default for k_pad > 1024), 'chain_f32' (the fp32 mode's fused
        chain), 'chain3_x3' (the bf16x3 mode's split-bf16 chain)."""
        return {-1: None, 0: "layered", 2: "chain", 3: "chain3", 4: "chain3_chunked", 5: "chain3_wide", 6: "chain_f32",
                7: "chain3_x3", 10: "chain3_zg"}[
            int(lib.inf_plan_last_step_path(self.handle))]

    def weight_generation(self) -> int:
        """inf_plan_weight_generation: changes whenever an update launch may have moved the
        weights; -1 once one was graph-captured (then nothing derived may be cached)."""
        return int(lib.inf_plan_weight_generation(self.handle))

    def grad_split(self) -> int:
        """inf_plan_grad_split: gradient bucket 1 = arena [split, P), bucket 2 = [0, split)."""
        return int(lib.inf_plan_grad_split(self.handle))

    def last_step_fused_update(self) -> bool:
        """inf_plan_last_step_fused_update: the last step's update ran inside the dW GEMM launch."""
        return int(lib.inf_plan_last_step_fused_update(self.handle)) == 1

    def last_part1_bucketed(self) -> int:
        """inf_plan_last_part1_bucketed: 1 if the last part=1 step split the gradient, 0 if it
        reduced all of it (part=2 then does nothing), -1 before any."""
        return int(lib.inf_plan_last_part1_bucketed(self.handle))

    def ctrl_advance(self):
        check(lib.inf_ctrl_advance(self.handle, stream_handle()), "ctrl_advance")


class RaySource:
    """Device-resident rays + eigenfunction table (ray_dataloader.py:58-98 moves the same
    arrays to the device once).  Keeps int32 vertex ids and packed GEMM-dtype tables."""

    def __init__(self, E: torch.Tensor, vids: torch.Tensor, bary: torch.Tensor, rgbs: torch.Tensor | None,
                 validate: bool = True):
        require_hip(E, vids, bary, rgbs)
        self.E = E
        self.vids = vids
        V = E.shape[0]
        # the reference's E[vids] raises IndexError on a bad id (mesh.py:319); the kernels
        # additionally read such rows as zero (validate=False exercises that guard)
        if validate and vids.numel() and (int(vids.min()) < 0 or int(vids.max()) >= V):
            raise ValueError("vertex id out of range of the eigenfunction table")
        self.vids32 = vids.to(torch.int32).contiguous()
        self.bary = bary.to(torch.float32).contiguous()
        self.rgbs = None if rgbs is None else rgbs.to(torch.float32).contiguous()
        self._tables = {}

    def table_for(self, plan: Plan) -> torch.Tensor:
        if plan.encoding is not None:  # the fp32 V x 3 vertex table of the xyz front-ends
            if self.E.dim() != 2 or self.E.shape[1] != 3:
                raise ValueError("an xyz/ff/rff model reads the V x 3 vertex table (ray_dataloader.py:28-30)")
            T = self._tables.get("xyz")
            if T is None:
                T = self.E.to(torch.float32).contiguous()
                self._tables["xyz"] = T
            return T
        key = (plan.in_pad, plan.gemm_dtype)
        T = self._tables.get(key)
        if T is None:
            if self.E.shape[1] != plan.desc.in_dim:
                raise ValueError(f"table has {self.E.shape[1]} columns, model expects {plan.desc.in_dim}")
            T = pack_table(self.E, plan.in_pad, plan.gemm_dtype)
            self._tables[key] = T
        return T


class Bvh:
    """A triangle mesh's BVH on the device (inf_bvh_create): the GPU replacement of the
    reference's trimesh/embree RayMeshIntersector (mesh.py:111-117)."""

    def __init__(self, vertices, faces):
        import numpy as np
        v = np.ascontiguousarray(np.asarray(vertices, dtype=np.float32).reshape(-1, 3))
        f = np.ascontiguousarray(np.asarray(faces, dtype=np.int64).reshape(-1, 3))
        h = c_void_p()
        check(lib.inf_bvh_create(v.ctypes.data, v.shape[0], f.ctypes.data, f.shape[0], ctypes.byref(h)),
              "bvh_create")
        self.handle = h
        self.num_vertices, self.num_faces = v.shape[0], f.shape[0]
        nf, nn, dp = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32()
        check(lib.inf_bvh_info(h, ctypes.byref(nf), ctypes.byref(nn), ctypes.byref(dp)), "bvh_info")
        self.num_nodes, self.depth = nn.value, dp.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            lib.inf_bvh_destroy(h)
            self.handle = None

    @staticmethod
    def _cam(camCv2world, K):
        import numpy as np
        cam = np.ascontiguousarray(np.asarray(torch.as_tensor(camCv2world).detach().cpu(), dtype=np.float32)[:3, :4])
        k = np.ascontiguousarray(np.asarray(torch.as_tensor(K).detach().cpu(), dtype=np.float32)[:3, :3])
        return cam, k

    def cast(self, camCv2world, K, H: int, W: int, pixel_idx: torch.Tensor | None = None, device="cuda"):
        """One ray per pixel (or per pixel_idx entry): per-ray hit face (-1 = miss), Cramer
        barycentrics and unit directions, on the device."""
        cam, k = self._cam(camCv2world, K)
        if pixel_idx is not None:
            require_hip(pixel_idx)
            pixel_idx = pixel_idx.to(torch.int64).contiguous()
            n = pixel_idx.shape[0]
        else:
            n = H * W
        face = torch.empty(n, dtype=torch.int32, device=device)
        bary = torch.empty((n, 3), dtype=torch.float32, device=device)
        dirs = torch.empty((n, 3), dtype=torch.float32, device=device)
        check(lib.inf_raycast(self.handle, cam.ctypes.data, k.ctypes.data, H, W, ptr(pixel_idx), n, ptr(face), ptr(bary),
                              ptr(dirs), stream_handle()), "raycast")
        return face, bary, dirs

    def cast_rays(self, origins: torch.Tensor, dirs: torch.Tensor):
        """Given rays (device [L][3] f32): per-ray hit face and barycentrics."""
        require_hip(origins, dirs)
        o = origins.to(torch.float32).contiguous()
        d = dirs.to(torch.float32).contiguous()
        n = o.shape[0]
        face = torch.empty(n, dtype=torch.int32, device=o.device)
        bary = torch.empty((n, 3), dtype=torch.float32, device=o.device)
        check(lib.inf_raycast_rays(self.handle, ptr(o), ptr(d), n, ptr(face), ptr(bary), stream_handle()),
              "raycast_rays")
        return face, bary

    def compact(self, face: torch.Tensor, bary: torch.Tensor):
        """The hit lists of mesh.ray_mesh_intersect, in ray order: (vids [M][3] int64,
        bary [M][3] f32, hit_ray_idxs [M] int64, face_idxs [M] int64)."""
        require_hip(face, bary)
        n = face.shape[0]
        dev = face.device
        scratch = torch.empty(max((n + 255) // 256, 1), dtype=torch.int32, device=dev)
        count = torch.zeros(1, dtype=torch.int64, device=dev)
        vids = torch.empty((n, 3), dtype=torch.int64, device=dev)
        ob = torch.empty((n, 3), dtype=torch.float32, device=dev)
        ray = torch.empty(n, dtype=torch.int64, device=dev)
        fc = torch.empty(n, dtype=torch.int64, device=dev)
        check(lib.inf_compact_hits(self.handle, ptr(face), ptr(bary), n, ptr(scratch), ptr(count), ptr(vids), ptr(ob),
                                   ptr(ray), ptr(fc), stream_handle()), "compact_hits")
        m = int(count.item())
        return vids[:m], ob[:m], ray[:m], fc[:m]


class StepPipeline:
    """Training steps with the NEXT batch's gather on a side HIP stream.

    Step n reads its features from pre-gather slot n % 2 (inf_train_step XSLOT flags); the
    side stream gathers batch n + 1 into the other slot (inf_prefetch_batch, batch offset
    from ctrl.prefetch_index) and the main stream's step n + 1 waits for it.  `lead`:
      0 -- the gather starts when step n's fused chain / dW / update launches are done, so it
           runs beside what follows them on the main stream: the data-parallel step's
           gradient all-reduce and Adam;
      1 -- it starts when step n - 1 is done (the last reader of its slot), beside step n's
           own kernels.
    Measured on one MI355X at 4096 rays, config B: lead 1 beside the single-GPU fused step
    costs +14 us per step (the gather's workgroups contend with the fused chain's, which
    hold every CU); lead 0 in the world-1 data-parallel step +17 us (94.2 vs 77.4 us: with
    an empty all-reduce the gather and two cross-queue signals sit on the critical path).
    So the in-kernel gather stays the default; the pipeline is opt-in (INF_PREFETCH=1) for
    multi-GPU runs, where it would run beside the all-reduce.  Events order the two
    streams, so the pattern is captured into a HIP graph as it is (a fork / join per step).
    `start()` gathers batch 0 into slot 0; a graph of an even number of steps leaves the
    slot parity as it found it."""

    def __init__(self, plan: Plan, batch: Batch, lead: int = 0):
        self.plan, self.batch, self.lead = plan, batch, lead
        self.side = torch.cuda.Stream(device=plan.device)
        self.enabled = True

    def start(self) -> bool:
        """Epoch start: prefetch index 0, batch 0 into slot 0 (current stream).  False when
        the plan cannot pre-gather this batch (then step without slots)."""
        self.plan.set_prefetch_index(0)
        self.enabled = self.plan.prefetch(self.batch, 0)
        return self.enabled

    def run(self, count: int, step_fn, first_slot: int = 0, tail_fn=None):
        """Issues `count` steps: step_fn(xslot) enqueues one step's fused launches, then
        tail_fn() what follows them (the data-parallel all-reduce / Adam / advance)."""
        if not self.enabled:
            for _ in range(count):
                step_fn(None)
                if tail_fn is not None:
                    tail_fn()
            return
        main = torch.cuda.current_stream()
        self.side.wait_stream(main)
        prev_done, ready = None, None
        for j in range(count):
            slot = (first_slot + j) % 2
            if ready is not None:
                main.wait_event(ready)
            step_fn(slot)
            done = torch.cuda.Event()
            done.record(main)
            after = done if self.lead == 0 else prev_done
            with torch.cuda.stream(self.side):
                if after is not None:
                    self.side.wait_event(after)
                self.plan.prefetch(self.batch, 1 - slot)
                ready = torch.cuda.Event()
                ready.record(self.side)
            if tail_fn is not None:
                tail_fn()
            prev_done = done
        main.wait_stream(self.side)
