"""Host mirror of the reference model.py (TextureField + make_model).

The module tree, parameter names/order and the seeded initialisation are the
reference's (model.py:12-96 TextureField.__init__, 194-258 init_weights/make_model),
so `state_dict()` files are interchangeable with the reference's.  The arithmetic of
`forward` (model.py:98-112) and of its autograd backward runs in libinf_hip.so: the
parameters live in one flat fp32 arena on the HIP device (each nn.Parameter is a view
into it), the kernels read packed GEMM-dtype copies that are refreshed whenever a
parameter changes, and a batch whose features were not materialised is gathered inside
the same launch sequence (mesh.py:313-324 fused into the forward).

Kernel arithmetic mode: `model_config["kernels"]["mode"]` ("fp32" exact f32 MFMA, the
default, or "bf16" MFMA with fp32 accumulation), overridable by INF_MODE.
"""
from __future__ import annotations

import os
import weakref

import numpy as np
import torch
import torch.nn as nn

from layers import FourierFeatEnc, LinearWithConcatAndActivation, RandomFourierFeatEnc

RGB_COLOR_DIM = 3

# arena base pointer -> runtime (lets the optimizer find the arena of its params)
_RUNTIMES: "weakref.WeakValueDictionary[int, _Runtime]" = weakref.WeakValueDictionary()


def _hip():
    from inf_hip import runtime  # raises if the HIP library is missing: no fallback
    return runtime


class _Runtime:
    """Device state of one TextureField: parameter arena, optimizer arenas, plan."""

    def __init__(self, module: "TextureField", device: torch.device, arena: torch.Tensor):
        self.module_ref = weakref.ref(module)
        self.device = device
        self.arena = arena
        self.grads = None
        self.exp_avg = None
        self.exp_avg_sq = None
        self.plan = None
        self.synced = None          # parameter versions the packed weights reflect
        self.gen = 0                # id of the last forward that saved activations
        self.saved_gen = None
        self.dev_step = None        # value of ctrl.step as last set/advanced
        self.dev_lr = None
        _RUNTIMES[arena.data_ptr()] = self

    def ensure_optimizer_arenas(self):
        if self.exp_avg is None:
            self.grads = torch.zeros_like(self.arena)
            self.exp_avg = torch.zeros_like(self.arena)
            self.exp_avg_sq = torch.zeros_like(self.arena)
            if self.plan is not None:
                self.plan.bind(self.grads, self.exp_avg, self.exp_avg_sq)


class TextureField(nn.Module):
    """Reference model.py:12-112.  Supported: feature strategies "efuncs" and the
    extrinsic "xyz" / "rff" (and "ff", which the reference's own constructor rejects),
    ReLU, batchnorm=False, sigmoid RGB head (every TextureField config in configs/)."""

    def __init__(self, num_layers, in_dim, hidden_dim, skip_layer_idx, input_feature_embed=None, embed_dim=None,
                 embed_include_input=True, embed_std=1., return_rgb=True, out_dim=RGB_COLOR_DIM, batchnorm=False,
                 activation=nn.ReLU):
        super().__init__()
        assert num_layers > 2 and 0 < skip_layer_idx and skip_layer_idx < num_layers - 1
        if batchnorm:
            raise NotImplementedError("batchnorm=True is not used by any intrinsic config and is not implemented")
        if activation is not nn.ReLU:
            raise NotImplementedError("only the ReLU activation is implemented")
        # the fused plan serves the sigmoid RGB head; the ReLU bottleneck of the view-dependent
        # field's spatial MLP (model.py:115-160) runs on the generic dense layers (dense.py)
        self.return_rgb = return_rgb
        self.dense_mode = not return_rgb or out_dim != RGB_COLOR_DIM
        self.skip_layer_idx = skip_layer_idx
        self.input_feature_embed = input_feature_embed
        # model.py:33-40: the encoder (and its RNG draw) precedes the layers
        if input_feature_embed == "ff":
            self.embedding = FourierFeatEnc(embed_dim, include_input=embed_include_input)
            in_dim = 3 * embed_dim * 2 + (3 if embed_include_input else 0)
        elif input_feature_embed == "rff":
            self.embedding = RandomFourierFeatEnc(embed_dim, std=embed_std, include_input=embed_include_input)
            in_dim = embed_dim * 2 + (3 if embed_include_input else 0)
        else:
            self.embedding = None
        self.num_layers = num_layers
        self.in_dim = in_dim
        self.hidden_dim = hidden_dim

        layers = [nn.Sequential(nn.Linear(in_dim, hidden_dim), activation())]
        for i in range(1, num_layers - 1):
            if i == skip_layer_idx:
                layers.append(LinearWithConcatAndActivation(hidden_dim, in_dim, hidden_dim, batchnorm=batchnorm,
                                                            activation=activation))
            else:
                layers.append(nn.Sequential(nn.Linear(hidden_dim, hidden_dim), activation()))
        layers.append(nn.Sequential(nn.Linear(hidden_dim, out_dim), nn.Sigmoid() if return_rgb else activation()))
        self.layers = nn.ModuleList(layers)

        self.kernel_mode = os.environ.get("INF_MODE", "fp32")
        self.max_batch_hint = 4096
        self._rt: _Runtime | None = None

    # ---- device binding ----------------------------------------------------------
    def _layout(self):
        params = list(self.parameters())
        offs, off = [], 0
        for p in params:
            offs.append(off)
            off += p.numel()
        return params, offs, off

    def hip_runtime(self) -> _Runtime:
        """Bind the parameters to a flat arena on their HIP device (once; re-binds after
        .to(), load_state_dict(assign=True) or any other re-pointing of .data)."""
        params, offs, P = self._layout()
        dev = params[0].device
        if dev.type != "cuda" or any(p.device != dev for p in params):
            raise RuntimeError("TextureField runs on one MI355X (HIP) device; move it with .to('cuda'). "
                               "There is no CPU fallback.")
        rt = self._rt
        if rt is None or rt.device != dev or rt.arena.numel() != P:
            with torch.no_grad():
                arena = torch.empty(P, dtype=torch.float32, device=dev)
                for p, o in zip(params, offs):
                    arena[o:o + p.numel()].copy_(p.detach().reshape(-1))
            rt = _Runtime(self, dev, arena)
            self._rt = rt
        base = rt.arena.data_ptr()
        for p, o in zip(params, offs):
            if p.data_ptr() != base + 4 * o or not p.is_contiguous() or p.dtype != torch.float32:
                with torch.no_grad():
                    rt.arena[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = rt.arena[o:o + p.numel()].view(p.shape)
                rt.synced = None
        return rt

    def _versions(self):
        return tuple(p._version for p in self.parameters())

    @property
    def extrinsic(self) -> bool:
        """Position-fed front-end (ray_dataloader.py:134-136) instead of eigenfunctions."""
        return self.input_feature_embed in ("ff", "rff", "xyz")

    def _encoding(self):
        if not self.extrinsic:
            return None
        rt = _hip()
        if self.input_feature_embed == "xyz":
            return rt.Encoding("xyz")
        e = self.embedding
        proj = e.B if self.input_feature_embed == "rff" else e.freq_bands
        if proj.dtype != torch.float32 or not proj.is_contiguous():
            raise ValueError("the encoder's projection must be a contiguous fp32 buffer")
        return rt.Encoding(self.input_feature_embed, proj.shape[-1], proj, e.include_input)

    def hip_plan(self, batch: int, loss: str = "L2"):
        rt = self.hip_runtime()
        plan = rt.plan
        if plan is None or batch > plan.max_batch or plan.mode != self.kernel_mode:
            mb = max(batch, self.max_batch_hint, 2 * plan.max_batch if plan is not None and batch > plan.max_batch
                     else 0)
            rt.plan = None  # free the old workspace first
            plan = _hip().Plan(self.in_dim, self.hidden_dim, self.num_layers, self.skip_layer_idx,
                               self.kernel_mode, loss, mb, rt.arena, rt.grads, rt.exp_avg, rt.exp_avg_sq)
            rt.plan = plan
            rt.synced = self._versions()
            rt.saved_gen = None
            rt.dev_step = 0
            rt.dev_lr = None
        versions = self._versions()
        if rt.synced != versions:
            plan.sync_shadow()
            rt.synced = versions
        plan.encoding = self._encoding()
        return plan

    # ---- forward (model.py:98-112) -----------------------------------------------
    def __deepcopy__(self, memo):
        """Copies parameters and structure, not the device runtime (plan handles and
        workspaces are per instance; the copy binds its own on first use)."""
        import copy as _copy
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            new.__dict__[k] = None if k == "_rt" else _copy.deepcopy(v, memo)
        return new

    def _input_features(self, batch):
        """model.py:98-104: the MLP input of a batch (materialised) for the dense path."""
        if self.extrinsic:
            x = batch["xyz"]
            if self.input_feature_embed == "xyz":
                return x.to(torch.float32)
            return self.embedding(x)
        return batch["eigenfunctions"].to(torch.float32)

    def _dense_forward(self, batch):
        import dense
        x = self._input_features(batch)
        if not x.is_cuda:
            raise RuntimeError("TextureField runs on MI355X (HIP) devices only. There is no CPU fallback.")
        h = x
        n = len(self.layers)
        for i, layer in enumerate(self.layers):
            if i == self.skip_layer_idx:
                h = dense.linear([(h, 0, 0), (x, 1, 0)], [layer.Lx.weight, layer.Ly.weight],
                                 [layer.Lx.bias, layer.Ly.bias], "relu")
            else:
                lin = layer[0]
                act = "relu" if i < n - 1 or not self.return_rgb else "sigmoid"
                h = dense.linear([(h, 0, 0)], [lin.weight], [lin.bias], act)
        return h

    def forward(self, batch):
        if self.dense_mode:
            return self._dense_forward(batch)
        params = list(self.parameters())
        needs = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        lazy = getattr(batch, "is_lazy_rays", None)
        if lazy is not None and lazy():
            feats, rays = None, batch.ray_args()
            if rays["extrinsic"] != self.extrinsic:
                raise ValueError("the loader's feature strategy does not match the model's input_feature_embed")
            B = rays["batch"]
        elif self.extrinsic:
            xyz = batch["xyz"]  # model.py:99-101
            if not xyz.is_cuda:
                raise RuntimeError("TextureField runs on MI355X (HIP) devices only; positions are on "
                                   f"{xyz.device}. There is no CPU fallback.")
            xyz = xyz.to(torch.float32).contiguous()
            rays = {"xyz": xyz}
            return _TextureFieldFn.apply(self, None, rays, xyz.shape[0], needs, *params)
        else:
            feats = batch["eigenfunctions"]
            if not feats.is_cuda:
                raise RuntimeError("TextureField runs on MI355X (HIP) devices only; features are on "
                                   f"{feats.device}. There is no CPU fallback.")
            if feats.requires_grad:
                raise NotImplementedError("gradients w.r.t. the eigenfunction features are not needed by the "
                                          "reference (they are data) and are not implemented")
            feats = feats.to(torch.float32).contiguous()
            rays, B = None, feats.shape[0]
        return _TextureFieldFn.apply(self, feats, rays, B, needs, *params)

    # ---- fused training step (used by trainer.Trainer) ------------------------------
    def fused_train_step(self, batch, optim, loss_type: str, want_pred: bool = True, loss_count: int = 0):
        """gather -> forward -> loss -> backward -> Adam in one launch sequence
        (trainer.py:71-84 with the loss of config.py:113-122).  Returns pred or None."""
        rays = batch.ray_args()
        B = rays["batch"]
        rt = self.hip_runtime()
        group = optim.fused_group_for(self)
        rt.ensure_optimizer_arenas()
        plan = self.hip_plan(B, loss_type)
        optim.sync_runtime_state(self, rt, plan, group)
        pred = torch.empty((B, 3), device=rt.device) if want_pred else None
        b = plan.make_batch(source=rays["source"], ray_idx=rays["ray_idx"], offset=rays["offset"], batch=B,
                            loss_count=loss_count, loss=loss_type)
        plan.train_step(b, pred, apply_adam=True)
        rt.saved_gen = None
        optim.after_fused_step(self, rt, group)
        return pred


def _make_batch(plan, feats, rays, B):
    if rays is None:
        return plan.make_batch(features=feats)
    if "xyz" in rays:
        return plan.make_batch(xyz=rays["xyz"])
    return plan.make_batch(source=rays["source"], ray_idx=rays["ray_idx"], offset=rays["offset"], batch=B)


class _TextureFieldFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, module, feats, rays, B, needs, *params):
        plan = module.hip_plan(B)
        rt = module._rt
        b = _make_batch(plan, feats, rays, B)
        pred = torch.empty((B, 3), device=rt.device)
        plan.forward(b, pred, save=needs)
        if needs:
            rt.gen += 1
            rt.saved_gen = rt.gen
            ctx.gen = rt.gen
            ctx.module = module
            ctx.rays = rays
            ctx.B = B
            ctx.plan = plan
            ctx.shapes = [p.shape for p in params]
            if feats is not None:
                ctx.save_for_backward(feats)
        else:
            rt.saved_gen = None
        return pred

    @staticmethod
    def backward(ctx, dpred):
        module, plan = ctx.module, ctx.plan
        rt = module._rt
        if rt.plan is not plan or rt.saved_gen != ctx.gen:
            # activations were overwritten by another forward: recompute them
            plan = module.hip_plan(ctx.B)
            b = _make_batch(plan, ctx.saved_tensors[0] if ctx.rays is None else None, ctx.rays, ctx.B)
            plan.forward(b, torch.empty((ctx.B, 3), device=rt.device), save=True)
            rt.gen += 1
            rt.saved_gen = rt.gen
            ctx.gen = rt.gen
        grads = torch.empty(plan.info.num_params, dtype=torch.float32, device=rt.device)
        plan.backward(dpred.to(torch.float32).contiguous(), grads)
        out = []
        for off, n, shape in zip(plan.offsets, plan.numels, ctx.shapes):
            out.append(grads[off:off + n].view(shape))
        return (None, None, None, None, None, *out)


class TextureFieldWithViewDependency(nn.Module):
    """Reference model.py:115-191: a TextureField with a ReLU bottleneck output, the
    viewing direction (its angle to the hit face's normal, "intrinsic", or the direction
    itself, "extrinsic") Fourier-encoded, and a two-layer directional MLP with a sigmoid
    RGB head.  Same module tree and parameter order as the reference; every layer runs on
    the generic fp32 dense kernels (dense.py / csrc/dense.hip) -- no config in configs/
    enables view dependence, so it is off the fused hot path."""

    def __init__(self, num_layers, in_dim, hidden_dim, skip_layer_idx, bottleneck_vec_dim, in_dim_view_dir,
                 include_view_dir, view_dir_embedding_size, directional_hidden_dim, input_feature_embed=None,
                 embed_dim=None, embed_include_input=True, embed_std=1., face_normals=None,
                 view_dir_strategy="intrinsic", batchnorm=False, activation=nn.ReLU):
        super().__init__()
        self.view_dir_strategy = view_dir_strategy
        if face_normals is not None:
            self.register_buffer("face_normals", face_normals, persistent=False)
        self.spatial_mlp = TextureField(num_layers, in_dim, hidden_dim, skip_layer_idx,
                                        input_feature_embed=input_feature_embed, embed_dim=embed_dim,
                                        embed_include_input=embed_include_input, embed_std=embed_std,
                                        return_rgb=False, out_dim=bottleneck_vec_dim, batchnorm=batchnorm,
                                        activation=activation)
        self.embedding = FourierFeatEnc(view_dir_embedding_size, include_input=include_view_dir, use_logspace=True)
        embedding_size = in_dim_view_dir * view_dir_embedding_size * 2 + (in_dim_view_dir if include_view_dir else 0)
        self.bottleneck_vec_dim = bottleneck_vec_dim
        self.directional_mlp = nn.Sequential(nn.Linear(bottleneck_vec_dim + embedding_size, directional_hidden_dim),
                                             activation(), nn.Linear(directional_hidden_dim, RGB_COLOR_DIM),
                                             nn.Sigmoid())

    def _get_embedded_view_dir(self, batch):
        """model.py:162-172."""
        import dense
        if self.view_dir_strategy == "intrinsic":
            angles = dense.view_angles(batch["unit_ray_dirs"], batch["hit_face_idxs"], self.face_normals)
            return self.embedding(angles.unsqueeze(-1))
        if self.view_dir_strategy == "extrinsic":
            return self.embedding(batch["unit_ray_dirs"].to(torch.float32))
        raise RuntimeError("Unknown viewing direction strategy.")

    def forward(self, batch):
        """model.py:174-177; the concatenation is two column ranges of the first
        directional weight."""
        import dense
        bottleneck = self.spatial_mlp(batch)
        view = self._get_embedded_view_dir(batch)
        l0, l2 = self.directional_mlp[0], self.directional_mlp[2]
        h = dense.linear([(bottleneck, 0, 0), (view, 0, self.bottleneck_vec_dim)], [l0.weight], [l0.bias], "relu")
        return dense.linear([(h, 0, 0)], [l2.weight], [l2.bias], "sigmoid")


def init_weights(m):
    """Reference model.py:194-196."""
    if isinstance(m, nn.Linear):
        torch.nn.init.xavier_uniform_(m.weight.data)


def make_model(model_config, mesh=None):
    """Reference model.py:199-258 for the TextureField configurations (efuncs, xyz, rff)."""
    view_dependence_config = model_config.get("view_dependence")
    feature_strategy = model_config.get("feature_strategy", "efuncs")
    if model_config.get("type") == "neutex":
        raise NotImplementedError("the NeuTex baseline is outside this build's scope")
    if feature_strategy == "xyz":
        in_dim = 3
    elif isinstance(model_config["k"], int):
        in_dim = model_config["k"]
    else:
        assert isinstance(model_config["k"], list)
        in_dim = len(model_config["k"])
    activation_fn = model_config.get("activation", "relu")
    if activation_fn != "relu":
        raise NotImplementedError(f"Activation function {activation_fn} not yet implemented.")
    if view_dependence_config is None:
        model = TextureField(model_config["num_layers"], in_dim, model_config["mlp_hidden_dim"],
                             model_config["skip_layer_idx"], input_feature_embed=feature_strategy,
                             embed_dim=model_config.get("k"),
                             embed_include_input=model_config.get("embed_include_input", True),
                             embed_std=model_config.get("embed_std", 1.),
                             batchnorm=model_config.get("batchnorm", False), activation=nn.ReLU)
    else:  # model.py:240-256
        assert mesh is not None
        face_normals = torch.from_numpy(np.array(mesh.face_normals, copy=True)).to(dtype=torch.float32)
        v = view_dependence_config
        model = TextureFieldWithViewDependency(model_config["num_layers"], in_dim, model_config["mlp_hidden_dim"],
                                               model_config["skip_layer_idx"], v["bottleneck_vec_dim"],
                                               v["in_dim_view_dir"], v["include_view_dir"], v["embed_size"],
                                               v["directional_hidden_dim"], input_feature_embed=feature_strategy,
                                               embed_dim=model_config.get("k"),
                                               embed_include_input=model_config.get("embed_include_input", True),
                                               embed_std=model_config.get("embed_std", 1.), face_normals=face_normals,
                                               view_dir_strategy=v["strategy"],
                                               batchnorm=model_config.get("batchnorm", False), activation=nn.ReLU)
    model.apply(init_weights)
    kernels = model_config.get("kernels") or {}
    model.kernel_mode = os.environ.get("INF_MODE", kernels.get("mode", "fp32"))
    if kernels.get("max_batch"):
        model.max_batch_hint = int(kernels["max_batch"])
    return model
