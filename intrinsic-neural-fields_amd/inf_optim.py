"""Adam on the HIP device for TextureField parameters.

Drop-in for the `torch.optim.Adam(model.parameters(), lr=...)` the reference creates at
config.py:108: it IS a torch.optim.Adam subclass, so param_groups, `zero_grad`,
`state_dict()` / `load_state_dict()` and the per-parameter state keys (`step`,
`exp_avg`, `exp_avg_sq`) are torch's own.  `step()` runs the single-tensor Adam formula
of torch 2.x in libinf_hip.so (csrc/adam.hip) over the model's flat arenas and refreshes
the packed GEMM weights in the same launch.  exp_avg / exp_avg_sq are views into the
runtime's device arenas.
"""
from __future__ import annotations

import torch

import model as _model


class Adam(torch.optim.Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, **kwargs):
        kwargs.pop("foreach", None)
        kwargs.pop("fused", None)
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         foreach=False, **kwargs)

    # ---- helpers -------------------------------------------------------------------
    @staticmethod
    def _check_group(group):
        if group["weight_decay"] != 0 or group["amsgrad"] or group.get("maximize", False) or \
                group.get("capturable", False) or group.get("differentiable", False):
            raise NotImplementedError("HIP Adam implements the reference's configuration: weight_decay=0, "
                                      "amsgrad=False, maximize=False")

    def _runtime_of(self, params):
        """(runtime, params) groups of arena-bound parameters, and the free ones (layers on
        the generic dense kernels, e.g. the view-dependent field)."""
        rts, free = {}, []
        for p in params:
            rt = None
            for base, r in list(_model._RUNTIMES.items()):
                if base <= p.data_ptr() < base + 4 * r.arena.numel():
                    rt = r
                    break
            if rt is None:
                if not p.is_cuda:
                    raise RuntimeError("HIP Adam updates device parameters only. There is no CPU fallback.")
                free.append(p)
                continue
            rts.setdefault(id(rt), (rt, []))[1].append(p)
        return list(rts.values()), free

    def _step_free(self, p, group):
        """torch.optim.Adam's single-tensor step for one parameter outside a plan arena
        (csrc/dense.hip inf_adam_dense, the plan update's arithmetic)."""
        import dense
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0, dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        step = int(st["step"].item()) + 1
        b1, b2 = group["betas"]
        g = p.grad.to(torch.float32).contiguous()
        dense.adam_step(p.data, g, st["exp_avg"], st["exp_avg_sq"], step, group["lr"], b1, b2, group["eps"])
        st["step"] += 1

    def _bind_state(self, module, rt, group):
        """Make every parameter's exp_avg/exp_avg_sq a view into the runtime's arenas
        (after load_state_dict, torch replaces them with fresh tensors: copy those in)."""
        rt.ensure_optimizer_arenas()
        params, offs, _ = module._layout()
        steps = set()
        for p, o in zip(params, offs):
            st = self.state[p]
            n = p.numel()
            m_view = rt.exp_avg[o:o + n].view(p.shape)
            v_view = rt.exp_avg_sq[o:o + n].view(p.shape)
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                m_view.zero_()
                v_view.zero_()
                st["exp_avg"] = m_view
                st["exp_avg_sq"] = v_view
            else:
                for key, view in (("exp_avg", m_view), ("exp_avg_sq", v_view)):
                    t = st[key]
                    if t.data_ptr() != view.data_ptr():
                        view.copy_(t.to(device=view.device, dtype=torch.float32).reshape(view.shape))
                        st[key] = view
            steps.add(float(st["step"]))
        if len(steps) != 1:
            raise RuntimeError("all TextureField parameters must share one Adam step count")
        return params, int(steps.pop())

    # ---- fused path (trainer.Trainer) ------------------------------------------------
    def fused_group_for(self, module):
        params = list(module.parameters())
        ids = {id(p) for p in params}
        for group in self.param_groups:
            gids = {id(p) for p in group["params"]}
            if ids <= gids:
                self._check_group(group)
                return group
        raise RuntimeError("optimizer does not hold all TextureField parameters in one group")

    @torch.no_grad()
    def sync_runtime_state(self, module, rt, plan, group):
        _, step = self._bind_state(module, rt, group)
        b1, b2 = group["betas"]
        plan.set_adam(float(b1), float(b2), float(group["eps"]))
        if rt.dev_step != step:
            plan.set_step(step)
            rt.dev_step = step
        lr = float(group["lr"])
        if rt.dev_lr != lr:
            plan.set_lr(lr)
            rt.dev_lr = lr

    def after_fused_step(self, module, rt, group):
        self.after_fused_steps(module, rt, group, 1)

    def after_fused_steps(self, module, rt, group, n):
        for p in module.parameters():
            self.state[p]["step"] += n
        rt.dev_step += n

    # ---- torch API -------------------------------------------------------------------
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            self._check_group(group)
            with_grad = [p for p in group["params"] if p.grad is not None]
            if not with_grad:
                continue
            groups, free = self._runtime_of(with_grad)
            for p in free:
                self._step_free(p, group)
            for rt, ps in groups:
                module = rt.module_ref()
                mparams, offs, _ = module._layout()
                if len(ps) != len(mparams):
                    raise NotImplementedError("HIP Adam updates a TextureField's parameters together; some "
                                              "have no gradient")
                _, step = self._bind_state(module, rt, group)
                plan = module.hip_plan(1)
                # gradients into the flat arena (autograd may hand back views of the backward's
                # flat buffer; a contiguous copy either way)
                flat = rt.grads
                for p, o in zip(mparams, offs):
                    g = p.grad
                    dst = flat[o:o + p.numel()]
                    if g.data_ptr() != dst.data_ptr():
                        dst.copy_(g.reshape(-1))
                b1, b2 = group["betas"]
                plan.set_adam(float(b1), float(b2), float(group["eps"]))
                plan.adam(step + 1, float(group["lr"]))
                for p in mparams:
                    self.state[p]["step"] += 1
                rt.dev_step = None  # host-driven step: re-sync ctrl before the next fused step
        return loss
