"""Debug: eager explicit-offset steps vs ctrl-offset steps on one plan."""
import os, sys
sys.path.insert(0, "/root/repo/intrinsic-neural-fields_amd"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
import numpy as np, torch
import config
from test_gpu_dp import _loaders
B, N = 1024, 2048
cfg = {"model": {"k": 64, "num_layers": 4, "mlp_hidden_dim": 128, "skip_layer_idx": 2, "kernels": {"mode": "fp32"}},
       "training": {"batch_size": B, "lr": 1e-3, "loss_type": "L1"}}
res = {}
for tag in ("explicit", "ctrl", "trainer_eager"):
    torch.manual_seed(0)
    model, optim = config.get_model_and_optim(cfg, None, "cuda")
    model.kernel_mode = "fp32"
    ld, _ = _loaders(B, N, True)
    torch.manual_seed(1)
    it = iter(ld)
    perm = ld.idxs.clone()
    rt = model.hip_runtime(); group = optim.fused_group_for(model); rt.ensure_optimizer_arenas()
    plan = model.hip_plan(B, "L1")
    optim.sync_runtime_state(model, rt, plan, group)
    if tag == "explicit":
        for i in range(2):
            plan.train_step(plan.make_batch(source=ld.source, ray_idx=perm, offset=i * B, batch=B, loss="L1"), None, apply_adam=True)
    elif tag == "ctrl":
        b = plan.make_batch(source=ld.source, ray_idx=perm, offset=0, batch=B, offset_from_ctrl=True, loss="L1")
        plan.set_batch_index(0)
        for i in range(2):
            plan.train_step(b, None, apply_adam=True, advance=True)
    else:
        for batch in it:
            print("batch offset", batch._offset, batch._count, batch._perm.data_ptr() == ld.idxs.data_ptr(), torch.equal(batch._perm, perm))
            model.fused_train_step(batch, optim, "L1", want_pred=False)
            print("ctrl", plan.read_ctrl())
    torch.cuda.synchronize()
    res[tag] = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
    print(tag, plan.read_ctrl())
print({k: float(np.abs(v - res["ctrl"]).max()) for k, v in res.items()})
