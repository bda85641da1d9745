"""The reference's two-step texture-reconstruction workflow through this build's CLIs:
training_scripts/train_cat_tex_recon.sh runs `train.py <config> --allow_checkpoint_loading`
and then `eval.py <out> <config> <dataset> test --uv_mesh_path <uv obj>` (reference
training_scripts/train_cat_tex_recon.sh:24-27), here on a synthetic dataset in the cat
config's layout (tests/synthetic_views.py; the cat is not available offline)."""
import json
import os
import pickle
import subprocess
import sys

import numpy as np
import pytest
import yaml

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_train_and_eval_scripts(tmp_path):
    import synthetic_views as S
    views = S.build(str(tmp_path))
    cfg = S.intrinsic_config(eval_views=views["val"][:1])
    cdir = tmp_path / "configs" / "texture_reconstruction"
    cdir.mkdir(parents=True)
    with open(cdir / "intrinsic_cat.yaml", "w") as fh:
        yaml.safe_dump(cfg, fh)
    env = dict(os.environ, PYTHON=sys.executable)
    r = subprocess.run(["bash", os.path.join(ROOT, "training_scripts", "train_cat_tex_recon.sh"), "intrinsic"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout[-3000:], r.stderr[-3000:])
    assert r.returncode == 0
    out = tmp_path / "out" / "texture_recon" / "intrinsic_cat"
    for f in ("model.pt", "model_last_epoch.pt", "checkpoint.pt"):
        assert (out / f).exists(), f
    # the trainer's visualisation rendered the validation view (trainer.py:285-300)
    tags = [json.loads(x)["tag"] for x in open(out / "logs" / "scalars.jsonl")]
    assert "img000_psnr" in tags and "img000_dist" in tags and "Val Epoch-PSNR" in tags
    ev = out / "test_eval"
    with open(ev / "evaluation_metrics.pkl", "rb") as fh:  # written by eval.py in this test
        metrics = pickle.load(fh)
    assert sorted(metrics) == ["000", "001"]
    for m in metrics.values():
        assert np.isfinite(m["psnr"]) and m["psnr"] > 10 and 0 <= m["dssim_rescaled"] < 50
    for i in ("000", "001"):
        for kind in ("fake_raw", "fake", "real"):
            assert (ev / f"{i}_{kind}.png").exists()
    assert (ev / "baked" / "texture.png").exists()
    assert "PSNR:" in r.stdout
