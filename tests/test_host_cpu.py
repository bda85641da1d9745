"""Host-side mirror of the reference surface, on CPU (no kernel launches)."""
import os

import numpy as np
import pytest
import torch

from conftest import golden

CFG = {"A": (64, 4, 128, 2), "R": (list(range(0, 256)) + list(range(1793, 2304)) + list(range(3840, 4096)), 6, 128, 3),
       "B": (1024, 8, 256, 4)}


@pytest.mark.parametrize("name", ["A", "R", "B"])
def test_make_model_seed0_init_matches_reference(name):
    """model.py:194-258: same module tree + xavier init -> bitwise the reference's weights."""
    import model as M
    k, L, H, s = CFG[name]
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s, "batchnorm": False})
    d = golden(f"g2_forward_{name}.npz")
    sd = m.state_dict()
    ref = {kk[2:]: d[kk] for kk in d.files if kk.startswith("w:")}
    assert list(sd.keys()) == list(ref.keys())
    for key in sd:
        np.testing.assert_array_equal(sd[key].numpy(), ref[key], err_msg=key)


def test_make_model_rejects_out_of_scope():
    import model as M
    with pytest.raises(NotImplementedError):
        M.make_model({"k": 8, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2, "activation": "sine"})
    with pytest.raises(AssertionError):  # model.py:243: view dependence needs the mesh's face normals
        M.make_model({"k": 8, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2,
                      "view_dependence": {"strategy": "intrinsic"}})
    with pytest.raises(AssertionError):
        M.make_model({"k": 8, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 3})


def test_forward_refuses_cpu_tensors():
    """No CPU fallback on the product path."""
    import model as M
    m = M.make_model({"k": 8, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2})
    with pytest.raises(RuntimeError, match="HIP"):
        m({"eigenfunctions": torch.zeros(4, 8)})
    mx = M.make_model({"k": 8, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2, "feature_strategy": "rff"})
    with pytest.raises(RuntimeError, match="HIP"):
        mx({"xyz": torch.zeros(4, 3)})


def test_load_first_k_eigenfunctions_matches_reference(tmp_path):
    import mesh
    d = golden("g1_load_efuncs.npz")
    p = tmp_path / "e.npy"
    np.save(p, d["table"])
    for strat in ("standard", "one-norm", "unscaled"):
        np.testing.assert_allclose(mesh.load_first_k_eigenfunctions(str(p), 24, strat).numpy(), d[f"int_{strat}"],
                                   rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(mesh.load_first_k_eigenfunctions(str(p), list(map(int, d["k_list"])), strat).numpy(),
                                   d[f"list_{strat}"], rtol=1e-6, atol=1e-7)


def test_preprocessed_format_roundtrip(tmp_path):
    import dataset
    rng = np.random.default_rng(0)
    v = rng.integers(0, 100, (20, 3))
    b = rng.random((20, 3)).astype(np.float32)
    c = rng.random((20, 3)).astype(np.float32)
    dataset.save_preprocessed_data(str(tmp_path), v, b, c, unit_ray_dirs=b, face_idxs=v[:, 0])
    data = dataset.load_preprocessed_data(str(tmp_path))
    assert data["vertex_idxs_of_hit_faces"].dtype == torch.int64
    np.testing.assert_array_equal(data["vertex_idxs_of_hit_faces"].numpy(), v)
    np.testing.assert_array_equal(data["barycentric_coords"].numpy(), b)
    assert data["face_idxs"].dtype == torch.int64 and data["unit_ray_dirs"].dtype == torch.float32


def test_metrics_match_reference():
    import evaluation_metrics as em
    d = golden("g6_psnr.npz")
    assert abs(em.psnr(d["a"], d["b"]) - float(d["psnr_full"])) < 1e-9
    assert abs(em.psnr(d["a"], d["b"], d["mask"]) - float(d["psnr_mask"])) < 1e-9
    assert abs(em.epoch_psnr(float(d["epoch_mse"])) - float(d["epoch_psnr"])) < 1e-12


def test_batchify_and_to_device():
    import utils
    data = {"a": torch.arange(10), "b": torch.arange(20).reshape(10, 2)}
    bs = utils.batchify_dict_data(data, 10, 4)
    assert [len(x["a"]) for x in bs] == [4, 4, 2]
    assert torch.equal(torch.cat([x["b"] for x in bs]), data["b"])
    out = utils.to_device({"x": torch.ones(2), "s": "name"}, device="cpu")
    assert out["s"] == "name"


def test_loss_fns_and_config(tmp_path):
    import config
    for lt in ("L2", "L1", "cauchy"):
        fn = config.get_loss_fn({"training": {"loss_type": lt}})
        assert fn.loss_type == lt
        p, t = torch.rand(8, 3), torch.rand(8, 3)
        from oracle import inf_oracle as O
        assert abs(float(fn(p, t)) - O.loss_value(p.numpy(), t.numpy(), lt)) < 1e-6
    with pytest.raises(RuntimeError):
        config.get_loss_fn({"training": {"loss_type": "L3"}})
    cfg_path = os.path.join(os.path.dirname(__file__), "..", "configs", "texture_reconstruction",
                            "intrinsic_cat_k1024_8x256.yaml")
    c = config.load_config(cfg_path)
    assert c["model"]["k"] == 1024 and c["model"]["num_layers"] == 8 and c["model"]["skip_layer_idx"] == 4
    assert config.get_seed(c) == 0


def test_dp_shard_span():
    import dp
    for B in (1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            spans = [dp.shard_span(B, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            for (a, b), (c, _) in zip(spans, spans[1:]):
                assert b == c
            # torch.chunk split (what DataParallel's scatter does)
            chunks = torch.arange(B).chunk(world)
            for r, ch in enumerate(chunks):
                assert spans[r] == (int(ch[0]), int(ch[-1]) + 1)


@pytest.mark.parametrize("tag", ["rff", "rffni", "xyz"])
def test_frontend_model_init_matches_reference(tag):
    """make_model for the extrinsic strategies (model.py:33-40,199-258): same parameter and
    buffer names, and the same seeded values -- the RFF matrix is drawn before the layers."""
    import model as M
    d = golden(f"g9_frontend_{tag}.npz")
    fe = {"rff": {"feature_strategy": "rff", "k": 16, "embed_std": 8.0, "embed_include_input": True},
          "rffni": {"feature_strategy": "rff", "k": 24, "embed_std": 2.0, "embed_include_input": False},
          "xyz": {"feature_strategy": "xyz", "k": 170}}[tag]
    torch.manual_seed(0)
    m = M.make_model(dict(fe, num_layers=4, mlp_hidden_dim=64, skip_layer_idx=2))
    sd = m.state_dict()
    ref = {k[2:]: d[k] for k in d.files if k.startswith("w:")}
    assert set(sd) == set(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), v, err_msg=k)


def test_ff_strategy_rejected_like_reference():
    """TextureField's FourierFeatEnc has no max_freq: the reference's constructor asserts."""
    import model as M
    assert bool(golden("g9_ff_encoder.npz")["ff_strategy_raises"])
    with pytest.raises(AssertionError):
        M.make_model({"feature_strategy": "ff", "k": 4, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2})


@pytest.mark.parametrize("strategy", ["intrinsic", "extrinsic"])
def test_viewdep_model_init_matches_reference(strategy):
    """make_model with view_dependence (model.py:240-256): the reference's module tree and
    seed-0 weights (G11), face normals as a non-persistent buffer."""
    import types

    import model as M
    d = golden(f"g11_viewdep_{strategy}.npz")
    torch.manual_seed(0)
    m = M.make_model({"k": 64, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2,
                      "view_dependence": {"bottleneck_vec_dim": 16, "in_dim_view_dir": 1 if strategy == "intrinsic"
                                          else 3, "include_view_dir": True, "embed_size": 4,
                                          "directional_hidden_dim": 32, "strategy": strategy}},
                     mesh=types.SimpleNamespace(face_normals=d["normals"].astype(np.float64)))
    sd = m.state_dict()
    ref = {k[2:]: d[k] for k in d.files if k.startswith("w:")}
    assert list(sd) == list(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), v, err_msg=k)


def test_config_guard_only_on_rank0(tmp_path):
    """config.load_config_file: the reference's "out_dir exists" guard (config.py:26-36)
    for the leading process; a data-parallel follower rank (train.py --data_parallel,
    RANK > 0) only reads the file -- rank 0 has created out_dir by then."""
    import yaml

    import config
    out = tmp_path / "out"
    path = tmp_path / "c.yaml"
    with open(path, "w") as fh:
        yaml.safe_dump({"training": {"out_dir": str(out)}, "model": {}}, fh)
    c0 = config.load_config_file(str(path))
    assert (out / "config.yaml").exists()
    with pytest.raises(RuntimeError):
        config.load_config_file(str(path))
    c1 = config.load_config_file(str(path), follower=True)
    assert c1 == c0
