"""A synthetic texture-reconstruction dataset in the reference's on-disk layout (test
infrastructure): the cat config's paths (configs/texture_reconstruction/intrinsic_cat.yaml
schema) filled with a torus instead of the cat, which is not available offline.

    data/cat_rescaled_rotated/12221_Cat_v1_l3.obj          mesh (positions)
    data/cat_tri/12221_Cat_v1_l3.obj (+ .mtl, texture.png)  UV mesh for baking
    data/preprocessed/cat_efuncs/eigenfunctions_*.npy        V x kmax table
    data/cat_dataset_v2_tiny/<view>/{depth/cameras.npz, depth/mask.png, image/000.png}
    data/cat_dataset_v2_tiny/{train,val,test}.lst
    data/preprocessed/cat_dataset_v2_tiny/{train,val}/*.npy (MeshViewPreProcessor)

Views are cast against the mesh on the device (csrc/raycast.hip) and coloured by a smooth
function of the hit position, so the field has something to learn.
"""
import os

import numpy as np
import torch

EFUNCS = "data/preprocessed/cat_efuncs/eigenfunctions_cotan_kmax4096_skip_first_efuncs.npy"
MESH = "data/cat_rescaled_rotated/12221_Cat_v1_l3.obj"
UV_MESH = "data/cat_tri/12221_Cat_v1_l3.obj"
DATASET = "data/cat_dataset_v2_tiny"
PREPROC = "data/preprocessed/cat_dataset_v2_tiny"


def torus(nu=48, nv=24, R=1.0, r=0.4):
    u = np.arange(nu) * 2 * np.pi / nu
    v = np.arange(nv) * 2 * np.pi / nv
    uu, vv = np.meshgrid(u, v, indexing="ij")
    V = np.stack([(R + r * np.cos(vv)) * np.cos(uu), (R + r * np.cos(vv)) * np.sin(uu), r * np.sin(vv)], -1)
    i, j = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    a, b = i * nv + j, ((i + 1) % nu) * nv + j
    c, d = ((i + 1) % nu) * nv + (j + 1) % nv, i * nv + (j + 1) % nv
    F = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    # UV grid with seam copies: corner (i, j) of a face -> vt row i' (nv + 1) + j'
    ti = np.stack([i, i + 1, i + 1], -1).reshape(-1, 3), np.stack([i, i + 1, i], -1).reshape(-1, 3)
    tj = np.stack([j, j, j + 1], -1).reshape(-1, 3), np.stack([j, j + 1, j + 1], -1).reshape(-1, 3)
    FT = np.concatenate([ti[0] * (nv + 1) + tj[0], ti[1] * (nv + 1) + tj[1]])
    gu, gv = np.meshgrid(np.arange(nu + 1) / nu, np.arange(nv + 1) / nv, indexing="ij")
    VT = np.stack([0.02 + 0.96 * gu, 0.02 + 0.96 * gv], -1).reshape(-1, 2)
    return V.reshape(-1, 3), F, VT, FT


def colour(p):
    return np.stack([0.5 + 0.45 * np.sin(4 * p[:, 0]), 0.5 + 0.45 * np.cos(3 * p[:, 1]),
                     0.5 + 0.45 * np.sin(5 * p[:, 2] + p[:, 0])], -1)


def look_at(eye, target=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0)):
    """OpenCV camera -> world (x right, y down, z forward), 4 x 4."""
    eye, target, up = (np.asarray(x, dtype=np.float64) for x in (eye, target, up))
    f = target - eye
    f /= np.linalg.norm(f)
    rgt = np.cross(f, up)
    rgt /= np.linalg.norm(rgt)
    down = np.cross(f, rgt)
    M = np.eye(4)
    M[:3, 0], M[:3, 1], M[:3, 2], M[:3, 3] = rgt, down, f, eye
    return M


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write(text)


def build(root, H=64, W=64, kmax=64, views=(6, 2, 2), seed=0):
    """Writes the dataset under `root`; returns {split: [view dirs]} (relative paths)."""
    from PIL import Image
    from inf_hip import runtime

    rng = np.random.default_rng(seed)
    V, F, VT, FT = torus()
    fmt = "v {:.6f} {:.6f} {:.6f}\n"
    vtxt = "".join(fmt.format(*p) for p in V)
    _write(os.path.join(root, MESH), vtxt + "".join(f"f {a + 1} {b + 1} {c + 1}\n" for a, b, c in F))
    _write(os.path.join(root, UV_MESH), "mtllib 12221_Cat_v1_l3.obj.mtl\n" + vtxt +
           "".join(f"vt {u:.6f} {v:.6f}\n" for u, v in VT) +
           "".join(f"f {a + 1}/{ta + 1} {b + 1}/{tb + 1} {c + 1}/{tc + 1}\n"
                   for (a, b, c), (ta, tb, tc) in zip(F, FT)))
    _write(os.path.join(root, UV_MESH + ".mtl"), "newmtl m\nmap_Kd texture.png\n")
    Image.fromarray(np.full((48, 48, 3), 128, np.uint8)).save(os.path.join(root, "data/cat_tri/texture.png"))
    V32 = np.asarray(np.loadtxt(os.path.join(root, MESH), usecols=(1, 2, 3), max_rows=len(V)), np.float64)
    # a smooth table: low-frequency functions of the vertex positions plus a little noise
    freq = rng.standard_normal((3, kmax)) * 1.5
    E = np.cos(V32 @ freq + rng.random(kmax) * 6.28) + 0.05 * rng.standard_normal((len(V), kmax))
    os.makedirs(os.path.dirname(os.path.join(root, EFUNCS)), exist_ok=True)
    np.save(os.path.join(root, EFUNCS), E.astype(np.float32))

    bvh = runtime.Bvh(V32, F)
    K = np.array([[W * 1.1, 0, W / 2], [0, H * 1.1, H / 2], [0, 0, 1]], np.float32)
    out = {}
    n = 0
    for split, count in zip(("train", "val", "test"), views):
        out[split] = []
        for _ in range(count):
            az, el = 2 * np.pi * n / sum(views) + 0.3, 0.6 + 0.3 * np.sin(n)
            n += 1
            eye = 3.0 * np.array([np.cos(az) * np.cos(el), np.sin(az) * np.cos(el), np.sin(el)])
            cam = look_at(eye).astype(np.float32)
            face, bary, _ = bvh.cast(torch.from_numpy(cam), torch.from_numpy(K), H, W)
            face, bary = face.cpu().numpy(), bary.cpu().numpy()
            mask = face >= 0
            img = np.ones((H * W, 3), np.float64)
            p = (V32[F[face[mask]]] * bary[mask][..., None]).sum(1)
            img[mask] = colour(p)
            name = f"cat_{split}{len(out[split]):03d}"
            view = os.path.join(root, DATASET, name)
            os.makedirs(os.path.join(view, "depth"), exist_ok=True)
            os.makedirs(os.path.join(view, "image"), exist_ok=True)
            np.savez(os.path.join(view, "depth", "cameras.npz"), world_mat_0=cam, camera_mat_0=K)
            Image.fromarray((mask.reshape(H, W) * 255).astype(np.uint8)).save(os.path.join(view, "depth", "mask.png"))
            Image.fromarray(np.round(img.reshape(H, W, 3) * 255).astype(np.uint8)).save(
                os.path.join(view, "image", "000.png"))
            out[split].append(os.path.join(DATASET, name))
        _write(os.path.join(root, DATASET, f"{split}.lst"), "".join(os.path.basename(v) + "\n" for v in out[split]))

    import mesh as MS
    from utils import imread, load_cameras, load_obj_mask_as_tensor
    m = MS.load_mesh(os.path.join(root, MESH))
    for split in ("train", "val"):
        pre = MS.MeshViewPreProcessor(None, os.path.join(root, PREPROC, split), mesh=m)
        for v in out[split]:
            view = os.path.join(root, v)
            cam, K_ = load_cameras(view)
            mask = load_obj_mask_as_tensor(view)
            img = imread(os.path.join(view, "image", "000.png"))[..., :3].astype(np.float32) / 255.
            pre.cache_single_view(cam, K_, mask, torch.from_numpy(img))
        pre.write_to_disk()
    return out


def intrinsic_config(k=32, epochs=4, batch=1024, H=64, W=64, eval_views=()):
    """The intrinsic_cat.yaml schema (reference configs/texture_reconstruction) at test size."""
    return {"seed": 0,
            "data": {"preproc_data_path_train": f"{PREPROC}/train", "preproc_data_path_eval": f"{PREPROC}/val",
                     "preproc_data_path_test": f"{PREPROC}/test", "eigenfunctions_path": EFUNCS,
                     "mesh_path": MESH, "img_height": H, "img_width": W,
                     "eval_render_input_paths": list(eval_views),
                     "eval_render_img_names": [os.path.basename(v) for v in eval_views]},
            "model": {"k": list(range(0, k // 2)) + list(range(40, 40 + k // 2)), "num_layers": 6,
                      "mlp_hidden_dim": 128, "skip_layer_idx": 3, "batchnorm": False},
            "training": {"out_dir": "out/texture_recon/intrinsic_cat", "batch_size": batch, "lr": 0.001,
                         "loss_type": "L1", "render_every": 2, "print_every": 1, "epochs": epochs,
                         "checkpoint_every": 25}}
