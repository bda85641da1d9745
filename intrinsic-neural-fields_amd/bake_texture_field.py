"""Host mirror of the reference bake_texture_field.py: bake a trained texture field into
the UV texture of a mesh, on the device.

Reference pipeline (bake_texture_field.py:334-420): per-vertex correspondence of the UV
mesh (vertices split per (v, vt) pair) to the eigenfunction mesh; texel -> UV triangle
search + barycentrics (:96-228); MLP colours of the texels' surface points (pred_rgbs
:267-319); hole filling (:245-264); 8-bit texture written under <out_dir>/baked/.

Here the texel search, barycentrics, compaction, feature gather / encoding + MLP
(the plan's render path) and hole filling run as HIP kernels (csrc/bake.hip,
csrc/raycast.hip, the plan).  The z-value colour-map debug texture (:372-398, viridis)
is not produced.  Texture files are read / written with PIL.
"""
from __future__ import annotations

import os
import shutil
from types import SimpleNamespace

import numpy as np
import torch

MIN_UV_AREA = 1e-4  # clean_tris (bake_texture_field.py:96)


def _no_tracer(*args, **kwargs):
    raise RuntimeError("baking renders precomputed texel hits only")


class UVMesh:
    """An OBJ with texture coordinates as trimesh loads it for baking: one vertex per
    distinct (position, uv) corner, faces over those, uv per vertex, and the material's
    diffuse map (map_Kd)."""

    def __init__(self, vertices, faces, uv, position_index, texture_path=None):
        self.vertices = vertices
        self.faces = faces
        self.uv = uv
        self.position_index = position_index  # the OBJ 'v' row of each split vertex
        self.texture_path = texture_path


def load_uv_mesh(path) -> UVMesh:
    pos, tex, faces = [], [], []
    corner_ids: dict = {}
    corners = []
    mtl = None
    with open(path) as fh:
        for line in fh:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                pos.append([float(x) for x in p[1:4]])
            elif p[0] == "vt":
                tex.append([float(x) for x in p[1:3]])
            elif p[0] == "mtllib":
                mtl = line.split(None, 1)[1].strip()
            elif p[0] == "f":
                ids = []
                for tok in p[1:]:
                    t = tok.split("/")
                    vi = int(t[0])
                    vi = vi - 1 if vi > 0 else len(pos) + vi
                    if len(t) < 2 or not t[1]:
                        raise ValueError(f"{path}: face corner '{tok}' has no texture coordinate")
                    ti = int(t[1])
                    ti = ti - 1 if ti > 0 else len(tex) + ti
                    key = (vi, ti)
                    if key not in corner_ids:
                        corner_ids[key] = len(corners)
                        corners.append(key)
                    ids.append(corner_ids[key])
                for j in range(1, len(ids) - 1):
                    faces.append([ids[0], ids[j], ids[j + 1]])
    pos = np.asarray(pos, dtype=np.float64)
    tex = np.asarray(tex, dtype=np.float64)
    c = np.asarray(corners, dtype=np.int64).reshape(-1, 2)
    texture = None
    mtl_path = os.path.join(os.path.dirname(path), mtl) if mtl is not None else path + ".mtl"
    if os.path.exists(mtl_path):
        texture = os.path.join(os.path.dirname(path), get_diffuse_color_map_file_name(path, mtl_path))
    return UVMesh(pos[c[:, 0]], np.asarray(faces, dtype=np.int64), tex[c[:, 1]], c[:, 0], texture)


def get_diffuse_color_map_file_name(uv_mesh_path, mtl_file_path=None):
    """Reference bake_texture_field.py:322-331 (the map_Kd entry of <mesh>.mtl)."""
    mtl_file_path = mtl_file_path or uv_mesh_path + ".mtl"
    with open(mtl_file_path) as fh:
        lines = [ln for ln in fh.readlines() if ln.startswith("map_Kd")]
    if len(lines) != 1:
        raise ValueError(f".mtl File {mtl_file_path} is missing 'map_Kd'")
    return os.path.basename(lines[0].split()[1].strip())


def correspondences(uv_mesh: UVMesh, ef_vertices) -> np.ndarray:
    """bake_texture_field.py:349-352: the eigenfunction-mesh vertex at the same position as
    each UV-mesh vertex (the reference's cKDTree query, asserted exact)."""
    ef = np.asarray(ef_vertices, dtype=np.float64)
    lut = {tuple(v): i for i, v in enumerate(ef)}
    try:
        return np.array([lut[tuple(v)] for v in uv_mesh.vertices], dtype=np.int64)
    except KeyError:
        raise ValueError("UV mesh vertex without an identical eigenfunction-mesh vertex") from None


def texel_hits(uv_mesh: UVMesh, H: int, W: int, device="cuda"):
    """Texel search + barycentrics (bake_texture_field.py:355-369): (texel_face [H*W],
    texel_bary [H*W, 3]) on the device; face -1 = no triangle."""
    from inf_hip import runtime
    pu = (W - 1) * uv_mesh.uv[:, 0]
    pv = (H - 1) * (1 - uv_mesh.uv[:, 1])
    uv_px = torch.from_numpy(np.stack([pu, pv], -1)).to(device)
    return runtime.uv_raster(uv_px, torch.from_numpy(uv_mesh.faces).to(device), H, W, MIN_UV_AREA)


@torch.no_grad()
def bake_texture_image(model, features, uv_mesh: UVMesh, idx_uv_to_ef, H: int, W: int, feature_strategy="efuncs"):
    """The baked texture (H x W x 3 uint8, and the filled fp32 texture) of a trained
    TextureField: pred_rgbs (:267-319) over the covered texels, then uv_fill_holes and
    (255 * CC).astype(uint8) (:406-416)."""
    from inf_hip import runtime
    from renderer import Renderer
    dev = torch.device("cuda")
    tf, tb = texel_hits(uv_mesh, H, W, device=dev)
    faces_ef = torch.from_numpy(np.asarray(idx_uv_to_ef)[uv_mesh.faces]).to(dev)
    vids, bary, texel, _ = runtime.compact_faces(faces_ef, tf, tb)
    if feature_strategy == "efuncs":
        r = Renderer(model, None, eigenfunctions=features, background="black", device=dev, H=H, W=W,
                     ray_tracer=_no_tracer)
    else:  # the xyz front-ends read the eigenfunction mesh's positions
        r = Renderer(model, SimpleNamespace(vertices=np.asarray(features)), feature_strategy=feature_strategy,
                     background="black", device=dev, H=H, W=W, ray_tracer=_no_tracer)
    img = r.render_hits(vids, bary, texel, return_tensor=True)
    u8, filled = runtime.uv_fill_holes(img)
    return u8, filled


def bake_texture(out_dir, uv_mesh_path, config_path):
    """Reference bake_texture_field.py:334-420 (without the colour-map debug texture)."""
    from PIL import Image

    from config import load_config
    from mesh import load_first_k_eigenfunctions, load_mesh
    from utils import load_trained_model
    assert not os.path.exists(out_dir)
    os.makedirs(out_dir)
    config = load_config(config_path)
    m = load_uv_mesh(uv_mesh_path)
    m_efs = load_mesh(config["data"]["mesh_path"])
    assert m_efs.faces.shape == m.faces.shape
    idx_uv_to_ef = correspondences(m, m_efs.vertices)
    if m.texture_path is None:
        raise ValueError(f"{uv_mesh_path}: no material texture (map_Kd) to size the bake")
    with Image.open(m.texture_path) as im:
        W, H = im.size
    if config["model"].get("view_dependence") is not None:
        raise NotImplementedError("Currently view dependence is not supported.")
    feature_strategy = config["model"].get("feature_strategy", "efuncs")
    if feature_strategy == "efuncs":
        features = load_first_k_eigenfunctions(config["data"]["eigenfunctions_path"], config["model"].get("k"),
                                               rescale_strategy=config["data"].get("rescale_strategy", "standard"),
                                               embed_strategy=config["data"].get("embed_strategy"),
                                               eigenvalues_path=config["data"].get("eigenvalues_path"))
    elif feature_strategy in ("xyz", "ff", "rff"):
        features = torch.from_numpy(np.asarray(m_efs.vertices)).to(torch.float32)
    else:
        raise ValueError(f"Unknown feature strategy: {feature_strategy}")
    model = load_trained_model(config["model"], os.path.join(config["training"]["out_dir"], "model.pt"), "cuda",
                               mesh=m_efs).eval()
    u8, _ = bake_texture_image(model, features, m, idx_uv_to_ef, H, W, feature_strategy)
    baked = os.path.join(out_dir, "baked")
    os.makedirs(baked, exist_ok=False)
    shutil.copyfile(uv_mesh_path, os.path.join(baked, os.path.basename(uv_mesh_path)))
    if os.path.exists(uv_mesh_path + ".mtl"):
        shutil.copyfile(uv_mesh_path + ".mtl", os.path.join(baked, os.path.basename(uv_mesh_path) + ".mtl"))
    Image.fromarray(u8.cpu().numpy()).save(os.path.join(baked, os.path.basename(m.texture_path)))
    return u8
