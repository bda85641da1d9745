"""Host mirror of the reference renderer.py.

The MLP slice of `Renderer.render` (reference renderer.py:112-146: batched inference
over the hit rays, then placement of each colour into a white/black image, then the
un-masking to H x W) runs on the HIP device in `render_hits`: gather + forward + scatter
in one launch sequence per 2^18-ray chunk (csrc/plan.hip inf_render), with the table
resident on the device instead of the reference's host-side M x k feature buffer.

Ray casting (reference renderer.py:71-81 -> mesh.ray_tracing, trimesh/embree) runs on
the GPU too (csrc/raycast.hip): given a mesh, `render()` casts
the view's camera rays against a device BVH and hands the hit lists to `render_hits`
without leaving the device.  A `ray_tracer` callable returning (vids, bary,
hit_ray_idxs) overrides it.
"""
from __future__ import annotations

import os

import torch

from mesh import load_first_k_eigenfunctions
from utils import load_trained_model

RENDER_CHUNK = 1 << 18
PROJECTED_CHUNK = 1 << 30


def make_renderer_with_trained_model(config, device="cuda"):
    """Reference renderer.py:9-32."""
    from mesh import load_mesh
    mesh = load_mesh(config["data"]["mesh_path"])
    efuncs = load_first_k_eigenfunctions(config["data"]["eigenfunctions_path"], config["model"].get("k"),
                                         rescale_strategy=config["data"].get("rescale_strategy", "standard"),
                                         embed_strategy=config["data"].get("embed_strategy"),
                                         eigenvalues_path=config["data"].get("eigenvalues_path"))
    weights_path = os.path.join(config["training"]["out_dir"], "model.pt")
    model = load_trained_model(config["model"], weights_path, device, mesh=None)
    return Renderer(model, mesh, eigenfunctions=efuncs, device=device, H=config["data"]["img_height"],
                    W=config["data"]["img_width"])


def _project_enabled(num_hits, num_vertices):
    """INF_RENDER_PROJECT=1 / 0 forces the projected-table render on / off; by default it
    runs when the frame has at least half as many hits as the table has vertices (the
    projection GEMM costs about what the per-hit input layers save at one hit per vertex)."""
    env = os.environ.get("INF_RENDER_PROJECT")
    if env is not None:
        return env != "0"
    return 2 * num_hits >= num_vertices


def _to_host(img):
    """Device image -> host tensor through page-locked memory (PyTorch's caching host
    allocator): the 2048^2 x 3 fp32 frame is ~50 MB, several times faster to copy than
    into pageable memory."""
    out = torch.empty(img.shape, dtype=img.dtype, pin_memory=True)
    out.copy_(img)
    return out


class Renderer:
    """Reference renderer.py:35-146."""

    def __init__(self, model, mesh, eigenfunctions=None, feature_strategy="efuncs", background="white", device="cpu",
                 *, H, W, ray_tracer=None):
        self.model = model
        self.mesh = mesh
        self.feature_strategy = feature_strategy
        if feature_strategy == "efuncs":
            self.features = eigenfunctions
        elif feature_strategy in ("ff", "rff", "xyz"):  # renderer.py:44-45: the vertex positions
            self.features = torch.as_tensor(mesh.vertices).to(dtype=torch.float32)
        else:
            raise ValueError(f"Unknown feature strategy: {feature_strategy}")
        self.H = H
        self.W = W
        self.background = background
        self.device = device
        self.ray_tracer = ray_tracer
        self.ray_mesh_intersector = None
        if ray_tracer is None and mesh is not None:
            from mesh import get_ray_mesh_intersector
            self.ray_mesh_intersector = get_ray_mesh_intersector(mesh)
        self._dev_features = None
        self._table_cache = {}

    def apply_mesh_transform(self, transform):
        """Reference renderer.py:62-64: transform the vertices, rebuild the intersector."""
        import numpy as np
        from mesh import get_ray_mesh_intersector
        T = np.asarray(transform, dtype=np.float64)
        v = np.concatenate([self.mesh.vertices, np.ones((self.mesh.vertices.shape[0], 1))], 1) @ T.T
        self.mesh.vertices = v[:, :3] / v[:, 3:4]
        self.ray_mesh_intersector = get_ray_mesh_intersector(self.mesh)

    def set_height(self, height):
        self.H = height

    def set_width(self, width):
        self.W = width

    def _features_on_device(self, device):
        # "cuda" (no index) names the current device: compare resolved devices, or the
        # table would be uploaded (and re-packed) on every frame
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        if self._dev_features is None or self._dev_features.device != device:
            self._dev_features = self.features.to(device=device, dtype=torch.float32).contiguous()
        return self._dev_features

    @torch.no_grad()
    def _render_generic(self, vids, bary, hit, face, unit_dirs, obj_mask_1d):
        """renderer.py:86-146 for models outside the fused plan (the view-dependent field):
        features of the hits, model(batch) over chunks (renderer.py:104-110), placement."""
        from inf_hip import runtime
        dev = vids.device
        feats = runtime.gather(self._features_on_device(dev), vids.contiguous(), bary.to(torch.float32).contiguous())
        key = "eigenfunctions" if self.feature_strategy == "efuncs" else "xyz"
        fill = 1.0 if self.background == "white" else 0.0
        img = torch.full((self.H * self.W, 3), fill, dtype=torch.float32, device=dev)
        preds = [self.model({key: feats[lo:lo + RENDER_CHUNK], "unit_ray_dirs": unit_dirs[lo:lo + RENDER_CHUNK],
                             "hit_face_idxs": face[lo:lo + RENDER_CHUNK]})
                 for lo in range(0, feats.shape[0], RENDER_CHUNK)]
        if preds:
            pix = hit if obj_mask_1d is None else torch.nonzero(torch.as_tensor(obj_mask_1d).to(dev)).reshape(-1)[hit]
            img[pix] = torch.cat(preds)
        return img.reshape(self.H, self.W, 3)

    @torch.no_grad()
    def render_hits(self, vertex_idxs_of_hit_faces, barycentric_coords, hit_ray_idxs, obj_mask_1d=None,
                    return_tensor=False):
        """Colours of precomputed hits placed into an H x W x 3 image (renderer.py:112-146)."""
        from inf_hip import runtime
        assert obj_mask_1d is None or obj_mask_1d.size()[0] == self.H * self.W
        self.model.eval()
        dev = torch.device(self.device) if not isinstance(self.device, torch.device) else self.device
        if dev.type != "cuda":
            raise RuntimeError("Renderer.render_hits runs on the HIP device; construct it with device='cuda'")
        E = self._features_on_device(dev)
        vids = vertex_idxs_of_hit_faces.to(dev)
        bary = barycentric_coords.to(dev, torch.float32)
        hit = hit_ray_idxs.to(dev, torch.int64).contiguous()
        num_rays = hit.shape[0]
        M = self.H * self.W
        fill = 1.0 if self.background == "white" else 0.0
        assert self.background in ("white", "black")
        img = torch.full((M, 3), fill, dtype=torch.float32, device=dev)
        if num_rays == 0:  # nothing hit: the reference's empty model call leaves the background
            img = img.reshape(self.H, self.W, 3)
            return img if return_tensor else img.cpu().numpy()
        pixel_map = None
        if obj_mask_1d is not None:
            assert obj_mask_1d.dtype == torch.bool
            pixel_map = torch.nonzero(obj_mask_1d.to(dev)).reshape(-1)
        # hit lists from the device caster are valid by construction; the packed GEMM-dtype
        # table is kept across calls (it depends only on the features and the plan)
        src = runtime.RaySource(E, vids, bary, None, validate=False)
        if self._table_cache.get("E") is not E:
            self._table_cache = {"E": E, "tables": {}}
        src._tables = self._table_cache["tables"]
        chunk = min(RENDER_CHUNK, num_rays)
        plan = self.model.hip_plan(chunk)
        # enough hits per vertex: interpolate the vertices' first-layer projections instead
        # of their features (inf_project_table).  The projected table is kept for the next
        # frame while the plan's weight generation is unchanged (several views of one
        # trained model: eval.py); recomputed whenever an update may have moved the weights
        proj = None
        if plan.can_project() and _project_enabled(num_rays, E.shape[0]):
            T = src.table_for(plan)
            gen = plan.weight_generation()
            pc = self._table_cache.get("proj")
            if pc is not None and gen >= 0 and pc[0] is plan and pc[1] == gen and pc[2] is T:
                proj = pc[3]
            else:
                proj = plan.project_table(T)
                self._table_cache["proj"] = (plan, gen, T, proj) if gen >= 0 else None
            chunk = min(num_rays, PROJECTED_CHUNK)  # no workspace: the frame in one persistent launch
        for low in range(0, num_rays, chunk):
            n = min(chunk, num_rays - low)
            b = plan.make_batch(source=src, offset=low, batch=n, projected=proj)
            plan.render(b, hit[low:low + n], pixel_map, img)
        self.model._rt.saved_gen = None
        img = img.reshape(self.H, self.W, 3)
        return img if return_tensor else _to_host(img).numpy()

    @torch.no_grad()
    def render(self, camCv2world, K, obj_mask_1d=None, eval_render=False, distortion_coeffs=None,
               distortion_type=None):
        """Reference renderer.py:64-146: camera rays cast on the device (or `self.ray_tracer`)."""
        img, hit_ray_idxs = self._render(camCv2world, K, obj_mask_1d, distortion_coeffs, distortion_type)
        if eval_render:
            return _to_host(img), hit_ray_idxs
        return _to_host(img).numpy()

    @torch.no_grad()
    def render_device(self, camCv2world, K, obj_mask_1d=None):
        """render() without the host read-back: the H x W x 3 image on the device."""
        return self._render(camCv2world, K, obj_mask_1d, None, None)[0]

    def _render(self, camCv2world, K, obj_mask_1d, distortion_coeffs, distortion_type):
        if not hasattr(self.model, "hip_plan"):  # view-dependent field: model(batch) per chunk
            if distortion_type is not None:
                raise NotImplementedError("lens undistortion (mesh.py:186-193) is outside this build's scope")
            from mesh import cast_camera_rays
            vids, bary, hit, face, dirs = cast_camera_rays(self.ray_mesh_intersector, camCv2world, K, obj_mask_1d,
                                                           H=self.H, W=self.W)
            return self._render_generic(vids, bary, hit, face, dirs[hit], obj_mask_1d), hit
        if self.ray_tracer is not None:
            vids, bary, hit_ray_idxs = self.ray_tracer(camCv2world, K, obj_mask_1d=obj_mask_1d, H=self.H, W=self.W,
                                                       distortion_coeffs=distortion_coeffs,
                                                       distortion_type=distortion_type)
        elif self.ray_mesh_intersector is not None:
            if distortion_type is not None:
                raise NotImplementedError("lens undistortion (mesh.py:186-193) is outside this build's scope")
            from mesh import cast_camera_rays
            vids, bary, hit_ray_idxs, _, _ = cast_camera_rays(self.ray_mesh_intersector, camCv2world, K, obj_mask_1d,
                                                              H=self.H, W=self.W)
        else:
            raise ValueError("Renderer.render needs a mesh (or a ray_tracer); render_hits takes precomputed hits")
        img = self.render_hits(vids, bary, hit_ray_idxs, obj_mask_1d, return_tensor=True)
        return img, hit_ray_idxs
