"""Host mirror of the reference ray_dataloader.py.

`RayDataLoader` (reference ray_dataloader.py:57-145) keeps the same constructor,
`len()`/iteration protocol, shuffling (`torch.randperm` on the device once per epoch,
:103-107), batch slicing (:109-113) and drop_last semantics (:88-95).  The arrays live
on the HIP device (:73-83).  Each batch is a `RayBatch`: a dict whose values are
computed on first access -- "eigenfunctions" by the HIP gather (mesh.py:313-324 fused
with the loader's index-select :122-129), or for the xyz/ff/rff strategies "xyz" by the
same gather over the V x 3 vertex positions (:134-136), "expected_rgbs" etc. by
index-select -- so a
consumer that reads `batch["eigenfunctions"]` sees exactly the reference's tensor, while
TextureField / Trainer hand the ray indices straight to the fused kernels and never
materialise the B x k feature matrix.
"""
from __future__ import annotations

import torch

from dataset import load_preprocessed_data
from mesh import load_first_k_eigenfunctions


def create_ray_dataloader(preproc_data_path, eigenfunctions_path, k, feature_strategy, mesh, rescale_strategy,
                          eigenvalues_path, embed_strategy, batch_size, shuffle, drop_last, device="cuda"):
    """Reference ray_dataloader.py:7-54."""
    if feature_strategy == "efuncs":
        features = load_first_k_eigenfunctions(eigenfunctions_path, k, rescale_strategy=rescale_strategy,
                                               embed_strategy=embed_strategy, eigenvalues_path=eigenvalues_path)
    elif feature_strategy in ("ff", "rff", "xyz"):
        # ray_dataloader.py:28-30: the vertex positions; the loader interpolates hit points
        features = torch.as_tensor(mesh.vertices).to(dtype=torch.float32)
    else:
        raise ValueError(f"Unknown input feature strategy: {feature_strategy}")
    data = load_preprocessed_data(preproc_data_path)
    return RayDataLoader(features, feature_strategy, data["vertex_idxs_of_hit_faces"], data["barycentric_coords"],
                         data["expected_rgbs"], data.get("unit_ray_dirs"), data.get("face_idxs"), batch_size, shuffle,
                         drop_last, device=device)


class RayBatch(dict):
    """A batch dict with lazily computed values (see module docstring)."""

    def __init__(self, loader: "RayDataLoader", idxs: torch.Tensor, offset: int, count: int):
        super().__init__()
        self._loader = loader
        self._perm = idxs          # the loader's index vector (identity or permutation)
        self._offset = offset
        self._count = count
        self._feat_key = "eigenfunctions" if loader.feature_strategy == "efuncs" else "xyz"
        self._keys = ["expected_rgbs", self._feat_key]
        if loader.unit_ray_dirs is not None:
            self._keys += ["unit_ray_dirs", "hit_face_idxs"]

    # ---- lazy dict protocol ----
    def _rows(self):
        return self._perm[self._offset:self._offset + self._count]

    def _compute(self, key):
        ld = self._loader
        if key == "xyz":  # ray_dataloader.py:134-136, the same barycentric sum over the V x 3 positions
            from inf_hip import runtime
            return runtime.gather(ld.features, ld.source.vids32, ld.source.bary, ray_idx=self._perm,
                                  offset=self._offset, batch=self._count)
        if key == "eigenfunctions":
            from inf_hip import runtime
            v = runtime.gather(ld.features, ld.source.vids32, ld.source.bary, ray_idx=self._perm, offset=self._offset,
                               batch=self._count)
            assert v.dtype == torch.float32
            return v
        rows = self._rows()
        if key == "expected_rgbs":
            return ld.expected_rgbs[rows]
        if key == "unit_ray_dirs":
            return ld.unit_ray_dirs[rows]
        if key == "hit_face_idxs":
            return ld.face_idxs[rows]
        raise KeyError(key)

    def __getitem__(self, key):
        if not dict.__contains__(self, key):
            if key not in self._keys:
                raise KeyError(key)
            dict.__setitem__(self, key, self._compute(key))
        return dict.__getitem__(self, key)

    def get(self, key, default=None):
        return self[key] if key in self else default

    def __contains__(self, key):
        return key in self._keys or dict.__contains__(self, key)

    def keys(self):
        return list(dict.fromkeys(self._keys + list(dict.keys(self))))

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self.keys())

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]

    # ---- fused-path hooks ----
    def is_lazy_rays(self):
        return not dict.__contains__(self, self._feat_key)

    def ray_args(self):
        return {"source": self._loader.source, "ray_idx": self._perm, "offset": self._offset, "batch": self._count,
                "extrinsic": self._feat_key == "xyz"}

    @property
    def batch_size(self):
        return self._count

    def to(self, device):
        return self


class RayDataLoader:
    """Reference ray_dataloader.py:57-145 (device-resident, shuffled by randperm)."""

    def __init__(self, features, feature_strategy, vertex_idxs_of_hit_faces, barycentric_coords, expected_rgbs,
                 unit_ray_dirs, face_idxs, batch_size, shuffle, drop_last, device="cuda"):
        if feature_strategy not in ("efuncs", "ff", "rff", "xyz"):
            raise ValueError(f"Unknown input feature strategy: {feature_strategy}")
        self.device = device
        self.features = features.to(self.device).to(torch.float32).contiguous()
        self.feature_strategy = feature_strategy
        self.vertex_idxs_of_hit_faces = vertex_idxs_of_hit_faces.to(self.device)
        self.barycentric_coords = barycentric_coords.to(self.device)
        self.expected_rgbs = expected_rgbs.to(self.device)
        self.unit_ray_dirs = unit_ray_dirs
        self.face_idxs = face_idxs
        if self.unit_ray_dirs is not None:
            assert self.face_idxs is not None
            self.unit_ray_dirs = self.unit_ray_dirs.to(self.device)
            self.face_idxs = self.face_idxs.to(self.device)

        from inf_hip import runtime
        self.source = runtime.RaySource(self.features, self.vertex_idxs_of_hit_faces, self.barycentric_coords,
                                        self.expected_rgbs)

        self.shuffle = shuffle
        self.drop_last = drop_last
        self.B = batch_size
        self.N = self.vertex_idxs_of_hit_faces.shape[0]
        if self.drop_last:
            self.num_batches = self.N // self.B
        else:
            self.num_batches = (self.N + self.B - 1) // self.B
        self.i = 0
        self.idxs = torch.arange(self.N, device=self.device)

    def __len__(self):
        return self.num_batches

    def __iter__(self):
        if self.shuffle:
            self.idxs = torch.randperm(self.N, device=self.device)
        self.i = 0
        return self

    def _get_next_batch_span(self):
        low = self.i * self.B
        high = min((self.i + 1) * self.B, self.N)
        self.i += 1
        return low, high

    def __next__(self):
        if self.i >= self.num_batches:
            raise StopIteration
        low, high = self._get_next_batch_span()
        return RayBatch(self, self.idxs, low, high - low)
