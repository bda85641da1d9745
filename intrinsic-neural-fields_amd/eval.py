"""Host mirror of the reference eval.py (CLI, eval.py:21-193).

    python eval.py <output_path> <config_path> <dataset_path> <split>
                   [--uv_mesh_path OBJ] [--background white]

Per view of the split: the camera rays are cast against the mesh on the device
(csrc/raycast.hip), the hits are shaded by the trained field (gather + MLP, the plan's
render path), the object mask is restricted to the pixels whose rays hit the mesh and the
background of both images is painted white, then PSNR over the mask and DSSIM x 100 are
computed on the device (csrc/metrics.hip) -- evaluation_metrics.evaluate_view.  The
rendered / real images are written as PNGs and the per-view metrics to
evaluation_metrics.pkl, as the reference does.  With --uv_mesh_path the field is first
baked into the UV texture (bake_texture_field.bake_texture, on the device).

LPIPS (eval.py:120, 161) needs AlexNet weights that cannot be fetched offline: it is
reported as None per view and "n/a" in the summary line.
"""
import argparse
import os
import pickle
import random

import numpy as np
import torch


def parse_args(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("output_path", type=str)
    parser.add_argument("config_path", type=str)
    parser.add_argument("dataset_path", type=str)
    parser.add_argument("split", type=str)
    parser.add_argument("--uv_mesh_path", type=str, default=None)
    parser.add_argument("--background", nargs='?', type=str, default="white")
    return parser.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    from bake_texture_field import bake_texture
    from config import get_seed, load_config
    from dataset import MeshroomRadialK3Dataset, MeshViewsDataset
    from evaluation_metrics import evaluate_view
    from mesh import load_first_k_eigenfunctions, load_mesh
    from renderer import Renderer
    from utils import load_trained_model

    if args.uv_mesh_path is not None:
        print("Baking texture into UV-map...")
        bake_texture(args.output_path, args.uv_mesh_path, args.config_path)
        print("Done.")

    config = load_config(args.config_path)
    if not torch.cuda.is_available():
        raise RuntimeError("eval.py renders on the MI355X (HIP) device; no GPU is visible. There is no CPU fallback.")
    device = "cuda"
    seed = get_seed(config)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)

    H, W = config["data"]["img_height"], config["data"]["img_width"]
    dataset_type = config["data"].get("type")
    if dataset_type is None:
        dataset = MeshViewsDataset(args.dataset_path, args.split, H=H, W=W, background=args.background)
    elif dataset_type == "meshroom_radial_k3":
        dataset = MeshroomRadialK3Dataset(args.dataset_path, args.split, H=H, W=W)
    else:
        raise NotImplementedError(f"Unknown dataset type: {dataset_type}")

    mesh = load_mesh(config["data"]["mesh_path"])
    feature_strategy = config["model"].get("feature_strategy", "efuncs")
    if feature_strategy == "efuncs":
        features = load_first_k_eigenfunctions(config["data"]["eigenfunctions_path"], config["model"].get("k"),
                                               rescale_strategy=config["data"].get("rescale_strategy", "standard"),
                                               embed_strategy=config["data"].get("embed_strategy"),
                                               eigenvalues_path=config["data"].get("eigenvalues_path"))
    elif feature_strategy in ("xyz", "ff", "rff"):
        features = None
    else:
        raise ValueError(f"Unknown feature strategy: {feature_strategy}")

    weights_path = os.path.join(config["training"]["out_dir"], "model.pt")
    model = load_trained_model(config["model"], weights_path, device, mesh=mesh).eval()
    os.makedirs(args.output_path, exist_ok=True)
    if feature_strategy == "efuncs":
        renderer = Renderer(model, mesh, eigenfunctions=features, feature_strategy=feature_strategy, H=H, W=W,
                            device=device)
    else:
        renderer = Renderer(model, mesh, feature_strategy=feature_strategy, H=H, W=W, device=device)

    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    results = {}
    total_psnr = total_dssim = 0.0
    total = 0
    with torch.no_grad():
        for i in range(len(dataset)):
            item = dataset[i]
            view_id = f"{i:03d}"
            if item.get("distortion_type") is not None:
                raise NotImplementedError("lens undistortion (meshroom_radial_k3 views) is outside this build's scope")
            metrics, fake_raw, fake, real = evaluate_view(renderer, item["camCv2world"], item["K"], item["img"],
                                                          item["obj_mask_1d"])
            metrics["lpips_rescaled"] = None  # LPIPS: AlexNet weights unavailable offline
            total_psnr += metrics["psnr"]
            total_dssim += metrics["dssim_rescaled"]
            total += 1
            results[view_id] = metrics
            plt.imsave(os.path.join(args.output_path, f"{view_id}_fake_raw.png"), np.clip(fake_raw, 0, 1))
            plt.imsave(os.path.join(args.output_path, f"{view_id}_fake.png"), np.clip(fake, 0, 1))
            plt.imsave(os.path.join(args.output_path, f"{view_id}_real.png"), np.clip(real, 0, 1))

    with open(os.path.join(args.output_path, "evaluation_metrics.pkl"), "wb") as f:
        pickle.dump(results, f)
    n = max(total, 1)
    print(f"PSNR: {total_psnr / n}, DSSIM: {total_dssim / n}, LPIPS: n/a (weights unavailable offline)")
    return results


if __name__ == "__main__":
    main()
