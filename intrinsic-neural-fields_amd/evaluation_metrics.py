"""Host mirror of the reference evaluation_metrics.py (evaluation_metrics.py:5-34).

psnr / epoch_psnr keep the reference's host arithmetic on numpy images (the renderer
returns host arrays, eval.py:140-176); given HIP tensors, psnr reduces on the device
(`inf_masked_sse`).  dssim -- scikit-image's structural_similarity in the reference,
absent from this image -- runs as the HIP kernel `inf_ssim` (csrc/metrics.hip) with
skimage's defaults; numpy inputs are copied to the device.
"""
import numpy as np
import torch


def _dev(x):
    t = torch.as_tensor(x)
    if not t.is_cuda:
        if not torch.cuda.is_available():
            raise RuntimeError("dssim runs on the HIP device (csrc/metrics.hip); no GPU is visible. "
                               "There is no CPU fallback.")
        t = t.cuda()
    return t


def psnr(fake_img, real_img, obj_mask_1d=None):
    """Reference evaluation_metrics.py:5-22 (MAX = 1)."""
    assert fake_img.shape == real_img.shape
    if isinstance(fake_img, torch.Tensor) and fake_img.is_cuda:
        from inf_hip import runtime
        mask = None if obj_mask_1d is None else _dev(obj_mask_1d).reshape(-1)
        sse, n = runtime.masked_sse(fake_img, _dev(real_img), mask)
        mse = sse / (3 * n) if n else float("nan")
    else:
        if obj_mask_1d is not None:
            fake_img = fake_img.reshape(-1, 3)[obj_mask_1d]
            real_img = real_img.reshape(-1, 3)[obj_mask_1d]
        mse = np.mean((fake_img - real_img) ** 2)
    if mse == 0:
        return float('inf')
    return 20 * np.log10(1.0 / np.sqrt(mse))


def epoch_psnr(epoch_mse):
    """Reference evaluation_metrics.py:25-26 (callers pass summed squared error / rays)."""
    return -10 * np.log10(epoch_mse)


def dssim(fake_image, real_image):
    """Reference evaluation_metrics.py:29-34: (1 - SSIM) / 2, SSIM as skimage's
    structural_similarity(multichannel=True) (data_range 2 for float images, 255 for
    uint8 ones -- skimage's dtype range)."""
    assert fake_image.shape == real_image.shape and fake_image.shape[2] == 3
    from inf_hip import runtime
    dt = fake_image.dtype
    is_u8 = dt in (np.uint8, torch.uint8)
    ssim = runtime.ssim(_dev(fake_image).to(torch.float32), _dev(real_image).to(torch.float32),
                        data_range=255.0 if is_u8 else 2.0)
    return (1 - ssim) / 2


@torch.no_grad()
def evaluate_view(renderer, camCv2world, K, real_img, obj_mask_1d):
    """eval.py:131-176 for one view without LPIPS (its AlexNet weights are not available
    offline): render, restrict the object mask to the pixels whose rays hit the mesh,
    paint the background white in both images, then psnr over the mask and dssim * 100.
    Returns (metrics, fake_img_raw, fake_img, real_img) as host arrays."""
    H, W = renderer.H, renderer.W
    fake, hit = renderer.render(camCv2world, K, eval_render=True)
    dev = hit.device if hit.is_cuda else torch.device("cuda")
    fake = torch.as_tensor(fake).to(dev, torch.float32)
    real = torch.as_tensor(real_img).to(dev, torch.float32).reshape(H * W, 3).clone()
    hit_mask = torch.zeros(H * W, dtype=torch.bool, device=dev)
    hit_mask[hit.to(dev)] = True
    mask = torch.logical_and(hit_mask, torch.as_tensor(obj_mask_1d).to(dev).reshape(-1).bool())
    fake_raw = fake.reshape(H, W, 3).cpu().numpy().copy()
    fake = fake.reshape(H * W, 3).clone()
    bg = ~mask
    fake[bg] = 1.0
    real[bg] = 1.0
    fake, real = fake.reshape(H, W, 3), real.reshape(H, W, 3)
    metrics = {"psnr": psnr(fake, real, mask), "dssim_rescaled": dssim(fake, real) * 100}
    return metrics, fake_raw, fake.cpu().numpy(), real.cpu().numpy()
