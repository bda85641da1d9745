"""Host mirror of the reference evaluation_metrics.py (evaluation_metrics.py:5-34).

psnr / epoch_psnr are host-side numpy on already-rendered images / summed errors, as
in the reference.  dssim needs scikit-image, which is absent from this image.
"""
import numpy as np


def psnr(fake_img, real_img, obj_mask_1d=None):
    """Reference evaluation_metrics.py:5-22 (MAX = 1)."""
    assert fake_img.shape == real_img.shape
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
    """Reference evaluation_metrics.py:29-34."""
    try:
        from skimage.metrics import structural_similarity
    except ImportError as e:  # pragma: no cover - environment dependent
        raise NotImplementedError("dssim needs scikit-image, which is not installed") from e
    assert fake_image.shape == real_image.shape and fake_image.shape[2] == 3
    return (1 - structural_similarity(fake_image, real_image, multichannel=True)) / 2
