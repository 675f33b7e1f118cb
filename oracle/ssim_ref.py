"""ORACLE -- test infrastructure only: the SSIM residual of the LM step.

A PyTorch CPU restatement of the reference's `disable_ssim=False` residual, pinned against the
reference's own `utils/loss_utils.py` functions by tests/golden/ssim_golden.npz:

  gaussian / create_window   utils/loss_utils.py:49-57  (11 taps, sigma 1.5, float32, 2-D = outer product)
  ssim_per_pixel             utils/loss_utils.py:91-122 (depthwise conv2d, zero padding 5, C1 = 0.01^2,
                             C2 = 0.03^2)
  l1_loss_per_pixel          utils/loss_utils.py:43-44
  residual block             solver/batch_training_loss.py:10-30 with FUSED_SSIM_AVAILABLE=False:
                               r1 = alpha_img sqrt(|x - gt| + 1e-6)
                               r2 = beta_img  sqrt(|1 - ssim(x, gt)| + 1e-6)
                             x = clamp01(render) * mask (batch_render.py:118, batch_training_loss.py:56-67),
                             alpha_img = sqrt((1 - lambda) / (3 H W)), beta_img = sqrt(lambda / (3 H W))
                             (batch_training_loss.py:69-77), lambda_dssim = 0.2 (arguments/__init__.py:90).
The residual vector is [r1; r2] (no aliasing), loss = ||r1||^2 + ||r2||^2 (loss_image_state.py:16-19).
"""
from math import exp

import torch
import torch.nn.functional as F

WINDOW = 11
SIGMA = 1.5
C1 = 0.01 ** 2
C2 = 0.03 ** 2
LAMBDA_DSSIM = 0.2


def gaussian_1d(window_size=WINDOW, sigma=SIGMA):
    g = torch.tensor([exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)],
                     dtype=torch.float32)
    return g / g.sum()


def create_window(window_size=WINDOW, channel=3):
    g1 = gaussian_1d(window_size).unsqueeze(1)
    w2 = g1.mm(g1.t()).float().unsqueeze(0).unsqueeze(0)
    return w2.expand(channel, 1, window_size, window_size).contiguous()


def ssim_per_pixel(img1, img2, window_size=WINDOW):
    """SSIM map of [.., C, H, W] images (per channel, same shape as the inputs)."""
    channel = img1.size(-3)
    window = create_window(window_size, channel).type_as(img1)
    pad = window_size // 2
    mu1 = F.conv2d(img1, window, padding=pad, groups=channel)
    mu2 = F.conv2d(img2, window, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = F.conv2d(img1 * img1, window, padding=pad, groups=channel) - mu1_sq
    sigma2_sq = F.conv2d(img2 * img2, window, padding=pad, groups=channel) - mu2_sq
    sigma12 = F.conv2d(img1 * img2, window, padding=pad, groups=channel) - mu1_mu2
    return ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))


def image_weights(H, W, lambda_dssim=LAMBDA_DSSIM):
    n = 3 * H * W
    return ((1.0 - lambda_dssim) / n) ** 0.5, (lambda_dssim / n) ** 0.5


def ssim_residuals(x, gt, lambda_dssim=LAMBDA_DSSIM):
    """(r1, r2) of one view; x = clamp01(render) * mask, [3, H, W]."""
    H, W = x.shape[-2:]
    a, b = image_weights(H, W, lambda_dssim)
    l1 = torch.abs(x - gt)
    s = ssim_per_pixel(x.unsqueeze(0), gt.unsqueeze(0)).squeeze(0)
    return a * torch.sqrt(l1 + 1e-6), b * torch.sqrt(torch.abs(1.0 - s) + 1e-6)
