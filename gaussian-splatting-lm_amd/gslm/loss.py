"""The first-order loss of train.py:119-125 (utils/loss_utils.py:40-89).

* `l1_loss(x, y)`  = mean |x - y|   (loss_utils.py:40-41; two elementwise torch ops)
* `ssim(x, y)`     = mean SSIM map, 11-tap Gaussian window (sigma 1.5), zero padding (loss_utils.py:59-89,
                     size_average=True), forward and backward as HIP kernels (csrc/ssim.hip
                     gslm_ssim_mean / gslm_ssim_mean_backward): the role of upstream's optional
                     `fused_ssim` (train.py:32-36).  GPU tensors only; no torch fallback.
"""
import torch

from gslm import _lib
from gslm._lib import lib, check


def l1_loss(network_output, gt):
    return torch.abs(network_output - gt).mean()


class _SsimMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, gt):
        if not img.is_cuda:
            raise RuntimeError("gslm.loss.ssim runs on the GPU (HIP kernel); got a CPU tensor")
        x = img.detach().to(torch.float32).contiguous()
        y = gt.detach().to(device=x.device, dtype=torch.float32).contiguous()
        if x.shape != y.shape:
            raise ValueError(f"ssim: image {tuple(x.shape)} and ground truth {tuple(y.shape)} differ")
        C, H, W = (int(d) for d in x.shape[-3:])
        C *= int(x.numel() // (C * H * W))  # a leading batch folds into the channel planes
        state = _lib.u8(lib.gslm_ssim_mean_state_bytes(C, H, W), x.device)
        out = torch.empty((), dtype=torch.float32, device=x.device)
        check(lib.gslm_ssim_mean(C, H, W, x.data_ptr(), y.data_ptr(), state.data_ptr(), state.numel(),
                                 out.data_ptr(), _lib.stream_handle(x.device)), "gslm_ssim_mean")
        ctx.save_for_backward(x, y, state)
        ctx.dims, ctx.in_dtype = (C, H, W), img.dtype
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, y, state = ctx.saved_tensors
        C, H, W = ctx.dims
        g = grad_out.detach().to(torch.float32).contiguous()
        grad = torch.empty_like(x)
        check(lib.gslm_ssim_mean_backward(C, H, W, x.data_ptr(), y.data_ptr(), state.data_ptr(), g.data_ptr(),
                                          grad.data_ptr(), _lib.stream_handle(x.device)), "gslm_ssim_mean_backward")
        return grad.to(ctx.in_dtype), None


def ssim(img1, img2, window_size=11, size_average=True):
    """utils/loss_utils.py:59-67 (window_size 11, size_average=True only, as train.py calls it)."""
    if window_size != 11 or not size_average:
        raise NotImplementedError("ssim: only window_size=11, size_average=True (the train.py call)")
    return _SsimMean.apply(img1, img2)
