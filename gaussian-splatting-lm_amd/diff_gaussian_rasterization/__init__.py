"""Drop-in `diff_gaussian_rasterization` for MI355X (HIP, gfx950).

Same surface as the package the reference imports at gaussian_renderer/__init__.py:14 (and, as
`diff_gaussian_rasterization_orig`, at gaussian_renderer/reference_render.py:14):

    GaussianRasterizationSettings(image_height, image_width, tanfovx, tanfovy, bg, scale_modifier,
                                  viewmatrix, projmatrix, sh_degree, campos, prefiltered, debug,
                                  antialiasing)                         # __init__.py:36-50
    GaussianRasterizer(raster_settings)(means3D=, means2D=, shs=, colors_precomp=, opacities=,
                                        scales=, rotations=, cov3D_precomp=[, dc=])
        -> (color[3,H,W], radii[P] int32, invdepth[1,H,W])           # __init__.py:90-110

The autograd Function implements `backward` (VJP, -> libgslm gslm_backward) and forward-mode `jvp`
(-> gslm_jvp, reusing the forward's sorted tile lists), which the reference's LM solver drives
through torch.autograd.forward_ad (solver/solver_functions.py:86-92).

`SparseGaussianAdam` (gslm.optim, one HIP launch per step) is exported as the accelerated upstream
rasterizer exports it (train.py:37-41, gaussian_model.py:29).  Its presence makes the reference's
train.py / train_jvp.py call render(..., separate_sh=True), which passes `dc=` and the SH rest
separately (gaussian_renderer/__init__.py:82-100): the rasterizer reads both in place (forward, VJP and
forward-mode JVP), so the LM path is unchanged by it.
"""
import ctypes
import os
from typing import NamedTuple

import torch
import torch.nn as nn

from gslm import _lib
from gslm._lib import lib, check

from gslm.optim import SparseGaussianAdam  # noqa: E402,F401

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "SparseGaussianAdam"]


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    antialiasing: bool = False


def _f32(t):
    if t is None or t.numel() == 0:
        return None
    if t.dtype != torch.float32:
        raise TypeError(f"rasterizer inputs must be float32, got {t.dtype}")
    return t.contiguous()


def _gaussians(P, means3D, opacities, scales, rotations, cov3D, sh, dc, colors):
    """gslm_gaussians for activated inputs; sh [P,K,3] (or rest [P,K-1,3] with dc [P,1,3])."""
    if dc is not None:
        dcp, dcs, rp, rs, K = _lib.sh_pointers(dc=dc, rest=sh)
    elif sh is not None:
        dcp, dcs, rp, rs, K = _lib.sh_pointers(shs=sh)
    else:
        dcp, dcs, rp, rs, K = None, 0, None, 0, 1
    return _lib.make_gaussians(P, means3D, opacities, scales, rotations, cov3D, dcp, dcs, rp, rs, K, colors, raw=False)


def forward_buffers(view, g, device):
    """Run gslm_preprocess / gslm_num_rendered / gslm_rasterize; returns outputs + saved buffers."""
    P, H, W = g.P, view.image_height, view.image_width
    stream = _lib.stream_handle(device)
    geom = _lib.u8(lib.gslm_geom_bytes(P), device)
    image = _lib.u8(lib.gslm_image_bytes(H, W), device)
    radii = torch.empty(P, dtype=torch.int32, device=device)  # gslm_preprocess writes every entry
    color = torch.empty(3, H, W, dtype=torch.float32, device=device)
    invdepth = torch.empty(1, H, W, dtype=torch.float32, device=device)
    check(lib.gslm_preprocess(ctypes.byref(view), ctypes.byref(g), geom.data_ptr(), geom.numel(),
                              radii.data_ptr(), stream), "gslm_preprocess")
    n = ctypes.c_int64(0)
    check(lib.gslm_num_rendered(geom.data_ptr(), P, ctypes.byref(n), stream), "gslm_num_rendered")
    N = int(n.value)
    binning = _lib.u8(lib.gslm_binning_bytes(N, H, W), device)
    check(lib.gslm_rasterize(ctypes.byref(view), P, geom.data_ptr(), binning.data_ptr(), binning.numel(), N,
                             image.data_ptr(), image.numel(), color.data_ptr(), invdepth.data_ptr(), stream),
          "gslm_rasterize")
    return color, radii, invdepth, geom, binning, image, N


_BWD_MEMO = os.environ.get("GSLM_BWD_MEMO", "1") != "0"


def _same_cotangent(a, b):
    """Equal cotangents (both absent, or the same shape and every element equal; one device compare and read-back)."""
    if a is None or b is None:
        return a is None and b is None
    return a.shape == b.shape and a.dtype == b.dtype and a.device == b.device and bool(torch.equal(a, b))


def _cpu_copy(args):
    return tuple(a.detach().cpu().clone() if isinstance(a, torch.Tensor) else a for a in args)


def _debug_call(settings, args, fn, which):
    """Upstream's debug protocol (diff_gaussian_rasterization/__init__.py of the CUDA rasterizer, the `debug` of
    arguments/__init__.py:70): copy the call's arguments to the host before the call, and on a failure save them to
    snapshot_<which>.dump, say so, and re-raise.  The library side of debug mode (gslm_view.debug) synchronises after
    every kernel so the failure is raised by the call that caused it."""
    if not settings.debug:
        return fn()
    cpu_args = _cpu_copy(args)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    except Exception:
        torch.save(cpu_args, f"snapshot_{which}.dump")
        print(f"\nAn error occured in {'forward' if which == 'fw' else 'backward'}. "
              f"Please forward snapshot_{which}.dump for debugging.")
        raise


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(means3D, means2D, sh, dc, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        device = means3D.device
        P = means3D.shape[0]
        view = _lib.view_from_settings(raster_settings)
        m = _f32(means3D)
        o = _f32(opacities.reshape(-1))
        s, r, c3 = _f32(scales), _f32(rotations), _f32(cov3Ds_precomp)
        shc, dcc, col = _f32(sh), _f32(dc), _f32(colors_precomp)
        g = _gaussians(P, m, o, s, r, c3, shc, dcc, col)
        color, radii, invdepth, geom, binning, image, N = _debug_call(
            raster_settings, (raster_settings.bg, means3D, colors_precomp, opacities, scales, rotations,
                              raster_settings.scale_modifier, cov3Ds_precomp, raster_settings.viewmatrix,
                              raster_settings.projmatrix, raster_settings.tanfovx, raster_settings.tanfovy,
                              raster_settings.image_height, raster_settings.image_width, sh, dc,
                              raster_settings.sh_degree, raster_settings.campos, raster_settings.prefiltered),
            lambda: forward_buffers(view, g, device), "fw")
        nr = torch.tensor([N], dtype=torch.int64)
        return color, radii, invdepth, geom, binning, image, nr

    @staticmethod
    def setup_context(ctx, inputs, output):
        (means3D, means2D, sh, dc, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
         raster_settings) = inputs
        color, radii, invdepth, geom, binning, image, nr = output
        ctx.raster_settings = raster_settings
        ctx.num_rendered = int(nr.item())
        # outputs the loss does not use reach backward as None, not as zero tensors: an unused inverse depth (the
        # reference's LM residual never reads it) then runs the backward without its gradient slot (9 values per row
        # instead of 10) and allocates no [1, H, W] of zeros
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(radii, geom, binning, image, nr)
        saved = (means3D, sh, dc, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, geom, binning, image)
        ctx.save_for_backward(*saved)
        ctx.save_for_forward(*saved)

    @staticmethod
    def backward(ctx, grad_color, _grad_radii, grad_invdepth, *_unused):
        # The reference's J^T v (solver_functions.py:101-132) calls backward twice on one graph, once per half of the
        # [r; r] pair (loss_image_state.py:93-97), and with disable_ssim the halves are the same image
        # (batch_training_loss.py:15-17), so every such pair of calls brings equal cotangents.  The VJP is a
        # deterministic function of the saved forward and the cotangent: a call whose cotangents equal the previous
        # call's, element for element (compared on the device), returns that call's gradients -- bitwise what the
        # kernels would produce again.  They stay referenced here until the graph is freed, so autograd clones them
        # before accumulating and never writes into them.  GSLM_BWD_MEMO=0 turns it off.
        memo = getattr(ctx, "bw_memo", None)
        if memo is not None and _same_cotangent(memo[0], grad_color) and _same_cotangent(memo[1], grad_invdepth):
            return memo[2]
        out = _RasterizeGaussians._backward(ctx, grad_color, grad_invdepth)
        if _BWD_MEMO:
            ctx.bw_memo = (None if grad_color is None else grad_color.detach().clone(),
                           None if grad_invdepth is None else grad_invdepth.detach().clone(), out)
        return out

    @staticmethod
    def _backward(ctx, grad_color, grad_invdepth):
        (means3D, sh, dc, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, geom, binning,
         image) = ctx.saved_tensors
        st = ctx.raster_settings
        device = means3D.device
        P = means3D.shape[0]
        N = ctx.num_rendered
        view = _lib.view_from_settings(st)
        m, o = _f32(means3D), _f32(opacities.reshape(-1))
        s, r, c3 = _f32(scales), _f32(rotations), _f32(cov3Ds_precomp)
        shc, dcc, col = _f32(sh), _f32(dc), _f32(colors_precomp)
        g = _gaussians(P, m, o, s, r, c3, shc, dcc, col)
        # gslm_backward overwrites every element of every output it is given (gslm_grads.accumulate = 0: invisible
        # Gaussians get their zeros from the kernel), so the buffers need no zero fill (~250 MB of fills per call at
        # 1M Gaussians SH 3)
        z = lambda t: None if t is None else torch.empty_like(t)
        d_means2D = torch.empty(P, 3, dtype=torch.float32, device=device)
        d_means3D = torch.empty_like(means3D)
        d_opac = torch.empty_like(opacities)
        d_scales, d_rot, d_cov = z(s), z(r), z(c3)
        d_sh, d_dc, d_col = z(shc), z(dcc), z(col)
        grads = _lib.make_grads(means2D=d_means2D, means3D=d_means3D, opacities=d_opac, scales=d_scales,
                                rotations=d_rot, cov3D=d_cov,
                                sh=(d_sh if d_dc is None else None), dc=d_dc,
                                rest=(d_sh if d_dc is not None else None), colors=d_col)
        scratch = _lib.u8(lib.gslm_scratch_bytes(P, N), device)
        gc = grad_color.contiguous() if grad_color is not None else torch.zeros(3, st.image_height, st.image_width, device=device)
        gi = grad_invdepth.contiguous() if grad_invdepth is not None else None
        _debug_call(st, (st.bg, means3D, opacities, scales, rotations, cov3Ds_precomp, sh, dc, colors_precomp, gc, gi,
                         geom, binning, image, N),
                    lambda: check(lib.gslm_backward(ctypes.byref(view), ctypes.byref(g), geom.data_ptr(),
                                                    binning.data_ptr(), N, image.data_ptr(), gc.data_ptr(),
                                                    None if gi is None else gi.data_ptr(), scratch.data_ptr(),
                                                    scratch.numel(), ctypes.byref(grads), _lib.stream_handle(device)),
                                  "gslm_backward"), "bw")
        sh_grad = d_sh if sh is not None and sh.numel() else None
        return (d_means3D, d_means2D, sh_grad, d_dc, d_col, d_opac, d_scales, d_rot, d_cov, None)

    @staticmethod
    def jvp(ctx, t_means3D, t_means2D, t_sh, t_dc, t_colors, t_opac, t_scales, t_rot, t_cov, _t_settings):
        (means3D, sh, dc, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, geom, binning,
         image) = ctx.saved_tensors
        st = ctx.raster_settings
        device = means3D.device
        P = means3D.shape[0]
        N = ctx.num_rendered
        view = _lib.view_from_settings(st)
        m, o = _f32(means3D), _f32(opacities.reshape(-1))
        s, r, c3 = _f32(scales), _f32(rotations), _f32(cov3Ds_precomp)
        shc, dcc, col = _f32(sh), _f32(dc), _f32(colors_precomp)
        g = _gaussians(P, m, o, s, r, c3, shc, dcc, col)
        tc = lambda t: None if t is None else t.contiguous()
        t_m, t_o = tc(t_means3D), (None if t_opac is None else t_opac.reshape(-1).contiguous())
        t_s, t_r, t_c3, t_col = tc(t_scales), tc(t_rot), tc(t_cov), tc(t_colors)
        t_shc, t_dcc = tc(t_sh), tc(t_dc)
        # tangent SH pointers follow the primal layout; a missing tangent is NULL (zero)
        if dcc is not None:
            tdcp = t_dcc.data_ptr() if t_dcc is not None else None
            trp = t_shc.data_ptr() if t_shc is not None else None
            _, dcs, _, rs, K = _lib.sh_pointers(dc=dcc, rest=shc)
            if tdcp is None and trp is not None:
                t_dcc = torch.zeros_like(dcc)
                tdcp = t_dcc.data_ptr()
            if trp is None and tdcp is not None and K > 1:
                t_shc = torch.zeros_like(shc)
                trp = t_shc.data_ptr()
        elif shc is not None and t_shc is not None:
            tdcp, dcs, trp, rs, K = _lib.sh_pointers(shs=t_shc)
        else:
            tdcp, dcs, trp, rs, K = None, 0, None, 0, g.max_coeffs
        tg = _lib.make_gaussians(P, t_m, t_o, t_s, t_r, t_c3, tdcp, dcs, trp, rs, K, t_col, raw=False)
        t_m2 = tc(t_means2D)
        scratch = _lib.u8(lib.gslm_scratch_bytes(P, N), device)
        color_t = torch.empty(3, st.image_height, st.image_width, dtype=torch.float32, device=device)
        inv_t = torch.empty(1, st.image_height, st.image_width, dtype=torch.float32, device=device)
        check(lib.gslm_jvp(ctypes.byref(view), ctypes.byref(g), ctypes.byref(tg),
                           None if t_m2 is None else t_m2.data_ptr(), geom.data_ptr(), binning.data_ptr(), N,
                           image.data_ptr(), scratch.data_ptr(), scratch.numel(), color_t.data_ptr(),
                           inv_t.data_ptr(), _lib.stream_handle(device)), "gslm_jvp")
        return color_t, None, inv_t, None, None, None, None


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings, dc=None):
    color, radii, invdepth, *_ = _RasterizeGaussians.apply(means3D, means2D, sh, dc, colors_precomp, opacities,
                                                           scales, rotations, cov3Ds_precomp, raster_settings)
    return color, radii, invdepth


def _none_if_empty(t):
    return None if (t is None or (isinstance(t, torch.Tensor) and t.numel() == 0)) else t


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        """Frustum test of the upstream in_frustum (p_view.z > 0.2), as a bool mask."""
        with torch.no_grad():
            V = self.raster_settings.viewmatrix
            pv = positions @ V[:3, :3] + V[3, :3]
            return pv[:, 2] > 0.2

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, dc=None):
        # upstream's exactly-one checks look at None, not at emptiness (an empty SH rest at degree 0 with dc=, or
        # every tensor of a P = 0 model, is a given argument); empty tensors become "absent" only afterwards
        has_sh = shs is not None or dc is not None
        if (not has_sh and colors_precomp is None) or (has_sh and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        shs, colors_precomp = _none_if_empty(shs), _none_if_empty(colors_precomp)
        scales, rotations, cov3D_precomp = _none_if_empty(scales), _none_if_empty(rotations), _none_if_empty(cov3D_precomp)
        dc = _none_if_empty(dc)
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, self.raster_settings, dc=dc)
