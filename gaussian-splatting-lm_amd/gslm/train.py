"""First-order training on the HIP rasterizer: `render()` and the loop of train.py.

* `render`             gaussian_renderer/__init__.py:18-130 -- the settings from the camera, the drop-in
                       GaussianRasterizer, exposure, clamp, and the returned dict (render,
                       viewspace_points, visibility_filter, radii, depth).
* `OptimizationParams` arguments/__init__.py:76-103 defaults (plain attributes, no argparse).
* `training_step`      one iteration of train.py:90-186: lr schedule, SH-degree bump, render, loss
                       (1 - lambda) L1 + lambda (1 - SSIM), backward, densification statistics
                       (gslm_densify_stats), densify / prune / opacity reset, and the optimizer step
                       (gslm_adam_step: FusedAdam, or SparseGaussianAdam on radii > 0).
* `training`           the loop over a camera list (random view order as train.py:98-103).

Logging, the network GUI, tensorboard, scene loading and the depth-regularisation branch (no
mono-depth maps on synthetic cameras) are not part of this path.
"""
import math
import random
from dataclasses import dataclass

import torch

from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
from gslm.loss import l1_loss, ssim


@dataclass
class PipelineParams:
    """arguments/__init__.py:63-70."""
    convert_SHs_python: bool = False
    compute_cov3D_python: bool = False
    debug: bool = False
    antialiasing: bool = False


@dataclass
class OptimizationParams:
    """arguments/__init__.py:72-103 defaults."""
    iterations: int = 30_000
    position_lr_init: float = 0.00016
    position_lr_final: float = 0.0000016
    position_lr_delay_mult: float = 0.01
    position_lr_max_steps: int = 30_000
    feature_lr: float = 0.0025
    opacity_lr: float = 0.025
    scaling_lr: float = 0.005
    rotation_lr: float = 0.001
    exposure_lr_init: float = 0.01
    exposure_lr_final: float = 0.001
    exposure_lr_delay_steps: int = 0
    exposure_lr_delay_mult: float = 0.0
    percent_dense: float = 0.01
    lambda_dssim: float = 0.2
    densification_interval: int = 100
    opacity_reset_interval: int = 3000
    densify_from_iter: int = 500
    densify_until_iter: int = 15_000
    densify_grad_threshold: float = 0.0002
    depth_l1_weight_init: float = 1.0
    depth_l1_weight_final: float = 0.01
    random_background: bool = False
    optimizer_type: str = "default"


def render(viewpoint_camera, pc, pipe, bg_color, scaling_modifier=1.0, separate_sh=False, override_color=None,
           use_trained_exp=False):
    """gaussian_renderer/__init__.py:18-130 (colour conversion in Python and cov3D_precomp supported)."""
    from gslm.model import eval_sh
    dev = pc.get_xyz.device
    screenspace_points = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True, device=dev) + 0
    try:
        screenspace_points.retain_grad()
    except RuntimeError:
        pass
    settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5),
        bg=bg_color, scale_modifier=scaling_modifier, viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform, sh_degree=pc.active_sh_degree,
        campos=viewpoint_camera.camera_center, prefiltered=False, debug=pipe.debug, antialiasing=pipe.antialiasing)
    rasterizer = GaussianRasterizer(raster_settings=settings)
    means3D, means2D, opacity = pc.get_xyz, screenspace_points, pc.get_opacity
    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales, rotations = pc.get_scaling, pc.get_rotation
    shs = colors_precomp = dc = None
    if override_color is None:
        if pipe.convert_SHs_python:
            shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = pc.get_xyz - viewpoint_camera.camera_center.repeat(pc.get_features.shape[0], 1)
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized) + 0.5, 0.0)
        elif separate_sh:
            dc, shs = pc.get_features_dc, pc.get_features_rest
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color
    kw = dict(means3D=means3D, means2D=means2D, shs=shs, colors_precomp=colors_precomp, opacities=opacity,
              scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp)
    if separate_sh:
        kw["dc"] = dc
    rendered_image, radii, depth_image = rasterizer(**kw)
    if use_trained_exp:
        exposure = pc.get_exposure_from_name(viewpoint_camera.image_name)
        rendered_image = torch.matmul(rendered_image.permute(1, 2, 0), exposure[:3, :3]).permute(2, 0, 1) + \
            exposure[:3, 3, None, None]
    rendered_image = rendered_image.clamp(0, 1)
    return {"render": rendered_image, "viewspace_points": screenspace_points,
            "visibility_filter": (radii > 0).nonzero(), "radii": radii, "depth": depth_image}


def batch_render(viewpoint_cameras, pc, pipe, bg_color, scaling_modifier=1.0, separate_sh=False, override_color=None,
                 use_trained_exp=False):
    """gaussian_renderer/batch_render.py:8-135: the batch settings, BatchGaussianRasterizer, clamp and the dict
    (render [B,3,maxH,maxW], viewspace_points, visibility_filter of radii.max(0), max_radii, depth, viewcount)."""
    from diff_gaussian_rasterization.batch_render import BatchGaussianRasterizationSettings, BatchGaussianRasterizer
    from gslm.model import eval_sh
    if use_trained_exp:
        raise NotImplementedError("Batch exposure not implemented yet")  # batch_render.py:117-118
    dev = pc.get_xyz.device
    screenspace_points = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True, device=dev) + 0
    try:
        screenspace_points.retain_grad()
    except RuntimeError:
        pass
    cams = list(viewpoint_cameras)
    settings = BatchGaussianRasterizationSettings(
        batch_size=len(cams), image_heights=[int(c.image_height) for c in cams],
        image_widths=[int(c.image_width) for c in cams], tanfovxs=[math.tan(c.FoVx * 0.5) for c in cams],
        tanfovys=[math.tan(c.FoVy * 0.5) for c in cams], bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrices=[c.world_view_transform for c in cams], projmatrices=[c.full_proj_transform for c in cams],
        sh_degree=pc.active_sh_degree, camposes=[c.camera_center for c in cams], prefiltered=False, debug=pipe.debug,
        antialiasing=pipe.antialiasing)
    rasterizer = BatchGaussianRasterizer(batch_raster_settings=settings)
    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales, rotations = pc.get_scaling, pc.get_rotation
    shs = colors_precomp = dc = None
    if override_color is None:
        if pipe.convert_SHs_python:
            # the reference's branch reads an undefined `viewpoint_camera` here (batch_render.py:77); one set of
            # colours for the whole batch needs one centre -- the first camera's
            shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = pc.get_xyz - cams[0].camera_center.repeat(pc.get_features.shape[0], 1)
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized) + 0.5, 0.0)
        elif separate_sh:
            dc, shs = pc.get_features_dc, pc.get_features_rest
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color
    kw = dict(means3D=pc.get_xyz, means2D=screenspace_points, shs=shs, colors_precomp=colors_precomp,
              opacities=pc.get_opacity, scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp)
    if separate_sh:
        kw["dc"] = dc
    rendered_image, radii, depth_image = rasterizer(**kw)
    rendered_image = rendered_image.clamp(0, 1)
    max_radii = radii.max(dim=0).values
    return {"render": rendered_image, "viewspace_points": screenspace_points,
            "visibility_filter": (max_radii > 0).nonzero(), "max_radii": max_radii, "depth": depth_image,
            "viewcount": (radii > 0).sum(dim=0)}


class Trainer:
    """State of train.py:training() between iterations (model, cameras, background, view stack)."""

    def __init__(self, gaussians, cameras, opt=None, pipe=None, background=None, cameras_extent=1.0,
                 white_background=False, train_test_exp=False, seed=0):
        self.gaussians, self.cameras = gaussians, list(cameras)
        self.opt = opt or OptimizationParams()
        self.pipe = pipe or PipelineParams()
        dev = gaussians.get_xyz.device
        bg = [1, 1, 1] if white_background else [0, 0, 0]
        self.background = background if background is not None else torch.tensor(bg, dtype=torch.float32, device=dev)
        self.cameras_extent = cameras_extent
        self.white_background = white_background
        self.train_test_exp = train_test_exp
        self.use_sparse_adam = self.opt.optimizer_type == "sparse_adam"
        self.separate_sh = True  # SparseGaussianAdam is available in this build (train.py:37-41, 111)
        self.rng = random.Random(seed)
        self.viewpoint_stack, self.viewpoint_indices = [], []
        self.last = None

    def next_camera(self):
        """train.py:98-103: a random camera from a stack that is refilled when empty."""
        if not self.viewpoint_stack:
            self.viewpoint_stack = self.cameras.copy()
            self.viewpoint_indices = list(range(len(self.viewpoint_stack)))
        i = self.rng.randint(0, len(self.viewpoint_indices) - 1)
        self.viewpoint_indices.pop(i)
        return self.viewpoint_stack.pop(i)

    def step(self, iteration, viewpoint_cam=None):
        """One iteration of train.py:90-186; returns the loss tensor (no host sync)."""
        g, opt = self.gaussians, self.opt
        g.update_learning_rate(iteration)
        if iteration % 1000 == 0:
            g.oneupSHdegree()
        cam = viewpoint_cam if viewpoint_cam is not None else self.next_camera()
        bg = torch.rand(3, device=self.background.device) if opt.random_background else self.background
        pkg = render(cam, g, self.pipe, bg, use_trained_exp=self.train_test_exp, separate_sh=self.separate_sh)
        image, viewspace_points, radii = pkg["render"], pkg["viewspace_points"], pkg["radii"]
        if cam.alpha_mask is not None:
            image = image * cam.alpha_mask
        gt = cam.original_image
        Ll1 = l1_loss(image, gt)
        loss = (1.0 - opt.lambda_dssim) * Ll1 + opt.lambda_dssim * (1.0 - ssim(image, gt))
        loss.backward()
        with torch.no_grad():
            if iteration < opt.densify_until_iter:
                # train.py:166-167 in one pass (max_radii2D, gradient accumulation, denominator)
                g.add_densification_stats(viewspace_points, radii=radii)
                if iteration > opt.densify_from_iter and iteration % opt.densification_interval == 0:
                    size_threshold = 20 if iteration > opt.opacity_reset_interval else None
                    g.densify_and_prune(opt.densify_grad_threshold, 0.005, self.cameras_extent, size_threshold, radii)
                if iteration % opt.opacity_reset_interval == 0 or (
                        self.white_background and iteration == opt.densify_from_iter):
                    g.reset_opacity()
            if iteration < opt.iterations:
                g.exposure_optimizer.step()
                g.exposure_optimizer.zero_grad(set_to_none=True)
                if self.use_sparse_adam:
                    visible = radii > 0
                    g.optimizer.step(visible, radii.shape[0])
                else:
                    g.optimizer.step()
                g.optimizer.zero_grad(set_to_none=True)
        self.last = pkg
        return loss.detach()


def training(gaussians, cameras, opt=None, pipe=None, first_iter=1, last_iter=None, **kw):
    """train.py:68-186 over `cameras` (the model must have been through `training_setup(opt)`)."""
    tr = Trainer(gaussians, cameras, opt=opt, pipe=pipe, **kw)
    last_iter = tr.opt.iterations if last_iter is None else last_iter
    losses = [tr.step(it) for it in range(first_iter, last_iter + 1)]
    return torch.stack(losses) if losses else torch.empty(0)
