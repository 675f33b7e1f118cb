"""Parameter container with the reference's tensor layout.

Mirrors the hot-path parts of `scene/gaussian_model.py`:
  * layout            :53-69, :256-266  (_xyz[P,3], _features_dc[P,1,3], _features_rest[P,K-1,3],
                                          _scaling[P,3] (log), _rotation[P,4] (wxyz), _opacity[P,1] (logit),
                                          _exposure[Ncam,3,4])
  * activations       :35-50, :192-233  (exp, sigmoid, L2-normalize, cat(dc, rest))
  * make_dual         :71-101
  * zero_grad         :122-129
  * update_step       :131-139
  * capture / restore :158-190
  * create_from_pcd   :236-265  (scales from distCUDA2 = gslm.knn, csrc/knn.hip)
  * save_ply / load_ply :329-397 (gslm.ply, numpy; plyfile is not a dependency)
  * first-order training:
      training_setup / update_learning_rate :268-313  (gslm.optim.FusedAdam / SparseGaussianAdam)
      reset_opacity, optimizer surgery, prune / clone / split :348-559
      add_densification_stats :561-563 (+ the max_radii2D update of train.py:166) = gslm_densify_stats
"""
from contextlib import contextmanager

import numpy as np
import torch
import torch.autograd.forward_ad as fwAD
import torch.nn as nn
import torch.nn.functional as F

C0 = 0.28209479177387814  # utils/sh_utils.py:26


def RGB2SH(rgb):
    """`utils/sh_utils.py:114`."""
    return (rgb - 0.5) / C0


def sh_basis(deg, dirs):
    """Real SH basis values [..., (deg+1)^2] at unit directions, deg <= 3, in the coefficient order and
    sign convention of utils/sh_utils.py:57-112 (constants :26-44)."""
    x, y, z = dirs[..., 0], dirs[..., 1], dirs[..., 2]
    b = [torch.full_like(x, C0)]
    if deg > 0:
        c1 = 0.4886025119029199
        b += [-c1 * y, c1 * z, -c1 * x]
    if deg > 1:
        xx, yy, zz = x * x, y * y, z * z
        b += [1.0925484305920792 * x * y, -1.0925484305920792 * y * z, 0.31539156525252005 * (2 * zz - xx - yy),
              -1.0925484305920792 * x * z, 0.5462742152960396 * (xx - yy)]
    if deg > 2:
        b += [-0.5900435899266435 * y * (3 * xx - yy), 2.890611442640554 * x * y * z,
              -0.4570457994644658 * y * (4 * zz - xx - yy), 0.3731763325901154 * z * (2 * zz - 3 * xx - 3 * yy),
              -0.4570457994644658 * x * (4 * zz - xx - yy), 1.445305721320277 * z * (xx - yy),
              -0.5900435899266435 * x * (xx - 3 * yy)]
    if deg > 3:
        raise ValueError("SH degree > 3 is not supported by the rasterizer")
    return torch.stack(b, dim=-1)


def eval_sh(deg, sh, dirs):
    """utils/sh_utils.py:57-112: sh [..., C, K >= (deg+1)^2], dirs [..., 3] -> [..., C]."""
    n = (deg + 1) ** 2
    return (sh[..., :n] * sh_basis(deg, dirs)[..., None, :]).sum(-1)


def inverse_sigmoid(x):
    """`utils/general_utils.py:19`."""
    return torch.log(x / (1 - x))


class _FirstOrder:
    """GaussianModel's first-order training methods (scene/gaussian_model.py:268-563), mixed in below."""

    def training_setup(self, training_args):
        """gaussian_model.py:268-301: six Adam groups (xyz lr scaled by spatial_lr_scale, f_rest at
        feature_lr / 20), eps 1e-15; optimizer_type "sparse_adam" -> SparseGaussianAdam; a separate
        Adam for the exposures; exponential xyz / exposure schedules."""
        from gslm.optim import FusedAdam, SparseGaussianAdam
        ta = training_args
        self.percent_dense = ta.percent_dense
        P, dev = self._xyz.shape[0], self._xyz.device
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros(P, device=dev)
        for name in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation", "_exposure"):
            setattr(self, name, nn.Parameter(getattr(self, name).detach().contiguous().requires_grad_(True)))
        groups = [
            {"params": [self._xyz], "lr": ta.position_lr_init * self.spatial_lr_scale, "name": "xyz"},
            {"params": [self._features_dc], "lr": ta.feature_lr, "name": "f_dc"},
            {"params": [self._features_rest], "lr": ta.feature_lr / 20.0, "name": "f_rest"},
            {"params": [self._opacity], "lr": ta.opacity_lr, "name": "opacity"},
            {"params": [self._scaling], "lr": ta.scaling_lr, "name": "scaling"},
            {"params": [self._rotation], "lr": ta.rotation_lr, "name": "rotation"},
        ]
        if self.optimizer_type == "sparse_adam":
            self.optimizer = SparseGaussianAdam(groups, lr=0.0, eps=1e-15)
        else:
            self.optimizer = FusedAdam(groups, lr=0.0, eps=1e-15)
        self.exposure_optimizer = FusedAdam([self._exposure])
        self.xyz_scheduler_args = get_expon_lr_func(ta.position_lr_init * self.spatial_lr_scale,
                                                    ta.position_lr_final * self.spatial_lr_scale,
                                                    lr_delay_mult=ta.position_lr_delay_mult,
                                                    max_steps=ta.position_lr_max_steps)
        self.exposure_scheduler_args = get_expon_lr_func(ta.exposure_lr_init, ta.exposure_lr_final,
                                                         lr_delay_steps=ta.exposure_lr_delay_steps,
                                                         lr_delay_mult=ta.exposure_lr_delay_mult,
                                                         max_steps=ta.iterations)

    def update_learning_rate(self, iteration):
        """gaussian_model.py:303-313 (returns the xyz lr)."""
        if self.pretrained_exposures is None:
            for g in self.exposure_optimizer.param_groups:
                g["lr"] = self.exposure_scheduler_args(iteration)
        for g in self.optimizer.param_groups:
            if g["name"] == "xyz":
                g["lr"] = self.xyz_scheduler_args(iteration)
                return g["lr"]

    # ---- optimizer surgery: swap a group's tensor, keeping (or resetting) its Adam moments ----
    def _swap_group(self, name, new_param, moments):
        """Replace group `name`'s tensor by `new_param`; moments(old_state) -> (exp_avg, exp_avg_sq) or None."""
        for group in self.optimizer.param_groups:
            if group["name"] != name:
                continue
            old = group["params"][0]
            state = self.optimizer.state.pop(old, None)
            param = nn.Parameter(new_param.contiguous().requires_grad_(True))
            group["params"][0] = param
            if state is not None:
                state["exp_avg"], state["exp_avg_sq"] = (t.contiguous() for t in moments(state))
                self.optimizer.state[param] = state
            return param
        raise KeyError(name)

    def replace_tensor_to_optimizer(self, tensor, name):
        """gaussian_model.py:406-419: new tensor, zeroed moments."""
        p = self._swap_group(name, tensor, lambda st: (torch.zeros_like(tensor), torch.zeros_like(tensor)))
        return {name: p}

    _GROUP_ATTR = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
                   "scaling": "_scaling", "rotation": "_rotation"}

    def _apply_to_groups(self, tensor_fn, moment_fn):
        for group in self.optimizer.param_groups:
            name = group["name"]
            old = group["params"][0]
            p = self._swap_group(name, tensor_fn(name, old.detach()),
                                 lambda st: (moment_fn(name, st["exp_avg"]), moment_fn(name, st["exp_avg_sq"])))
            setattr(self, self._GROUP_ATTR[name], p)

    @torch.no_grad()
    def reset_opacity(self):
        """gaussian_model.py:348-351: opacity = min(opacity, 0.01), moments zeroed."""
        new = inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01))
        self._opacity = self.replace_tensor_to_optimizer(new.detach(), "opacity")["opacity"]

    @torch.no_grad()
    def prune_points(self, mask):
        """gaussian_model.py:421-454: drop the Gaussians where mask is True (parameters, moments, stats)."""
        keep = ~mask
        self._apply_to_groups(lambda n, t: t[keep], lambda n, m: m[keep])
        self.xyz_gradient_accum = self.xyz_gradient_accum[keep]
        self.denom = self.denom[keep]
        self.max_radii2D = self.max_radii2D[keep]
        if getattr(self, "tmp_radii", None) is not None:
            self.tmp_radii = self.tmp_radii[keep]

    def densification_postfix(self, new_xyz, new_features_dc, new_features_rest, new_opacities, new_scaling,
                              new_rotation, new_tmp_radii):
        """gaussian_model.py:456-497: append Gaussians (zero moments), reset the statistics."""
        ext = {"xyz": new_xyz, "f_dc": new_features_dc, "f_rest": new_features_rest, "opacity": new_opacities,
               "scaling": new_scaling, "rotation": new_rotation}
        self._apply_to_groups(lambda n, t: torch.cat((t, ext[n].detach())),
                              lambda n, m: torch.cat((m, torch.zeros_like(ext[n]))))
        self.tmp_radii = torch.cat((self.tmp_radii, new_tmp_radii))
        P, dev = self._xyz.shape[0], self._xyz.device
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros(P, device=dev)

    @torch.no_grad()
    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2):
        """gaussian_model.py:499-523: large high-gradient Gaussians -> N samples at scale / (0.8 N)."""
        P, dev = self._xyz.shape[0], self._xyz.device
        padded = torch.zeros(P, device=dev)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = (padded >= grad_threshold) & (self.get_scaling.max(dim=1).values > self.percent_dense * scene_extent)
        stds = self.get_scaling[sel].repeat(N, 1)
        samples = self._split_samples(stds)
        rots = build_rotation(self._rotation[sel]).repeat(N, 1, 1)
        new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self.get_xyz[sel].repeat(N, 1)
        new_scaling = self.scaling_inverse_activation(self.get_scaling[sel].repeat(N, 1) / (0.8 * N))
        self.densification_postfix(new_xyz, self._features_dc[sel].repeat(N, 1, 1),
                                   self._features_rest[sel].repeat(N, 1, 1), self._opacity[sel].repeat(N, 1),
                                   new_scaling, self._rotation[sel].repeat(N, 1), self.tmp_radii[sel].repeat(N))
        prune = torch.cat((sel, torch.zeros(N * int(sel.sum()), device=dev, dtype=torch.bool)))
        self.prune_points(prune)

    def _split_samples(self, stds):
        """The N(0, stds) offsets of densify_and_split (gaussian_model.py:509-511)."""
        return torch.normal(mean=torch.zeros((stds.size(0), 3), device=stds.device), std=stds)

    @torch.no_grad()
    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        """gaussian_model.py:525-540: small high-gradient Gaussians are duplicated."""
        sel = (torch.norm(grads, dim=-1) >= grad_threshold) & (
            self.get_scaling.max(dim=1).values <= self.percent_dense * scene_extent)
        self.densification_postfix(self._xyz[sel], self._features_dc[sel], self._features_rest[sel],
                                   self._opacity[sel], self._scaling[sel], self._rotation[sel], self.tmp_radii[sel])

    @torch.no_grad()
    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, radii):
        """gaussian_model.py:542-559."""
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.tmp_radii = radii
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent)
        prune = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            big_vs = self.max_radii2D > max_screen_size
            big_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
            prune = prune | big_vs | big_ws
        self.prune_points(prune)
        self.tmp_radii = None

    def add_densification_stats(self, viewspace_point_tensor, update_filter=None, radii=None):
        """gaussian_model.py:561-563 on the HIP kernel gslm_densify_stats.  The reference passes
        update_filter = radii > 0 (render()'s visibility_filter); pass `radii` to take the mask from it and
        fold train.py:166's max_radii2D update into the same pass."""
        from gslm._lib import lib, check, stream_handle
        g = viewspace_point_tensor.grad
        if radii is None:
            if update_filter is None:
                raise ValueError("add_densification_stats needs update_filter or radii")
            m = torch.zeros(self._xyz.shape[0], dtype=torch.bool, device=g.device)
            m[update_filter.reshape(-1) if update_filter.dtype != torch.bool else update_filter] = True
            radii, max_r = m.to(torch.int32), None
        else:
            max_r = self.max_radii2D
        g = g.contiguous()
        radii = radii.to(torch.int32).contiguous()
        check(lib.gslm_densify_stats(g.shape[0], g.data_ptr(), g.shape[1], radii.data_ptr(),
                                     None if max_r is None else max_r.data_ptr(),
                                     self.xyz_gradient_accum.data_ptr(), self.denom.data_ptr(),
                                     stream_handle(g.device)), "gslm_densify_stats")


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:30-63: log-linear decay from lr_init (step 0) to lr_final (max_steps), with
    an optional sine-eased delay."""
    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        return delay_rate * np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
    return helper


class GaussianModel(_FirstOrder):
    def __init__(self, sh_degree, optimizer_type="default"):
        self.active_sh_degree = 0
        self.optimizer_type = optimizer_type
        self.max_sh_degree = sh_degree
        self._xyz = torch.empty(0)
        self._features_dc = torch.empty(0)
        self._features_rest = torch.empty(0)
        self._scaling = torch.empty(0)
        self._rotation = torch.empty(0)
        self._opacity = torch.empty(0)
        self._exposure = torch.empty(0)
        self.max_radii2D = torch.empty(0)
        self.xyz_gradient_accum = torch.empty(0)
        self.denom = torch.empty(0)
        self.optimizer = None
        self.spatial_lr_scale = 0
        self.scaling_activation = torch.exp
        self.scaling_inverse_activation = torch.log
        self.opacity_activation = torch.sigmoid
        self.inverse_opacity_activation = inverse_sigmoid
        self.rotation_activation = F.normalize
        self.exposure_mapping = {}
        self.pretrained_exposures = None

    # ---- activations (gaussian_model.py:192-233) ----
    @property
    def get_scaling(self):
        return self.scaling_activation(self._scaling)

    @property
    def get_rotation(self):
        return self.rotation_activation(self._rotation)

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_features_dc(self):
        return self._features_dc

    @property
    def get_features_rest(self):
        return self._features_rest

    @property
    def get_opacity(self):
        return self.opacity_activation(self._opacity)

    @property
    def get_exposure(self):
        return self._exposure

    def get_exposure_from_name(self, image_name):
        if self.pretrained_exposures is None:
            return self._exposure[self.exposure_mapping[image_name]]
        return self.pretrained_exposures[image_name]

    def get_covariance(self, scaling_modifier=1):
        """cov3D upper triangle of L L^T, L = R(q) diag(s) (gaussian_model.py:36-40)."""
        s = scaling_modifier * self.get_scaling
        R = build_rotation(self._rotation)
        L = R * s[:, None, :]
        S = L @ L.transpose(1, 2)
        return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], dim=1)

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    @property
    def num_gaussians(self):
        return self._xyz.shape[0]

    def params(self):
        return [self._xyz, self._features_dc, self._features_rest, self._scaling,
                self._rotation, self._opacity, self._exposure]

    def set_params(self, xyz, dc, rest, scaling, rotation, opacity, exposure=None, requires_grad=True):
        def leaf(t):
            return t.detach().clone().contiguous().requires_grad_(requires_grad)
        self._xyz, self._features_dc, self._features_rest = leaf(xyz), leaf(dc), leaf(rest)
        self._scaling, self._rotation, self._opacity = leaf(scaling), leaf(rotation), leaf(opacity)
        if exposure is None:
            exposure = torch.eye(3, 4, device=xyz.device)[None]
        self._exposure = leaf(exposure)
        P = xyz.shape[0]
        self.max_radii2D = torch.zeros(P, device=xyz.device)
        return self

    # ---- LM protocol (gaussian_model.py:71-139) ----
    @contextmanager
    def make_dual(self, v):
        orig = (self._xyz, self._features_dc, self._features_rest, self._scaling,
                self._rotation, self._opacity, self._exposure)
        self._xyz = fwAD.make_dual(self._xyz, v.xyz_grad)
        self._features_dc = fwAD.make_dual(self._features_dc, v.features_dc_grad)
        self._features_rest = fwAD.make_dual(self._features_rest, v.features_rest_grad)
        self._scaling = fwAD.make_dual(self._scaling, v.scaling_grad)
        self._rotation = fwAD.make_dual(self._rotation, v.rotation_grad)
        self._opacity = fwAD.make_dual(self._opacity, v.opacity_grad)
        self._exposure = fwAD.make_dual(self._exposure, v.exposure_grad)
        try:
            yield
        finally:
            (self._xyz, self._features_dc, self._features_rest, self._scaling,
             self._rotation, self._opacity, self._exposure) = orig

    def zero_grad(self):
        for t in self.params():
            t.grad = None

    def update_step(self, s):
        self._xyz.data += s.xyz_grad
        self._features_dc.data += s.features_dc_grad
        self._features_rest.data += s.features_rest_grad
        self._scaling.data += s.scaling_grad
        self._rotation.data += s.rotation_grad
        self._opacity.data += s.opacity_grad
        self._exposure.data += s.exposure_grad

    def capture(self):
        """gaussian_model.py:158-172 (the reference drops _exposure; so do we)."""
        return (self.active_sh_degree, self._xyz, self._features_dc, self._features_rest,
                self._scaling, self._rotation, self._opacity, self.max_radii2D,
                self.xyz_gradient_accum, self.denom, None, self.spatial_lr_scale)

    def restore(self, model_args, training_args=None):
        (self.active_sh_degree, self._xyz, self._features_dc, self._features_rest,
         self._scaling, self._rotation, self._opacity, self.max_radii2D,
         self.xyz_gradient_accum, self.denom, _opt, self.spatial_lr_scale) = model_args

    # ---- initialisation and on-disk formats ----
    def create_from_pcd(self, points, colors, n_cams=1, spatial_lr_scale=0.0, device="cuda"):
        """gaussian_model.py:236-265: SH DC from the point colours, scales log(sqrt(mean 3-NN squared
        distance)) clamped at 1e-7, identity rotations, opacity 0.1, one eye(3, 4) exposure per camera."""
        from gslm.knn import distCUDA2
        self.spatial_lr_scale = spatial_lr_scale
        pts = torch.as_tensor(points, dtype=torch.float32).to(device)
        rgb = torch.as_tensor(colors, dtype=torch.float32).to(device)
        P, K = pts.shape[0], (self.max_sh_degree + 1) ** 2
        features = torch.zeros((P, 3, K), dtype=torch.float32, device=device)
        features[:, :3, 0] = RGB2SH(rgb)
        dist2 = torch.clamp_min(distCUDA2(pts), 0.0000001)
        scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
        rots = torch.zeros((P, 4), device=device)
        rots[:, 0] = 1
        opacities = inverse_sigmoid(0.1 * torch.ones((P, 1), dtype=torch.float32, device=device))
        exposure = torch.eye(3, 4, device=device)[None].repeat(n_cams, 1, 1)
        self.set_params(pts, features[:, :, 0:1].transpose(1, 2), features[:, :, 1:].transpose(1, 2), scales, rots,
                        opacities, exposure)
        return self

    def save_ply(self, path):
        from gslm.ply import save_ply
        save_ply(self, path)

    def load_ply(self, path, device="cuda"):
        from gslm.ply import load_ply
        return load_ply(self, path, device=device)

    def to(self, device):
        rg = self._xyz.requires_grad
        self.set_params(*(t.detach().to(device) for t in self.params()), requires_grad=rg)
        return self


def build_rotation(r):
    """`utils/general_utils.py:79-99` (normalises, then the quaternion matrix), device-agnostic."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.view(-1, 3, 3)


def synthetic_gaussians(P, sh_degree, seed=0, s0=0.005, device="cpu", n_cams=1):
    """Seeded synthetic model, SURVEY §8(d) (generator seed 0):
    xyz ~ U[-1,1]^3; log-scale = log(s0*U[0.5,1.5]); rotation ~ N(0,I4); opacity = logit(U[0.05,0.95]);
    f_dc = RGB2SH(U[0,1]); f_rest ~ N(0, 0.05^2); exposure = eye(3,4) per camera."""
    g = torch.Generator().manual_seed(seed)
    K = (sh_degree + 1) ** 2
    xyz = torch.rand(P, 3, generator=g) * 2 - 1
    scaling = torch.log(s0 * (torch.rand(P, 3, generator=g) + 0.5))
    rotation = torch.randn(P, 4, generator=g)
    opacity = inverse_sigmoid(torch.rand(P, 1, generator=g) * 0.9 + 0.05)
    dc = RGB2SH(torch.rand(P, 1, 3, generator=g))
    rest = torch.randn(P, K - 1, 3, generator=g) * 0.05
    exposure = torch.eye(3, 4)[None].repeat(n_cams, 1, 1)
    m = GaussianModel(sh_degree)
    m.set_params(*(t.to(device) for t in (xyz, dc, rest, scaling, rotation, opacity, exposure)))
    m.active_sh_degree = sh_degree
    return m
