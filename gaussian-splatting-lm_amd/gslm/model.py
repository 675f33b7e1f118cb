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
Densification and optimizer setup are out of scope.
"""
from contextlib import contextmanager

import torch
import torch.autograd.forward_ad as fwAD
import torch.nn.functional as F

C0 = 0.28209479177387814  # utils/sh_utils.py:26


def RGB2SH(rgb):
    """`utils/sh_utils.py:114`."""
    return (rgb - 0.5) / C0


def inverse_sigmoid(x):
    """`utils/general_utils.py:19`."""
    return torch.log(x / (1 - x))


class GaussianModel:
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
