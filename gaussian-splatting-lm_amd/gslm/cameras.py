"""Camera conventions of the reference, restated for the MI355X build.

Follows `utils/graphics_utils.py:38-71` (getWorld2View2, getProjectionMatrix) and
`scene/cameras.py:19-89` (Camera: world_view_transform, full_proj_transform,
camera_center).  Matrices are stored exactly as the reference stores them: the
row-major torch storage of the *transposed* world-to-view matrix, which the
rasterizer reads as a column-major 4x4.

The reference Camera loads images with cv2/PIL; here the image is handed in as
a tensor, everything else (field names, matrix construction) is the same so
`render()` / `batch_render()` / `batch_training_loss()` can consume it.
"""
import math

import numpy as np
import torch


def get_world2view2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    """`utils/graphics_utils.py:38-49`: R is the camera-to-world rotation (COLMAP R^T),
    t the world-to-camera translation."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = C2W[:3, 3]
    cam_center = (cam_center + translate) * scale
    C2W[:3, 3] = cam_center
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def get_projection_matrix(znear, zfar, fovX, fovY):
    """`utils/graphics_utils.py:51-71`."""
    tanHalfFovY = math.tan(fovY / 2)
    tanHalfFovX = math.tan(fovX / 2)
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def fov2focal(fov, pixels):
    return pixels / (2 * math.tan(fov / 2))


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


class Camera:
    """Matrix-side mirror of `scene/cameras.py:19-89`.

    `image` is a [3,H,W] float tensor in [0,1] (or None: a zero image of the given size).
    """

    def __init__(self, R, T, FoVx, FoVy, image=None, width=None, height=None,
                 image_name="", uid=0, alpha_mask=None, trans=np.array([0.0, 0.0, 0.0]),
                 scale=1.0, device="cpu"):
        self.uid = uid
        self.colmap_id = uid
        self.R = R
        self.T = T
        self.FoVx = FoVx
        self.FoVy = FoVy
        self.image_name = image_name or f"view_{uid:05d}"
        if image is None:
            image = torch.zeros(3, int(height), int(width))
        self.original_image = image.clamp(0.0, 1.0).to(device)
        self.image_width = self.original_image.shape[2]
        self.image_height = self.original_image.shape[1]
        # cameras.py:46-49 -- an all-ones mask when the image has no alpha channel
        self.alpha_mask = (alpha_mask.to(device) if alpha_mask is not None
                           else torch.ones_like(self.original_image[0:1]))
        self.invdepthmap = None
        self.depth_reliable = False
        self.zfar = 100.0
        self.znear = 0.01
        self.trans = trans
        self.scale = scale
        # cameras.py:86-89
        self.world_view_transform = torch.tensor(get_world2view2(R, T, trans, scale)).transpose(0, 1).to(device)
        self.projection_matrix = get_projection_matrix(znear=self.znear, zfar=self.zfar,
                                                       fovX=self.FoVx, fovY=self.FoVy).transpose(0, 1).to(device)
        self.full_proj_transform = (self.world_view_transform.unsqueeze(0)
                                    .bmm(self.projection_matrix.unsqueeze(0))).squeeze(0)
        self.camera_center = self.world_view_transform.inverse()[3, :3]

    def to(self, device):
        for name in ("original_image", "alpha_mask", "world_view_transform", "projection_matrix",
                     "full_proj_transform", "camera_center"):
            setattr(self, name, getattr(self, name).to(device))
        return self


def look_at(eye, target=(0.0, 0.0, 0.0), world_up=(0.0, 0.0, 1.0)):
    """COLMAP-convention pose (x right, y down, z forward) looking from `eye` at `target`.
    Returns (R, T) in the reference Camera convention: R = camera-to-world rotation, T = w2c translation."""
    eye = np.asarray(eye, dtype=np.float64)
    f = np.asarray(target, dtype=np.float64) - eye
    f /= np.linalg.norm(f)
    r = np.cross(f, np.asarray(world_up, dtype=np.float64))
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    R_w2c = np.stack([r, d, f], axis=0)
    T = -R_w2c @ eye
    return R_w2c.T.copy(), T


def orbit_cameras(n, width, height, fovx_deg=60.0, radius=3.0, seed=1, device="cpu", images=None):
    """Seeded cameras on a sphere of `radius` looking at the origin (seed 1)."""
    g = np.random.default_rng(seed)
    fovx = math.radians(fovx_deg)
    fovy = focal2fov(fov2focal(fovx, width), height)
    cams = []
    for i in range(n):
        while True:
            v = g.normal(size=3)
            v /= np.linalg.norm(v)
            if abs(v[2]) < 0.85:
                break
        R, T = look_at(radius * v)
        img = None if images is None else images[i]
        cams.append(Camera(R, T, fovx, fovy, image=img, width=width, height=height, uid=i, device=device))
    return cams
