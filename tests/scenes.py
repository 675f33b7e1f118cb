"""Seeded test scenes shared by the CPU and GPU tests (SURVEY §8(d) input recipe)."""
import math

import torch

from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from oracle import torch_raster as tr

# name -> (P, sh_degree, W, H, s0, n_views)
SCENES = {
    "cfg1_2k_sh0_256": (2000, 0, 256, 256, 0.005, 1),     # BASELINE config 1 (sparse)
    "dense_2k_sh3_64x48": (2000, 3, 64, 48, 0.03, 1),      # many overlaps, early termination
    "mid_8k_sh1_96x80": (8000, 1, 96, 80, 0.02, 1),        # ragged tiles (96x80 = 6x5 tiles)
    "tiny_300_sh2_40x33": (300, 2, 40, 33, 0.06, 2),       # partial tiles both axes, 2 views
}


def make_scene(name, device="cpu"):
    P, D, W, H, s0, nv = SCENES[name]
    model = synthetic_gaussians(P, D, seed=0, s0=s0, device="cpu", n_cams=nv)
    cams = orbit_cameras(nv, W, H, seed=1)
    return model, cams


def activated(model):
    """The tensors render() hands to the rasterizer (gaussian_renderer/__init__.py:54-73)."""
    with torch.no_grad():
        return dict(means3D=model.get_xyz.detach().clone(), opacities=model.get_opacity.detach().clone(),
                    scales=model.get_scaling.detach().clone(), rotations=model.get_rotation.detach().clone(),
                    shs=model.get_features.detach().clone())


def oracle_settings(cam, D, bg=None, scale_modifier=1.0, antialiasing=False):
    bg = torch.zeros(3) if bg is None else bg
    return tr.settings_from_camera(cam, bg, D, scale_modifier=scale_modifier, antialiasing=antialiasing)


def gpu_settings(cam, D, bg=None, device="cuda", scale_modifier=1.0, antialiasing=False):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    bg = torch.zeros(3) if bg is None else bg
    return GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg.to(device),
        scale_modifier=float(scale_modifier), viewmatrix=cam.world_view_transform.to(device),
        projmatrix=cam.full_proj_transform.to(device), sh_degree=D, campos=cam.camera_center.to(device),
        prefiltered=False, debug=False, antialiasing=bool(antialiasing))
