"""Experiment: where the drop-in path's time goes (bench.py dropin_solver_ops, tests/test_jvp_timing.py:71-106 call
shapes) at the headline size: 1M Gaussians SH 3, one 1080p view.  Host-timed medians (each call synchronised):
  activations   the GaussianModel get_* tensors render() builds (sigmoid / exp / normalize / cat of the SH)
  settings      diff_gaussian_rasterization's host copy of the settings tensors (view_from_settings)
  raster_fwd    GaussianRasterizer forward on precomputed activations (no grad)
  render_fwd    gslm.train.render forward (no grad)
  raw_fwd       the same HIP forward on the raw leaves (ViewRaster.forward: activations fused, pair count read back)
  matvec / matvec_T / forward   bench.py's three drop-in timings
    python tools/exp/dropin_breakdown.py [--P 1000000] [--reps 7]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=7)
a = ap.parse_args()
import bench  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from gslm import _lib  # noqa: E402
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import ViewRaster  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.params import raw_gaussians  # noqa: E402
from gslm.train import PipelineParams, render  # noqa: E402
import math  # noqa: E402

dev = torch.device("cuda", 0)
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu").to(dev)
cam = orbit_cameras(1, 1920, 1080, seed=1)[0].to(dev)
bg = torch.zeros(3, device=dev)
pipe = PipelineParams()


def med(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return 1e3 * sorted(ts)[len(ts) // 2]


def acts():
    return (model.get_xyz, model.get_opacity, model.get_scaling, model.get_rotation, model.get_features)


settings = GaussianRasterizationSettings(
    image_height=1080, image_width=1920, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg,
    scale_modifier=1.0, viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, sh_degree=3,
    campos=cam.camera_center, prefiltered=False, debug=False, antialiasing=False)
out = {"P": a.P}
with torch.no_grad():
    out["activations_ms"] = med(acts)
    out["settings_ms"] = med(lambda: _lib.view_from_settings(settings))
    xyz, op, sc, rot, sh = acts()
    m2 = torch.zeros_like(xyz)
    rz = GaussianRasterizer(settings)
    out["raster_fwd_ms"] = med(lambda: rz(means3D=xyz, means2D=m2, shs=sh, opacities=op, scales=sc, rotations=rot))
    out["render_fwd_ms"] = med(lambda: render(cam, model, pipe, bg))
    vr = ViewRaster(_lib.view_from_camera(cam, torch.zeros(3), 3), dev)
    g = raw_gaussians(model)
    out["raw_fwd_ms"] = med(lambda: vr.forward(g, _lib.stream_handle(dev)))
cam.original_image = torch.rand(3, 1080, 1920, device=dev)
out.update(bench.time_dropin_solver_ops(model, cam, torch.zeros(3), reps=a.reps))
print(json.dumps(out), flush=True)
