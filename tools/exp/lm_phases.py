"""Experiment: where a configs[2] LM step's wall time goes (bench.py's lm_step scene: 1M Gaussians SH 3, one 1080p
training view, the reference's 50 validation views, 10 CGLS iterations).  Untimed steps (wall clock, as bench.py's
`ms`) next to steps with timing=True (device synchronised at the phase boundaries), xyz left untouched between steps
as in train_jvp.py's loop.
    python tools/exp/lm_phases.py [--reps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.environ.get("GSLM_PKG_DIR", os.path.join(ROOT, "gaussian-splatting-lm_amd"))]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--val-batch", type=int, default=8, help="lm_step's val_batch (1: one stream, solo kernel times)")
ap.add_argument("--copy-xyz", action="store_true", help="restore xyz too between steps (drops the cached depth orders)")
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem, lm_step  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402

dev = torch.device("cuda", 0)
bg = torch.zeros(3)
pert = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1)
g2 = torch.Generator().manual_seed(2)
with torch.no_grad():
    pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
    pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
    pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
pert.to(dev)
cams = [c.to(dev) for c in orbit_cameras(1, 1920, 1080, seed=1)]
val = [c.to(dev) for c in orbit_cameras(50, 1920, 1080, seed=5)]
for chunk in [cams] + [val[i:i + 8] for i in range(0, 50, 8)]:
    vp = LMProblem(pert, chunk, bg, device=dev)
    vp.evaluate()
    for c, vr in zip(chunk, vp.views):
        c.original_image = vr.color.clamp(0, 1).clone()
    del vp
del pert
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(dev)
saved = [t.detach().clone() for t in model.params()]


def restore():
    with torch.no_grad():
        for t, s0 in zip(model.params(), saved):
            if a.copy_xyz or t is not model._xyz:
                t.copy_(s0)


out = {"copy_xyz": a.copy_xyz, "untimed_ms": [], "timed": []}
lm_step(model, cams, val, bg, max_iter=10, restart_iter=10, val_batch=a.val_batch)
restore()
for _ in range(a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lm_step(model, cams, val, bg, max_iter=10, restart_iter=10, val_batch=a.val_batch)
    torch.cuda.synchronize()
    out["untimed_ms"].append(round(1e3 * (time.perf_counter() - t0), 2))
    restore()
for _ in range(a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    o = lm_step(model, cams, val, bg, max_iter=10, restart_iter=10, timing=True, val_batch=a.val_batch)
    wall = 1e3 * (time.perf_counter() - t0)
    restore()
    out["timed"].append({"wall_ms": round(wall, 2), **{k: round(v, 2) for k, v in o["timing"].items()}})
print(json.dumps(out), flush=True)
