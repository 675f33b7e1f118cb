"""Experiment: the line search's validation loss (gslm.lm.LossEvaluator) at bench.py's scene -- 1M Gaussians, SH 3,
V 1080p views -- by stream count, and against LMProblem.evaluate (the residual path).
    python tools/exp/val_time.py [--views 50] [--reps 5]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--views", type=int, default=50)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--streams", type=int, nargs="*", default=[1, 2, 3, 4])
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--readback", action="store_true", help="also time the per-batch count read-back path (device_count=False)")
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LossEvaluator  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402

dev = torch.device("cuda", 0)
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu").to(dev)
cams = orbit_cameras(a.views, 1920, 1080, seed=5)
for c in cams:
    c.to(dev)
    c.original_image = torch.rand(3, 1080, 1920, device=dev)
out = {"views": a.views, "P": a.P, "batch": a.batch}
ref = None
runs = [(ns, True) for ns in a.streams] + ([(ns, False) for ns in a.streams] if a.readback else [])
for ns, dc in runs:
    ev = LossEvaluator(model, cams, torch.zeros(3), device=dev, streams=ns, batch=max(a.batch, ns), device_count=dc)
    v = float(ev.evaluate())  # sorts the depth orders
    ref = v if ref is None else ref
    for _ in range(2):
        ev.evaluate()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        ev.evaluate()
    torch.cuda.synchronize()
    tag = f"streams{ns}" + ("" if dc else "_readback")
    out[f"{tag}_ms_per_view"] = 1e3 * (time.perf_counter() - t0) / a.reps / a.views
    out[f"{tag}_rel_diff"] = abs(v - ref) / abs(ref)
    del ev
print(json.dumps(out), flush=True)
