"""Experiment: the line search's final point (train_jvp.py:278-279) through the kept union lists (LossEvaluator.
evaluate_final) against its exact render (evaluate()), at bench.py's lm_step scene (1M Gaussians SH 3, 50 1080p
validation views, val_batch 8): wall time of each after evaluate_points(keep=True) over six points.
    python tools/exp/final_eval.py [--reps 5]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--views", type=int, default=50)
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LossEvaluator, param_snapshot, update_params  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.params import ParamLayout  # noqa: E402

dev = torch.device("cuda", 0)
bg = torch.zeros(3)
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(dev)
val = [c.to(dev) for c in orbit_cameras(a.views, 1920, 1080, seed=5)]
for i, c in enumerate(val):
    c.original_image = torch.rand(3, 1080, 1920, generator=torch.Generator().manual_seed(100 + i)).to(dev)
lay = ParamLayout(a.P, 16, model._exposure.shape[0])
s = torch.zeros(lay.numel, device=dev)
v = lay.views(s)
gen = torch.Generator(device=dev).manual_seed(3)
for name, sd in (("features_dc", 0.02), ("features_rest", 0.005), ("scaling", 0.05), ("rotation", 0.05),
                 ("opacity", 0.2)):
    v[name].copy_(sd * torch.randn(v[name].shape, generator=gen, device=dev))
ev = LossEvaluator(model, val, bg, device=dev, batch=8)
alpha = 2.0
update_params(model, lay, s, alpha, skip_xyz=True)
sets = []
for _ in range(6):
    sets.append(param_snapshot(model))
    update_params(model, lay, s, 0.5 * alpha - alpha, skip_xyz=True)
    alpha *= 0.5
update_params(model, lay, s, 1.0 - alpha, skip_xyz=True)
out = {"P": a.P, "views": a.views}


def wall(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps, r


ev.evaluate()  # depth orders, exact-path workspaces
out["points_keep_ms"], _ = wall(lambda: ev.evaluate_points(sets, keep=True), 2)
out["final_union_ms"], lu = wall(lambda: ev.evaluate_final(), a.reps)
out["final_exact_ms"], lx = wall(lambda: ev.evaluate(), a.reps)
out["equal"] = float(lu) == float(lx)
out["final_exact_views"] = len(ev.final_exact)
out["points_nokeep_ms"], _ = wall(lambda: ev.evaluate_points(sets), 2)
print(json.dumps(out), flush=True)
