"""Experiment: the LM step's final point on the kept union lists (LossEvaluator.evaluate_final) against the exact
render (evaluate), and evaluate_points with and without keep, at bench.py's configs[2] line-search scene (1M Gaussians,
50 1080p validation views, a 10-iteration CGLS step).
    python tools/exp/final_ab.py [--reps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--views", type=int, default=50)
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem, LossEvaluator, cgls_fused, param_snapshot, update_params  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.params import ParamLayout  # noqa: E402

dev = torch.device("cuda", 0)
bg = torch.zeros(3)
P = 1_000_000
pert = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu")
g2 = torch.Generator().manual_seed(2)
with torch.no_grad():
    pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
    pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
    pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
pert.to(dev)
cams = [c.to(dev) for c in orbit_cameras(1, 1920, 1080, seed=1)]
val = [c.to(dev) for c in orbit_cameras(a.views, 1920, 1080, seed=5)]
for chunk in [cams] + [val[i:i + 8] for i in range(0, len(val), 8)]:
    vp = LMProblem(pert, chunk, bg, device=dev)
    vp.evaluate()
    for c, vr in zip(chunk, vp.views):
        c.original_image = vr.color.clamp(0, 1).clone()
    del vp
del pert
model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu").to(dev)
prob = LMProblem(model, cams, bg, device=dev, sh_projection="auto")
prob.evaluate()
s, _ = cgls_fused(prob, prob.rhs(prob.zeros()), max_iter=10, restart_iter=10, check_every=True)
s = prob.expand(s)
del prob
full = ParamLayout(P, 16, model._exposure.shape[0])
ev = LossEvaluator(model, val, bg, device=dev)
alpha = 2.0
update_params(model, full, s, alpha, skip_xyz=True)
sets = []
for _ in range(6):
    sets.append(param_snapshot(model))
    update_params(model, full, s, 0.5 * alpha - alpha, skip_xyz=True)
    alpha *= 0.5
update_params(model, full, s, 1.0 - alpha, skip_xyz=True)  # the final point at best_alpha = 1


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        r = fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / a.reps, r


out = {}
for keep in (False, True, False, True):
    ev.evaluate_points(sets, keep=keep)
    out[f"points_keep{int(keep)}_ms"], _ = timed(lambda: [float(x) for x in ev.evaluate_points(sets, keep=keep)])
ev.evaluate_points(sets, keep=True)
out["final_union_ms"], fu = timed(lambda: float(ev.evaluate_final(model)))
out["final_exact_ms"], fx = timed(lambda: float(ev.evaluate()))
out["final_union_ms_2"], _ = timed(lambda: float(ev.evaluate_final(model)))
out["equal"] = fu == fx
out["fallbacks"] = len(ev.final_fallbacks)
print(json.dumps(out), flush=True)
