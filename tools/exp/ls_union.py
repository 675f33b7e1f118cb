"""Experiment: the line search's union binning (LossEvaluator.evaluate_points) against the exact per-point renders, at
bench.py's configs[2] scene: 1M Gaussians SH 3, one 1080p training view, V 1080p validation views with the GT rendered
from the perturbed model, the step s from 10 CGLS iterations.  Reports the list lengths (each point's N against the
union's) and the wall time of both paths; run under rocprofv3 --kernel-trace --stats for the per-kernel split.
    python tools/exp/ls_union.py [--views 50] [--reps 3] [--mode both|union|exact]"""
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
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--mode", default="both")
ap.add_argument("--streams", type=int, default=8)
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem, LossEvaluator, cgls_fused, param_snapshot, update_params  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.params import ParamLayout  # noqa: E402

dev = torch.device("cuda", 0)
bg = torch.zeros(3)
pert = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu")
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
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu").to(dev)
prob = LMProblem(model, cams, bg, device=dev, sh_projection="auto")
prob.evaluate()
s, _ = cgls_fused(prob, prob.rhs(prob.zeros()), max_iter=10, restart_iter=10, check_every=True)
s = prob.expand(s)
del prob
full = ParamLayout(a.P, 16, model._exposure.shape[0])
saved = [t.detach().clone() for t in model.params()]


def restore():
    with torch.no_grad():
        for t, s0 in zip(model.params(), saved):
            t.copy_(s0)


out = {"views": a.views, "P": a.P}
ev_x = LossEvaluator(model, val, bg, device=dev, streams=a.streams)
ev_u = LossEvaluator(model, val, bg, device=dev, streams=a.streams)
# the points and, per point, every view's exact pair count
alpha = 2.0
update_params(model, full, s, alpha, skip_xyz=True)
sets, exact, counts = [], [], []
for _ in range(6):
    sets.append(param_snapshot(model))
    exact.append(float(ev_x.evaluate()))
    counts.append(list(ev_x.num_rendered))
    update_params(model, full, s, 0.5 * alpha - alpha, skip_xyz=True)
    alpha *= 0.5
got = [float(x) for x in ev_u.evaluate_points(sets)]
out["equal"] = got == exact
NU = list(ev_u.union_counts)
out["N_point_mean"] = [sum(c) / len(c) for c in counts]
out["N_union_mean"] = sum(NU) / len(NU)
out["N_union_over_max_point"] = sum(NU) / sum(max(c[i] for c in counts) for i in range(len(NU)))
restore()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / a.reps


if a.mode in ("both", "exact"):
    out["exact_6_points_ms"] = timed(lambda: [ev_x.evaluate() for _ in range(6)])
if a.mode in ("both", "union"):
    ev_u.loss_sets = 1
    out["union_6_points_ms"] = timed(lambda: ev_u.evaluate_points(sets))  # the default: per-set blends
    ev_u.loss_sets = 8
    out["union_6_points_all_sets_blend_ms"] = timed(lambda: ev_u.evaluate_points(sets))
    ev_u.loss_sets = 1
    out["snapshot_ms"] = timed(lambda: [param_snapshot(model) for _ in range(6)])
print(json.dumps(out), flush=True)
