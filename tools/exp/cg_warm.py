"""Experiment helper: the CG iteration time of bench.py's problem (1M Gaussians SH 3, one 1080p view, projected
SH-rest layout) as a function of how the GPU was kept busy before it: after 2 s idle, untimed full forwards or CG
calls for a while, then cgls_fused(10) timed three times.  python tools/exp/cg_warm.py"""
import json
import os
import sys
import time

import torch

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gaussian-splatting-lm_amd")]
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem, cgls_fused  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402

dev = torch.device("cuda", 0)
W, H, P = 1920, 1080, 1_000_000
cams = orbit_cameras(1, W, H, seed=1)
pert = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1)
g2 = torch.Generator().manual_seed(2)
with torch.no_grad():
    pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
    pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
    pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
pert.to(dev)
gp = LMProblem(pert, [c.to(dev) for c in cams], torch.zeros(3), device=dev)
gp.evaluate()
cams[0].original_image = gp.views[0].color.clamp(0, 1).clone()
del gp, pert
model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(dev)
prob = LMProblem(model, cams, torch.zeros(3), device=dev, sh_projection="auto")
prob.evaluate()
g = prob.rhs(prob.zeros())
torch.cuda.synchronize()


def timed(k=10, warm=5):
    cgls_fused(prob, g, max_iter=warm, restart_iter=warm, check_every=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cgls_fused(prob, g, max_iter=k, restart_iter=k, check_every=False)
    torch.cuda.synchronize()
    return round(1e3 * (time.perf_counter() - t0) / k, 4)


from gslm.params import raw_gaussians  # noqa: E402

graw = raw_gaussians(model)
vr = prob.views[0]


def settle_forwards(sec):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < sec:
        for _ in range(8):
            vr.forward(graw, prob.stream)
        torch.cuda.synchronize()


def settle_cg(sec):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < sec:
        cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=False)
        torch.cuda.synchronize()


out = {}
for name, fn, sec in (("forwards_150ms", settle_forwards, 0.15), ("forwards_500ms", settle_forwards, 0.5),
                      ("cg_150ms", settle_cg, 0.15), ("none", None, 0.0)):
    time.sleep(2.0)
    if fn:
        fn(sec)
    out[name] = [timed() for _ in range(3)]
print(json.dumps(out))
