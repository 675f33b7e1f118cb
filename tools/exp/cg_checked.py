"""Experiment: the CG iteration with the reference's stopping tests on the device (cgls_fused check_every=True)
against benchmark mode (check_every=False), bench.py's configs[2] scene (1M Gaussians SH 3, one 1080p view,
projected SH-rest layout).  Host-timed calls of 10 iterations, each mode alternately; under
`rocprofv3 --kernel-trace` the calls are separated by 20 ms idle so tools/exp/cg_trace.py sees one run per call.
    python tools/exp/cg_checked.py [--reps 6]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--P", type=int, default=1_000_000)
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem, cgls_fused  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402

dev = torch.device("cuda", 0)
bg = torch.zeros(3)
pert = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1)
g2 = torch.Generator().manual_seed(2)
with torch.no_grad():
    pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
    pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
pert.to(dev)
cams = [c.to(dev) for c in orbit_cameras(1, 1920, 1080, seed=1)]
vp = LMProblem(pert, cams, bg, device=dev)
vp.evaluate()
cams[0].original_image = vp.views[0].color.clamp(0, 1).clone()
del vp, pert
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(dev)
prob = LMProblem(model, cams, bg, device=dev, sh_projection="auto")
prob.evaluate()
g = prob.rhs(prob.zeros())
for _ in range(20):  # clocks
    cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=False)
torch.cuda.synchronize()
out = {"unchecked_ms": [], "checked_ms": [], "info": None}
for _ in range(a.reps):
    for mode in (False, True):
        time.sleep(0.02)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, info = cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=mode)
        torch.cuda.synchronize()
        out["checked_ms" if mode else "unchecked_ms"].append(round(1e3 * (time.perf_counter() - t0), 3))
        if mode:
            out["info"] = {k: v for k, v in info.items() if k != "residuals"}
print(json.dumps(out), flush=True)
