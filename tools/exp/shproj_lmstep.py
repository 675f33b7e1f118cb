"""Experiment: lm_step trajectories with and without the projected SH-rest layout at the bench scene."""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gaussian-splatting-lm_amd")]
import torch
from gslm.cameras import orbit_cameras
from gslm.lm import LMProblem, lm_step, cgls_fused
from gslm.model import synthetic_gaussians
W, H, P = 1920, 1080, 1_000_000
cams = [c.to("cuda") for c in orbit_cameras(1, W, H, seed=1)]
pert = synthetic_gaussians(P, 3, seed=0, s0=0.005, n_cams=1)
g2 = torch.Generator().manual_seed(2)
with torch.no_grad():
    pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
    pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
    pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
pert.to("cuda")
gp = LMProblem(pert, cams, torch.zeros(3)); gp.evaluate()
cams[0].original_image = gp.views[0].color.clamp(0, 1).clone()
del gp, pert
for proj in (False, True):
    m = synthetic_gaussians(P, 3, seed=0, s0=0.005, n_cams=1).to("cuda")
    for it in range(3):
        out = lm_step(m, cams, cams, torch.zeros(3), max_iter=10, restart_iter=10, check_every=True, sh_projection=proj)
        print(proj, it, out["start_loss"], out["final_val_loss"], out["best_alpha"], out["cg"]["iters"],
              [f"{r:.6e}" for r in out["cg"]["residuals"][:3]], out["cg"]["residuals"][-1])
    # the CG solution itself on a fresh model
    m = synthetic_gaussians(P, 3, seed=0, s0=0.005, n_cams=1).to("cuda")
    pr = LMProblem(m, cams, torch.zeros(3), sh_projection=proj); pr.evaluate()
    x, _ = cgls_fused(pr, pr.rhs(pr.zeros()), max_iter=10, restart_iter=10, check_every=False)
    x = pr.expand(x)
    if proj:
        print("rel diff of x", float((x.double() - x0.double()).norm() / x0.double().norm()))
    else:
        x0 = x.clone()
