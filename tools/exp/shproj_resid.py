"""Experiment: how far the full-layout CG solution's SH-rest rows are from the view's span, and the normal-
equation residual of both solutions under the full operator (bench scene, first LM step)."""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gaussian-splatting-lm_amd")]
import torch
from gslm.cameras import orbit_cameras
from gslm.lm import LMProblem, cgls_fused
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
m = synthetic_gaussians(P, 3, seed=0, s0=0.005, n_cams=1).to("cuda")
pf = LMProblem(m, cams, torch.zeros(3), sh_projection=False); pf.evaluate()
pp = LMProblem(m, cams, torch.zeros(3), sh_projection=True); pp.evaluate()
gf = pf.rhs(pf.zeros()); gpj = pp.rhs(pp.zeros())
a, b = pf.full_layout.offsets["features_rest"]


def offspan(v):
    e = pp.expand(pp.project(v))
    return float((v[a:b] - e[a:b]).norm() / v[a:b].norm())


print("g off-span", offspan(gf), "g vs expand(gp)", float((pp.expand(gpj) - gf).norm() / gf.norm()))
gf2 = gf * (1 + 1e-7 * torch.randn_like(gf))
for iters in (5, 6, 7, 8, 9, 10):
    xf, inf = cgls_fused(pf, gf, max_iter=iters, restart_iter=iters, check_every=True)
    xn, inn = cgls_fused(pf, gf2, max_iter=iters, restart_iter=iters, check_every=True)
    xp, inp = cgls_fused(pp, gpj, max_iter=iters, restart_iter=iters, check_every=True)
    xe = pp.expand(xp)
    res = lambda x: float((pf.matvec(x, pf.zeros()) - gf).norm() / gf.norm())
    print(iters, "proj-full", float((xe - xf).norm() / xf.norm()), "noisy-full", float((xn - xf).norm() / xf.norm()),
          "resid full/noisy/proj", res(xf), res(xn), res(xe))
print("monitor full ", inf["residuals"])
print("monitor noisy", inn["residuals"])
print("monitor proj ", inp["residuals"])
