"""Experiment: LM vectors of the bench scene (loss, J^T b, A v, 10-iteration CG) with the library GSLM_LIB
points at, saved to gpurun_out/<tag>.pt, to compare two library builds.
    GSLM_LIB=.../libgslm.so python tools/exp/dump_lm_vectors.py <tag> [proj]"""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gaussian-splatting-lm_amd")]
import torch
from gslm.cameras import orbit_cameras
from gslm.lm import LMProblem, cgls_fused
from gslm.model import synthetic_gaussians
tag = sys.argv[1]
proj = len(sys.argv) > 2 and sys.argv[2] == "proj"
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
pr = LMProblem(m, cams, torch.zeros(3), sh_projection=proj)
loss = float(pr.evaluate())
g = pr.rhs(pr.zeros())
torch.cuda.synchronize()
print("NaN in g after rhs", int(torch.isnan(g).sum()), "inf", int(torch.isinf(g).sum()))
bad = torch.nonzero(~torch.isfinite(g)).flatten()
if bad.numel():
    views = pr.layout.views(g)
    a0 = pr.layout.offsets["features_rest"][0]
    gi = int((bad[0] - a0) // 45)
    for name, t in views.items():
        if name != "exposure":
            print(name, t[gi].flatten().tolist()[:12])
    print("tiles", int(pr.views[0].radii[gi]), "xyz", m._xyz[gi].tolist())
    g2 = pr.rhs(pr.zeros(), fused=False)
    print("drop-in rhs finite:", bool(torch.isfinite(g2).all()), "rest of that Gaussian", g2[a0 + 45 * gi: a0 + 45 * gi + 6].tolist())
gen = torch.Generator(device="cuda").manual_seed(3)
v = torch.randn(pr.layout.numel, device="cuda", generator=gen)
for grp in ("xyz", "exposure"):
    a, b = pr.layout.offsets[grp]
    v[a:b] = 0
y = pr.matvec(v, pr.zeros())
torch.cuda.synchronize()
print("NaN in g after matvec", int(torch.isnan(g).sum()), "in y", int(torch.isnan(y).sum()))
x, info = cgls_fused(pr, g, max_iter=10, restart_iter=10, check_every=True)
for name, (a, b) in pr.layout.offsets.items():
    seg = g[a:b]
    nn = int(torch.isnan(seg).sum())
    if nn:
        w = (b - a) // pr.layout.P if name != "exposure" else 1
        idx = torch.nonzero(torch.isnan(seg)).flatten()[:8] // max(w, 1)
        print("NaN in g", name, nn, "first Gaussians", idx.tolist())
print(tag, loss, float(g.norm()), float(y.norm()), float(x.norm()), info["residuals"][-1])
