"""Experiment: locate the SSIM-mode LM product mismatch (J v image, u, per view)."""
import os, sys, ctypes, numpy as np, torch
import torch.autograd.forward_ad as fwAD
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd"), os.path.join(ROOT, "tests")]
import test_gpu_ssim as T
from gslm.lm import LMProblem
from oracle.lm_ref import OracleLMProblem
from oracle import torch_raster as tr
from gslm.params import GROUPS
ds, m, cams = T._load()
prob = LMProblem(m, cams, torch.zeros(3), ssim=True)
prob.evaluate(); prob.rhs(prob.zeros())
v = torch.from_numpy(ds["v"]).cuda()
y = prob.matvec(v, prob.zeros())
torch.cuda.synchronize()
# oracle
mc = m.__class__(m.active_sh_degree)
mc.set_params(*[t.detach().cpu() for t in (m._xyz, m._features_dc, m._features_rest, m._scaling, m._rotation, m._opacity, m._exposure)])
mc.active_sh_degree = m.active_sh_degree
cc = [c for c in T._load()[2]]
for c in cc: c.to("cpu")
op = OracleLMProblem(mc, cc, torch.zeros(3), ssim=True)
views = op.layout.views(v.cpu())
leaves = op._leaves()
with torch.no_grad(), fwAD.dual_level():
    (mc._xyz, mc._features_dc, mc._features_rest, mc._scaling, mc._rotation, mc._opacity, mc._exposure) = [
        fwAD.make_dual(t.detach(), views[gname].to(t.dtype)) for t, gname in zip(leaves, GROUPS)]
    jvs = []
    for c in cc:
        img, _, _, raw = tr.render_model(mc, c, torch.zeros(3))
        jvs.append(fwAD.unpack_dual(raw).tangent)
    (mc._xyz, mc._features_dc, mc._features_rest, mc._scaling, mc._rotation, mc._opacity, mc._exposure) = leaves
for b in range(len(cc)):
    g = prob._jv[b].cpu()
    r = jvs[b]
    print("view", b, "jv rel err", ((g - r).abs().max() / r.abs().max()).item(), "max", r.abs().max().item())
yo = op.matvec(v.cpu(), op.zeros())
print("Av rel (oracle vs golden)", np.abs(yo.numpy() - ds["Av"]).max() / np.abs(ds["Av"]).max())
print("Av rel (gpu vs oracle)", (np.abs(y.cpu().numpy() - yo.numpy()).max() / np.abs(yo.numpy()).max()))
o = prob.layout.offsets
for gname in GROUPS:
    a, bb = o[gname]
    if bb > a:
        e = np.abs(y.cpu().numpy()[a:bb] - yo.numpy()[a:bb]).max(); s = np.abs(yo.numpy()[a:bb]).max()
        print(gname, e, s)
