"""Experiment helper: dump the bench view's sorted lists and render records for offline analysis
of tile-pass work (quadrant hit patterns, per-pixel blend counts)."""
import os, sys, ctypes, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
from gslm import _lib
from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from gslm.lm import LMProblem
W, H, P = 1920, 1080, 1_000_000
cams = orbit_cameras(1, W, H, seed=1)
m = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to("cuda")
prob = LMProblem(m, [c.to("cuda") for c in cams], torch.zeros(3))
prob.evaluate()
vr = prob.views[0]
N = vr.N
ntiles = ((W + 15) // 16) * ((H + 15) // 16)
pl = torch.zeros(N, dtype=torch.int32, device="cuda")
rg = torch.zeros(ntiles * 2, dtype=torch.int32, device="cuda")
nc = torch.zeros(H * W, dtype=torch.int32, device="cuda")
rec = torch.zeros(P * 12, dtype=torch.float32, device="cuda")
_lib.check(_lib.lib.gslm_inspect(vr.geom.data_ptr(), P, vr.binning.data_ptr(), N, H, W, vr.image.data_ptr(),
                                 pl.data_ptr(), rg.data_ptr(), None, None, nc.data_ptr(), rec.data_ptr(),
                                 _lib.stream_handle()))
torch.cuda.synchronize()
r = rec.view(P, 12)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "geom.npz"), pl=pl.cpu().numpy(), ranges=rg.cpu().numpy(),
                    n_contrib=nc.cpu().numpy(), rec=r[:, :8].cpu().numpy(), tq=r[:, 11].cpu().numpy())
print("N", N)
