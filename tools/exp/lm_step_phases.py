"""Experiment: host-timed phases of one LM step at the bench config (1M, SH3, 1080p, 1 view)."""
import os, sys, time, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from gslm.lm import LMProblem, cgls_fused, update_params
W, H = 1920, 1080
cams = [c.to("cuda") for c in orbit_cameras(1, W, H, seed=1)]
m = synthetic_gaussians(1_000_000, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to("cuda")
for c in cams:
    c.original_image = torch.rand(3, H, W, device="cuda")
def T():
    torch.cuda.synchronize(); return time.perf_counter()
for rep in range(3):
    t0 = T(); prob = LMProblem(m, cams, torch.zeros(3)); t1 = T()
    prob.evaluate(); t2 = T()
    g = prob.rhs(prob.zeros()); t3 = T()
    s, info = cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=True); t4 = T()
    s2, _ = cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=False); t5 = T()
    val = LMProblem(m, cams, torch.zeros(3)); t6 = T()
    for _ in range(7):
        float(val.evaluate())
    t7 = T()
    print(f"rep {rep}: ctor {1e3*(t1-t0):.2f} eval {1e3*(t2-t1):.2f} rhs {1e3*(t3-t2):.2f} cg(check) {1e3*(t4-t3):.2f} "
          f"cg(nocheck) {1e3*(t5-t4):.2f} val-ctor {1e3*(t6-t5):.2f} 7 evals {1e3*(t7-t6):.2f}  iters {info['iters']}")
