"""Experiment: the Gaussian-sharded exchange's kernels on one GPU (one rank: the all-to-alls are copies).

    python tools/exp/gshard_time.py [--views 8] [--P 1000000] [--reps 5]

One rank holding V 1080p views runs the pipeline a rank of a V-GPU job runs per product, but over all P
Gaussians instead of P / V: gslm_tangent_views (V views), RENDER | SCREEN per view, gslm_gather_screen (V views).
The per-kernel times (rocprofv3 --kernel-trace --stats around this script) divided by V are the per-rank costs
of the tangent / gather side at V GPUs; k_render_matvec is one view's as at N = 1."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--views", type=int, default=8)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.parallel import GaussianShardedOperator  # noqa: E402

dev = torch.device("cuda", 0)
cams = [c.to(dev) for c in orbit_cameras(a.views, 1920, 1080, seed=1)]
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=a.views).to(dev)
prob = LMProblem(model, cams, torch.zeros(3), device=dev, sh_projection=False)
prob.evaluate()
g = prob.rhs(prob.zeros())
op = GaussianShardedOperator(prob, all_cams=prob.cams)
op._exchange_flags()
v = op.shard(g)
y = op.zeros()
op.matvec(v, y)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    op.matvec(v, y)
torch.cuda.synchronize()
print(f"views {a.views} P {a.P}: sharded-pipeline product {1e3 * (time.perf_counter() - t0) / a.reps:.3f} ms")
