"""Experiment: one rank's kernels of an n-GPU LM CG iteration (Gaussian-sharded exchange), emulated on one GPU.

    python tools/exp/rank_emulate.py [--ranks 8] [--P 1000000] [--steps 20]

Rank r of n (one 1080p view per rank, configs[3]): tangent records of its Gaussian shard (P / n) for all n views,
the tile pass of its own view over the exchanged [P][8] table, the screen row sums, the shard's gather over n views,
the CG update on the shard -- with every collective replaced by a local copy of the same shape
(GaussianShardedOperator(emulate=(r, n))).  Prints per-stage times (HIP events) and the CG iteration without
communication, next to the single-view N = 1 iteration (projected and full layouts)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem, cgls_fused  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.parallel import GaussianShardedOperator  # noqa: E402

dev = torch.device("cuda", 0)
n, r = a.ranks, a.rank
cams = [c.to(dev) for c in orbit_cameras(n, 1920, 1080, seed=1)]
for c in cams:
    c.original_image = torch.rand(3, 1080, 1920, device=dev)
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=n).to(dev)
out = {"ranks": n, "rank": r, "P": a.P}


def cg_ms(prob, g, steps):
    cgls_fused(prob, g, max_iter=3, restart_iter=3, check_every=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cgls_fused(prob, g, max_iter=steps, restart_iter=steps, check_every=False)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


local = LMProblem(model, [cams[r]], torch.zeros(3), device=dev, sh_projection=False)
local.evaluate()
op = GaussianShardedOperator(local, all_cams=cams, emulate=(r, n))
op._exchange_flags()
gs = op.rhs(op.zeros())
for _ in range(30):  # clocks
    cg_ms(op, gs, 10)
out["emulated_rank_cg_ms"] = cg_ms(op, gs, a.steps)
out["emulated_rank_stage_ms"] = op.stage_times(gs, reps=a.steps)
out["bytes_per_rank_all_to_all"] = {"trec": 32 * op.S * n * (n - 1) // n, "screen": 32 * op.S * n * (n - 1) // n}
del op, local
torch.cuda.empty_cache()
for proj in (True, False):
    p1 = LMProblem(model, [cams[r]], torch.zeros(3), device=dev, sh_projection=proj)
    p1.evaluate()
    g1 = p1.rhs(p1.zeros())
    cg_ms(p1, g1, 10)
    out["n1_cg_ms_" + ("projected" if proj else "full")] = cg_ms(p1, g1, a.steps)
    del p1, g1
print(json.dumps(out), flush=True)
