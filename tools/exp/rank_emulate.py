"""Experiment: one rank's kernels of an n-GPU LM CG iteration (Gaussian-sharded exchange), emulated on one GPU.

    python tools/exp/rank_emulate.py [--ranks 8] [--P 1000000] [--steps 20] [--per 1] [--W 1920 --H 1080]
    configs[4] (5M Gaussians, 32 4K views over n ranks): --P 5000000 --W 3840 --H 2160 --per $((32 / n)) --ranks n

Rank r of n (--per views per rank; configs[3]: one 1080p view per rank): tangent records of its Gaussian shard (P / n)
for all n per views,
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
ap.add_argument("--per", type=int, default=1, help="views per rank")
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--no-n1", action="store_true", help="skip the single-view N = 1 reference iterations")
a = ap.parse_args()
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem, cgls_fused  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.parallel import GaussianShardedOperator  # noqa: E402

dev = torch.device("cuda", 0)
n, r = a.ranks, a.rank
cams = [c.to(dev) for c in orbit_cameras(n * a.per, a.W, a.H, seed=1)]
for c in cams:
    c.original_image = torch.rand(3, a.H, a.W, device=dev)
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=n * a.per).to(dev)
out = {"ranks": n, "rank": r, "P": a.P, "views_per_rank": a.per, "W": a.W, "H": a.H}


def cg_ms(prob, g, steps):
    cgls_fused(prob, g, max_iter=3, restart_iter=3, check_every=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cgls_fused(prob, g, max_iter=steps, restart_iter=steps, check_every=False)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


mine = cams[r * a.per:(r + 1) * a.per]
local = LMProblem(model, mine, torch.zeros(3), device=dev, sh_projection=False)
local.evaluate()
op = GaussianShardedOperator(local, all_cams=cams, emulate=(r, n))
op._exchange_flags()
# visible fraction of the shard's Gaussians per view (the flags' top bit): what compressing the exchange to visible
# Gaussians (batch_render.py:124 viewcount > 0) could save
fl = op._buffers()["flags"]
out["visible_frac"] = [round(float(((fl[k] >> 31) != 0).float().mean()), 4) for k in range(fl.shape[0])]
gs = op.rhs(op.zeros())
t_warm = time.perf_counter()
while time.perf_counter() - t_warm < 1.0:  # clocks: ~1 s of CG load first
    cg_ms(op, gs, 5)
out["emulated_rank_cg_ms"] = cg_ms(op, gs, a.steps)
out["emulated_rank_stage_ms"] = op.stage_times(gs, reps=a.steps)
# each of the per view groups' two all-to-alls moves 32 B per Gaussian of the table in and out, (n - 1) / n of it
# across links
out["bytes_per_rank_all_to_all"] = {"trec": a.per * 32 * op.S * (n - 1), "screen": a.per * 32 * op.S * (n - 1)}
out["rest_views"] = op.rest_views
out["num_rendered"] = [vr.N for vr in local.views]
del op, local
torch.cuda.empty_cache()
for proj in (() if a.no_n1 else (True, False)):
    p1 = LMProblem(model, [cams[r]], torch.zeros(3), device=dev, sh_projection=proj)
    p1.evaluate()
    g1 = p1.rhs(p1.zeros())
    cg_ms(p1, g1, 10)
    out["n1_cg_ms_" + ("projected" if proj else "full")] = cg_ms(p1, g1, a.steps)
    del p1, g1
print(json.dumps(out), flush=True)
