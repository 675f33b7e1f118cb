"""Experiment: the wave imbalance of the VJP pass's block-synchronous batches (vjp_tile: 128 list entries per batch,
block barriers around each), at the bench config (1M Gaussians SH3, 1080p), on the CPU oracle.

Per sampled tile and quadrant wave w, the visits are the list positions below the wave's largest n_contrib whose
alpha region reaches a pixel of the quadrant (a lower bound of the quadrant cull's visits).  Compares the wave
iterations of the per-batch barrier schedule (sum over batches of the busiest wave) with free-running waves (the
busiest wave's total) and with perfect balance (the mean).
    python tools/exp/batch_imbalance.py [tile stride, default 23]"""
import sys
import numpy as np
import torch
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from oracle import torch_raster as tr  # noqa: E402

torch.set_num_threads(8)
W, H = 1920, 1080
m = synthetic_gaussians(1_000_000, 3, seed=0, s0=0.005, device="cpu")
cam = orbit_cameras(1, W, H, seed=1)[0]
st = tr.settings_from_camera(cam, torch.zeros(3), 3)
with torch.no_grad():
    pre = tr.preprocess(m.get_xyz, torch.zeros_like(m.get_xyz), m.get_opacity, m.get_features, None, m.get_scaling,
                        m.get_rotation, None, st)
pl, ts, rg = tr.binning(pre)
pl, rg = pl.numpy(), rg.numpy()
xy, conic, opac = pre["xy"].numpy().astype(np.float32), pre["conic"].numpy().astype(np.float32), pre["opacity"].numpy().astype(np.float32)
gx, gy = pre["grid"]
tiles = range(0, gx * gy, int(sys.argv[1]) if len(sys.argv) > 1 else 23)
S = dict(sync=0.0, free=0.0, mean=0.0, tiles=0)
for t in tiles:
    s, e = int(rg[t, 0]), int(rg[t, 1])
    if e <= s:
        continue
    tx, ty = t % gx, t // gx
    L = pl[s:e]
    yy, xx = np.meshgrid(np.arange(16) + 16 * ty, np.arange(16) + 16 * tx, indexing="ij")
    inside = (xx < W) & (yy < H)
    px, py = xx.reshape(-1).astype(np.float32), yy.reshape(-1).astype(np.float32)
    dx = xy[L, 0][None, :] - px[:, None]
    dy = xy[L, 1][None, :] - py[:, None]
    a, b, c = conic[L, 0][None], conic[L, 1][None], conic[L, 2][None]
    power = np.float32(-0.5) * (a * dx * dx + c * dy * dy) - b * dx * dy
    alpha = np.minimum(np.float32(0.99), opac[L][None] * np.exp(power))
    ok = (power <= 0) & (alpha >= 1 / 255.0)
    om = np.where(ok, 1 - alpha, 1.0)
    Tinc = np.cumprod(om.astype(np.float64), axis=1)
    stop = ok & (Tinc < 1e-4)
    n = len(L)
    idx = np.arange(n)[None]
    first = np.where(stop, idx, n).min(axis=1)
    contrib = ok & (idx < first[:, None])
    last = np.where(contrib, idx + 1, 0).max(axis=1)
    last[~inside.reshape(-1)] = 0
    reach = ok & inside.reshape(-1)[:, None]
    q = ((yy.reshape(-1) - 16 * ty) >= 8) * 2 + ((xx.reshape(-1) - 16 * tx) >= 8)
    wm = [int(last[q == w].max()) for w in range(4)]
    neff = max(wm)
    if neff == 0:
        continue
    hit = np.stack([reach[q == w].any(axis=0) & (np.arange(n) < wm[w]) for w in range(4)])[:, :neff]
    bidx = (neff - 1 - np.arange(neff)) // 128  # batches of 128 from the back, as vjp_tile
    hw = np.stack([np.bincount(bidx, weights=hit[w], minlength=bidx.max() + 1) for w in range(4)])
    S["sync"] += hw.max(axis=0).sum()
    S["free"] += hw.sum(axis=1).max()
    S["mean"] += hw.mean(axis=0).sum()
    S["tiles"] += 1
S.update(sync_over_free=S["sync"] / S["free"], sync_over_mean=S["sync"] / S["mean"], free_over_mean=S["free"] / S["mean"])
print(S)
