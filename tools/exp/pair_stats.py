"""Experiment: how many of a quadrant wave's tile-pass visits could share one iteration with the next visit, at the
bench config (1M Gaussians SH3, 1080p), on the CPU oracle.

Two consecutive visits of a wave whose valid lane sets (power <= 0, alpha >= 1/255, position < n_contrib) are
disjoint touch no common pixel, so each lane can run whichever of the two entries it blends: per pixel the same
operations in the same order.  Counts the wave iterations of a greedy pairing schedule (and of greedy groups of up
to K mutually disjoint consecutive visits) against the one-visit-per-iteration schedule."""
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
tiles = range(0, gx * gy, int(sys.argv[1]) if len(sys.argv) > 1 else 41)
KS = (2, 3, 4)
tot = dict(visits=0, empty=0, valid=0, **{f"g{k}": 0 for k in KS}, **{f"g{k}_nonempty": 0 for k in KS})
hist = np.zeros(65, np.int64)
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
    valid = reach & (idx < last[:, None])
    pix = np.arange(256).reshape(16, 16)
    for q in range(4):
        qp = pix[8 * (q >> 1):8 * (q >> 1) + 8, 8 * (q & 1):8 * (q & 1) + 8].reshape(-1)
        wmax = last[qp].max()
        hit = reach[qp].any(axis=0) & (np.arange(n) < wmax)
        v = valid[qp][:, hit]  # [64, nv] in visit order
        nv = v.shape[1]
        tot["visits"] += nv
        cnt = v.sum(axis=0)
        tot["valid"] += int(cnt.sum())
        tot["empty"] += int((cnt == 0).sum())
        np.add.at(hist, cnt, 1)
        for K in KS:
            for drop_empty in (False, True):
                vv = v[:, cnt > 0] if drop_empty else v
                i, it = 0, 0
                while i < vv.shape[1]:
                    u = vv[:, i].copy()
                    j = i + 1
                    while j < vv.shape[1] and j - i < K and not (u & vv[:, j]).any():
                        u |= vv[:, j]
                        j += 1
                    it += 1
                    i = j
                tot[f"g{K}" + ("_nonempty" if drop_empty else "")] += it
print(tot)
V = tot["visits"]
print(f"valid lane fraction {tot['valid'] / (64 * V):.3f}; visits with no valid lane {tot['empty'] / V:.3f}")
for K in KS:
    print(f"greedy groups of <= {K} disjoint consecutive visits: {tot[f'g{K}'] / V:.3f} of the iterations; "
          f"empty visits dropped first: {tot[f'g{K}_nonempty'] / V:.3f}")
print("valid lanes per visit, deciles:", np.searchsorted(np.cumsum(hist) / hist.sum(), np.linspace(0.1, 0.9, 9)))
