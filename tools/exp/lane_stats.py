"""Experiment: where the tile passes' lanes go at the bench config (1M Gaussians SH3, 1080p), on the CPU oracle.

For a strided sample of tiles: per pixel the exact valid set (power <= 0, alpha >= 1/255, position < n_contrib),
then, per 8x8 quadrant wave, the visits the current schedule makes (entries whose alpha region reaches a
quadrant pixel, positions below the wave's max n_contrib) and why their invalid lanes are invalid; and the
iteration count of alternative schedules."""
import os
import sys

import numpy as np
import torch

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
tot = dict(visits=0, lanes=0, valid=0, inv_alpha=0, inv_last=0, inv_outside=0, sub_iters=0, sub_lane_visits=0,
           pair_iters=0, ent=0, vis_ent=0, half_iters=0, blend_visits=0, fwd_visits=0)
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
    reach = ok & inside.reshape(-1)[:, None]  # alpha region reaches the pixel (exact; quad_mask is conservative)
    valid = reach & (idx < last[:, None])
    tot["ent"] += n
    tot["vis_ent"] += int(last.max())
    pix = np.arange(256).reshape(16, 16)
    for q in range(4):
        qp = pix[8 * (q >> 1):8 * (q >> 1) + 8, 8 * (q & 1):8 * (q & 1) + 8].reshape(-1)
        wmax = last[qp].max()
        hit = reach[qp].any(axis=0) & (np.arange(n) < wmax)
        nv = int(hit.sum())
        tot["visits"] += nv
        tot["lanes"] += 64 * nv
        tot["blend_visits"] += int(valid[qp].any(axis=0).sum())  # visits some lane of the quadrant blends
        # the forward blend (no n_contrib yet): hits until every lane has stopped (the stopping entry included),
        # the whole list when some pixel never reaches T < 1e-4
        fst = np.where(inside.reshape(-1)[qp], first[qp], -1)
        fend = fst.max() if (fst < n).all() else n - 1
        tot["fwd_visits"] += int((reach[qp].any(axis=0) & (np.arange(n) <= fend)).sum())
        v = valid[qp][:, hit]
        tot["valid"] += int(v.sum())
        r = reach[qp][:, hit]
        ins = inside.reshape(-1)[qp][:, None]
        tot["inv_outside"] += int((~ins).sum() * nv)
        tot["inv_alpha"] += int((~r & ins).sum())
        tot["inv_last"] += int((r & ~v).sum())
        # 4x4 sub-quadrants processed by 16-lane groups, each on its own hit list: wave iterations = max count
        cnts = []
        for sq in range(4):
            sp = qp.reshape(8, 8)[4 * (sq >> 1):4 * (sq >> 1) + 4, 4 * (sq & 1):4 * (sq & 1) + 4].reshape(-1)
            smax = last[sp].max()
            cnts.append(int((reach[sp].any(axis=0) & (np.arange(n) < smax)).sum()))
        tot["sub_iters"] += max(cnts)
        # 8x4 halves processed by 32-lane groups
        cnth = []
        for hh in range(2):
            sp = qp.reshape(8, 8)[4 * hh:4 * hh + 4, :].reshape(-1)
            smax = last[sp].max()
            cnth.append(int((reach[sp].any(axis=0) & (np.arange(n) < smax)).sum()))
        tot["half_iters"] += max(cnth)
    # two quadrants per wave (16x8 halves): union visits
    for hq in (0, 1):
        hp = pix[8 * hq:8 * hq + 8, :].reshape(-1)
        wmax = last[hp].max()
        tot["pair_iters"] += int((reach[hp].any(axis=0) & (np.arange(n) < wmax)).sum())
print({k: v for k, v in tot.items()})
lanes = tot["lanes"]
print(f"valid lane fraction {tot['valid'] / lanes:.3f}; invalid: alpha region {tot['inv_alpha'] / lanes:.3f}, "
      f"past own n_contrib {tot['inv_last'] / lanes:.3f}, outside image {tot['inv_outside'] / lanes:.3f}")
print(f"visits per wave (quadrant) schedule {tot['visits']}; 4x4 sub-quadrant groups {tot['sub_iters']} "
      f"({tot['sub_iters'] / tot['visits']:.3f}); 16x8 half-tile waves {tot['pair_iters']} x2 px/lane")
print(f"8x4 half groups (32 lanes) {tot['half_iters']} ({tot['half_iters'] / tot['visits']:.3f})")
print(f"visits some lane blends {tot['blend_visits']} ({tot['blend_visits'] / tot['visits']:.3f} of the exact-reach schedule)")
print(f"forward blend visits {tot['fwd_visits']} ({tot['fwd_visits'] / tot['visits']:.3f} of the JVP/VJP schedule)")
print(f"visited entries / N_dup {tot['vis_ent'] / tot['ent']:.3f}")
