"""Experiment: how many quadrant bits the round-2 rectangle test and the round-3 band test keep (float32 numpy
restatements of gslm_kernels.hpp's quad_mask, bench scene subset).  python tools/exp/quadmask_count.py [P]"""
import sys
import numpy as np
import torch

sys.path[:0] = [".", "gaussian-splatting-lm_amd"]
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from oracle import torch_raster as tr  # noqa: E402

f32 = np.float32
P = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
m = synthetic_gaussians(P, 3, seed=0, s0=0.005)
cam = orbit_cameras(1, 1920, 1080, seed=1)[0]
st = tr.settings_from_camera(cam, torch.zeros(3), 3)
with torch.no_grad():
    pre = tr.preprocess(m.get_xyz, torch.zeros_like(m.get_xyz), m.get_opacity, m.get_features, None, m.get_scaling,
                        m.get_rotation, None, st)
vis = (pre["tiles_touched"] > 0).numpy()
xy = pre["xy"].numpy()[vis].astype(f32)
con = pre["conic"].numpy()[vis].astype(f32)
op = pre["opacity"].numpy()[vis].reshape(-1).astype(f32)
rect = [r.numpy()[vis] for r in pre["rect"]] if isinstance(pre["rect"], (tuple, list)) else None
tq = (2.0 * np.log(255.0 * op.astype(np.float64)) * 1.02 + 1e-4).astype(f32)
A, B, C = con[:, 0], con[:, 1], con[:, 2]
e = f32(32 * 5.9604644775390625e-8) * (A + C)
a, c = A - e, C - e
det = a * c - B * B
ok = (a > 0) & (c > 0) & (det > f32(1e-6) * a * c) & (op * 255 > 1)


def q_lower(x, y, b):
    ax, by, bx, cy = a_ * x, b * y, b * x, c_ * y
    val = (ax + 2 * by) * x + cy * y
    mag = (np.abs(ax) + 2 * np.abs(by)) * np.abs(x) + np.abs(cy * y)
    grad = 2 * (np.abs(ax) + np.abs(by) + np.abs(bx) + np.abs(cy))
    return val - (f32(2e-6) * mag + grad * dpos_ + f32(1e-5))


def rect_qmin(x0, x1, y0, y1, b):
    in_x = (x0 <= 0) & (x1 >= 0)
    in_y = (y0 <= 0) & (y1 >= 0)
    best = np.full(x0.shape, np.inf, dtype=f32)
    xe = np.where(x0 > 0, x0, x1)
    v1 = q_lower(xe, np.minimum(np.maximum(nbc_ * xe, y0), y1), b)
    best = np.where(~in_x, v1, best)
    ye = np.where(y0 > 0, y0, y1)
    v2 = q_lower(np.minimum(np.maximum(nba_ * ye, x0), x1), ye, b)
    best = np.where(~in_y, np.minimum(best, v2), best)
    return np.where(in_x & in_y, f32(0), best)


def band(ya, yb):
    y0 = np.maximum(ya, -ydom)
    y1 = np.minimum(yb, ydom)
    hit = y0 <= y1
    yh = np.minimum(np.maximum(yr, y0), y1)
    yl = np.minimum(np.maximum(-yr, y0), y1)
    sh = np.sqrt(np.maximum(ta - det_ * yh * yh, 0))
    sl = np.sqrt(np.maximum(ta - det_ * yl * yl, 0))
    bh, bl = b_ * yh, b_ * yl
    hi = (sh - bh) * ia + f32(1e-4) * (np.abs(bh) + sh) * ia + sqm + f32(0.01)
    lo = -(sl + bl) * ia - (f32(1e-4) * (np.abs(bl) + sl) * ia + sqm + f32(0.01))
    return hit, lo, hi


old_bits = new_bits = entries = exact_bits = 0
PXO = np.meshgrid(np.arange(8, dtype=f32), np.arange(8, dtype=f32))  # pixel offsets in a quadrant
H, W = 1080, 1920
gx_, gy_ = xy[:, 0], xy[:, 1]
for k in np.nonzero(ok)[0][:20000]:
    r = (pre["radii"].numpy()[vis][k])
    x0t = max(0, int((gx_[k] - r) / 16)); x1t = min(120, int((gx_[k] + r + 15) / 16))
    y0t = max(0, int((gy_[k] - r) / 16)); y1t = min(68, int((gy_[k] + r + 15) / 16))
    a_, c_, b_ = a[k], c[k], B[k]
    nba_, nbc_ = -b_ / a_, -b_ / c_
    dpos_ = f32(4e-7) * (abs(gx_[k]) + abs(gy_[k]) + 8192)
    det_ = det[k]; ta = tq[k] * a_; ia = f32(1) / a_
    ydom = np.sqrt(ta / det_) * f32(1.0001) + f32(0.01)
    yr = -b_ * np.sqrt(tq[k] * c_ / det_) / c_
    sqm = np.sqrt(f32(1e-6) * ta) * ia
    for ty in range(y0t, y1t):
        for tx in range(x0t, x1t):
            entries += 1
            bx, by = f32(tx * 16) - gx_[k], f32(ty * 16) - gy_[k]
            for s in range(4):
                xa, ya = bx + 8 * (s & 1), by + 8 * (s >> 1)
                xa, ya = np.array([xa], f32), np.array([ya], f32)
                if not (rect_qmin(xa, xa + 7, ya, ya + 7, b_)[0] > tq[k]):
                    old_bits += 1
                hit, lo, hi = band(ya, ya + 7)
                if hit[0] and xa[0] <= hi[0] and xa[0] + 7 >= lo[0]:
                    new_bits += 1
                    # exact: some pixel centre of the quadrant with power <= 0 and alpha >= 1/255 (float32)
                    dx = (gx_[k] - (f32(tx * 16 + 8 * (s & 1)) + PXO[0])).astype(f32)
                    dy = (gy_[k] - (f32(ty * 16 + 8 * (s >> 1)) + PXO[1])).astype(f32)
                    pw = f32(-0.5) * (A[k] * dx * dx + C[k] * dy * dy) - B[k] * dx * dy
                    al = np.minimum(f32(0.99), op[k] * np.exp(pw))
                    inside = ((f32(tx * 16 + 8 * (s & 1)) + PXO[0]) < W) & ((f32(ty * 16 + 8 * (s >> 1)) + PXO[1]) < H)
                    if np.any((pw <= 0) & (al >= f32(1 / 255.0)) & inside):
                        exact_bits += 1
print(f"entries {entries}: old kept {old_bits} ({old_bits / entries:.3f}/entry), new kept {new_bits} "
      f"({new_bits / entries:.3f}/entry), exact (a pixel centre reached) {exact_bits} ({exact_bits / entries:.3f}/entry)")
