"""Experiment helper: head rows per Gaussian at the bench config (1M Gaussians SH 3, one 1080p view) and the
load balance of k_gather_lm's per-thread row sums (a block of 256 consecutive Gaussians waits for its longest
row run).  python tools/exp/row_stats.py"""
import json
import os
import sys

import torch

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gaussian-splatting-lm_amd")]
from gslm import _lib  # noqa: E402
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.lm import LMProblem  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402

W, H, P = 1920, 1080, 1_000_000
cams = orbit_cameras(1, W, H, seed=1)
model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to("cuda")
prob = LMProblem(model, [c.to("cuda") for c in cams], torch.zeros(3))
prob.evaluate()
vr = prob.views[0]
N = vr.N
gy, gx = (H + 15) // 16, (W + 15) // 16
pl = torch.zeros(N, dtype=torch.int32, device="cuda")
rg = torch.zeros(gy * gx * 2, dtype=torch.int32, device="cuda")
tiles = torch.zeros(P, dtype=torch.int32, device="cuda")
nc = torch.zeros(H * W, dtype=torch.int32, device="cuda")
_lib.check(_lib.lib.gslm_inspect(vr.geom.data_ptr(), P, vr.binning.data_ptr(), N, H, W, vr.image.data_ptr(),
                                 pl.data_ptr(), rg.data_ptr(), tiles.data_ptr(), None, nc.data_ptr(), None,
                                 _lib.stream_handle()))
torch.cuda.synchronize()
pad = torch.zeros(gy * 16, gx * 16, dtype=torch.int64, device="cuda")
pad[:H, :W] = nc.view(H, W).long()
neff = pad.view(gy, 16, gx, 16).amax(dim=(1, 3)).reshape(-1)
r = rg.view(-1, 2).long()
# tile id of every list position, and its position inside the tile's range
tid = torch.repeat_interleave(torch.arange(r.shape[0], device="cuda"), r[:, 1] - r[:, 0])
pos = torch.arange(N, device="cuda") - r[tid, 0]
head = pos < neff[tid]
gid = (pl.long() & ((1 << 28) - 1))[head]
h = torch.bincount(gid, minlength=P).double()
t = tiles.double()
out = {"N": N, "head_rows": int(h.sum()), "gaussians_with_rows": int((h > 0).sum())}
for name, x in (("head_rows", h), ("tiles", t)):
    xb = x[: (P // 256) * 256].view(-1, 256)
    mx, mean = xb.max(dim=1).values, xb.mean(dim=1)
    q = torch.quantile(x[x > 0], torch.tensor([0.5, 0.9, 0.99, 0.999], dtype=torch.float64, device="cuda"))
    out[name] = {"mean_nonzero": float(x[x > 0].mean()), "quantiles_50_90_99_999": [float(v) for v in q],
                 "max": float(x.max()),
                 "block_serial_over_balanced": float(mx.sum() / mean.sum()),
                 "blocks_with_max_over_64": int((mx > 64).sum()), "blocks": int(xb.shape[0])}
print(json.dumps(out))
