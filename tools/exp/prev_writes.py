"""Experiment: what bounds k_preprocess_views in depth space (the line search's per-set render records).
The same launch (1M Gaussians SH 3, 1080p views) with the real depth positions (scattered 64-B record writes) and
with identity positions (coalesced writes), for 1 and 8 views per launch.
    python tools/exp/prev_writes.py [--reps 10]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--P", type=int, default=1_000_000)
a = ap.parse_args()
from gslm import _lib  # noqa: E402
from gslm._lib import check, lib  # noqa: E402
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.params import raw_gaussians  # noqa: E402

dev = torch.device("cuda", 0)
bg = torch.zeros(3)
P = a.P
model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu").to(dev)
cams = orbit_cameras(8, 1920, 1080, seed=5)
vws = [_lib.view_from_camera(c.to(dev), bg, 3) for c in cams]
g = raw_gaussians(model)
st = _lib.stream_handle(dev)
nb = lib.gslm_geom_bytes(P)
geoms = [_lib.u8(nb, dev) for _ in range(8)]
pos = []
for k in range(8):
    order = torch.empty(P, dtype=torch.int32, device=dev)
    p = torch.empty(P, dtype=torch.int32, device=dev)
    check(lib.gslm_preprocess_ordered(ctypes.byref(vws[k]), ctypes.byref(g), geoms[k].data_ptr(), nb, None,
                                      order.data_ptr(), 1, st))
    check(lib.gslm_depth_positions(order.data_ptr(), P, p.data_ptr(), st))
    pos.append(p)
ident = torch.arange(P, dtype=torch.int32, device=dev)


def run(nv, positions):
    vv = (_lib.GslmView * nv)(*vws[:nv])
    pp = (ctypes.c_void_p * nv)(*[positions[k].data_ptr() for k in range(nv)])
    ge = (ctypes.c_void_p * nv)(*[geoms[k].data_ptr() for k in range(nv)])
    check(lib.gslm_preprocess_views(vv, nv, ctypes.byref(g), ge, nb, pp, st))


def ev_ms(fn):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.reps


out = {"P": P}
for nv in (1, 8):
    out[f"depth_pos_{nv}v_ms"] = ev_ms(lambda: run(nv, pos))
    out[f"identity_{nv}v_ms"] = ev_ms(lambda: run(nv, [ident] * 8))
# index-space preprocess of one view (k_preprocess_dma + depth sort + scans) for scale
out["preprocess_ordered_reuse_ms"] = ev_ms(lambda: check(lib.gslm_preprocess_ordered(
    ctypes.byref(vws[0]), ctypes.byref(g), geoms[0].data_ptr(), nb, None, pos[0].data_ptr(), 2, st)))
print(json.dumps(out), flush=True)
