"""Experiment: the line search's union-list stages for ONE 1080p view on one stream (HIP events), at bench.py's configs[2]
scene (1M Gaussians SH 3, the six points of a 10-iteration CGLS step), next to the exact per-point render:
  preprocess_views (6 sets, depth space), union_geometry, union_binning, the six slot blends / the all-sets blend.
    python tools/exp/union_kernels.py [--reps 10]"""
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
from gslm.lm import LMProblem, cgls_fused, param_snapshot, update_params  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.params import ParamLayout, raw_gaussians  # noqa: E402

dev = torch.device("cuda", 0)
bg = torch.zeros(3)
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu").to(dev)
cam = orbit_cameras(1, 1920, 1080, seed=1)[0].to(dev)
cam.original_image = torch.rand(3, 1080, 1920, device=dev)
val = orbit_cameras(1, 1920, 1080, seed=5)[0].to(dev)
gt = torch.rand(3, 1080, 1920, device=dev)
prob = LMProblem(model, [cam], bg, device=dev, sh_projection="auto")
prob.evaluate()
s, _ = cgls_fused(prob, prob.rhs(prob.zeros()), max_iter=10, restart_iter=10, check_every=True)
s = prob.expand(s)
del prob
full = ParamLayout(a.P, 16, model._exposure.shape[0])
alpha = 2.0
update_params(model, full, s, alpha, skip_xyz=True)
sets = []
for _ in range(6):
    sets.append(param_snapshot(model))
    update_params(model, full, s, 0.5 * alpha - alpha, skip_xyz=True)
    alpha *= 0.5
gs = [raw_gaussians(t) for t in sets]
P, n = a.P, 6
vw = _lib.view_from_camera(val, bg, 3)
st = _lib.stream_handle(dev)
nb = lib.gslm_geom_bytes(P)
geoms = [_lib.u8(nb, dev) for _ in range(n)]
ugeom = _lib.u8(nb, dev)
order = torch.empty(P, dtype=torch.int32, device=dev)
pos = torch.empty(P, dtype=torch.int32, device=dev)
check(lib.gslm_preprocess_ordered(ctypes.byref(vw), ctypes.byref(gs[0]), geoms[0].data_ptr(), nb, None,
                                  order.data_ptr(), 1, st))
check(lib.gslm_depth_positions(order.data_ptr(), P, pos.data_ptr(), st))
vws = (_lib.GslmView * 1)(vw)
pp = (ctypes.c_void_p * 1)(pos.data_ptr())
ge = (ctypes.c_void_p * n)(*[g.data_ptr() for g in geoms])
losses = torch.zeros(n, dtype=torch.float64, device=dev)
scr = torch.empty(lib.gslm_loss_sets_scratch_bytes(n, 1080, 1920) // 8 + 1, dtype=torch.float64, device=dev)
box = {}


def pre():
    for k in range(n):
        g1 = (ctypes.c_void_p * 1)(geoms[k].data_ptr())
        check(lib.gslm_preprocess_views(vws, 1, ctypes.byref(gs[k]), g1, nb, pp, st))


def ugeo():
    check(lib.gslm_union_geometry(ctypes.byref(vw), P, ge, n, nb, ugeom.data_ptr(), nb, st))


def ubin():
    N = box["N"]
    check(lib.gslm_union_binning(ctypes.byref(vw), P, ugeom.data_ptr(), box["bin"].data_ptr(), box["bin"].numel(), N, ge,
                                 n, nb, st))


def blends():
    N = box["N"]
    for k in range(n):
        check(lib.gslm_rasterize_loss_slot(ctypes.byref(vw), P, geoms[k].data_ptr(), nb, box["bin"].data_ptr(),
                                           box["bin"].numel(), N, k, n, gt.data_ptr(), None, scr.data_ptr(), scr.numel() * 8,
                                           losses.data_ptr() + 8 * k, 0, st))


def blend_sets():
    N = box["N"]
    lp = (ctypes.c_void_p * n)(*[losses.data_ptr() + 8 * k for k in range(n)])
    check(lib.gslm_rasterize_loss_sets(ctypes.byref(vw), P, ge, n, 0, nb, box["bin"].data_ptr(), box["bin"].numel(), N,
                                       gt.data_ptr(), None, scr.data_ptr(), scr.numel() * 8, lp, 0, st))


pre()
ugeo()
Nt = ctypes.c_int64()
check(lib.gslm_num_rendered(ugeom.data_ptr(), P, ctypes.byref(Nt), st))
box["N"] = int(Nt.value)
box["bin"] = _lib.u8(lib.gslm_union_binning_bytes(box["N"], 1080, 1920), dev)
ubin()
out = {"P": P, "N_union": box["N"]}


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


out["preprocess_6_sets_ms"] = ev_ms(pre)
out["union_geometry_ms"] = ev_ms(ugeo)
out["union_binning_ms"] = ev_ms(ubin)
out["blends_6_slot_ms"] = ev_ms(blends)
out["blend_all_sets_ms"] = ev_ms(blend_sets)


# the exact per-point render of the same view (preprocess with the cached order, binning, blend + loss)
def exact():
    for k in range(n):
        check(lib.gslm_preprocess_ordered(ctypes.byref(vw), ctypes.byref(gs[k]), geoms[k].data_ptr(), nb, None,
                                          order.data_ptr(), 2, st))
        N = box["Ne"][k]
        check(lib.gslm_rasterize_loss(ctypes.byref(vw), P, geoms[k].data_ptr(), box["ebin"].data_ptr(),
                                      box["ebin"].numel(), N, gt.data_ptr(), None, scr.data_ptr(), scr.numel() * 8,
                                      losses.data_ptr() + 8 * k, 0, st))


box["Ne"] = []
for k in range(n):
    check(lib.gslm_preprocess_ordered(ctypes.byref(vw), ctypes.byref(gs[k]), geoms[k].data_ptr(), nb, None,
                                      order.data_ptr(), 2, st))
    check(lib.gslm_num_rendered(geoms[k].data_ptr(), P, ctypes.byref(Nt), st))
    box["Ne"].append(int(Nt.value))
box["ebin"] = _lib.u8(lib.gslm_binning_bytes(max(box["Ne"]), 1080, 1920), dev)
out["exact_6_points_ms"] = ev_ms(exact)
print(json.dumps(out), flush=True)
