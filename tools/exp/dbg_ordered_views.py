"""Debug: gslm_preprocess_ordered (order_mode 2) against gslm_preprocess_ordered_views on the same depth order, per SH
degree: geometry workspaces byte-compared and the records / tile counts through gslm_inspect."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402
from gslm import _lib  # noqa: E402
from gslm._lib import check, lib  # noqa: E402
from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.params import raw_gaussians  # noqa: E402

for D in (3, 2, 1, 0):
    m = synthetic_gaussians(3000, D, seed=0, s0=0.03).to("cuda")
    cam = orbit_cameras(1, 56, 40, seed=7)[0].to("cuda")
    v = _lib.view_from_camera(cam, torch.zeros(3), m.active_sh_degree)
    g = raw_gaussians(m)
    P = g.P
    nb = lib.gslm_geom_bytes(P)
    st = _lib.stream_handle()
    order = torch.empty(P, dtype=torch.int32, device="cuda")
    ga = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    gb = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    gc = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    check(lib.gslm_preprocess_ordered(ctypes.byref(v), ctypes.byref(g), gc.data_ptr(), nb, None, order.data_ptr(), 1, st))
    check(lib.gslm_preprocess_ordered(ctypes.byref(v), ctypes.byref(g), ga.data_ptr(), nb, None, order.data_ptr(), 2, st))
    vws = (_lib.GslmView * 1)(v)
    ge = (ctypes.c_void_p * 1)(gb.data_ptr())
    od = (ctypes.c_void_p * 1)(order.data_ptr())
    check(lib.gslm_preprocess_ordered_views(vws, 1, ctypes.byref(g), ge, nb, od, st))
    torch.cuda.synchronize()
    d = (ga != gb).nonzero().flatten()
    recs = []
    for w in (ga, gb):
        rec = torch.zeros(P * 12, dtype=torch.float32, device="cuda")
        tiles = torch.zeros(P, dtype=torch.int32, device="cuda")
        check(lib.gslm_inspect(w.data_ptr(), P, None, 0, 40, 56, None, None, None, tiles.data_ptr(), None, None,
                               rec.data_ptr(), st))
        torch.cuda.synchronize()
        recs.append((rec.view(P, 12).cpu(), tiles.cpu()))
    vis = recs[0][1] > 0
    rd = (recs[0][0][vis] != recs[1][0][vis]).any(dim=1)
    print(f"D={D} active={m.active_sh_degree} M={1 + m._features_rest.shape[1]} bytes differing {d.numel()} "
          f"(first offsets {d[:8].tolist()}), tiles equal {torch.equal(recs[0][1], recs[1][1])}, "
          f"visible {int(vis.sum())}, records differing {int(rd.sum())}", flush=True)
    if rd.any():
        k = int(rd.nonzero()[0])
        print("  first:", recs[0][0][vis][k].tolist(), "\n  views:", recs[1][0][vis][k].tolist(), flush=True)
