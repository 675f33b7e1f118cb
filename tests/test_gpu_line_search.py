"""GPU: the line search with one binning per validation view and LM step (ABI 8, include/gslm.h "shared binning";
gslm.lm.LossEvaluator.evaluate_points).

train_jvp.py:262-277 renders every validation view at six points theta + alpha s with xyz masked (:221-227).  The
union path bins each view once over the union of the points' rects and blends every point through that list with
its own per-entry quadrant bits (carried through the tile sort).  The claim is exactness, so every comparison here is `==` against the exact renders
(gslm_rasterize_loss with the point's own binning, LossEvaluator.evaluate), not a tolerance:
  * each of the six points' losses, with steps large enough that radii and rects change between points, at 320x208
    and at 1080p / 200k Gaussians, over several batch and stream counts;
  * alpha masks, and points that cull Gaussians others keep (empty quadrant masks, zero-area rects);
  * lm_step(line_search="union") against lm_step(line_search="exact"): trace, best_alpha, final loss and the
    stepped parameters bitwise, and the reference-solver golden (test_gpu_lm_step.py) through the union path.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _scene(P=20000, W=320, H=208, nviews=5, seed=0, D=3, s0=0.01):
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    m = synthetic_gaussians(P, D, seed=seed, s0=s0).to("cuda")
    cams = orbit_cameras(nviews, W, H, seed=7)
    for i, c in enumerate(cams):
        c.original_image = torch.rand(3, H, W, generator=torch.Generator().manual_seed(60 + i))
        c.to("cuda")
    return m, cams


def _step(m, seed=3, scale=1.0):
    """A step on every group but xyz, large enough that scales (hence radii and rects) and opacities (hence quadrant
    masks) differ between the line-search points."""
    from gslm.params import ParamLayout
    P, K = m._xyz.shape[0], 1 + m._features_rest.shape[1]
    lay = ParamLayout(P, K, m._exposure.shape[0])
    s = torch.zeros(lay.numel, device="cuda")
    v = lay.views(s)
    gen = torch.Generator(device="cuda").manual_seed(seed)
    for name, sd in (("features_dc", 0.1), ("features_rest", 0.02), ("scaling", 0.25), ("rotation", 0.2),
                     ("opacity", 0.8)):
        v[name].copy_(scale * sd * torch.randn(v[name].shape, generator=gen, device="cuda"))
    return lay, s


def _points(m, lay, s, ev_exact):
    """The six points as lm_step forms them, with each point's exact loss and pair counts."""
    from gslm.lm import param_snapshot, update_params
    alpha = 2.0
    update_params(m, lay, s, alpha, skip_xyz=True)
    sets, exact, counts = [], [], []
    for _ in range(6):
        sets.append(param_snapshot(m))
        exact.append(float(ev_exact.evaluate()))
        counts.append(list(ev_exact.num_rendered))
        update_params(m, lay, s, 0.5 * alpha - alpha, skip_xyz=True)
        alpha *= 0.5
    return sets, exact, counts, alpha


@pytest.mark.parametrize("batch,streams", [(2, 2), (8, 8), (1, 1)])
def test_evaluate_points_equal_exact_renders(batch, streams):
    from gslm.lm import LossEvaluator
    m, cams = _scene()
    lay, s = _step(m)
    ev_x = LossEvaluator(m, cams, torch.zeros(3), batch=batch, streams=streams)
    ev_u = LossEvaluator(m, cams, torch.zeros(3), batch=batch, streams=streams)
    sets, exact, counts, alpha = _points(m, lay, s, ev_x)
    got = [float(x) for x in ev_u.evaluate_points(sets)]
    assert got == exact
    # the union list holds every point's list and is longer than some (the test moves rects)
    for i, N in enumerate(ev_u.union_counts):
        assert N >= max(c[i] for c in counts)
    assert any(N > min(c[i] for c in counts) for i, N in enumerate(ev_u.union_counts))
    # the blends over groups of sets (all sets in one pass; pairs and triples, with a ragged last group) give the same
    # losses as the per-set blends (the default)
    for k in (8, 2, 4):
        ev_u.loss_sets = k
        assert [float(x) for x in ev_u.evaluate_points(sets)] == exact, k
    ev_u.loss_sets = 3
    # fewer points, and a second LM step on the same evaluator (buffers reused, depth orders cached)
    assert [float(x) for x in ev_u.evaluate_points(sets[2:5])] == exact[2:5]
    sets2, exact2, _, _ = _points(m, lay, s, ev_x)
    assert [float(x) for x in ev_u.evaluate_points(sets2)] == exact2


def test_evaluate_points_batch_above_eight_views():
    """A batch of more views than one gslm_preprocess_views call takes (8): the batch's depth-space preprocesses go in
    chunks of 8 (lm_step(val_batch=12) raised before round 5's fix)."""
    from gslm.lm import LossEvaluator
    m, cams = _scene(P=5000, nviews=11)
    lay, s = _step(m)
    ev_x = LossEvaluator(m, cams, torch.zeros(3), batch=11, streams=3)
    ev_u = LossEvaluator(m, cams, torch.zeros(3), batch=11, streams=3)
    sets, exact, _, _ = _points(m, lay, s, ev_x)
    assert [float(x) for x in ev_u.evaluate_points(sets)] == exact


@pytest.mark.parametrize("D", [0, 1])
def test_evaluate_points_equal_exact_renders_low_sh_degree(D):
    """SH degree 0 (no SH-rest leaf: the preprocess cannot stage SH rows and runs its unstaged form, which must still
    write the records at their depth positions -- ADVICE r04) and degree 1."""
    from gslm.lm import LossEvaluator
    m, cams = _scene(D=D)
    lay, s = _step(m)
    ev_x = LossEvaluator(m, cams, torch.zeros(3), batch=2, streams=2)
    ev_u = LossEvaluator(m, cams, torch.zeros(3), batch=2, streams=2)
    sets, exact, _, _ = _points(m, lay, s, ev_x)
    assert [float(x) for x in ev_u.evaluate_points(sets)] == exact
    ev_u.loss_sets = 8
    assert [float(x) for x in ev_u.evaluate_points(sets)] == exact


def test_evaluate_points_with_alpha_masks_and_culled_sets():
    """Alpha masks on the residual, and points where some Gaussians are culled (opacity driven below 1/255, so their
    quadrant masks are empty, and scales driven to zero-area rects) while other points keep them."""
    from gslm.lm import LossEvaluator, param_snapshot
    m, cams = _scene(nviews=3)
    masks = [(torch.rand(1, c.image_height, c.image_width, generator=torch.Generator().manual_seed(9 + i)) > 0.3).float()
             for i, c in enumerate(cams)]
    ev_x = LossEvaluator(m, cams, torch.zeros(3), batch=2, streams=2, alpha_masks=masks)
    ev_u = LossEvaluator(m, cams, torch.zeros(3), batch=2, streams=2, alpha_masks=masks)
    sets, exact = [], []
    for k in range(4):
        with torch.no_grad():
            m._opacity[k::4] -= 12.0      # below the 1/255 cut: reaches no pixel
            m._scaling[(k + 1)::4] += 0.7  # larger footprints
            m._scaling[(k + 2)::9] -= 9.0  # vanishing footprints
        sets.append(param_snapshot(m))
        exact.append(float(ev_x.evaluate()))
    assert [float(x) for x in ev_u.evaluate_points(sets)] == exact


def test_evaluate_points_1080p_200k():
    """At the bench's resolution (1080p, 200k Gaussians at the bench's footprint scale, 3 views): every point equal."""
    from gslm.lm import LossEvaluator
    m, cams = _scene(P=200_000, W=1920, H=1080, nviews=3, s0=0.005)
    lay, s = _step(m, seed=11, scale=0.5)
    ev_x = LossEvaluator(m, cams, torch.zeros(3))
    ev_u = LossEvaluator(m, cams, torch.zeros(3))
    sets, exact, _, _ = _points(m, lay, s, ev_x)
    assert [float(x) for x in ev_u.evaluate_points(sets)] == exact


def test_lm_step_union_equals_exact_line_search():
    from gslm.cameras import orbit_cameras
    from gslm.lm import lm_step
    from gslm.model import synthetic_gaussians
    outs, params = [], []
    for ls in ("union", "exact"):
        m = synthetic_gaussians(30000, 3, seed=0, s0=0.01).to("cuda")
        cams = orbit_cameras(1, 320, 208, seed=1)
        val = orbit_cameras(6, 320, 208, seed=4)
        for i, c in enumerate(cams + val):
            c.original_image = torch.rand(3, 208, 320, generator=torch.Generator().manual_seed(80 + i))
            c.to("cuda")
        outs.append(lm_step(m, cams, val, torch.zeros(3), max_iter=10, restart_iter=10, line_search=ls,
                            val_at_start=True))
        params.append([t.detach().clone() for t in (m._features_dc, m._features_rest, m._scaling, m._rotation,
                                                     m._opacity, m._xyz)])
    u, x = outs
    assert u["line_search"] == "union" and x["line_search"] == "exact"
    assert u["trace"] == x["trace"]
    assert u["best_alpha"] == x["best_alpha"]
    assert u["final_val_loss"] == x["final_val_loss"]
    assert u["val_start_loss"] == x["val_start_loss"]
    for a, b in zip(*params):
        assert torch.equal(a, b)


def test_union_lm_step_matches_reference_golden():
    """The reference-solver golden of test_gpu_lm_step.py, through the union line search (lm_step's default)."""
    import test_gpu_lm_step as t
    d, L, m, cams, val = t._setup()
    from gslm.lm import lm_step
    out = lm_step(m, cams, val, torch.zeros(3), max_iter=10, restart_iter=10, check_every=True, line_search="union")
    assert out["line_search"] == "union"
    assert out["best_alpha"] == float(L["ten_best_alpha"])
    losses = np.array([v for _, v in out["trace"]])
    ref = L["ten_trace_loss"]
    assert np.abs(losses - ref).max() <= 1e-4 * ref.max()
    fin = float(L["ten_final_val_loss"])
    assert abs(out["final_val_loss"] - fin) <= 1e-4 * fin


@pytest.mark.parametrize("nviews", [1, 3, 8])
def test_preprocess_views_equals_per_view_preprocess(nviews):
    """gslm_preprocess_views (one pass over the Gaussians for several views) writes each view's records, tile counts
    and rects bitwise as gslm_preprocess does (ragged P, mixed image sizes); with depth positions, the same records at
    each Gaussian's depth position (the rect slot zero when culled)."""
    import ctypes
    from gslm import _lib
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    from gslm.params import raw_gaussians
    lib = _lib.lib
    m = synthetic_gaussians(10_007, 3, seed=1, s0=0.02).to("cuda")
    g = raw_gaussians(m)
    cams = orbit_cameras(nviews, 96, 80, seed=3)
    if nviews > 1:
        cams[1] = orbit_cameras(2, 130, 57, seed=9)[1]
    views = (_lib.GslmView * nviews)(*[_lib.view_from_camera(c, torch.zeros(3), 3) for c in cams])
    nb = lib.gslm_geom_bytes(g.P)
    a = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(nviews)]
    b = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(nviews)]
    for k in range(nviews):
        assert lib.gslm_preprocess(ctypes.byref(views[k]), ctypes.byref(g), a[k].data_ptr(), nb, None, None) == 0
    ge = (ctypes.c_void_p * nviews)(*[t.data_ptr() for t in b])
    assert lib.gslm_preprocess_views(views, nviews, ctypes.byref(g), ge, nb, None, None) == 0, lib.gslm_last_error()
    torch.cuda.synchronize()
    P = g.P
    rec = 64 * P  # render records [P][4] float4
    keys = 4 * P
    for k in range(nviews):
        ra, rb = a[k][:rec].view(torch.float32).view(P, 16), b[k][:rec].view(torch.float32).view(P, 16)
        tiles_a = a[k][_off(rec, keys):_off(rec, keys) + keys].view(torch.int32)
        tiles_b = b[k][_off(rec, keys):_off(rec, keys) + keys].view(torch.int32)
        assert torch.equal(tiles_a, tiles_b)
        vis = tiles_a > 0
        assert int(vis.sum()) > 0
        assert torch.equal(ra[vis].view(torch.int32), rb[vis].view(torch.int32))
        # rects (the depth keys are not comparable: gslm_preprocess's depth sort reuses their buffer)
        r0 = _off(rec, keys) + _al(keys)
        rect_a = a[k][r0:r0 + 8 * P].view(torch.int64)
        rect_b = b[k][r0:r0 + 8 * P].view(torch.int64)
        assert torch.equal(rect_a[vis], rect_b[vis])
    # depth space: each view's records at its Gaussians' depth positions, the rect slot zero when culled
    orders, poss, c = [], [], [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(nviews)]
    for k in range(nviews):
        o = torch.empty(P, dtype=torch.int32, device="cuda")
        assert lib.gslm_preprocess_ordered(ctypes.byref(views[k]), ctypes.byref(g), a[k].data_ptr(), nb, None,
                                           o.data_ptr(), 1, None) == 0
        pos = torch.empty(P, dtype=torch.int32, device="cuda")
        assert lib.gslm_depth_positions(o.data_ptr(), P, pos.data_ptr(), None) == 0
        orders.append(o)
        poss.append(pos)
    pp = (ctypes.c_void_p * nviews)(*[t.data_ptr() for t in poss])
    gc = (ctypes.c_void_p * nviews)(*[t.data_ptr() for t in c])
    assert lib.gslm_preprocess_views(views, nviews, ctypes.byref(g), gc, nb, pp, None) == 0, lib.gslm_last_error()
    torch.cuda.synchronize()
    for k in range(nviews):
        o = orders[k].long()
        assert torch.equal(poss[k].long()[o], torch.arange(P, device="cuda"))  # pos is the order's inverse
        ra = b[k][:rec].view(torch.float32).view(P, 16)
        rc = c[k][:rec].view(torch.float32).view(P, 16)[poss[k].long()]  # back in index order
        tiles = b[k][_off(rec, keys):_off(rec, keys) + keys].view(torch.int32)
        vis = tiles > 0
        assert torch.equal(rc[vis][:, :12].view(torch.int32), ra[vis][:, :12].view(torch.int32))
        r0 = _off(rec, keys) + _al(keys)
        rect = b[k][r0:r0 + 8 * P].view(torch.int64)
        assert torch.equal(rc[vis][:, 12:14].contiguous().view(torch.int64).reshape(-1), rect[vis])
        assert bool((rc[~vis][:, 12:14] == 0).all())


def _al(x):
    return (x + 255) // 256 * 256


def _off(rec, keys):
    """Byte offset of the tile counts in the geometry layout (rec, depth_key, tiles, ...; 256-B aligned, api.hip)."""
    return _al(rec) + _al(keys)


@pytest.mark.parametrize("P", [1, 5, 63, 65, 129])
def test_evaluate_points_tiny_and_ragged(P):
    """The union path at a handful of Gaussians (block tails of the 64-Gaussian duplicate blocks and the 8-item payload
    sort, views where the union list is empty) equals the exact renders."""
    from gslm.lm import LossEvaluator
    m, cams = _scene(P=P, nviews=3, s0=0.05)
    lay, s = _step(m, seed=7)
    ev_x = LossEvaluator(m, cams, torch.zeros(3), batch=2, streams=2)
    ev_u = LossEvaluator(m, cams, torch.zeros(3), batch=2, streams=2)
    sets, exact, _, _ = _points(m, lay, s, ev_x)
    assert [float(x) for x in ev_u.evaluate_points(sets)] == exact


def test_loss_slot_past_the_recorded_set_count_is_nan():
    """ADVICE r04 (ABI 9): gslm_union_binning records the set count its masks were built for; a slot at or past it
    (a caller passing a larger n_sets than the binning's) renders a NaN loss, not a plausible background-only one."""
    import ctypes
    import math
    from gslm import _lib
    from gslm.lm import LossEvaluator, param_snapshot
    lib = _lib.lib
    m, cams = _scene(nviews=1)
    ev = LossEvaluator(m, cams, torch.zeros(3), batch=1, streams=1)
    sets = [param_snapshot(m), param_snapshot(m)]
    got = [float(x) for x in ev.evaluate_points(sets)]
    assert got[0] == got[1] == float(ev.evaluate())
    # the evaluator's last union binning (batch position 0, view 0) was built for n = 2
    sl, binning, vw = ev.uslots[0][0], ev.ubins[0], ev.views[0]
    P, N = m._xyz.shape[0], ev.union_counts[0]
    loss = torch.zeros(1, dtype=torch.float64, device="cuda")
    scr = ev.loss_scratch[0]
    for slot, want_nan in ((1, False), (2, True), (5, True)):
        _lib.check(lib.gslm_rasterize_loss_slot(ctypes.byref(vw), P, sl["geoms"][0].data_ptr(), sl["geoms"][0].numel(),
                                                binning.data_ptr(), binning.numel(), N, slot, 6, ev.gts[0].data_ptr(),
                                                None, scr.data_ptr(), scr.numel() * 8, loss.data_ptr(), 0,
                                                _lib.stream_handle()))
        v = float(loss)
        assert math.isnan(v) == want_nan, (slot, v)
    # the all-sets entry point honours the same recorded count -- a group reaching past the binning's 2 sets
    # gets NaN losses there (not background-only ones), and its sets inside the count are the slot form's values
    H, W = int(vw.image_height), int(vw.image_width)
    ref = []
    for slot in (0, 1):
        _lib.check(lib.gslm_rasterize_loss_slot(ctypes.byref(vw), P, sl["geoms"][slot].data_ptr(), sl["geoms"][0].numel(),
                                                binning.data_ptr(), binning.numel(), N, slot, 2, ev.gts[0].data_ptr(),
                                                None, scr.data_ptr(), scr.numel() * 8, loss.data_ptr(), 0,
                                                _lib.stream_handle()))
        ref.append(float(loss))
    for first, n, want in ((0, 4, (False, False, True, True)), (1, 2, (False, True)), (0, 2, (False, False))):
        nb = lib.gslm_loss_sets_scratch_bytes(n, H, W)
        sscr = torch.empty(nb // 8 + 1, dtype=torch.float64, device="cuda")
        out = torch.zeros(n, dtype=torch.float64, device="cuda")
        gg = (ctypes.c_void_p * n)(*[sl["geoms"][min(first + a, 1)].data_ptr() for a in range(n)])
        lp = (ctypes.c_void_p * n)(*[out.data_ptr() + 8 * a for a in range(n)])
        _lib.check(lib.gslm_rasterize_loss_sets(ctypes.byref(vw), P, gg, n, first, sl["geoms"][0].numel(),
                                                binning.data_ptr(), binning.numel(), N, ev.gts[0].data_ptr(), None,
                                                sscr.data_ptr(), sscr.numel() * 8, lp, 0, _lib.stream_handle()))
        got = [float(x) for x in out.cpu()]
        assert [math.isnan(x) for x in got] == list(want), (first, n, got)
        for a, x in enumerate(got):
            if not want[a]:
                assert x == ref[first + a], (first, a, x, ref)
