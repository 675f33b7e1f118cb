"""GPU: the device-count rasterize forms (ABI 7: gslm_rasterize_dev / gslm_rasterize_loss_dev) -- the pair count stays
on the device between the preprocess and the binning.  When the count fits the list capacity they give gslm_rasterize's
image and gslm_rasterize_loss's loss bitwise and report the count; a count past the capacity is reported (no write past
the list) and the line-search evaluator renders that view again exactly."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _scene(P=20000, W=320, H=208, seed=0):
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    m = synthetic_gaussians(P, 3, seed=seed, s0=0.01).to("cuda")
    cams = orbit_cameras(3, W, H, seed=3)
    for c in cams:
        c.to("cuda")
    return m, cams


def test_rasterize_dev_equals_rasterize_and_reports_the_count():
    from gslm import _lib
    from gslm.lm import ViewRaster
    from gslm.params import raw_gaussians
    m, cams = _scene()
    g = raw_gaussians(m)
    st = _lib.stream_handle("cuda")
    for c in cams:
        vr = ViewRaster(_lib.view_from_camera(c, torch.zeros(3), 3), "cuda")
        ref = vr.forward(g, st).clone()
        ref_inv = vr.invdepth.clone()
        N = vr.N
        assert N > 0 and vr.capacity() >= N
        n = torch.full((2,), -1, dtype=torch.int32, device="cuda")
        img = vr.forward_dev(g, st, n_out=n.data_ptr())
        torch.cuda.synchronize()
        assert int(n[0]) == N and vr.N is None
        assert torch.equal(img, ref) and torch.equal(vr.invdepth, ref_inv)
        # the count copied out on its own (stream ordered, no sync inside)
        assert _lib.lib.gslm_num_rendered_copy(vr.geom.data_ptr(), g.P, n.data_ptr() + 4, st) == 0
        torch.cuda.synchronize()
        assert int(n[1]) == N
        # a list too short for the count: reported, nothing written past the list (the guard bytes stay put)
        need = _lib.lib.gslm_binning_bytes(N // 2, vr.H, vr.W)
        buf = torch.full((need + 4096,), 0xA5, dtype=torch.uint8, device="cuda")
        cap = _lib.lib.gslm_binning_capacity(need, vr.H, vr.W)
        assert N // 2 <= cap < N
        out = torch.empty_like(ref)
        rc = _lib.lib.gslm_rasterize_dev(ctypes.byref(vr.view), g.P, vr.geom.data_ptr(), buf.data_ptr(), need,
                                         vr.image.data_ptr(), vr.image.numel(), out.data_ptr(), None, n.data_ptr(), st)
        assert rc == 0, _lib.lib.gslm_last_error()
        torch.cuda.synchronize()
        assert int(n[0]) == N > cap
        assert bool((buf[need:] == 0xA5).all())


def test_loss_evaluator_device_count_renders_and_overflow():
    """With device_count=True later evaluations run gslm_rasterize_loss_dev; a slot whose list is too short for a view is caught by the
    end-of-evaluation count check and that view is rendered again exactly: the loss is unchanged, bitwise."""
    from gslm.lm import LossEvaluator
    m, cams = _scene(P=8000, W=200, H=136, seed=1)
    gts = [torch.rand(3, 136, 200, generator=torch.Generator().manual_seed(40 + i)) for i in range(len(cams))]
    for c, gt in zip(cams, gts):
        c.original_image = gt.cuda()
    ev = LossEvaluator(m, cams, torch.zeros(3), batch=2, streams=2, device_count=True)
    first = float(ev.evaluate())  # sizes the slots (counts read back)
    counts = list(ev.num_rendered)
    assert float(ev.evaluate()) == first  # device-count renders
    assert ev.num_rendered == counts
    # shrink slot 1's list below every view's count: its views overflow and are rendered again exactly
    from gslm import _lib
    small = min(counts) // 3
    ev.slots[1]["binning"] = _lib.u8(_lib.lib.gslm_binning_bytes(small, 136, 200), "cuda")
    assert float(ev.evaluate()) == first
    assert ev.num_rendered == counts
    assert _lib.lib.gslm_binning_capacity(ev.slots[1]["binning"].numel(), 136, 200) >= max(counts[1::2])  # grown
    assert float(ev.evaluate()) == first
