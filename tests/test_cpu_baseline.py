"""The CPU baseline leg of bench.py (oracle/cpu_baseline.py): the per-tile blend it times on a tile sample is the
full-frame blend's arithmetic on those tiles, and its split J^T u (autograd cut at the screen-space tensors)
is the unsplit one."""
import torch
import torch.autograd.forward_ad as fwAD

from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from oracle import cpu_baseline as cb
from oracle import torch_raster as tr


def _scene():
    model = synthetic_gaussians(300, 1, seed=0, s0=0.03, device="cpu")
    cam = orbit_cameras(1, 64, 48, seed=1)[0]
    st = tr.settings_from_camera(cam, torch.zeros(3), model.active_sh_degree)
    return model, cam, st


def test_blend_tiles_matches_blend():
    model, cam, st = _scene()
    with torch.no_grad():
        pre, pl, ranges = cb._preprocess_binning(model, st)
        color = tr.blend(pre, pl, ranges, st.image_height, st.image_width, st.bg)[0]
        gx = pre["grid"][0]
        tiles = [t for t in range(gx * pre["grid"][1]) if ranges[t, 1] > ranges[t, 0]][:5]
        assert tiles
        sub = tr.blend_tiles(pre, pl, ranges, st.image_height, st.image_width, st.bg, tiles)
    ref = []
    for t in tiles:
        py, px = tr._tile_pixels(t, gx, st.image_height, st.image_width)
        ref.append(color[:, py, px].t())
    assert torch.equal(sub, torch.cat(ref, 0))


def test_split_backward_equals_unsplit():
    model, cam, st = _scene()
    H, W = st.image_height, st.image_width
    pre, pl, ranges = cb._preprocess_binning(model, st)
    tiles = list(range(pre["grid"][0] * pre["grid"][1]))
    u = torch.randn(tr.blend_tiles(pre, pl, ranges, H, W, st.bg, tiles).shape, generator=torch.Generator().manual_seed(5))
    model.zero_grad()
    (tr.blend_tiles(pre, pl, ranges, H, W, st.bg, tiles) * u).sum().backward()
    ref = [p.grad.clone() for p in (model._features_dc, model._opacity, model._scaling, model._rotation)]
    model.zero_grad()
    pre, pl, ranges = cb._preprocess_binning(model, st)
    leaves = {k: pre[k].detach().requires_grad_(pre[k].requires_grad) for k in cb._SCREEN}
    (tr.blend_tiles(dict(pre, **leaves), pl, ranges, H, W, st.bg, tiles) * u).sum().backward()
    outs = [(pre[k], leaves[k].grad) for k in cb._SCREEN if leaves[k].grad is not None]
    torch.autograd.backward([o for o, _ in outs], [g for _, g in outs])
    got = [p.grad for p in (model._features_dc, model._opacity, model._scaling, model._rotation)]
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


def test_cpu_matvec_rate_runs():
    model, cam, _ = _scene()
    r = cb.cpu_matvec_rate(model, cam, torch.zeros(3), n_tiles=4, repeats=1, threads=2)
    assert r["n_tiles"] == 4 and r["ntiles"] == 12
    assert r["t_gauss"] > 0 and r["t_tiles"] > 0 and r["matvec_s"] > r["t_gauss"]
    assert r["forward_s"] > 0
