"""GPU parity at BASELINE.json's full sizes, checked against the CPU oracle on a sample of tiles.

configs[1] (100k Gaussians, SH 3, one 1920x1080 view) and configs[2] (1M Gaussians, same view) are
too large for the dense oracle blend over the whole frame, but every stage before the blend is per
Gaussian or a sort, and the blend is per tile.  So:

  * integer / index work over the WHOLE view is bit-exact: radii, tiles_touched, num_rendered, the
    sorted point list (4.87M entries at 1M) and every tile range -- and so is every visible
    Gaussian's render record (screen position, conic, opacity, colour, 1/depth);
  * the blend is compared on a tile sample (strided over the frame, plus the longest list and the
    ragged bottom-right corner tile): n_contrib bit-exact, colour / invdepth within 1e-4, final_T 1e-5;
  * the VJP is driven by dL/dcolor ~ N(0, 1) (seed 4) that is ZERO outside the sampled tiles, so the
    GPU's full-frame backward must equal the oracle's autograd through the sampled tiles only
    (every Gaussian's gradient, 1e-4 of the tensor's max);
  * the fused LM product (J^T W J + D) v is checked the same way: W (the per-pixel weight
    m^2 1[0 <= R <= 1]) is zeroed outside the sampled tiles, and the oracle computes 2 J^T (W J v) with
    forward-AD + autograd on the raw GaussianModel leaves (1e-4 of the vector's max).
"""
import math

import numpy as np
import pytest
import torch
import torch.autograd.forward_ad as fwAD

from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from oracle import torch_raster as tr
from margins import record
from scenes import activated, gpu_settings, oracle_settings

pytestmark = pytest.mark.gpu
DEV = "cuda"
W, H = 1920, 1080
CONFIGS = {"cfg1_100k_sh3_1080p": 100_000, "cfg2_1M_sh3_1080p": 1_000_000}


def _sample_tiles(ranges, n=24):
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ntiles = gx * gy
    lens = (ranges[:, 1] - ranges[:, 0]).numpy()
    sub = set(range(ntiles // (2 * n), ntiles, ntiles // n))
    sub.add(int(np.argmax(lens)))  # the longest list
    sub.add(ntiles - 1)            # ragged corner tile (1080 = 67.5 tiles)
    return sub


def _tile_pixel_mask(sub):
    gx = (W + 15) // 16
    m = torch.zeros(H, W, dtype=torch.bool)
    for t in sub:
        ty, tx = divmod(t, gx)
        m[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16] = True
    return m


def _scene(P):
    model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1)
    cam = orbit_cameras(1, W, H, seed=1)[0]
    return model, cam


def _l2_rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _rel_err(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-8)).item()


def _gpu_records(model, cam):
    from diff_gaussian_rasterization import _gaussians, forward_buffers
    from gslm import _lib
    a = {k: v.to(DEV) for k, v in activated(model).items()}
    view = _lib.view_from_settings(gpu_settings(cam, 3))
    P = a["means3D"].shape[0]
    g = _gaussians(P, a["means3D"], a["opacities"].reshape(-1).contiguous(), a["scales"], a["rotations"], None,
                   a["shs"], None, None)
    _, _, _, geom, binning, image, N = forward_buffers(view, g, DEV)
    rec = torch.zeros(P * 12, dtype=torch.float32, device=DEV)
    _lib.check(_lib.lib.gslm_inspect(geom.data_ptr(), P, binning.data_ptr(), N, H, W, image.data_ptr(), None, None,
                                     None, None, None, rec.data_ptr(), _lib.stream_handle()))
    torch.cuda.synchronize()
    return rec.view(P, 12).cpu()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fullsize_forward(name):
    from test_gpu_raster import _gpu_forward_internals
    model, cam = _scene(CONFIGS[name])
    a = activated(model)
    st = oracle_settings(cam, 3)
    with torch.no_grad():
        pre = tr.preprocess(a["means3D"], torch.zeros_like(a["means3D"]), a["opacities"], a["shs"], None,
                            a["scales"], a["rotations"], None, st)
        pl, _, ranges = tr.binning(pre)
    G = _gpu_forward_internals(model, cam, 3)
    assert torch.equal(G["radii"], pre["radii"]), "radii must match exactly"
    assert torch.equal(G["tiles"], pre["tiles_touched"].long()), "tiles_touched must match exactly"
    assert G["N"] == pl.numel(), "num_rendered must match"
    assert torch.equal(G["point_list"], pl), "sorted point list must match exactly"
    assert torch.equal(G["ranges"], ranges.long()), "tile ranges must match exactly"
    # every visible Gaussian's render record is bit-identical to the restatement's (preprocess mirrors
    # its operation order; both use correctly rounded float32 division and sqrt)
    rec = _gpu_records(model, cam)
    vis = pre["radii"] > 0
    for name, col, ref in (("x", 0, pre["xy"][:, 0]), ("y", 1, pre["xy"][:, 1]), ("conic.a", 2, pre["conic"][:, 0]),
                           ("conic.b", 3, pre["conic"][:, 1]), ("conic.c", 4, pre["conic"][:, 2]),
                           ("opacity", 5, pre["opacity"]), ("r", 6, pre["rgb"][:, 0]), ("g", 7, pre["rgb"][:, 1]),
                           ("b", 8, pre["rgb"][:, 2]), ("1/z", 9, 1.0 / pre["depth"])):
        assert torch.equal(rec[vis, col], ref[vis]), f"record field {name} differs"
    sub = _sample_tiles(ranges)
    with torch.no_grad():
        color, invd, fT, nc = tr.blend(pre, pl, ranges, H, W, st.bg, tile_subset=sub)
    m = _tile_pixel_mask(sub)
    assert torch.equal(G["n_contrib"][m].long(), nc[m].long()), "n_contrib must match exactly"
    assert (G["final_T"][m] - fT[m]).abs().max() <= 1e-5
    assert (G["color"][:, m] - color[:, m]).abs().max() <= 1e-4
    assert (G["invdepth"][:, m] - invd[:, m]).abs().max() <= 1e-4


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fullsize_backward(name):
    from diff_gaussian_rasterization import GaussianRasterizer
    model, cam = _scene(CONFIGS[name])
    a0 = activated(model)
    st = oracle_settings(cam, 3)
    with torch.no_grad():
        pre = tr.preprocess(a0["means3D"], torch.zeros_like(a0["means3D"]), a0["opacities"], a0["shs"], None,
                            a0["scales"], a0["rotations"], None, st)
        _, _, ranges = tr.binning(pre)
    sub = _sample_tiles(ranges)
    g = torch.Generator().manual_seed(4)
    dcol = torch.randn(3, H, W, generator=g) * _tile_pixel_mask(sub)

    # oracle: autograd through the sampled tiles' blend and every Gaussian's preprocess
    a = {k: v.clone().requires_grad_(True) for k, v in a0.items()}
    m2 = torch.zeros_like(a0["means3D"], requires_grad=True)
    pre = tr.preprocess(a["means3D"], m2, a["opacities"], a["shs"], None, a["scales"], a["rotations"], None, st)
    pl, _, ranges = tr.binning(pre)
    color, _, _, _ = tr.blend(pre, pl, ranges, H, W, st.bg, tile_subset=sub)
    (color * dcol).sum().backward()
    ref = {k: v.grad for k, v in a.items()} | {"means2D": m2.grad}

    ag = {k: v.to(DEV).requires_grad_(True) for k, v in a0.items()}
    m2g = torch.zeros_like(ag["means3D"], requires_grad=True)
    c, _, _ = GaussianRasterizer(gpu_settings(cam, 3))(means3D=ag["means3D"], means2D=m2g, shs=ag["shs"],
                                                       opacities=ag["opacities"], scales=ag["scales"],
                                                       rotations=ag["rotations"])
    c.backward(dcol.to(DEV))
    got = {k: v.grad.cpu() for k, v in ag.items()} | {"means2D": m2g.grad.cpu()}
    for k in ref:
        err = record(f"test_fullsize_backward[{name}]", f"grad {k} (of max)", _rel_err(got[k], ref[k]), 1e-4)
        assert err < 1e-4, f"grad {k}: rel err {err:.3e}"


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fullsize_lm_matvec(name):
    from gslm.lm import LMProblem
    model, cam = _scene(CONFIGS[name])
    zero_damp = {k: 0.0 for k in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity",
                                  "exposure")}
    gm = synthetic_gaussians(CONFIGS[name], 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(DEV)
    cg = orbit_cameras(1, W, H, seed=1)[0].to(DEV)
    prob = LMProblem(gm, [cg], torch.zeros(3), gts=[torch.zeros(3, H, W, device=DEV)],
                     alpha_masks=[torch.ones(1, H, W, device=DEV)], damp=zero_damp)
    prob.evaluate()
    ranges = None
    with torch.no_grad():
        st = oracle_settings(cam, 3)
        pre = tr.preprocess(model.get_xyz, torch.zeros_like(model.get_xyz), model.get_opacity, model.get_features,
                            None, model.get_scaling, model.get_rotation, None, st)
        _, _, ranges = tr.binning(pre)
    sub = _sample_tiles(ranges)
    tm = _tile_pixel_mask(sub)
    prob.weights[0].mul_(tm.to(DEV).to(torch.float32))
    w = prob.weights[0].cpu()

    gen = torch.Generator().manual_seed(3)
    v = torch.randn(prob.layout.numel, generator=gen)
    o = prob.layout.offsets
    v[o["xyz"][0]:o["xyz"][1]] = 0
    v[o["exposure"][0]:o["exposure"][1]] = 0
    y = prob.matvec(v.to(DEV), prob.zeros()).cpu()

    # oracle on the raw leaves: q = J v (forward-AD), then J^T (2 w q) (autograd)
    groups = ["features_dc", "features_rest", "scaling", "rotation", "opacity"]
    leaves = {"features_dc": "_features_dc", "features_rest": "_features_rest", "scaling": "_scaling",
              "rotation": "_rotation", "opacity": "_opacity"}
    tang = {gname: v[o[gname][0]:o[gname][1]].reshape(getattr(model, leaves[gname]).shape) for gname in groups}

    def render():
        st = oracle_settings(cam, 3)
        pre = tr.preprocess(model.get_xyz, torch.zeros_like(model.get_xyz), model.get_opacity,
                            model.get_features, None, model.get_scaling, model.get_rotation, None, st)
        pl, _, rg = tr.binning(pre)
        color, _, _, _ = tr.blend(pre, pl, rg, H, W, st.bg, tile_subset=sub)
        return color

    with torch.no_grad(), fwAD.dual_level():
        saved = {gname: getattr(model, leaves[gname]) for gname in groups}
        try:
            for gname in groups:
                setattr(model, leaves[gname], fwAD.make_dual(saved[gname], tang[gname]))
            q = fwAD.unpack_dual(render()).tangent
        finally:
            for gname in groups:
                setattr(model, leaves[gname], saved[gname])
    for gname in groups:
        getattr(model, leaves[gname]).requires_grad_(True)
    (render() * (2.0 * w * q)).sum().backward()
    for gname in groups:
        ref = getattr(model, leaves[gname]).grad.reshape(-1)
        got = y[o[gname][0]:o[gname][1]]
        err = record(f"test_fullsize_lm_matvec[{name}]", f"group {gname} (of max)", _rel_err(got, ref), 1e-4)
        assert err < 1e-4, f"group {gname}: rel err {err:.3e}"
    assert y[o["xyz"][0]:o["xyz"][1]].abs().max() == 0


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fullsize_forward_whole_frame(name):
    """The blend over EVERY tile of the 1080p frame (not a sample), against the oracle's dense blend (~10 s at 100k,
    ~40 s at 1M on the host): n_contrib bit-exact, colour / inverse depth within 1e-4 and final_T within 1e-5 at every
    pixel except where one Gaussian's alpha sits at the 1/255 cut (or T at the 1e-4 stop) and the two exponentials (the GPU's
    v_exp_f32, ~2 ulp -- shared by every GPU tile pass, so their decisions agree among themselves -- and torch's CPU
    exp) decide it differently: such a flip scales the pixel's later transmittance by (1 - alpha) ~ 1 - 1/255.  Those
    pixels must be rare (<= 1e-4 of the frame) and their error that of one flip (<= 0.01)."""
    from test_gpu_raster import _gpu_forward_internals
    model, cam = _scene(CONFIGS[name])
    a = activated(model)
    st = oracle_settings(cam, 3)
    with torch.no_grad():
        pre = tr.preprocess(a["means3D"], torch.zeros_like(a["means3D"]), a["opacities"], a["shs"], None,
                            a["scales"], a["rotations"], None, st)
        pl, _, ranges = tr.binning(pre)
        color, invd, fT, nc = tr.blend(pre, pl, ranges, H, W, st.bg)
    G = _gpu_forward_internals(model, cam, 3)
    dN = G["n_contrib"].long() != nc.long()
    dT = (G["final_T"] - fT).abs()
    dC = (G["color"] - color).abs().amax(0)
    dD = (G["invdepth"] - invd).abs()[0]
    flip = dN | (dT > 1e-5) | (dC > 1e-4) | (dD > 1e-4)
    nflip = int(flip.sum())
    print(f"{name}: {nflip} of {H * W} pixels off (alpha-cut flips; n_contrib differs at {int(dN.sum())}); "
          f"max |dT| {float(dT.max()):.2e}, |dC| {float(dC.max()):.2e}; elsewhere |dC| {float(dC[~flip].max()):.2e}")
    record(f"test_fullsize_forward_whole_frame[{name}]", "pixels off (of H W)", nflip / (H * W), 1e-4)
    record(f"test_fullsize_forward_whole_frame[{name}]", "|dC| elsewhere", float(dC[~flip].max()), 1e-4)
    assert nflip <= 1e-4 * H * W, nflip
    assert float(dT.max()) <= 0.01 and float(dC.max()) <= 0.01, (float(dT.max()), float(dC.max()))


def test_fullsize_backward_whole_frame_100k():
    """configs[1]'s backward with dL/dcolor ~ N(0, 1) over the WHOLE frame against the oracle's autograd through every
    tile (every Gaussian's gradient, 1e-4 of each tensor's max)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    model, cam = _scene(CONFIGS["cfg1_100k_sh3_1080p"])
    a0 = activated(model)
    st = oracle_settings(cam, 3)
    dcol = torch.randn(3, H, W, generator=torch.Generator().manual_seed(4))
    a = {k: v.clone().requires_grad_(True) for k, v in a0.items()}
    m2 = torch.zeros_like(a0["means3D"], requires_grad=True)
    pre = tr.preprocess(a["means3D"], m2, a["opacities"], a["shs"], None, a["scales"], a["rotations"], None, st)
    pl, _, ranges = tr.binning(pre)
    color, _, _, _ = tr.blend(pre, pl, ranges, H, W, st.bg)
    (color * dcol).sum().backward()
    ref = {k: v.grad for k, v in a.items()} | {"means2D": m2.grad}
    ag = {k: v.to(DEV).requires_grad_(True) for k, v in a0.items()}
    m2g = torch.zeros_like(ag["means3D"], requires_grad=True)
    c, _, _ = GaussianRasterizer(gpu_settings(cam, 3))(means3D=ag["means3D"], means2D=m2g, shs=ag["shs"],
                                                       opacities=ag["opacities"], scales=ag["scales"],
                                                       rotations=ag["rotations"])
    c.backward(dcol.to(DEV))
    got = {k: v.grad.cpu() for k, v in ag.items()} | {"means2D": m2g.grad.cpu()}
    # over the whole frame a handful of (entry, pixel) alpha tests sit within an ulp of the 1/255 cut, where the GPU's
    # v_exp_f32 and the oracle's exp decide differently (the forward's flipped pixels above): each moves the gradients
    # of the Gaussians behind that pixel, so the max-based error is set by the worst flip.  Measured (round 5,
    # profiles/r05/parity_margins*.jsonl): the kept kernels 3.8e-6 L2 / 7.6e-5 per element (SH gradient, the worst);
    # round 4's rejected log2e-prescaled exponent -- one more rounding in every alpha -- 2.1e-5 / 3.8e-4 (scales).  A
    # wrong derivative is O(1).  Asserted (round 6: no bound looser than round 4's except on flip-touched elements): the
    # error over every Gaussian (L2 rel 3e-5); per element round 4's 1e-4 of the max for all but at most 1e-4 of the
    # elements (the Gaussians behind a flipped pixel), and those within a flip-sized 1e-3.
    for k in ref:
        T = "test_fullsize_backward_whole_frame_100k"
        l2 = record(T, f"grad {k} (L2 rel)", _l2_rel(got[k], ref[k]), 3e-5)
        err = record(T, f"grad {k} (of max, per element, flip guard)", _rel_err(got[k], ref[k]), 1e-3)
        d = (got[k] - ref[k]).abs()
        n_over = int((d > 1e-4 * ref[k].abs().max().clamp_min(1e-8)).sum())
        frac_over = record(T, f"grad {k} elements beyond 1e-4 of max (fraction)", n_over / d.numel(), 1e-4)
        assert l2 <= 3e-5 and err < 1e-3 and frac_over <= 1e-4, f"grad {k}: L2 {l2:.3e}, max {err:.3e}, over {n_over}"


def test_fullsize_lm_matvec_whole_frame_100k():
    """configs[1]'s fused LM product (J^T W J v, xyz masked, zero damping) with the per-pixel weights of the WHOLE
    frame (no tile sample) against the oracle's forward-AD J v and autograd J^T over every tile (1e-4 of each group's
    max)."""
    from gslm.lm import LMProblem
    name = "cfg1_100k_sh3_1080p"
    model, cam = _scene(CONFIGS[name])
    zero_damp = {k: 0.0 for k in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity",
                                  "exposure")}
    gm = synthetic_gaussians(CONFIGS[name], 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(DEV)
    cg = orbit_cameras(1, W, H, seed=1)[0].to(DEV)
    prob = LMProblem(gm, [cg], torch.zeros(3), gts=[torch.zeros(3, H, W, device=DEV)],
                     alpha_masks=[torch.ones(1, H, W, device=DEV)], damp=zero_damp)
    prob.evaluate()
    w = prob.weights[0].cpu()
    gen = torch.Generator().manual_seed(3)
    v = torch.randn(prob.layout.numel, generator=gen)
    o = prob.layout.offsets
    v[o["xyz"][0]:o["xyz"][1]] = 0
    v[o["exposure"][0]:o["exposure"][1]] = 0
    y = prob.matvec(v.to(DEV), prob.zeros()).cpu()
    groups = ["features_dc", "features_rest", "scaling", "rotation", "opacity"]
    leaves = {g: "_" + g for g in groups}
    tang = {g: v[o[g][0]:o[g][1]].reshape(getattr(model, leaves[g]).shape) for g in groups}

    def render():
        st = oracle_settings(cam, 3)
        pre = tr.preprocess(model.get_xyz, torch.zeros_like(model.get_xyz), model.get_opacity,
                            model.get_features, None, model.get_scaling, model.get_rotation, None, st)
        pl, _, rg = tr.binning(pre)
        color, _, _, _ = tr.blend(pre, pl, rg, H, W, st.bg)
        return color

    with torch.no_grad(), fwAD.dual_level():
        saved = {g: getattr(model, leaves[g]) for g in groups}
        try:
            for g in groups:
                setattr(model, leaves[g], fwAD.make_dual(saved[g], tang[g]))
            q = fwAD.unpack_dual(render()).tangent
        finally:
            for g in groups:
                setattr(model, leaves[g], saved[g])
    for g in groups:
        getattr(model, leaves[g]).requires_grad_(True)
    (render() * (2.0 * w * q)).sum().backward()
    for g in groups:
        err = record("test_fullsize_lm_matvec_whole_frame_100k", f"group {g} (of max)",
                     _rel_err(y[o[g][0]:o[g][1]], getattr(model, leaves[g]).grad.reshape(-1)), 1e-4)
        assert err < 1e-4, f"group {g}: rel err {err:.3e}"
    assert y[o["xyz"][0]:o["xyz"][1]].abs().max() == 0
