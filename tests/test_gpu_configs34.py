"""GPU parity at the per-GPU slices of BASELINE.json configs[3] and configs[4] (the multi-GPU configs).

configs[3] is 1M Gaussians with a batch of 8 x 1080p views, one view per GPU; configs[4] is 5M Gaussians SH 3
with 32 x 3840x2160 views over 8 GPUs (4 per GPU).  One rank of those runs holds the whole model and renders
its views with the full SH-rest layout (no single-view projection), so the slices tested here are:

  * configs[3]: 1M Gaussians, two 1080p views in one LMProblem (multi-view, full layout): the fused product
    sum_b 2 J_b^T W_b J_b v against the oracle's forward-AD + autograd on a tile sample of each view (W zeroed
    outside the sample, as tests/test_gpu_fullsize.py does for one view); and the Gaussian-sharded pipeline of
    the 8-GPU exchange (gslm_tangent_views -> exchanged records -> RENDER | SCREEN -> gslm_gather_screen) on the
    same two views equals that product;
  * configs[4]: 5M Gaussians, one 3840x2160 view: the forward's integer work bit-exact over the whole view
    (radii, tiles_touched, num_rendered, tile ranges), the blend on sampled tiles (n_contrib exact, colour
    1e-4), and the LM product on sampled tiles against the oracle (1e-4 of the vector's max).
"""
import numpy as np
import pytest
import torch
import torch.autograd.forward_ad as fwAD

from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from oracle import torch_raster as tr
from scenes import oracle_settings

pytestmark = pytest.mark.gpu
DEV = "cuda"
GROUPS = ["features_dc", "features_rest", "scaling", "rotation", "opacity"]
LEAVES = {"features_dc": "_features_dc", "features_rest": "_features_rest", "scaling": "_scaling",
          "rotation": "_rotation", "opacity": "_opacity"}
ZERO_DAMP = {k: 0.0 for k in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure")}


def _sample_tiles(ranges, W, H, n):
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ntiles = gx * gy
    lens = (ranges[:, 1] - ranges[:, 0]).numpy()
    sub = set(range(ntiles // (2 * n), ntiles, ntiles // n))
    sub.add(int(np.argmax(lens)))
    sub.add(ntiles - 1)
    return sub


def _tile_mask(sub, W, H):
    gx = (W + 15) // 16
    m = torch.zeros(H, W, dtype=torch.bool)
    for t in sub:
        ty, tx = divmod(t, gx)
        m[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16] = True
    return m


def _rel_err(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-8)).item()


def _direction(layout, seed=3):
    v = torch.randn(layout.numel, generator=torch.Generator().manual_seed(seed))
    o = layout.offsets
    v[o["xyz"][0]:o["xyz"][1]] = 0
    v[o["exposure"][0]:o["exposure"][1]] = 0
    return v


def _oracle_product(model, cams, subs, weights, v, layout):
    """sum_b 2 J_b^T (w_b J_b v) on the raw leaves, each view's blend restricted to its tile sample."""
    o = layout.offsets
    tang = {g: v[o[g][0]:o[g][1]].reshape(getattr(model, LEAVES[g]).shape) for g in GROUPS}

    def render(cam, sub):
        st = oracle_settings(cam, 3)
        pre = tr.preprocess(model.get_xyz, torch.zeros_like(model.get_xyz), model.get_opacity, model.get_features,
                            None, model.get_scaling, model.get_rotation, None, st)
        pl, _, rg = tr.binning(pre)
        color, _, _, _ = tr.blend(pre, pl, rg, cam.image_height, cam.image_width, st.bg, tile_subset=sub)
        return color

    qs = []
    with torch.no_grad(), fwAD.dual_level():
        saved = {g: getattr(model, LEAVES[g]) for g in GROUPS}
        try:
            for g in GROUPS:
                setattr(model, LEAVES[g], fwAD.make_dual(saved[g], tang[g]))
            for cam, sub in zip(cams, subs):
                qs.append(fwAD.unpack_dual(render(cam, sub)).tangent)
        finally:
            for g in GROUPS:
                setattr(model, LEAVES[g], saved[g])
    for g in GROUPS:
        getattr(model, LEAVES[g]).requires_grad_(True)
        getattr(model, LEAVES[g]).grad = None
    obj = sum((render(cam, sub) * (2.0 * w * q)).sum() for cam, sub, w, q in zip(cams, subs, weights, qs))
    obj.backward()
    return {g: getattr(model, LEAVES[g]).grad.reshape(-1).clone() for g in GROUPS}


def _sampled_problem(P, cams_cpu, W, H, ntiles):
    """GPU LMProblem (full layout, zero damping) over the views with each view's weight zeroed outside a tile
    sample; returns (problem, model on the CPU, tile samples, CPU weights)."""
    from gslm.lm import LMProblem
    model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=len(cams_cpu))
    gm = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=len(cams_cpu)).to(DEV)
    cams = [c.to(DEV) for c in orbit_cameras(len(cams_cpu), W, H, seed=1)]
    prob = LMProblem(gm, cams, torch.zeros(3), gts=[torch.zeros(3, H, W, device=DEV) for _ in cams],
                     alpha_masks=[torch.ones(1, H, W, device=DEV) for _ in cams], damp=ZERO_DAMP,
                     sh_projection=False)
    prob.evaluate()
    subs, weights = [], []
    for b, cam in enumerate(cams_cpu):
        with torch.no_grad():
            st = oracle_settings(cam, 3)
            pre = tr.preprocess(model.get_xyz, torch.zeros_like(model.get_xyz), model.get_opacity,
                                model.get_features, None, model.get_scaling, model.get_rotation, None, st)
            _, _, ranges = tr.binning(pre)
        sub = _sample_tiles(ranges, W, H, ntiles)
        prob.weights[b].mul_(_tile_mask(sub, W, H).to(DEV).to(torch.float32))
        subs.append(sub)
        weights.append(prob.weights[b].cpu())
    return prob, model, subs, weights


def test_config3_slice_multiview_product_and_gaussian_exchange():
    """configs[3] per-GPU slice: 1M Gaussians, two 1080p views, full layout."""
    from gslm.parallel import GaussianShardedOperator
    W, H = 1920, 1080
    cams_cpu = orbit_cameras(2, W, H, seed=1)
    prob, model, subs, weights = _sampled_problem(1_000_000, cams_cpu, W, H, 10)
    assert not prob.layout.rest_projected
    # the Gaussian-sharded exchange's pipeline over the same views (one rank: the exchanges are copies), SH-rest
    # group in the two views' coordinates: the direction's SH-rest part projected onto their span first
    op = GaussianShardedOperator(prob, all_cams=prob.cams)
    op._exchange_flags()
    assert op.rest_views == 2
    v = op.gather_full(op.shard(_direction(prob.layout).to(DEV))).cpu()
    y = prob.matvec(v.to(DEV), prob.zeros())
    ys = op.gather_full(op.matvec(op.shard(v.to(DEV)), op.zeros()))
    torch.cuda.synchronize()
    y, ys = y.cpu(), ys.cpu()
    assert (ys - y).abs().max() <= 1e-5 * y.abs().max()
    ref = _oracle_product(model, cams_cpu, subs, weights, v, prob.layout)
    o = prob.layout.offsets
    for g in GROUPS:
        err = _rel_err(y[o[g][0]:o[g][1]], ref[g])
        assert err < 1e-4, f"group {g}: rel err {err:.3e}"
    assert y[o["xyz"][0]:o["xyz"][1]].abs().max() == 0


def test_config4_slice_5M_4k_forward_and_product():
    """configs[4] per-GPU slice: 5M Gaussians SH 3, one 3840x2160 view."""
    from test_gpu_raster import _gpu_forward_internals
    W, H, P = 3840, 2160, 5_000_000
    cam = orbit_cameras(1, W, H, seed=1)[0]
    model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1)
    st = oracle_settings(cam, 3)
    with torch.no_grad():
        pre = tr.preprocess(model.get_xyz, torch.zeros_like(model.get_xyz), model.get_opacity, model.get_features,
                            None, model.get_scaling, model.get_rotation, None, st)
        pl, _, ranges = tr.binning(pre)
    G = _gpu_forward_internals(model, cam, 3)
    assert torch.equal(G["radii"], pre["radii"])
    assert torch.equal(G["tiles"], pre["tiles_touched"].long())
    assert G["N"] == pl.numel()
    assert torch.equal(G["ranges"], ranges.long())
    sub = _sample_tiles(ranges, W, H, 12)
    with torch.no_grad():
        color, _, fT, nc = tr.blend(pre, pl, ranges, H, W, st.bg, tile_subset=sub)
    m = _tile_mask(sub, W, H)
    assert torch.equal(G["n_contrib"][m].long(), nc[m].long())
    assert (G["color"][:, m] - color[:, m]).abs().max() <= 1e-4
    del G, pre, pl, color, fT, nc
    torch.cuda.empty_cache()

    prob, model, subs, weights = _sampled_problem(P, [cam], W, H, 8)
    v = _direction(prob.layout)
    y = prob.matvec(v.to(DEV), prob.zeros()).cpu()
    ref = _oracle_product(model, [cam], subs, weights, v, prob.layout)
    o = prob.layout.offsets
    for g in GROUPS:
        err = _rel_err(y[o[g][0]:o[g][1]], ref[g])
        assert err < 1e-4, f"group {g}: rel err {err:.3e}"
