"""GPU edge cases of the drop-in rasterizer and the LM product, against the CPU oracle (the HIP-path
counterpart of tests/test_oracle_properties.py::test_empty_and_culled_inputs): no Gaussians, every Gaussian
culled, one-pixel / one-row / one-column images, a Gaussian covering the whole frame, Gaussians straddling the
image border, and an LM problem with nothing visible.

Tolerances as tests/test_gpu_raster.py: index work and n_contrib bit-exact, images 1e-4 L-inf, gradients and
tangents 1e-4 relative to the tensor's max magnitude; exact zeros where the math gives zeros.
"""
import math

import pytest
import torch
import torch.autograd.forward_ad as fwAD

from oracle import torch_raster as tr
from scenes import activated, gpu_settings, oracle_settings
from test_gpu_raster import _gpu_forward_internals, _rel_err

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _model(P, D, s0, seed=0):
    from gslm.model import synthetic_gaussians
    return synthetic_gaussians(P, D, seed=seed, s0=s0, device="cpu", n_cams=1)


def _cam(W, H, seed=1):
    from gslm.cameras import orbit_cameras
    return orbit_cameras(1, W, H, seed=seed)[0]


def _rasterize_gpu(a, cam, D, bg, m2=None):
    from diff_gaussian_rasterization import GaussianRasterizer
    m2 = torch.zeros_like(a["means3D"]) if m2 is None else m2
    return GaussianRasterizer(gpu_settings(cam, D, bg))(means3D=a["means3D"], means2D=m2, shs=a["shs"],
                                                        opacities=a["opacities"], scales=a["scales"],
                                                        rotations=a["rotations"])


def _rasterize_cpu(a, cam, D, bg, m2=None):
    m2 = torch.zeros_like(a["means3D"]) if m2 is None else m2
    return tr.rasterize(a["means3D"], m2, a["opacities"], oracle_settings(cam, D, bg), shs=a["shs"],
                        scales=a["scales"], rotations=a["rotations"])


def _check_forward_backward_jvp(model, cam, bg, seed=5):
    """Forward internals exact, image / gradients / tangents within the suite's tolerances.  Returns the
    oracle's preprocess state (for the callers' checks that the scene exercises what it means to)."""
    D = model.active_sh_degree
    st = oracle_settings(cam, D, bg)
    a0 = activated(model)
    with torch.no_grad():
        c, r, d, I = tr.rasterize(a0["means3D"], torch.zeros_like(a0["means3D"]), a0["opacities"], st, shs=a0["shs"],
                                  scales=a0["scales"], rotations=a0["rotations"], return_internals=True)
    G = _gpu_forward_internals(model, cam, D, bg)
    assert torch.equal(G["radii"], r)
    assert G["N"] == I["point_list"].numel()
    assert torch.equal(G["point_list"], I["point_list"])
    assert torch.equal(G["ranges"], I["ranges"])
    assert torch.equal(G["n_contrib"].long(), I["n_contrib"].long())
    assert (G["color"] - c).abs().max() <= 1e-4
    assert (G["invdepth"] - d).abs().max() <= 1e-4
    H, W = cam.image_height, cam.image_width
    gen = torch.Generator().manual_seed(seed)
    dcol, ddep = torch.randn(3, H, W, generator=gen), torch.randn(1, H, W, generator=gen)

    def grads(dev, fn):
        a = {k: v.detach().to(dev).clone().requires_grad_(True) for k, v in a0.items()}  # fresh leaves per run
        m2 = torch.zeros_like(a["means3D"], requires_grad=True)
        cc, _, dd = fn(a, cam, D, bg.to(dev), m2)
        loss = (cc * dcol.to(dev)).sum() + (dd * ddep.to(dev)).sum()
        if loss.requires_grad:  # the oracle's graph is empty when nothing is visible
            loss.backward()
        z = lambda t: (t.grad if t.grad is not None else torch.zeros_like(t)).detach().cpu()  # noqa: E731
        return {k: z(v) for k, v in a.items()} | {"means2D": z(m2)}

    ref, got = grads("cpu", _rasterize_cpu), grads(DEV, _rasterize_gpu)
    for k in ref:
        if float(ref[k].abs().max()) == 0.0:
            assert float(got[k].abs().max()) == 0.0, k
        else:
            assert _rel_err(got[k], ref[k]) < 1e-4, f"grad {k}: {_rel_err(got[k], ref[k]):.3e}"
    tang = {k: torch.randn(v.shape, generator=gen) for k, v in a0.items()}

    def tangents(dev, fn):
        with torch.no_grad(), fwAD.dual_level():
            a = {k: fwAD.make_dual(v.to(dev), tang[k].to(dev)) for k, v in a0.items()}
            cc, _, dd = fn(a, cam, D, bg.to(dev))
            return fwAD.unpack_dual(cc).tangent, fwAD.unpack_dual(dd).tangent

    (rc, rd), (gc, gd) = tangents("cpu", _rasterize_cpu), tangents(DEV, _rasterize_gpu)
    for x, y, name in ((gc, rc, "color"), (gd, rd, "invdepth")):
        x = torch.zeros_like(y) if x is None else x.cpu()
        y = torch.zeros_like(x) if y is None else y
        if float(y.abs().max()) == 0.0:
            assert float(x.abs().max()) == 0.0, name
        else:
            assert _rel_err(x, y) < 1e-4, f"{name} tangent: {_rel_err(x, y):.3e}"
    return I["pre"]


def test_no_gaussians():
    """P = 0: the background everywhere, no radii, empty gradients, zero tangent."""
    model = _model(0, 1, 0.02)
    cam = _cam(40, 33)
    bg = torch.tensor([0.25, 0.5, 0.75])
    a = {k: v.to(DEV).requires_grad_(True) for k, v in activated(model).items()}
    c, r, d = _rasterize_gpu(a, cam, model.active_sh_degree, bg.to(DEV))
    assert r.numel() == 0
    assert torch.equal(c.cpu(), bg.view(3, 1, 1).expand(3, 33, 40))
    assert float(d.abs().max()) == 0.0
    (c.sum() + d.sum()).backward()
    for k, v in a.items():
        assert v.grad is None or v.grad.numel() == 0, k


def test_every_gaussian_culled():
    """Every mean at the camera centre (view-space z = 0 <= 0.2): the background, zero radii, exact-zero
    gradients and tangent, as the oracle."""
    model = _model(500, 2, 0.03)
    cam = _cam(48, 40)
    with torch.no_grad():
        model._xyz[:] = cam.camera_center.view(1, 3)
    bg = torch.tensor([0.1, 0.6, 0.3])
    _check_forward_backward_jvp(model, cam, bg)
    G = _gpu_forward_internals(model, cam, model.active_sh_degree, bg)
    assert G["N"] == 0 and int(G["radii"].abs().sum()) == 0


@pytest.mark.parametrize("W,H", [(1, 1), (17, 1), (1, 23), (16, 16), (33, 17)])
def test_degenerate_image_sizes(W, H):
    """One-pixel, one-row, one-column, exactly one tile, one tile plus one pixel on each axis."""
    model = _model(300, 2, 0.06)
    _check_forward_backward_jvp(model, _cam(W, H), torch.tensor([0.3, 0.2, 0.1]))


def test_frame_filling_and_border_gaussians():
    """One large Gaussian in front of the camera covering every tile (long lists, early termination), others
    centred outside the image whose footprints straddle its border (rect clamping)."""
    model = _model(200, 3, 0.02, seed=3)
    cam = _cam(72, 56)
    with torch.no_grad():
        centre = cam.camera_center
        fwd = -centre / centre.norm()  # orbit cameras look at the origin
        model._xyz[0] = centre + 2.0 * fwd
        model._scaling[0] = math.log(1.5)
        model._opacity[0] = 2.0
        # a ring of Gaussians just outside the frustum's side planes
        k = torch.arange(1, 40, dtype=torch.float32)
        up = torch.tensor([0.0, 0.0, 1.0])
        side = torch.linalg.cross(fwd, up)
        side = side / side.norm()
        up2 = torch.linalg.cross(side, fwd)
        ang = 2 * math.pi * k / 39
        model._xyz[1:40] = (centre + 3.0 * fwd + (torch.cos(ang)[:, None] * side + torch.sin(ang)[:, None] * up2)
                            * 1.6 * math.tan(cam.FoVx * 0.5) * 3.0)
        model._scaling[1:40] = math.log(0.15)
    pre = _check_forward_backward_jvp(model, cam, torch.tensor([0.0, 0.0, 0.0]))
    gx, gy = pre["grid"]
    assert int(pre["tiles_touched"][0]) == gx * gy, "Gaussian 0 must cover every tile"
    xy = pre["xy"].detach()
    outside = (xy[:, 0] < 0) | (xy[:, 0] >= cam.image_width) | (xy[:, 1] < 0) | (xy[:, 1] >= cam.image_height)
    straddling = outside & (pre["tiles_touched"] > 0)
    assert int(straddling[1:40].sum()) >= 5, "ring Gaussians centred outside the frame must reach into it"


def test_lm_product_nothing_visible():
    """An LM problem whose Gaussians are all culled: J = 0, so J^T b = 0 and (J^T J + D) v = D v exactly."""
    from gslm.lm import LMProblem
    model = _model(700, 3, 0.03).to(DEV)
    cam = _cam(64, 48)
    with torch.no_grad():
        model._xyz[:] = cam.camera_center.to(DEV).view(1, 3)
    cam.original_image = torch.rand(3, 48, 64)
    prob = LMProblem(model, [cam.to(DEV)], torch.zeros(3), device=DEV, sh_projection=False)
    prob.evaluate()
    assert prob.num_rendered() == [0]
    g = prob.rhs(prob.zeros())
    assert float(g.abs().max()) == 0.0
    v = torch.randn(prob.layout.numel, generator=torch.Generator().manual_seed(2)).to(DEV)
    for name in ("xyz", "exposure"):
        lo, hi = prob.layout.offsets[name]
        v[lo:hi] = 0
    y = prob.zeros()
    prob.matvec(v, y)
    dv = torch.zeros_like(v)
    for name, d in prob.damp.items():
        if name in prob.layout.offsets:
            lo, hi = prob.layout.offsets[name]
            dv[lo:hi] = float(d) * v[lo:hi]
    assert torch.allclose(y, dv, rtol=0, atol=0), float((y - dv).abs().max())


@pytest.mark.parametrize("max_deg,active,W,H", [(0, 0, 40, 33), (1, 1, 64, 48), (2, 2, 17, 23), (3, 1, 48, 40)])
@pytest.mark.parametrize("projected", [False, True])
def test_lm_product_sh_degrees_and_sizes(max_deg, active, W, H, projected):
    """The LM loss, J^T b and (J^T J + D) v against the oracle's operator for SH degrees 0-2, an active degree
    below the stored one (train_jvp.py's progressive oneupSHdegree), ragged images, and the single-view
    projected SH-rest layout where it applies (1e-4 of the vector's max, loss rel 1e-5)."""
    import copy
    from gslm.lm import LMProblem
    from oracle.lm_ref import OracleLMProblem
    model = _model(1500, max_deg, 0.04, seed=11)
    model.active_sh_degree = active
    cam = _cam(W, H, seed=4)
    cam.original_image = torch.rand(3, H, W, generator=torch.Generator().manual_seed(8))
    mc, cc = copy.deepcopy(model), copy.deepcopy(cam)
    op = OracleLMProblem(mc, [cc], torch.zeros(3))
    lo = float(op.evaluate())
    prob = LMProblem(model.to(DEV), [cam.to(DEV)], torch.zeros(3), device=DEV, sh_projection=projected)
    assert prob.layout.rest_projected == (projected and max_deg > 0)
    assert abs(float(prob.evaluate()) - lo) <= 1e-5 * lo
    assert prob.num_rendered()[0] > 1000
    g = prob.rhs(prob.zeros())
    go = op.rhs()
    full = prob.expand(g).cpu() if prob.layout.rest_projected else g.cpu()
    assert _rel_err(full, go) < 1e-4, _rel_err(full, go)
    v = torch.randn(prob.layout.numel, generator=torch.Generator().manual_seed(9)).to(DEV)
    for name in ("xyz", "exposure"):
        a, b = prob.layout.offsets[name]
        v[a:b] = 0
    y = prob.matvec(v, prob.zeros())
    vf = prob.expand(v) if prob.layout.rest_projected else v
    yo = op.zeros()
    op.matvec(vf.cpu(), yo)
    yf = prob.expand(y).cpu() if prob.layout.rest_projected else y.cpu()
    assert _rel_err(yf, yo) < 1e-4, _rel_err(yf, yo)


@pytest.mark.parametrize("W,H", [(5, 7), (17, 23), (40, 33)])
def test_lm_ssim_product_small_and_ragged_images(W, H):
    """The SSIM residual's loss, J^T b and (J^T J + D) v (batch_training_loss.py:18-30) against the oracle on
    images smaller than the 11-tap window and on ragged sizes (the separable window's border handling)."""
    import copy
    from gslm.lm import LMProblem
    from oracle.lm_ref import OracleLMProblem
    model = _model(800, 2, 0.05, seed=12)
    cam = _cam(W, H, seed=6)
    cam.original_image = torch.rand(3, H, W, generator=torch.Generator().manual_seed(10))
    mc, cc = copy.deepcopy(model), copy.deepcopy(cam)
    op = OracleLMProblem(mc, [cc], torch.zeros(3), ssim=True)
    lo = float(op.evaluate())
    prob = LMProblem(model.to(DEV), [cam.to(DEV)], torch.zeros(3), device=DEV, ssim=True, sh_projection=False)
    assert abs(float(prob.evaluate()) - lo) <= 1e-5 * lo
    assert prob.num_rendered()[0] > 0
    g = prob.rhs(prob.zeros())
    go = op.rhs()
    assert _rel_err(g.cpu(), go) < 1e-4, _rel_err(g.cpu(), go)
    v = torch.randn(prob.layout.numel, generator=torch.Generator().manual_seed(9)).to(DEV)
    for name in ("xyz", "exposure"):
        a, b = prob.layout.offsets[name]
        v[a:b] = 0
    y = prob.matvec(v, prob.zeros())
    yo = op.zeros()
    op.matvec(v.cpu(), yo)
    assert _rel_err(y.cpu(), yo) < 1e-4, _rel_err(y.cpu(), yo)
