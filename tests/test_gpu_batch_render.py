"""`batch_render` / `BatchGaussianRasterizer` relations the reference's own tests pin, on the GPU.

tests/test_batch_render.py:72-89: every batch slice equals the single-view render (render and depth,
atol 1e-6), `max_radii` equals the running max of the single-view radii and `visibility_filter` the
union of their visible sets.  tests/test_batch_training_loss.py:74-110: the batch loss's gradients equal
the sum of the single-view gradients (1e-5).  Views of different sizes are padded to maxH x maxW
(batch_render.py:33-50); the padding must be zero.  Each slice is also checked against the CPU oracle
(1e-4 L-inf) and the batch JVP against the single-view JVPs.
"""
import pytest
import torch
import torch.autograd.forward_ad as fwAD

from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from gslm.train import PipelineParams, batch_render, render
from oracle import torch_raster as tr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _absmax(t):
    return float(t.abs().max()) if t.numel() else 0.0


def _scene(sh=2, P=6000):
    m = synthetic_gaussians(P, sh, seed=0, s0=0.02, n_cams=5).to(DEV)
    cams = orbit_cameras(2, 96, 80, seed=1) + orbit_cameras(2, 64, 48, seed=5) + orbit_cameras(1, 40, 33, seed=9)
    for c in cams:
        c.to(DEV)
    return m, cams


@pytest.mark.parametrize("pipe_kw", [{}, {"antialiasing": True}, {"compute_cov3D_python": True},
                                     {"convert_SHs_python": True}])
@pytest.mark.parametrize("separate_sh", [False, True])
def test_batch_equals_single(pipe_kw, separate_sh):
    if separate_sh and pipe_kw.get("convert_SHs_python"):
        pytest.skip("colours precomputed: no SH split")
    m, cams = _scene()
    pipe = PipelineParams(**pipe_kw)
    bg = torch.tensor([0.2, 0.3, 0.4], device=DEV)
    if pipe_kw.get("convert_SHs_python"):
        cams = [c for c in cams if c is cams[0]] + cams[1:2]  # one colour set per batch: a shared centre
        cams[1].camera_center = cams[0].camera_center
    with torch.no_grad():
        bpkg = batch_render(cams, m, pipe, bg, separate_sh=separate_sh)
        maxH = max(c.image_height for c in cams)
        maxW = max(c.image_width for c in cams)
        assert bpkg["render"].shape == (len(cams), 3, maxH, maxW)
        assert bpkg["depth"].shape == (len(cams), 1, maxH, maxW)
        P = m.get_xyz.shape[0]
        max_radii = torch.zeros(P, dtype=torch.int32, device=DEV)
        vis = torch.zeros(P, dtype=torch.bool, device=DEV)
        count = torch.zeros(P, dtype=torch.int64, device=DEV)
        for i, c in enumerate(cams):
            pkg = render(c, m, pipe, bg, separate_sh=separate_sh)
            H, W = c.image_height, c.image_width
            for key in ("render", "depth"):
                assert torch.allclose(bpkg[key][i, :, :H, :W], pkg[key], atol=1e-6), f"{key} differs for camera {i}"
                assert _absmax(bpkg[key][i, :, H:, :]) == 0.0, "padding rows must be zero"
                assert _absmax(bpkg[key][i, :, :, W:]) == 0.0, "padding columns must be zero"
            max_radii = torch.max(max_radii, pkg["radii"])
            vis[pkg["visibility_filter"]] = True
            count += (pkg["radii"] > 0).to(torch.int64)
        assert torch.equal(bpkg["max_radii"], max_radii)
        assert torch.equal(bpkg["visibility_filter"], vis.nonzero())
        assert torch.equal(bpkg["viewcount"], count)


def test_batch_slices_match_oracle():
    m, cams = _scene()
    pipe = PipelineParams()
    bg = torch.tensor([0.1, 0.6, 0.2])
    with torch.no_grad():
        bpkg = batch_render(cams, m, pipe, bg.to(DEV))
    mc = synthetic_gaussians(6000, 2, seed=0, s0=0.02, n_cams=5)
    for i, c in enumerate(orbit_cameras(2, 96, 80, seed=1) + orbit_cameras(2, 64, 48, seed=5)
                          + orbit_cameras(1, 40, 33, seed=9)):
        img, radii, invd, _ = tr.render_model(mc, c, bg)
        H, W = c.image_height, c.image_width
        assert (bpkg["render"][i, :, :H, :W].cpu() - img).abs().max() <= 1e-4
        assert (bpkg["depth"][i, :, :H, :W].cpu() - invd).abs().max() <= 1e-4


def test_batch_loss_gradients_equal_sum_of_single():
    """tests/test_batch_training_loss.py:104-110: grads of a loss over the batch == sum over views (1e-5)."""
    m, cams = _scene()
    pipe = PipelineParams()
    bg = torch.zeros(3, device=DEV)
    g = torch.Generator().manual_seed(12)
    maxH = max(c.image_height for c in cams)
    maxW = max(c.image_width for c in cams)
    wts = torch.randn(len(cams), 3, maxH, maxW, generator=g).to(DEV)
    leaves = m.params()
    for t in leaves:
        t.grad = None
    bpkg = batch_render(cams, m, pipe, bg)
    (bpkg["render"] * wts).sum().backward()
    gb = [t.grad.detach().clone() if t.grad is not None else torch.zeros_like(t) for t in leaves]
    for t in leaves:
        t.grad = None
    for i, c in enumerate(cams):
        pkg = render(c, m, pipe, bg)
        H, W = c.image_height, c.image_width
        (pkg["render"] * wts[i, :, :H, :W]).sum().backward()
    gs = [t.grad.detach().clone() if t.grad is not None else torch.zeros_like(t) for t in leaves]
    assert float(gs[1].abs().max()) > 0 and float(gs[3].abs().max()) > 0, "gradients must reach the leaves"
    for a, b in zip(gb, gs):
        scale = max(float(b.abs().max()), 1e-8)
        assert float((a - b).abs().max()) <= 1e-5 * max(scale, 1.0)


def test_batch_jvp_equals_single_jvps():
    from diff_gaussian_rasterization.batch_render import BatchGaussianRasterizationSettings, BatchGaussianRasterizer
    from scenes import gpu_settings
    import math
    m, cams = _scene()
    bg = torch.zeros(3, device=DEV)
    a0 = {"means3D": m.get_xyz.detach(), "opacities": m.get_opacity.detach(), "scales": m.get_scaling.detach(),
          "rotations": m.get_rotation.detach(), "shs": m.get_features.detach().contiguous()}
    gen = torch.Generator().manual_seed(13)
    tang = {k: torch.randn(v.shape, generator=gen).to(DEV) for k, v in a0.items()}
    st = BatchGaussianRasterizationSettings(
        batch_size=len(cams), image_heights=[c.image_height for c in cams], image_widths=[c.image_width for c in cams],
        tanfovxs=[math.tan(c.FoVx * 0.5) for c in cams], tanfovys=[math.tan(c.FoVy * 0.5) for c in cams], bg=bg,
        scale_modifier=1.0, viewmatrices=[c.world_view_transform for c in cams],
        projmatrices=[c.full_proj_transform for c in cams], sh_degree=m.active_sh_degree,
        camposes=[c.camera_center for c in cams], prefiltered=False, debug=False, antialiasing=False)
    from diff_gaussian_rasterization import GaussianRasterizer
    with torch.no_grad(), fwAD.dual_level():
        a = {k: fwAD.make_dual(v, tang[k]) for k, v in a0.items()}
        c, _, d = BatchGaussianRasterizer(st)(means2D=torch.zeros_like(a0["means3D"]), **a)
        bt = fwAD.unpack_dual(c).tangent.clone()
        for i, cam in enumerate(cams):
            ci, _, _ = GaussianRasterizer(gpu_settings(cam, m.active_sh_degree, bg))(
                means2D=torch.zeros_like(a0["means3D"]), **a)
            ti = fwAD.unpack_dual(ci).tangent
            H, W = cam.image_height, cam.image_width
            assert torch.allclose(bt[i, :, :H, :W], ti, atol=1e-6)
            assert _absmax(bt[i, :, H:, :]) == 0.0 and _absmax(bt[i, :, :, W:]) == 0.0
