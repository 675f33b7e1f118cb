"""GPU parity of the drop-in rasterizer (forward / VJP / JVP) against the CPU oracle.

Tolerances: images within 1e-4 L-inf per channel (BASELINE north_star); integer / index work
(radii, tiles_touched, num_rendered, sorted point list, tile ranges, n_contrib) bit-exact;
gradients / tangents within 1e-4 relative to the tensor's max magnitude (the reference's own grad
check uses 1e-5 absolute on unit-scale losses, tests/test_batch_training_loss.py:104-110).
"""
import ctypes
import math

import pytest
import torch
import torch.autograd.forward_ad as fwAD

from oracle import torch_raster as tr
from scenes import SCENES, activated, gpu_settings, make_scene, oracle_settings

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _gpu_forward_internals(model, cam, D, bg=None):
    from diff_gaussian_rasterization import _gaussians, forward_buffers
    from gslm import _lib
    a = {k: v.to(DEV) for k, v in activated(model).items()}
    st = gpu_settings(cam, D, bg)
    view = _lib.view_from_settings(st)
    P = a["means3D"].shape[0]
    g = _gaussians(P, a["means3D"], a["opacities"].reshape(-1).contiguous(), a["scales"], a["rotations"], None,
                   a["shs"], None, None)
    color, radii, invd, geom, binning, image, N = forward_buffers(view, g, DEV)
    H, W = st.image_height, st.image_width
    ntiles = ((W + 15) // 16) * ((H + 15) // 16)
    pl = torch.zeros(max(N, 1), dtype=torch.int32, device=DEV)
    rg = torch.zeros(ntiles * 2, dtype=torch.int32, device=DEV)
    tiles = torch.zeros(P, dtype=torch.int32, device=DEV)
    fT = torch.zeros(H * W, dtype=torch.float32, device=DEV)
    nc = torch.zeros(H * W, dtype=torch.int32, device=DEV)
    _lib.check(_lib.lib.gslm_inspect(geom.data_ptr(), P, binning.data_ptr(), N, H, W, image.data_ptr(),
                                     pl.data_ptr(), rg.data_ptr(), tiles.data_ptr(), fT.data_ptr(), nc.data_ptr(),
                                     None, _lib.stream_handle()))
    torch.cuda.synchronize()
    return dict(color=color.cpu(), radii=radii.cpu(), invdepth=invd.cpu(), N=N, point_list=pl[:N].cpu().long(),
                ranges=rg.view(-1, 2).cpu().long(), tiles=tiles.cpu().long(), final_T=fT.view(H, W).cpu(),
                n_contrib=nc.view(H, W).cpu())


@pytest.mark.parametrize("name", list(SCENES))
def test_forward_parity(name):
    model, cams = make_scene(name)
    D = model.active_sh_degree
    for cam in cams:
        st = oracle_settings(cam, D)
        a = activated(model)
        with torch.no_grad():
            c, r, d, I = tr.rasterize(a["means3D"], torch.zeros_like(a["means3D"]), a["opacities"], st, shs=a["shs"],
                                      scales=a["scales"], rotations=a["rotations"], return_internals=True)
        G = _gpu_forward_internals(model, cam, D)
        assert torch.equal(G["radii"], r), "radii must match exactly"
        assert torch.equal(G["tiles"], I["pre"]["tiles_touched"]), "tiles_touched must match exactly"
        assert G["N"] == I["point_list"].numel(), "num_rendered must match"
        assert torch.equal(G["point_list"], I["point_list"]), "sorted point list must match exactly"
        assert torch.equal(G["ranges"], I["ranges"]), "tile ranges must match exactly"
        assert torch.equal(G["n_contrib"].long(), I["n_contrib"].long()), "n_contrib must match exactly"
        assert (G["final_T"] - I["final_T"]).abs().max() <= 1e-5
        assert (G["color"] - c).abs().max() <= 1e-4
        assert (G["invdepth"] - d).abs().max() <= 1e-4


def _rel_err(a, b):
    scale = b.abs().max().clamp_min(1e-8)
    return ((a - b).abs().max() / scale).item()


@pytest.mark.parametrize("name", ["dense_2k_sh3_64x48", "mid_8k_sh1_96x80", "tiny_300_sh2_40x33"])
@pytest.mark.parametrize("with_depth", [False, True])
def test_backward_parity(name, with_depth):
    from diff_gaussian_rasterization import GaussianRasterizer
    model, cams = make_scene(name)
    D = model.active_sh_degree
    cam = cams[0]
    bg = torch.tensor([0.2, 0.5, 0.9])
    g = torch.Generator().manual_seed(4)
    H, W = cam.image_height, cam.image_width
    dcol = torch.randn(3, H, W, generator=g)
    ddep = torch.randn(1, H, W, generator=g) if with_depth else torch.zeros(1, H, W)

    def run(dev, rast_fn):
        a = {k: v.to(dev).requires_grad_(True) for k, v in activated(model).items()}
        m2 = torch.zeros_like(a["means3D"], requires_grad=True)
        c, _, d = rast_fn(a, m2)
        (c * dcol.to(dev)).sum().__add__((d * ddep.to(dev)).sum()).backward()
        return {k: v.grad.detach().cpu() for k, v in a.items()} | {"means2D": m2.grad.detach().cpu()}

    ref = run("cpu", lambda a, m2: tr.rasterize(a["means3D"], m2, a["opacities"], oracle_settings(cam, D, bg),
                                                 shs=a["shs"], scales=a["scales"], rotations=a["rotations"]))
    got = run(DEV, lambda a, m2: GaussianRasterizer(gpu_settings(cam, D, bg))(
        means3D=a["means3D"], means2D=m2, shs=a["shs"], opacities=a["opacities"], scales=a["scales"],
        rotations=a["rotations"]))
    for k in ref:
        assert _rel_err(got[k], ref[k]) < 1e-4, f"grad {k}: rel err {_rel_err(got[k], ref[k]):.3e}"


@pytest.mark.parametrize("name", ["dense_2k_sh3_64x48", "mid_8k_sh1_96x80", "tiny_300_sh2_40x33"])
def test_jvp_parity(name):
    from diff_gaussian_rasterization import GaussianRasterizer
    model, cams = make_scene(name)
    D = model.active_sh_degree
    cam = cams[0]
    bg = torch.tensor([0.3, 0.1, 0.7])
    a0 = activated(model)
    gen = torch.Generator().manual_seed(3)
    tang = {k: torch.randn(v.shape, generator=gen) for k, v in a0.items()}
    t_m2 = torch.randn(a0["means3D"].shape, generator=gen)

    def run(dev, rast_fn):
        with torch.no_grad(), fwAD.dual_level():
            a = {k: fwAD.make_dual(v.to(dev), tang[k].to(dev)) for k, v in a0.items()}
            m2 = fwAD.make_dual(torch.zeros_like(a0["means3D"]).to(dev), t_m2.to(dev))
            c, _, d = rast_fn(a, m2)
            return fwAD.unpack_dual(c).tangent.cpu(), fwAD.unpack_dual(d).tangent.cpu()

    rc, rd = run("cpu", lambda a, m2: tr.rasterize(a["means3D"], m2, a["opacities"], oracle_settings(cam, D, bg),
                                                   shs=a["shs"], scales=a["scales"], rotations=a["rotations"]))
    gc, gd = run(DEV, lambda a, m2: GaussianRasterizer(gpu_settings(cam, D, bg))(
        means3D=a["means3D"], means2D=m2, shs=a["shs"], opacities=a["opacities"], scales=a["scales"],
        rotations=a["rotations"]))
    assert _rel_err(gc, rc) < 1e-4, f"color tangent rel err {_rel_err(gc, rc):.3e}"
    assert _rel_err(gd, rd) < 1e-4, f"invdepth tangent rel err {_rel_err(gd, rd):.3e}"


@pytest.mark.parametrize("name", ["dense_2k_sh3_64x48", "mid_8k_sh1_96x80"])
def test_adjoint_identity_gpu(name):
    """<u, J v> == <J^T u, v> on the GPU kernels (the tests/test_matvec.py:51-86 criterion, rel 1e-4)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    model, cams = make_scene(name)
    D = model.active_sh_degree
    cam = cams[0]
    st = gpu_settings(cam, D, torch.tensor([0.1, 0.2, 0.3]))
    a0 = {k: v.to(DEV) for k, v in activated(model).items()}
    gen = torch.Generator().manual_seed(7)
    v = {k: torch.randn(x.shape, generator=gen).to(DEV) for k, x in a0.items()}
    H, W = cam.image_height, cam.image_width
    u_c = torch.randn(3, H, W, generator=gen).to(DEV)
    u_d = torch.randn(1, H, W, generator=gen).to(DEV)
    rast = GaussianRasterizer(st)
    with torch.no_grad(), fwAD.dual_level():
        a = {k: fwAD.make_dual(x, v[k]) for k, x in a0.items()}
        c, _, d = rast(means3D=a["means3D"], means2D=torch.zeros_like(a0["means3D"]), shs=a["shs"],
                       opacities=a["opacities"], scales=a["scales"], rotations=a["rotations"])
        lhs = (fwAD.unpack_dual(c).tangent * u_c).sum() + (fwAD.unpack_dual(d).tangent * u_d).sum()
    a = {k: x.clone().requires_grad_(True) for k, x in a0.items()}
    c, _, d = rast(means3D=a["means3D"], means2D=torch.zeros_like(a0["means3D"]), shs=a["shs"],
                   opacities=a["opacities"], scales=a["scales"], rotations=a["rotations"])
    ((c * u_c).sum() + (d * u_d).sum()).backward()
    rhs = sum((a[k].grad * v[k]).sum() for k in a)
    assert abs(lhs.item() - rhs.item()) <= 1e-4 * max(abs(lhs.item()), abs(rhs.item())), (lhs.item(), rhs.item())
