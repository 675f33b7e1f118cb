"""CPU: the oracle's linearisation -- forward-AD JVP vs central finite differences,
and the adjoint identity <u, J v> = <J^T u, v> between its JVP and its autograd VJP (the
tests/test_matvec.py:51-86 criterion), in float64."""
import pytest
import torch
import torch.autograd.forward_ad as fwAD

from oracle import torch_raster as tr
from scenes import activated, make_scene, oracle_settings


def _inputs(name, dtype=torch.float64):
    model, cams = make_scene(name)
    a = {k: v.to(dtype) for k, v in activated(model).items()}
    return model, cams[0], a


def _render(a, st, m2=None):
    m2 = torch.zeros_like(a["means3D"]) if m2 is None else m2
    c, _, d = tr.rasterize(a["means3D"], m2, a["opacities"], st, shs=a["shs"], scales=a["scales"],
                           rotations=a["rotations"])
    return c, d


@pytest.mark.parametrize("name", ["dense_2k_sh3_64x48", "tiny_300_sh2_40x33"])
def test_jvp_matches_central_differences(name):
    model, cam, a = _inputs(name)
    st = oracle_settings(cam, model.active_sh_degree, torch.tensor([0.2, 0.4, 0.6], dtype=torch.float64))
    g = torch.Generator().manual_seed(9)
    v = {k: torch.randn(x.shape, generator=g, dtype=torch.float64) for k, x in a.items()}
    v["means3D"] *= 1e-2  # keep the xyz direction comparable in pixels
    with torch.no_grad(), fwAD.dual_level():
        ad = {k: fwAD.make_dual(x, v[k]) for k, x in a.items()}
        c, d = _render(ad, st)
        jc, jd = fwAD.unpack_dual(c).tangent, fwAD.unpack_dual(d).tangent
    eps = 1e-7
    with torch.no_grad():
        cp, dp = _render({k: x + eps * v[k] for k, x in a.items()}, st)
        cm, dm = _render({k: x - eps * v[k] for k, x in a.items()}, st)
    fc, fd = (cp - cm) / (2 * eps), (dp - dm) / (2 * eps)
    # threshold crossings (alpha = 1/255, T = 1e-4, tan-FoV clamp) are measure-zero; allow a few pixels
    bad = ((jc - fc).abs() > 1e-5 * (1 + fc.abs())).sum().item()
    assert bad <= 3, bad
    assert ((jd - fd).abs() > 1e-5 * (1 + fd.abs())).sum().item() <= 3


@pytest.mark.parametrize("name", ["dense_2k_sh3_64x48", "mid_8k_sh1_96x80"])
def test_adjoint_identity(name):
    model, cam, a = _inputs(name)
    st = oracle_settings(cam, model.active_sh_degree, torch.tensor([0.1, 0.2, 0.3], dtype=torch.float64))
    g = torch.Generator().manual_seed(10)
    v = {k: torch.randn(x.shape, generator=g, dtype=torch.float64) for k, x in a.items()}
    H, W = cam.image_height, cam.image_width
    uc = torch.randn(3, H, W, generator=g, dtype=torch.float64)
    ud = torch.randn(1, H, W, generator=g, dtype=torch.float64)
    with torch.no_grad(), fwAD.dual_level():
        ad = {k: fwAD.make_dual(x, v[k]) for k, x in a.items()}
        c, d = _render(ad, st)
        lhs = (fwAD.unpack_dual(c).tangent * uc).sum() + (fwAD.unpack_dual(d).tangent * ud).sum()
    ar = {k: x.clone().requires_grad_(True) for k, x in a.items()}
    c, d = _render(ar, st)
    ((c * uc).sum() + (d * ud).sum()).backward()
    rhs = sum((ar[k].grad * v[k]).sum() for k in ar)
    assert abs(lhs.item() - rhs.item()) <= 1e-10 * max(1.0, abs(rhs.item()))


def test_alpha_clamp_is_pass_through():
    """Upstream backward: dL/dopacity = G * dL/dalpha with no mask at the 0.99 clamp (App. B)."""
    x = torch.tensor([2.0], dtype=torch.float64, requires_grad=True)
    alpha = x + (torch.clamp_max(x, 0.99) - x).detach()
    alpha.backward()
    assert alpha.item() == 0.99 and x.grad.item() == 1.0


def test_empty_and_culled_inputs():
    """P = 0 and all-culled inputs render the background with zero radii (edge cases)."""
    _, cam, a = _inputs("tiny_300_sh2_40x33", torch.float32)
    st = oracle_settings(cam, 2, torch.tensor([0.25, 0.5, 0.75]))
    empty = {k: v[:0] for k, v in a.items()}
    c, r, d = tr.rasterize(empty["means3D"], empty["means3D"].clone(), empty["opacities"], st, shs=empty["shs"],
                           scales=empty["scales"], rotations=empty["rotations"])
    assert r.numel() == 0 and torch.allclose(c, torch.tensor([0.25, 0.5, 0.75]).view(3, 1, 1).expand_as(c))
    behind = dict(a)
    behind["means3D"] = cam.camera_center.view(1, 3).expand_as(a["means3D"]).clone()  # z_view = 0 <= 0.2
    c, r, d = tr.rasterize(behind["means3D"], torch.zeros_like(behind["means3D"]), behind["opacities"], st,
                           shs=behind["shs"], scales=behind["scales"], rotations=behind["rotations"])
    assert (r == 0).all() and (d == 0).all()


def _rest_basis(model, cam):
    """Unit SH-rest basis directions Bh_i = B_rest(dir_i) / |B_rest(dir_i)| [P, K-1] (utils/sh_utils.py basis)."""
    D = model.active_sh_degree
    K = (D + 1) ** 2
    d = model._xyz.detach().double() - cam.camera_center.double()
    d = d / d.norm(dim=1, keepdim=True)
    eye = torch.eye(K, dtype=torch.float64).expand(d.shape[0], 1, K, K)[:, 0]  # [P, K, K]: coefficient k = e_k
    B = torch.stack([tr.eval_sh(D, eye[:, :, k:k + 1].expand(-1, -1, 3), d)[:, 0] for k in range(K)], 1)  # [P, K]
    Br = B[:, 1:]
    return Br / Br.norm(dim=1, keepdim=True)


@pytest.mark.parametrize("ssim", [False, True])
def test_single_view_krylov_space_keeps_sh_rest_in_basis_span(ssim):
    """The claim behind GSLM_MV_SH_REST_PROJECTED: with one view, J^T b and (J^T J + D) applied to any
    vector whose SH-rest rows are Bh_i (x) c_i keep the SH-rest rows in span{Bh_i (x) e_c}, so CG from
    x0 = 0 never leaves it (checked on the oracle's autograd / forward-AD operator, float32)."""
    from oracle.lm_ref import OracleLMProblem
    model, cams = make_scene("tiny_300_sh2_40x33")
    cam = cams[0]
    cam.original_image = torch.rand(3, cam.image_height, cam.image_width, generator=torch.Generator().manual_seed(3))
    op = OracleLMProblem(model, [cam], torch.zeros(3), ssim=ssim)
    op.evaluate()
    Bh = _rest_basis(model, cam).float()  # [P, K-1]
    a, b = op.layout.offsets["features_rest"]
    P, Km1 = Bh.shape

    def off_span(vec):
        R = vec[a:b].view(P, Km1, 3)
        coef = (Bh[:, :, None] * R).sum(1)  # [P, 3]
        resid = R - Bh[:, :, None] * coef[:, None, :]
        return float(resid.abs().max()), float(R.abs().max())

    g = op.rhs()
    r, scale = off_span(g)
    assert scale > 0 and r <= 1e-5 * scale
    y = op.zeros()
    op.matvec(g, y)
    r, scale = off_span(y)
    assert scale > 0 and r <= 1e-5 * scale
    # and a generic vector of the span (random coefficients in every group)
    v = torch.randn(op.layout.numel, generator=torch.Generator().manual_seed(4))
    v[a:b] = (Bh[:, :, None] * torch.randn(P, 1, 3, generator=torch.Generator().manual_seed(5))).reshape(-1)
    op.matvec(v, y)
    r, scale = off_span(y)
    assert r <= 1e-5 * scale
