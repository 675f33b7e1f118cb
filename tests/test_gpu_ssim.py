"""GPU parity of the SSIM residual path against the CPU oracle and the goldens the
reference's own solver produced with the disable_ssim=False residual (tests/golden/solver_ssim_golden.npz).

Tolerances: the SSIM map / residuals 1e-5 relative to the image's max (separable 11 + 11 taps here vs
the reference's 121-tap conv2d: summation order), loss 1e-5, image-space operator 1e-4 of its max, LM
vectors vs the goldens 1e-4 of the vector's max, CG solution 2e-3 (rel, norm) -- as tests/test_gpu_lm.py.
"""
import numpy as np
import pytest
import torch
import torch.autograd.forward_ad as fwAD

from oracle import ssim_ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def _state(H, W):
    from gslm import _lib
    return _lib.u8(_lib.lib.gslm_ssim_state_bytes(H, W), "cuda")


@pytest.mark.parametrize("with_mask", [False, True])
def test_ssim_residual_and_seed(with_mask):
    """r1, r2, loss and the J^T b seed of one view against the oracle's autograd (renders with values
    outside [0, 1], a random alpha mask)."""
    from gslm import _lib
    H, W = 45, 70
    g = torch.Generator().manual_seed(12)
    R = torch.rand(3, H, W, generator=g) * 1.2 - 0.1
    gt = torch.rand(3, H, W, generator=g)
    m = torch.rand(1, H, W, generator=g) if with_mask else torch.ones(1, H, W)
    # oracle
    Rr = R.clone().requires_grad_(True)
    x = Rr.clamp(0, 1) * m
    r1, r2 = ssim_ref.ssim_residuals(x, gt)
    loss = (r1.double() ** 2).sum() + (r2.double() ** 2).sum()
    (0.5 * ((r1 * r1).sum() + (r2 * r2).sum())).backward()
    seed_ref = -Rr.grad
    # GPU
    st = _state(H, W)
    Rg, gtg = R.cuda(), gt.cuda()
    mg = m.cuda() if with_mask else None
    o1, o2, seed = (torch.empty(3, H, W, device="cuda") for _ in range(3))
    lg = torch.zeros((), dtype=torch.float64, device="cuda")
    _lib.check(_lib.lib.gslm_ssim_residual(H, W, Rg.data_ptr(), gtg.data_ptr(), None if mg is None else mg.data_ptr(),
                                           0.2, st.data_ptr(), st.numel(), o1.data_ptr(), o2.data_ptr(),
                                           seed.data_ptr(), lg.data_ptr(), 0, _lib.stream_handle()))
    torch.cuda.synchronize()
    assert _rel(o1.cpu(), r1.detach()) < 1e-5
    assert _rel(o2.cpu(), r2.detach()) < 1e-5
    assert abs(lg.item() - loss.item()) <= 1e-5 * loss.item()
    assert _rel(seed.cpu(), seed_ref) < 1e-4


def test_ssim_normal_operator():
    """u = M (d1^2 + S^T c2^2 S) M jv equals the oracle's J_x^T J_x jv (forward-AD then autograd through
    the clamp, mask, l1 and SSIM residuals) and is symmetric: <a, N b> = <N a, b>."""
    from gslm import _lib
    H, W = 40, 57
    g = torch.Generator().manual_seed(13)
    R = torch.rand(3, H, W, generator=g) * 1.2 - 0.1
    gt = torch.rand(3, H, W, generator=g)
    m = torch.rand(1, H, W, generator=g)
    jv = torch.randn(3, H, W, generator=g)

    def res(Rt):
        r1, r2 = ssim_ref.ssim_residuals(Rt.clamp(0, 1) * m, gt)
        return r1, r2

    with fwAD.dual_level():
        d1, d2 = res(fwAD.make_dual(R, jv))
        t1, t2 = fwAD.unpack_dual(d1).tangent, fwAD.unpack_dual(d2).tangent
    Rr = R.clone().requires_grad_(True)
    r1, r2 = res(Rr)
    ((r1 * t1).sum() + (r2 * t2).sum()).backward()
    u_ref = Rr.grad

    st = _state(H, W)
    Rg, gtg, mg = R.cuda(), gt.cuda(), m.cuda()
    lg = torch.zeros((), dtype=torch.float64, device="cuda")
    seed = torch.empty(3, H, W, device="cuda")
    _lib.check(_lib.lib.gslm_ssim_residual(H, W, Rg.data_ptr(), gtg.data_ptr(), mg.data_ptr(), 0.2, st.data_ptr(),
                                           st.numel(), None, None, seed.data_ptr(), lg.data_ptr(), 0,
                                           _lib.stream_handle()))

    def N(a):
        u = torch.empty(3, H, W, device="cuda")
        _lib.check(_lib.lib.gslm_ssim_normal(H, W, gtg.data_ptr(), st.data_ptr(), a.data_ptr(), u.data_ptr(),
                                             _lib.stream_handle()))
        torch.cuda.synchronize()
        return u

    u = N(jv.cuda())
    assert _rel(u.cpu(), u_ref) < 1e-4
    a, b = torch.randn(3, H, W, generator=g).cuda(), torch.randn(3, H, W, generator=g).cuda()
    lhs, rhs = (a.double() * N(b).double()).sum().item(), (N(a).double() * b.double()).sum().item()
    assert abs(lhs - rhs) <= 1e-4 * max(abs(lhs), abs(rhs))


def _load():
    import os
    from gslm.cameras import orbit_cameras
    from gslm.model import GaussianModel
    here = os.path.dirname(os.path.abspath(__file__))
    d = np.load(os.path.join(here, "golden", "solver_golden.npz"))
    ds = np.load(os.path.join(here, "golden", "solver_ssim_golden.npz"))
    P, D, W, H, s0, nv = d["scene"]
    m = GaussianModel(int(D))
    t = lambda k: torch.from_numpy(d[f"in_{k}"]).cuda()
    m.set_params(t("xyz"), t("features_dc"), t("features_rest"), t("scaling"), t("rotation"), t("opacity"),
                 t("exposure"))
    m.active_sh_degree = int(D)
    cams = orbit_cameras(int(nv), int(W), int(H), seed=1, images=[torch.from_numpy(ds[f"gt{i}"]) for i in range(int(nv))])
    for c in cams:
        c.to("cuda")
    return ds, m, cams


def test_ssim_lm_matches_reference_solver():
    """LMProblem(ssim=True): loss, J^T b, (J^T J + D) v and 10 CGLS iterations vs the reference solver's
    disable_ssim=False run (solver_ssim_golden.npz)."""
    from gslm.lm import LMProblem, cgls_fused
    ds, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3), ssim=True)
    loss = float(prob.evaluate())
    assert abs(loss - float(ds["loss"])) <= 1e-5 * float(ds["loss"])
    g = prob.rhs(prob.zeros())
    assert _rel(g.cpu().numpy(), ds["Jtb"]) < 1e-4
    y = prob.matvec(torch.from_numpy(ds["v"]).cuda(), prob.zeros())
    assert _rel(y.cpu().numpy(), ds["Av"]) < 1e-4
    x, _ = cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=True)
    err = np.linalg.norm(x.cpu().numpy().astype(np.float64) - ds["x_ten"]) / np.linalg.norm(ds["x_ten"])
    assert err < 2e-3, err
