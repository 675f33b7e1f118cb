"""GPU: the projected SH-rest layout of single-view LM problems (GSLM_MV_SH_REST_PROJECTED).

With one view the SH-rest rows of J^T b and of (J^T J + D) v stay in span{Bh_i (x) e_c} (Bh_i the unit
SH-rest basis direction of Gaussian i: tests/test_oracle_properties.py checks the claim on the oracle),
so the CG vectors carry 3 coordinates per Gaussian instead of 3(K-1).  Here the projected products,
J^T b and CGLS solutions, expanded back to the reference layout, must equal the unprojected path's
(1e-5 of the vector's max; solutions rel 1e-4 in norm) and the oracle's (1e-4 of the max)."""
import copy

import numpy as np
import pytest
import torch

from test_gpu_lm import _load

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max()) <= tol * max(float(b.abs().max()), 1e-12)


def _one_view(ssim):
    from gslm.lm import LMProblem
    if ssim:
        # solver_ssim_golden's ground truth: near x ~ gt the sqrt(|x - gt| + 1e-6) residual's curvature makes
        # J^T J sensitive to 1-ulp render differences; that fixture's pixels keep clear of it
        from test_gpu_ssim import _load as _load_ssim
        _, m, cams = _load_ssim()
    else:
        _, m, cams = _load()
    cam = cams[0]
    pf = LMProblem(m, [cam], torch.zeros(3), ssim=ssim, sh_projection=False)
    pp = LMProblem(m, [cam], torch.zeros(3), ssim=ssim, sh_projection=True)
    assert pp.layout.rest_projected and pp.layout.numel < pf.layout.numel
    return m, cam, pf, pp


@pytest.mark.parametrize("ssim", [False, True])
def test_projected_rhs_and_matvec_match_full_and_oracle(ssim):
    from oracle.lm_ref import OracleLMProblem
    m, cam, pf, pp = _one_view(ssim)
    assert abs(float(pf.evaluate()) - float(pp.evaluate())) <= 1e-7 * float(pf.loss)
    gf = pf.rhs(pf.zeros())
    gp = pp.rhs(pp.zeros())
    assert _close(pp.expand(gp), gf, 1e-5)
    assert _close(pp.project(gf), gp, 1e-5)
    # the unfused (drop-in backward) J^T b, projected
    assert _close(pp.rhs(pp.zeros(), fused=False), gp, 1e-5)
    # oracle (reference layout, CPU autograd)
    mc = copy.deepcopy(m).to("cpu")
    cc = copy.deepcopy(cam).to("cpu")
    op = OracleLMProblem(mc, [cc], torch.zeros(3), ssim=ssim)
    op.evaluate()
    assert _close(pp.expand(gp), op.rhs(), 1e-4)
    # a random vector of the projected layout (xyz and exposure zero, as in every LM iterate)
    g = torch.Generator(device="cuda").manual_seed(7)
    v = torch.randn(pp.layout.numel, device="cuda", generator=g)
    for grp in ("xyz", "exposure"):
        a, b = pp.layout.offsets[grp]
        v[a:b] = 0
    yp = pp.matvec(v, pp.zeros())
    vf = pp.expand(v)
    yf = pf.matvec(vf, pf.zeros())
    assert _close(pp.expand(yp), yf, 1e-5)
    yo = op.zeros()
    op.matvec(vf.cpu(), yo)
    assert _close(pp.expand(yp), yo, 1e-4)


@pytest.mark.parametrize("check_every", [True, False])
def test_projected_cgls_matches_full(check_every):
    from gslm.lm import cgls_fused
    m, cam, pf, pp = _one_view(False)
    for p in (pf, pp):
        p.evaluate()
    xf, inf = cgls_fused(pf, pf.rhs(pf.zeros()), max_iter=10, restart_iter=10, check_every=check_every)
    xp, inp = cgls_fused(pp, pp.rhs(pp.zeros()), max_iter=10, restart_iter=10, check_every=check_every)
    assert inf["iters"] == inp["iters"]
    xe = pp.expand(xp)
    err = float((xe.double() - xf.double()).norm() / xf.double().norm())
    assert err < 1e-4, err
    if check_every:
        np.testing.assert_allclose(inp["residuals"], inf["residuals"], rtol=1e-4)


def test_projected_lm_step_matches_full():
    from gslm.lm import lm_step
    d, m, cams = _load()
    m2 = copy.deepcopy(m)
    a = lm_step(m, cams[:1], cams[:1], torch.zeros(3), max_iter=10, restart_iter=10, sh_projection=False)
    b = lm_step(m2, cams[:1], cams[:1], torch.zeros(3), max_iter=10, restart_iter=10, sh_projection=True)
    assert a["best_alpha"] == b["best_alpha"]
    assert abs(a["final_val_loss"] - b["final_val_loss"]) <= 1e-4 * a["final_val_loss"]
    for t1, t2 in zip(m.params(), m2.params()):
        assert _close(t2.detach(), t1.detach(), 1e-4)


def test_projected_and_full_cgls_against_float64_oracle():
    """Both float32 GPU layouts against the float64 oracle CGLS of the same single-view problem: the
    projected solution is as accurate as the full one (rel 2e-3 in norm, the reference-schedule bar)."""
    from gslm.lm import cgls_fused
    from oracle.lm_ref import OracleLMProblem, cgls_ref
    m, cam, pf, pp = _one_view(False)
    mc = copy.deepcopy(m).to("cpu")
    for t in mc.params():
        t.data = t.data.double()
    cc = copy.deepcopy(cam).to("cpu")
    for k in ("original_image", "alpha_mask", "world_view_transform", "projection_matrix", "full_proj_transform",
              "camera_center"):
        setattr(cc, k, getattr(cc, k).double())
    op = OracleLMProblem(mc, [cc], torch.zeros(3, dtype=torch.float64))
    op.evaluate()
    x64 = cgls_ref(op, op.rhs(), 10, 10)
    errs = {}
    for name, p in (("full", pf), ("proj", pp)):
        p.evaluate()
        x, _ = cgls_fused(p, p.rhs(p.zeros()), max_iter=10, restart_iter=10, check_every=True)
        errs[name] = float((p.expand(x).double().cpu() - x64).norm() / x64.norm())
    assert errs["full"] < 2e-3 and errs["proj"] < 2e-3, errs
    assert errs["proj"] <= 2 * errs["full"] + 1e-4, errs
