"""GPU parity of the fused LM operator and device CG against the reference solver's golden vectors.

tests/golden/solver_golden.npz was produced by the reference's own cgls_damped /
LinearSolverFunctions / GaussianModelState (imported from /root/reference, make_golden.py) around
the CPU oracle renderer.  Here the same scene runs through libgslm (raw-parameter preprocess,
fused JVP->VJP matvec, gather-sum backward, device scalars) and must reproduce:
  loss (rel 1e-5), J^T b and (J^T J + D) v (1e-5 of the vector's max), and the CGLS solutions of
  the reference schedule (max_iter=2, restart_iter=1) and of 10 iterations: the LM model decrease of the step (one-
  sided, at most 1e-6 relative less than the reference step's) and the step itself (rel 1e-5 in norm for the 2 x 1
  schedule, 1e-4 for 10 x 10; see CGLS_CASES).
  The CPU oracle itself reaches 1.6e-7 / 1.3e-6 on the same goldens (tests/test_oracle_golden.py).
"""
import os

import numpy as np
import pytest
import torch

from gslm.cameras import orbit_cameras
from gslm.model import GaussianModel
from margins import record

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _load():
    d = np.load(os.path.join(HERE, "golden", "solver_golden.npz"))
    P, D, W, H, s0, nv = d["scene"]
    P, D, W, H, nv = int(P), int(D), int(W), int(H), int(nv)
    m = GaussianModel(D)
    t = lambda k: torch.from_numpy(d[f"in_{k}"]).cuda()
    m.set_params(t("xyz"), t("features_dc"), t("features_rest"), t("scaling"), t("rotation"), t("opacity"),
                 t("exposure"))
    m.active_sh_degree = D
    cams = orbit_cameras(nv, W, H, seed=1, images=[torch.from_numpy(d[f"gt{i}"]) for i in range(nv)])
    for c in cams:
        c.to("cuda")
    return d, m, cams


def _err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-12)


def _close(a, b, tol):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() <= tol * max(np.abs(b).max(), 1e-12)


def test_loss_rhs_matvec_match_reference_solver():
    from gslm.lm import LMProblem
    d, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3))
    loss = float(prob.evaluate())
    T = "test_loss_rhs_matvec_match_reference_solver"
    assert record(T, "loss rel", abs(loss - float(d["loss"])) / float(d["loss"]), 1e-5) <= 1e-5
    g = prob.rhs(prob.zeros())
    assert record(T, "J^T b (of max)", _err(g.cpu().numpy(), d["Jtb"]), 1e-5) <= 1e-5
    v = torch.from_numpy(d["v"]).cuda()
    y = prob.matvec(v, prob.zeros())
    assert record(T, "(J^T J + D) v (of max)", _err(y.cpu().numpy(), d["Av"]), 1e-5) <= 1e-5


def _model_gap(prob, g, x, ref, signed=False):
    """(m(x) - m(ref)) / |m(ref)| for the LM model m(v) = 1/2 v^T A v - g^T v on this (GPU) operator (its absolute
    value unless `signed`): how much less (positive) or more (negative) the step decreases the model than the reference
    solver's step -- second order in their difference, so stable where the coordinates of an ill-conditioned solve are
    not."""
    def mval(v):
        av = prob.matvec(v, prob.zeros()).double()
        return float(0.5 * (v.double() * av).sum() - (g.double() * v.double()).sum())
    mr = mval(torch.from_numpy(np.asarray(ref, dtype=np.float32)).cuda())
    d = (mval(x) - mr) / abs(mr)
    return d if signed else abs(d)


# The reference solver's iterates (solver_golden.npz, float32 on the CPU oracle).  Primary: the LM model decrease of
# the step, ONE-SIDED (round 6): (m(x) - m(ref)) / |m(ref)| <= MODEL_BEHIND -- the GPU step may
# decrease the model more than the reference solver's step by any amount, less by at most 1e-6 (worst measured: 5.6e-8
# in magnitude, 10 x 10); |gap| <= 1e-4 stays as a gross-error guard.  The coordinates are held to round 4's bounds:
# 1e-5 for the 2 x 1 schedule (measured 8.7e-6 of the norm: the GPU operator's hardware exp / rcp) and 1e-4
# for 10 x 10 (measured 1.6e-5).  Every kernel is deterministic, so these are reproducible run to run.
CGLS_CASES = [((2, 1), "x_ref_schedule", 1e-5), ((10, 10), "x_ten", 1e-4)]
MODEL_BEHIND = 1e-6


@pytest.mark.parametrize("sched,key,tol", CGLS_CASES)
def test_cgls_matches_reference_schedule(sched, key, tol):
    from gslm.lm import LMProblem, cgls_fused
    d, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    g = prob.rhs(prob.zeros())
    x, info = cgls_fused(prob, g, max_iter=sched[0], restart_iter=sched[1], check_every=True)
    ref = d[key]
    err = np.linalg.norm(x.cpu().numpy().astype(np.float64) - ref) / np.linalg.norm(ref)
    T = "test_cgls_matches_reference_schedule"
    gap = _model_gap(prob, g, x, ref, signed=True)
    record(T, f"CGLS {sched} model decrease behind (rel)", max(gap, 0.0), MODEL_BEHIND)
    record(T, f"CGLS {sched} model decrease |gap| (guard)", abs(gap), 1e-4)
    assert record(T, f"CGLS {sched} iterate rel", err, tol) < tol, err
    assert gap <= MODEL_BEHIND and abs(gap) <= 1e-4, gap


def test_cg_nocheck_matches_checked():
    """Benchmark mode (no host sync per iteration) produces the same iterates."""
    from gslm.lm import LMProblem, cgls_fused
    d, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    g = prob.rhs(prob.zeros())
    x1, _ = cgls_fused(prob, g, max_iter=5, restart_iter=5, check_every=True)
    x2, _ = cgls_fused(prob, g, max_iter=5, restart_iter=5, check_every=False)
    assert torch.equal(x1, x2)


def test_matvec_deterministic():
    """No float atomics: two applications are bitwise identical."""
    from gslm.lm import LMProblem
    d, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    v = torch.from_numpy(d["v"]).cuda()
    y1 = prob.matvec(v, prob.zeros()).clone()
    y2 = prob.matvec(v, prob.zeros())
    assert torch.equal(y1, y2)


def test_fused_dot_and_cg_update():
    """<v, A v> fused into the gather and the one-pass CG update match plain torch algebra."""
    from gslm import _lib
    from gslm.lm import LMProblem
    d, m, cams = _load()
    prob = LMProblem(m, cams[:1], torch.zeros(3))
    prob.evaluate()
    v = torch.from_numpy(d["v"]).cuda()
    sc = torch.zeros(4, dtype=torch.float64, device="cuda")
    y = prob.zeros()
    assert prob.matvec_dot(v, y, sc.data_ptr())
    ref = (v.double() * y.double()).sum()
    assert abs(sc[0].item() - ref.item()) <= 1e-9 * abs(ref.item())
    # x += a p ; s -= a q ; gamma' = <s, s>
    g = torch.Generator().manual_seed(5)
    p, q, x, s = (torch.randn(v.numel(), generator=g).cuda() for _ in range(4))
    x0, s0 = x.clone(), s.clone()
    sc[1], sc[2] = 3.0, 2.0
    _lib.check(_lib.lib.gslm_cg_update(v.numel(), sc.data_ptr() + 8, sc.data_ptr() + 16, p.data_ptr(), q.data_ptr(),
                                       x.data_ptr(), s.data_ptr(), prob.dot_scratch.data_ptr(), sc.data_ptr() + 24,
                                       _lib.stream_handle()))
    torch.cuda.synchronize()
    assert torch.allclose(x, x0 + 1.5 * p, atol=1e-6) and torch.allclose(s, s0 - 1.5 * q, atol=1e-6)
    assert abs(sc[3].item() - (s.double() ** 2).sum().item()) <= 1e-9 * sc[3].item()


def test_lm_step_decreases_loss():
    from gslm.lm import lm_step
    d, m, cams = _load()
    out = lm_step(m, cams, cams, torch.zeros(3), max_iter=2, restart_iter=1)
    assert out["final_val_loss"] <= out["start_loss"]


def test_fused_xpby_matches_separate():
    """The deferred CG direction update p = s + beta p fused into the tangent kernel (all groups and
    the exposure tail) gives the same p and the same (J^T J + D) p, bitwise, as gslm_xpby_dev + matvec."""
    from gslm import _lib
    from gslm.lm import LMProblem
    d, m, cams = _load()
    prob = LMProblem(m, cams[:1], torch.zeros(3))
    prob.evaluate()
    n = prob.layout.numel
    g = torch.Generator().manual_seed(8)
    s = torch.randn(n, generator=g).cuda()
    p = torch.randn(n, generator=g).cuda()
    lo, hi = prob.layout.offsets["xyz"]
    s[lo:hi] = 0
    p[lo:hi] = 0
    sc = torch.tensor([3.0, 7.0], dtype=torch.float64, device="cuda")  # beta = 3 / 7
    num, den = sc.data_ptr(), sc.data_ptr() + 8
    p1 = p.clone()
    _lib.check(_lib.lib.gslm_xpby_dev(n, s.data_ptr(), num, den, p1.data_ptr(), _lib.stream_handle()))
    y1 = prob.matvec(p1, prob.zeros()).clone()
    p2 = p.clone()
    y2 = prob.zeros()
    prob.matvec_dot(p2, y2, None, pre=(s, num, den))
    torch.cuda.synchronize()
    assert torch.equal(p1, p2)
    assert torch.equal(y1, y2)


def test_tail_rows_written_once_per_geometry():
    """GSLM_MV_TAIL_CLEAN: the zero rows of never-blended entries are written by the first product on a
    geometry and skipped afterwards.  A scratch poisoned with NaN before the first product, a second
    product reusing the tail, and a product after the drop-in rhs (whose backward reuses the scratch
    with 48-byte rows) must all equal a fresh problem's product bitwise."""
    from gslm.lm import LMProblem
    d, m, cams = _load()
    v = torch.from_numpy(d["v"]).cuda()
    fresh = LMProblem(m, cams, torch.zeros(3))
    fresh.evaluate()
    ref = fresh.matvec(v, fresh.zeros()).clone()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    for vr in prob.views:
        vr.scratch.view(torch.float32)[: vr.scratch.numel() // 4].fill_(float("nan"))
    y1 = prob.matvec(v, prob.zeros()).clone()
    assert all(vr.tail_clean for vr in prob.views)
    y2 = prob.matvec(v, prob.zeros()).clone()
    prob.rhs(prob.zeros(), fused=False)  # the drop-in backward's 48-byte rows overwrite the scratch
    assert not any(vr.tail_clean for vr in prob.views)
    y3 = prob.matvec(v, prob.zeros())
    assert torch.equal(y1, ref) and torch.equal(y2, ref) and torch.equal(y3, ref)


@pytest.mark.parametrize("with_mask", [False, True])
def test_fused_residual_matches_reference_formulas(with_mask):
    """gslm_lm_residual against the reference's torch expressions (batch_render.py:118 clamp,
    batch_training_loss.py:10-17 / 56-67, loss_image_state.py:16-19): r, weight and the J^T b seed
    bit-identical, loss = 2 ||r||^2 to 1e-12, on renders with values outside [0, 1]."""
    from gslm import _lib
    H, W = 37, 53
    g = torch.Generator().manual_seed(11)
    R = (torch.rand(3, H, W, generator=g) * 2.0 - 0.5).cuda()
    gt = torch.rand(3, H, W, generator=g).cuda()
    m = torch.rand(1, H, W, generator=g).cuda() if with_mask else None
    res, w, seed = (torch.empty_like(R) for _ in range(3))
    loss = torch.full((), 5.0, dtype=torch.float64, device="cuda")
    scratch = torch.empty(_lib.lib.gslm_residual_scratch_bytes(H, W) // 8, dtype=torch.float64, device="cuda")
    for acc in (0, 1):
        _lib.check(_lib.lib.gslm_lm_residual(H, W, R.data_ptr(), gt.data_ptr(), None if m is None else m.data_ptr(),
                                             res.data_ptr(), w.data_ptr(), seed.data_ptr(), scratch.data_ptr(),
                                             scratch.numel() * 8, loss.data_ptr(), acc, _lib.stream_handle()))
    torch.cuda.synchronize()
    mm = torch.ones(1, H, W, device="cuda") if m is None else m
    inside = ((R >= 0) & (R <= 1)).to(torch.float32)
    r_ref = mm * R.clamp(0, 1) - gt
    assert torch.equal(res, r_ref)
    assert torch.equal(w, mm * mm * inside)
    assert torch.equal(seed, -2.0 * mm * inside * r_ref)
    ref_loss = 2.0 * 2.0 * (r_ref.double() ** 2).sum().item()  # written once, then accumulated once
    assert abs(loss.item() - ref_loss) <= 1e-12 * ref_loss


def test_fused_rhs_matches_dropin_backward():
    """J^T b on the LM path (seeded back-to-front pass into LM rows + LM gather) equals the drop-in
    gslm_backward's (general rows), up to summation order; then the matvec reusing the tail rows the
    fused rhs wrote matches a fresh problem's product bitwise."""
    from gslm.lm import LMProblem
    d, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    g_fused = prob.rhs(prob.zeros()).clone()
    assert all(vr.tail_clean for vr in prob.views)
    v = torch.from_numpy(d["v"]).cuda()
    y = prob.matvec(v, prob.zeros()).clone()
    g_drop = prob.rhs(prob.zeros(), fused=False)
    assert _close(g_fused.cpu().numpy(), g_drop.cpu().numpy(), 1e-5)
    fresh = LMProblem(m, cams, torch.zeros(3))
    fresh.evaluate()
    assert torch.equal(y, fresh.matvec(v, fresh.zeros()))


def test_culled_gaussians_get_exact_zero_rows():
    """Gaussians the forward culls (radii 0: behind the camera) have exactly zero J^T b and (J^T J) v rows
    in every group -- the SH epilogue stages them too (a NaN there once came from an unset register)."""
    from gslm.lm import LMProblem
    d, m, cams = _load()
    P = m._xyz.shape[0]
    behind = cams[0].camera_center.cuda() * 1.5  # past the camera, looking away from the scene
    with torch.no_grad():
        xyz = m._xyz.detach().clone()
        xyz[::3] = behind + 0.01 * torch.randn_like(xyz[::3])
    m.set_params(xyz, m._features_dc, m._features_rest, m._scaling, m._rotation, m._opacity, m._exposure)
    for proj in (False, True):
        prob = LMProblem(m, cams[:1], torch.zeros(3), sh_projection=proj)
        prob.evaluate()
        culled = prob.views[0].radii == 0
        assert int(culled.sum()) >= P // 3
        g = prob.rhs(prob.zeros())
        v = torch.randn(prob.layout.numel, device="cuda")
        y = prob.matvec(v, prob.zeros())
        assert torch.isfinite(g).all() and torch.isfinite(y).all()
        views = prob.layout.views(g)
        for name in ("features_dc", "features_rest", "scaling", "rotation", "opacity"):
            assert float(views[name][culled].abs().max()) == 0.0, name


@pytest.mark.parametrize("sched,key,tol", CGLS_CASES)
def test_cgls_residual_matches_reference_schedule(sched, key, tol):
    """The reference's own recursion (conjugate_gradient.py:93-104: r -= alpha q, fresh J^T r - D x, fresh
    residual monitor) on the HIP operator against the reference solver's iterates."""
    from gslm.lm import LMProblem, cgls_residual
    d, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    x, info = cgls_residual(prob, max_iter=sched[0], restart_iter=sched[1])
    ref = d[key]
    err = np.linalg.norm(x.cpu().numpy().astype(np.float64) - ref) / np.linalg.norm(ref)
    T = "test_cgls_residual_matches_reference_schedule"
    g = prob.rhs(prob.zeros())
    gap = _model_gap(prob, g, x, ref, signed=True)
    record(T, f"residual-space CGLS {sched} model decrease behind (rel)", max(gap, 0.0), MODEL_BEHIND)
    record(T, f"residual-space CGLS {sched} model decrease |gap| (guard)", abs(gap), 1e-4)
    assert record(T, f"residual-space CGLS {sched} rel", err, tol) < tol, err
    assert gap <= MODEL_BEHIND and abs(gap) <= 1e-4, gap


def test_recursions_against_float64_oracle():
    """10 CGLS iterations of the two float32 recursions (fused normal-equation, residual-space) against the float64
    oracle's CGLS on the golden scene: both decrease the LM model as the float64 step does (rel 1e-5), their
    coordinates stay within 1e-4 of it (measured 9.2e-5) and within 1e-4 of each other (DESIGN.md reports the
    drift)."""
    import copy
    from gslm.lm import LMProblem, cgls_fused, cgls_residual
    from oracle.lm_ref import OracleLMProblem, cgls_ref
    d, m, cams = _load()
    mc = copy.deepcopy(m).to("cpu")
    for t in mc.params():
        t.data = t.data.double()
    ccs = []
    for c in cams:
        cc = copy.deepcopy(c).to("cpu")
        for k in ("original_image", "alpha_mask", "world_view_transform", "projection_matrix", "full_proj_transform",
                  "camera_center"):
            setattr(cc, k, getattr(cc, k).double())
        ccs.append(cc)
    op = OracleLMProblem(mc, ccs, torch.zeros(3, dtype=torch.float64))
    op.evaluate()
    x64 = cgls_ref(op, op.rhs(), 10, 10)
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    xf, _ = cgls_fused(prob, prob.rhs(prob.zeros()), max_iter=10, restart_iter=10, check_every=True)
    xr, _ = cgls_residual(prob, max_iter=10, restart_iter=10)
    ef = float((xf.double().cpu() - x64).norm() / x64.norm())
    er = float((xr.double().cpu() - x64).norm() / x64.norm())
    efr = float((xf.double() - xr.double()).norm().cpu() / x64.norm())
    print(f"10-iteration drift vs float64 oracle: fused {ef:.3e}, residual-space {er:.3e}, between {efr:.3e}")
    T = "test_recursions_against_float64_oracle"
    # primary: the steps' LM model decrease against the float64 step's (on this operator; second order in their
    # difference); the coordinates against the float64 oracle carry the float32 operator's rounding amplified by 10
    # iterations (9.2e-5, the log2e-perturbed build 9.2e-5 too) and are held to round 4's 1e-4 again (round 5 had
    # widened it to 1e-3); the two float32 recursions on the same operator stay tight
    gf = prob.rhs(prob.zeros())
    x64f = x64.float().cuda()
    mf = record(T, "fused: model decrease rel vs float64", _model_gap(prob, gf, xf, x64f.cpu().numpy()), 1e-5)
    mr = record(T, "residual-space: model decrease rel vs float64", _model_gap(prob, gf, xr, x64f.cpu().numpy()), 1e-5)
    record(T, "fused vs float64 oracle (coordinates)", ef, 1e-4)
    record(T, "residual-space vs float64 oracle (coordinates)", er, 1e-4)
    record(T, "fused vs residual-space", efr, 1e-4)
    assert mf <= 1e-5 and mr <= 1e-5, (mf, mr)
    assert ef < 1e-4 and er < 1e-4 and efr < 1e-4, (ef, er, efr)
