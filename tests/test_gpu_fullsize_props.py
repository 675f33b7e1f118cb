"""Whole-frame properties of the products at BASELINE.json's full sizes (configs[2]: 1M Gaussians SH 3, one 1080p
view; the configs[4] slice: 5M Gaussians, one 3840x2160 view), where the oracle's dense blend over every tile is
too slow for a test (its forward-AD + autograd product takes ~2 min on the host at 100k and ~10x that at 1M; the
oracle comparisons at these sizes run on tile samples, tests/test_gpu_fullsize.py and test_gpu_configs34.py).

Every pixel of the frame enters each check, and each is size-independent:

  * energy identity of the fused LM product, per parameter group:  <v, A v> = 2 ||W^(1/2) J v||^2 with
    A = 2 J^T W J (zero damping), v nonzero in one group only.  The left side is k_render_matvec's JVP pass
    feeding its VJP pass and the LM gather; the right side is the J v pass alone (k_render_jv_wave, jv_out).
    A contribution the VJP drops or mis-scales anywhere in the frame moves <v, A v> by its share of the sum,
    so the 2e-6 bound resolves one tile of the 8,160 at 1080p (1.2e-4 of the sum) or of the 32,400 at 4K.
    Measured: 2.2-2.5e-7 in every group at both sizes -- a consistent offset rather than noise, most likely the
    back-to-front pass recovering the transmittance with v_rcp_f32, whose rounding compounds over a pixel's list;
  * the fused product against its two-pass decomposition, elementwise: A v = 2 J^T (W (J v)) with the J v pass
    and the seeded back-to-front pass (pixel_seed, the J^T b kernel of LMProblem.rhs) as separate launches
    (1e-5 of each group's max; measured: bitwise equal);
  * symmetry <u, A v> = <A u, v> (1e-7 of sqrt(<u, A u> <v, A v>); measured 0.4-1.2e-9);
  * the drop-in pair that an unchanged train_jvp.py drives (`render()` under forward-mode AD, then autograd's
    backward): <u, J^T (J u)> = ||J u||^2 per raw GaussianModel leaf, xyz included -- the screen-position
    tangents and gradients (k_render_jvp<true>, k_render_bwd) over the whole frame (2e-6; measured 2.2-2.3e-7).

The J v pass, the product and the drop-in JVP / VJP are each checked against the oracle on tile samples at these
sizes and over the whole frame at 100k (test_gpu_fullsize.py); these identities extend the whole-frame evidence
to 1M and 5M / 4K.
"""
import types

import pytest
import torch
import torch.autograd.forward_ad as fwAD

from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians

pytestmark = pytest.mark.gpu
DEV = "cuda"
GROUPS = ["features_dc", "features_rest", "scaling", "rotation", "opacity"]
ZERO_DAMP = {k: 0.0 for k in ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure")}
CASES = {
    "cfg2_1M_1080p_projected": (1_000_000, 1920, 1080, True),
    "cfg2_1M_1080p_full": (1_000_000, 1920, 1080, False),
    "cfg4_5M_4K_full": (5_000_000, 3840, 2160, False),
}
TOL = 1e-5         # elementwise, of each group's max
TOL_ENERGY = 2e-6  # relative, of ||J v||^2
TOL_SYM = 1e-7     # relative, of sqrt(<u, A u> <v, A v>)


def _problem(P, W, H, proj):
    from gslm.lm import LMProblem
    gm = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(DEV)
    cam = orbit_cameras(1, W, H, seed=1)[0].to(DEV)
    prob = LMProblem(gm, [cam], torch.zeros(3), gts=[torch.zeros(3, H, W, device=DEV)],
                     alpha_masks=[torch.ones(1, H, W, device=DEV)], damp=ZERO_DAMP, sh_projection=proj)
    prob.evaluate()
    return prob


def _group_direction(layout, group, seed):
    v = torch.zeros(layout.numel)
    a, b = layout.offsets[group]
    v[a:b] = torch.randn(b - a, generator=torch.Generator().manual_seed(seed))
    return v.to(DEV)


def _dot(a, b):
    return float((a.double() * b.double()).sum())


@pytest.mark.parametrize("case", list(CASES))
def test_lm_product_whole_frame_identities(case):
    P, W, H, proj = CASES[case]
    prob = _problem(P, W, H, proj)
    assert prob.layout.rest_projected == proj
    rm = prob.residual_masks()
    # alpha mask 1: the weight m^2 1[0 <= R <= 1] is the residual mask itself (0 / 1)
    assert torch.equal(prob.weights[0], rm[0].expand_as(prob.weights[0]))
    jv = [torch.empty(3, H, W, device=DEV)]
    o = prob.layout.offsets
    for k, g in enumerate(GROUPS):
        v = _group_direction(prob.layout, g, seed=10 + k)
        y = prob.matvec(v, prob.zeros())
        prob.jv_residual(v, rm, jv)                 # W^(1/2) J v (mask 0 / 1)
        lhs, rhs = _dot(v, y), 2.0 * _dot(jv[0], jv[0])
        assert rhs > 0
        print(f"{case} {g}: energy rel {abs(lhs - rhs) / rhs:.2e}", end="")
        assert abs(lhs - rhs) <= TOL_ENERGY * rhs, f"{g}: <v, A v> {lhs:.9e} vs 2 ||J v||_W^2 {rhs:.9e}"
        y2 = prob.jt_residual(jv, rm, prob.zeros())  # 2 J^T (W J v), seeded back-to-front pass
        for h in GROUPS:
            a, b = o[h]
            scale = float(y[a:b].abs().max())
            err = float((y2[a:b] - y[a:b]).abs().max())
            print(f", {h} {err / max(scale, 1e-30):.1e}", end="")
            assert err <= TOL * max(scale, 1e-30), f"v in {g}: group {h} differs by {err:.3e} (max {scale:.3e})"
        print()
        assert float(y[o["xyz"][0]:o["xyz"][1]].abs().max()) == 0.0
    # symmetry over a direction in every LM group at once
    u = sum(_group_direction(prob.layout, g, seed=20 + k) for k, g in enumerate(GROUPS))
    v = sum(_group_direction(prob.layout, g, seed=30 + k) for k, g in enumerate(GROUPS))
    Au, Av = prob.matvec(u, prob.zeros()), prob.matvec(v, prob.zeros())
    uAu, vAv = _dot(u, Au), _dot(v, Av)
    assert uAu > 0 and vAv > 0
    print(f"{case} symmetry rel {abs(_dot(u, Av) - _dot(Au, v)) / (uAu * vAv) ** 0.5:.2e}")
    assert abs(_dot(u, Av) - _dot(Au, v)) <= TOL_SYM * (uAu * vAv) ** 0.5


def test_dropin_jvp_vjp_energy_whole_frame_1M():
    """render() under forward-mode AD (J u) and autograd's backward (J^T g) through the drop-in rasterizer, per raw
    leaf: <u, J^T (J u)> = ||J u||^2 over the whole 1080p frame at 1M Gaussians."""
    from gslm.train import PipelineParams, render
    W, H = 1920, 1080
    model = synthetic_gaussians(1_000_000, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(DEV)
    cam = orbit_cameras(1, W, H, seed=1)[0].to(DEV)
    bg = torch.zeros(3, device=DEV)
    pipe = PipelineParams()
    names = ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure")
    leaves = dict(zip(names, model.params()))
    for k, name in enumerate(names[:-1]):  # exposure does not enter render() (use_trained_exp=False)
        gen = torch.Generator().manual_seed(40 + k)
        u = types.SimpleNamespace(**{f"{n}_grad": (torch.randn(t.shape, generator=gen).to(DEV) if n == name
                                                   else torch.zeros_like(t)) for n, t in leaves.items()})
        with torch.no_grad(), fwAD.dual_level(), model.make_dual(u):
            ju = fwAD.unpack_dual(render(cam, model, pipe, bg)["render"]).tangent
        model.zero_grad()
        render(cam, model, pipe, bg)["render"].backward(ju)
        lhs = _dot(getattr(u, f"{name}_grad"), getattr(model, f"_{name}").grad)
        rhs = _dot(ju, ju)
        assert rhs > 0
        print(f"drop-in {name}: energy rel {abs(lhs - rhs) / rhs:.2e}")
        assert abs(lhs - rhs) <= TOL_ENERGY * rhs, f"{name}: <u, J^T J u> {lhs:.9e} vs ||J u||^2 {rhs:.9e}"
