"""GPU: how far the float32 CG iterates drift at the bench size (BASELINE configs[2]: 1M Gaussians SH 3, one 1080p
view, 10 CGLS iterations), in both layouts of the CG vectors.

The reference's solver runs cgls_damped in float32 tensors with float64 scalars (conjugate_gradient.py:51-127).  The
headline and every single-view LM step carry the SH-rest group projected (3 coordinates along the view's SH-rest
direction): an exact Krylov-subspace restriction in exact arithmetic, but its float32 rounding differs
from the full layout's.  The yardstick here is the same recursion in float64 (vectors, dots, updates) on the same
device operator (each product the float32 fused kernels applied to the float64 direction rounded to float32): what
is left is the float32 recursion's own rounding.  Both float32 layouts must stay within DRIFT_TOL of it after 10
iterations, and the projected one no worse than the full one (by more than a hair).  DESIGN.md §5 states the bound.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DRIFT_TOL = 2e-3  # relative, after 10 iterations (measured values in DESIGN.md §5)


def _bench_scene(P=1_000_000, W=1920, H=1080):
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem
    from gslm.model import synthetic_gaussians
    bg = torch.zeros(3)
    pert = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu")
    g2 = torch.Generator().manual_seed(2)
    with torch.no_grad():
        pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
        pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
        pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
    pert.to("cuda")
    cams = [c.to("cuda") for c in orbit_cameras(1, W, H, seed=1)]
    gp = LMProblem(pert, cams, bg)
    gp.evaluate()
    cams[0].original_image = gp.views[0].color.clamp(0, 1).clone()
    del gp, pert
    model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu").to("cuda")
    return model, cams, bg


def _cg64(prob, g32, iters):
    """CG on the normal equations (cgls_fused's recursion, x0 = 0, no restart within `iters`) with float64 vectors and
    dots; each product is prob.matvec on the direction rounded to float32."""
    x = torch.zeros(g32.numel(), dtype=torch.float64, device=g32.device)
    s = g32.double().clone()
    p = s.clone()
    gam = float((s * s).sum())
    q32 = torch.zeros_like(g32)
    for _ in range(iters):
        prob.matvec(p.float().contiguous(), q32)
        q = q32.double()
        alpha = gam / float((p * q).sum())
        x += alpha * p
        s -= alpha * q
        gam_new = float((s * s).sum())
        p = s + (gam_new / gam) * p
        gam = gam_new
    return x


def test_projected_and_full_layout_drift_at_bench_size():
    from gslm.lm import LMProblem, cgls_fused
    model, cams, bg = _bench_scene()
    out = {}
    for name, proj in (("full", False), ("projected", True)):
        prob = LMProblem(model, cams, bg, sh_projection=proj)
        prob.evaluate()
        g = prob.rhs(prob.zeros())
        x32, _ = cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=False)
        x64 = _cg64(prob, g, 10)
        expand = getattr(prob, "expand", None) if proj else None
        # compare in the reference layout (the projected step expanded; its float64 yardstick expanded the same way)
        a = expand(x32).double() if expand else x32.double()
        b = expand(x64.float()).double() if expand else x64
        out[name] = float((a - b).norm() / b.norm())
        out[name + "_x64"] = b
        del prob
        torch.cuda.empty_cache()
    # the two float64 yardsticks are the same step (the Krylov restriction), up to the float32 operator's rounding
    ref_gap = float((out["full_x64"] - out["projected_x64"]).norm() / out["full_x64"].norm())
    print(f"10-iteration drift at 1M / 1080p against float64 CG on the same operator: full {out['full']:.3e}, "
          f"projected {out['projected']:.3e}; float64 yardsticks apart {ref_gap:.3e}")
    assert out["full"] <= DRIFT_TOL and out["projected"] <= DRIFT_TOL, out
    assert out["projected"] <= 1.5 * out["full"] + 1e-5, (out["projected"], out["full"])
