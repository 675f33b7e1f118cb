"""The quadrant cull is an exact-results optimisation: with it (default) and without it
(gslm_view.debug = 1, the reference's exhaustive traversal) every output must be BITWISE identical --
forward image / inverse depth, VJP gradients, JVP tangents and the fused LM matvec.

The scene is built to stress the cull's conservative bound (gslm_kernels.hpp, quad_mask4):
needle-like splats (condition numbers ~1e7), splats larger than the image, opacities straddling
the 1/255 threshold, and the antialiasing opacity rescale."""
import math

import pytest
import torch
import torch.autograd.forward_ad as fwAD

from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from scenes import activated

pytestmark = pytest.mark.gpu
DEV = "cuda"
W, H = 112, 72


def _adversarial_model(P=4000, sh=2):
    m = synthetic_gaussians(P, sh, seed=7, s0=0.02, n_cams=2)
    g = torch.Generator().manual_seed(11)
    q = P // 5
    with torch.no_grad():
        # needles: one long axis, two ~1e-4 axes, random orientation
        m._scaling[:q] = torch.log(torch.tensor([0.4, 1e-4, 1e-4])) + 0.1 * torch.randn(q, 3, generator=g)
        # splats wider than the frame
        m._scaling[q:2 * q] = math.log(0.8) + 0.2 * torch.randn(q, 3, generator=g)
        # opacity around the 1/255 blend threshold
        op = (1.0 / 255.0) * (0.6 + 0.8 * torch.rand(q, 1, generator=g))
        m._opacity[2 * q:3 * q] = torch.log(op / (1 - op))
        # flat, strongly anisotropic discs
        m._scaling[3 * q:4 * q] = torch.log(torch.tensor([0.08, 0.01, 0.0005])) + 0.1 * torch.randn(q, 3, generator=g)
    return m


def _settings(cam, D, debug, antialiasing, bg):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    return GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        bg=bg.to(DEV), scale_modifier=1.0, viewmatrix=cam.world_view_transform.to(DEV),
        projmatrix=cam.full_proj_transform.to(DEV), sh_degree=D, campos=cam.camera_center.to(DEV),
        prefiltered=False, debug=debug, antialiasing=antialiasing)


@pytest.mark.parametrize("antialiasing", [False, True])
def test_cull_forward_backward_jvp_bitwise(antialiasing):
    from diff_gaussian_rasterization import GaussianRasterizer
    m = _adversarial_model()
    D = m.active_sh_degree
    cam = orbit_cameras(1, W, H, seed=3)[0]
    bg = torch.tensor([0.1, 0.4, 0.8])
    a0 = {k: v.to(DEV) for k, v in activated(m).items()}
    gen = torch.Generator().manual_seed(5)
    dcol = torch.randn(3, H, W, generator=gen).to(DEV)
    ddep = torch.randn(1, H, W, generator=gen).to(DEV)
    tang = {k: torch.randn(v.shape, generator=gen).to(DEV) for k, v in a0.items()}

    def run(debug):
        rast = GaussianRasterizer(_settings(cam, D, debug, antialiasing, bg))
        a = {k: v.clone().requires_grad_(True) for k, v in a0.items()}
        m2 = torch.zeros_like(a["means3D"], requires_grad=True)
        c, radii, d = rast(means3D=a["means3D"], means2D=m2, shs=a["shs"], opacities=a["opacities"],
                           scales=a["scales"], rotations=a["rotations"])
        ((c * dcol).sum() + (d * ddep).sum()).backward()
        out = {"color": c.detach(), "invdepth": d.detach(), "radii": radii} | \
              {f"grad_{k}": v.grad for k, v in a.items()} | {"grad_means2D": m2.grad}
        with torch.no_grad(), fwAD.dual_level():
            ad = {k: fwAD.make_dual(v, tang[k]) for k, v in a0.items()}
            c, _, d = rast(means3D=ad["means3D"], means2D=torch.zeros_like(a0["means3D"]), shs=ad["shs"],
                           opacities=ad["opacities"], scales=ad["scales"], rotations=ad["rotations"])
            out["jvp_color"] = fwAD.unpack_dual(c).tangent.clone()
            out["jvp_invdepth"] = fwAD.unpack_dual(d).tangent.clone()
        return out

    culled, exhaustive = run(False), run(True)
    assert (culled["radii"] > 0).sum() > 1000
    for k in exhaustive:
        assert torch.equal(culled[k], exhaustive[k]), f"{k} differs between culled and exhaustive traversal"


def test_cull_lm_matvec_bitwise():
    from gslm.lm import LMProblem
    m = _adversarial_model().to(DEV)
    cams = orbit_cameras(2, W, H, seed=3, images=[torch.rand(3, H, W, generator=torch.Generator().manual_seed(i))
                                                   for i in range(2)])
    for c in cams:
        c.to(DEV)
    v = None
    ys = []
    for debug in (0, 1):
        prob = LMProblem(m, cams, torch.zeros(3))
        for vr in prob.views:
            vr.view.debug = debug
        prob.evaluate()
        g = prob.rhs(prob.zeros())
        if v is None:
            v = torch.randn(g.numel(), generator=torch.Generator().manual_seed(9)).to(DEV)
            for grp in ("xyz", "exposure"):
                lo, hi = prob.layout.offsets[grp]
                v[lo:hi] = 0
        ys.append((g.clone(), prob.matvec(v, prob.zeros()).clone()))
    assert torch.equal(ys[0][0], ys[1][0]), "J^T r differs between culled and exhaustive traversal"
    assert torch.equal(ys[0][1], ys[1][1]), "(J^T J + D) v differs between culled and exhaustive traversal"
