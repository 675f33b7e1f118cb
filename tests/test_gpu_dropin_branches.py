"""GPU parity of the drop-in rasterizer's optional branches against the CPU oracle.

The reference's render() / batch_render() reach these through PipelineParams and the camera settings
(gaussian_renderer/__init__.py:36-110, batch_render.py:33-108, arguments/__init__.py:63-70):
  * antialiasing=True            (pipe.antialiasing: opacity rescaled by h = sqrt(det0 / det))
  * scale_modifier != 1          (render(..., scaling_modifier))
  * cov3D_precomp                (pipe.compute_cov3D_python: pc.get_covariance(scaling_modifier))
  * colors_precomp               (pipe.convert_SHs_python / override_color)
  * dc= split                    (separate_sh=True, the SparseGaussianAdam configuration; dc [P,1,3] and the
                                  SH rest [P,K-1,3] passed separately) -- forward, VJP and forward-mode JVP
Each case runs the forward (image 1e-4 L-inf, radii exact), the VJP (every input's gradient within 1e-4 of
its max) and the JVP (colour / inverse-depth tangents within 1e-4 of their max) on the GPU and on the
oracle (oracle/torch_raster.py, autograd / forward-AD) with the same inputs and tangents.
"""
import pytest
import torch
import torch.autograd.forward_ad as fwAD

from oracle import torch_raster as tr
from scenes import activated, gpu_settings, make_scene, oracle_settings

pytestmark = pytest.mark.gpu
DEV = "cuda"

# case -> (antialiasing, scale_modifier, cov3D_precomp, colors_precomp, dc split)
CASES = {
    "antialiasing": (True, 1.0, False, False, False),
    "scale_modifier_0.8": (False, 0.8, False, False, False),
    "cov3D_precomp": (False, 1.0, True, False, False),
    "colors_precomp": (False, 1.0, False, True, False),
    "cov3D_and_colors_precomp": (False, 1.0, True, True, False),
    "dc_split": (False, 1.0, False, False, True),
    "dc_split_aa_scale0.7": (True, 0.7, False, False, True),
    "cov3D_precomp_aa": (True, 1.0, True, False, False),
}


def _inputs(model, case):
    aa, smod, use_cov, use_col, split = CASES[case]
    a = activated(model)
    out = {"means3D": a["means3D"], "opacities": a["opacities"]}
    if use_cov:
        # pc.get_covariance(scaling_modifier) (gaussian_model.py:36-40): the modifier is baked into the cov
        with torch.no_grad():
            out["cov3D_precomp"] = tr.compute_cov3d(a["scales"], smod, a["rotations"]).contiguous()
    else:
        out["scales"], out["rotations"] = a["scales"], a["rotations"]
    if use_col:
        g = torch.Generator().manual_seed(21)
        out["colors_precomp"] = torch.rand(a["means3D"].shape[0], 3, generator=g)
    elif split:
        out["dc"] = a["shs"][:, :1].contiguous()
        out["shs"] = a["shs"][:, 1:].contiguous()
    else:
        out["shs"] = a["shs"]
    return out


def _oracle_call(inp, m2, st):
    shs = inp.get("shs")
    if "dc" in inp:
        shs = torch.cat([inp["dc"], inp["shs"]], dim=1)
    return tr.rasterize(inp["means3D"], m2, inp["opacities"], st, shs=shs, colors_precomp=inp.get("colors_precomp"),
                        scales=inp.get("scales"), rotations=inp.get("rotations"),
                        cov3D_precomp=inp.get("cov3D_precomp"))


def _gpu_call(inp, m2, st):
    from diff_gaussian_rasterization import GaussianRasterizer
    return GaussianRasterizer(st)(means3D=inp["means3D"], means2D=m2, opacities=inp["opacities"], shs=inp.get("shs"),
                                  colors_precomp=inp.get("colors_precomp"), scales=inp.get("scales"),
                                  rotations=inp.get("rotations"), cov3D_precomp=inp.get("cov3D_precomp"),
                                  dc=inp.get("dc"))


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-8)).item()


def _settings(cam, D, case, bg):
    aa, smod, use_cov, _, _ = CASES[case]
    # with cov3D_precomp the modifier is already inside the covariance; the rasterizer ignores it then
    return (oracle_settings(cam, D, bg, scale_modifier=smod, antialiasing=aa),
            gpu_settings(cam, D, bg, scale_modifier=smod, antialiasing=aa))


@pytest.mark.parametrize("scene", ["dense_2k_sh3_64x48", "mid_8k_sh1_96x80"])
@pytest.mark.parametrize("case", list(CASES))
def test_branch_forward_backward(scene, case):
    model, cams = make_scene(scene)
    D = model.active_sh_degree
    cam = cams[0]
    bg = torch.tensor([0.25, 0.5, 0.75])
    ost, gst = _settings(cam, D, case, bg)
    inp0 = _inputs(model, case)
    H, W = cam.image_height, cam.image_width
    g = torch.Generator().manual_seed(4)
    dcol = torch.randn(3, H, W, generator=g)
    ddep = torch.randn(1, H, W, generator=g)

    def run(dev, fn, st):
        inp = {k: v.detach().clone().to(dev).requires_grad_(True) for k, v in inp0.items()}
        m2 = torch.zeros_like(inp["means3D"], requires_grad=True)
        c, r, d = fn(inp, m2, st)
        ((c * dcol.to(dev)).sum() + (d * ddep.to(dev)).sum()).backward()
        grads = {k: v.grad.detach().cpu() for k, v in inp.items()}
        grads["means2D"] = m2.grad.detach().cpu()
        return c.detach().cpu(), r.cpu(), d.detach().cpu(), grads

    oc, orr, od, og = run("cpu", _oracle_call, ost)
    gc, gr, gd, gg = run(DEV, _gpu_call, gst)
    assert torch.equal(gr, orr), "radii must match exactly"
    assert (gc - oc).abs().max() <= 1e-4, f"colour L-inf {(gc - oc).abs().max():.3e}"
    assert (gd - od).abs().max() <= 1e-4, f"invdepth L-inf {(gd - od).abs().max():.3e}"
    for k in og:
        assert _rel(gg[k], og[k]) < 1e-4, f"grad {k}: rel err {_rel(gg[k], og[k]):.3e}"


@pytest.mark.parametrize("scene", ["dense_2k_sh3_64x48", "mid_8k_sh1_96x80"])
@pytest.mark.parametrize("case", list(CASES))
def test_branch_jvp(scene, case):
    model, cams = make_scene(scene)
    D = model.active_sh_degree
    cam = cams[0]
    bg = torch.tensor([0.3, 0.1, 0.7])
    ost, gst = _settings(cam, D, case, bg)
    inp0 = _inputs(model, case)
    gen = torch.Generator().manual_seed(3)
    tang = {k: torch.randn(v.shape, generator=gen) for k, v in inp0.items()}
    t_m2 = torch.randn(inp0["means3D"].shape, generator=gen)

    def run(dev, fn, st):
        with torch.no_grad(), fwAD.dual_level():
            inp = {k: fwAD.make_dual(v.to(dev), tang[k].to(dev)) for k, v in inp0.items()}
            m2 = fwAD.make_dual(torch.zeros_like(inp0["means3D"]).to(dev), t_m2.to(dev))
            c, _, d = fn(inp, m2, st)
            return fwAD.unpack_dual(c).tangent.cpu(), fwAD.unpack_dual(d).tangent.cpu()

    rc, rd = run("cpu", _oracle_call, ost)
    gc, gd = run(DEV, _gpu_call, gst)
    assert _rel(gc, rc) < 1e-4, f"colour tangent rel err {_rel(gc, rc):.3e}"
    assert _rel(gd, rd) < 1e-4, f"invdepth tangent rel err {_rel(gd, rd):.3e}"


def test_dc_split_jvp_with_partial_tangents():
    """separate_sh under forward-mode AD with a tangent on dc only (rest primal-only) and on the rest only:
    the missing tangent is zero (the jvp's NULL-tangent path), equal to the oracle with a zero tangent."""
    model, cams = make_scene("dense_2k_sh3_64x48")
    D = model.active_sh_degree
    cam = cams[0]
    bg = torch.zeros(3)
    ost, gst = _settings(cam, D, "dc_split", bg)
    inp0 = _inputs(model, "dc_split")
    gen = torch.Generator().manual_seed(9)
    for which in ("dc", "shs"):
        tang = {which: torch.randn(inp0[which].shape, generator=gen)}

        def run(dev, fn, st):
            with torch.no_grad(), fwAD.dual_level():
                inp = {k: (fwAD.make_dual(v.to(dev), tang[k].to(dev)) if k in tang else v.to(dev))
                       for k, v in inp0.items()}
                c, _, d = fn(inp, torch.zeros_like(inp0["means3D"]).to(dev), st)
                return fwAD.unpack_dual(c).tangent.cpu()

        rc = run("cpu", _oracle_call, ost)
        gc = run(DEV, _gpu_call, gst)
        assert _rel(gc, rc) < 1e-4, f"{which}: colour tangent rel err {_rel(gc, rc):.3e}"


def test_debug_mode_same_results_and_snapshot_on_failure(tmp_path, monkeypatch):
    """settings.debug (arguments/__init__.py:70, forwarded by render()): upstream's debug mode.  The library then
    synchronises after every kernel of the call (gslm_view.debug, a failing launch reported at its source line) and
    walks every list entry in every wave; the Python side copies the arguments to the host first and, on a failure,
    saves them to snapshot_fw.dump / snapshot_bw.dump and re-raises.  Results are bitwise those of the normal mode."""
    from diff_gaussian_rasterization import GaussianRasterizer
    model, cams = make_scene("dense_2k_sh3_64x48")
    cam = cams[0]
    D = model.max_sh_degree
    monkeypatch.chdir(tmp_path)
    outs = []
    for debug in (False, True):
        st = gpu_settings(cam, D)._replace(debug=debug)
        inp = {k: v.to(DEV).detach().requires_grad_(True) for k, v in _inputs(model, "scale_modifier_0.8").items()}
        m2 = torch.zeros_like(inp["means3D"], requires_grad=True)
        color, radii, invd = GaussianRasterizer(st)(means2D=m2, **inp)
        (color.square().sum() + invd.sum()).backward()
        outs.append([color.detach(), radii, invd.detach(), m2.grad] + [inp[k].grad for k in sorted(inp)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert not (tmp_path / "snapshot_fw.dump").exists()
    # an invalid call (SH degree out of range): raised by the call, arguments dumped as upstream does
    bad = gpu_settings(cam, D)._replace(debug=True, sh_degree=7)
    inp = {k: v.to(DEV) for k, v in _inputs(model, "scale_modifier_0.8").items()}
    with pytest.raises(RuntimeError):
        GaussianRasterizer(bad)(means2D=torch.zeros_like(inp["means3D"]), **inp)
    snap = torch.load(tmp_path / "snapshot_fw.dump", weights_only=True)
    assert torch.equal(snap[1], inp["means3D"].cpu())
