"""CPU: the oracle (and the host-side camera / model code) against the golden fixtures produced by the
reference's own Python (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest
import torch

from gslm.cameras import orbit_cameras
from gslm.model import GaussianModel, build_rotation
from oracle import torch_raster as tr

HERE = os.path.dirname(os.path.abspath(__file__))


def _g(name):
    return np.load(os.path.join(HERE, "golden", name))


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_eval_sh_matches_reference(deg):
    d = _g("sh_golden.npz")
    sh = torch.from_numpy(d[f"sh{deg}"]).transpose(1, 2)  # reference layout [..., C, K] -> [P, K, C]
    dirs = torch.from_numpy(d[f"dirs{deg}"])
    got = tr.eval_sh(deg, sh, dirs)
    assert np.allclose(got.numpy(), d[f"rgb{deg}"], rtol=0, atol=1e-12)


def test_rgb2sh_matches_reference():
    from gslm.model import RGB2SH
    d = _g("sh_golden.npz")
    assert np.allclose(RGB2SH(torch.from_numpy(d["rgb2sh_in"])).numpy(), d["rgb2sh_out"], atol=1e-15)


def test_covariance_matches_reference():
    d = _g("cov_golden.npz")
    s, q = torch.from_numpy(d["scales"]), torch.from_numpy(d["rotations"])
    qn = q / q.norm(dim=1, keepdim=True)  # build_rotation normalises; the kernel receives normalised q
    got = tr.compute_cov3d(s, 1.0, qn)
    assert np.allclose(got.numpy(), d["cov6"], rtol=1e-5, atol=1e-9)
    assert np.allclose(build_rotation(q).numpy(), d["R"], atol=1e-6)
    m = GaussianModel(0)
    m.set_params(torch.zeros(64, 3), torch.zeros(64, 1, 3), torch.zeros(64, 0, 3), torch.log(s), q, torch.zeros(64, 1))
    assert np.allclose(m.get_covariance().detach().numpy(), d["cov6"], rtol=1e-5, atol=1e-9)


def test_camera_matrices_match_reference():
    d = _g("camera_golden.npz")
    cams = orbit_cameras(4, 64, 48, seed=1)
    for i, c in enumerate(cams):
        assert np.allclose(c.R, d[f"R{i}"]) and np.allclose(c.T, d[f"T{i}"])
        assert np.allclose(c.world_view_transform.numpy(), d[f"world_view{i}"], atol=1e-6)
        assert np.allclose(c.full_proj_transform.numpy(), d[f"full_proj{i}"], atol=1e-6)
        assert np.allclose(c.camera_center.numpy(), d[f"center{i}"], atol=1e-5)


def test_raster_fixture_regression():
    """The restatement itself is stable: config-1 forward equals its committed fixture."""
    from scenes import activated, make_scene, oracle_settings
    d = _g("raster_cfg1.npz")
    model, cams = make_scene("cfg1_2k_sh0_256")
    a = activated(model)
    with torch.no_grad():
        c, r, dep, I = tr.rasterize(a["means3D"], torch.zeros_like(a["means3D"]), a["opacities"],
                                    oracle_settings(cams[0], 0), shs=a["shs"], scales=a["scales"],
                                    rotations=a["rotations"], return_internals=True)
    assert np.array_equal(r.numpy(), d["radii"])
    assert np.array_equal(I["point_list"].numpy().astype(np.int32), d["point_list"])
    assert np.array_equal(I["n_contrib"].numpy(), d["n_contrib"])
    assert np.abs(c.numpy() - d["color"]).max() <= 1e-6
    assert np.abs(dep.numpy() - d["invdepth"]).max() <= 1e-6


def _solver_scene():
    d = _g("solver_golden.npz")
    P, D, W, H, s0, nv = d["scene"]
    P, D, W, H, nv = int(P), int(D), int(W), int(H), int(nv)
    m = GaussianModel(D)
    t = lambda k: torch.from_numpy(d[f"in_{k}"])
    m.set_params(t("xyz"), t("features_dc"), t("features_rest"), t("scaling"), t("rotation"), t("opacity"),
                 t("exposure"))
    m.active_sh_degree = D
    cams = orbit_cameras(nv, W, H, seed=1, images=[torch.from_numpy(d[f"gt{i}"]) for i in range(nv)])
    return d, m, cams


def _close(a, b, tol):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() <= tol * max(np.abs(b).max(), 1e-12)


def test_oracle_lm_algebra_matches_reference_solver():
    """Loss, J^T b and (J^T J + D) v restated on the oracle equal the reference solver's outputs."""
    from oracle.lm_ref import OracleLMProblem
    d, m, cams = _solver_scene()
    op = OracleLMProblem(m, cams, torch.zeros(3))
    assert abs(float(op.evaluate()) - float(d["loss"])) <= 1e-6 * float(d["loss"])
    assert _close(op.rhs().numpy(), d["Jtb"], 1e-5)
    y = op.matvec(torch.from_numpy(d["v"]), op.zeros())
    assert _close(y.numpy(), d["Av"], 1e-5)


@pytest.mark.parametrize("sched,key", [((2, 1), "x_ref_schedule"), ((10, 10), "x_ten")])
def test_oracle_cgls_matches_reference_schedule(sched, key):
    """CG on A = J^T J + D with the reference's restart schedule reproduces cgls_damped's iterates."""
    from oracle.lm_ref import OracleLMProblem, cgls_ref
    d, m, cams = _solver_scene()
    op = OracleLMProblem(m, cams, torch.zeros(3))
    op.evaluate()
    x = cgls_ref(op, op.rhs(), sched[0], sched[1])
    err = np.linalg.norm(x.numpy().astype(np.float64) - d[key]) / np.linalg.norm(d[key])
    assert err < 1e-3, err


def test_ssim_oracle_matches_reference():
    """oracle/ssim_ref.py's SSIM map equals the reference's utils/loss_utils.py ssim_per_pixel on random
    pairs and on the solver scene's renders (ssim_golden.npz)."""
    from oracle import ssim_ref
    d = _g("ssim_golden.npz")
    for a, b, ref in (("rand_a", "rand_b", "rand_ssim"), ("scene_x", "scene_gt", "scene_ssim")):
        got = ssim_ref.ssim_per_pixel(torch.from_numpy(d[a]), torch.from_numpy(d[b])).numpy()
        assert np.abs(got - d[ref]).max() <= 1e-6, ref
    assert np.array_equal(np.abs(d["rand_a"] - d["rand_b"]), d["rand_l1"])


def test_oracle_ssim_lm_algebra_matches_reference_solver():
    """The disable_ssim=False residual: loss, J^T b, (J^T J + D) v and 10 CGLS iterations of the
    oracle equal the reference solver's (solver_ssim_golden.npz)."""
    from oracle.lm_ref import OracleLMProblem, cgls_ref
    _, m, cams = _solver_scene()
    d = _g("solver_ssim_golden.npz")
    for i, c in enumerate(cams):
        c.original_image = torch.from_numpy(d[f"gt{i}"])
    op = OracleLMProblem(m, cams, torch.zeros(3), ssim=True)
    # the reference's loss_scalar sums r^2 in float32 (loss_image_state.py:16-19), the oracle in float64
    assert abs(float(op.evaluate()) - float(d["loss"])) <= 1e-5 * float(d["loss"])
    g = op.rhs()
    assert _close(g.numpy(), d["Jtb"], 1e-5)
    y = op.matvec(torch.from_numpy(d["v"]), op.zeros())
    assert _close(y.numpy(), d["Av"], 1e-5)
    x = cgls_ref(op, g, 10, 10)
    err = np.linalg.norm(x.numpy().astype(np.float64) - d["x_ten"]) / np.linalg.norm(d["x_ten"])
    assert err < 1e-3, err


@pytest.mark.parametrize("tag", ["ref", "ten"])
def test_oracle_line_search_matches_lm_step_golden(tag):
    """oracle/lm_ref.py:line_search_ref (train_jvp.py:262-279) with the oracle's flat-vector update on the golden's
    CG step reproduces the golden's (alpha, val loss) trace, best_alpha, final loss and stepped parameters."""
    from gslm.lm import update_params
    from gslm.params import ParamLayout
    from oracle.lm_ref import OracleLMProblem, line_search_ref
    d, L = _g("solver_golden.npz"), _g("lm_step_golden.npz")
    P, D, W, H, s0, nv = (int(x) if i != 4 else x for i, x in enumerate(d["scene"]))
    names = ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure")
    m = GaussianModel(D)
    m.set_params(*(torch.from_numpy(d[f"in_{k}"]) for k in names))
    m.active_sh_degree = D
    nval = sum(1 for k in L.files if k.startswith("val_gt"))
    val = orbit_cameras(nval, W, H, seed=4, images=[torch.from_numpy(L[f"val_gt{i}"]) for i in range(nval)])
    layout = ParamLayout(P, (D + 1) ** 2, m._exposure.shape[0])
    s = torch.from_numpy(L[f"{tag}_s"])
    op = OracleLMProblem(m, val, torch.zeros(3))
    best, final, trace = line_search_ref(lambda a: update_params(m, layout, s, a), lambda: float(op.evaluate()))
    assert best == float(L[f"{tag}_best_alpha"])
    assert [a for a, _ in trace] == list(L[f"{tag}_trace_alpha"])
    assert np.allclose([v for _, v in trace], L[f"{tag}_trace_loss"], rtol=1e-6, atol=0)
    assert abs(final - float(L[f"{tag}_final_val_loss"])) <= 1e-6 * float(L[f"{tag}_final_val_loss"])
    for k, t in zip(names, m.params()):
        assert np.allclose(t.detach().numpy(), L[f"{tag}_out_{k}"], rtol=0, atol=1e-6), k
