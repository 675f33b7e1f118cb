"""Generate the committed golden fixtures from the reference's own Python (run in the build container).

    python tests/golden/make_golden.py          # needs /root/reference (read-only)

What is pinned by the *reference's code* (imported from /root/reference, never copied):
  * sh_golden.npz      utils/sh_utils.py eval_sh / RGB2SH on random coefficients and directions
  * cov_golden.npz     utils/general_utils.py build_scaling_rotation / strip_symmetric (the covariance
                       the rasterizer's computeCov3D must reproduce; the reference hard-codes
                       device="cuda" at :66,:84,:103, so the allocation calls are redirected to CPU
                       for this script only -- the arithmetic is the reference's)
  * camera_golden.npz  utils/graphics_utils.py getWorld2View2 / getProjectionMatrix for the seeded
                       orbit cameras
  * solver_golden.npz  solver/conjugate_gradient.py cgls_damped + solver/solver_functions.py
                       LinearSolverFunctions + solver/gaussian_model_state.py + loss_image_state.py,
                       run around the CPU oracle renderer (oracle/torch_raster.py) exactly as
                       train_jvp.py:221-258 drives them (disable_ssim residual, xyz mask, damping):
                       loss, J^T b, (J^T J + D) v, and the CGLS solutions for the reference schedule
                       (max_iter=2, restart_iter=1) and for max_iter=restart_iter=10.
  * ssim_golden.npz    utils/loss_utils.py ssim_per_pixel / l1_loss_per_pixel on random image pairs
                       and on the solver scene's renders (the SSIM residual)
  * solver_ssim_golden.npz  the same solver run with the disable_ssim=False residual
                       (solver/batch_training_loss.py:18-30, restated around the reference's own
                       l1_loss_per_pixel / ssim_per_pixel): loss, J^T b, (J^T J + D) v, 10-iteration CGLS
  * lm_step_golden.npz one LM step of train_jvp.py:237-279: the reference's cgls_damped (schedule 2 x 1) on the
                       solver scene, then the restated backtracking line search (oracle/lm_ref.py) on three
                       validation views stepping the model by the reference's GaussianModelState arithmetic:
                       best_alpha, the (alpha, val loss) trace, the final val loss and the stepped parameters
  * train_golden.npz   the first-order step: utils/general_utils.py get_expon_lr_func
                       at the schedules GaussianModel.training_setup builds (scene/gaussian_model.py:293-301,
                       OptimizationParams defaults of arguments/__init__.py:76-90), and the trajectory of
                       torch.optim.Adam -- the optimizer the reference steps (gaussian_model.py:283,
                       train.py:184-186) -- over the six parameter groups with their default lrs
The rasterizer itself has no reference binary here (absent submodule): its numerics are pinned by
the oracle restatement, finite differences and the adjoint identity (tests/test_oracle.py).
"""
import contextlib
import math
import os
import sys
from functools import partial

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-lm_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(1, os.path.join(ROOT, "tests"))

from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from oracle import torch_raster as tr  # noqa: E402

SOLVER_SCENE = dict(P=400, D=1, W=32, H=32, s0=0.06, views=2)


@contextlib.contextmanager
def reference_on_path():
    sys.path.insert(0, REF)
    try:
        yield
    finally:
        sys.path.remove(REF)


def sh_golden():
    with reference_on_path():
        from utils.sh_utils import RGB2SH, eval_sh
    g = torch.Generator().manual_seed(11)
    out = {}
    for deg in range(4):
        K = (deg + 1) ** 2
        sh = torch.randn(64, 3, K, generator=g, dtype=torch.float64)
        d = torch.randn(64, 3, generator=g, dtype=torch.float64)
        d = d / d.norm(dim=1, keepdim=True)
        out[f"sh{deg}"] = sh.numpy()
        out[f"dirs{deg}"] = d.numpy()
        out[f"rgb{deg}"] = eval_sh(deg, sh, d).numpy()
    rgb = torch.rand(16, 3, generator=g, dtype=torch.float64)
    out["rgb2sh_in"], out["rgb2sh_out"] = rgb.numpy(), RGB2SH(rgb).numpy()
    np.savez(os.path.join(HERE, "sh_golden.npz"), **out)


def cov_golden():
    with reference_on_path():
        import utils.general_utils as gu
    zeros = torch.zeros

    def cpu_zeros(*a, **k):
        k.pop("device", None)
        return zeros(*a, **k)

    g = torch.Generator().manual_seed(12)
    s = torch.exp(torch.randn(64, 3, generator=g)) * 0.1
    q = torch.randn(64, 4, generator=g)
    old = torch.zeros
    torch.zeros = cpu_zeros  # redirect the reference's device="cuda" allocations to CPU for this script
    try:
        L = gu.build_scaling_rotation(s, q)
        cov = gu.strip_symmetric(L @ L.transpose(1, 2))
        R = gu.build_rotation(q)
    finally:
        torch.zeros = old
    np.savez(os.path.join(HERE, "cov_golden.npz"), scales=s.numpy(), rotations=q.numpy(), cov6=cov.numpy(),
             R=R.numpy())


def camera_golden():
    with reference_on_path():
        from utils.graphics_utils import getProjectionMatrix, getWorld2View2
    cams = orbit_cameras(4, 64, 48, seed=1)
    out = {}
    for i, c in enumerate(cams):
        wv = torch.tensor(getWorld2View2(c.R, c.T, c.trans, c.scale)).transpose(0, 1)
        pr = getProjectionMatrix(znear=c.znear, zfar=c.zfar, fovX=c.FoVx, fovY=c.FoVy).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pr.unsqueeze(0)).squeeze(0)
        out[f"R{i}"], out[f"T{i}"] = c.R, c.T
        out[f"fov{i}"] = np.array([c.FoVx, c.FoVy])
        out[f"world_view{i}"], out[f"full_proj{i}"] = wv.numpy(), full.numpy()
        out[f"center{i}"] = wv.inverse()[3, :3].numpy()
    np.savez(os.path.join(HERE, "camera_golden.npz"), **out)


def solver_scene():
    sc = SOLVER_SCENE
    model = synthetic_gaussians(sc["P"], sc["D"], seed=0, s0=sc["s0"], n_cams=sc["views"])
    cams = orbit_cameras(sc["views"], sc["W"], sc["H"], seed=1)
    # GT (seed 2): render of the model with f_dc / opacity / scaling perturbed by N(0, 0.01^2)
    g = torch.Generator().manual_seed(2)
    pert = synthetic_gaussians(sc["P"], sc["D"], seed=0, s0=sc["s0"], n_cams=sc["views"])
    with torch.no_grad():
        pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g)
        pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g)
        pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g)
        for c in cams:
            img, _, _, _ = tr.render_model(pert, c, torch.zeros(3))
            c.original_image = img.detach().clone()
    return model, cams


def oracle_batch_loss(gaussians, viewpoint_cams, batch_stats=None, BatchLossImageState=None):
    """batch_training_loss(disable_ssim=True) (solver/batch_training_loss.py:33-105) on the oracle renderer."""
    bg = torch.zeros(3)
    imgs = []
    for vc in viewpoint_cams:
        img, _, _, _ = tr.render_model(gaussians, vc, bg)
        imgs.append(img)
    images = torch.stack(imgs)
    gt = torch.stack([vc.original_image for vc in viewpoint_cams])
    masks = torch.stack([vc.alpha_mask for vc in viewpoint_cams])
    r = images * masks - gt
    depth = torch.zeros((0,), dtype=r.dtype, requires_grad=True)
    sizes = [(vc.image_height, vc.image_width) for vc in viewpoint_cams]
    return BatchLossImageState(r, r, depth, sizes, False)


def oracle_batch_loss_ssim(gaussians, viewpoint_cams, batch_stats=None, BatchLossImageState=None, ref=None,
                           lambda_dssim=0.2):
    """batch_training_loss(disable_ssim=False, FUSED_SSIM_AVAILABLE=False) (solver/batch_training_loss.py:
    10-30, 56-81) on the oracle renderer, with the reference's l1_loss_per_pixel / ssim_per_pixel."""
    l1_loss_per_pixel, ssim_per_pixel = ref
    bg = torch.zeros(3)
    images = torch.stack([tr.render_model(gaussians, vc, bg)[0] for vc in viewpoint_cams])
    gt = torch.stack([vc.original_image for vc in viewpoint_cams])
    masks = torch.stack([vc.alpha_mask for vc in viewpoint_cams])
    images = images * masks
    alphas, betas = [], []
    for vc in viewpoint_cams:
        n = 3 * int(vc.image_height) * int(vc.image_width)
        alphas.append(math.sqrt((1.0 - lambda_dssim) / n))
        betas.append(math.sqrt(lambda_dssim / n))
    alphas = torch.tensor(alphas, dtype=images.dtype).view(-1, 1, 1, 1)
    betas = torch.tensor(betas, dtype=images.dtype).view(-1, 1, 1, 1)
    l1 = l1_loss_per_pixel(images, gt)
    ssim_loss = (1.0 - ssim_per_pixel(images, gt)).abs()
    r1 = alphas * torch.sqrt(l1 + 1e-6)
    r2 = betas * torch.sqrt(ssim_loss + 1e-6)
    depth = torch.zeros((0,), dtype=r1.dtype, requires_grad=True)
    sizes = [(vc.image_height, vc.image_width) for vc in viewpoint_cams]
    return BatchLossImageState(r1, r2, depth, sizes, False)


def ssim_golden():
    with reference_on_path():
        from utils.loss_utils import l1_loss_per_pixel, ssim_per_pixel
    g = torch.Generator().manual_seed(21)
    out = {}
    a = torch.rand(2, 3, 37, 53, generator=g)
    b = (a + 0.1 * torch.randn(2, 3, 37, 53, generator=g)).clamp(0, 1)
    out["rand_a"], out["rand_b"] = a.numpy(), b.numpy()
    out["rand_ssim"] = ssim_per_pixel(a, b).numpy()
    out["rand_l1"] = l1_loss_per_pixel(a, b).numpy()
    model, cams = solver_scene()
    imgs = torch.stack([tr.render_model(model, c, torch.zeros(3))[0].detach() for c in cams])
    gts = torch.stack([c.original_image for c in cams])
    out["scene_x"], out["scene_gt"] = imgs.numpy(), gts.numpy()
    out["scene_ssim"] = ssim_per_pixel(imgs, gts).numpy()
    np.savez_compressed(os.path.join(HERE, "ssim_golden.npz"), **out)


def solver_ssim_golden():
    with reference_on_path():
        from solver.conjugate_gradient import cgls_damped
        from solver.gaussian_model_state import (GaussianModelDampMatrix, GaussianModelParamGroupMask,
                                                 GaussianModelState)
        from solver.loss_image_state import BatchLossImageState
        from solver.solver_functions import LinearSolverFunctions
        from utils.loss_utils import l1_loss_per_pixel, ssim_per_pixel
    model, cams = solver_scene()
    # Ground truth = independent uniform images (seed 22), not the perturbed render: r1 = a sqrt(|x - gt| + 1e-6)
    # has d r1 / dx ~ 1 / sqrt(|x - gt|), so pixels where the render is within ~1e-6 of the ground truth
    # turn 1-ulp render differences into O(1) changes of J^T J; a perturbed-render ground truth has many
    # such pixels and makes the golden host-dependent (0.3% on (J^T J + D) v between two CPUs).
    g = torch.Generator().manual_seed(22)
    for c in cams:
        c.original_image = torch.rand(3, c.image_height, c.image_width, generator=g)
    loss_func = partial(oracle_batch_loss_ssim, BatchLossImageState=BatchLossImageState,
                        ref=(l1_loss_per_pixel, ssim_per_pixel))
    param_mask = GaussianModelParamGroupMask(mask_xyz=True)
    damp = GaussianModelDampMatrix(xyz_damp=5e2, features_dc_damp=5e-2, features_rest_damp=5e-2, scaling_damp=5e-2,
                                   rotation_damp=5e-2, opacity_damp=5e-2, exposure_damp=1e1)
    out = {}
    st = LinearSolverFunctions(loss_func, model, cams, batch_size=20, param_mask=param_mask)
    out["loss"] = np.array(float(st.evaluate_loss().loss_scalar))
    with torch.no_grad():
        b = -1 * st.loss
        out["Jtb"] = st.matvec_T(b).as_1d_tensor().detach().numpy()
        gen = torch.Generator().manual_seed(3)
        v = GaussianModelState.from_gaussians(model, param_mask=param_mask)
        vv = v.as_1d_tensor()
        vv.copy_(torch.randn(vv.shape, generator=gen))
        v.load_1d_tensor(vv)
        v = GaussianModelState(v.xyz_grad, v.features_dc_grad, v.features_rest_grad, v.scaling_grad, v.rotation_grad,
                               v.opacity_grad, v.exposure_grad.zero_(), param_mask=param_mask)
        Av = st.matvec_T(st.matvec(v)) + v * damp
        out["v"] = v.as_1d_tensor().detach().numpy()
        out["Av"] = Av.as_1d_tensor().detach().numpy()
        x0 = st.get_initial_solution()
        x = cgls_damped(matvec=st.matvec, matvec_T=st.matvec_T, dot=st.dot, saxpy=st.saxpy, b=b, x0=x0, damp=damp,
                        tol=1e-10, atol=0.0, max_iter=10, restart_iter=10, verbose=False)
        out["x_ten"] = x.as_1d_tensor().detach().numpy()
    for i, c in enumerate(cams):
        out[f"gt{i}"] = c.original_image.numpy()
    np.savez(os.path.join(HERE, "solver_ssim_golden.npz"), **out)


def solver_golden():
    with reference_on_path():
        from solver.conjugate_gradient import cgls_damped
        from solver.gaussian_model_state import (GaussianModelDampMatrix, GaussianModelParamGroupMask,
                                                 GaussianModelState)
        from solver.loss_image_state import BatchLossImageState
        from solver.solver_functions import LinearSolverFunctions
    model, cams = solver_scene()
    loss_func = partial(oracle_batch_loss, BatchLossImageState=BatchLossImageState)
    # train_jvp.py:221-235
    param_mask = GaussianModelParamGroupMask(mask_xyz=True)
    damp = GaussianModelDampMatrix(xyz_damp=5e2, features_dc_damp=5e-2, features_rest_damp=5e-2, scaling_damp=5e-2,
                                   rotation_damp=5e-2, opacity_damp=5e-2, exposure_damp=1e1)
    out = {}
    st = LinearSolverFunctions(loss_func, model, cams, batch_size=20, param_mask=param_mask)
    out["loss"] = np.array(float(st.evaluate_loss().loss_scalar))
    with torch.no_grad():
        b = -1 * st.loss
        # J^T b (matvec_T zeroes the xyz group through the param mask)
        out["Jtb"] = st.matvec_T(b).as_1d_tensor().detach().numpy()
        # (J^T J + D) v for a seeded tangent (seed 3: N(0,1) on every group but xyz and exposure)
        gen = torch.Generator().manual_seed(3)
        v = GaussianModelState.from_gaussians(model, param_mask=param_mask)
        vv = v.as_1d_tensor()
        vv.copy_(torch.randn(vv.shape, generator=gen))
        v.load_1d_tensor(vv)
        v = GaussianModelState(v.xyz_grad, v.features_dc_grad, v.features_rest_grad, v.scaling_grad, v.rotation_grad,
                               v.opacity_grad, v.exposure_grad.zero_(), param_mask=param_mask)
        Jv = st.matvec(v)
        JtJv = st.matvec_T(Jv)
        Av = JtJv + v * damp
        out["v"] = v.as_1d_tensor().detach().numpy()
        out["Av"] = Av.as_1d_tensor().detach().numpy()
        for name, (mi, ri) in {"ref_schedule": (2, 1), "ten": (10, 10)}.items():
            x0 = st.get_initial_solution()
            x = cgls_damped(matvec=st.matvec, matvec_T=st.matvec_T, dot=st.dot, saxpy=st.saxpy, b=b, x0=x0, damp=damp,
                            tol=1e-10, atol=0.0, max_iter=mi, restart_iter=ri, verbose=False)
            out[f"x_{name}"] = x.as_1d_tensor().detach().numpy()
    # inputs
    for k, t in zip(("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure"),
                    model.params()):
        out[f"in_{k}"] = t.detach().numpy()
    for i, c in enumerate(cams):
        out[f"gt{i}"] = c.original_image.numpy()
    out["scene"] = np.array([SOLVER_SCENE[k] for k in ("P", "D", "W", "H", "s0", "views")], dtype=np.float64)
    np.savez(os.path.join(HERE, "solver_golden.npz"), **out)


LM_VAL_VIEWS = 3  # validation cameras of the line-search golden (seed 4), GT from the same perturbed model


def lm_step_golden():
    """One LM step as train_jvp.py:237-279 runs it: the reference's LinearSolverFunctions + cgls_damped (reference
    schedule max_iter=2, restart_iter=1, and 10 x 10) on the solver scene, then the backtracking line search (restated in
    oracle/lm_ref.py:line_search_ref -- train_jvp.py is a script) on separate validation views, stepping the model
    with the reference's own GaussianModelState arithmetic (gaussians.update_step(alpha * s)).
    Pins best_alpha, every (alpha, val loss) pair, the final val loss and the stepped parameters."""
    from oracle.lm_ref import line_search_ref
    with reference_on_path():
        from solver.conjugate_gradient import cgls_damped
        from solver.gaussian_model_state import GaussianModelDampMatrix, GaussianModelParamGroupMask
        from solver.loss_image_state import BatchLossImageState
        from solver.solver_functions import LinearSolverFunctions
    model, cams = solver_scene()
    sc = SOLVER_SCENE
    val_cams = orbit_cameras(LM_VAL_VIEWS, sc["W"], sc["H"], seed=4)
    g = torch.Generator().manual_seed(2)
    pert = synthetic_gaussians(sc["P"], sc["D"], seed=0, s0=sc["s0"], n_cams=sc["views"])
    with torch.no_grad():
        pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g)
        pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g)
        pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g)
        for c in val_cams:
            c.original_image = tr.render_model(pert, c, torch.zeros(3))[0].detach().clone()
    loss_func = partial(oracle_batch_loss, BatchLossImageState=BatchLossImageState)
    param_mask = GaussianModelParamGroupMask(mask_xyz=True)
    damp = GaussianModelDampMatrix(xyz_damp=5e2, features_dc_damp=5e-2, features_rest_damp=5e-2, scaling_damp=5e-2,
                                   rotation_damp=5e-2, opacity_damp=5e-2, exposure_damp=1e1)
    out = {}
    base = [t.detach().clone() for t in model.params()]
    for tag, (mi, ri) in {"ref": (2, 1), "ten": (10, 10)}.items():
        model.set_params(*base)
        st = LinearSolverFunctions(loss_func, model, cams, batch_size=20, param_mask=param_mask)
        out[f"{tag}_start_loss"] = np.array(float(st.evaluate_loss().loss_scalar))
        with torch.no_grad():
            b = -1 * st.loss
            s = cgls_damped(matvec=st.matvec, matvec_T=st.matvec_T, dot=st.dot, saxpy=st.saxpy, b=b,
                            x0=st.get_initial_solution(), damp=damp, tol=1e-10, atol=0.0, max_iter=mi,
                            restart_iter=ri, verbose=False)
            del st
            out[f"{tag}_s"] = s.as_1d_tensor().detach().numpy()
            val_loss_func = partial(loss_func, gaussians=model, viewpoint_cams=val_cams)
            best_alpha, final, trace = line_search_ref(lambda a: model.update_step(a * s),
                                                       lambda: val_loss_func().loss_scalar)
        out[f"{tag}_best_alpha"] = np.array(best_alpha)
        out[f"{tag}_final_val_loss"] = np.array(final)
        out[f"{tag}_trace_alpha"] = np.array([a for a, _ in trace])
        out[f"{tag}_trace_loss"] = np.array([v for _, v in trace])
        for k, t in zip(("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure"),
                        model.params()):
            out[f"{tag}_out_{k}"] = t.detach().numpy()
    for i, c in enumerate(val_cams):
        out[f"val_gt{i}"] = c.original_image.numpy()
    np.savez(os.path.join(HERE, "lm_step_golden.npz"), **out)


TRAIN_STEPS = [0, 1, 2, 10, 100, 500, 1000, 7000, 15000, 29999, 30000, 45000]
ADAM_P = 37  # odd: every group's float count is exercised with a ragged float4 tail


def train_golden():
    with reference_on_path():
        from utils.general_utils import get_expon_lr_func
    out = {"steps": np.array(TRAIN_STEPS)}
    # position schedule (spatial_lr_scale 2.5), exposure schedule (delay 0), and a delayed variant
    scheds = {"xyz": get_expon_lr_func(0.00016 * 2.5, 0.0000016 * 2.5, lr_delay_mult=0.01, max_steps=30_000),
              "exposure": get_expon_lr_func(0.01, 0.001, lr_delay_steps=0, lr_delay_mult=0.0, max_steps=30_000),
              "delayed": get_expon_lr_func(0.01, 0.001, lr_delay_steps=1000, lr_delay_mult=0.1, max_steps=30_000)}
    for k, f in scheds.items():
        out[f"lr_{k}"] = np.array([f(s) for s in TRAIN_STEPS], np.float64)
    # torch.optim.Adam over the training_setup groups (lr as gaussian_model.py:273-280 with the defaults)
    g = torch.Generator().manual_seed(31)
    P = ADAM_P
    shapes = {"xyz": (P, 3), "f_dc": (P, 1, 3), "f_rest": (P, 15, 3), "opacity": (P, 1), "scaling": (P, 3),
              "rotation": (P, 4)}
    lrs = {"xyz": 0.00016 * 2.5, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025, "scaling": 0.005,
           "rotation": 0.001}
    params = {k: torch.nn.Parameter(torch.randn(shp, generator=g)) for k, shp in shapes.items()}
    for k, t in params.items():
        out[f"adam_p0_{k}"] = t.detach().numpy().copy()
    opt = torch.optim.Adam([{"params": [params[k]], "lr": lrs[k], "name": k} for k in shapes], lr=0.0, eps=1e-15)
    n_steps = 4
    for it in range(n_steps):
        for k, t in params.items():
            gr = torch.randn(t.shape, generator=g) * (10.0 ** (it - 2))
            out[f"adam_g{it}_{k}"] = gr.numpy()
            t.grad = gr
        opt.step()
    for k, t in params.items():
        st = opt.state[t]
        out[f"adam_p_{k}"] = t.detach().numpy().copy()
        out[f"adam_m_{k}"] = st["exp_avg"].numpy().copy()
        out[f"adam_v_{k}"] = st["exp_avg_sq"].numpy().copy()
        out[f"adam_lr_{k}"] = np.array(lrs[k])
    out["adam_steps"] = np.array(n_steps)
    np.savez(os.path.join(HERE, "train_golden.npz"), **out)


def raster_fixture():
    """Oracle forward outputs of BASELINE config 1 (2k Gaussians, SH0, 256x256): a regression fixture
    of the restatement itself (not a reference-binary vector, see module docstring)."""
    from scenes import activated, make_scene, oracle_settings
    model, cams = make_scene("cfg1_2k_sh0_256")
    a = activated(model)
    with torch.no_grad():
        c, r, d, I = tr.rasterize(a["means3D"], torch.zeros_like(a["means3D"]), a["opacities"],
                                  oracle_settings(cams[0], 0), shs=a["shs"], scales=a["scales"],
                                  rotations=a["rotations"], return_internals=True)
    np.savez_compressed(os.path.join(HERE, "raster_cfg1.npz"), color=c.numpy(), radii=r.numpy(), invdepth=d.numpy(),
                        point_list=I["point_list"].numpy().astype(np.int32), n_contrib=I["n_contrib"].numpy())


if __name__ == "__main__":
    torch.set_num_threads(8)
    if len(sys.argv) > 1:  # e.g. `make_golden.py solver_ssim_golden`
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    sh_golden()
    cov_golden()
    camera_golden()
    solver_golden()
    ssim_golden()
    solver_ssim_golden()
    train_golden()
    raster_fixture()
    lm_step_golden()
    print("golden fixtures written to", HERE)
