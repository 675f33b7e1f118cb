"""GPU parity of the first-order training row: gslm_adam_step (FusedAdam /
SparseGaussianAdam), gslm_densify_stats, gslm_ssim_mean, and one full train.py iteration.

Tolerances: Adam and the densification statistics follow the oracle's float32 operation order (rel 1e-6;
the statistics bit-exact); SSIM value 1e-6 and its gradient 1e-5 of the gradient's max against the
oracle's autograd; a training step's leaf gradients 1e-4 of each group's max (the rasterizer VJP bar)."""
import copy

import numpy as np
import pytest
import torch

from oracle import train_ref as ref
from oracle import torch_raster as tr
from oracle.ssim_ref import ssim_per_pixel
from scenes import make_scene

pytestmark = pytest.mark.gpu
DEV = "cuda"
GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def _gold():
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_golden.npz"))


def test_fused_adam_matches_torch_adam_golden_and_oracle():
    from gslm.optim import FusedAdam
    G = _gold()
    params = {k: torch.nn.Parameter(torch.from_numpy(G[f"adam_p0_{k}"]).to(DEV)) for k in GROUPS}
    opt = FusedAdam([{"params": [params[k]], "lr": float(G[f"adam_lr_{k}"]), "name": k} for k in GROUPS], lr=0.0,
                    eps=1e-15)
    ora = {k: (G[f"adam_p0_{k}"].copy(), np.zeros_like(G[f"adam_p0_{k}"]), np.zeros_like(G[f"adam_p0_{k}"]))
           for k in GROUPS}
    for it in range(int(G["adam_steps"])):
        for k in GROUPS:
            params[k].grad = torch.from_numpy(G[f"adam_g{it}_{k}"]).to(DEV)
            p, m, v = ora[k]
            ora[k] = ref.adam_dense_ref(p, G[f"adam_g{it}_{k}"], m, v, float(G[f"adam_lr_{k}"]), it + 1, eps=1e-15)
        opt.step()
    torch.cuda.synchronize()
    for k in GROUPS:
        st = opt.state[params[k]]
        assert float(st["step"]) == float(G["adam_steps"])
        got = (params[k].detach().cpu().numpy(), st["exp_avg"].cpu().numpy(), st["exp_avg_sq"].cpu().numpy())
        for name, a, o, gold in zip(("p", "m", "v"), got, ora[k], (G[f"adam_p_{k}"], G[f"adam_m_{k}"], G[f"adam_v_{k}"])):
            np.testing.assert_allclose(a, o, rtol=1e-6, atol=1e-9, err_msg=f"{k}.{name} vs oracle")
            np.testing.assert_allclose(a, gold, rtol=1e-5, atol=1e-7, err_msg=f"{k}.{name} vs torch.optim.Adam golden")


def test_fused_adam_matches_torch_adam_on_gpu_large():
    """A 100k-Gaussian SH-3 model's groups, 3 steps, against torch.optim.Adam (foreach) on the same GPU."""
    from gslm.optim import FusedAdam
    g = torch.Generator(device=DEV).manual_seed(0)
    P = 100_003
    shapes = {"xyz": (P, 3), "f_dc": (P, 1, 3), "f_rest": (P, 15, 3), "opacity": (P, 1), "scaling": (P, 3),
              "rotation": (P, 4)}
    lrs = {"xyz": 4e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 0.025, "scaling": 5e-3, "rotation": 1e-3}
    a = {k: torch.nn.Parameter(torch.randn(s, device=DEV, generator=g)) for k, s in shapes.items()}
    b = {k: torch.nn.Parameter(t.detach().clone()) for k, t in a.items()}
    oa = FusedAdam([{"params": [a[k]], "lr": lrs[k], "name": k} for k in shapes], lr=0.0, eps=1e-15)
    ob = torch.optim.Adam([{"params": [b[k]], "lr": lrs[k], "name": k} for k in shapes], lr=0.0, eps=1e-15)
    for _ in range(3):
        for k in shapes:
            gr = torch.randn(shapes[k], device=DEV, generator=g)
            a[k].grad, b[k].grad = gr, gr.clone()
        oa.step()
        ob.step()
    for k in shapes:
        torch.testing.assert_close(a[k].detach(), b[k].detach(), rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(oa.state[a[k]]["exp_avg_sq"], ob.state[b[k]]["exp_avg_sq"], rtol=1e-5, atol=1e-9)
    # grad None groups are skipped, as torch does
    a["xyz"].grad = None
    before = a["xyz"].detach().clone()
    oa.step()
    assert torch.equal(before, a["xyz"].detach())


@pytest.mark.parametrize("P", [37, 10_000])
def test_sparse_adam_matches_oracle(P):
    from gslm.optim import SparseGaussianAdam
    g = torch.Generator().manual_seed(P)
    shapes = {"xyz": (P, 3), "f_dc": (P, 1, 3), "f_rest": (P, 15, 3), "opacity": (P, 1), "scaling": (P, 3),
              "rotation": (P, 4)}
    lrs = {"xyz": 4e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 0.025, "scaling": 5e-3, "rotation": 1e-3}
    host = {k: torch.randn(s, generator=g) for k, s in shapes.items()}
    params = {k: torch.nn.Parameter(t.to(DEV)) for k, t in host.items()}
    opt = SparseGaussianAdam([{"params": [params[k]], "lr": lrs[k], "name": k} for k in shapes], lr=0.0, eps=1e-15)
    ora = {k: (host[k].numpy().copy(), np.zeros(shapes[k], np.float32), np.zeros(shapes[k], np.float32)) for k in shapes}
    for it in range(3):
        vis = torch.rand(P, generator=g) < 0.6
        for k in shapes:
            gr = torch.randn(shapes[k], generator=g)
            params[k].grad = gr.to(DEV)
            p, m, v = ora[k]
            ora[k] = ref.sparse_adam_ref(p, gr.numpy(), m, v, vis.numpy(), lrs[k], eps=1e-15)
        opt.step(vis.to(DEV), P)
    torch.cuda.synchronize()
    for k in shapes:
        st = opt.state[params[k]]
        np.testing.assert_allclose(params[k].detach().cpu().numpy(), ora[k][0], rtol=1e-6, atol=1e-9, err_msg=k)
        np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), ora[k][1], rtol=1e-6, atol=1e-9, err_msg=k)
        np.testing.assert_allclose(st["exp_avg_sq"].cpu().numpy(), ora[k][2], rtol=1e-6, atol=1e-12, err_msg=k)
    with pytest.raises(ValueError):
        opt.step(torch.ones(P + 1, dtype=torch.bool, device=DEV), P + 1)


def test_densify_stats_matches_oracle():
    from gslm.model import synthetic_gaussians
    P = 5000
    m = synthetic_gaussians(P, 0, seed=0, device=DEV)
    rng = np.random.default_rng(1)
    grad = rng.normal(size=(P, 3)).astype(np.float32)
    radii = rng.integers(-2, 6, size=P).astype(np.int32)
    m.xyz_gradient_accum = torch.from_numpy(rng.random((P, 1)).astype(np.float32)).to(DEV)
    m.denom = torch.from_numpy(rng.integers(0, 5, (P, 1)).astype(np.float32)).to(DEV)
    m.max_radii2D = torch.from_numpy((rng.random(P) * 4).astype(np.float32)).to(DEV)
    mr0, acc0, den0 = (t.cpu().numpy() for t in (m.max_radii2D, m.xyz_gradient_accum, m.denom))
    vsp = torch.from_numpy(grad).to(DEV).requires_grad_(True)
    vsp.grad = vsp.detach().clone()
    m.add_densification_stats(vsp, radii=torch.from_numpy(radii).to(DEV))
    mr, acc, den = ref.densify_stats_ref(grad, radii, mr0, acc0, den0)
    assert np.array_equal(m.max_radii2D.cpu().numpy(), mr)
    assert np.array_equal(m.denom.cpu().numpy(), den)
    np.testing.assert_allclose(m.xyz_gradient_accum.cpu().numpy(), acc, rtol=2e-7, atol=0)
    # the reference's call form: a visibility index tensor (render()'s (radii > 0).nonzero())
    m.denom.zero_()
    m.add_densification_stats(vsp, torch.from_numpy(radii > 0).nonzero().to(DEV))
    assert np.array_equal(m.denom.cpu().numpy()[:, 0], (radii > 0).astype(np.float32))


@pytest.mark.parametrize("shape", [(3, 64, 48), (3, 37, 53), (1, 3, 96, 80)])
def test_ssim_loss_matches_oracle(shape):
    from gslm.loss import ssim
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.rand(shape, generator=g)
    y = (x + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1)
    xo = x.clone().double().requires_grad_(True)
    so = ssim_per_pixel(xo.reshape(-1, *shape[-3:]), y.double().reshape(-1, *shape[-3:])).mean()
    (0.2 * (1.0 - so)).backward()
    xg = x.to(DEV).requires_grad_(True)
    sg = ssim(xg, y.to(DEV))
    (0.2 * (1.0 - sg)).backward()
    assert abs(float(sg.detach()) - float(so.detach())) < 1e-6
    gref = xo.grad.float()
    assert (xg.grad.cpu() - gref).abs().max() <= 1e-5 * gref.abs().max()


def _train_scene(P=2000, D=1, W=64, H=48, views=3, s0=0.04, pert_dc=0.2, pert_opacity=0.5):
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    model = synthetic_gaussians(P, D, seed=0, s0=s0, n_cams=views)
    cams = orbit_cameras(views, W, H, seed=1)
    pert = synthetic_gaussians(P, D, seed=0, s0=s0, n_cams=views)
    gg = torch.Generator().manual_seed(2)
    with torch.no_grad():
        pert._features_dc += pert_dc * torch.randn(pert._features_dc.shape, generator=gg)
        pert._opacity += pert_opacity * torch.randn(pert._opacity.shape, generator=gg)
        for c in cams:
            img, _, _, _ = tr.render_model(pert, c, torch.zeros(3))
            c.original_image = img.detach().clone()
    return model, cams


def test_training_step_gradients_and_update_match_oracle():
    """One train.py iteration (no densification) on the GPU vs the oracle: render + (1-l) L1 + l (1-SSIM) +
    autograd on the CPU restatement, then adam_dense_ref."""
    from gslm.train import OptimizationParams, Trainer
    model, cams = _train_scene()
    cam = cams[0]
    D = model.active_sh_degree
    # oracle: leaf gradients of the same loss through the restated rasterizer
    om = copy.deepcopy(model)
    leaves = [om._xyz, om._features_dc, om._features_rest, om._opacity, om._scaling, om._rotation]
    img, _, _, _ = tr.render_model(om, cam, torch.zeros(3))
    gt = cam.original_image
    s = ssim_per_pixel(img.unsqueeze(0), gt.unsqueeze(0)).mean()
    loss_o = 0.8 * torch.abs(img - gt).mean() + 0.2 * (1.0 - s)
    loss_o.backward()
    # GPU
    opt = OptimizationParams(densify_until_iter=0)
    gm = model.to(DEV)
    gm.spatial_lr_scale = 1.0
    gm.training_setup(opt)
    for c in cams:
        c.to(DEV)
    trn = Trainer(gm, cams, opt=opt)
    g_params = [gm._xyz, gm._features_dc, gm._features_rest, gm._opacity, gm._scaling, gm._rotation]
    p0 = [p.detach().clone() for p in g_params]
    grads = {}
    # capture the leaf gradients between backward and the optimizer step
    orig_step = gm.optimizer.step

    def spy_step(*a, **k):
        for name, p in zip(GROUPS, g_params):
            grads[name] = p.grad.detach().clone()
        return orig_step(*a, **k)
    gm.optimizer.step = spy_step
    loss_g = trn.step(1, viewpoint_cam=cam)
    torch.cuda.synchronize()
    assert abs(float(loss_g) - float(loss_o.detach())) < 1e-5
    for name, lo in zip(GROUPS, leaves):
        ref_g = lo.grad
        got = grads[name].cpu()
        scale = ref_g.abs().max()
        assert (got - ref_g).abs().max() <= 1e-4 * scale + 1e-12, name
    # Adam step 1 from the GPU's own gradients (the oracle's float32 operation order)
    lrs = {g["name"]: g["lr"] for g in gm.optimizer.param_groups}
    for name, p, q0 in zip(GROUPS, g_params, p0):
        gr = grads[name].cpu().numpy()
        z = np.zeros_like(gr)
        exp_p, _, _ = ref.adam_dense_ref(q0.cpu().numpy(), gr, z, z, lrs[name], 1, eps=1e-15)
        np.testing.assert_allclose(p.detach().cpu().numpy(), exp_p, rtol=1e-6, atol=1e-9, err_msg=name)


def _eval_loss(gm, cams):
    from gslm.loss import l1_loss, ssim
    from gslm.train import PipelineParams, render
    tot = 0.0
    with torch.no_grad():
        for c in cams:
            img = render(c, gm, PipelineParams(), torch.zeros(3, device=DEV), separate_sh=True)["render"]
            tot += float(0.8 * l1_loss(img, c.original_image) + 0.2 * (1.0 - ssim(img, c.original_image)))
    return tot / len(cams)


@pytest.mark.parametrize("optimizer_type", ["default", "sparse_adam"])
def test_training_loop_with_densification(optimizer_type):
    """80 iterations of train.py's loop from a model far from the ground truth, densifying at iterations
    20 and 40: finite, the loss over all views falls, the model grows, optimizer state tracks the parameters."""
    from gslm.train import OptimizationParams, training
    model, cams = _train_scene(P=1500, pert_dc=0.8, pert_opacity=1.5)
    for c in cams:
        c.to(DEV)
    gm = model.to(DEV)
    gm.optimizer_type = optimizer_type
    gm.spatial_lr_scale = 1.0
    opt = OptimizationParams(iterations=80, densify_from_iter=10, densification_interval=20,
                             opacity_reset_interval=1000, densify_until_iter=45, position_lr_max_steps=80,
                             optimizer_type=optimizer_type)
    gm.training_setup(opt)
    sizes = []
    orig = gm.densify_and_prune

    def track(max_grad, *a, **k):
        # threshold at the 95th percentile of the accumulated screen-space gradients, so that clone and
        # split both fire on this small synthetic scene whatever its gradient scale
        acc = (gm.xyz_gradient_accum / gm.denom)[gm.denom > 0]
        orig(float(torch.quantile(acc, 0.95)), *a, **k)
        sizes.append(gm._xyz.shape[0])
    gm.densify_and_prune = track
    before = _eval_loss(gm, cams)
    losses = training(gm, cams, opt=opt, cameras_extent=3.0).cpu()
    after = _eval_loss(gm, cams)
    assert torch.isfinite(losses).all()
    assert after < 0.8 * before, (before, after)
    assert len(sizes) == 2 and sizes[0] > 1500, sizes
    for grp in gm.optimizer.param_groups:
        p = grp["params"][0]
        assert torch.isfinite(p).all()
        st = gm.optimizer.state.get(p)
        if st:
            assert st["exp_avg"].shape == p.shape and st["exp_avg_sq"].shape == p.shape
