"""CPU: the first-order training row -- oracle against the reference's golden vectors,
and the host-side logic of GaussianModel (schedules, optimizer groups, densification) against the oracle.

The HIP kernels (gslm_adam_step, gslm_densify_stats, gslm_ssim_mean) are checked in test_gpu_train.py."""
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from gslm.model import GaussianModel, eval_sh, get_expon_lr_func, synthetic_gaussians
from oracle import train_ref as ref

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "train_golden.npz"))
GROUP_SHAPES = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def test_lr_schedules_match_reference():
    steps = GOLD["steps"]
    f = {"xyz": get_expon_lr_func(0.00016 * 2.5, 0.0000016 * 2.5, lr_delay_mult=0.01, max_steps=30_000),
         "exposure": get_expon_lr_func(0.01, 0.001, lr_delay_steps=0, lr_delay_mult=0.0, max_steps=30_000),
         "delayed": get_expon_lr_func(0.01, 0.001, lr_delay_steps=1000, lr_delay_mult=0.1, max_steps=30_000)}
    for k, fn in f.items():
        got = np.array([fn(int(s)) for s in steps])
        np.testing.assert_allclose(got, GOLD[f"lr_{k}"], rtol=1e-15, atol=0)
    assert get_expon_lr_func(0.0, 0.0)(5) == 0.0 and get_expon_lr_func(1e-3, 1e-4)(-1) == 0.0


def test_dense_adam_oracle_matches_torch_adam_golden():
    """adam_dense_ref over 4 steps equals torch.optim.Adam's trajectory (the reference's optimizer)."""
    n = int(GOLD["adam_steps"])
    for k in GROUP_SHAPES:
        p = GOLD[f"adam_p0_{k}"].copy()
        m, v = np.zeros_like(p), np.zeros_like(p)
        for it in range(n):
            p, m, v = ref.adam_dense_ref(p, GOLD[f"adam_g{it}_{k}"], m, v, float(GOLD[f"adam_lr_{k}"]), it + 1,
                                         eps=1e-15)
        np.testing.assert_allclose(m, GOLD[f"adam_m_{k}"], rtol=1e-5, atol=1e-8)  # CPU lerp may fuse
        np.testing.assert_allclose(v, GOLD[f"adam_v_{k}"], rtol=2e-6, atol=1e-12)
        np.testing.assert_allclose(p, GOLD[f"adam_p_{k}"], rtol=2e-6, atol=1e-7)


def test_sparse_adam_oracle_semantics():
    """Visible rows follow the bias-free upstream update, invisible rows are untouched."""
    rng = np.random.default_rng(0)
    N, per = 13, 3
    p, g = rng.normal(size=(N, per)).astype(np.float32), rng.normal(size=(N, per)).astype(np.float32)
    m, v = rng.normal(size=(N, per)).astype(np.float32), rng.random((N, per)).astype(np.float32)
    vis = rng.random(N) < 0.5
    p2, m2, v2 = ref.sparse_adam_ref(p, g, m, v, vis, lr=0.01, eps=1e-15)
    assert np.array_equal(p2[~vis], p[~vis]) and np.array_equal(m2[~vis], m[~vis]) and np.array_equal(v2[~vis], v[~vis])
    mm = 0.9 * m + 0.1 * g
    vv = 0.999 * v + 0.001 * g * g
    np.testing.assert_allclose(m2[vis], mm[vis], rtol=1e-6)
    np.testing.assert_allclose(v2[vis], vv[vis], rtol=1e-6)
    np.testing.assert_allclose(p2[vis], (p - 0.01 * mm / (np.sqrt(vv) + 1e-15))[vis], rtol=1e-5, atol=1e-7)


def test_python_sh_path_matches_reference_golden():
    """render(convert_SHs_python=True) evaluates utils/sh_utils.eval_sh (golden from the reference)."""
    d = np.load(os.path.join(HERE, "golden", "sh_golden.npz"))
    for deg in range(4):
        got = eval_sh(deg, torch.from_numpy(d[f"sh{deg}"]), torch.from_numpy(d[f"dirs{deg}"]))
        np.testing.assert_allclose(got.numpy(), d[f"rgb{deg}"], rtol=0, atol=1e-12)


def _opt_args(**kw):
    from gslm.train import OptimizationParams
    o = OptimizationParams()
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _cpu_setup(model, opt):
    """training_setup's groups with torch's own Adam on CPU (the surgery code is optimizer-agnostic)."""
    model.training_setup(opt)
    groups = [{"params": g["params"], "lr": g["lr"], "name": g["name"]} for g in model.optimizer.param_groups]
    model.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
    return model


def test_training_setup_groups_match_reference():
    m = synthetic_gaussians(20, 3, seed=0)
    m.spatial_lr_scale = 2.5
    opt = _opt_args()
    m.training_setup(opt)
    lrs = {g["name"]: g["lr"] for g in m.optimizer.param_groups}
    # gaussian_model.py:273-280
    assert lrs == {"xyz": 0.00016 * 2.5, "f_dc": 0.0025, "f_rest": 0.0025 / 20.0, "opacity": 0.025,
                   "scaling": 0.005, "rotation": 0.001}
    assert all(g["eps"] == 1e-15 for g in m.optimizer.param_groups)
    assert m.xyz_gradient_accum.shape == (20, 1) and m.denom.shape == (20, 1) and m.max_radii2D.shape == (20,)
    assert m.update_learning_rate(0) == pytest.approx(0.00016 * 2.5)
    assert m.update_learning_rate(30_000) == pytest.approx(0.0000016 * 2.5)
    from gslm.optim import FusedAdam, SparseGaussianAdam
    assert type(m.optimizer) is FusedAdam
    m2 = synthetic_gaussians(20, 3, seed=0)
    m2.optimizer_type = "sparse_adam"
    m2.training_setup(opt)
    assert type(m2.optimizer) is SparseGaussianAdam


@pytest.mark.parametrize("max_screen_size", [None, 20])
def test_densify_and_prune_matches_oracle(max_screen_size):
    torch.manual_seed(0)
    P = 300
    m = synthetic_gaussians(P, 2, seed=5, s0=0.02)
    with torch.no_grad():
        m._scaling += torch.log(torch.rand(P, 3) * 3 + 0.2)  # mix of clone (small) and split (large) sizes
        m._opacity[::7] = -6.0  # some below min_opacity after densification
    m.spatial_lr_scale = 1.0
    _cpu_setup(m, _opt_args())
    # populate Adam moments: one step on random gradients
    for grp in m.optimizer.param_groups:
        grp["params"][0].grad = torch.randn_like(grp["params"][0])
    m.optimizer.step()
    m.optimizer.zero_grad(set_to_none=True)
    accum = torch.rand(P, 1) * 4e-4
    denom = torch.randint(0, 4, (P, 1)).float()
    m.xyz_gradient_accum, m.denom = accum.clone(), denom.clone()
    m.max_radii2D = torch.rand(P) * 40
    radii = torch.randint(0, 30, (P,), dtype=torch.int32)
    extent = 3.0
    params0 = {k: getattr(m, m._GROUP_ATTR[k]).detach().numpy().copy() for k in GROUP_SHAPES}
    moments0 = {}
    for grp in m.optimizer.param_groups:
        st = m.optimizer.state[grp["params"][0]]
        moments0[grp["name"]] = (st["exp_avg"].numpy().copy(), st["exp_avg_sq"].numpy().copy())
    rng = torch.Generator().manual_seed(7)
    draws = []

    def samples(stds):
        s = torch.randn(stds.shape, generator=rng, dtype=stds.dtype) * stds
        draws.append(s.clone())
        return s
    m._split_samples = samples
    m.densify_and_prune(0.0002, 0.005, extent, max_screen_size, radii)
    P_ref, M_ref, n_clone, n_split, n_pruned = ref.densify_and_prune_ref(
        params0, moments0, accum.numpy(), denom.numpy(), m.max_radii2D.numpy(), radii.numpy(), 0.0002, 0.005,
        extent, max_screen_size, 0.01, lambda stds: draws[0].double().numpy())
    assert n_clone > 0 and n_split > 0 and n_pruned > 0, (n_clone, n_split, n_pruned)
    for k in GROUP_SHAPES:
        got = getattr(m, m._GROUP_ATTR[k]).detach().double().numpy()
        assert got.shape == P_ref[k].shape, (k, got.shape, P_ref[k].shape)
        np.testing.assert_allclose(got, P_ref[k], rtol=1e-6, atol=1e-6, err_msg=k)
    for grp in m.optimizer.param_groups:
        st = m.optimizer.state[grp["params"][0]]
        assert st["exp_avg"].shape == grp["params"][0].shape
        np.testing.assert_allclose(st["exp_avg"].double().numpy(), M_ref[grp["name"]][0], rtol=0, atol=0)
        np.testing.assert_allclose(st["exp_avg_sq"].double().numpy(), M_ref[grp["name"]][1], rtol=0, atol=0)
    n = m._xyz.shape[0]
    assert m.xyz_gradient_accum.shape == (n, 1) and m.denom.shape == (n, 1) and m.max_radii2D.shape == (n,)
    assert float(m.xyz_gradient_accum.abs().sum()) == 0.0 and m.tmp_radii is None


def test_reset_opacity_and_state_surgery():
    m = synthetic_gaussians(50, 1, seed=1)
    _cpu_setup(m, _opt_args())
    for grp in m.optimizer.param_groups:
        grp["params"][0].grad = torch.ones_like(grp["params"][0])
    m.optimizer.step()
    before = m.get_opacity.detach().clone()
    m.reset_opacity()
    after = m.get_opacity.detach()
    torch.testing.assert_close(after, torch.minimum(before, torch.full_like(before, 0.01)), rtol=1e-5, atol=1e-7)
    grp = next(g for g in m.optimizer.param_groups if g["name"] == "opacity")
    assert grp["params"][0] is m._opacity
    st = m.optimizer.state[m._opacity]
    assert float(st["exp_avg"].abs().sum()) == 0.0 and float(st["exp_avg_sq"].abs().sum()) == 0.0
    # the other groups keep their moments and the same Parameter objects
    xyz_grp = next(g for g in m.optimizer.param_groups if g["name"] == "xyz")
    assert xyz_grp["params"][0] is m._xyz and float(m.optimizer.state[m._xyz]["exp_avg"].abs().sum()) > 0
    # a checkpoint round trip of the optimizer state (gaussian_model.py:158-190)
    sd = m.optimizer.state_dict()
    assert {"exp_avg", "exp_avg_sq", "step"} <= set(sd["state"][0])


def test_densify_stats_oracle():
    rng = np.random.default_rng(3)
    P = 100
    grad = rng.normal(size=(P, 3)).astype(np.float32)
    radii = rng.integers(-1, 5, size=P).astype(np.int32)
    mr, acc, den = rng.random(P).astype(np.float32) * 3, np.zeros((P, 1), np.float32), np.zeros((P, 1), np.float32)
    mr2, acc2, den2 = ref.densify_stats_ref(grad, radii, mr, acc, den)
    vis = radii > 0
    assert np.array_equal(den2[:, 0], vis.astype(np.float32))
    np.testing.assert_allclose(acc2[vis, 0], np.linalg.norm(grad[vis, :2], axis=1), rtol=1e-6)
    assert np.array_equal(mr2[~vis], mr[~vis]) and np.all(mr2[vis] >= radii[vis])
