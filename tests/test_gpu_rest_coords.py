"""GPU: the SH-rest coordinates of the Gaussian-sharded exchange (include/gslm.h, gslm_rest_basis /
gslm_rest_coords).

The CG iterate's SH-rest group lies in span{B_rest(dir_b)} over the job's views; the exchange stores 3 V
coordinates per Gaussian in an orthonormal basis Q of that span, B = Q R.  Checked here against a float64
restatement on the host (the oracle's eval_sh evaluated on one-hot coefficients gives the basis vectors):
  - R is the upper Cholesky factor of the views' Gram matrix, in view order, with a repeated camera's row
    dropped (zero) and its column equal to the original's;
  - project -> expand is the orthogonal projection onto the span (idempotent, residual orthogonal to every
    B_b), expand -> project the identity on coordinates, and the coordinates' norm the vector's norm.
The product in these coordinates against the reference layout's is in test_gpu_dist.py / test_gpu_configs34.py.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
W, H = 64, 48


def _setup(P=3000, nv=4, repeat=1):
    from gslm import _lib
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    from gslm.params import raw_gaussians
    cams = orbit_cameras(nv, W, H, seed=1)
    cams = cams + [cams[repeat]]  # a repeated camera: its SH-rest direction adds nothing to the span
    model = synthetic_gaussians(P, 3, seed=0, s0=0.03, n_cams=len(cams)).to("cuda")
    views = (_lib.GslmView * len(cams))()
    for k, c in enumerate(cams):
        views[k] = _lib.view_from_camera(c, torch.zeros(3), 3)
    return model, cams, views, raw_gaussians(model)


def _basis(model, cams):
    """[V, P, 15] float64: B_rest(dir_b) of every Gaussian (the oracle's eval_sh on one-hot coefficients)."""
    from oracle.torch_raster import eval_sh
    xyz = model._xyz.detach().double().cpu()
    out = []
    for c in cams:
        d = xyz - c.camera_center.double().cpu()
        d = d / d.norm(dim=1, keepdim=True)
        rows = []
        for k in range(1, 16):
            sh = torch.zeros(xyz.shape[0], 16, 1, dtype=torch.float64)
            sh[:, k, 0] = 1.0
            rows.append(eval_sh(3, sh, d)[:, 0])
        out.append(torch.stack(rows, 1))
    return torch.stack(out).numpy()


def _cholesky_ref(B):
    """Column-wise upper Cholesky of G = B B^T per Gaussian with the kernel's drop rule; packed by columns."""
    V, P, _ = B.shape
    G = np.einsum("apk,bpk->pab", B, B)
    R = np.zeros((P, V, V))
    for b in range(V):
        d = G[:, b, b].copy()
        for j in range(b):
            keep = R[:, j, j] != 0
            r = G[:, j, b] - np.einsum("pq,pq->p", R[:, :j, j], R[:, :j, b])
            R[:, j, b] = np.where(keep, r / np.where(keep, R[:, j, j], 1.0), 0.0)
            d -= R[:, j, b] ** 2
        R[:, b, b] = np.where((G[:, b, b] > 0) & (d > 1e-7 * G[:, b, b]), np.sqrt(np.maximum(d, 0)), 0.0)
    return np.concatenate([R[:, :b + 1, b] for b in range(V)], axis=1)


def _rest_basis(views, V, g, P):
    from gslm import _lib
    R = torch.zeros(P * V * (V + 1) // 2, device="cuda")
    assert _lib.lib.gslm_rest_basis(views, V, ctypes.byref(g), R.data_ptr(), None) == 0, _lib.lib.gslm_last_error()
    return R


def _coords(views, V, g, R, mode, x, P):
    from gslm import _lib
    out = torch.zeros(P, 3 * V if mode == 1 else 45, device="cuda")
    assert _lib.lib.gslm_rest_coords(views, V, ctypes.byref(g), R.data_ptr(), mode, x.data_ptr(), x.shape[1],
                                     out.data_ptr(), out.shape[1], None) == 0, _lib.lib.gslm_last_error()
    return out


def test_rest_basis_is_the_cholesky_factor_of_the_views_gram():
    model, cams, views, g = _setup()
    P, V = model._xyz.shape[0], len(cams)
    R = _rest_basis(views, V, g, P).reshape(P, -1).cpu().double().numpy()
    ref = _cholesky_ref(_basis(model, cams))
    assert np.abs(R - ref).max() <= 1e-5 * np.abs(ref).max()
    # the repeated camera (view 4 = view 1): diagonal dropped, column = the original's
    col4 = R[:, 10:15]
    assert np.all(col4[:, 4] == 0)
    assert np.abs(col4[:, :2] - R[:, 1:3]).max() <= 1e-5 * np.abs(R[:, 1:3]).max()
    assert np.abs(col4[:, 2:4]).max() <= 1e-4


def test_rest_coords_projection_and_roundtrip():
    model, cams, views, g = _setup()
    P, V = model._xyz.shape[0], len(cams)
    R = _rest_basis(views, V, g, P)
    gen = torch.Generator().manual_seed(0)
    t = torch.randn(P, 45, generator=gen).cuda()
    c = _coords(views, V, g, R, 1, t, P)
    t2 = _coords(views, V, g, R, 0, c, P)
    c2 = _coords(views, V, g, R, 1, t2, P)
    t3 = _coords(views, V, g, R, 0, c2, P)
    torch.cuda.synchronize()
    assert (c2 - c).abs().max() <= 1e-5 * c.abs().max()          # expand -> project = identity on coordinates
    assert (t3 - t2).abs().max() <= 1e-5 * t2.abs().max()        # the projection is idempotent
    # coordinates in an orthonormal basis: |c| = |Q c| per Gaussian
    n_c, n_t = c.double().norm(dim=1), t2.double().norm(dim=1)
    assert ((n_c - n_t).abs() <= 1e-5 * n_t.max()).all()
    assert c.view(P, V, 3)[:, 4].abs().max() == 0                 # the dropped view's coordinate stays 0
    # the residual t - Pt is orthogonal to every view's SH-rest direction (per channel)
    B = torch.from_numpy(_basis(model, cams))                      # [V, P, 15]
    res = (t - t2).double().cpu().view(P, 15, 3)
    dots = torch.einsum("vpk,pkc->vpc", B, res)
    assert dots.abs().max() <= 1e-5 * t.abs().max() * B.abs().max()
    # a vector in the span is reproduced: t = sum_b B_b y_b
    y = torch.randn(V, P, 3, generator=gen, dtype=torch.float64)
    ts = torch.einsum("vpk,vpc->pkc", B, y).reshape(P, 45).float().cuda()
    back = _coords(views, V, g, R, 0, _coords(views, V, g, R, 1, ts, P), P)
    torch.cuda.synchronize()
    assert (back - ts).abs().max() <= 1e-5 * ts.abs().max()


def test_nearly_collinear_views_expand_consistently():
    """Views whose SH-rest directions are nearly parallel (a camera moved by 1e-4 .. 1e-2 of the orbit radius): the
    expansion of coordinates c is what the CG kernels assume it is -- B_b^T expand(c) = (R^T c)_b for every view b
    (view b's colour tangent from the coordinates) -- to 1e-3 of |B| |c|, kept views and dropped ones alike (the float
    R's rounding is amplified by 1 / R[b][b], which the drop cut bounds)."""
    from gslm import _lib
    from gslm.cameras import Camera, orbit_cameras
    from gslm.model import synthetic_gaussians
    from gslm.params import raw_gaussians
    base = orbit_cameras(3, W, H, seed=2)
    cams = list(base)
    for k, eps in enumerate((1e-4, 1e-3, 1e-2)):
        c0 = base[k]
        # the same camera translated along its own x axis by eps of the orbit radius (3)
        T_ = np.asarray(c0.T, dtype=np.float64) + np.array([3.0 * eps, 0.0, 0.0])
        cams.append(Camera(np.asarray(c0.R), T_, c0.FoVx, c0.FoVy, width=W, height=H))
    model = synthetic_gaussians(4000, 3, seed=0, s0=0.03, n_cams=len(cams)).to("cuda")
    views = (_lib.GslmView * len(cams))()
    for k, c in enumerate(cams):
        views[k] = _lib.view_from_camera(c, torch.zeros(3), 3)
    g = raw_gaussians(model)
    P, V = model._xyz.shape[0], len(cams)
    R = _rest_basis(views, V, g, P)
    c = torch.randn(P, 3 * V, generator=torch.Generator().manual_seed(5)).cuda()
    t = _coords(views, V, g, R, 0, c, P)
    torch.cuda.synchronize()
    B = torch.from_numpy(_basis(model, cams))                       # [V, P, 15]
    lhs = torch.einsum("vpk,pkc->pvc", B, t.double().cpu().view(P, 15, 3))
    Rp = R.double().cpu().view(P, -1)
    rhs = torch.zeros(P, V, 3, dtype=torch.float64)
    cc = c.double().cpu().view(P, V, 3)
    for b in range(V):
        for j in range(b + 1):
            rhs[:, b] += Rp[:, b * (b + 1) // 2 + j, None] * cc[:, j]
    scale = B.norm(dim=2).max() * cc.norm(dim=(1, 2)).max()
    assert ((lhs - rhs).abs().max() / scale).item() <= 1e-3
