"""CPU restatement of the first-order training step's per-Gaussian work.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of csrc/optim.hip and of
GaussianModel's densification (gslm/model.py); never by the product path.

  adam_dense_ref      torch.optim.Adam's step as the reference steps it (train.py:184-186,
                      scene/gaussian_model.py:282-283): the foreach op sequence in float32 --
                      exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
                      denom = sqrt(v) / sqrt(1-b2^t) + eps; p.addcdiv_(m, denom, -lr/(1-b1^t)).
                      Pinned by tests/golden/train_golden.npz (torch.optim.Adam's own trajectory).
  sparse_adam_ref     SparseGaussianAdam.step(visible, N) (train.py:180-183; the class comes from the
                      accelerated rasterizer, gaussian_model.py:29 -- absent here, so its adamUpdate
                      kernel is restated from the upstream 3dgs_accel release: only visible Gaussians,
                      b1 0.9, b2 0.999, no bias correction).  Parity unpinned against that binary.
  densify_stats_ref   train.py:166-167 + gaussian_model.py:561-563.
  densify_and_prune_ref  gaussian_model.py:478-559 (clone, split with given samples, prune), moments
                      carried as _prune_optimizer / cat_tensors_to_optimizer do (:421-476).
"""
import numpy as np

F32 = np.float32
GROUPS = ("xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation")


def adam_dense_ref(p, g, m, v, lr, step, b1=0.9, b2=0.999, eps=1e-8):
    """One torch.optim.Adam step (step = the count after its increment); returns new (p, m, v)."""
    p, g, m, v = (np.asarray(t, F32).copy() for t in (p, g, m, v))
    w1, w2 = F32(1.0 - b1), F32(1.0 - b2)  # torch's Python-float scalars, rounded once
    m = m + w1 * (g - m)
    v = v * F32(b2)
    v = v + (w2 * g) * g
    bc1 = 1.0 - b1 ** step
    bc2_sqrt = F32((1.0 - b2 ** step) ** 0.5)
    step_size = F32(-(lr / bc1))
    denom = np.sqrt(v) / bc2_sqrt + F32(eps)
    p = p + step_size * (m / denom)
    return p, m, v


def sparse_adam_ref(p, g, m, v, visible, lr, eps=1e-15, b1=0.9, b2=0.999):
    """Upstream adamUpdate over [N, per] rows; rows with visible[i] == False are untouched."""
    p, g, m, v = (np.asarray(t, F32).copy() for t in (p, g, m, v))
    N = visible.shape[0]
    shp = p.shape
    p, g, m, v = (t.reshape(N, -1) for t in (p, g, m, v))
    vis = np.asarray(visible, bool)
    b1, b2, lr, eps = F32(b1), F32(b2), F32(lr), F32(eps)  # upstream's float kernel arguments
    mn = b1 * m[vis] + (F32(1) - b1) * g[vis]
    vn = b2 * v[vis] + ((F32(1) - b2) * g[vis]) * g[vis]
    p[vis] = p[vis] + (-lr * mn / (np.sqrt(vn) + eps))
    m[vis], v[vis] = mn, vn
    return p.reshape(shp), m.reshape(shp), v.reshape(shp)


def densify_stats_ref(grad2d, radii, max_radii, accum, denom):
    """train.py:166 (max_radii2D) and gaussian_model.py:561-563 for vis = radii > 0."""
    grad2d = np.asarray(grad2d, F32)
    vis = np.asarray(radii) > 0
    max_radii, accum, denom = (np.asarray(t, F32).copy() for t in (max_radii, accum, denom))
    max_radii[vis] = np.maximum(max_radii[vis], np.asarray(radii, F32)[vis])
    gx, gy = grad2d[vis, 0], grad2d[vis, 1]
    accum[vis, 0] = accum[vis, 0] + np.sqrt(gx * gx + gy * gy)
    denom[vis, 0] = denom[vis, 0] + F32(1)
    return max_radii, accum, denom


def _rotation(q):
    """utils/general_utils.py:79-99 (normalise, quaternion matrix)."""
    q = q / np.sqrt((q * q).sum(1, keepdims=True))
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1)
    return R.reshape(-1, 3, 3)


def densify_and_prune_ref(params, moments, accum, denom, max_radii, radii, max_grad, min_opacity, extent,
                          max_screen_size, percent_dense, split_samples, N=2):
    """gaussian_model.py:542-559 on float64 copies.

    params: dict group -> [P, ...] array (raw leaves: xyz, f_dc, f_rest, opacity (logit), scaling (log),
    rotation); moments: dict group -> (exp_avg, exp_avg_sq); split_samples: function(stds) -> the
    N(0, stds) draws of densify_and_split (:509-511).  Returns (params, moments, n_clone, n_split, n_pruned)."""
    P = {k: np.asarray(v, np.float64) for k, v in params.items()}
    M = {k: tuple(np.asarray(t, np.float64) for t in mv) for k, mv in moments.items()}
    with np.errstate(divide="ignore", invalid="ignore"):
        grads = np.asarray(accum, np.float64) / np.asarray(denom, np.float64)
    grads[np.isnan(grads)] = 0.0
    tmp_radii = np.asarray(radii)
    scaling = lambda: np.exp(P["scaling"])

    def postfix(new):
        for k in GROUPS:
            P[k] = np.concatenate([P[k], new[k]])
            M[k] = tuple(np.concatenate([t, np.zeros_like(new[k])]) for t in M[k])

    def prune(mask):
        keep = ~mask
        for k in GROUPS:
            P[k] = P[k][keep]
            M[k] = tuple(t[keep] for t in M[k])

    # clone (:525-540)
    sel = (np.linalg.norm(grads, axis=-1) >= max_grad) & (scaling().max(1) <= percent_dense * extent)
    n_clone = int(sel.sum())
    postfix({k: P[k][sel] for k in GROUPS})
    tmp_radii = np.concatenate([tmp_radii, tmp_radii[sel]])
    # split (:499-523): the statistics were reset by the clone's postfix, but `grads` is the padded copy
    n = P["xyz"].shape[0]
    padded = np.zeros(n)
    padded[:grads.shape[0]] = grads.squeeze(-1)
    sel = (padded >= max_grad) & (scaling().max(1) > percent_dense * extent)
    n_split = int(sel.sum())
    stds = np.tile(scaling()[sel], (N, 1))
    samples = np.asarray(split_samples(stds), np.float64)
    rots = np.tile(_rotation(P["rotation"][sel]), (N, 1, 1))
    new = {k: np.tile(P[k][sel], (N,) + (1,) * (P[k].ndim - 1)) for k in GROUPS}
    new["xyz"] = np.einsum("nij,nj->ni", rots, samples) + np.tile(P["xyz"][sel], (N, 1))
    new["scaling"] = np.log(np.tile(scaling()[sel], (N, 1)) / (0.8 * N))
    postfix(new)
    prune(np.concatenate([sel, np.zeros(N * n_split, bool)]))
    # prune (:548-555): the postfix reset max_radii2D to zero, so only opacity / world size matter
    mask = (1 / (1 + np.exp(-P["opacity"])) < min_opacity).squeeze(-1)
    if max_screen_size:
        mask = mask | (np.zeros(P["xyz"].shape[0]) > max_screen_size) | (scaling().max(1) > 0.1 * extent)
    n_pruned = int(mask.sum())
    prune(mask)
    return P, M, n_clone, n_split, n_pruned
