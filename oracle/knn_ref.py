"""ORACLE -- test infrastructure only: distCUDA2 (simple-knn, called at scene/gaussian_model.py:249) on the CPU.

The submodule is absent; its published algorithm returns, per point, the mean of the squared
distances to its 3 nearest other points, each squared distance evaluated in float32 as
d.x*d.x + d.y*d.y + d.z*d.z and the mean as (b0 + b1 + b2) / 3.  Neighbours are found exactly with
scipy's KD-tree (float64); the value is then formed in float32 with that arithmetic."""
import numpy as np
from scipy.spatial import cKDTree


def dist_cuda2_ref(points):
    p = np.asarray(points, dtype=np.float32)
    n = p.shape[0]
    k = min(4, n)
    _, idx = cKDTree(p.astype(np.float64)).query(p.astype(np.float64), k=k)
    idx = idx.reshape(n, k)
    own = idx == np.arange(n)[:, None]
    # drop the point itself (a duplicate may come first: drop exactly one self entry per row)
    keep = np.ones_like(own)
    first_self = own.argmax(axis=1)
    has_self = own.any(axis=1)
    keep[np.arange(n)[has_self], first_self[has_self]] = False
    rows = [idx[i][keep[i]][:3] for i in range(n)]
    best = np.full((n, 3), np.finfo(np.float32).max, dtype=np.float32)
    for i, r in enumerate(rows):
        d = p[r] - p[i]
        ds = np.sort((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
        best[i, :len(ds)] = ds
    return ((best[:, 0] + best[:, 1]) + best[:, 2]) / np.float32(3.0)
