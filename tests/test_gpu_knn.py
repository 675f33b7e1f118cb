"""distCUDA2 (csrc/knn.hip) against the exact CPU oracle (oracle/knn_ref.py: scipy KD-tree neighbours,
float32 distance arithmetic of simple-knn's updateKBest), and create_from_pcd's scale initialisation
(scene/gaussian_model.py:236-265).  Same float32 formula on both sides: the values must agree to 1e-6."""
import numpy as np
import pytest
import torch

from oracle.knn_ref import dist_cuda2_ref

pytestmark = pytest.mark.gpu


def _clouds():
    g = np.random.default_rng(31)
    cube = g.random((100_000, 3), dtype=np.float32) * 4 - 2
    plane = np.concatenate([g.random((40_000, 2), dtype=np.float32), np.zeros((40_000, 1), np.float32)], 1)
    blobs = np.concatenate([g.normal(c, 0.01, (3000, 3)) for c in ((0, 0, 0), (5, 0, 0), (0, 7, -3))]).astype(np.float32)
    dup = g.random((500, 3), dtype=np.float32)
    dup = np.concatenate([dup, dup[:20]])                  # exact duplicates: distance 0 neighbours
    line = np.stack([np.linspace(0, 1, 777, dtype=np.float32)] + [np.zeros(777, np.float32)] * 2, 1)
    return {"cube_100k": cube, "plane_40k": plane, "blobs": blobs, "duplicates": dup, "line": line}


@pytest.mark.parametrize("name", list(_clouds()))
def test_knn3_matches_exact_oracle(name):
    from gslm.knn import distCUDA2
    p = _clouds()[name]
    got = distCUDA2(torch.from_numpy(p).cuda()).cpu().numpy()
    ref = dist_cuda2_ref(p)
    scale = np.maximum(np.abs(ref), 1e-30)
    assert np.max(np.abs(got - ref) / scale) <= 1e-6


def test_knn3_fewer_than_four_points():
    from gslm.knn import distCUDA2
    p = np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0]], np.float32)
    got = distCUDA2(torch.from_numpy(p).cuda()).cpu().numpy()
    assert np.array_equal(got, dist_cuda2_ref(p))           # one missing neighbour: FLT_MAX / 3 terms


def test_create_from_pcd_scales():
    from gslm.knn import distCUDA2
    from gslm.model import GaussianModel
    g = np.random.default_rng(32)
    pts = g.random((5000, 3), dtype=np.float32)
    cols = g.random((5000, 3), dtype=np.float32)
    m = GaussianModel(3).create_from_pcd(pts, cols, n_cams=2)
    d2 = torch.clamp_min(torch.from_numpy(dist_cuda2_ref(pts)), 0.0000001)
    ref = torch.log(torch.sqrt(d2))[:, None].repeat(1, 3)
    assert torch.allclose(m._scaling.detach().cpu(), ref, rtol=0, atol=1e-6)
    assert m._features_rest.shape == (5000, 15, 3) and float(m._features_rest.abs().max()) == 0.0
    assert torch.allclose(m.get_opacity.detach().cpu(), torch.full((5000, 1), 0.1), atol=1e-6)
    assert m._exposure.shape == (2, 3, 4)
    assert distCUDA2(torch.from_numpy(pts).cuda()).shape == (5000,)


def test_simple_knn_module_matches_oracle():
    """The reference's import path (scene/gaussian_model.py:22, :249) reaches the same kernel."""
    from simple_knn._C import distCUDA2
    p = _clouds()["blobs"]
    got = torch.clamp_min(distCUDA2(torch.from_numpy(p).float().cuda()), 0.0000001).cpu().numpy()
    ref = np.maximum(dist_cuda2_ref(p), 0.0000001)
    assert np.abs(got - ref).max() <= 1e-6 * np.abs(ref).max()
