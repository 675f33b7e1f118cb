"""PLY / checkpoint formats (scene/gaussian_model.py:315-397, train_jvp.py:82-84, 339-341).

plyfile (the reference's PLY library) is not installed here, so the file layout is checked against the
reference's construct_list_of_attributes order and plyfile's binary_little_endian vertex encoding as
restated in gslm/ply.py; round trips are bit-exact."""
import numpy as np
import pytest
import torch

from gslm.model import GaussianModel, synthetic_gaussians
from gslm import ply


def _same(a, b):
    return all(torch.equal(x, y) for x, y in zip(a.params()[:6], b.params()[:6]))


@pytest.mark.parametrize("D", [0, 1, 3])
def test_ply_round_trip_bit_exact(tmp_path, D):
    m = synthetic_gaussians(257, D, seed=4)
    path = str(tmp_path / "point_cloud" / "iteration_7" / "point_cloud.ply")
    m.save_ply(path)
    m2 = GaussianModel(D).load_ply(path, device="cpu")
    assert m2.active_sh_degree == D
    assert _same(m, m2)


def test_ply_layout_matches_reference_attribute_order(tmp_path):
    D, P = 2, 5
    K = (D + 1) ** 2
    m = synthetic_gaussians(P, D, seed=5)
    path = str(tmp_path / "m.ply")
    m.save_ply(path)
    raw = open(path, "rb").read()
    header, body = raw.split(b"end_header\n", 1)
    lines = header.decode().splitlines()
    assert lines[:3] == ["ply", "format binary_little_endian 1.0", f"element vertex {P}"]
    names = [ln.split()[2] for ln in lines if ln.startswith("property")]
    # gaussian_model.py:315-327
    ref = ["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)] + \
          [f"f_rest_{i}" for i in range(3 * (K - 1))] + ["opacity"] + [f"scale_{i}" for i in range(3)] + \
          [f"rot_{i}" for i in range(4)]
    assert names == ref
    assert all(ln.split()[1] == "float" for ln in lines if ln.startswith("property"))
    rec = np.frombuffer(body, dtype=np.dtype([(n, "<f4") for n in names]))
    rest = m._features_rest.detach().numpy()                     # [P, K-1, 3]
    for i in range(3 * (K - 1)):                                 # channel-major flattening (:332-333)
        assert np.array_equal(rec[f"f_rest_{i}"], rest[:, i % (K - 1), i // (K - 1)])
    assert np.array_equal(rec["f_dc_1"], m._features_dc.detach().numpy()[:, 0, 1])
    assert np.all(rec["nx"] == 0) and np.array_equal(rec["rot_3"], m._rotation.detach().numpy()[:, 3])


def test_ply_reads_ascii_and_shuffled_properties(tmp_path):
    """load_ply sorts f_rest_* / scale_* / rot_* by suffix (gaussian_model.py:370-389) and reads ascii."""
    D, P = 1, 3
    m = synthetic_gaussians(P, D, seed=6)
    names = ply.attribute_names(4)
    path = str(tmp_path / "b.ply")
    m.save_ply(path)
    cols = ply.read_ply_vertices(path)
    order = names[::-1]
    with open(str(tmp_path / "a.ply"), "w") as f:
        f.write(f"ply\nformat ascii 1.0\ncomment shuffled\nelement vertex {P}\n")
        f.writelines(f"property float {n}\n" for n in order)
        f.write("end_header\n")
        for i in range(P):
            f.write(" ".join(repr(float(cols[n][i])) for n in order) + "\n")
    m2 = GaussianModel(D).load_ply(str(tmp_path / "a.ply"), device="cpu")
    assert _same(m, m2)


def test_checkpoint_round_trip_weights_only(tmp_path):
    m = synthetic_gaussians(64, 2, seed=7)
    path = str(tmp_path / "chkpnt30000.pth")
    ply.save_checkpoint(m, 30000, path)
    m2 = GaussianModel(2)
    assert ply.load_checkpoint(m2, path, device="cpu") == 30000   # torch.load(..., weights_only=True)
    assert m2.active_sh_degree == m.active_sh_degree and _same(m, m2)


def test_ply_rejects_wrong_sh_degree(tmp_path):
    m = synthetic_gaussians(8, 1, seed=8)
    path = str(tmp_path / "m.ply")
    m.save_ply(path)
    with pytest.raises(ValueError):
        GaussianModel(3).load_ply(path, device="cpu")
