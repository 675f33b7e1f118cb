"""Gaussian PLY files and the checkpoint tuple.

The reference writes and reads its models with `plyfile` (scene/gaussian_model.py:315-404), which is not
installed here; this module reads and writes the same files with numpy alone:

  * one `vertex` element, float32 properties in construct_list_of_attributes order
    (gaussian_model.py:315-327): x y z nx ny nz f_dc_0..2 f_rest_0..3(K-1)-1 opacity scale_0..2 rot_0..3;
  * f_dc / f_rest are the (P, 3, K) channel-major flattening of the [P, K, 3] leaves
    (`features.transpose(1, 2).flatten(1)`, :332-333), so f_rest_i = rest[:, i % (K-1), i // (K-1)];
  * normals are written as zeros (:330) and ignored on load;
  * plyfile's default output is `binary_little_endian 1.0` (native order on x86); load_ply also accepts
    `ascii 1.0` and `binary_big_endian 1.0` vertex-only files and sorts f_rest_* / scale_* / rot_* by their
    numeric suffix as the reference does (:370-389), so files written by either implementation load in both.
The scene-loading point clouds (scene/dataset_readers.py:120-136, fetchPly / storePly: x y z nx ny nz
red green blue) use the same reader via `read_ply_vertices`.
"""
import os

import numpy as np
import torch

_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def attribute_names(K):
    """construct_list_of_attributes (gaussian_model.py:315-327) for K SH coefficients per channel."""
    names = ["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)]
    names += [f"f_rest_{i}" for i in range(3 * (K - 1))]
    names += ["opacity"] + [f"scale_{i}" for i in range(3)] + [f"rot_{i}" for i in range(4)]
    return names


def write_ply_vertices(path, names, columns):
    """Binary little-endian PLY with one `vertex` element of float32 properties."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    n = columns[0].shape[0]
    rec = np.empty(n, dtype=[(nm, "<f4") for nm in names])
    for nm, col in zip(names, columns):
        rec[nm] = col
    header = "ply\nformat binary_little_endian 1.0\n" + f"element vertex {n}\n"
    header += "".join(f"property float {nm}\n" for nm in names) + "end_header\n"
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(rec.tobytes())


def read_ply_vertices(path):
    """{property name: numpy column} of the `vertex` element (any other element must come after it)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, props, count, elem, first = None, [], 0, None, None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii").split()
            if not tok or tok[0] in ("comment", "obj_info"):
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                elem = tok[1]
                if first is None:
                    first = elem
                if elem == "vertex":
                    count = int(tok[2])
            elif tok[0] == "property":
                if tok[1] == "list":
                    if elem == "vertex":
                        raise ValueError(f"{path}: list properties in the vertex element are not supported")
                    continue
                if elem == "vertex":
                    props.append((tok[2], _PLY_TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        if first != "vertex":
            raise ValueError(f"{path}: the vertex element must come first")
        if fmt == "ascii":
            data = np.loadtxt(f, dtype=np.float64, max_rows=count, ndmin=2)
            return {nm: data[:, i].astype(np.dtype(t)) for i, (nm, t) in enumerate(props)}
        if fmt not in ("binary_little_endian", "binary_big_endian"):
            raise ValueError(f"{path}: unsupported PLY format {fmt}")
        order = "<" if fmt == "binary_little_endian" else ">"
        dt = np.dtype([(nm, order + t) for nm, t in props])
        rec = np.frombuffer(f.read(dt.itemsize * count), dtype=dt, count=count)
        return {nm: rec[nm].astype(np.dtype(t).newbyteorder("=")) for nm, t in props}


def _sorted_suffix(cols, prefix):
    names = [n for n in cols if n.startswith(prefix)]
    return sorted(names, key=lambda x: int(x.split("_")[-1]))


def save_ply(model, path):
    """GaussianModel.save_ply (gaussian_model.py:329-345)."""
    xyz = model._xyz.detach().cpu().numpy()
    P = xyz.shape[0]
    f_dc = model._features_dc.detach().transpose(1, 2).reshape(P, -1).contiguous().cpu().numpy()
    f_rest = model._features_rest.detach().transpose(1, 2).reshape(P, -1).contiguous().cpu().numpy()
    K = 1 + model._features_rest.shape[1]
    cols = [xyz[:, 0], xyz[:, 1], xyz[:, 2]] + [np.zeros(P, np.float32)] * 3
    cols += [f_dc[:, i] for i in range(3)] + [f_rest[:, i] for i in range(f_rest.shape[1])]
    cols += [model._opacity.detach().cpu().numpy()[:, 0]]
    sc, rot = model._scaling.detach().cpu().numpy(), model._rotation.detach().cpu().numpy()
    cols += [sc[:, i] for i in range(3)] + [rot[:, i] for i in range(4)]
    write_ply_vertices(path, attribute_names(K), cols)


def load_ply(model, path, device="cuda"):
    """GaussianModel.load_ply (gaussian_model.py:352-397) without the exposure.json side file
    (use_train_test_exp=False); sets active_sh_degree = max_sh_degree."""
    c = read_ply_vertices(path)
    P = c["x"].shape[0]
    K = (model.max_sh_degree + 1) ** 2
    xyz = np.stack([c["x"], c["y"], c["z"]], axis=1)
    dc = np.stack([c["f_dc_0"], c["f_dc_1"], c["f_dc_2"]], axis=1)[:, None, :]      # [P, 1, 3]
    rest_names = _sorted_suffix(c, "f_rest_")
    if len(rest_names) != 3 * K - 3:
        raise ValueError(f"{path}: {len(rest_names)} f_rest properties, expected {3 * K - 3} for SH degree "
                         f"{model.max_sh_degree}")
    rest = np.stack([c[n] for n in rest_names], axis=1) if rest_names else np.zeros((P, 0), np.float32)
    rest = rest.reshape(P, 3, K - 1).transpose(0, 2, 1)                                # [P, K-1, 3]
    scale = np.stack([c[n] for n in _sorted_suffix(c, "scale_")], axis=1)
    rot = np.stack([c[n] for n in _sorted_suffix(c, "rot")], axis=1)
    opac = c["opacity"][:, None]
    t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float32, device=device)
    n_cams = model._exposure.shape[0] if model._exposure.numel() else 1
    model.set_params(t(xyz), t(dc), t(rest), t(scale), t(rot), t(opac),
                     torch.eye(3, 4, device=device)[None].repeat(n_cams, 1, 1))
    model.active_sh_degree = model.max_sh_degree
    return model


def save_checkpoint(model, iteration, path):
    """torch.save((gaussians.capture(), iteration), path) as train_jvp.py:339-341 does (tensors only,
    so torch.load(..., weights_only=True) reads it back)."""
    torch.save((model.capture(), iteration), path)


def load_checkpoint(model, path, device="cuda"):
    """train_jvp.py:82-84: (model_params, first_iter) = torch.load(checkpoint); gaussians.restore(...)."""
    model_args, iteration = torch.load(path, weights_only=True, map_location=device)
    model.restore(model_args)
    return iteration
