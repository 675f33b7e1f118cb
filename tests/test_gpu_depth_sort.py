"""GPU: the depth sort over the frame's key span (radix_sort_pairs(key_range), sort.hip KeyRange).

The preprocess's depth sort (upstream's cub::DeviceRadixSort over (tile | depth) keys)
sorts key - min over the keys other than 0xFFFFFFFF (Gaussians behind the near plane, which sort last in index order)
and runs the passes past the span's bytes as copies.  The claim is the 32-bit stable order exactly, so the order is
compared with numpy's stable argsort of the raw keys the same preprocess writes (gslm_preprocess_views leaves them
unsorted), at depth spans that need 1, 2, 3 and 4 working passes, with ties, with every Gaussian behind the near
plane and with a single one in front, at a ragged P and on the 16-item path (P >= 4M).  The tile counts the last
pass gathers in depth order are checked too, and the working pass count the sort recorded against the one the keys
need.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _al(x):
    return (x + 255) // 256 * 256


def _layout(P):
    """Byte offsets in the geometry workspace (api.hip geom_layout: 256-B aligned regions)."""
    off, o = {}, 0
    for name, size in (("rec", 64 * P), ("depth_key", 4 * P), ("tiles", 4 * P), ("rect", 8 * P),
                       ("vals_init", 4 * P), ("keys_alt", 4 * P), ("vals_alt", 4 * P), ("offsets", 4 * P),
                       ("goff", 4 * P), ("hist", 0)):
        off[name] = o
        o += _al(size)
    items = 16 if -(-P // 4096) >= 1024 else 8  # gslm_internal.hpp sort_items
    nb = -(-P // (256 * items))
    off["range_w"] = off["hist"] + 4 * 256 * nb + 4 * 256  # after the [RADIX][nb] counts and the RADIX totals
    return off


def _passes(keys):
    """The working pass count of sort.hip's KeyRange for these keys."""
    valid = keys[keys != 0xFFFFFFFF]
    if valid.size == 0:
        return 1
    kmin, hi = int(valid.min()), int(valid.max())
    r1 = hi - kmin + 1
    t = r1 + ((((0xFF - kmin) & 0xFF) - r1) & 0xFF)
    return max(1, (t.bit_length() + 7) // 8)


def _depths(kind, P, gen):
    u = torch.rand(P, generator=gen, dtype=torch.float64)
    if kind == "span24":   # the bench scene's 1.3-4.7: 3 passes
        return 1.3 + 3.4 * u
    if kind == "span16":   # ~4e4 distinct floats: 2 passes
        return 2.0 + 0.01 * u
    if kind == "narrow":   # ~40 distinct floats: 1 or 2 passes, the rest copies
        return 2.0 + 1e-5 * u
    if kind == "ties":     # seven depths, each shared by ~P/7 Gaussians (stability)
        return torch.tensor([0.7, 1.1, 1.1000001, 2.5, 3.0, 9.0, 40.0], dtype=torch.float64)[(u * 7).long()]
    if kind == "wide":     # 0.21-5000 log-uniform, 10% behind the near plane: 4 passes
        d = torch.exp(np.log(0.21) + (np.log(5000.0) - np.log(0.21)) * u)
        behind = torch.rand(P, generator=gen) < 0.1
        d[behind] = -3.0 + 3.1 * u[behind]
        return d
    if kind == "behind":   # nothing in front of the near plane
        return -2.0 + 2.15 * u
    if kind == "one":      # one Gaussian in front
        d = -2.0 + 2.15 * u
        d[P // 3] = 1.0
        return d
    raise ValueError(kind)


@pytest.mark.parametrize("kind,P", [("span24", 100_003), ("span16", 100_003), ("narrow", 100_003),
                                    ("ties", 100_003), ("wide", 100_003), ("behind", 70_001), ("one", 5_000),
                                    ("span24", 4_300_001), ("wide", 4_300_001)])
def test_depth_sort_equals_stable_argsort(kind, P):
    from gslm import _lib
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    from gslm.params import raw_gaussians
    lib = _lib.lib
    gen = torch.Generator().manual_seed(11)
    m = synthetic_gaussians(P, 1, seed=4, s0=0.01)
    cam = orbit_cameras(1, 160, 96, seed=3)[0]
    # move each Gaussian along its ray from the camera centre to the wanted view depth
    W = cam.world_view_transform.double()
    c = cam.camera_center.double()
    xyz = m._xyz.detach().double()
    d = (torch.cat([xyz, torch.ones(P, 1, dtype=torch.float64)], 1) @ W)[:, 2]
    assert bool((d > 0.5).all())
    want = _depths(kind, P, gen)
    with torch.no_grad():
        m._xyz.copy_((c + (xyz - c) * (want / d)[:, None]).float())
    m = m.to("cuda")
    g = raw_gaussians(m)
    view = _lib.view_from_camera(cam, torch.zeros(3), 1)
    nb = lib.gslm_geom_bytes(P)
    a = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    b = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    # raw keys and tile counts (gslm_preprocess_views: no sort)
    ge = (ctypes.c_void_p * 1)(b.data_ptr())
    assert lib.gslm_preprocess_views(ctypes.byref(view), 1, ctypes.byref(g), ge, nb, None, None) == 0, \
        lib.gslm_last_error()
    order = torch.empty(P, dtype=torch.int32, device="cuda")
    assert lib.gslm_preprocess_ordered(ctypes.byref(view), ctypes.byref(g), a.data_ptr(), nb, None, order.data_ptr(),
                                       1, None) == 0, lib.gslm_last_error()
    torch.cuda.synchronize()
    off = _layout(P)
    keys = b[off["depth_key"]:off["depth_key"] + 4 * P].view(torch.int32).cpu().numpy().view(np.uint32)
    tiles = b[off["tiles"]:off["tiles"] + 4 * P].view(torch.int32).cpu().numpy()
    want_order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(order.cpu().numpy(), want_order.astype(np.int32))
    # the last pass's gather: the tile counts in depth order, where the sorted keys would be (4 passes: no ping-pong)
    tiles_sorted = a[off["depth_key"]:off["depth_key"] + 4 * P].view(torch.int32).cpu().numpy()
    np.testing.assert_array_equal(tiles_sorted, tiles[want_order])
    w = a[off["range_w"]:off["range_w"] + 12].view(torch.int32).cpu().numpy().view(np.uint32)
    assert int(w[2]) == _passes(keys), (kind, w)
    expect = {"span24": 3, "span16": 2, "behind": 1, "wide": 4}  # (narrow / one: 1 or 2, by the low byte of the min)
    if kind in expect:
        assert int(w[2]) == expect[kind], (kind, w)
