"""CPU: libgslm.so loads, exports every function include/gslm.h declares, and its host-side argument
checks / workspace queries behave (no kernel is launched: there is no GPU in this container)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "gslm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gslm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from gslm import _lib
    names = _declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(_lib.lib, n)]
    assert not missing, missing
    # the ctypes table covers the header too (so the Python host binds every entry point)
    assert set(names) <= set(_lib.EXPORTS), set(names) - set(_lib.EXPORTS)


def test_abi_version_and_sizes():
    from gslm import _lib
    lib = _lib.lib
    assert lib.gslm_abi_version() == _lib.ABI_VERSION == 9
    g1, g2 = lib.gslm_geom_bytes(1000), lib.gslm_geom_bytes(2000)
    assert 0 < g1 < g2
    assert lib.gslm_binning_bytes(10_000, 1080, 1920) > 10_000 * 16
    assert lib.gslm_image_bytes(1080, 1920) >= 1080 * 1920 * 8
    assert lib.gslm_scratch_bytes(1000, 5000) >= 1000 * 48 + 5000 * 48


def test_binning_capacity_is_the_largest_fitting_list():
    """gslm_binning_capacity (ABI 7, the device-count rasterize forms): the largest pair count whose binning layout fits
    the workspace -- host arithmetic only."""
    from gslm import _lib
    lib = _lib.lib
    for H, W in ((1080, 1920), (40, 56), (2160, 3840)):
        for n in (0, 1, 4095, 4096, 4_867_236, 6_000_000):
            b = lib.gslm_binning_bytes(n, H, W)
            for extra in (0, 3, 4096):
                cap = lib.gslm_binning_capacity(b + extra, H, W)
                assert cap >= n
                assert lib.gslm_binning_bytes(cap, H, W) <= b + extra < lib.gslm_binning_bytes(cap + 1, H, W)
        assert lib.gslm_binning_capacity(lib.gslm_binning_bytes(0, H, W) - 1, H, W) == 0
    assert lib.gslm_num_rendered_copy(None, 5, None, None) == _lib.GSLM_ERR_INVALID


def test_invalid_arguments_return_error_codes():
    from gslm import _lib
    lib = _lib.lib
    assert lib.gslm_preprocess(None, None, None, 0, None, None) == _lib.GSLM_ERR_INVALID
    assert b"view" in lib.gslm_last_error()
    view = _lib.make_view(0, 64, 0.5, 0.5, [0, 0, 0], 1.0, [0.0] * 16, [0.0] * 16, 0, [0, 0, 0])
    g = _lib.make_gaussians(0)
    assert lib.gslm_preprocess(ctypes.byref(view), ctypes.byref(g), None, 0, None, None) == _lib.GSLM_ERR_INVALID
    view = _lib.make_view(64, 64, 0.5, 0.5, [0, 0, 0], 1.0, [0.0] * 16, [0.0] * 16, 4, [0, 0, 0])
    assert lib.gslm_preprocess(ctypes.byref(view), ctypes.byref(g), None, 0, None, None) == _lib.GSLM_ERR_INVALID
    assert b"sh_degree" in lib.gslm_last_error()
    view = _lib.make_view(64, 64, 0.5, 0.5, [0, 0, 0], 1.0, [0.0] * 16, [0.0] * 16, 0, [0, 0, 0])
    g = _lib.make_gaussians(10)  # P > 0 but no tensors
    assert lib.gslm_preprocess(ctypes.byref(view), ctypes.byref(g), None, 0, None, None) == _lib.GSLM_ERR_INVALID
    assert lib.gslm_damp_add(10, None, None, None, 9, None, None) == _lib.GSLM_ERR_INVALID
    # Gaussian-sharded exchange entry points (ABI v3)
    assert lib.gslm_view_flags(None, 10, None, None) == _lib.GSLM_ERR_INVALID
    assert b"view_flags" in lib.gslm_last_error()
    views = (_lib.GslmView * 17)(*([view] * 17))
    g = _lib.make_gaussians(0)
    v = _lib.GslmGrads()
    for n in (0, 17):
        assert lib.gslm_tangent_views(views, n, ctypes.byref(g), ctypes.byref(v), 1, None, 0, None, 0, None,
                                      None) == _lib.GSLM_ERR_INVALID
        assert b"nviews" in lib.gslm_last_error()
    # SH-rest coordinates (ABI v6): argument checks only (no GPU here)
    for n in (0, _lib.GSLM_MAX_REST_VIEWS + 1):
        assert lib.gslm_rest_basis(views, n, ctypes.byref(g), None, None) == _lib.GSLM_ERR_INVALID
        assert b"nviews" in lib.gslm_last_error()
    assert lib.gslm_rest_coords(views, 2, ctypes.byref(g), None, 2, None, 0, None, 0, None) == _lib.GSLM_ERR_INVALID
    assert b"mode" in lib.gslm_last_error()
    opts = _lib.GslmMatvecOpts()
    opts.rest_basis, opts.rest_views, opts.view_base = 16, 2, 1
    g.raw = 1
    assert lib.gslm_tangent_views(views, 2, ctypes.byref(g), ctypes.byref(v), 1, None, 0, None, 0, ctypes.byref(opts),
                                  None) == _lib.GSLM_ERR_INVALID
    assert b"rest_views" in lib.gslm_last_error()


def test_union_binning_argument_checks():
    """The line search's shared binning (ABI 8; ABI 9 adds each set workspace's size and n_sets): set counts outside
    1..8, slots outside [0, n_sets), set workspaces below gslm_depth_records_bytes(P), NULL workspaces and short buffers
    are refused before any launch (host-side checks only: no GPU here)."""
    from gslm import _lib
    lib = _lib.lib
    view = _lib.make_view(64, 64, 0.5, 0.5, [0, 0, 0], 1.0, [0.0] * 16, [0.0] * 16, 0, [0, 0, 0])
    vp = ctypes.byref(view)
    geoms = (ctypes.c_void_p * 9)(*([None] * 9))
    gb = lib.gslm_geom_bytes(10)
    rb = lib.gslm_depth_records_bytes(10)
    assert 10 * 64 <= rb < gb  # the depth-space sets hold their 64-B records only
    for n in (0, 9):
        assert lib.gslm_union_geometry(vp, 10, geoms, n, rb, 16, gb, None) == _lib.GSLM_ERR_INVALID
        assert b"parameter sets" in lib.gslm_last_error()
    assert lib.gslm_union_geometry(vp, 10, geoms, 2, rb, 16, gb - 1, None) == _lib.GSLM_ERR_CAPACITY
    assert lib.gslm_union_geometry(vp, 10, geoms, 2, rb - 1, 16, gb, None) == _lib.GSLM_ERR_CAPACITY
    assert b"gslm_depth_records_bytes" in lib.gslm_last_error()
    assert lib.gslm_union_geometry(vp, 10, geoms, 2, rb, 16, gb, None) == _lib.GSLM_ERR_INVALID
    assert b"NULL geometry" in lib.gslm_last_error()
    assert lib.gslm_depth_positions(None, 10, None, None) == _lib.GSLM_ERR_INVALID
    views = (_lib.GslmView * 9)(*([view] * 9))
    g = _lib.make_gaussians(0)
    for n in (0, 9):
        assert lib.gslm_preprocess_views(views, n, ctypes.byref(g), geoms, gb, None, None) == _lib.GSLM_ERR_INVALID
    # the union list carries two more words per entry than a binning (the per-set masks' sort ping-pong)
    nb = lib.gslm_union_binning_bytes(100, 64, 64)
    assert nb >= lib.gslm_binning_bytes(100, 64, 64) + 2 * 100 * 4
    assert lib.gslm_union_binning(vp, 10, 16, 16, nb - 1, 100, geoms, 2, rb, None) == _lib.GSLM_ERR_CAPACITY
    assert lib.gslm_union_binning(vp, 10, 16, 16, nb, 100, geoms, 0, rb, None) == _lib.GSLM_ERR_INVALID
    assert lib.gslm_union_binning(vp, 10, 16, 16, nb, 100, geoms, 2, rb - 1, None) == _lib.GSLM_ERR_CAPACITY
    for slot, n_sets in ((-1, 6), (8, 8), (6, 6), (2, 2), (0, 0), (0, 9)):
        assert lib.gslm_rasterize_loss_slot(vp, 10, 16, rb, 16, nb, 100, slot, n_sets, 16, None, 16, 1 << 20, 16, 0,
                                            None) == _lib.GSLM_ERR_INVALID, (slot, n_sets)
        assert b"slot" in lib.gslm_last_error()
    assert lib.gslm_rasterize_loss_slot(vp, 10, 16, rb - 1, 16, nb, 100, 0, 6, 16, None, 16, 1 << 20, 16, 0,
                                        None) == _lib.GSLM_ERR_CAPACITY
    assert lib.gslm_rasterize_loss_slot(vp, 10, 16, rb, 16, nb - 1, 100, 0, 6, 16, None, 16, 1 << 20, 16, 0,
                                        None) == _lib.GSLM_ERR_CAPACITY
    assert lib.gslm_rasterize_loss_slot(vp, 10, 16, rb, 16, nb, 100, 0, 6, None, None, 16, 1 << 20, 16, 0,
                                        None) == _lib.GSLM_ERR_INVALID


def test_dropin_modules_import_with_reference_names():
    import diff_gaussian_rasterization as d
    import diff_gaussian_rasterization.batch_render as b
    import diff_gaussian_rasterization_orig as o
    assert d.GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug", "antialiasing")
    assert b.BatchGaussianRasterizationSettings._fields[:5] == (
        "batch_size", "image_heights", "image_widths", "tanfovxs", "tanfovys")
    assert o.GaussianRasterizer is d.GaussianRasterizer
    # exported like the accelerated upstream rasterizer's (train.py:37-41): render() then passes dc= separately
    from gslm.optim import SparseGaussianAdam
    assert d.SparseGaussianAdam is SparseGaussianAdam and issubclass(SparseGaussianAdam, __import__("torch").optim.Adam)


def test_rasterizer_argument_validation():
    import torch
    from diff_gaussian_rasterization import GaussianRasterizer
    r = GaussianRasterizer(None)
    x = torch.zeros(4, 3)
    with pytest.raises(Exception, match="one of either SHs or precomputed colors"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), scales=x, rotations=torch.zeros(4, 4))
    with pytest.raises(Exception, match="scale/rotation pair"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), colors_precomp=x)
    # upstream's checks test for None, not emptiness: an empty colors_precomp beside shs is a second colour
    # source (raises), while an empty SH rest beside dc= (separate_sh at degree 0) or the empty tensors of a
    # P = 0 model are given arguments (tests/test_gpu_edge.py renders those)
    with pytest.raises(Exception, match="one of either SHs or precomputed colors"):
        r(means3D=x, means2D=x, opacities=torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), colors_precomp=torch.zeros(0),
          scales=x, rotations=torch.zeros(4, 4))


def test_simple_knn_module_binds_the_hip_kernel():
    """scene/gaussian_model.py:22 imports `from simple_knn._C import distCUDA2` at module load: the build ships
    that module, bound to the HIP kernel (gslm.knn), and it rejects host tensors instead of computing on the CPU."""
    import torch
    from simple_knn._C import distCUDA2
    from gslm import knn
    assert distCUDA2 is knn.distCUDA2
    with pytest.raises(ValueError, match="GPU tensor"):
        distCUDA2(torch.zeros(8, 3))
    with pytest.raises(ValueError, match=r"\[N, 3\]"):
        distCUDA2(torch.zeros(8, 2))


def test_shipped_library_exports_only_declared_entry_points():
    """The product .so carries no experiment / debug entry points (the round-2 gslm_dbg_* counters lived behind
    GSLM_EXPERIMENT_* defines that the product build now refuses): every exported gslm_* symbol is one
    include/gslm.h declares."""
    import subprocess
    from gslm import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = sorted({ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith("gslm_")})
    assert not [n for n in exported if n.startswith("gslm_dbg")], exported
    assert set(exported) <= set(_declared()), set(exported) - set(_declared())


def test_product_build_refuses_experiment_flags():
    import subprocess
    csrc = os.path.join(ROOT, "gaussian-splatting-lm_amd", "csrc")
    r = subprocess.run(["make", "-n", "-C", csrc, "EXTRA=-DGSLM_EXPERIMENT_SKIP_JVP"], capture_output=True, text=True)
    assert r.returncode != 0 and "not part of the product build" in (r.stdout + r.stderr)
    src = open(os.path.join(csrc, "gslm_device.hpp")).read()
    assert "#error" in src and "GSLM_EXPERIMENT_SKIP_VJP" in src


def test_no_product_kernel_uses_scratch(tmp_path):
    """Every kernel of the shipped gfx950 code object has a zero private segment: no register spills and no
    local array indexed at run time (which the compiler places in scratch memory, one memory round trip per
    access).  Read from the code object's AMDGPU metadata notes."""
    import re
    import shutil
    import subprocess
    from gslm import _lib
    llvm = "/opt/rocm/lib/llvm/bin"
    tools = [f"{llvm}/{t}" for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(shutil.which(t) for t in tools):
        pytest.skip("ROCm LLVM tools not available")
    fat = tmp_path / "fat.bin"
    subprocess.run([tools[0], f"--dump-section=.hip_fatbin={fat}", _lib.LIB_PATH, str(tmp_path / "x.so")], check=True)
    # one offload bundle per translation unit, concatenated
    blob = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
    notes = ""
    for k, a in enumerate(starts):
        part, co = tmp_path / f"b{k}.bin", tmp_path / f"b{k}.co"
        part.write_bytes(blob[a:starts[k + 1] if k + 1 < len(starts) else len(blob)])
        subprocess.run([tools[1], "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes += subprocess.run([tools[2], "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    names = re.findall(r"^\s+\.name:\s+(\S+)", notes, re.M)
    sizes = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)]
    assert len(names) == len(sizes) and len(names) > 50
    assert [n for n, s in zip(names, sizes) if s] == []


def test_comm_entry_points_check_arguments():
    """The C-ABI RCCL communicator (gslm_comm_*, gslm_allreduce_sum_*, gslm_alltoall): the id size, and NULL handles /
    bad ranks refused with GSLM_ERR_INVALID before RCCL is touched (no GPU here; tests/test_gpu_rccl.py runs them)."""
    import ctypes as C
    from gslm import _lib
    lib = _lib.lib
    assert lib.gslm_comm_id_bytes() == 128
    h = C.c_void_p()
    buf = (C.c_uint8 * 128)()
    assert lib.gslm_comm_init(None, 1, 0, C.byref(h)) == -1
    assert lib.gslm_comm_init(C.addressof(buf), 2, 2, C.byref(h)) == -1
    assert lib.gslm_comm_init(C.addressof(buf), 0, 0, C.byref(h)) == -1
    assert lib.gslm_comm_unique_id(None) == -1
    assert lib.gslm_allreduce_sum_f32(None, None, 4, None) == -1
    assert lib.gslm_allreduce_sum_f64(None, None, 4, None) == -1
    assert lib.gslm_alltoall(None, None, None, 16, None) == -1
    assert lib.gslm_allgather(None, None, None, 16, None) == -1
    assert b"NULL" in lib.gslm_last_error()
    assert lib.gslm_comm_destroy(None) == 0


def test_loss_set_group_env_is_validated(monkeypatch):
    """the line search's sets-per-blend-pass knob is GSLM_LOSS_SET_GROUP (1..8); the round-4/5 spelling
    GSLM_LOSS_SETS, whose meaning changed between those rounds, is refused, and so are out-of-range values."""
    from gslm.lm import loss_set_group
    monkeypatch.delenv("GSLM_LOSS_SETS", raising=False)
    monkeypatch.delenv("GSLM_LOSS_SET_GROUP", raising=False)
    assert loss_set_group() == 1
    for k in (1, 3, 8):
        monkeypatch.setenv("GSLM_LOSS_SET_GROUP", str(k))
        assert loss_set_group() == k
    for bad in ("0", "9", "-1", "all", ""):
        monkeypatch.setenv("GSLM_LOSS_SET_GROUP", bad)
        with pytest.raises(ValueError):
            loss_set_group()
    monkeypatch.setenv("GSLM_LOSS_SET_GROUP", "2")
    monkeypatch.setenv("GSLM_LOSS_SETS", "1")
    with pytest.raises(ValueError, match="GSLM_LOSS_SET_GROUP"):
        loss_set_group()
