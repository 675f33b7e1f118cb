"""ctypes binding of libgslm.so (C ABI in include/gslm.h).

There is deliberately no fallback: if the HIP library is missing the import fails loudly, so no
caller can silently run a CPU or eager-PyTorch path in its place.
"""
import ctypes
import math
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(os.path.dirname(_HERE), "build", "libgslm.so")
LIB_PATH = os.environ.get("GSLM_LIB", _DEFAULT_LIB)

GSLM_OK = 0
GSLM_ERR_INVALID = -1
GSLM_ERR_HIP = -2
GSLM_ERR_CAPACITY = -3
GSLM_MAX_REST_VIEWS = 8  # include/gslm.h


class GslmView(ctypes.Structure):
    _fields_ = [
        ("image_height", ctypes.c_int32), ("image_width", ctypes.c_int32),
        ("tanfovx", ctypes.c_double), ("tanfovy", ctypes.c_double), ("scale_modifier", ctypes.c_double),
        ("viewmatrix", ctypes.c_float * 16), ("projmatrix", ctypes.c_float * 16),
        ("campos", ctypes.c_float * 3), ("bg", ctypes.c_float * 3),
        ("sh_degree", ctypes.c_int32), ("prefiltered", ctypes.c_int32),
        ("antialiasing", ctypes.c_int32), ("debug", ctypes.c_int32),
    ]


class GslmGaussians(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int64), ("max_coeffs", ctypes.c_int32), ("raw", ctypes.c_int32),
        ("means3D", ctypes.c_void_p), ("opacities", ctypes.c_void_p), ("scales", ctypes.c_void_p),
        ("rotations", ctypes.c_void_p), ("cov3D_precomp", ctypes.c_void_p),
        ("sh_dc", ctypes.c_void_p), ("sh_dc_stride", ctypes.c_int64),
        ("sh_rest", ctypes.c_void_p), ("sh_rest_stride", ctypes.c_int64),
        ("colors_precomp", ctypes.c_void_p),
    ]


class GslmGrads(ctypes.Structure):
    _fields_ = [
        ("means2D", ctypes.c_void_p), ("means3D", ctypes.c_void_p), ("opacities", ctypes.c_void_p),
        ("scales", ctypes.c_void_p), ("rotations", ctypes.c_void_p), ("cov3D", ctypes.c_void_p),
        ("sh_dc", ctypes.c_void_p), ("sh_dc_stride", ctypes.c_int64),
        ("sh_rest", ctypes.c_void_p), ("sh_rest_stride", ctypes.c_int64),
        ("colors", ctypes.c_void_p), ("accumulate", ctypes.c_int32),
    ]


class GslmMatvecOpts(ctypes.Structure):
    _fields_ = [
        ("stages", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("damp7", ctypes.POINTER(ctypes.c_double)), ("dot_vy", ctypes.c_void_p),
        ("dot_scratch", ctypes.c_void_p), ("dot_scratch_bytes", ctypes.c_size_t),
        ("xpby_s", ctypes.c_void_p), ("beta_num", ctypes.c_void_p), ("beta_den", ctypes.c_void_p),
        ("xpby_tail_v", ctypes.c_void_p), ("xpby_tail_s", ctypes.c_void_p), ("xpby_tail_n", ctypes.c_int64),
        ("screen_out", ctypes.c_void_p), ("pixel_seed", ctypes.c_void_p), ("jv_out", ctypes.c_void_p),
        ("alpha_num", ctypes.c_void_p), ("alpha_den", ctypes.c_void_p), ("xpby_x_offset", ctypes.c_int64),
        ("trec_in", ctypes.c_void_p), ("screen_stride", ctypes.c_int64),
        ("cg_ctl", ctypes.c_void_p),
        ("rest_basis", ctypes.c_void_p), ("rest_views", ctypes.c_int32), ("view_base", ctypes.c_int32),
    ]


class GslmAdamGroup(ctypes.Structure):
    _fields_ = [
        ("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
        ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_int64), ("floats_per_gaussian", ctypes.c_int32),
        ("_pad", ctypes.c_int32), ("lr", ctypes.c_double), ("step", ctypes.c_int64),
    ]


ADAM_MAX_GROUPS = 8  # GSLM_ADAM_MAX_GROUPS


# Every symbol include/gslm.h declares; tests check the library exports each of them.
EXPORTS = {
    "gslm_geom_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "gslm_image_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "gslm_binning_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "gslm_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int64]),
    "gslm_preprocess": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians), ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_num_rendered": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                         ctypes.c_void_p]),
    "gslm_preprocess_ordered": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians),
                                               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_int32, ctypes.c_void_p]),
    "gslm_preprocess_views": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int32, ctypes.POINTER(GslmGaussians),
                                             ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "gslm_depth_positions": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_num_rendered_many": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                                              ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "gslm_rasterize": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_loss_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "gslm_rasterize_loss": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int32,
                                           ctypes.c_void_p]),
    "gslm_binning_capacity": (ctypes.c_int64, [ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32]),
    "gslm_rasterize_dev": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_rasterize_loss_dev": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int32,
                                               ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_num_rendered_copy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_union_binning_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "gslm_depth_records_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "gslm_union_geometry": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.c_int32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p]),
    "gslm_union_binning": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.c_int32, ctypes.c_size_t, ctypes.c_void_p]),
    "gslm_rasterize_loss_slot": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64, ctypes.c_void_p,
                                                ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64,
                                                ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int32,
                                                ctypes.c_void_p]),
    "gslm_loss_sets_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "gslm_rasterize_loss_sets": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int64,
                                                ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, ctypes.c_int32,
                                                ctypes.c_size_t,
                                                ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, ctypes.c_void_p]),
    "gslm_forward": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians), ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "gslm_backward": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians), ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(GslmGrads), ctypes.c_void_p]),
    "gslm_jvp": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians),
                                ctypes.POINTER(GslmGaussians), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_matvec_view": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians),
                                        ctypes.POINTER(GslmGrads), ctypes.c_void_p, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(GslmGrads),
                                        ctypes.c_void_p]),
    "gslm_matvec_view_ex": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians),
                                           ctypes.POINTER(GslmGrads), ctypes.c_void_p, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(GslmGrads),
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_sh_rest_project": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.POINTER(GslmGaussians), ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p]),
    "gslm_rest_basis": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int32, ctypes.POINTER(GslmGaussians),
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_rest_coords": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int32, ctypes.POINTER(GslmGaussians),
                                        ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "gslm_gather_screen": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int32, ctypes.POINTER(GslmGaussians),
                                          ctypes.c_void_p, ctypes.POINTER(GslmGrads), ctypes.POINTER(GslmGrads),
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_view_flags": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_tangent_views": (ctypes.c_int, [ctypes.POINTER(GslmView), ctypes.c_int32, ctypes.POINTER(GslmGaussians),
                                          ctypes.POINTER(GslmGrads), ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_cg_update": (ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_cg_update_monitor": (ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_cg_monitor": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    "gslm_dot_finalize": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_dot_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "gslm_dot": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                ctypes.POINTER(ctypes.c_double), ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_axpy_dev": (ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_xpby_dev": (ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_damp_add": (ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                                     ctypes.POINTER(ctypes.c_double), ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p]),
    "gslm_comm_id_bytes": (ctypes.c_int32, []),
    "gslm_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "gslm_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(ctypes.c_void_p)]),
    "gslm_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "gslm_allreduce_sum_f32": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "gslm_allreduce_sum_f64": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "gslm_alltoall": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_void_p]),
    "gslm_allgather": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_void_p]),
    "gslm_residual_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "gslm_lm_residual": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int32,
                                        ctypes.c_void_p]),
    "gslm_ssim_state_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "gslm_ssim_residual": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int32, ctypes.c_void_p]),
    "gslm_ssim_normal": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_ssim_mean_state_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "gslm_ssim_mean": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_ssim_mean_backward": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p]),
    "gslm_knn_scratch_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "gslm_knn3_mean_dist": (ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p]),
    "gslm_adam_step": (ctypes.c_int, [ctypes.POINTER(GslmAdamGroup), ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_void_p]),
    "gslm_densify_stats": (ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_inspect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p]),
    "gslm_selftest": (ctypes.c_int, [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_selftest_scan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "gslm_last_error": (ctypes.c_char_p, []),
    "gslm_abi_version": (ctypes.c_int, []),
}


ABI_VERSION = 9  # GSLM_ABI_VERSION of include/gslm.h these structs mirror


class GslmError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libgslm.so not found at {LIB_PATH}: build it with "
                          f"`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    ab_mode = os.environ.get("GSLM_ABI_ANY") == "1" and "GSLM_LIB" in os.environ and LIB_PATH != _DEFAULT_LIB
    for name, (restype, argtypes) in EXPORTS.items():
        if ab_mode and not hasattr(lib, name):
            continue  # an older A/B build without this entry point (only the A/B tools load those)
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    if lib.gslm_abi_version() != ABI_VERSION:
        # GSLM_ABI_ANY=1 with an explicit GSLM_LIB (the A/B tools timing an older build whose structs are
        # unchanged): accepted with a warning.  Never for the in-tree product library.
        if not (os.environ.get("GSLM_ABI_ANY") == "1" and "GSLM_LIB" in os.environ and LIB_PATH != _DEFAULT_LIB):
            raise ImportError(f"{LIB_PATH} has C ABI version {lib.gslm_abi_version()}, these bindings need "
                              f"{ABI_VERSION}: rebuild it")
        import warnings
        warnings.warn(f"gslm: GSLM_ABI_ANY=1 loads {LIB_PATH} (ABI {lib.gslm_abi_version()}) into ABI "
                      f"{ABI_VERSION} bindings: A/B timing only, struct layouts are not checked", RuntimeWarning)
    return lib


lib = _load()


def check(status, what=""):
    if status != GSLM_OK:
        msg = lib.gslm_last_error().decode(errors="replace")
        raise GslmError(f"{what or 'gslm'} failed ({status}): {msg}")


def ptr(t):
    """Device pointer of a tensor (or None -> NULL).  Tensors must be fp32/int32 contiguous."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None):
    return torch.cuda.current_stream(device).cuda_stream


# Host copies of settings tensors (viewmatrix, projmatrix, campos, bg): a device tensor costs a device-to-host copy and
# a stream synchronisation per read, and the drop-in Function reads the settings in its forward, backward and jvp.  A
# camera's matrices are the same tensors call after call, so the copy is cached per tensor object, valid while the
# tensor lives at the same version (any in-place write bumps it).
# The key is the tensor object, its storage address and its version counter.  A write that bypasses the version counter
# (through `t.data`, or an alias with a counter of its own) is not seen: set_host_cache(False) (or GSLM_HOST_CACHE=0)
# turns the cache off for code that moves cameras that way (the reference never does: its Camera matrices are built
# once, scene/cameras.py:80-89), and clear_host_cache() drops every entry.
_HOST_CACHE = {}
_HOST_CACHE_ON = [os.environ.get("GSLM_HOST_CACHE", "1") != "0"]


def set_host_cache(enabled):
    _HOST_CACHE_ON[0] = bool(enabled)
    if not enabled:
        _HOST_CACHE.clear()


def clear_host_cache():
    _HOST_CACHE.clear()


def _host_floats(t, n):
    if isinstance(t, torch.Tensor):
        hit = _HOST_CACHE.get(id(t)) if _HOST_CACHE_ON[0] else None
        if (hit is not None and hit[0]() is t and hit[1] == t._version and hit[2] == n and
                hit[4] == t.data_ptr()):
            return hit[3]
        vals = [float(x) for x in t.detach().reshape(-1).to("cpu", torch.float32).tolist()][:n]
        if t.is_cuda and _HOST_CACHE_ON[0]:
            import weakref
            key = id(t)
            try:
                ref = weakref.ref(t, lambda _r, key=key: _HOST_CACHE.pop(key, None))
            except TypeError:
                return vals
            _HOST_CACHE[key] = (ref, t._version, n, vals, t.data_ptr())
        return vals
    return [float(x) for x in list(t)][:n]


def make_view(H, W, tanfovx, tanfovy, bg, scale_modifier, viewmatrix, projmatrix, sh_degree, campos,
              prefiltered=False, antialiasing=False, debug=False):
    v = GslmView()
    v.image_height, v.image_width = int(H), int(W)
    v.tanfovx, v.tanfovy, v.scale_modifier = float(tanfovx), float(tanfovy), float(scale_modifier)
    v.viewmatrix[:] = _host_floats(viewmatrix, 16)
    v.projmatrix[:] = _host_floats(projmatrix, 16)
    v.campos[:] = _host_floats(campos, 3)
    v.bg[:] = _host_floats(bg, 3)
    v.sh_degree = int(sh_degree)
    v.prefiltered, v.antialiasing, v.debug = int(bool(prefiltered)), int(bool(antialiasing)), int(bool(debug))
    return v


def view_from_settings(s):
    """GaussianRasterizationSettings -> GslmView (gaussian_renderer/__init__.py:36-50 field names)."""
    return make_view(s.image_height, s.image_width, s.tanfovx, s.tanfovy, s.bg, s.scale_modifier,
                     s.viewmatrix, s.projmatrix, s.sh_degree, s.campos, s.prefiltered, s.antialiasing, s.debug)


def view_from_camera(cam, bg, sh_degree, scale_modifier=1.0, antialiasing=False):
    """The settings render() builds from a Camera (gaussian_renderer/__init__.py:33-50)."""
    return make_view(cam.image_height, cam.image_width, math.tan(cam.FoVx * 0.5), math.tan(cam.FoVy * 0.5),
                     bg, scale_modifier, cam.world_view_transform, cam.full_proj_transform, sh_degree,
                     cam.camera_center, antialiasing=antialiasing)


def make_gaussians(P, means3D=None, opacities=None, scales=None, rotations=None, cov3D=None, sh_dc=None,
                   sh_dc_stride=0, sh_rest=None, sh_rest_stride=0, max_coeffs=1, colors=None, raw=False):
    g = GslmGaussians()
    g.P = int(P)
    g.max_coeffs = int(max_coeffs)
    g.raw = int(bool(raw))
    g.means3D, g.opacities, g.scales = ptr(means3D), ptr(opacities), ptr(scales)
    g.rotations, g.cov3D_precomp = ptr(rotations), ptr(cov3D)
    g.sh_dc, g.sh_dc_stride = sh_dc, int(sh_dc_stride)
    g.sh_rest, g.sh_rest_stride = sh_rest, int(sh_rest_stride)
    g.colors_precomp = ptr(colors)
    return g


def sh_pointers(shs=None, dc=None, rest=None):
    """(dc_ptr, dc_stride, rest_ptr, rest_stride, K) for a [P,K,3] shs tensor or a (dc, rest) pair."""
    if shs is not None:
        K = shs.shape[1]
        base = shs.data_ptr()
        return base, 3 * K, (base + 12 if K > 1 else None), 3 * K, K
    if dc is not None:
        K = 1 + (rest.shape[1] if rest is not None else 0)
        return dc.data_ptr(), 3, (rest.data_ptr() if rest is not None and K > 1 else None), 3 * (K - 1), K
    return None, 0, None, 0, 1


def make_grads(means2D=None, means3D=None, opacities=None, scales=None, rotations=None, cov3D=None,
               sh=None, dc=None, rest=None, colors=None, accumulate=False):
    g = GslmGrads()
    g.means2D, g.means3D, g.opacities = ptr(means2D), ptr(means3D), ptr(opacities)
    g.scales, g.rotations, g.cov3D, g.colors = ptr(scales), ptr(rotations), ptr(cov3D), ptr(colors)
    dcp, dcs, rp, rs, _ = sh_pointers(sh, dc, rest)
    g.sh_dc, g.sh_dc_stride, g.sh_rest, g.sh_rest_stride = dcp, dcs, rp, rs
    g.accumulate = int(bool(accumulate))
    return g


def u8(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
