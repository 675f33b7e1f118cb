"""Flat param-space layout of a GaussianModelState (solver/gaussian_model_state.py:162-172).

Group order xyz, features_dc, features_rest, scaling, rotation, opacity, exposure; each group is
the row-major [P, width] tensor of the reference, so `as_1d_tensor()` of the reference and our flat
device buffer are the same bytes and group views are zero-copy.
"""
import ctypes

import torch

GROUPS = ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure")


class ParamLayout:
    """rest_projected: the SH-rest group holds 3 floats per Gaussian -- its coordinates along one view's unit
    basis direction (GSLM_MV_SH_REST_PROJECTED, gslm_sh_rest_project) -- instead of 3(K-1).
    rest_views = V > 0: the SH-rest group holds 3 V floats per Gaussian, its coordinates in an orthonormal basis
    of the V views' SH-rest directions (the Gaussian-sharded exchange, gslm_rest_basis / gslm_rest_coords)."""

    def __init__(self, P, sh_coeffs, n_exposure=1, rest_projected=False, rest_views=0):
        self.P, self.K, self.n_exposure = int(P), int(sh_coeffs), int(n_exposure)
        K = self.K
        self.rest_projected = bool(rest_projected) and K > 1
        self.rest_views = int(rest_views) if K > 1 else 0
        if self.rest_projected and self.rest_views:
            raise ValueError("rest_projected and rest_views are exclusive")
        rest_rows = self.rest_views or (1 if self.rest_projected else K - 1)
        self.rest_rows = rest_rows
        self.shapes = {
            "xyz": (P, 3), "features_dc": (P, 1, 3), "features_rest": (P, rest_rows, 3), "scaling": (P, 3),
            "rotation": (P, 4), "opacity": (P, 1), "exposure": (n_exposure, 3, 4)}
        self.offsets, off = {}, 0
        for g in GROUPS:
            n = 1
            for s in self.shapes[g]:
                n *= s
            self.offsets[g] = (off, off + n)
            off += n
        self.numel = off

    @property
    def floats_per_gaussian(self):
        """F = 11 + 3K: xyz 3, dc 3, rest 3(K-1), scaling 3, rotation 4, opacity 1 (17 when projected, 14 + 3V
        in rest_views coordinates)."""
        return 14 + 3 * self.rest_rows if self.K > 1 else 14

    def views(self, flat):
        """dict group -> view of the flat tensor with the reference shape."""
        return {g: flat[a:b].view(self.shapes[g]) for g, (a, b) in self.offsets.items()}

    def bounds(self):
        return [self.offsets[g][0] for g in GROUPS] + [self.numel]

    def group_damp_arrays(self, damp):
        """(int64[8], double[7]) host arrays for the gslm_dot / gslm_damp_add group weights.
        damp: mapping group -> scalar (GaussianModelDampMatrix fields) or a scalar."""
        vals = []
        for g in GROUPS:
            if isinstance(damp, (int, float)):
                vals.append(float(damp))
            elif isinstance(damp, dict):
                vals.append(float(damp[g]))
            else:
                vals.append(float(getattr(damp, g + "_damp")))
        b = (ctypes.c_int64 * 8)(*self.bounds())
        d = (ctypes.c_double * 7)(*vals)
        return b, d

    def grads_struct(self, flat, accumulate=False):
        """gslm_grads whose group pointers point into the flat vector (raw-parameter groups)."""
        from gslm import _lib
        base = flat.data_ptr()
        f = 4
        g = _lib.GslmGrads()
        g.means2D = None
        g.means3D = base + f * self.offsets["xyz"][0]
        g.opacities = base + f * self.offsets["opacity"][0]
        g.scales = base + f * self.offsets["scaling"][0]
        g.rotations = base + f * self.offsets["rotation"][0]
        g.cov3D = None
        g.sh_dc = base + f * self.offsets["features_dc"][0]
        g.sh_dc_stride = 3
        g.sh_rest = (base + f * self.offsets["features_rest"][0]) if self.K > 1 else None
        g.sh_rest_stride = 3 * self.rest_rows
        g.colors = None
        g.accumulate = int(bool(accumulate))
        return g


def raw_gaussians(model):
    """gslm_gaussians over the GaussianModel leaves (raw = 1: activations fused into the kernels)."""
    from gslm import _lib
    P = model._xyz.shape[0]
    K = 1 + model._features_rest.shape[1]
    for t in (model._xyz, model._features_dc, model._features_rest, model._scaling, model._rotation, model._opacity):
        assert t.is_contiguous() and t.dtype == torch.float32, "GaussianModel leaves must be contiguous fp32"
    return _lib.make_gaussians(
        P, model._xyz, model._opacity, model._scaling, model._rotation, None,
        model._features_dc.data_ptr(), 3, model._features_rest.data_ptr() if K > 1 else None, 3 * (K - 1), K,
        None, raw=True)
