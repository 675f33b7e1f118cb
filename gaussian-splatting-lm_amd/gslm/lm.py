"""Matrix-free Levenberg-Marquardt on the HIP rasterizer: the hot path of train_jvp.py's LM branch.

Reference semantics:
  * residual (batch_training_loss.py:10-17, disable_ssim=True):  r_b = m_b * clamp01(R_b) - gt_b, and
    the "ssim" slot aliases r, so the residual vector is [r; r]: loss = 2 ||r||^2, J^T J = 2 J_r^T J_r.
  * cgls_damped (conjugate_gradient.py:51-127) solves (J^T J + D) x = J^T b with b = -[r; r]
    (train_jvp.py:243), D the per-group diagonal of GaussianModelDampMatrix (train_jvp.py:229-235),
    xyz frozen by the param mask (train_jvp.py:221-227).
  * line search: alpha = 2, 1, ..., 1/16 on the validation views, keep the best (train_jvp.py:264-279).

MI355X design: the operator A = J^T J + D is applied by one fused HIP pass per view (gslm_matvec_view:
tangent preprocess -> JVP tile pass -> weight -> VJP tile pass -> gather-sum preprocess backward) on
geometry cached once per LM step (the sort is not redone per matvec).  CG runs on flat param-space
vectors with its scalars in device memory (gslm_dot / gslm_axpy_dev / gslm_xpby_dev): with
`check=False` an iteration has no host synchronisation at all.  CGLS on (J, D) and CG on A generate
the same iterates in exact arithmetic; the reference's restart schedule and stopping tests are kept.
"""
import ctypes
import math
import os

import torch

from gslm import _lib
from gslm._lib import check, lib
from gslm.params import GROUPS, ParamLayout, raw_gaussians

# train_jvp.py:229-235
STAGE_ALL = 7
STAGE_OVERWRITE = 8
MV_TAIL_CLEAN = 1  # gslm_matvec_opts.flags: GSLM_MV_TAIL_CLEAN
MV_SH_REST_PROJECTED = 2  # GSLM_MV_SH_REST_PROJECTED

DEFAULT_DAMP = {"xyz": 5e2, "features_dc": 5e-2, "features_rest": 5e-2, "scaling": 5e-2, "rotation": 5e-2,
                "opacity": 5e-2, "exposure": 1e1}


class ViewRaster:
    """Primal forward of one view on raw GaussianModel leaves + the buffers the matvec reuses."""

    def __init__(self, view, device):
        self.view = view
        self.H, self.W = view.image_height, view.image_width
        self.device = device
        self.N = 0
        self.geom = self.binning = self.image = self.scratch = None
        # the scratch's gradient rows of never-blended entries hold the zeros of an earlier fused
        # product on the current geometry (GSLM_MV_TAIL_CLEAN): false after a forward or a backward
        self.tail_clean = False

    def forward(self, g, stream, want_invdepth=True):
        """The full forward (the drop-in's gslm_preprocess + gslm_rasterize).  want_invdepth=False: the LM paths,
        which never read the inverse depth -- the blend then skips its accumulation (and its image)."""
        P = g.P
        dev = self.device
        self.tail_clean = False
        if self.geom is None or self.geom.numel() < lib.gslm_geom_bytes(P):
            self.geom = _lib.u8(lib.gslm_geom_bytes(P), dev)
            self.image = _lib.u8(lib.gslm_image_bytes(self.H, self.W), dev)
            self.color = torch.empty(3, self.H, self.W, dtype=torch.float32, device=dev)
            self.invdepth = torch.empty(1, self.H, self.W, dtype=torch.float32, device=dev)
            self.radii = torch.empty(P, dtype=torch.int32, device=dev)
        check(lib.gslm_preprocess(ctypes.byref(self.view), ctypes.byref(g), self.geom.data_ptr(), self.geom.numel(),
                                  self.radii.data_ptr(), stream), "gslm_preprocess")
        n = ctypes.c_int64(0)
        check(lib.gslm_num_rendered(self.geom.data_ptr(), P, ctypes.byref(n), stream), "gslm_num_rendered")
        self.N = int(n.value)
        need = lib.gslm_binning_bytes(self.N, self.H, self.W)
        if self.binning is None or self.binning.numel() < need:
            self.binning = _lib.u8(int(need * 1.25) + 4096, dev)
        check(lib.gslm_rasterize(ctypes.byref(self.view), P, self.geom.data_ptr(), self.binning.data_ptr(),
                                 self.binning.numel(), self.N, self.image.data_ptr(), self.image.numel(),
                                 self.color.data_ptr(), self.invdepth.data_ptr() if want_invdepth else None, stream),
              "gslm_rasterize")
        need = lib.gslm_scratch_bytes(P, self.N)
        if self.scratch is None or self.scratch.numel() < need:
            self.scratch = _lib.u8(int(need * 1.25) + 4096, dev)
        return self.color


    def forward_dev(self, g, stream, want_invdepth=True, n_out=None):
        """forward() without the pair-count read-back between the preprocess and the binning (gslm_rasterize_dev):
        the binning workspace of an earlier forward() is used as a list of its capacity, the count stays on the
        device, and n_out (device or pinned uint32 address, or None) receives it in stream order.  The image is valid
        when the count fits `capacity()`.  The binning then serves this render only: an LM product on this view needs
        a forward() first (self.N is None until then)."""
        if self.binning is None or self.geom is None or self.geom.numel() < lib.gslm_geom_bytes(g.P):
            raise RuntimeError("forward_dev: the workspaces of an earlier forward() at this P are required")
        P = g.P
        self.tail_clean = False
        self.N = None
        check(lib.gslm_preprocess(ctypes.byref(self.view), ctypes.byref(g), self.geom.data_ptr(), self.geom.numel(),
                                  self.radii.data_ptr(), stream), "gslm_preprocess")
        check(lib.gslm_rasterize_dev(ctypes.byref(self.view), P, self.geom.data_ptr(), self.binning.data_ptr(),
                                     self.binning.numel(), self.image.data_ptr(), self.image.numel(),
                                     self.color.data_ptr(), self.invdepth.data_ptr() if want_invdepth else None,
                                     n_out, stream), "gslm_rasterize_dev")
        return self.color

    def capacity(self):
        """List capacity of the binning workspace (forward_dev renders at most this many pairs)."""
        return 0 if self.binning is None else int(lib.gslm_binning_capacity(self.binning.numel(), self.H, self.W))


class LMProblem:
    """The LM normal equations of one camera batch (one LM step's worth of cached geometry)."""

    def __init__(self, model, cams, bg, gts=None, alpha_masks=None, mask_xyz=True, damp=None, device="cuda",
                 ssim=False, lambda_dssim=0.2, sh_projection=False):
        """ssim=False: the residual train_jvp.py uses (disable_ssim=True, [r; r]); ssim=True: the
        [r1; r2] residual with the SSIM term (batch_training_loss.py:18-30, gslm_ssim_*).

        sh_projection: param-space vectors carry the SH-rest group as 3 coordinates per Gaussian along the
        view's unit basis direction (GSLM_MV_SH_REST_PROJECTED; one view only -- with one view the CG
        iterates of (J^T J + D) x = J^T b never leave that span).  True / False / "auto" (= one camera and
        SH degree > 0).  `expand` / `project` convert to and from the reference's layout (`full_layout`)."""
        self.model = model
        self.ssim, self.lambda_dssim = bool(ssim), float(lambda_dssim)
        if self.ssim and not mask_xyz:
            raise ValueError("the SSIM residual path runs on the LM rows (mask_xyz=True, train_jvp.py:221-227)")
        self.cams = cams
        self.device = device
        self.bg = bg
        self.mask_xyz = bool(mask_xyz)
        P = model._xyz.shape[0]
        K = 1 + model._features_rest.shape[1]
        if sh_projection == "auto":
            sh_projection = len(cams) == 1 and K > 1 and model.active_sh_degree > 0
        if sh_projection and len(cams) != 1:
            raise ValueError("sh_projection is a single-view mode (the Krylov space of one view's J)")
        self.full_layout = ParamLayout(P, K, model._exposure.shape[0])
        self.layout = ParamLayout(P, K, model._exposure.shape[0], rest_projected=bool(sh_projection))
        self.mv_flags = MV_SH_REST_PROJECTED if self.layout.rest_projected else 0
        self.damp = DEFAULT_DAMP if damp is None else damp
        self._bounds, self._damps = self.layout.group_damp_arrays(self.damp)
        self.gts = [c.original_image.to(device) for c in cams] if gts is None else gts
        self.masks = [c.alpha_mask.to(device) for c in cams] if alpha_masks is None else alpha_masks
        self.views = [ViewRaster(_lib.view_from_camera(c, bg, model.active_sh_degree), device) for c in cams]
        self.stream = _lib.stream_handle(device)
        # >= 3 x 1024 doubles: gslm_cg_update_monitor's three partial sums
        self.dot_scratch = torch.empty(max(lib.gslm_dot_scratch_bytes(max(P, self.layout.numel)) // 8, 3 * 1024) + 8,
                                       dtype=torch.float64, device=device)
        self.weights = [None] * len(cams)
        self.residuals = [None] * len(cams)
        self.seeds = [None] * len(cams)
        self.ssim_state = [None] * len(cams)
        self._jv = [None] * len(cams)
        self._u = [None] * len(cams)
        self.res_scratch = torch.empty(lib.gslm_residual_scratch_bytes(1, 1) // 8, dtype=torch.float64,
                                       device=device)

    # -------------------------------------------------------------- residual (A8)
    def evaluate(self):
        """Primal forward of every view; residuals, per-pixel weights and the J^T b seeds from one fused
        epilogue per view (gslm_lm_residual); loss = 2 sum ||r||^2 (device double)."""
        g = raw_gaussians(self.model)
        loss = torch.zeros((), dtype=torch.float64, device=self.device)
        for b, vr in enumerate(self.views):
            R = vr.forward(g, self.stream, want_invdepth=False)
            if self.residuals[b] is None or self.residuals[b].shape != R.shape:
                self.residuals[b] = torch.empty_like(R)
                self.weights[b] = torch.empty_like(R)
                self.seeds[b] = torch.empty_like(R)
            m = self.masks[b]
            gt = self.gts[b]
            if m is not None:
                m = m.to(torch.float32).contiguous()
                if m.numel() != vr.H * vr.W:
                    raise ValueError("alpha mask must be [1, H, W]")
            if gt.shape != R.shape or gt.dtype != torch.float32:
                raise ValueError(f"ground truth must be float32 {tuple(R.shape)}, got {gt.dtype} {tuple(gt.shape)}")
            gt = gt.contiguous()
            if self.ssim:
                if self.ssim_state[b] is None:
                    self.ssim_state[b] = _lib.u8(lib.gslm_ssim_state_bytes(vr.H, vr.W), self.device)
                    self._jv[b] = torch.empty_like(R)
                    self._u[b] = torch.empty_like(R)
                st = self.ssim_state[b]
                check(lib.gslm_ssim_residual(vr.H, vr.W, R.data_ptr(), gt.data_ptr(),
                                             None if m is None else m.data_ptr(), self.lambda_dssim, st.data_ptr(),
                                             st.numel(), None, None, self.seeds[b].data_ptr(), loss.data_ptr(),
                                             int(b > 0), self.stream), "gslm_ssim_residual")
                continue
            check(lib.gslm_lm_residual(vr.H, vr.W, R.data_ptr(), gt.data_ptr(), None if m is None else m.data_ptr(),
                                       self.residuals[b].data_ptr(), self.weights[b].data_ptr(),
                                       self.seeds[b].data_ptr(), self.res_scratch.data_ptr(),
                                       self.res_scratch.numel() * 8, loss.data_ptr(), int(b > 0), self.stream),
                  "gslm_lm_residual")
        self.loss = loss
        return loss

    def num_rendered(self):
        return [v.N for v in self.views]

    # -------------------------------------------------------------- J^T b
    def rhs(self, out, fused=True):
        """out = J^T b = -2 sum_b J_b^T (m (.) 1[0<=R<=1] (.) r_b) in the flat layout (xyz, exposure zeroed).

        fused: the LM path -- a back-to-front pass seeded with gslm_lm_residual's seed into the LM
        rows, then the LM gather (gslm_matvec_view_ex with pixel_seed); otherwise the drop-in
        gslm_backward (general rows, every parameter group)."""
        g = raw_gaussians(self.model)
        if fused and self.mask_xyz:
            ys = self.layout.grads_struct(out)
            for b, vr in enumerate(self.views):
                opts = _lib.GslmMatvecOpts()
                opts.stages = 2 | 4 | (STAGE_OVERWRITE if b == 0 else 0)  # RENDER | GATHER
                opts.flags = (MV_TAIL_CLEAN if vr.tail_clean else 0) | self.mv_flags
                opts.pixel_seed = self.seeds[b].data_ptr()
                check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(ys),
                                              self.seeds[b].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                              vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                              ctypes.byref(ys), ctypes.byref(opts), self.stream), "gslm_matvec_view_ex")
                vr.tail_clean = True
            if not self.views:
                out.zero_()
            e0, e1 = self.layout.offsets["exposure"]
            out[e0:e1].zero_()
            return self._mark_rhs(out)
        if self.layout.rest_projected:
            full = torch.zeros(self.full_layout.numel, dtype=torch.float32, device=self.device)
            self.rhs_full(full)
            return self._mark_rhs(self.project(full, out))
        return self._mark_rhs(self.rhs_full(out))

    def _mark_rhs(self, out):
        """Remember the J^T b this problem produced (exposure slice zeroed): cgls_fused may then skip the exposure
        slice's D v in every product without checking it (exposure_is_zero)."""
        self._rhs_token = (out.data_ptr(), out._version)
        return out

    def exposure_is_zero(self, g):
        """Whether the exposure slice of the right-hand side g is zero, so that every CG iterate's is (J has no
        exposure column): true without a device read for the rhs() this problem produced and nobody modified
        since; otherwise checked on the device (one host sync per solve)."""
        if getattr(self, "_rhs_token", None) == (g.data_ptr(), g._version):
            return True
        e0, e1 = self.layout.offsets["exposure"]
        return not bool(g[e0:e1].any())

    def rhs_full(self, out):
        """J^T b through the drop-in gslm_backward, in the reference's layout (full_layout)."""
        g = raw_gaussians(self.model)
        out.zero_()
        grads = self.full_layout.grads_struct(out, accumulate=True)
        for b, vr in enumerate(self.views):
            dL = self.seeds[b]  # -2 m 1[0 <= R <= 1] r, from gslm_lm_residual
            check(lib.gslm_backward(ctypes.byref(vr.view), ctypes.byref(g), vr.geom.data_ptr(), vr.binning.data_ptr(),
                                    vr.N, vr.image.data_ptr(), dL.data_ptr(), None, vr.scratch.data_ptr(),
                                    vr.scratch.numel(), ctypes.byref(grads), self.stream), "gslm_backward")
            vr.tail_clean = False
        self._apply_mask(out, self.full_layout)
        return out

    # -------------------------------------------------------------- SH-rest projection (sh_projection)
    def _rest_convert(self, mode, src, dst, src_layout, dst_layout):
        if self.layout.K < 2:
            return
        g = raw_gaussians(self.model)
        a0 = src_layout.offsets["features_rest"][0]
        b0 = dst_layout.offsets["features_rest"][0]
        src_w = 3 * src_layout.shapes["features_rest"][1]
        dst_w = 3 * dst_layout.shapes["features_rest"][1]
        check(lib.gslm_sh_rest_project(ctypes.byref(self.views[0].view), ctypes.byref(g), mode,
                                       src.data_ptr() + 4 * a0, src_w, dst.data_ptr() + 4 * b0, dst_w, self.stream),
              "gslm_sh_rest_project")

    def _copy_other_groups(self, src, dst, src_layout, dst_layout):
        for name in GROUPS:
            if name == "features_rest":
                continue
            a0, a1 = src_layout.offsets[name]
            b0, b1 = dst_layout.offsets[name]
            dst[b0:b1].copy_(src[a0:a1])

    def expand(self, x, out=None):
        """A vector of this problem's layout in the reference's (full_layout); x itself when not projected."""
        if not self.layout.rest_projected:
            return x
        out = torch.empty(self.full_layout.numel, dtype=torch.float32, device=x.device) if out is None else out
        self._copy_other_groups(x, out, self.layout, self.full_layout)
        self._rest_convert(0, x, out, self.layout, self.full_layout)
        return out

    def project(self, x_full, out=None):
        """full_layout -> this problem's layout (the orthogonal projection onto the view's SH-rest span)."""
        if not self.layout.rest_projected:
            return x_full if out is None else out.copy_(x_full)
        out = torch.empty(self.layout.numel, dtype=torch.float32, device=x_full.device) if out is None else out
        self._copy_other_groups(x_full, out, self.full_layout, self.layout)
        self._rest_convert(1, x_full, out, self.full_layout, self.layout)
        return out

    def _apply_mask(self, vec, layout=None):
        o = (layout or self.layout).offsets
        if self.mask_xyz:
            vec[o["xyz"][0]:o["xyz"][1]].zero_()
        vec[o["exposure"][0]:o["exposure"][1]].zero_()

    # -------------------------------------------------------------- (J^T J + D) v
    def matvec(self, v, y, cg_ctl=None):
        """y = sum_b 2 J_b^T W_b J_b v + D v (fused per view; D v folded into the first view's gather)."""
        self.matvec_dot(v, y, None, cg_ctl=cg_ctl)
        return y

    # cgls_fused may pass exposure_zero=True (see matvec_dot) and the device CG control block (cg_ctl)
    supports_exposure_zero = True
    supports_cg_ctl = True

    def matvec_dot(self, v, y, dot_out, pre=None, exposure_zero=False, cg_ctl=None):
        """matvec, and when possible <v, y> -> device double* dot_out fused into the gather (single
        view; exposure components of v zero, as in every LM iterate).  Returns True if fused.
        pre = (s, beta_num_ptr, beta_den_ptr): first v <- s + beta v (the deferred CG direction
        update), fused into the first view's tangent kernel.
        exposure_zero: the caller guarantees that the exposure components of v (after pre) and of y are
        zero already -- true of every CG iterate (J has no exposure column, x0 = 0, y is the solver's own
        q) -- so y's exposure slice D v = 0 is left as it is (no elementwise launch per product).
        cg_ctl: device pointer of cgls_fused's CG control block (gslm_cg_monitor): once its stopping tests
        have fired the product's kernels return at once (gslm_matvec_opts.cg_ctl)."""
        fuse = dot_out is not None and len(self.views) == 1
        self.local_normal_matvec(v, y, damp=True, dot_out=dot_out if fuse else None, pre=pre,
                                 exposure_zero=exposure_zero, cg_ctl=cg_ctl)
        return fuse

    def local_normal_matvec(self, v, y, damp=False, dot_out=None, pre=None, exposure_zero=False, cg_ctl=None):
        """y = [D v +] sum over this problem's views of 2 J_b^T W_b J_b v  (overwrites y).
        pre, exposure_zero, cg_ctl: see matvec_dot."""
        g = raw_gaussians(self.model)
        vs = self.layout.grads_struct(v)
        ys = self.layout.grads_struct(y)
        if pre is not None and not self.views:
            self._pre_without_views(v, pre)
            pre = None
        if not self.views:
            y.zero_()
            if damp:
                self.damp_add(v, y)
            return y
        last = len(self.views) - 1
        e0, e1 = self.layout.offsets["exposure"]
        for b, vr in enumerate(self.views):
            opts = _lib.GslmMatvecOpts()
            opts.stages = STAGE_ALL | (STAGE_OVERWRITE if b == 0 else 0)
            opts.flags = (MV_TAIL_CLEAN if vr.tail_clean else 0) | self.mv_flags
            opts.damp7 = self._damps if (damp and b == 0) else None
            opts.cg_ctl = cg_ctl
            if pre is not None and b == 0:
                ss = self._pre_opts(opts, v, pre)  # noqa: F841  (kept alive for the call)
            if dot_out is not None and b == last:
                opts.dot_vy = dot_out
                opts.dot_scratch = self.dot_scratch.data_ptr()
                opts.dot_scratch_bytes = self.dot_scratch.numel() * 8
            if self.ssim:
                self._ssim_product(b, vr, g, vs, ys, opts)
                continue
            check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                          self.weights[b].data_ptr(), int(self.mask_xyz), vr.geom.data_ptr(),
                                          vr.binning.data_ptr(), vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(),
                                          vr.scratch.numel(), ctypes.byref(ys), ctypes.byref(opts), self.stream),
                  "gslm_matvec_view_ex")
            vr.tail_clean = True
        if exposure_zero:
            pass  # y[e0:e1] = D v[e0:e1] = 0 already (matvec_dot)
        elif damp:
            torch.mul(v[e0:e1], float(self._damps[6]), out=y[e0:e1])  # J has no exposure column
        else:
            y[e0:e1].zero_()
        return y

    # pre = (s, beta_num, beta_den[, x, alpha_num, alpha_den]): before the product, [x += alpha v then]
    # v = s + beta v -- the CG direction update (and the deferred x update) of the previous iteration
    def _pre_opts(self, opts, v, pre):
        s, num, den = pre[:3]
        e0, e1 = self.layout.offsets["exposure"]
        ss = self.layout.grads_struct(s)
        opts.xpby_s = ctypes.addressof(ss)
        opts.beta_num, opts.beta_den = num, den
        opts.xpby_tail_v = v.data_ptr() + 4 * e0
        opts.xpby_tail_s = s.data_ptr() + 4 * e0
        opts.xpby_tail_n = e1 - e0
        if len(pre) > 3 and pre[3] is not None:
            x, anum, aden = pre[3:]
            opts.alpha_num, opts.alpha_den = anum, aden
            opts.xpby_x_offset = x.data_ptr() - v.data_ptr()
        return ss

    def _pre_without_views(self, v, pre):
        s, num, den = pre[:3]
        if len(pre) > 3 and pre[3] is not None:
            x, anum, aden = pre[3:]
            check(lib.gslm_axpy_dev(v.numel(), anum, aden, 1.0, v.data_ptr(), x.data_ptr(), self.stream),
                  "gslm_axpy_dev")
        check(lib.gslm_xpby_dev(v.numel(), s.data_ptr(), num, den, v.data_ptr(), self.stream), "gslm_xpby_dev")

    def _ssim_product(self, b, vr, g, vs, ys, opts):
        """One view's J^T J v with the SSIM residual: J v (jv_out) -> image-space factor
        M (d1^2 + S^T c2^2 S) M (gslm_ssim_normal) -> seeded back-to-front pass + LM gather.
        opts carries this view's gather options (overwrite, damping, dot) and the fused xpby."""
        jv, u = self._jv[b], self._u[b]
        o1 = _lib.GslmMatvecOpts()
        o1.stages = 1 | 2  # TANGENT | RENDER
        o1.flags = self.mv_flags
        o1.jv_out = jv.data_ptr()
        o1.xpby_s, o1.beta_num, o1.beta_den = opts.xpby_s, opts.beta_num, opts.beta_den
        o1.xpby_tail_v, o1.xpby_tail_s, o1.xpby_tail_n = opts.xpby_tail_v, opts.xpby_tail_s, opts.xpby_tail_n
        o1.alpha_num, o1.alpha_den, o1.xpby_x_offset = opts.alpha_num, opts.alpha_den, opts.xpby_x_offset
        o1.cg_ctl = opts.cg_ctl
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs), jv.data_ptr(), 1,
                                      vr.geom.data_ptr(), vr.binning.data_ptr(), vr.N, vr.image.data_ptr(),
                                      vr.scratch.data_ptr(), vr.scratch.numel(), ctypes.byref(ys), ctypes.byref(o1),
                                      self.stream), "gslm_matvec_view_ex(jv)")
        check(lib.gslm_ssim_normal(vr.H, vr.W, self.gts[b].data_ptr(), self.ssim_state[b].data_ptr(), jv.data_ptr(),
                                   u.data_ptr(), self.stream), "gslm_ssim_normal")
        o2 = _lib.GslmMatvecOpts()
        o2.stages = 2 | 4 | (opts.stages & STAGE_OVERWRITE)  # RENDER | GATHER
        o2.flags = (MV_TAIL_CLEAN if vr.tail_clean else 0) | self.mv_flags
        o2.pixel_seed = u.data_ptr()
        o2.damp7 = opts.damp7
        o2.dot_vy, o2.dot_scratch, o2.dot_scratch_bytes = opts.dot_vy, opts.dot_scratch, opts.dot_scratch_bytes
        o2.cg_ctl = opts.cg_ctl
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs), u.data_ptr(), 1,
                                      vr.geom.data_ptr(), vr.binning.data_ptr(), vr.N, vr.image.data_ptr(),
                                      vr.scratch.data_ptr(), vr.scratch.numel(), ctypes.byref(ys), ctypes.byref(o2),
                                      self.stream), "gslm_matvec_view_ex(seed)")
        vr.tail_clean = True

    # -------------------------------------------------------------- view-sharded exchange (gslm.parallel)
    def views_for(self, cams, pad_to=None):
        """ctypes array of the gslm_view of every camera in `cams` (the whole sharded batch), padded
        with copies of the last to `pad_to` entries (padded slots carry no screen data)."""
        vs = [_lib.view_from_camera(c, self.bg, self.model.active_sh_degree) for c in cams]
        vs += [vs[-1]] * max(0, (pad_to or len(vs)) - len(vs))
        arr = (_lib.GslmView * len(vs))()
        for k, vw in enumerate(vs):
            arr[k] = vw
        return arr

    def screen_products(self, v, screen, pre=None, cg_ctl=None):
        """screen[b] = this rank's view b's per-Gaussian screen-space sums S_b^T W_b J_b v (P x 8,
        GSLM_STAGE_SCREEN); pre as in matvec_dot (applied with the first view)."""
        g = raw_gaussians(self.model)
        vs = self.layout.grads_struct(v)
        ys = self.layout.grads_struct(v)  # unused by the SCREEN stage
        e0, e1 = self.layout.offsets["exposure"]
        if pre is not None and not self.views:
            self._pre_without_views(v, pre)
        for b, vr in enumerate(self.views):
            opts = _lib.GslmMatvecOpts()
            opts.stages = 1 | 2 | 16  # TANGENT | RENDER | SCREEN
            opts.flags = MV_TAIL_CLEAN if vr.tail_clean else 0
            opts.screen_out = screen[b].data_ptr()
            opts.cg_ctl = cg_ctl
            if pre is not None and b == 0:
                ss = self._pre_opts(opts, v, pre)  # noqa: F841
            check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                          self.weights[b].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                          vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                          ctypes.byref(ys), ctypes.byref(opts), self.stream), "gslm_matvec_view_ex")
            vr.tail_clean = True

    def gather_screen(self, views, screen_all, v, y, dot_out=None, chunk=16):
        """y = sum over all views b of C_b^T screen_all[b] + D v (exposure: D v only); <v, y> fused
        into dot_out when given."""
        g = raw_gaussians(self.model)
        vs = self.layout.grads_struct(v)
        ys = self.layout.grads_struct(y)
        n = len(views)
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            opts = _lib.GslmMatvecOpts()
            opts.stages = (STAGE_ALL | STAGE_OVERWRITE) if c0 == 0 else STAGE_ALL
            opts.damp7 = self._damps if c0 == 0 else None
            if dot_out is not None and c1 == n:
                opts.dot_vy = dot_out
                opts.dot_scratch = self.dot_scratch.data_ptr()
                opts.dot_scratch_bytes = self.dot_scratch.numel() * 8
            vptr = ctypes.cast(ctypes.byref(views, c0 * ctypes.sizeof(_lib.GslmView)), ctypes.POINTER(_lib.GslmView))
            check(lib.gslm_gather_screen(vptr, c1 - c0, ctypes.byref(g), screen_all[c0].data_ptr(), ctypes.byref(vs),
                                         ctypes.byref(ys), ctypes.byref(opts), self.stream), "gslm_gather_screen")
        e0, e1 = self.layout.offsets["exposure"]
        torch.mul(v[e0:e1], float(self._damps[6]), out=y[e0:e1])  # J has no exposure column
        return y

    def damp_add(self, v, y):
        check(lib.gslm_damp_add(v.numel(), v.data_ptr(), self._bounds, self._damps, 7, y.data_ptr(), self.stream))

    # -------------------------------------------------------------- residual-space J and J^T (cgls_residual)
    def residual_masks(self):
        """Per view m (.) 1[0 <= R <= 1]: the Jacobian of r = m clamp01(R) - gt w.r.t. the render R."""
        out = []
        for b, vr in enumerate(self.views):
            R = vr.color
            inside = ((R >= 0) & (R <= 1)).to(torch.float32)
            m = self.masks[b]
            out.append(inside if m is None else inside * m.to(torch.float32).reshape(1, vr.H, vr.W))
        return out

    def jv_residual(self, v, rmasks, out):
        """out[b] = J_r,b v = m 1[0 <= R <= 1] (.) (d R_b / d theta) v  (the `matvec` of solver_functions.py:83-93,
        one copy of the [r; r] pair)."""
        if self.ssim:
            raise ValueError("jv_residual: the disable_ssim residual only")
        g = raw_gaussians(self.model)
        vs = self.layout.grads_struct(v)
        for b, vr in enumerate(self.views):
            opts = _lib.GslmMatvecOpts()
            opts.stages = 1 | 2  # TANGENT | RENDER with jv_out: the colour tangent
            opts.flags = self.mv_flags
            opts.jv_out = out[b].data_ptr()
            check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                          out[b].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(), vr.N,
                                          vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                          ctypes.byref(vs), ctypes.byref(opts), self.stream), "gslm_matvec_view_ex(jv)")
            out[b].mul_(rmasks[b])
        return out

    def jt_residual(self, r, rmasks, out):
        """out = J^T [r; r] = 2 sum_b J_r,b^T r_b (the `matvec_T` of solver_functions.py:101-132), xyz and exposure
        groups zero.  Overwrites out."""
        g = raw_gaussians(self.model)
        ys = self.layout.grads_struct(out)
        for b, vr in enumerate(self.views):
            seed = (2.0 * rmasks[b]) * r[b]
            opts = _lib.GslmMatvecOpts()
            opts.stages = 2 | 4 | (STAGE_OVERWRITE if b == 0 else 0)  # RENDER | GATHER, seeded
            opts.flags = (MV_TAIL_CLEAN if vr.tail_clean else 0) | self.mv_flags
            opts.pixel_seed = seed.data_ptr()
            check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(ys), seed.data_ptr(), 1,
                                          vr.geom.data_ptr(), vr.binning.data_ptr(), vr.N, vr.image.data_ptr(),
                                          vr.scratch.data_ptr(), vr.scratch.numel(), ctypes.byref(ys),
                                          ctypes.byref(opts), self.stream), "gslm_matvec_view_ex(seed)")
            vr.tail_clean = True
        if not self.views:
            out.zero_()
        self._apply_mask(out)
        return out

    # -------------------------------------------------------------- device scalar algebra
    def dot(self, a, b, out_slot, damped=False):
        if damped:
            check(lib.gslm_dot(a.data_ptr(), b.data_ptr(), self._bounds, self._damps, 7, a.numel(),
                               self.dot_scratch.data_ptr(), out_slot, self.stream))
        else:
            check(lib.gslm_dot(a.data_ptr(), b.data_ptr(), None, None, 0, a.numel(), self.dot_scratch.data_ptr(),
                               out_slot, self.stream))

    def zeros(self):
        return torch.zeros(self.layout.numel, dtype=torch.float32, device=self.device)


class NonFiniteError(AssertionError):
    """A NaN or Inf reached the normal equations.  The reference's only failure detection on the LM path is
    matvec_T's `assert not torch.isnan(self.gaussians._<group>.grad).any(), "NaN detected in gaussians._<group>.grad"`
    (solver/solver_functions.py:125-130), which aborts the step before the parameters move; this is raised at the
    same point of the fused solve (an AssertionError, with the reference's message), before update_params."""


CG_STOP_NONFINITE = 4  # gslm_cg_monitor's stop code (include/gslm.h GSLM_CG_STOP_NONFINITE)


def raise_nonfinite(prob, g, what="the normal-equations product (J^T J + D) p"):
    """Raises NonFiniteError naming the parameter groups of J^T b (= g) that hold a NaN / Inf, as the reference's
    asserts do; when J^T b is finite the failure came later in the solve (a product or the iterate)."""
    names = []
    try:
        for k, v in prob.layout.views(g).items():
            if k != "exposure" and v.numel() and not bool(torch.isfinite(v).all()):
                names.append(k)
    except (AttributeError, RuntimeError, TypeError):
        pass
    if names:
        raise NonFiniteError("; ".join(f"NaN detected in gaussians._{k}.grad" for k in names))
    raise NonFiniteError(f"NaN detected in {what} during CGLS (J^T b is finite)")


def cgls_fused(prob, g, max_iter=10, restart_iter=10, tol=1e-10, atol=0.0, check_every=True, verbose=False,
               callback=None, host_checks=None):
    """cgls_damped (conjugate_gradient.py:51-127) on the fused operator, x0 = 0.

    Returns (x, info).  check_every: the reference's stopping tests (delta < 1e-20, residual increase, gamma
    tolerance).  They run on the device by default (gslm_cg_monitor: a control block the update and product
    kernels test, one read-back at the end, no host synchronisation inside the loop -- the host enqueues the
    whole max_iter x restart_iter schedule and a stopped solve's remaining launches return at once);
    host_checks=True (or verbose / a callback, which need the values each iteration) reads the scalars back
    every iteration instead.  Both give the same iterates, stop and history.  With check_every=False the tests
    are skipped (benchmark mode); the iterates are identical while no test fires."""
    n = prob.layout.numel
    dev = prob.device
    st = prob.stream
    # With the xyz mask (train_jvp.py:221-227) the xyz group is zero in every iterate: the vector
    # updates and dots run on [lo, n) only (lo rounded down to a float4 boundary for the update kernel).
    lo = (3 * prob.layout.P // 4) * 4 if getattr(prob, "mask_xyz", False) else 0
    na = n - lo
    off = lambda t: t.data_ptr() + 4 * lo
    sc = torch.zeros(16, dtype=torch.float64, device=dev)
    ptr = lambda i: sc.data_ptr() + 8 * i
    GAM, GAMN, DEL, XG, XS = 0, 1, 2, 3, 4  # gamma / gamma' ping-pong between slots 0 and 1
    x = torch.zeros(n, dtype=torch.float32, device=dev)
    s = torch.empty_like(x)
    p = torch.empty_like(x)
    q = torch.zeros_like(x)
    if host_checks is None:
        host_checks = verbose or callback is not None
    on_device = check_every and not host_checks
    ctl = None
    if on_device:
        # [stop, iters, last_res, n_hist, history...] (gslm_cg_monitor)
        ctl = torch.full((4 + max_iter,), math.nan, dtype=torch.float64, device=dev)
        ctl[:4] = torch.tensor([0.0, 0.0, math.inf, 0.0], dtype=torch.float64)
        loss = prob.loss
        b2_dev = loss if (torch.is_tensor(loss) and loss.is_cuda and loss.dtype == torch.float64 and
                          loss.numel() == 1) else torch.tensor(float(loss), dtype=torch.float64, device=dev)
    cg_ctl = ctl.data_ptr() if ctl is not None else None
    ctl_kw = {"cg_ctl": cg_ctl} if (cg_ctl is not None and getattr(prob, "supports_cg_ctl", False)) else {}
    b2 = float(prob.loss) if (check_every and not on_device) else None  # ||b||^2 = loss
    iter_total, last_res, history = 0, math.inf, []
    # Benchmark mode defers x += alpha p into the next product's xpby pass (gslm_matvec_opts.alpha_num):
    # the update kernel then streams s and q only; the iterates are bitwise those of the undeferred loop.
    defer = not check_every and callback is None
    pend = None  # (alpha_num, alpha_den) of a deferred x update not yet applied
    # Gaussian-sharded operators (gslm.parallel.GaussianShardedOperator) hold a shard of every vector: each
    # dot / update pass leaves a per-shard partial that is summed over the ranks before it is used
    red = getattr(prob, "allreduce_scalars", None)

    def reduce(*slots):
        if red is not None:
            red(sc, slots)

    def flush():
        nonlocal pend
        if pend is not None:
            check(lib.gslm_axpy_dev(na, pend[0], pend[1], 1.0, off(p), off(x), st), "gslm_axpy_dev")
            pend = None

    # the products may leave y's exposure slice (D v there) unwritten only when g's is zero (exposure_zero)
    ez = {"exposure_zero": True} if (getattr(prob, "supports_exposure_zero", False) and
                                     prob.exposure_is_zero(g)) else {}
    first = True
    while iter_total < max_iter:
        if first:
            s.copy_(g)  # s0 = J^T b - D x0 with x0 = 0
            first = False
        else:
            flush()
            prob.matvec(x, q, **ctl_kw)
            torch.sub(g, q, out=s)
        p.copy_(s)
        prob.dot(s[lo:], s[lo:], ptr(GAM))
        reduce(GAM)
        stop = False
        pre = None
        for _ in range(restart_iter):
            # [p = s + beta p and the deferred x += alpha p, both fused into this product's tangent kernel]
            # q = A p and delta = <p, A p> (= |J p|^2 + p.D.p), fused into the gather when possible
            full = None if pre is None else pre + ((x, pend[0], pend[1]) if pend is not None else (None, None, None))
            if full is not None:
                pend = None
            # (q was allocated zero; with g's exposure slice zero every iterate's is: J has no exposure column
            # and x0 = 0)
            if not prob.matvec_dot(p, q, ptr(DEL), pre=full, **ez, **ctl_kw):
                prob.dot(p[lo:], q[lo:], ptr(DEL))
            reduce(DEL)
            if check_every and not on_device and not math.isfinite(sc[DEL].item()):
                raise_nonfinite(prob, g)
            if check_every and not on_device and sc[DEL].item() < 1e-20:
                if verbose:
                    print("Early termination: delta is too small.")
                stop = True
                break
            # [x += alpha p ;] s -= alpha q ; gamma' = <s, s> [; <x, g>, <x, s> for the monitor]  (one pass)
            if check_every:
                check(lib.gslm_cg_update_monitor(na, ptr(GAM), ptr(DEL), off(p), off(q), off(x), off(s), off(g),
                                                 prob.dot_scratch.data_ptr(), prob.dot_scratch.numel() * 8,
                                                 ptr(GAMN), ptr(XG), ptr(XS), cg_ctl, st))
                reduce(GAMN, XG, XS)
                if on_device:  # the stopping tests of :88-117 on the device (gslm_cg_monitor)
                    check(lib.gslm_cg_monitor(ptr(GAM), ptr(GAMN), ptr(DEL), ptr(XG), ptr(XS), b2_dev.data_ptr(),
                                              float(tol), float(atol), cg_ctl, max_iter, st), "gslm_cg_monitor")
            elif defer:
                check(lib.gslm_cg_update(na, ptr(GAM), ptr(DEL), off(p), off(q), None, off(s),
                                         prob.dot_scratch.data_ptr(), ptr(GAMN), st))
                pend = (ptr(GAM), ptr(DEL))  # alpha = gamma / delta, read before either slot is rewritten
                reduce(GAMN)
            else:
                check(lib.gslm_cg_update(na, ptr(GAM), ptr(DEL), off(p), off(q), off(x), off(s),
                                         prob.dot_scratch.data_ptr(), ptr(GAMN), st))
                reduce(GAMN)
            # beta = gamma' / gamma; after the slot swap below these are the GAM / GAMN slots
            pre = (s, ptr(GAMN), ptr(GAM))
            if check_every and not on_device:
                vals = sc[:5].tolist()
                if not all(math.isfinite(vals[k]) for k in (GAM, GAMN, XG, XS)):
                    raise_nonfinite(prob, g)
                res = b2 - vals[XG] - vals[XS]  # ||b - J x||^2 + x^T D x  (monitor of conjugate_gradient.py:103-104)
                history.append(res)
                if verbose:
                    print(f"[Iter {iter_total + 1}] res: {res:.2e}")
                if res > last_res:
                    stop = True
                    break
                last_res = res
                if vals[GAMN] < max(tol * math.sqrt(vals[GAM]), atol):
                    stop = True
                    break
            if callback is not None:
                callback(x, s, iter_total + 1)
            GAM, GAMN = GAMN, GAM
            iter_total += 1
            if iter_total >= max_iter:
                stop = True
                break
        if stop:
            break
    flush()
    if on_device:
        c = ctl.tolist()  # the solve's one read-back
        if int(c[0]) == CG_STOP_NONFINITE:  # (the monitor's inputs are all-reduced first: every rank raises here)
            raise_nonfinite(prob, g)
        iter_total, nh = int(c[1]), int(c[3])
        history = c[4:4 + min(nh, max_iter)]
        return x, {"iters": iter_total, "residuals": history, "stop": int(c[0])}
    return x, {"iters": iter_total, "residuals": history}


def cgls_residual(prob, max_iter=10, restart_iter=10, tol=1e-10, atol=0.0, verbose=False, callback=None):
    """cgls_damped (conjugate_gradient.py:51-127) in the reference's own recursion, on the HIP operator: residual-
    space r (one [3,H,W] image per view standing for the [r; r] pair, so its dots count twice), r -= alpha q with
    q = J p, a fresh s = J^T r - D x every iteration, and the residual monitor from a fresh J x -- two tangent
    passes and one seeded adjoint pass per iteration, where cgls_fused runs one fused (J^T J + D) p and updates s
    algebraically.  Equal iterates in exact arithmetic; this mode keeps long float32 solves on the reference's
    rounding path.  b = -[r; r] (train_jvp.py:243), x0 = 0.  Returns (x, info)."""
    if getattr(prob, "ssim", False):
        raise ValueError("cgls_residual: the disable_ssim residual only")
    dev = prob.device
    rm = prob.residual_masks()
    b = [-r for r in prob.residuals]  # b = -[r; r]: one copy per view

    def dot2(u, v):  # <[u; u], [v; v]> over the views, reduced in float64 on the device (the .item() of :138-146)
        return 2.0 * sum(float((a.double() * c.double()).sum()) for a, c in zip(u, v))

    n = prob.layout.numel
    dvec = torch.empty(n, dtype=torch.float64, device=dev)
    bounds = list(prob._bounds)
    for k in range(7):
        dvec[bounds[k]:bounds[k + 1]] = float(prob._damps[k])

    def ddot(u, v):  # dot(x, y, damp) of GaussianModelState (gaussian_model_state.py:262-269)
        return float((u.double() * v.double() * dvec).sum())

    def Dx(x):
        return (x.double() * dvec).to(torch.float32)

    jv = [torch.empty_like(t) for t in b]
    x = torch.zeros(n, dtype=torch.float32, device=dev)
    s = torch.empty_like(x)
    iter_total, last_res, history = 0, math.inf, []
    stop = False
    while iter_total < max_iter and not stop:
        prob.jv_residual(x, rm, jv)
        r = [bb - q for bb, q in zip(b, jv)]                         # r0 = b - A x0
        prob.jt_residual(r, rm, s)
        s -= Dx(x)                                                    # s0 = A^T r0 - D x0
        p = s.clone()
        gamma = float((s.double() * s.double()).sum())
        for _ in range(restart_iter):
            q = [t.clone() for t in prob.jv_residual(p, rm, jv)]      # q = A p
            delta = dot2(q, q) + ddot(p, p)
            if delta < 1e-20:
                if verbose:
                    print("Early termination: delta is too small.")
                stop = True
                break
            alpha = gamma / delta
            x += alpha * p
            r = [rr - alpha * qq for rr, qq in zip(r, q)]
            prob.jt_residual(r, rm, s)
            s -= Dx(x)                                                # s = A^T r - D x
            gamma_prev, gamma = gamma, float((s.double() * s.double()).sum())
            p = s + (gamma / gamma_prev) * p
            prob.jv_residual(x, rm, jv)
            cur = [bb - q for bb, q in zip(b, jv)]                   # cur_r = b - A x
            res = dot2(cur, cur) + ddot(x, x)
            history.append(res)
            if verbose:
                print(f"[Iter {iter_total + 1}] res: {res:.2e}")
            if res > last_res:
                stop = True
                break
            last_res = res
            if callback is not None:
                callback(x, s, iter_total + 1)
            if gamma < max(tol * math.sqrt(gamma_prev), atol):
                stop = True
                break
            iter_total += 1
            if iter_total >= max_iter:
                stop = True
                break
    return x, {"iters": iter_total, "residuals": history}


def loss_set_group():
    """Sets per blend pass of the line search (GSLM_LOSS_SET_GROUP, 1..8; default 1 = one pass per set).

    The variable was GSLM_LOSS_SETS until round 5, whose meaning changed between rounds (round 4: 1 = all sets; round
    5: 1 = per set): the old spelling is refused rather than silently read with either meaning, and so is a value
    outside 1..8."""
    if "GSLM_LOSS_SETS" in os.environ:
        raise ValueError("GSLM_LOSS_SETS is no longer read: set GSLM_LOSS_SET_GROUP=k (k sets per blend pass, 1..8; "
                         "1 = per set, the default; 8 = all sets in one pass)")
    raw = os.environ.get("GSLM_LOSS_SET_GROUP", "1")
    try:
        k = int(raw)
    except ValueError:
        k = 0
    if not 1 <= k <= 8:
        raise ValueError(f"GSLM_LOSS_SET_GROUP={raw!r}: sets per blend pass must be an integer in 1..8")
    return k


class LossEvaluator:
    """The line search's validation loss: `val_loss_func().loss_scalar` of train_jvp.py:258,268,279 (batch_training_loss
    with disable_ssim=True over the validation views: 2 sum_b ||m_b clamp01(R_b) - gt_b||^2) on the HIP forward.

    Per view: gslm_preprocess_ordered -> gslm_rasterize_loss (binning, then the blend with the residual's loss fused
    into its epilogue: no image is written).
      * Depth order: it depends on xyz alone, which the LM step freezes (train_jvp.py:221-227), so each view's order
        is sorted at its first evaluation and reused while model._xyz is the same tensor at the same version (the
        same point list, bitwise).
      * Batches: views run in batches of `batch` workspaces.  The first evaluation sizes the binnings: a batch's
        preprocesses are enqueued first and one gslm_num_rendered_many read-back sizes them all (one host round trip
        per batch).  With device_count=True later evaluations render through gslm_rasterize_loss_dev instead (the
        pair count stays on the device, no host round trip inside the evaluation); the counts land in one device
        array read once at the end, and a view whose count exceeded its slot's list capacity is rendered again
        exactly (its slot grown).
      * Streams: consecutive views of a batch run on `streams` HIP streams, so one view's short serial kernels
        (scans, the tile launch order, the loss reduction) and its blend's tail overlap another view's work.  Three
        by default: with the main stream that is the 4 hardware queues HIP gives a process (GPU_MAX_HW_QUEUES), and
        the LM step measured 91-93 ms at 3 side streams against 94-96 at 8 (profiles/r05/ab/val_streams_kept/; more
        queues or higher-priority streams were slower still).
    Each view's loss lands in its own device double; the total is their sum (view order fixed, so run to run the
    same).  `reduce`: a callable summing it over the ranks that hold the other views (gslm.parallel.allreduce_loss)."""

    def __init__(self, model, cams, bg, device="cuda", batch=8, gts=None, alpha_masks=None, reduce=None, streams=3,
                 device_count=False):
        self.model = model
        # True: evaluations after the first render through gslm_rasterize_loss_dev (no count read-back per batch).
        # Measured at 50 1080p views, 8 streams: 0.347 ms per view against 0.339 with the per-batch read-back
        # (profiles/r03/val_loss_devcount.json) -- the read-back costs less than the capacity-sized tile sort
        self.device_count = device_count
        self.device = device
        self.reduce = reduce
        self.gts = [c.original_image.to(device) for c in cams] if gts is None else gts
        ms = [c.alpha_mask for c in cams] if alpha_masks is None else alpha_masks
        self.masks = [None if m is None else m.to(device=device, dtype=torch.float32).contiguous() for m in ms]
        self.views = [_lib.view_from_camera(c, bg, model.active_sh_degree) for c in cams]
        for vw, gt, m in zip(self.views, self.gts, self.masks):
            H, W = vw.image_height, vw.image_width
            if gt.shape != (3, H, W) or gt.dtype != torch.float32:
                raise ValueError(f"ground truth must be float32 (3, {H}, {W}), got {gt.dtype} {tuple(gt.shape)}")
            if m is not None and m.numel() != H * W:
                raise ValueError("alpha mask must be [1, H, W]")
        self.batch = max(1, min(int(batch), len(cams) or 1))
        nstr = max(1, min(int(streams), self.batch))
        self.streams = [torch.cuda.Stream(device) for _ in range(nstr)] if nstr > 1 else [None]
        self.slots = [dict(geom=None, binning=None) for _ in range(self.batch)]
        nb = max([lib.gslm_loss_scratch_bytes(v.image_height, v.image_width) for v in self.views] + [8])
        self.loss_scratch = [torch.empty(nb // 8 + 1, dtype=torch.float64, device=device) for _ in self.streams]
        self.num_rendered = [0] * len(cams)
        self._order_key, self._orders = None, [None] * len(cams)
        self._pos = [None] * len(cams)  # the depth orders' inverses (gslm_depth_positions), for evaluate_points
        # the shared binning of evaluate_points (gslm_union_*): per batch position k its sets' geometries, the union
        # geometry and the union list
        self.uslots = [[dict(geoms=[], ugeom=None) for _ in range(self.batch)] for _ in range(2)]
        self.ubins = [None] * self.batch
        self.sets_scratch = [None] * self.batch
        # the six points' blends: one pass per set over each union list (gslm_rasterize_loss_slot; loss_sets = 1), or
        # passes over groups of loss_sets sets each (gslm_rasterize_loss_sets) -- the same losses bitwise.  Per set is
        # the default: the all-sets pass wins when evaluate_points runs back to back (69.8 against 74.8 ms for the six
        # points over 50 views) but not inside lm_step, where it holds the CUs longer against the next batch's sorts
        # on the other streams (profiles/r04/ab/all_sets_default/, profiles/r05/ab/loss_set_groups/).
        # GSLM_LOSS_SET_GROUP=k (1..8) selects groups of k (1 = per set, 8 = all sets in one pass).
        self.loss_sets = loss_set_group()
        self.union_counts = []

    def _slot(self, k, P):
        sl = self.slots[k]
        if sl["geom"] is None or sl["geom"].numel() < lib.gslm_geom_bytes(P):
            sl["geom"] = _lib.u8(lib.gslm_geom_bytes(P), self.device)
        return sl

    def _stream(self, k):
        """(torch stream or None, hipStream_t) of batch position k."""
        st = self.streams[k % len(self.streams)]
        return st, (st.cuda_stream if st is not None else _lib.stream_handle(self.device))

    def _render_exact(self, g, i, losses):
        """View i's loss into losses[i] with the count read back first (slot 0 grown as needed; main stream)."""
        P = g.P
        sl = self._slot(0, P)
        vw = self.views[i]
        main_h = torch.cuda.current_stream(self.device).cuda_stream
        check(lib.gslm_preprocess_ordered(ctypes.byref(vw), ctypes.byref(g), sl["geom"].data_ptr(), sl["geom"].numel(),
                                          None, self._orders[i].data_ptr(), 2, main_h), "gslm_preprocess_ordered")
        n = ctypes.c_int64(0)
        check(lib.gslm_num_rendered(sl["geom"].data_ptr(), P, ctypes.byref(n), main_h), "gslm_num_rendered")
        N = int(n.value)
        self.num_rendered[i] = N
        need = lib.gslm_binning_bytes(N, vw.image_height, vw.image_width)
        if sl["binning"] is None or sl["binning"].numel() < need:
            sl["binning"] = _lib.u8(int(need * 1.25) + 4096, self.device)
        m = self.masks[i]
        scr = self.loss_scratch[0]
        check(lib.gslm_rasterize_loss(ctypes.byref(vw), P, sl["geom"].data_ptr(), sl["binning"].data_ptr(),
                                      sl["binning"].numel(), N, self.gts[i].data_ptr(), None if m is None else m.data_ptr(),
                                      scr.data_ptr(), scr.numel() * 8, losses.data_ptr() + 8 * i, 0, main_h),
              "gslm_rasterize_loss")

    def evaluate(self):
        """Device double: the loss over this evaluator's views (summed over the ranks with `reduce`)."""
        g = raw_gaussians(self.model)
        P = g.P
        V = len(self.views)
        losses = torch.zeros(max(V, 1), dtype=torch.float64, device=self.device)
        main = torch.cuda.current_stream(self.device)
        main_h = main.cuda_stream
        xyz = self.model._xyz
        key = (xyz.data_ptr(), xyz._version, P)
        if key != self._order_key:  # xyz moved: sort again
            self._order_key, self._orders = key, [None] * V
            self._pos = [None] * V
        # device-count renders' pair counts: allocated and zeroed on the main stream BEFORE the side streams wait on
        # it, so no stream's k_ranges count write can precede the zero fill
        counts = torch.zeros(max(V, 1), dtype=torch.int32, device=self.device)
        for st in self.streams:  # the parameters (and the zeroed losses and counts) as the main stream left them
            if st is not None:
                st.wait_stream(main)
        caps = {}  # view -> list capacity it was rendered with (device-count renders)
        for b0 in range(0, V, self.batch):
            idx = list(range(b0, min(V, b0 + self.batch)))
            slots = [self._slot(k, P) for k in range(len(idx))]
            if self.device_count and all(sl["binning"] is not None for sl in slots):
                # device-count renders: per view preprocess -> binning + blend + loss on its stream, no read-back
                for k, (sl, i) in enumerate(zip(slots, idx)):
                    vw = self.views[i]
                    mode = 2 if self._orders[i] is not None else 1
                    if mode == 1:
                        self._orders[i] = torch.empty(max(P, 1), dtype=torch.int32, device=self.device)
                    _, sh = self._stream(k)
                    check(lib.gslm_preprocess_ordered(ctypes.byref(vw), ctypes.byref(g), sl["geom"].data_ptr(),
                                                      sl["geom"].numel(), None, self._orders[i].data_ptr(), mode, sh),
                          "gslm_preprocess_ordered")
                    caps[i] = (k, int(lib.gslm_binning_capacity(sl["binning"].numel(), vw.image_height,
                                                                   vw.image_width)))
                    m = self.masks[i]
                    scr = self.loss_scratch[k % len(self.streams)]
                    check(lib.gslm_rasterize_loss_dev(ctypes.byref(vw), P, sl["geom"].data_ptr(), sl["binning"].data_ptr(),
                                                      sl["binning"].numel(), self.gts[i].data_ptr(),
                                                      None if m is None else m.data_ptr(), scr.data_ptr(),
                                                      scr.numel() * 8, losses.data_ptr() + 8 * i, 0,
                                                      counts.data_ptr() + 4 * i, sh), "gslm_rasterize_loss_dev")
                continue
            for k, (sl, i) in enumerate(zip(slots, idx)):
                mode = 2 if self._orders[i] is not None else 1
                if mode == 1:
                    self._orders[i] = torch.empty(max(P, 1), dtype=torch.int32, device=self.device)
                _, sh = self._stream(k)
                check(lib.gslm_preprocess_ordered(ctypes.byref(self.views[i]), ctypes.byref(g), sl["geom"].data_ptr(),
                                                  sl["geom"].numel(), None, self._orders[i].data_ptr(), mode, sh),
                      "gslm_preprocess_ordered")
            for st in self.streams:
                if st is not None:
                    main.wait_stream(st)
            geoms = (ctypes.c_void_p * len(idx))(*[sl["geom"].data_ptr() for sl in slots])
            Ps = (ctypes.c_int64 * len(idx))(*([P] * len(idx)))
            Ns = (ctypes.c_int64 * len(idx))()
            check(lib.gslm_num_rendered_many(geoms, Ps, len(idx), Ns, main_h), "gslm_num_rendered_many")
            for k, (sl, i) in enumerate(zip(slots, idx)):
                vw = self.views[i]
                H, W, N = vw.image_height, vw.image_width, int(Ns[k])
                self.num_rendered[i] = N
                st, sh = self._stream(k)
                need = lib.gslm_binning_bytes(N, H, W)
                if sl["binning"] is None or sl["binning"].numel() < need:
                    if sl["binning"] is not None and st is not None:
                        main.wait_stream(st)  # the old buffer is freed on the main stream: after its last use
                    sl["binning"] = _lib.u8(int(need * 1.25) + 4096, self.device)
                m = self.masks[i]
                scr = self.loss_scratch[k % len(self.streams)]
                check(lib.gslm_rasterize_loss(ctypes.byref(vw), P, sl["geom"].data_ptr(), sl["binning"].data_ptr(),
                                              sl["binning"].numel(), N, self.gts[i].data_ptr(),
                                              None if m is None else m.data_ptr(), scr.data_ptr(), scr.numel() * 8,
                                              losses.data_ptr() + 8 * i, 0, sh), "gslm_rasterize_loss")
        for st in self.streams:
            if st is not None:
                main.wait_stream(st)
        if caps:
            ns = counts.tolist()  # the evaluation's one read-back
            for i in caps:
                self.num_rendered[i] = ns[i]
            for i, (k, cap) in caps.items():
                if ns[i] > cap:  # a list past its slot's capacity: this view again, exactly, on the main stream
                    self._render_exact(g, i, losses)
                    vw = self.views[i]
                    need = lib.gslm_binning_bytes(ns[i], vw.image_height, vw.image_width)
                    if self.slots[k]["binning"].numel() < need:  # and its slot's list grown for the next evaluation
                        self.slots[k]["binning"] = _lib.u8(int(need * 1.25) + 4096, self.device)
        loss = losses[:V].sum() if V else losses[0]
        if self.reduce is not None:
            self.reduce(loss)
        return loss

    # ---- the line search's six points with one binning per view (include/gslm.h "shared binning", ABI 8) ----
    def _sets_scratch(self, k, n, H, W):
        """Batch position k's per-tile partials of the all-sets blend (its stream's own buffer)."""
        nb = lib.gslm_loss_sets_scratch_bytes(n, H, W)
        t = self.sets_scratch[k]
        if t is None or t.numel() * 8 < nb:
            t = self.sets_scratch[k] = torch.empty(nb // 8 + 1, dtype=torch.float64, device=self.device)
        return t

    def _uslot(self, par, k, n, P):
        """Batch position k's depth-space records (n sets, gslm_depth_records_bytes(P) = 64 B per Gaussian each) and
        union geometry (gslm_geom_bytes(P), ~112 B per Gaussian), of slot set `par` (two sets alternate over the
        batches: a batch's preprocesses overwrite the slots of the batch before the previous one).  Peak device memory
        of evaluate_points: 2 x batch x (64 n + 112) B per Gaussian (7.9 GB at 1M Gaussians, batch 8, n = 6; until
        round 5 every set held a whole geometry workspace: 12.5 GB), plus the snapshots' five moving leaves per point
        (param_snapshot) and one sort geometry; clear_val_cache() releases an evaluator lm_step kept."""
        sl = self.uslots[par][k]
        nr, nb = lib.gslm_depth_records_bytes(P), lib.gslm_geom_bytes(P)
        while len(sl["geoms"]) < n:
            sl["geoms"].append(None)
        for a in range(n):
            if sl["geoms"][a] is None or sl["geoms"][a].numel() < nr:
                sl["geoms"][a] = _lib.u8(nr, self.device)
        if sl["ugeom"] is None or sl["ugeom"].numel() < nb:
            sl["ugeom"] = _lib.u8(nb, self.device)
        return sl

    def _sort_geom(self, P):
        """The full geometry workspace of the depth sorts of evaluate_points (main stream only)."""
        t = getattr(self, "_sgeom", None)
        if t is None or t.numel() < lib.gslm_geom_bytes(P):
            t = self._sgeom = _lib.u8(lib.gslm_geom_bytes(P), self.device)
        return t

    def refresh_views(self, cams, bg, sh_degree):
        """Rebuild the views from the cameras (their matrices now) and drop the cached depth order of every view whose
        camera moved -- a kept evaluator (lm_step's _VAL_CACHE) then never renders with a stale pose."""
        for i, c in enumerate(cams):
            v = _lib.view_from_camera(c, bg, sh_degree)
            if bytes(v) != bytes(self.views[i]):
                self.views[i] = v
                self._orders[i] = None
                self._pos[i] = None

    def evaluate_points(self, sets):
        """The validation loss at each of n <= 8 parameter sets (snapshots sharing the model's frozen xyz: the six
        line-search points of train_jvp.py:262-277, param_snapshot), as a list of device doubles -- each bitwise equal
        to evaluate() with the model at that set.  Per view: the n sets' render records in depth space
        (gslm_preprocess_views with the view's depth positions: one pass over the Gaussians per set for the batch's
        views), ONE binning over the union of the sets' rects (gslm_union_geometry / gslm_union_binning: 4 mask bits
        per set and list entry, carried through the tile sort), then the n blends + losses through it
        (gslm_rasterize_loss_slot).
        Pipelining: a batch's preprocesses, union geometries and pair-count read-back run on the main stream while the
        previous batch's binnings and blends run on the side streams (two alternating slot sets), so the read-back does
        not drain the device.  union_counts[i]: view i's union list length (the last call)."""
        n = len(sets)
        if not 1 <= n <= 8:
            raise ValueError("evaluate_points takes 1..8 parameter sets")
        xyz = sets[0]._xyz
        if any(st._xyz is not xyz for st in sets):
            raise ValueError("evaluate_points: every set shares the frozen xyz tensor")
        gs = [raw_gaussians(st) for st in sets]
        P = gs[0].P
        V = len(self.views)
        main = torch.cuda.current_stream(self.device)
        main_h = main.cuda_stream
        key = (xyz.data_ptr(), xyz._version, P)
        if key != self._order_key:
            self._order_key, self._orders = key, [None] * V
            self._pos = [None] * V
        losses = [torch.zeros(max(V, 1), dtype=torch.float64, device=self.device) for _ in range(n)]
        self.union_counts = [0] * V
        side = [st for st in self.streams if st is not None]
        done = [None, None]  # per slot set: events after the side streams' last use of its slots
        for bi, b0 in enumerate(range(0, V, self.batch)):
            par = bi & 1
            idx = list(range(b0, min(V, b0 + self.batch)))
            if done[par] is not None:  # the batch before the previous one has finished with these slots
                for ev in done[par]:
                    main.wait_event(ev)
            slots = [self._uslot(par, k, n, P) for k in range(len(idx))]
            # 1. each view's depth order (sorted once while xyz is unchanged) and its inverse, the depth positions
            for k, i in enumerate(idx):
                if self._orders[i] is None:  # the depth sort (set 0's geometry; only the order is kept)
                    self._orders[i] = torch.empty(max(P, 1), dtype=torch.int32, device=self.device)
                    sg = self._sort_geom(P)
                    check(lib.gslm_preprocess_ordered(ctypes.byref(self.views[i]), ctypes.byref(gs[0]),
                                                      sg.data_ptr(), sg.numel(), None, self._orders[i].data_ptr(), 1,
                                                      main_h), "gslm_preprocess_ordered")
                    self._pos[i] = None
                if self._pos[i] is None:
                    self._pos[i] = torch.empty(max(P, 1), dtype=torch.int32, device=self.device)
                    check(lib.gslm_depth_positions(self._orders[i].data_ptr(), P, self._pos[i].data_ptr(), main_h),
                          "gslm_depth_positions")
            # 2. the sets' render records in depth space: one pass over the Gaussians per set for the batch's views
            # (gslm_preprocess_views takes at most 8 views per call: a batch above 8 goes in chunks)
            for c0 in range(0, len(idx), 8):
                cidx = idx[c0:c0 + 8]
                vws = (_lib.GslmView * len(cidx))(*[self.views[i] for i in cidx])
                pos = (ctypes.c_void_p * len(cidx))(*[self._pos[i].data_ptr() for i in cidx])
                for a in range(n):
                    ge = (ctypes.c_void_p * len(cidx))(*[sl["geoms"][a].data_ptr() for sl in slots[c0:c0 + 8]])
                    check(lib.gslm_preprocess_views(vws, len(cidx), ctypes.byref(gs[a]), ge,
                                                    slots[0]["geoms"][a].numel(), pos, main_h), "gslm_preprocess_views")
            # 3. union geometries and their pair counts (main stream; the read-back waits for main only)
            for k, i in enumerate(idx):
                ge = (ctypes.c_void_p * n)(*[slots[k]["geoms"][a].data_ptr() for a in range(n)])
                check(lib.gslm_union_geometry(ctypes.byref(self.views[i]), P, ge, n, slots[k]["geoms"][0].numel(),
                                              slots[k]["ugeom"].data_ptr(), slots[k]["ugeom"].numel(), main_h),
                      "gslm_union_geometry")
            ugeoms = (ctypes.c_void_p * len(idx))(*[sl["ugeom"].data_ptr() for sl in slots])
            Ps = (ctypes.c_int64 * len(idx))(*([P] * len(idx)))
            Ns = (ctypes.c_int64 * len(idx))()
            check(lib.gslm_num_rendered_many(ugeoms, Ps, len(idx), Ns, main_h), "gslm_num_rendered_many")
            # 4. binning + the n blends of each view on its side stream
            for st in side:
                st.wait_stream(main)
            for k, (sl, i) in enumerate(zip(slots, idx)):
                vw = self.views[i]
                H, W, N = vw.image_height, vw.image_width, int(Ns[k])
                self.union_counts[i] = N
                st, sh = self._stream(k)
                need = lib.gslm_union_binning_bytes(N, H, W)
                bins = self.ubins
                if bins[k] is None or bins[k].numel() < need:
                    if bins[k] is not None and st is not None:
                        main.wait_stream(st)  # freed on the main stream: after its last use
                    bins[k] = _lib.u8(int(need * 1.25) + 4096, self.device)
                binning = bins[k]
                ge = (ctypes.c_void_p * n)(*[sl["geoms"][a].data_ptr() for a in range(n)])
                sb = sl["geoms"][0].numel()
                check(lib.gslm_union_binning(ctypes.byref(vw), P, sl["ugeom"].data_ptr(), binning.data_ptr(),
                                             binning.numel(), N, ge, n, sb, sh), "gslm_union_binning")
                m = self.masks[i]
                if self.loss_sets > 1:  # groups of loss_sets sets, one pass over the union list each
                    gsz = min(self.loss_sets, n)
                    scr = self._sets_scratch(k, gsz, H, W)
                    for a0 in range(0, n, gsz):
                        na = min(gsz, n - a0)
                        gg = (ctypes.c_void_p * na)(*[sl["geoms"][a].data_ptr() for a in range(a0, a0 + na)])
                        lp = (ctypes.c_void_p * na)(*[losses[a].data_ptr() + 8 * i for a in range(a0, a0 + na)])
                        check(lib.gslm_rasterize_loss_sets(ctypes.byref(vw), P, gg, na, a0, sb, binning.data_ptr(),
                                                           binning.numel(), N, self.gts[i].data_ptr(),
                                                           None if m is None else m.data_ptr(), scr.data_ptr(),
                                                           scr.numel() * 8, lp, 0, sh), "gslm_rasterize_loss_sets")
                    continue
                scr = self.loss_scratch[k % len(self.streams)]
                for a in range(n):
                    check(lib.gslm_rasterize_loss_slot(ctypes.byref(vw), P, sl["geoms"][a].data_ptr(), sb,
                                                       binning.data_ptr(), binning.numel(), N, a, n, self.gts[i].data_ptr(),
                                                       None if m is None else m.data_ptr(), scr.data_ptr(),
                                                       scr.numel() * 8, losses[a].data_ptr() + 8 * i, 0, sh),
                          "gslm_rasterize_loss_slot")
            if side:
                evs = []
                for st in side:
                    ev = torch.cuda.Event()
                    ev.record(st)
                    evs.append(ev)
                done[par] = evs
        for st in side:
            main.wait_stream(st)
        out = []
        for a in range(n):
            loss = losses[a][:V].sum() if V else losses[a][0]
            if self.reduce is not None:
                self.reduce(loss)
            out.append(loss)
        return out


_LS_GROUPS = ("_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity")


def param_snapshot(model):
    """A line-search point's parameters for LossEvaluator.evaluate_points: clones of the groups the LM step moves,
    the model's own (frozen) xyz tensor.  The exposure group is not rendered by the validation loss."""
    import types
    ns = types.SimpleNamespace(_xyz=model._xyz, active_sh_degree=model.active_sh_degree)
    with torch.no_grad():
        for k in _LS_GROUPS:
            setattr(ns, k, getattr(model, k).detach().clone())
    return ns


def update_params(model, layout, step, scale, skip_xyz=False):
    """GaussianModel.update_step(scale * s) (gaussian_model.py:131-139) from a flat step.  skip_xyz: the step's xyz
    group is zero by construction (the LM step's param mask, train_jvp.py:221-227), so adding it would change no
    value -- it is left alone, which keeps model._xyz's version (the line search's cached depth orders)."""
    v = layout.views(step)
    with torch.no_grad():
        if not skip_xyz:
            model._xyz.add_(v["xyz"], alpha=scale)
        model._features_dc.add_(v["features_dc"], alpha=scale)
        model._features_rest.add_(v["features_rest"], alpha=scale)
        model._scaling.add_(v["scaling"], alpha=scale)
        model._rotation.add_(v["rotation"], alpha=scale)
        model._opacity.add_(v["opacity"], alpha=scale)
        model._exposure.add_(v["exposure"], alpha=scale)


_VAL_CACHE = {}  # lm_step's last validation evaluator: {"last": (key, evaluator)}


def clear_val_cache():
    """Release the validation evaluator lm_step keeps between LM steps (its workspaces -- evaluate_points' peak, see
    LossEvaluator._uslot -- the views' depth orders, and its references to the model and the validation cameras)."""
    _VAL_CACHE.clear()


def lm_step(model, cams, val_cams, bg, max_iter=2, restart_iter=1, damp=None, mask_xyz=True, check_every=True,
            verbose=False, device="cuda", sh_projection="auto", recursion="fused", exchange="auto", group=None,
            val_batch=8, timing=False, backend=None, line_search="union", val_at_start=False, cache_val=True):
    """One LM step of train_jvp.py:237-289: loss, CGLS on the normal equations, backtracking line search.

    Single process: LMProblem over `cams` (with one training view the SH-rest group of the CG vectors is carried
    projected).  Under torch.distributed (several ranks, or GSLM_FORCE_COLLECTIVES=1 at one rank) the step runs
    sharded, every rank calling lm_step with the same arguments: the training views are split over the ranks
    (gslm.parallel.ShardedLMProblem -- Gaussian-sharded CG vectors when every rank holds as many views, else the
    replicated-vector exchanges), the step is gathered whole on every rank (gather_full), the validation views are
    split the same way and each line-search loss is one 8-byte all-reduce, and every rank applies the identical
    update_step -- the replicas stay bitwise equal.
    recursion: "fused" (cgls_fused, one fused (J^T J + D) p per iteration) or "cgls" (cgls_residual, the
    reference's residual-space recursion; single process only).  check_every: the reference's stopping tests,
    on the device (cgls_fused).  timing=True adds wall-clock phases (evaluate + J^T b, CG, line search) to the
    result, synchronising the device at their boundaries.
    line_search: "union" (xyz masked: the six points' parameters are formed first by the same update_step sequence
    and their validation losses come from ONE binning per view, LossEvaluator.evaluate_points -- bitwise the losses of
    the sequential renders; the final point, known only after them, is rendered as before) or "exact" (train_jvp.py's
    order: update, render, update, ...).  val_at_start: also report the validation loss at the starting parameters
    (one more evaluation, outside the reference's algorithm: it shows whether the step descends).  cache_val: keep the
    validation evaluator for the next LM step (its workspaces and cached depth orders; clear_val_cache() releases it;
    the views are rebuilt from the cameras every step, so a moved camera is rendered at its new pose).
    backend: (problem_cls, evaluator_cls, solver) replacing (LMProblem, LossEvaluator, cgls_fused) -- the CPU
    multi-process tests run this same driver, sharding and reductions on the oracle restatement."""
    import time
    from gslm.parallel import ShardedLMProblem, allreduce_loss, collectives_on, shard_views, world
    rank, n = world()
    sharded = collectives_on(n)
    problem_cls, evaluator_cls, solver = backend if backend is not None else (LMProblem, LossEvaluator, cgls_fused)
    t = {}
    clock = [time.perf_counter()]

    def lap(name):
        if timing:
            if torch.device(device).type == "cuda":
                torch.cuda.synchronize(device)
            now = time.perf_counter()
            t[name] = 1e3 * (now - clock[0])
            clock[0] = now

    if sharded:
        if recursion != "fused":
            raise ValueError("the sharded LM step runs cgls_fused")
        mine = [cams[i] for i in shard_views(len(cams), rank, n)]
        prob = ShardedLMProblem(model, mine, bg, group=group, all_cams=cams, exchange=exchange, mask_xyz=mask_xyz,
                                damp=damp, device=device, problem_cls=problem_cls)
    else:
        prob = problem_cls(model, cams, bg, mask_xyz=mask_xyz, damp=damp, device=device, sh_projection=sh_projection)
    start_loss = prob.evaluate()
    if recursion == "cgls":
        lap("evaluate_rhs_ms")
        s, info = cgls_residual(prob, max_iter=max_iter, restart_iter=restart_iter, verbose=verbose)
    elif recursion == "fused":
        g = prob.rhs(prob.zeros())
        lap("evaluate_rhs_ms")
        s, info = solver(prob, g, max_iter=max_iter, restart_iter=restart_iter, check_every=check_every,
                         verbose=verbose)
    else:
        raise ValueError(f"recursion must be 'fused' or 'cgls', got {recursion!r}")
    # the whole step in the reference's layout, identical on every rank
    s = prob.gather_full(s) if getattr(prob, "exchange", None) == "gaussian" else getattr(prob, "expand", lambda v: v)(s)
    if not bool(torch.isfinite(s).all()):
        # the reference's NaN asserts (solver_functions.py:125-130) on the step itself, before update_params touches the
        # model -- for solves without the device stopping tests (which raise inside cgls_fused, naming the groups);
        # s is the gathered step, the same on every rank, so every rank raises here and none waits in a collective
        raise NonFiniteError("NaN detected in the LM step (the CGLS solution)")
    start_loss = float(start_loss)
    del prob
    lap("cg_ms")
    full = ParamLayout(model._xyz.shape[0], 1 + model._features_rest.shape[1], model._exposure.shape[0])
    mine_val = [val_cams[i] for i in shard_views(len(val_cams), rank, n)] if sharded else val_cams
    # the validation evaluator (its workspaces and the views' cached depth orders) is kept from one LM step to the
    # next while the model, the validation cameras (held by it, so their ids stay theirs) and the settings are the same
    imgs = [(getattr(c, "original_image", None), getattr(c, "alpha_mask", None)) for c in mine_val]
    vkey = (id(model), model.active_sh_degree, tuple(id(c) for c in mine_val), tuple(id(t) for p in imgs for t in p),
            str(device), val_batch, evaluator_cls, sharded, id(group),
            tuple(float(x) for x in torch.as_tensor(bg).reshape(-1).tolist()))
    hit = _VAL_CACHE.get("last") if cache_val else None
    if hit is not None and hit[0] == vkey:
        val = hit[1]
        if hasattr(val, "refresh_views"):
            val.refresh_views(mine_val, bg, model.active_sh_degree)
    else:
        _VAL_CACHE.pop("last", None)
        val = evaluator_cls(model, mine_val, bg, device=device, batch=val_batch,
                            reduce=(lambda x: allreduce_loss(x, group)) if sharded else None,
                            # (GSLM_VAL_STREAMS: the side-stream count, an A/B override of LossEvaluator's default)
                            **({"streams": int(os.environ["GSLM_VAL_STREAMS"])} if "GSLM_VAL_STREAMS" in os.environ else {}))
        if cache_val:
            val.held = (model, list(mine_val), imgs)
            _VAL_CACHE["last"] = (vkey, val)
    val_start = float(val.evaluate()) if val_at_start else None
    if val_at_start:
        lap("val_start_ms")
    if line_search not in ("union", "exact"):
        raise ValueError(f"line_search must be 'union' or 'exact', got {line_search!r}")
    union = line_search == "union" and mask_xyz and hasattr(val, "evaluate_points")
    # train_jvp.py:262-279: alpha = 2, 1, ..., 1/16 on the validation views, keep the best, step to it
    alpha = 2.0
    best_alpha, best_loss = alpha, math.inf
    trace = []
    update_params(model, full, s, alpha, skip_xyz=mask_xyz)
    if union:
        # the same update_step sequence, the six points' parameters kept; their losses from one binning per view
        points = []
        for _ in range(6):
            points.append((alpha, param_snapshot(model)))
            new_alpha = alpha * 0.5
            update_params(model, full, s, new_alpha - alpha, skip_xyz=mask_xyz)
            alpha = new_alpha
        alphas = [a for a, _ in points]
        vls = [float(v) for v in val.evaluate_points([p for _, p in points])]
        del points
        for a, vl in zip(alphas, vls):
            trace.append((a, vl))
            if vl < best_loss:
                best_loss, best_alpha = vl, a
    else:
        for _ in range(6):
            vl = float(val.evaluate())
            trace.append((alpha, vl))
            if vl < best_loss:
                best_loss, best_alpha = vl, alpha
            new_alpha = alpha * 0.5
            update_params(model, full, s, new_alpha - alpha, skip_xyz=mask_xyz)
            alpha = new_alpha
    update_params(model, full, s, best_alpha - alpha, skip_xyz=mask_xyz)
    final = float(val.evaluate())
    lap("line_search_ms")
    out = dict(start_loss=start_loss, final_val_loss=final, best_alpha=best_alpha, cg=info, step=s, trace=trace,
               val_views=len(val_cams), ranks=n if sharded else 1, line_search="union" if union else "exact")
    if val_at_start:
        out["val_start_loss"] = val_start
    if union and getattr(val, "union_counts", None):
        out["union_pairs"] = sum(val.union_counts)
    if timing:
        out["timing"] = t
    return out
