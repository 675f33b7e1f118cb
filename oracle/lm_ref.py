"""ORACLE -- test infrastructure only: the LM normal equations on the CPU oracle renderer.

A PyTorch restatement of the reference LM algebra around
oracle/torch_raster.py, used to (1) check the oracle-side solver semantics against the golden
vectors the reference's own solver produced (tests/golden/solver_golden.npz) and (2) stand in for
the HIP operator in multi-process (gloo) tests of the view sharding:

  residual        r_b = m_b * clamp01(R_b) - gt_b, residual vector [r; r]
                  (batch_training_loss.py:10-17, disable_ssim=True); with ssim=True the vector is
                  [r1; r2] of oracle/ssim_ref.py (batch_training_loss.py:18-30)
  J^T b           -2 sum_b J_r^T r_b                      (solver_functions.py:101-132 with b = -[r; r])
  (J^T J + D) v   2 sum_b J_r^T J_r v + D v               (matvec, matvec_T, GaussianModelDampMatrix)
  CGLS            conjugate_gradient.py:51-127 in its normal-equations form, float64 scalars
"""
import math

import torch
import torch.autograd.forward_ad as fwAD

from gslm.params import GROUPS, ParamLayout
from oracle import ssim_ref
from oracle import torch_raster as tr

DEFAULT_DAMP = {"xyz": 5e2, "features_dc": 5e-2, "features_rest": 5e-2, "scaling": 5e-2, "rotation": 5e-2,
                "opacity": 5e-2, "exposure": 1e1}


class OracleLMProblem:
    def __init__(self, model, cams, bg, mask_xyz=True, damp=None, ssim=False, lambda_dssim=0.2, device="cpu",
                 sh_projection=False):
        # (device / sh_projection: the HIP LMProblem's keywords, accepted so gslm.lm.lm_step can build either;
        # the oracle runs on the CPU in the reference's full layout)
        self.model, self.cams, self.bg = model, cams, bg
        self.mask_xyz = mask_xyz
        self.ssim, self.lambda_dssim = ssim, lambda_dssim
        self.damp = DEFAULT_DAMP if damp is None else damp
        P = model._xyz.shape[0]
        K = 1 + model._features_rest.shape[1]
        self.layout = ParamLayout(P, K, model._exposure.shape[0])

    def _leaves(self):
        m = self.model
        return [m._xyz, m._features_dc, m._features_rest, m._scaling, m._rotation, m._opacity, m._exposure]

    def _residuals(self):
        """Residual blocks; each enters the loss and J^T J with factor self._fac (2: the [r; r] aliasing)."""
        out = []
        for c in self.cams:
            img, _, _, _ = tr.render_model(self.model, c, self.bg)
            x = img * c.alpha_mask
            if self.ssim:
                out.extend(ssim_ref.ssim_residuals(x, c.original_image, self.lambda_dssim))
            else:
                out.append(x - c.original_image)
        return out

    @property
    def _fac(self):
        return 1.0 if self.ssim else 2.0

    def evaluate(self):
        with torch.no_grad():
            self.loss = torch.zeros((), dtype=torch.float64)
            for r in self._residuals():
                self.loss = self.loss + self._fac * (r.double() ** 2).sum()
        return self.loss

    def _flatten(self, tensors):
        return torch.cat([t.reshape(-1) for t in tensors])

    def _mask(self, vec):
        o = self.layout.offsets
        if self.mask_xyz:
            vec[o["xyz"][0]:o["xyz"][1]] = 0
        vec[o["exposure"][0]:o["exposure"][1]] = 0
        return vec

    def rhs(self, out=None):
        leaves = self._leaves()
        for t in leaves:
            t.grad = None
        res = list(self._residuals())
        if not res:  # a rank holding no views (an uneven split): J^T b = 0
            g = torch.zeros(self.layout.numel)
            if out is not None:
                out.copy_(g)
                return out
            return g
        loss = sum((0.5 * self._fac) * (r * r).sum() for r in res)  # J^T b = -grad
        grads = torch.autograd.grad(loss, leaves, allow_unused=True)
        g = self._flatten([-(gr if gr is not None else torch.zeros_like(t)) for gr, t in zip(grads, leaves)])
        g = self._mask(g.detach())
        if out is not None:
            out.copy_(g)
            return out
        return g

    def _jr_v(self, v):
        views = self.layout.views(v)
        m = self.model
        saved = self._leaves()
        with torch.no_grad(), fwAD.dual_level():
            (m._xyz, m._features_dc, m._features_rest, m._scaling, m._rotation, m._opacity, m._exposure) = [
                fwAD.make_dual(t.detach(), views[gname].to(t.dtype)) for t, gname in zip(saved, GROUPS)]
            try:
                tangents = [fwAD.unpack_dual(r).tangent for r in self._residuals()]
            finally:
                (m._xyz, m._features_dc, m._features_rest, m._scaling, m._rotation, m._opacity, m._exposure) = saved
        return [t if t is not None else torch.zeros(3, c.image_height, c.image_width)
                for t, c in zip(tangents, [c for c in self.cams for _ in range(2 if self.ssim else 1)])]

    def damp_add(self, v, y):
        for gname in GROUPS:
            a, b = self.layout.offsets[gname]
            y[a:b] += self.damp[gname] * v[a:b]
        return y

    def local_normal_matvec(self, v, y, damp=False):
        """y = [D v +] sum_b 2 J_r^T J_r v (overwrites y)."""
        v = self._mask(v.clone())
        if not self.cams:  # no views: J^T J v = 0
            y.zero_()
            if damp:
                self.damp_add(v, y)
            return y
        jv = self._jr_v(v)
        leaves = self._leaves()
        res = self._residuals()
        obj = sum((r * (self._fac * t.detach())).sum() for r, t in zip(res, jv))
        grads = torch.autograd.grad(obj, leaves, allow_unused=True)
        out = self._flatten([gr if gr is not None else torch.zeros_like(t) for gr, t in zip(grads, leaves)])
        y.copy_(self._mask(out.detach()))
        if damp:
            self.damp_add(v, y)
        return y

    def matvec(self, v, y):
        return self.local_normal_matvec(v, y, damp=True)

    def matvec_dot(self, v, y, dot_out):
        self.matvec(v, y)
        return False

    def zeros(self):
        return torch.zeros(self.layout.numel)


class OracleLossEvaluator:
    """The line search's validation loss on the oracle (gslm.lm.LossEvaluator's interface): 2 sum_b ||m_b
    clamp01(R_b) - gt_b||^2 over `cams`, summed over the ranks by `reduce`."""

    def __init__(self, model, cams, bg, device="cpu", batch=8, reduce=None):
        self.prob = OracleLMProblem(model, cams, bg)
        self.reduce = reduce

    def evaluate(self):
        loss = self.prob.evaluate().clone()
        if self.reduce is not None:
            self.reduce(loss)
        return loss

    def evaluate_points(self, sets):
        """gslm.lm.LossEvaluator.evaluate_points' interface: the loss at each parameter snapshot (gslm.lm.param_snapshot),
        the model's leaves swapped for the snapshot's while it renders."""
        m = self.prob.model
        names = ("_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity")
        saved = [getattr(m, k) for k in names]
        out = []
        try:
            for st in sets:
                for k in names:
                    setattr(m, k, getattr(st, k))
                out.append(self.evaluate())
        finally:
            for k, t in zip(names, saved):
                setattr(m, k, t)
        return out


def cgls_solver(op, g, max_iter=10, restart_iter=10, check_every=True, verbose=False):
    """cgls_ref in gslm.lm.lm_step's solver interface: (x, info)."""
    return cgls_ref(op, g, max_iter, restart_iter), {"iters": None}


def cgls_ref(op, g, max_iter, restart_iter, tol=1e-10, atol=0.0):
    """cgls_damped (conjugate_gradient.py:51-127) written on A = J^T J + D in float64 scalars.
    Same restart schedule and stopping tests as gslm.lm.cgls_fused.  An operator whose vectors are shards of
    the whole (gslm.parallel.GaussianShardedOperator) supplies the global inner product as op.vdot."""
    vdot = getattr(op, "vdot", None) or (lambda a, b: float((a.double() * b.double()).sum()))
    n = g.numel()
    x = torch.zeros(n, dtype=g.dtype)
    b2 = float(op.loss)
    iter_total, last_res, first = 0, math.inf, True
    q = torch.zeros_like(x)
    while iter_total < max_iter:
        if first:
            s = g.clone()
            first = False
        else:
            s = g - op.matvec(x, q)
        p = s.clone()
        gamma = vdot(s, s)
        stop = False
        for _ in range(restart_iter):
            op.matvec(p, q)
            delta = vdot(p, q)
            if delta < 1e-20:
                stop = True
                break
            alpha = gamma / delta
            x = x + alpha * p
            s = s - alpha * q
            gamma_new = vdot(s, s)
            p = s + (gamma_new / gamma) * p
            res = b2 - vdot(x, g) - vdot(x, s)
            if res > last_res:
                stop = True
                break
            last_res = res
            if gamma_new < max(tol * math.sqrt(gamma), atol):
                stop = True
                break
            gamma = gamma_new
            iter_total += 1
            if iter_total >= max_iter:
                stop = True
                break
        if stop:
            break
    return x


def line_search_ref(apply_step, val_loss, alpha=2.0, halvings=6):
    """The backtracking line search of train_jvp.py:262-279, restated (train_jvp.py is a script and cannot be
    imported).  apply_step(a) performs gaussians.update_step(a * s); val_loss() evaluates the validation batch's
    loss_scalar.  The model is left at best_alpha * s.  Returns (best_alpha, final_val_loss, [(alpha, loss)])."""
    best_alpha, best_loss = alpha, math.inf
    apply_step(alpha)                                # gaussians.update_step(alpha * s)        :266
    trace = []
    for _ in range(halvings):                        # for i in range(6)                       :267
        vl = float(val_loss())
        trace.append((alpha, vl))
        if vl < best_loss:                           # strict: the first (largest) alpha wins ties
            best_loss, best_alpha = vl, alpha
        new_alpha = alpha * 0.5
        apply_step(new_alpha - alpha)                # update_step(alpha_update * s)           :274-275
        alpha = new_alpha
    apply_step(best_alpha - alpha)                   # update_step(best_update * s)            :277-278
    return best_alpha, float(val_loss()), trace      # val_loss = val_loss_func().loss_scalar  :279
