"""First-order optimizers of the reference's training loop on one HIP launch per step.

* `FusedAdam` is `torch.optim.Adam` (the optimizer `GaussianModel.training_setup` builds,
  scene/gaussian_model.py:282-283,291, stepped at train.py:184-186) with `step()` replaced by
  `gslm_adam_step`: every parameter group in one launch, 28 B of HBM traffic per float instead of the
  ~7 passes of torch's foreach implementation.  State keys (`step`, `exp_avg`, `exp_avg_sq`), param
  groups, `state_dict()` / `load_state_dict()` are torch's own (it subclasses torch.optim.Adam), so the
  reference's optimizer surgery (`replace_tensor_to_optimizer`, `_prune_optimizer`,
  `cat_tensors_to_optimizer`, gaussian_model.py:406-476) and checkpoint capture work unchanged.
* `SparseGaussianAdam` is the class the reference imports from the accelerated rasterizer
  (gaussian_model.py:29, :284-289; train.py:180-183): `step(visibility, N)` updates only the Gaussians
  with `visibility[g]` set, betas (0.9, 0.999), no bias correction (upstream 3dgs_accel adamUpdate,
  absent here: semantics restated; see include/gslm.h).

Parameters, gradients and moments must be contiguous float32 on the GPU; there is no torch fallback.
"""
import torch

from gslm import _lib
from gslm._lib import lib, check

__all__ = ["FusedAdam", "SparseGaussianAdam"]


def _contig_f32(t, what):
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise TypeError(f"{what} must be a contiguous float32 tensor (got {t.dtype}, contiguous={t.is_contiguous()})")
    if not t.is_cuda:
        raise RuntimeError(f"{what} must live on the GPU (gslm_adam_step is a HIP kernel)")
    return t


class FusedAdam(torch.optim.Adam):
    """torch.optim.Adam(params, lr, betas, eps) whose step is `gslm_adam_step` (dense, bias-corrected)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay != 0.0:
            raise ValueError("FusedAdam: weight_decay is not used by the reference (gaussian_model.py:283)")
        super().__init__(params, lr=lr, betas=betas, eps=eps)

    def _state(self, p):
        state = self.state[p]
        if len(state) == 0:
            # torch.optim.Adam's lazy initialisation (CPU float step counter, preserve_format moments)
            state["step"] = torch.tensor(0.0, dtype=torch.float32)
            state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return state

    def _launch(self, descs, betas, eps, visible=None, num_gaussians=0):
        for i in range(0, len(descs), _lib.ADAM_MAX_GROUPS):
            chunk = descs[i:i + _lib.ADAM_MAX_GROUPS]
            arr = (_lib.GslmAdamGroup * len(chunk))(*chunk)
            check(lib.gslm_adam_step(arr, len(chunk), float(betas[0]), float(betas[1]), float(eps),
                                     None if visible is None else visible.data_ptr(), int(num_gaussians),
                                     0 if visible is None else 1, _lib.stream_handle()), "gslm_adam_step")

    @staticmethod
    def _desc(p, state, lr, step=0, per_gauss=1):
        d = _lib.GslmAdamGroup()
        d.param, d.grad = p.data_ptr(), p.grad.data_ptr()
        d.exp_avg, d.exp_avg_sq = state["exp_avg"].data_ptr(), state["exp_avg_sq"].data_ptr()
        d.n, d.floats_per_gaussian, d.lr, d.step = p.numel(), int(per_gauss), float(lr), int(step)
        return d

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        by_hyper = {}
        for group in self.param_groups:
            if group.get("amsgrad") or group.get("maximize") or group.get("weight_decay", 0.0):
                raise ValueError("FusedAdam: amsgrad / maximize / weight_decay are not supported")
            for p in group["params"]:
                if p.grad is None:
                    continue
                _contig_f32(p, "parameter")
                _contig_f32(p.grad, "gradient")
                state = self._state(p)
                state["step"] += 1
                key = (tuple(group["betas"]), group["eps"])
                by_hyper.setdefault(key, []).append(
                    (self._desc(p, state, group["lr"], step=int(state["step"].item())), (p, state)))
        for (betas, eps), items in by_hyper.items():
            self._launch([d for d, _ in items], betas, eps)
        return loss


class SparseGaussianAdam(FusedAdam):
    """`diff_gaussian_rasterization.SparseGaussianAdam(params, lr, eps)`; `step(visibility, N)`."""

    def __init__(self, params, lr, eps):
        super().__init__(params, lr=lr, eps=eps)

    @torch.no_grad()
    def step(self, visibility, N):
        N = int(N)
        vis = visibility.reshape(-1)
        if vis.numel() != N:
            raise ValueError(f"SparseGaussianAdam: visibility has {vis.numel()} entries, N = {N}")
        vis = vis.to(torch.bool).contiguous()
        by_eps = {}
        for group in self.param_groups:
            assert len(group["params"]) == 1, "more than one tensor in group"
            p = group["params"][0]
            if p.grad is None:
                continue
            _contig_f32(p, "parameter")
            _contig_f32(p.grad, "gradient")
            if p.numel() % max(N, 1):
                raise ValueError(f"SparseGaussianAdam: group '{group.get('name')}' has {p.numel()} floats, "
                                 f"not a multiple of N = {N}")
            state = self._state(p)
            by_eps.setdefault(group["eps"], []).append(self._desc(p, state, group["lr"],
                                                                  per_gauss=p.numel() // max(N, 1)))
        # the upstream kernel hard-codes b1 = 0.9, b2 = 0.999 and takes the group's lr and eps
        for eps, descs in by_eps.items():
            self._launch(descs, (0.9, 0.999), eps, visible=vis, num_gaussians=N)
