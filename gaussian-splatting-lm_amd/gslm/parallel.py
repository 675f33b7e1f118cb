"""View-sharded LM operator over torch.distributed (RCCL over xGMI on MI355X; gloo for CPU tests).

The reference has no distributed code: its LinearSolverFunctions renders a view batch
serially on one GPU (solver_functions.py:38-41,88-93,110-121).  Here every rank owns a disjoint
slice of the camera batch; the parameters theta (59 fp32 per Gaussian at SH 3) are replicated.
  * J v and the per-view weights never leave the GPU that renders the view;
  * the only exchange per CG iteration is ONE all-reduce (sum) of the partial J^T W J v over the
    param-space vector; D v is added after the reduction, once;
  * J^T b and the loss are all-reduced once per LM step.
All-reduce results are bitwise identical on every rank, so the CG scalars (computed redundantly on
each rank, device-resident) stay consistent without a further broadcast.
"""
import torch
import torch.distributed as dist

from gslm.lm import LMProblem


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_views(n_views, rank, world_size):
    """Contiguous block of view indices owned by `rank` (weak scaling: equal blocks)."""
    per = (n_views + world_size - 1) // world_size
    lo = min(rank * per, n_views)
    return list(range(lo, min(lo + per, n_views)))


class ShardedLMProblem(LMProblem):
    def __init__(self, model, cams, bg, group=None, **kw):
        super().__init__(model, cams, bg, **kw)
        self.group = group
        self.rank, self.world_size = world()

    def _allreduce(self, t):
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def evaluate(self):
        loss = super().evaluate()
        return self._allreduce(loss)

    def rhs(self, out):
        super().rhs(out)
        return self._allreduce(out)

    def matvec_dot(self, v, y, dot_out):
        if self.world_size == 1:
            return super().matvec_dot(v, y, dot_out)
        self.local_normal_matvec(v, y, damp=False)
        self._allreduce(y)
        self.damp_add(v, y)
        return False
