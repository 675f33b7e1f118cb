"""View-sharded LM operator over torch.distributed (RCCL over xGMI on MI355X; gloo for CPU tests).

The reference has no distributed code: its LinearSolverFunctions renders a view batch
serially on one GPU (solver_functions.py:38-41,88-93,110-121).  Here every rank owns a disjoint
block of the camera batch; the parameters theta (59 fp32 per Gaussian at SH 3) are replicated.
  * J v and the per-view weights never leave the GPU that renders the view;
  * the only exchange per CG iteration is ONE all-reduce (sum) of the partial J^T W J v over the
    param-space vector; D v is added after the reduction, once;
  * J^T b and the loss are all-reduced once per LM step.
All-reduce results are bitwise identical on every rank, so the CG scalars (computed redundantly on
each rank, device-resident) stay consistent without a further broadcast.

`ShardedOperator` wraps any per-rank operator with the LMProblem protocol (gslm.lm.LMProblem on
the GPU, oracle.lm_ref.OracleLMProblem in the CPU tests).
"""
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_views(n_views, rank, world_size):
    """Contiguous block of view indices owned by `rank` (weak scaling: equal blocks)."""
    per = (n_views + world_size - 1) // world_size
    lo = min(rank * per, n_views)
    return list(range(lo, min(lo + per, n_views)))


class ShardedOperator:
    def __init__(self, local, group=None):
        self.local = local
        self.group = group
        self.rank, self.world_size = world()

    def __getattr__(self, name):  # layout, dot, zeros, stream, dot_scratch, views, ...
        return getattr(self.local, name)

    def _allreduce(self, t):
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def evaluate(self):
        loss = self.local.evaluate()
        self._allreduce(loss)
        self.local.loss = loss
        return loss

    @property
    def loss(self):
        return self.local.loss

    def rhs(self, out):
        self.local.rhs(out)
        return self._allreduce(out)

    def matvec_dot(self, v, y, dot_out, pre=None):
        kw = {} if pre is None else {"pre": pre}
        if self.world_size == 1:
            return self.local.matvec_dot(v, y, dot_out, **kw)
        # every rank holds the same s, p and scalars, so the deferred p update stays rank-local
        self.local.local_normal_matvec(v, y, damp=False, **kw)
        self._allreduce(y)
        self.local.damp_add(v, y)
        return False

    def matvec(self, v, y):
        self.matvec_dot(v, y, None)
        return y


def ShardedLMProblem(model, cams, bg, group=None, **kw):
    """LMProblem over this rank's views, wrapped for the cross-rank reductions."""
    from gslm.lm import LMProblem
    return ShardedOperator(LMProblem(model, cams, bg, **kw), group=group)
