"""View-sharded LM operator over torch.distributed (RCCL over xGMI on MI355X; gloo for CPU tests).

The reference has no distributed code: its LinearSolverFunctions renders a view batch
serially on one GPU (solver_functions.py:38-41,88-93,110-121).  Here every rank owns a disjoint
block of the camera batch; the parameters theta (59 fp32 per Gaussian at SH 3) are replicated.
  * J v and the per-view weights never leave the GPU that renders the view;
  * per CG iteration ONE collective combines the ranks' partial products:
      - "screen" exchange (default when it moves less data): ranks all-gather 8 floats per
        (view, Gaussian) of screen-space sums and every rank applies all views' chains itself
        (gslm_gather_screen, exchange.hip) -- at 1 view per GPU that is 32 B/Gaussian/rank instead
        of the 2 (n-1)/n * 236 B/Gaussian an all-reduce of the param-space vector moves;
      - "allreduce": one all-reduce (sum) of the partial J^T W J v over the param-space vector,
        D v added after the reduction, once;
  * J^T b and the loss are all-reduced once per LM step.
Collective results are bitwise identical on every rank (and the screen gather sums the views in
index order on every rank), so the CG scalars, computed redundantly on each rank in device memory,
stay consistent without a further broadcast.

`ShardedOperator` wraps any per-rank operator with the LMProblem protocol (gslm.lm.LMProblem on
the GPU, oracle.lm_ref.OracleLMProblem in the CPU tests; the screen exchange needs the former).
"""
import torch
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


def _all_gather_into(out, inp, group=None):
    """out[r * len(inp):(r + 1) * len(inp)] = rank r's inp (dim 0 blocks)."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    ho = out.cpu() if out.is_cuda else out
    hi = inp.cpu() if inp.is_cuda else inp
    dist.all_gather(list(ho.chunk(dist.get_world_size(group))), hi, group=group)
    if out.is_cuda:
        out.copy_(ho)


def _staged(fn, *tensors):
    """gloo has no device all_gather: run the collective on host copies of CUDA tensors (tests)."""
    if tensors[0].is_cuda and dist.get_backend() == "gloo":
        host = [t.cpu() for t in tensors]
        fn(*host)
        for t, h in zip(tensors, host):
            t.copy_(h)
    else:
        fn(*tensors)


class ShardedOperator:
    SCREEN_FLOATS = 8  # per (view, Gaussian) in the screen exchange

    def __init__(self, local, group=None, all_cams=None, exchange="auto"):
        self.local = local
        self.group = group
        self.rank, self.world_size = world()
        self.all_cams = all_cams
        self.exchange = self._pick_exchange(exchange)
        self._screen = None

    def _pick_exchange(self, mode):
        if self.world_size == 1 or mode == "allreduce":
            return "allreduce"
        capable = self.all_cams is not None and getattr(self.local, "mask_xyz", False) and \
            hasattr(self.local, "screen_products") and not getattr(self.local, "ssim", False)
        if mode == "screen":
            if not capable:
                raise ValueError("screen exchange needs the GPU LMProblem, mask_xyz=True and all_cams")
            return "screen"
        if not capable:
            return "allreduce"
        per = (len(self.all_cams) + self.world_size - 1) // self.world_size
        F = self.local.layout.floats_per_gaussian
        # per rank and Gaussian an all-gather receives (n - 1) per 8 floats, a ring all-reduce moves
        # 2 (n - 1) / n F: the screen exchange wins while n per 8 < 2 F (up to 14 views at SH 3)
        return "screen" if self.world_size * per * self.SCREEN_FLOATS < 2 * F else "allreduce"

    def __getattr__(self, name):  # layout, dot, zeros, stream, dot_scratch, views, ...
        return getattr(self.local, name)

    def _allreduce(self, t):
        if self.world_size > 1:
            _staged(lambda x: dist.all_reduce(x, op=dist.ReduceOp.SUM, group=self.group), t)
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
        if self.exchange == "screen":
            return self._matvec_screen(v, y, dot_out, pre)
        # every rank holds the same s, p and scalars, so the deferred p update stays rank-local
        self.local.local_normal_matvec(v, y, damp=False, **kw)
        self._allreduce(y)
        self.local.damp_add(v, y)
        return False

    def _matvec_screen(self, v, y, dot_out, pre):
        per = (len(self.all_cams) + self.world_size - 1) // self.world_size
        P = self.local.layout.P
        if self._screen is None:
            dev = v.device
            self._screen = torch.zeros(per, P, self.SCREEN_FLOATS, dtype=torch.float32, device=dev)
            self._screen_all = torch.empty(self.world_size * per, P, self.SCREEN_FLOATS, dtype=torch.float32,
                                           device=dev)
            self._views_all = self.local.views_for(self.all_cams, pad_to=self.world_size * per)
        self.local.screen_products(v, self._screen, pre=pre)
        _all_gather_into(self._screen_all, self._screen, self.group)
        self.local.gather_screen(self._views_all, self._screen_all, v, y, dot_out)
        return dot_out is not None

    def matvec(self, v, y):
        self.matvec_dot(v, y, None)
        return y


def ShardedLMProblem(model, cams, bg, group=None, all_cams=None, exchange="auto", **kw):
    """LMProblem over this rank's views, wrapped for the cross-rank reductions.  all_cams (every
    rank's views, in rank order) enables the screen exchange."""
    from gslm.lm import LMProblem
    if world()[1] > 1 or (all_cams is not None and len(all_cams) > 1):
        kw["sh_projection"] = False  # the SH-rest span is one view's: the global batch has several
    return ShardedOperator(LMProblem(model, cams, bg, **kw), group=group, all_cams=all_cams, exchange=exchange)
