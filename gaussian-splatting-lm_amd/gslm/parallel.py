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
import ctypes
import math
import os

import torch
import torch.distributed as dist

from gslm.params import GROUPS, ParamLayout


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def collectives_on(world_size):
    """Whether the cross-rank collectives run: several ranks, or GSLM_FORCE_COLLECTIVES=1 with one rank -- the
    one-rank RCCL rehearsal on a one-GPU box (tests/test_gpu_rccl.py): every device-tensor collective of the
    multi-GPU path then goes through the backend (a copy with one rank) instead of the single-rank shortcut."""
    return world_size > 1 or os.environ.get("GSLM_FORCE_COLLECTIVES") == "1"


_NATIVE = {}


def native_comm(group=None, device=None):
    """The GSLM_COMM=native communicator of `group` (gslm.comm.NativeComm over the C-ABI RCCL entry points), made on
    first use -- a collective call, reached in the same program order on every rank -- or None (torch.distributed)."""
    from gslm import comm
    if not comm.enabled():
        return None
    key = id(group)
    if key not in _NATIVE:
        _NATIVE[key] = comm.NativeComm(group, device)
    return _NATIVE[key]


def close_native_comms():
    """Destroy the GSLM_COMM=native communicators, in creation order, after the device's work: call it on every rank
    at the same point of an orderly shutdown (before destroy_process_group) -- NativeComm.__del__ does not run at
    interpreter teardown."""
    if _NATIVE:
        torch.cuda.synchronize()
    for key in list(_NATIVE):
        _NATIVE.pop(key).close()


def _device_allreduce(t, group):
    """In-place sum over the ranks: the native communicator for device tensors under GSLM_COMM=native, otherwise
    torch.distributed (host-staged under gloo)."""
    nc = native_comm(group, t.device) if t.is_cuda else None
    if nc is not None:
        nc.all_reduce_(t)
    else:
        _staged(lambda x: dist.all_reduce(x, op=dist.ReduceOp.SUM, group=group), t)


def allreduce_loss(t, group=None):
    """Sum a device (or host) double over the ranks in place: the multi-GPU line search's validation loss, one
    8-byte all-reduce per evaluation (every rank gets the bitwise same sum, so every rank takes the same
    line-search decisions)."""
    if collectives_on(world()[1]):
        _device_allreduce(t.view(1), group)
    return t


def shard_views(n_views, rank, world_size):
    """Contiguous block of view indices owned by `rank` (weak scaling: equal blocks)."""
    per = (n_views + world_size - 1) // world_size
    lo = min(rank * per, n_views)
    return list(range(lo, min(lo + per, n_views)))


def _all_gather_into(out, inp, group=None):
    """out[r * len(inp):(r + 1) * len(inp)] = rank r's inp (dim 0 blocks)."""
    nc = native_comm(group, out.device) if out.is_cuda else None
    if nc is not None:
        nc.all_gather(out, inp)
        return
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
    supports_cg_ctl = True  # cgls_fused's device control block, passed to the local products

    @property
    def supports_exposure_zero(self):
        """Without collectives (one rank) the products are the local problem's, its exposure-slice skip included;
        the exchanges' products write y themselves."""
        return (not collectives_on(self.world_size)) and getattr(self.local, "supports_exposure_zero", False)

    def __init__(self, local, group=None, all_cams=None, exchange="auto"):
        self.local = local
        self.group = group
        self.rank, self.world_size = world()
        self.all_cams = all_cams
        self.exchange = self._pick_exchange(exchange)
        self._screen = None

    def _pick_exchange(self, mode):
        if not collectives_on(self.world_size) or mode == "allreduce":
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
        if collectives_on(self.world_size):
            _device_allreduce(t, self.group)
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

    def matvec_dot(self, v, y, dot_out, pre=None, cg_ctl=None, exposure_zero=False):
        kw = {} if pre is None else {"pre": pre}
        if cg_ctl is not None:
            kw["cg_ctl"] = cg_ctl
        if not collectives_on(self.world_size):
            if exposure_zero:
                kw["exposure_zero"] = True
            return self.local.matvec_dot(v, y, dot_out, **kw)
        if self.exchange == "screen":
            return self._matvec_screen(v, y, dot_out, pre, cg_ctl)
        # every rank holds the same s, p and scalars, so the deferred p update stays rank-local
        self.local.local_normal_matvec(v, y, damp=False, **kw)
        self._allreduce(y)
        self.local.damp_add(v, y)
        return False

    def _matvec_screen(self, v, y, dot_out, pre, cg_ctl=None):
        per = (len(self.all_cams) + self.world_size - 1) // self.world_size
        P = self.local.layout.P
        if self._screen is None:
            dev = v.device
            self._screen = torch.zeros(per, P, self.SCREEN_FLOATS, dtype=torch.float32, device=dev)
            self._screen_all = torch.empty(self.world_size * per, P, self.SCREEN_FLOATS, dtype=torch.float32,
                                           device=dev)
            self._views_all = self.local.views_for(self.all_cams, pad_to=self.world_size * per)
        self.local.screen_products(v, self._screen, pre=pre, cg_ctl=cg_ctl)
        _all_gather_into(self._screen_all, self._screen, self.group)
        self.local.gather_screen(self._views_all, self._screen_all, v, y, dot_out)
        return dot_out is not None

    def matvec(self, v, y, cg_ctl=None):
        self.matvec_dot(v, y, None, cg_ctl=cg_ctl)
        return y


def ShardedLMProblem(model, cams, bg, group=None, all_cams=None, exchange="auto", problem_cls=None, **kw):
    """LMProblem over this rank's views, wrapped for the cross-rank reductions.  all_cams (every
    rank's views, in rank order) enables the screen and Gaussian-sharded exchanges.  problem_cls: the per-rank
    problem (gslm.lm.LMProblem; the CPU tests pass oracle.lm_ref.OracleLMProblem).

    exchange: "gaussian" (GaussianShardedOperator: CG vectors sharded by Gaussian, two all-to-alls per
    product), "screen" / "allreduce" (ShardedOperator: vectors replicated), or "auto" -- "gaussian" when
    several ranks render the same number of views each with the disable_ssim residual, else
    ShardedOperator's own choice."""
    if problem_cls is None:
        from gslm.lm import LMProblem as problem_cls
    rank, n = world()
    if n > 1 or (all_cams is not None and len(all_cams) > 1) or exchange == "gaussian":
        # the SH-rest span is one view's: the global batch has several (and the Gaussian-sharded exchange
        # runs on the full layout)
        kw["sh_projection"] = False
    local = problem_cls(model, cams, bg, **kw)
    if exchange == "auto" and n > 1 and all_cams is not None and len(cams) >= 1 and \
            len(all_cams) == n * len(cams) and local.mask_xyz and not local.ssim:
        exchange = "gaussian"
    if exchange == "gaussian":
        if local.ssim or not local.mask_xyz:
            raise ValueError("the Gaussian-sharded exchange runs the disable_ssim product with xyz frozen")
        return GaussianShardedOperator(local, group=group, all_cams=all_cams if all_cams is not None else cams)
    return ShardedOperator(local, group=group, all_cams=all_cams, exchange=exchange)


def _slice_gaussians(g, lo, hi):
    """gslm_gaussians over Gaussians [lo, hi) of `g` (pointer offsets into the same leaves)."""
    from gslm import _lib
    out = _lib.GslmGaussians()
    ctypes.pointer(out)[0] = g
    out.P = hi - lo
    for name, w in (("means3D", 3), ("opacities", 1), ("scales", 3), ("rotations", 4)):
        p = getattr(g, name)
        if p:
            setattr(out, name, p + 4 * w * lo)
    if g.sh_dc:
        out.sh_dc = g.sh_dc + 4 * g.sh_dc_stride * lo
    if g.sh_rest:
        out.sh_rest = g.sh_rest + 4 * g.sh_rest_stride * lo
    return out


class GaussianShardedOperator:
    """The Gaussian-sharded exchange (exchange "gaussian").

    Views stay sharded as in ShardedOperator (rank r renders its block of `per` views), and in addition
    the Gaussians are cut into n contiguous shards: rank r owns Gaussians [lo, hi) = [r S, (r+1) S) of
    every CG vector (x, s, p, q and J^T b are shard-sized, `layout`) and the per-Gaussian work on them.
    Per product (matvec_dot), with b = (k, t) running over every view (k-th view of rank t):
      1. gslm_tangent_views: this shard's tangent render records for every view (the fused direction
         update p = s + beta p [, x += alpha p] on the shard first) -> trec[k][t][S][8];
      2. all_to_all per k: rank t receives every shard's records of its k-th view = a [P][8] table;
      3. RENDER | SCREEN with opts.trec_in: the view's fused JVP -> VJP tile pass and row sums -> [P][8];
      4. all_to_all per k: rank r receives the [S][8] slices of its shard from every view;
      5. gslm_gather_screen over the shard, every view's chain, + D v, <v, y> partial.
    The CG scalars are sums over shards: one small all-reduce each (DEL, GAMN [, monitor dots]) via
    `allreduce_scalars`, which gslm.lm.cgls_fused calls.  A rank receives (32 + 32) (n - 1) / n bytes per
    Gaussian per view instead of the screen all-gather's 32 (n - 1), and runs 1/n of the chains, gathers
    and vector algebra.  J^T b and the loss are all-reduced once per LM step (full layout), then sliced.

    With a per-rank operator that has no HIP views (oracle.lm_ref.OracleLMProblem in the CPU tests) the
    product falls back to all-gather v -> local sum_b 2 J_b^T W_b J_b v -> all-reduce -> slice + D v on
    the shard, which exercises the same shard layout, scalar reductions and gathers."""

    exchange = "gaussian"
    supports_exposure_zero = False  # (not forwarded to the local problem by __getattr__)
    supports_cg_ctl = True  # cgls_fused's device control block: the tile pass of a stopped solve returns at once

    def __init__(self, local, group=None, all_cams=None, emulate=None):
        """emulate=(rank, n): timing only -- run rank `rank` of an n-rank job's per-rank kernels in one process, each
        collective replaced by a local copy of the same shape (the products are NOT the n-rank job's; the kernels'
        sizes and control flow are: tile-pass decisions are frozen at the primal, independent of tangent values)."""
        self.local = local
        self.group = group
        self._emulate = emulate is not None
        self.rank, self.world_size = emulate if self._emulate else world()
        self._slot_index = {}  # allreduce_scalars' device index tensors, per slot tuple
        full = local.layout
        if getattr(full, "rest_projected", False):
            raise ValueError("the Gaussian-sharded exchange runs on the full SH-rest layout")
        self.full_layout = full
        self.P = full.P
        n = self.world_size
        self.S = max(1, -(-self.P // n))
        self.lo = min(self.rank * self.S, self.P)
        self.hi = min(self.lo + self.S, self.P)
        self.mask_xyz = getattr(local, "mask_xyz", True)
        self.device = getattr(local, "device", "cpu")
        self.kernel_path = hasattr(local, "views") and all_cams is not None
        self.all_cams = all_cams
        # SH-rest coordinates (gslm_rest_basis): with V <= GSLM_MAX_REST_VIEWS views in the job every CG iterate's
        # SH-rest group lies in the span of the V views' SH-rest directions, 3 V floats per Gaussian instead of
        # 3(K-1) in the shard's vectors (GSLM_SHARD_REST=full keeps the reference's layout)
        V = len(all_cams) if self.kernel_path else 0
        from gslm._lib import GSLM_MAX_REST_VIEWS
        self.rest_views = V if (full.K > 1 and 0 < V <= GSLM_MAX_REST_VIEWS and 3 * V < 3 * (full.K - 1)
                                and os.environ.get("GSLM_SHARD_REST", "coords") != "full") else 0
        self._rest_R = None  # [S][V (V + 1) / 2] factors, per geometry (evaluate)
        # the exposure group (zero in every LM iterate: J has no exposure column) lives on rank 0
        self.layout = ParamLayout(self.hi - self.lo, full.K, full.n_exposure if self.rank == 0 else 0,
                                  rest_views=self.rest_views)
        if self.kernel_path:
            self.per = len(local.views)
            if self.per < 1 or len(all_cams) != n * self.per:
                raise ValueError("gaussian exchange: every rank renders the same number (>= 1) of views "
                                 f"(got {self.per} here, {len(all_cams)} in all for {n} ranks)")
            # view order b = k n + t (the k-th view of rank t): the all-to-all blocks of one k are contiguous
            self.cams_kt = [all_cams[t * self.per + k] for k in range(self.per) for t in range(n)]
            self.views_kt = local.views_for(self.cams_kt)
            self._bufs = None
        if hasattr(local, "_damps"):
            self._damps = local._damps
        self._events = None  # stage_times: HIP events recorded between the product's stages

    def __getattr__(self, name):  # stream, dot_scratch, views, weights, model, ...
        return getattr(self.local, name)

    # ------------------------------------------------------------------ collectives
    def _allreduce(self, t):
        if collectives_on(self.world_size) and not self._emulate:
            _device_allreduce(t, self.group)
        return t

    def _native(self, t):
        return native_comm(self.group, t.device) if t.is_cuda else None

    def _all_to_all(self, out, inp):
        if not collectives_on(self.world_size) or self._emulate:
            out.copy_(inp)
            return
        nc = self._native(out)
        if nc is not None:
            nc.all_to_all(out, inp)
            return
        _staged(lambda o, i: dist.all_to_all_single(o, i, group=self.group), out, inp)

    def _overlap(self):
        """Whether the product's all-to-alls run asynchronously, overlapped with the tile passes of the other views
        (a device backend: RCCL runs the collective on its own stream, ordered after the kernels enqueued before it
        was issued; Work.wait() orders the compute stream after it).  gloo stages through the host: synchronous."""
        if self._emulate or not collectives_on(self.world_size) or os.environ.get("GSLM_OVERLAP", "1") == "0":
            return False
        from gslm import comm
        return dist.get_backend(self.group) == "nccl" or (comm.enabled() and
                                                         torch.device(self.device).type == "cuda")

    def _all_to_all_async(self, out, inp):
        """all_to_all_single issued without waiting: the Work to wait on, or None once done (synchronous paths)."""
        if self._overlap():
            nc = self._native(out)
            if nc is not None:
                return nc.all_to_all_async(out, inp)
            return dist.all_to_all_single(out, inp, group=self.group, async_op=True)
        self._all_to_all(out, inp)
        return None

    def allreduce_scalars(self, sc, slots):
        """Sum the CG scalars sc[slots] (device doubles, per-shard partials) over the ranks.  One slot (the CG
        loop's delta and gamma' without the residual monitor): in place on the 8-byte view, no gather / scatter
        kernels and no host-to-device index copy around the collective."""
        if not collectives_on(self.world_size) or self._emulate:
            return
        slots = tuple(slots)
        if len(slots) == 1:
            self._allreduce(sc[slots[0]:slots[0] + 1])
            return
        idx = self._slot_index.get(slots)
        if idx is None:
            idx = self._slot_index[slots] = torch.tensor(slots, device=sc.device)
        t = sc.index_select(0, idx)
        self._allreduce(t)
        sc.index_copy_(0, idx, t)

    # ------------------------------------------------------------------ shard <-> full layout
    def _group_rows(self, layout, vec):
        return {name: t.reshape(t.shape[0], math.prod(t.shape[1:])) for name, t in layout.views(vec).items()}

    # ------------------------------------------------------------------ SH-rest coordinates
    def _rest_args(self):
        from gslm import _lib
        from gslm.params import raw_gaussians
        gs = _slice_gaussians(raw_gaussians(self.local.model), self.lo, self.hi)
        vptr = ctypes.cast(ctypes.byref(self.views_kt, 0), ctypes.POINTER(_lib.GslmView))
        return gs, vptr

    def rest_basis(self):
        """gslm_rest_basis of this shard's Gaussians over the job's views (recomputed per geometry)."""
        if self._rest_R is None:
            from gslm._lib import check, lib
            V, S = self.rest_views, self.hi - self.lo
            self._rest_R = torch.zeros(max(1, S * V * (V + 1) // 2), dtype=torch.float32, device=self.device)
            gs, vptr = self._rest_args()
            check(lib.gslm_rest_basis(vptr, V, ctypes.byref(gs), self._rest_R.data_ptr(), self.local.stream),
                  "gslm_rest_basis")
        return self._rest_R

    def _rest_convert(self, mode, src, dst):
        """mode 0: coordinates [S][V][3] -> the reference's [S][K-1][3] rows; 1: the reverse (projection)."""
        from gslm._lib import check, lib
        if self.hi == self.lo:
            return
        R = self.rest_basis()
        gs, vptr = self._rest_args()
        check(lib.gslm_rest_coords(vptr, self.rest_views, ctypes.byref(gs), R.data_ptr(), mode, src.data_ptr(),
                                   src.shape[1], dst.data_ptr(), dst.shape[1], self.local.stream), "gslm_rest_coords")

    def shard(self, full_vec, out=None):
        """This rank's shard of a full-layout vector (SH-rest coordinates: its projection onto the views' span)."""
        out = self.zeros() if out is None else out
        src = self._group_rows(self.full_layout, full_vec)
        dst = self._group_rows(self.layout, out)
        for name in GROUPS:
            if name == "exposure":
                if self.layout.n_exposure:
                    dst[name].copy_(src[name])
                continue
            if name == "features_rest" and self.rest_views:
                self._rest_convert(1, src[name][self.lo:self.hi].contiguous(), dst[name])
                continue
            dst[name].copy_(src[name][self.lo:self.hi])
        return out

    def gather_full(self, vec):
        """The full-layout vector whose shards the ranks hold (all-gather of the Gaussian rows, rank 0's
        exposure group)."""
        n, S = self.world_size, self.S
        names = [g for g in GROUPS if g != "exposure"]
        rows = self._group_rows(self.layout, vec)
        if self.rest_views:
            full_rest = torch.zeros(self.hi - self.lo, 3 * (self.full_layout.K - 1), dtype=vec.dtype, device=vec.device)
            self._rest_convert(0, rows["features_rest"], full_rest)
            rows["features_rest"] = full_rest
        widths = [math.prod(self.full_layout.shapes[g][1:]) for g in names]
        F = sum(widths)
        pack = torch.zeros(S, F, dtype=vec.dtype, device=vec.device)
        c = 0
        for name, w in zip(names, widths):
            pack[:self.hi - self.lo, c:c + w] = rows[name]
            c += w
        allp = torch.empty(n * S, F, dtype=vec.dtype, device=vec.device)
        if self._emulate:
            allp.copy_(pack.repeat(n, 1))
        elif collectives_on(n):
            _all_gather_into(allp, pack, self.group)
        else:
            allp.copy_(pack)
        out = torch.zeros(self.full_layout.numel, dtype=vec.dtype, device=vec.device)
        dst = self._group_rows(self.full_layout, out)
        c = 0
        for name, w in zip(names, widths):
            dst[name].copy_(allp[:self.P, c:c + w])
            c += w
        e0, e1 = self.full_layout.offsets["exposure"]
        if self.layout.n_exposure:
            a0, a1 = self.layout.offsets["exposure"]
            out[e0:e1] = vec[a0:a1]
        if collectives_on(n) and not self._emulate:
            ex = out[e0:e1].clone()
            self._allreduce(ex)
            out[e0:e1] = ex
        return out

    def zeros(self):
        return torch.zeros(self.layout.numel, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ LM protocol
    @property
    def loss(self):
        return self.local.loss

    def evaluate(self):
        loss = self.local.evaluate()
        self._allreduce(loss)
        self.local.loss = loss
        if self.kernel_path:
            self._exchange_flags()
            self._rest_R = None  # the geometry (xyz) may have changed: SH-rest factors recomputed on first use
        return loss

    def rhs(self, out):
        full = self.local.rhs(self.local.zeros())
        self._allreduce(full)
        return self.shard(full, out)

    def vdot(self, a, b):
        """<a, b> over the whole vector (host float; the oracle CG of the CPU tests)."""
        t = (a.double() * b.double()).sum().reshape(1)
        self._allreduce(t)
        return float(t)

    def dot(self, a, b, out_slot, damped=False):
        """This shard's partial of <a, b> [damped] into a device double (cgls_fused all-reduces it)."""
        from gslm._lib import check, lib
        bounds, damps = self.layout.group_damp_arrays(self.local.damp) if damped else (None, None)
        check(lib.gslm_dot(a.data_ptr(), b.data_ptr(), bounds, damps, 7 if damped else 0, a.numel(),
                           self.local.dot_scratch.data_ptr(), out_slot, self.local.stream), "gslm_dot")

    def damp_add_shard(self, v, y):
        dv = self._group_rows(self.layout, v)
        dy = self._group_rows(self.layout, y)
        damp = self.local.damp
        for name in GROUPS:
            d = float(damp[name]) if isinstance(damp, dict) else float(damp)
            dy[name].add_(dv[name], alpha=d)
        return y

    def matvec(self, v, y, cg_ctl=None):
        self.matvec_dot(v, y, None, cg_ctl=cg_ctl)
        return y

    def matvec_dot(self, v, y, dot_out, pre=None, cg_ctl=None):
        if not self.kernel_path:
            if pre is not None:
                raise ValueError("the fused direction update needs the HIP operator")
            vf = self.gather_full(v)
            yf = self.local.local_normal_matvec(vf, torch.zeros_like(vf), damp=False)
            self._allreduce(yf)
            self.shard(yf, y)
            self.damp_add_shard(v, y)
            return False
        return self._matvec_kernels(v, y, dot_out, pre, cg_ctl)

    # ------------------------------------------------------------------ HIP path
    def _buffers(self):
        if self._bufs is None:
            n, S, per, dev = self.world_size, self.S, self.per, self.device
            self._bufs = dict(
                flags_local=torch.zeros(per, n * S, dtype=torch.int32, device=dev),
                flags=torch.zeros(per, n * S, dtype=torch.int32, device=dev),
                # the LM rows' compact tangent records: 8 floats per Gaussian (gslm_tangent_views with mask_xyz)
                trec_send=torch.zeros(per, n * S, 8, dtype=torch.float32, device=dev),
                trec_recv=torch.zeros(per, n * S, 8, dtype=torch.float32, device=dev),
                screen_send=torch.zeros(per, n * S, 8, dtype=torch.float32, device=dev),
                screen_recv=torch.zeros(per, n * S, 8, dtype=torch.float32, device=dev))
        return self._bufs

    def _exchange_flags(self):
        """Once per geometry: visibility / SH-clamp words of this shard's Gaussians in every view."""
        from gslm._lib import check, lib
        b = self._buffers()
        b["flags_local"].zero_()
        for k, vr in enumerate(self.local.views):
            check(lib.gslm_view_flags(vr.geom.data_ptr(), self.P, b["flags_local"][k].data_ptr(), self.local.stream),
                  "gslm_view_flags")
        for k in range(self.per):
            self._all_to_all(b["flags"][k], b["flags_local"][k])

    def _pre_opts(self, opts, v, pre):
        s, num, den = pre[:3]
        ss = self.layout.grads_struct(s)
        opts.xpby_s = ctypes.addressof(ss)
        opts.beta_num, opts.beta_den = num, den
        e0, e1 = self.layout.offsets["exposure"]
        if e1 > e0:
            opts.xpby_tail_v = v.data_ptr() + 4 * e0
            opts.xpby_tail_s = s.data_ptr() + 4 * e0
            opts.xpby_tail_n = e1 - e0
        if len(pre) > 3 and pre[3] is not None:
            x, anum, aden = pre[3:]
            opts.alpha_num, opts.alpha_den = anum, aden
            opts.xpby_x_offset = x.data_ptr() - v.data_ptr()
        return ss

    STAGES = ("tangent_views", "all_to_all_trec", "render_screen", "all_to_all_screen", "gather_screen")

    def stage_times(self, v, reps=10):
        """Per-stage time of this rank's product (ms, mean over `reps` products of direction v): HIP events on the
        product's stream between the five stages of _matvec_kernels (the all-to-alls include their wait)."""
        y = self.zeros()
        evs = []
        for _ in range(reps):
            self._events = [torch.cuda.Event(enable_timing=True) for _ in range(len(self.STAGES) + 1)]
            self.matvec_dot(v, y, None)
            evs.append(self._events)
            self._events = None
        torch.cuda.synchronize()
        out = {name: sum(e[k].elapsed_time(e[k + 1]) for e in evs) / reps for k, name in enumerate(self.STAGES)}
        out["total"] = sum(e[0].elapsed_time(e[-1]) for e in evs) / reps
        return out

    def _mark(self, k):
        if self._events is not None:
            self._events[k].record()

    def _matvec_kernels(self, v, y, dot_out, pre, cg_ctl=None):
        from gslm import _lib
        from gslm._lib import check, lib
        from gslm.params import raw_gaussians
        self._mark(0)
        loc = self.local
        b = self._buffers()
        n, S, per, P = self.world_size, self.S, self.per, self.P
        nv = n * per
        chunk = 16  # views per gslm_tangent_views / gslm_gather_screen call
        g = raw_gaussians(loc.model)
        gs = _slice_gaussians(g, self.lo, self.hi)
        vs = self.layout.grads_struct(v)
        ys = self.layout.grads_struct(y)
        vsz = ctypes.sizeof(_lib.GslmView)
        keep = []
        if pre is not None and self.hi == self.lo:
            # empty shard: the direction update has nothing here but rank 0's exposure tail, which an empty
            # shard never holds (rank 0 owns Gaussians whenever P > 0)
            pre = None
        # The views are ordered b = k n + t (the k-th view of rank t), so view group k = [k n, (k + 1) n) is one
        # all-to-all's worth.  With several views per rank the stages are pipelined over the groups (SURVEY 8(e)
        # "overlap the reduce-scatter of view k's contribution with view k+1's JVP/VJP"): the records of group k are
        # sent while group k+1's are written, view k renders while group k+1's records are in flight, and view k's
        # screen sums are sent while view k+1 renders.  Same kernels, same buffers, same order of every sum: the
        # products are bitwise those of the unpipelined schedule (GSLM_OVERLAP=0).
        R = self.rest_basis() if self.rest_views else None
        overlap = self._overlap() and per > 1
        tchunk = n if overlap else chunk  # one tangent call per view group, its all-to-all issued at once
        works = []
        # 1. tangent records of this shard for every view (direction update fused into the first call)
        for c0 in range(0, nv, tchunk):
            c1 = min(nv, c0 + tchunk)
            opts = None
            if (pre is not None and c0 == 0) or R is not None or cg_ctl is not None:
                opts = _lib.GslmMatvecOpts()
                opts.cg_ctl = cg_ctl  # a stopped solve's tangent kernel returns at once
            if pre is not None and c0 == 0:
                keep.append(self._pre_opts(opts, v, pre))
            if R is not None:
                opts.rest_basis, opts.rest_views, opts.view_base = R.data_ptr(), self.rest_views, c0
            vptr = ctypes.cast(ctypes.byref(self.views_kt, c0 * vsz), ctypes.POINTER(_lib.GslmView))
            check(lib.gslm_tangent_views(vptr, c1 - c0, ctypes.byref(gs), ctypes.byref(vs), int(self.mask_xyz),
                                         b["flags"].data_ptr() + 4 * c0 * S, S,
                                         b["trec_send"].data_ptr() + 32 * c0 * S, S,
                                         None if opts is None else ctypes.byref(opts), loc.stream),
                  "gslm_tangent_views")
            if overlap:  # 2. (pipelined) every shard's records of my view of group c0 / n
                k = c0 // n
                works.append(self._all_to_all_async(b["trec_recv"][k], b["trec_send"][k]))
        self._mark(1)
        # 2. every shard's records of my k-th view
        if not overlap:
            for k in range(per):
                self._all_to_all(b["trec_recv"][k], b["trec_send"][k])
        self._mark(2)
        # 3. render my views from the exchanged tables: per-Gaussian screen-space sums
        swork = []
        for k, vr in enumerate(loc.views):
            if overlap and works[k] is not None:
                works[k].wait()  # the compute stream waits for view k's table only
            opts = _lib.GslmMatvecOpts()
            opts.stages = 2 | 16  # RENDER | SCREEN
            opts.flags = 1 if vr.tail_clean else 0  # GSLM_MV_TAIL_CLEAN
            opts.screen_out = b["screen_send"][k].data_ptr()
            opts.trec_in = b["trec_recv"][k].data_ptr()
            opts.cg_ctl = cg_ctl
            check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                          loc.weights[k].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                          vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                          ctypes.byref(vs), ctypes.byref(opts), loc.stream), "gslm_matvec_view_ex")
            vr.tail_clean = True
            if overlap:  # 4. (pipelined) view k's screen sums leave while view k+1 renders
                swork.append(self._all_to_all_async(b["screen_recv"][k], b["screen_send"][k]))
        self._mark(3)
        # 4. my shard's slices of every view's screen sums
        if overlap:
            for w in swork:
                if w is not None:
                    w.wait()
        else:
            for k in range(per):
                self._all_to_all(b["screen_recv"][k], b["screen_send"][k])
        self._mark(4)
        # 5. every view's chain over my shard, + D v, <v, y>
        fuse = dot_out is not None and self.hi > self.lo
        for c0 in range(0, nv, chunk):
            c1 = min(nv, c0 + chunk)
            opts = _lib.GslmMatvecOpts()
            opts.stages = 7 | (8 if c0 == 0 else 0)
            opts.damp7 = self._damps if c0 == 0 else None
            opts.screen_stride = S
            opts.cg_ctl = cg_ctl  # as the tangent and tile kernels: nothing runs once the solve has stopped
            if R is not None:
                opts.rest_basis, opts.rest_views, opts.view_base = R.data_ptr(), self.rest_views, c0
            if fuse and c1 == nv:
                opts.dot_vy = dot_out
                opts.dot_scratch = loc.dot_scratch.data_ptr()
                opts.dot_scratch_bytes = loc.dot_scratch.numel() * 8
            vptr = ctypes.cast(ctypes.byref(self.views_kt, c0 * vsz), ctypes.POINTER(_lib.GslmView))
            check(lib.gslm_gather_screen(vptr, c1 - c0, ctypes.byref(gs), b["screen_recv"].data_ptr() + 32 * c0 * S,
                                         ctypes.byref(vs), ctypes.byref(ys), ctypes.byref(opts), loc.stream),
                  "gslm_gather_screen")
        e0, e1 = self.layout.offsets["exposure"]
        if e1 > e0:
            torch.mul(v[e0:e1], float(self._damps[6]), out=y[e0:e1])  # J has no exposure column
        self._mark(5)
        return fuse
