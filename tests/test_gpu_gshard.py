"""GPU parity of the Gaussian-sharded exchange's building blocks (include/gslm.h, "Gaussian-sharded exchange").

On the reference solver's golden scene (tests/golden/solver_golden.npz, several views) the product is
split the way a rank of the Gaussian-sharded exchange computes it, with the Gaussians cut into two
shards inside one process:
  gslm_view_flags -> gslm_tangent_views per shard -> RENDER | SCREEN with opts.trec_in
must reproduce the unsharded screen rows of LMProblem.screen_products (TANGENT | RENDER | SCREEN), and
gslm_gather_screen over each shard (strided screen, opts.screen_stride = P) must reproduce the
unsharded gather. Same chain_jvp / gather code on both sides, so the tolerance is 1e-6 of the max.
"""
import ctypes

import numpy as np
import pytest
import torch

from test_gpu_lm import _load

pytestmark = pytest.mark.gpu

_G_WIDTH = {"means3D": 3, "opacities": 1, "scales": 3, "rotations": 4, "sh_dc": 3}


def _slice(struct, cls, s0, s1, rest_w, with_p):
    out = cls()
    ctypes.pointer(out)[0] = struct  # copy every field
    for k, w in _G_WIDTH.items():
        p = getattr(struct, k)
        if p:
            setattr(out, k, p + 4 * w * s0)
    if struct.sh_rest:
        out.sh_rest = struct.sh_rest + 4 * rest_w * s0
    if with_p:
        out.P = s1 - s0
    return out


def test_gaussian_sharded_product_matches_unsharded():
    from gslm import _lib
    from gslm.lm import LMProblem, MV_TAIL_CLEAN, STAGE_ALL, STAGE_OVERWRITE, check
    from gslm.params import raw_gaussians
    lib = _lib.lib
    d, m, cams = _load()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    prob.rhs(prob.zeros())
    P, n = m._xyz.shape[0], len(prob.views)
    K = 1 + m._features_rest.shape[1]
    R = 3 * (K - 1)
    gen = torch.Generator(device="cpu").manual_seed(0)
    v = (torch.randn(prob.zeros().numel(), generator=gen) * 1e-2).cuda()
    x0, x1 = prob.layout.offsets["xyz"]
    v[x0:x1] = 0
    ref = torch.zeros(n, P, 8, device="cuda")
    prob.screen_products(v, ref)

    flags = torch.zeros(n, P, dtype=torch.int32, device="cuda")
    for b, vr in enumerate(prob.views):
        check(lib.gslm_view_flags(vr.geom.data_ptr(), P, flags[b].data_ptr(), prob.stream), "gslm_view_flags")
    views = prob.views_for(cams)
    g = raw_gaussians(m)
    vs = prob.layout.grads_struct(v)
    trec = torch.zeros(n, P, 8, device="cuda")  # the LM rows' compact records (mask_xyz)
    cut = (P * 3) // 7  # not a multiple of the 256-Gaussian block
    shards = [(0, cut), (cut, P)]
    for s0, s1 in shards:
        gs = _slice(g, _lib.GslmGaussians, s0, s1, R, True)
        vss = _slice(vs, _lib.GslmGrads, s0, s1, R, False)
        check(lib.gslm_tangent_views(views, n, ctypes.byref(gs), ctypes.byref(vss), 1,
                                     flags.data_ptr() + 4 * s0, P, trec.data_ptr() + 32 * s0, P, None,
                                     prob.stream), "gslm_tangent_views")
    got = torch.zeros(n, P, 8, device="cuda")
    for b, vr in enumerate(prob.views):
        opts = _lib.GslmMatvecOpts()
        opts.stages = 2 | 16  # RENDER | SCREEN
        opts.flags = MV_TAIL_CLEAN if vr.tail_clean else 0
        opts.screen_out = got[b].data_ptr()
        opts.trec_in = trec[b].data_ptr()
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                      prob.weights[b].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                      vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                      ctypes.byref(vs), ctypes.byref(opts), prob.stream), "gslm_matvec_view_ex")
    torch.cuda.synchronize()
    r, o = ref.cpu().numpy(), got.cpu().numpy()
    assert np.array_equal(r[..., 7].view(np.uint32), o[..., 7].view(np.uint32))
    assert (r[..., 7].view(np.uint32) >> 31).sum() > 0
    scale = max(np.abs(r[..., :7]).max(), 1e-12)
    assert np.abs(r[..., :7] - o[..., :7]).max() <= 1e-6 * scale

    # gather over each shard from the strided screen rows == the unsharded gather
    y_ref = prob.gather_screen(views, ref, v, prob.zeros())
    y = prob.zeros()
    ys = prob.layout.grads_struct(y)
    for s0, s1 in shards:
        gs = _slice(g, _lib.GslmGaussians, s0, s1, R, True)
        vss = _slice(vs, _lib.GslmGrads, s0, s1, R, False)
        yss = _slice(ys, _lib.GslmGrads, s0, s1, R, False)
        opts = _lib.GslmMatvecOpts()
        opts.stages = STAGE_ALL | STAGE_OVERWRITE
        opts.damp7 = prob._damps
        opts.screen_stride = P
        check(lib.gslm_gather_screen(views, n, ctypes.byref(gs), ref[0, s0].data_ptr(), ctypes.byref(vss),
                                     ctypes.byref(yss), ctypes.byref(opts), prob.stream), "gslm_gather_screen")
    e0, e1 = prob.layout.offsets["exposure"]
    torch.mul(v[e0:e1], float(prob._damps[6]), out=y[e0:e1])
    torch.cuda.synchronize()
    a, b = y.cpu().numpy(), y_ref.cpu().numpy()
    assert np.abs(a - b).max() <= 1e-6 * max(np.abs(b).max(), 1e-12)


def _xpby_opts(layout, s, v, x, sc, tail):
    """gslm_matvec_opts with the fused direction update v = s + beta v and the deferred x += alpha v
    (beta = sc[0] / sc[1], alpha = sc[2] / sc[3]); the flat exposure tail only when `tail`."""
    from gslm import _lib
    opts = _lib.GslmMatvecOpts()
    ss = layout.grads_struct(s)
    opts.xpby_s = ctypes.addressof(ss)
    opts.beta_num, opts.beta_den = sc.data_ptr(), sc.data_ptr() + 8
    opts.alpha_num, opts.alpha_den = sc.data_ptr() + 16, sc.data_ptr() + 24
    opts.xpby_x_offset = x.data_ptr() - v.data_ptr()
    if tail:
        e0, e1 = layout.offsets["exposure"]
        opts.xpby_tail_v = v.data_ptr() + 4 * e0
        opts.xpby_tail_s = s.data_ptr() + 4 * e0
        opts.xpby_tail_n = e1 - e0
    return opts, ss


def test_tangent_views_fused_direction_update_matches_tangent_stage():
    """gslm_tangent_views with the fused p = s + beta p and x += alpha p, run per shard on private p / x
    copies (the shard cut inside a 256-Gaussian block, the tail with the first shard only), equals the
    TANGENT stage of gslm_matvec_view_ex with the same update: p and x bitwise, and the screen rows rendered
    from the exchanged records equal the unsharded product's."""
    from gslm import _lib
    from gslm.lm import MV_TAIL_CLEAN, check
    from gslm.params import raw_gaussians
    lib = _lib.lib
    d, m, cams = _load()
    from gslm.lm import LMProblem
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    prob.rhs(prob.zeros())
    P, n = m._xyz.shape[0], len(prob.views)
    K = 1 + m._features_rest.shape[1]
    R = 3 * (K - 1)
    gen = torch.Generator(device="cpu").manual_seed(5)
    lay = prob.layout
    x0, x1 = lay.offsets["xyz"]

    def vec():
        t = torch.randn(lay.numel, generator=gen) * 1e-2
        t[x0:x1] = 0
        return t.cuda()
    s, p0, xv0 = vec(), vec(), vec()
    sc = torch.tensor([0.7, 1.3, 0.25, 0.9], dtype=torch.float64, device="cuda")
    g = raw_gaussians(m)
    views = prob.views_for(cams)

    # reference: the TANGENT stage of the first view's product carries the update
    p_ref, x_ref = p0.clone(), xv0.clone()
    ref = torch.zeros(n, P, 8, device="cuda")
    for b, vr in enumerate(prob.views):
        vs = lay.grads_struct(p_ref)
        opts, keep = _xpby_opts(lay, s, p_ref, x_ref, sc, True) if b == 0 else (_lib.GslmMatvecOpts(), None)
        opts.stages = 1 | 2 | 16
        opts.flags = MV_TAIL_CLEAN if vr.tail_clean else 0
        opts.screen_out = ref[b].data_ptr()
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                      prob.weights[b].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                      vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                      ctypes.byref(vs), ctypes.byref(opts), prob.stream), "gslm_matvec_view_ex")
        vr.tail_clean = True

    flags = torch.zeros(n, P, dtype=torch.int32, device="cuda")
    for b, vr in enumerate(prob.views):
        check(lib.gslm_view_flags(vr.geom.data_ptr(), P, flags[b].data_ptr(), prob.stream), "gslm_view_flags")
    trec = torch.zeros(n, P, 8, device="cuda")
    cut = (P * 3) // 7
    shards = [(0, cut), (cut, P)]
    p_out, x_out = p0.clone(), xv0.clone()
    for si, (s0, s1) in enumerate(shards):
        p_sh, x_sh = p0.clone(), xv0.clone()  # this shard's private copies (a rank's vectors)
        opts, keep = _xpby_opts(lay, s, p_sh, x_sh, sc, si == 0)
        # the shard's view of s as well: its pointers must sit at the same Gaussian offset as v's
        keep_s = _slice(keep, _lib.GslmGrads, s0, s1, R, False)
        opts.xpby_s = ctypes.addressof(keep_s)
        gs = _slice(g, _lib.GslmGaussians, s0, s1, R, True)
        vss = _slice(lay.grads_struct(p_sh), _lib.GslmGrads, s0, s1, R, False)
        check(lib.gslm_tangent_views(views, n, ctypes.byref(gs), ctypes.byref(vss), 1,
                                     flags.data_ptr() + 4 * s0, P, trec.data_ptr() + 32 * s0, P, ctypes.byref(opts),
                                     prob.stream), "gslm_tangent_views")
        torch.cuda.synchronize()
        pv, xv, po, xo = lay.views(p_sh), lay.views(x_sh), lay.views(p_out), lay.views(x_out)
        for name in ("features_dc", "features_rest", "scaling", "rotation", "opacity"):
            po[name][s0:s1] = pv[name][s0:s1]
            xo[name][s0:s1] = xv[name][s0:s1]
        if si == 0:
            po["exposure"].copy_(pv["exposure"])
            xo["exposure"].copy_(xv["exposure"])
    torch.cuda.synchronize()
    assert torch.equal(p_out, p_ref)
    assert torch.equal(x_out, x_ref)
    assert not torch.equal(p_ref, p0)  # the update ran
    got = torch.zeros(n, P, 8, device="cuda")
    for b, vr in enumerate(prob.views):
        opts = _lib.GslmMatvecOpts()
        opts.stages = 2 | 16
        opts.flags = MV_TAIL_CLEAN
        opts.screen_out = got[b].data_ptr()
        opts.trec_in = trec[b].data_ptr()
        vs = lay.grads_struct(p_ref)
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                      prob.weights[b].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                      vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                      ctypes.byref(vs), ctypes.byref(opts), prob.stream), "gslm_matvec_view_ex")
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("mask_xyz", [1, 0])
def test_render_gather_from_trec_in_matches_full_product(mask_xyz):
    """RENDER | GATHER reading an exchanged tangent table (opts.trec_in) equals TANGENT | RENDER | GATHER, on
    the LM rows (mask_xyz = 1) and on the xyz-including template (mask_xyz = 0, k_render_matvec<true>)."""
    from gslm import _lib
    from gslm.lm import LMProblem, check
    from gslm.params import raw_gaussians
    lib = _lib.lib
    d, m, cams = _load()
    prob = LMProblem(m, cams[:1], torch.zeros(3), mask_xyz=bool(mask_xyz))
    prob.evaluate()
    P = m._xyz.shape[0]
    vr = prob.views[0]
    lay = prob.layout
    gen = torch.Generator(device="cpu").manual_seed(9)
    v = (torch.randn(lay.numel, generator=gen) * 1e-2).cuda()
    e0, e1 = lay.offsets["exposure"]
    v[e0:e1] = 0
    if mask_xyz:
        x0, x1 = lay.offsets["xyz"]
        v[x0:x1] = 0
    g = raw_gaussians(m)
    vs = lay.grads_struct(v)

    def product(stages, trec_in=None):
        y = prob.zeros()
        ys = lay.grads_struct(y)
        opts = _lib.GslmMatvecOpts()
        opts.stages = stages | 8
        opts.trec_in = trec_in
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(g), ctypes.byref(vs),
                                      prob.weights[0].data_ptr(), mask_xyz, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                      vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                      ctypes.byref(ys), ctypes.byref(opts), prob.stream), "gslm_matvec_view_ex")
        return y
    ref = product(7)
    flags = torch.zeros(P, dtype=torch.int32, device="cuda")
    check(lib.gslm_view_flags(vr.geom.data_ptr(), P, flags.data_ptr(), prob.stream), "gslm_view_flags")
    trec = torch.zeros(P, 8 if mask_xyz else 12, device="cuda")
    views = prob.views_for(cams[:1])
    check(lib.gslm_tangent_views(views, 1, ctypes.byref(g), ctypes.byref(vs), mask_xyz, flags.data_ptr(), P,
                                 trec.data_ptr(), P, None, prob.stream), "gslm_tangent_views")
    got = product(2 | 4, trec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
