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
    trec = torch.zeros(n, P, 12, device="cuda")
    cut = (P * 3) // 7  # not a multiple of the 256-Gaussian block
    shards = [(0, cut), (cut, P)]
    for s0, s1 in shards:
        gs = _slice(g, _lib.GslmGaussians, s0, s1, R, True)
        vss = _slice(vs, _lib.GslmGrads, s0, s1, R, False)
        check(lib.gslm_tangent_views(views, n, ctypes.byref(gs), ctypes.byref(vss), 1,
                                     flags.data_ptr() + 4 * s0, P, trec.data_ptr() + 48 * s0, P, None,
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
