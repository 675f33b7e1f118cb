"""Experiment: k_render_matvec's two passes timed apart at the bench config (1M Gaussians SH 3, one 1080p view; the
scene of tools/mv_ab.py), for the split profile VERDICT r04 asked for.  Each runs --reps times back to back on one
stream, so a kernel trace / PMC pass sees three kernels with the same scene and geometry:
  k_render_matvec<false>      the fused product as the CG loop runs it (J v pass -> u = 2 w (.) J v -> VJP pass)
  k_render_jv_wave            the J v pass alone (gslm_matvec_view_ex with jv_out: the same per-wave walk)
  k_render_bwd<false,false,2> the VJP pass alone: the seeded back-to-front pass of the LM step's J^T b (pixel_seed,
                              the same vjp_tile with the LM rows), driven by a per-pixel seed image
    python tools/exp/split_passes.py [--reps 20] [--out gpurun_out/split.json]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from gslm import _lib
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem
    from gslm.model import synthetic_gaussians
    from gslm.params import raw_gaussians
    dev = torch.device("cuda", 0)
    W, H, P = 1920, 1080, 1_000_000
    cams = orbit_cameras(1, W, H, seed=1)
    pert = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1)
    g2 = torch.Generator().manual_seed(2)
    with torch.no_grad():
        pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
        pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
        pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
    pert.to(dev)
    gp = LMProblem(pert, [c.to(dev) for c in cams], torch.zeros(3), device=dev)
    gp.evaluate()
    cams[0].original_image = gp.views[0].color.clamp(0, 1).clone()
    del gp, pert
    model = synthetic_gaussians(P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(dev)
    prob = LMProblem(model, cams, torch.zeros(3), device=dev)
    prob.evaluate()
    g = prob.rhs(prob.zeros())
    y = prob.zeros()
    prob.matvec(g, y)
    torch.cuda.synchronize()
    lib, check = _lib.lib, _lib.check
    vr = prob.views[0]
    graw = raw_gaussians(model)
    vs = prob.layout.grads_struct(g)
    ys = prob.layout.grads_struct(prob.zeros(), accumulate=True)
    jv = torch.zeros(3, H, W, device=dev)
    seed = torch.randn(3, H, W, generator=torch.Generator().manual_seed(7)).to(dev)

    def call(stages, jv_out=None, pixel_seed=None):
        opts = _lib.GslmMatvecOpts()
        opts.stages = stages
        opts.flags = 1 | prob.mv_flags
        if jv_out is not None:
            opts.jv_out = jv_out.data_ptr()
        if pixel_seed is not None:
            opts.pixel_seed = pixel_seed.data_ptr()
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(graw), ctypes.byref(vs),
                                      prob.weights[0].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                      vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                      ctypes.byref(ys), ctypes.byref(opts), prob.stream))

    legs = {"matvec": lambda: call(2), "jv_pass": lambda: call(2, jv_out=jv), "vjp_pass": lambda: call(2, pixel_seed=seed)}
    res = {"N": vr.N}
    for name, fn in legs.items():
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_ms"] = e0.elapsed_time(e1) / a.reps
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
