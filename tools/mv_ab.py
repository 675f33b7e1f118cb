"""A/B harness for the tile-pass kernels at the bench config (1M Gaussians SH3, one 1080p view).

    GSLM_LIB=<path to libgslm.so> python tools/mv_ab.py <tag> [--reps N] [--out DIR]

Builds bench.py's scene (seeded model, GT = render of the perturbed model), runs one LM problem with the
single-view SH-rest projection, and reports HIP-event times of: the fused (J^T J + D) p product's stages
(tangent, k_render_matvec, gather), a full CG iteration, and the full forward (preprocess + sort + binning +
blend).  Saves the product y = A g and the forward image to DIR/<tag>.pt so builds can be compared
(`python tools/mv_ab.py --compare DIR tagA tagB ...`)."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]

import torch  # noqa: E402


def compare(out_dir, tags):
    base = torch.load(os.path.join(out_dir, tags[0] + ".pt"), weights_only=True)
    for t in tags[1:]:
        d = torch.load(os.path.join(out_dir, t + ".pt"), weights_only=True)
        for k in base:
            a, b = base[k].double(), d[k].double()
            rel = float((a - b).abs().max() / max(float(a.abs().max()), 1e-30))
            print(f"{t} vs {tags[0]}: {k} max rel diff {rel:.3e} equal={torch.equal(base[k], d[k])}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag", nargs="?")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="/tmp/gslm_ab")
    ap.add_argument("--compare", nargs="+")
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--full", action="store_true", help="the reference's full SH-rest layout (no projection)")
    ap.add_argument("--stagger", type=int, nargs="*", default=[],
                    help="also time the gather with its output vector offset by K floats (HBM channel alignment)")
    ap.add_argument("--ramp", type=int, default=0, help="also time N single CG iterations back to back (clock ramp)")
    ap.add_argument("--cg-scan", type=int, nargs="*", default=[],
                    help="also time cgls_fused calls of K iterations: wall clock per iteration and the host's enqueue time")
    a = ap.parse_args()
    if a.compare:
        compare(a.compare[0], a.compare[1:])
        return
    from gslm import _lib
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem, cgls_fused
    from gslm.model import synthetic_gaussians
    from gslm.params import raw_gaussians
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    cams = orbit_cameras(1, W, H, seed=1)
    pert = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1)
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
    model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(dev)
    prob = LMProblem(model, cams, torch.zeros(3), device=dev, sh_projection=False if a.full else "auto")
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

    def stage(mask, jv_out=False):
        opts = _lib.GslmMatvecOpts()
        opts.stages = mask | (8 if mask == 4 else 0)
        if jv_out:
            opts.jv_out = jv.data_ptr()
        opts.flags = 1 | prob.mv_flags
        opts.damp7 = prob._damps if mask == 4 else None
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(graw), ctypes.byref(vs),
                                      prob.weights[0].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                      vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                      ctypes.byref(ys), ctypes.byref(opts), prob.stream))

    def ev(fn, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    res = {"tag": a.tag, "N": vr.N}
    res["tangent_ms"] = ev(lambda: stage(1), a.reps)
    res["render_matvec_ms"] = ev(lambda: stage(2), a.reps)
    res["gather_ms"] = ev(lambda: stage(4), a.reps)
    for k in a.stagger:
        ybuf = torch.zeros(prob.layout.numel + k, dtype=torch.float32, device=dev)
        vbuf = torch.zeros(prob.layout.numel + 2 * k, dtype=torch.float32, device=dev)
        vbuf[2 * k:].copy_(g)
        ys_save, vs_save = ys, vs
        ys = prob.layout.grads_struct(ybuf[k:], accumulate=True)
        res[f"gather_ms_ystagger{k}"] = ev(lambda: stage(4), a.reps)
        vs = prob.layout.grads_struct(vbuf[2 * k:])
        res[f"gather_ms_yvstagger{k}"] = ev(lambda: stage(4), a.reps)
        ys, vs = ys_save, vs_save
        del ybuf, vbuf
    res["jv_ms"] = ev(lambda: stage(2, jv_out=True), a.reps)
    # k_render_matvec as the CG loop runs it: between the tangent and gather passes, which stream the vectors
    # through the caches (the back-to-back timing above replays it with its inputs cache-warm)
    evs = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stage(1)
        e0.record()
        stage(2)
        e1.record()
        stage(4)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    res["render_matvec_loop_ms"] = sum(e0.elapsed_time(e1) for e0, e1 in evs) / a.reps
    cgls_fused(prob, g, max_iter=2, restart_iter=2, check_every=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cgls_fused(prob, g, max_iter=a.reps, restart_iter=a.reps, check_every=False)
    torch.cuda.synchronize()
    res["cg_iter_ms"] = 1e3 * (time.perf_counter() - t0) / a.reps
    for k in a.cg_scan:
        cgls_fused(prob, g, max_iter=3, restart_iter=3, check_every=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cgls_fused(prob, g, max_iter=k, restart_iter=k, check_every=False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[f"cg{k}_iter_ms"] = round(1e3 * (t2 - t0) / k, 4)
        res[f"cg{k}_enqueue_ms_per_iter"] = round(1e3 * (t1 - t0) / k, 4)
    if a.ramp:
        # per-iteration device time of N consecutive CG iterations, launched without host syncs
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.ramp)]
        for e0, e1 in evs:
            e0.record()
            cgls_fused(prob, g, max_iter=1, restart_iter=1, check_every=False)
            e1.record()
        torch.cuda.synchronize()
        ts = [e0.elapsed_time(e1) for e0, e1 in evs]
        res["ramp_ms"] = [round(t, 4) for t in ts[:5]] + [round(sum(ts[i:i + 25]) / len(ts[i:i + 25]), 4)
                                                          for i in range(5, len(ts), 25)]
    vr.forward(graw, prob.stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        vr.forward(graw, prob.stream)
    torch.cuda.synchronize()
    res["forward_ms"] = 1e3 * (time.perf_counter() - t0) / a.reps
    os.makedirs(a.out, exist_ok=True)
    torch.save({"y": y.cpu(), "color": vr.color.cpu(), "jv": jv.cpu(), "image": vr.image.cpu()}, os.path.join(a.out, a.tag + ".pt"))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
