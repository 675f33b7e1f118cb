"""ORACLE -- test infrastructure only: the CPU baseline leg of bench.py.

Times the CPU restatement (oracle/torch_raster.py, PyTorch on the host cores) on a BOUNDED sample
of the benchmark workload and scales it to the full frame:

  * the per-Gaussian stages (activations, preprocess, binning, and their forward-AD / autograd
    passes) run on ALL P Gaussians and are timed as they are (t_gauss);
  * the per-tile blend (forward-AD, autograd forward + backward to the screen-space tensors) runs
    on `n_tiles` tiles spread uniformly over the frame and is timed on its own (t_tiles); the
    full-frame time is t_gauss + t_tiles * ntiles / n_tiles.

One "matvec" here is the reference's J v (torch forward-AD, solver_functions.py:83-99) plus
J^T u (autograd backward, solver_functions.py:101-132) of one view -- the CPU analogue of one
gslm_matvec_view.  The reference itself has no CPU renderer (gaussian_renderer/reference_render.py
wraps the CUDA `_orig` rasterizer), so kind = "port".
"""
import os
import time

import torch
import torch.autograd.forward_ad as fwAD

from oracle import torch_raster as tr


_SCREEN = ("xy", "conic", "opacity", "rgb")


def _preprocess_binning(model, st):
    m2 = torch.zeros_like(model.get_xyz)
    pre = tr.preprocess(model.get_xyz, m2, model.get_opacity, model.get_features, None, model.get_scaling,
                        model.get_rotation, None, st)
    pl, _, ranges = tr.binning(pre)
    return pre, pl, ranges


def _matvec_phases(model, cam, bg, tiles, tangents):
    """One J v + J^T (2 J v) of the view restricted to `tiles`, timed per phase (seconds):
    per-Gaussian work on all P (preprocess + binning under forward-AD, again under autograd, and the autograd
    backward from the screen-space tensors to the parameters) and per-tile work on the sampled tiles only
    (blend under forward-AD, blend + its backward to the screen-space tensors)."""
    st = tr.settings_from_camera(cam, bg, model.active_sh_degree)
    H, W = st.image_height, st.image_width
    names = ("_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity")
    saved = tuple(getattr(model, n) for n in names)
    # J v (forward mode, solver_functions.py:83-99)
    with torch.no_grad(), fwAD.dual_level():
        for n, p, t in zip(names, saved, tangents):
            setattr(model, n, fwAD.make_dual(p, t))
        try:
            t0 = time.perf_counter()
            pre, pl, ranges = _preprocess_binning(model, st)
            t1 = time.perf_counter()
            q = fwAD.unpack_dual(tr.blend_tiles(pre, pl, ranges, H, W, st.bg, tiles)).tangent
            t2 = time.perf_counter()
        finally:
            for n, p in zip(names, saved):
                setattr(model, n, p)
    q = torch.zeros(0, 3) if q is None else q
    # J^T (2 q) (reverse mode, solver_functions.py:101-132), the graph cut at the screen-space tensors
    model.zero_grad()
    t3 = time.perf_counter()
    pre, pl, ranges = _preprocess_binning(model, st)
    t4 = time.perf_counter()
    leaves = {k: pre[k].detach().requires_grad_(pre[k].requires_grad) for k in _SCREEN}
    color = tr.blend_tiles(dict(pre, **leaves), pl, ranges, H, W, st.bg, tiles)
    if color.requires_grad:
        (color * (2.0 * q)).sum().backward()
    t5 = time.perf_counter()
    outs = [(pre[k], leaves[k].grad) for k in _SCREEN if leaves[k].grad is not None]
    if outs:
        torch.autograd.backward([o for o, _ in outs], [g for _, g in outs])
    t6 = time.perf_counter()
    return (t1 - t0) + (t4 - t3) + (t6 - t5), (t2 - t1) + (t5 - t4)


def _forward_phases(model, cam, bg, tiles):
    st = tr.settings_from_camera(cam, bg, model.active_sh_degree)
    with torch.no_grad():
        t0 = time.perf_counter()
        pre, pl, ranges = _preprocess_binning(model, st)
        t1 = time.perf_counter()
        tr.blend_tiles(pre, pl, ranges, st.image_height, st.image_width, st.bg, tiles)
        t2 = time.perf_counter()
    return t1 - t0, t2 - t1


def cpu_matvec_rate(model, cam, bg, n_tiles=64, repeats=3, threads=None):
    """Seconds per full-frame matvec / forward on the host cores from a bounded sample: the per-Gaussian phases
    run on all P Gaussians and are timed as they are; the per-tile phases run on `n_tiles` tiles spread uniformly
    over the frame, timed on their own (no difference of two noisy totals) and scaled by ntiles / n_tiles.
    Each phase is the median of `repeats` runs.  Returns dict(matvec_s, forward_s, t_gauss, t_tiles, f_gauss,
    f_tiles, n_tiles, ntiles, threads, cpu_model)."""
    if threads:
        torch.set_num_threads(threads)
    th = torch.get_num_threads()
    W, H = cam.image_width, cam.image_height
    ntiles = ((W + 15) // 16) * ((H + 15) // 16)
    stride = max(1, ntiles // n_tiles)
    tiles = list(range(stride // 2, ntiles, stride))[:n_tiles]
    g = torch.Generator().manual_seed(3)
    tangents = [torch.randn(t.shape, generator=g) for t in
                (model._features_dc, model._features_rest, model._scaling, model._rotation, model._opacity)]

    def med(xs):
        return sorted(xs)[len(xs) // 2]

    mv = [_matvec_phases(model, cam, bg, tiles, tangents) for _ in range(repeats)]
    fw = [_forward_phases(model, cam, bg, tiles) for _ in range(repeats)]
    t_gauss, t_tiles = med([a for a, _ in mv]), med([b for _, b in mv])
    f_gauss, f_tiles = med([a for a, _ in fw]), med([b for _, b in fw])
    scale = ntiles / len(tiles)
    return dict(matvec_s=t_gauss + t_tiles * scale, forward_s=f_gauss + f_tiles * scale,
                t_gauss=t_gauss, t_tiles=t_tiles, f_gauss=f_gauss, f_tiles=f_tiles, n_tiles=len(tiles),
                ntiles=ntiles, threads=th, cpu_model=_cpu_model())


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_config0_times(repeats=5, threads=None):
    """BASELINE.json configs[0] (BASELINE.md "CPU baseline plan"): 2k synthetic Gaussians, SH 0, one 256x256 view,
    on the oracle renderer with no sampling or extrapolation: forward, JVP (forward-AD over every activated input,
    the tangent seed 3) and VJP (autograd with dL/dcolor ~ N(0,1), seed 4); 1 warm-up then the median of
    `repeats` timed runs of each.  Returns seconds per call and the thread count."""
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    if threads:
        torch.set_num_threads(threads)
    model = synthetic_gaussians(2000, 0, seed=0, s0=0.005)
    cam = orbit_cameras(1, 256, 256, seed=1)[0]
    st = tr.settings_from_camera(cam, torch.zeros(3), 0)
    with torch.no_grad():
        a = dict(means3D=model.get_xyz.detach().clone(), opacities=model.get_opacity.detach().clone(),
                 scales=model.get_scaling.detach().clone(), rotations=model.get_rotation.detach().clone(),
                 shs=model.get_features.detach().clone())
    g3 = torch.Generator().manual_seed(3)
    tang = {k: torch.randn(v.shape, generator=g3) for k, v in a.items()}
    dcol = torch.randn(3, 256, 256, generator=torch.Generator().manual_seed(4))

    def call(inp):
        return tr.rasterize(inp["means3D"], torch.zeros_like(a["means3D"]), inp["opacities"], st, shs=inp["shs"],
                            scales=inp["scales"], rotations=inp["rotations"])[0]

    def fwd():
        with torch.no_grad():
            call(a)

    def jvp():
        with torch.no_grad(), fwAD.dual_level():
            fwAD.unpack_dual(call({k: fwAD.make_dual(v, tang[k]) for k, v in a.items()})).tangent

    def vjp():
        leaves = {k: v.clone().requires_grad_(True) for k, v in a.items()}
        (call(leaves) * dcol).sum().backward()

    out = {}
    for name, fn in (("forward", fwd), ("jvp", jvp), ("vjp", vjp)):
        fn()
        ts = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        out[name + "_s"] = sorted(ts)[len(ts) // 2]
    out["threads"] = torch.get_num_threads()
    return out


def host_info():
    """os.cpu_count(), the CPU model and the cores this process may run on (the GPU box's CPU share)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"os_cpu_count": os.cpu_count(), "affinity_cpus": affinity, "cpu_model": _cpu_model(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_config1_forward(repeats=5, threads=None, P=100_000, W=1920, H=1080, s0=0.005):
    """BASELINE.json configs[1]'s forward on the host cores, timed whole (SURVEY 8(d) "CPU baseline": config 2's
    forward on the CPU when it finishes in minutes): P = 100k synthetic Gaussians, SH 3, one 1080p view through the
    full oracle rasterizer (preprocess, binning, every tile's blend), no sampling or extrapolation; 1 warm-up then
    the median of `repeats`.  Returns seconds per forward, Mpix/s and the thread count."""
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    if threads:
        torch.set_num_threads(threads)
    model = synthetic_gaussians(P, 3, seed=0, s0=s0)
    cam = orbit_cameras(1, W, H, seed=1)[0]
    st = tr.settings_from_camera(cam, torch.zeros(3), 3)
    with torch.no_grad():
        a = dict(means3D=model.get_xyz, opacities=model.get_opacity, scales=model.get_scaling,
                 rotations=model.get_rotation, shs=model.get_features)

        def fwd():
            tr.rasterize(a["means3D"], torch.zeros_like(a["means3D"]), a["opacities"], st, shs=a["shs"],
                         scales=a["scales"], rotations=a["rotations"])

        fwd()
        ts = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            fwd()
            ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    return {"forward_s": t, "mpix_s": W * H / t / 1e6, "threads": torch.get_num_threads(), "repeats": repeats,
            "config": f"BASELINE configs[1] forward: {P} Gaussians SH3, one {W}x{H} view, oracle rasterizer timed "
                      "whole (1 warm-up + median)"}
