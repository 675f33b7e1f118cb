"""ORACLE -- test infrastructure only: the CPU baseline leg of bench.py.

Times the CPU restatement (oracle/torch_raster.py, PyTorch on the host cores) on a BOUNDED sample
of the benchmark workload and scales it to the full frame:

  * the per-Gaussian stages (activations, preprocess, binning, and their forward-AD / autograd
    passes) run on ALL P Gaussians -- measured once with an empty tile set (t_pre);
  * the per-tile blend (forward, JVP, VJP) runs on `n_tiles` tiles spread uniformly over the
    frame (t_sub); the full-frame time is t_pre + (t_sub - t_pre) * ntiles / n_tiles.

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


def _render_subset(model, cam, bg, subset, means2D=None):
    st = tr.settings_from_camera(cam, bg, model.active_sh_degree)
    m2 = torch.zeros_like(model.get_xyz) if means2D is None else means2D
    pre = tr.preprocess(model.get_xyz, m2, model.get_opacity, model.get_features, None, model.get_scaling,
                        model.get_rotation, None, st)
    pl, _, ranges = tr.binning(pre)
    color, _, _, _ = tr.blend(pre, pl, ranges, st.image_height, st.image_width, st.bg, tile_subset=subset)
    # keep the per-Gaussian stage in the autograd graph even when no tile of the sample touches it
    anchor = pre["xy"].sum() + pre["conic"].sum() + pre["opacity"].sum() + pre["rgb"].sum()
    return color + 0.0 * anchor


def _matvec_once(model, cam, bg, subset, tangents):
    # J v (forward mode)
    with torch.no_grad(), fwAD.dual_level():
        saved = (model._features_dc, model._features_rest, model._scaling, model._rotation, model._opacity)
        model._features_dc = fwAD.make_dual(saved[0], tangents[0])
        model._features_rest = fwAD.make_dual(saved[1], tangents[1])
        model._scaling = fwAD.make_dual(saved[2], tangents[2])
        model._rotation = fwAD.make_dual(saved[3], tangents[3])
        model._opacity = fwAD.make_dual(saved[4], tangents[4])
        try:
            q = fwAD.unpack_dual(_render_subset(model, cam, bg, subset)).tangent
        finally:
            (model._features_dc, model._features_rest, model._scaling, model._rotation, model._opacity) = saved
    q = torch.zeros(3, cam.image_height, cam.image_width) if q is None else q
    # J^T (2 q) (reverse mode)
    model.zero_grad()
    color = _render_subset(model, cam, bg, subset)
    (color * (2.0 * q)).sum().backward()
    return q


def cpu_matvec_rate(model, cam, bg, n_tiles=32, repeats=1, threads=None):
    """Returns dict(matvec_s, forward_s, t_pre, t_sub, n_tiles, ntiles, threads)."""
    if threads:
        torch.set_num_threads(threads)
    th = torch.get_num_threads()
    W, H = cam.image_width, cam.image_height
    ntiles = ((W + 15) // 16) * ((H + 15) // 16)
    stride = max(1, ntiles // n_tiles)
    subset = set(range(stride // 2, ntiles, stride))
    g = torch.Generator().manual_seed(3)
    tangents = [torch.randn(t.shape, generator=g) for t in
                (model._features_dc, model._features_rest, model._scaling, model._rotation, model._opacity)]

    def timed(fn):  # median of `repeats` runs
        ts = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]

    t_pre = timed(lambda: _matvec_once(model, cam, bg, set(), tangents))
    t_sub = timed(lambda: _matvec_once(model, cam, bg, subset, tangents))
    with torch.no_grad():
        f_pre = timed(lambda: _render_subset(model, cam, bg, set()))
        f_sub = timed(lambda: _render_subset(model, cam, bg, subset))
    scale = ntiles / len(subset)
    return dict(matvec_s=t_pre + max(t_sub - t_pre, 0.0) * scale, forward_s=f_pre + max(f_sub - f_pre, 0.0) * scale,
                t_pre=t_pre, t_sub=t_sub, n_tiles=len(subset), ntiles=ntiles, threads=th,
                cpu_model=_cpu_model())


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
