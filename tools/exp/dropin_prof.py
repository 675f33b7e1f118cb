"""Experiment: where the drop-in solver ops' time goes (bench.time_dropin_solver_ops: matvec / matvec_T / forward through
render() at 1M Gaussians SH 3, one 1080p view).  For each op: the host-timed median, the GPU busy time (sum of kernel
durations in a torch.profiler trace of one call) and the top device kernels / host ops.
    python tools/exp/dropin_prof.py [--P 1000000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]
import torch  # noqa: E402
import torch.autograd.forward_ad as fwAD  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--P", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=7)
a = ap.parse_args()
import types  # noqa: E402

from gslm.cameras import orbit_cameras  # noqa: E402
from gslm.model import synthetic_gaussians  # noqa: E402
from gslm.train import PipelineParams, render  # noqa: E402

dev = torch.device("cuda", 0)
model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu").to(dev)
cam = orbit_cameras(1, 1920, 1080, seed=1)[0].to(dev)
cam.original_image = torch.rand(3, 1080, 1920, device=dev)
bg = torch.zeros(3, device=dev)
pipe = PipelineParams()
gt = cam.original_image
g3 = torch.Generator().manual_seed(3)
u = types.SimpleNamespace(**{f"{k}_grad": torch.randn(t.shape, generator=g3).to(dev) for k, t in
                             zip(("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure"),
                                 model.params())})
v = torch.randn(gt.shape, generator=torch.Generator().manual_seed(4)).to(dev)


def residual():
    return render(cam, model, pipe, bg)["render"] - gt


def matvec():
    with torch.no_grad(), fwAD.dual_level(), model.make_dual(u):
        return fwAD.unpack_dual(residual()).tangent


def matvec_T():
    model.zero_grad()
    r = residual()
    r.backward(v, retain_graph=True)
    r.backward(v)
    return model._opacity.grad


def forward():
    with torch.no_grad():
        r = residual()
        return 2.0 * (r.double() ** 2).sum()


out = {}
for name, fn in (("matvec", matvec), ("matvec_T", matvec_T), ("forward", forward)):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    rec = {"ms": 1e3 * sorted(ts)[len(ts) // 2]}
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    ev = prof.key_averages()
    dev_rows = sorted([e for e in ev if e.device_time_total > 0 and e.cpu_time_total == 0 or
                       (getattr(e, "device_type", None) is not None and str(e.device_type).endswith("CUDA"))],
                      key=lambda e: -e.self_device_time_total)
    kern = [(e.key[:60], round(e.self_device_time_total / 1e3, 4), e.count) for e in
            sorted(ev, key=lambda e: -e.self_device_time_total)[:14] if e.self_device_time_total > 0]
    rec["gpu_busy_ms"] = round(sum(e.self_device_time_total for e in ev) / 1e3, 4)
    rec["top_device"] = kern
    rec["top_host"] = [(e.key[:60], round(e.self_cpu_time_total / 1e3, 4), e.count) for e in
                       sorted(ev, key=lambda e: -e.self_cpu_time_total)[:14]]
    out[name] = rec
    print(name, json.dumps(rec), flush=True)
with open(os.path.join(ROOT, "gpurun_out", "dropin_prof.json"), "w") as f:
    json.dump(out, f, indent=1)
