"""GPU: device memory of the configs[2] LM step (the reference measures a batch loss's memory,
/root/reference/tests/test_render_backward_mem.py:201-205).

BASELINE configs[2] as bench.py runs it: 1M Gaussians SH 3, one 1080p training view, the reference's 50 validation
views (train_jvp.py:214-216), CGLS 10 iterations with the stopping tests, the 7-point line search.  The torch allocator's
peak over the step (every gslm workspace is a torch allocation: geometry, binning, image state, scratch, the validation
evaluator's slot workspaces and union lists, the CG vectors) must stay within LM_STEP_BUDGET_GB above what was resident
before it (the model, its GT images).  Measured on MI355X (round 6): 11.5 GB above resident -- most of it the kept
validation evaluator (8 batch positions x 2 alternating slot sets x 6 parameter sets of 64-B depth-space render
records per Gaussian, the union geometries and union lists); the budget is that plus ~20% (a workspace that starts
growing per view or per set shows up here first)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
LM_STEP_BUDGET_GB = 14.0


def test_configs2_lm_step_peak_memory():
    from margins import record
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem, clear_val_cache, lm_step
    from gslm.model import synthetic_gaussians
    from test_gpu_drift import _bench_scene
    model, cams, bg = _bench_scene()
    pert = synthetic_gaussians(1_000_000, 3, seed=0, s0=0.005, device="cpu")
    g2 = torch.Generator().manual_seed(2)
    with torch.no_grad():
        pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
        pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
        pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
    pert.to("cuda")
    val = [c.to("cuda") for c in orbit_cameras(50, 1920, 1080, seed=5)]
    for c0 in range(0, 50, 8):
        vp = LMProblem(pert, val[c0:c0 + 8], bg)
        vp.evaluate()
        for c, vr in zip(val[c0:c0 + 8], vp.views):
            c.original_image = vr.color.clamp(0, 1).clone()
        del vp
    del pert
    clear_val_cache()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    resident = torch.cuda.memory_allocated()
    out = lm_step(model, cams, val, bg, max_iter=10, restart_iter=10)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated()
    above = (peak - resident) / 1e9
    print(f"configs[2] LM step: resident {resident / 1e9:.3f} GB, peak {peak / 1e9:.3f} GB, above resident {above:.3f} GB "
          f"(best_alpha {out['best_alpha']})")
    record("test_configs2_lm_step_peak_memory", "LM step peak above resident (GB)", above, LM_STEP_BUDGET_GB)
    clear_val_cache()
    assert above <= LM_STEP_BUDGET_GB, above
