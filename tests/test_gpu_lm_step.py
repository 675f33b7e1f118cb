"""GPU parity of one whole LM step (train_jvp.py:237-279) against tests/golden/lm_step_golden.npz.

The golden comes from the reference's own LinearSolverFunctions + cgls_damped on the CPU oracle renderer (schedule
2 x 1 as train_jvp.py:254-256, and 10 x 10), followed by the backtracking line search (restated in
oracle/lm_ref.py:line_search_ref) on three validation views, the model stepped with the reference's
GaussianModelState arithmetic.  gslm.lm.lm_step must pick the same best_alpha, reproduce every (alpha, val loss)
pair of the search and the final validation loss (rel 1e-4: the GPU's CG step differs from the golden's by ~1e-7,
so the stepped parameters differ by ulps, and a splat whose alpha sits at the 1/255 cut or a radius at a ceil()
boundary can flip at one alpha -- measured 6.6e-5 once, 1e-6 otherwise), and leave the parameters where the
reference's step leaves them (1e-4 of the step's max).
"""
import os

import numpy as np
import pytest
import torch

from gslm.cameras import orbit_cameras
from gslm.model import GaussianModel

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GROUPS = ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure")


def _setup():
    d = np.load(os.path.join(HERE, "golden", "solver_golden.npz"))
    L = np.load(os.path.join(HERE, "golden", "lm_step_golden.npz"))
    P, D, W, H, s0, nv = d["scene"]
    D, W, H, nv = int(D), int(W), int(H), int(nv)
    m = GaussianModel(D)
    m.set_params(*(torch.from_numpy(d[f"in_{k}"]).cuda() for k in GROUPS))
    m.active_sh_degree = D
    cams = orbit_cameras(nv, W, H, seed=1, images=[torch.from_numpy(d[f"gt{i}"]) for i in range(nv)])
    nval = sum(1 for k in L.files if k.startswith("val_gt"))
    val = orbit_cameras(nval, W, H, seed=4, images=[torch.from_numpy(L[f"val_gt{i}"]) for i in range(nval)])
    for c in cams + val:
        c.to("cuda")
    return d, L, m, cams, val


@pytest.mark.parametrize("tag,sched", [("ref", (2, 1)), ("ten", (10, 10))])
def test_lm_step_matches_reference_line_search(tag, sched):
    from gslm.lm import lm_step
    d, L, m, cams, val = _setup()
    out = lm_step(m, cams, val, torch.zeros(3), max_iter=sched[0], restart_iter=sched[1], check_every=True)
    assert abs(out["start_loss"] - float(L[f"{tag}_start_loss"])) <= 1e-5 * float(L[f"{tag}_start_loss"])
    s_ref = L[f"{tag}_s"].astype(np.float64)
    s = out["step"].cpu().numpy().astype(np.float64)
    assert np.linalg.norm(s - s_ref) <= 1e-4 * np.linalg.norm(s_ref), np.linalg.norm(s - s_ref) / np.linalg.norm(s_ref)
    assert out["best_alpha"] == float(L[f"{tag}_best_alpha"])
    alphas = [a for a, _ in out["trace"]]
    losses = np.array([v for _, v in out["trace"]])
    assert alphas == list(L[f"{tag}_trace_alpha"])
    ref = L[f"{tag}_trace_loss"]
    assert np.abs(losses - ref).max() <= 1e-4 * ref.max(), np.abs(losses - ref).max() / ref.max()
    fin = float(L[f"{tag}_final_val_loss"])
    assert abs(out["final_val_loss"] - fin) <= 1e-4 * fin
    # the stepped parameters: theta0 + best_alpha * s (update_step arithmetic), against the reference's
    scale = float(L[f"{tag}_best_alpha"]) * np.abs(s_ref).max()
    for k, t in zip(GROUPS, m.params()):
        err = np.abs(t.detach().cpu().numpy().astype(np.float64) - L[f"{tag}_out_{k}"]).max()
        assert err <= 1e-4 * scale + 1e-6, (k, err, scale)


def _check_against_golden(out, params, L, tag):
    assert abs(out["start_loss"] - float(L[f"{tag}_start_loss"])) <= 1e-5 * float(L[f"{tag}_start_loss"])
    s_ref = L[f"{tag}_s"].astype(np.float64)
    s = out["step"].cpu().numpy().astype(np.float64)
    assert np.linalg.norm(s - s_ref) <= 1e-4 * np.linalg.norm(s_ref), np.linalg.norm(s - s_ref) / np.linalg.norm(s_ref)
    assert out["best_alpha"] == float(L[f"{tag}_best_alpha"])
    assert [a for a, _ in out["trace"]] == list(L[f"{tag}_trace_alpha"])
    ref = L[f"{tag}_trace_loss"]
    losses = np.array([v for _, v in out["trace"]])
    assert np.abs(losses - ref).max() <= 1e-4 * ref.max(), np.abs(losses - ref).max() / ref.max()
    fin = float(L[f"{tag}_final_val_loss"])
    assert abs(out["final_val_loss"] - fin) <= 1e-4 * fin
    scale = float(L[f"{tag}_best_alpha"]) * np.abs(s_ref).max()
    for k, t in zip(GROUPS, params):
        err = np.abs(t.detach().cpu().numpy().astype(np.float64) - L[f"{tag}_out_{k}"]).max()
        assert err <= 1e-4 * scale + 1e-6, (k, err, scale)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dist_worker(rank, world, port, out_path, tag, sched):
    import sys
    import torch.distributed as dist
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gaussian-splatting-lm_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gslm.lm import lm_step
    d, L, m, cams, val = _setup()
    out = lm_step(m, cams, val, torch.zeros(3), max_iter=sched[0], restart_iter=sched[1], check_every=True)
    torch.save({"out": {k: out[k] for k in ("start_loss", "final_val_loss", "best_alpha", "trace", "ranks")},
                "step": out["step"].cpu(), "params": [t.detach().cpu() for t in m.params()],
                "exchange": "gaussian"}, out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("tag,sched", [("ref", (2, 1)), ("ten", (10, 10))])
def test_sharded_lm_step_two_processes_matches_golden(tmp_path, tag, sched):
    """The multi-GPU LM step (train_jvp.py:237-279) with two ranks on the one GPU (gloo, host-staged
    collectives): one training view per rank through the Gaussian-sharded HIP pipeline, the validation views split
    2 + 1 with an all-reduced loss per line-search point, the gathered step applied on both ranks.  Both ranks end
    bitwise equal and match the reference's step and line search (lm_step_golden.npz)."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "r")
    mp.start_processes(_dist_worker, args=(2, _free_port(), out, tag, sched), nprocs=2, start_method="spawn",
                       join=True)
    r0, r1 = (torch.load(out + f".{r}", weights_only=True) for r in (0, 1))
    for a, b in zip(r0["params"], r1["params"]):
        assert torch.equal(a, b)
    assert r0["out"]["ranks"] == 2
    L = np.load(os.path.join(HERE, "golden", "lm_step_golden.npz"))
    _check_against_golden(dict(r0["out"], step=r0["step"]), r0["params"], L, tag)


@pytest.mark.parametrize("sched,kw", [((2, 1), {}), ((10, 10), {}), ((10, 10), {"atol": 1e30}),
                                      ((10, 5), {"tol": 1e-2})])
def test_device_stopping_tests_equal_host(sched, kw):
    """cgls_fused's stopping tests on the device (gslm_cg_monitor; no host read inside the loop) against the
    host-side tests: the same iterate, iteration count and residual history -- also when a test fires early
    (atol huge: stops after the first step; tol 1e-2 with restarts)."""
    from gslm.lm import LMProblem, cgls_fused
    d, L, m, cams, val = _setup()
    prob = LMProblem(m, cams, torch.zeros(3))
    prob.evaluate()
    g = prob.rhs(prob.zeros())
    xh, ih = cgls_fused(prob, g, max_iter=sched[0], restart_iter=sched[1], host_checks=True, **kw)
    xd, idv = cgls_fused(prob, g, max_iter=sched[0], restart_iter=sched[1], host_checks=False, **kw)
    assert torch.equal(xh, xd)
    assert ih["iters"] == idv["iters"]
    assert ih["residuals"] == idv["residuals"]
    if "atol" in kw:
        assert idv["stop"] == 3 and idv["iters"] == 0 and len(idv["residuals"]) == 1


def test_loss_evaluator_equals_lmproblem_evaluate():
    """The line search's loss-only evaluator (batched preprocesses, one num_rendered read-back per batch, the loss
    fused into the blend's epilogue: gslm_rasterize_loss) gives LMProblem.evaluate's loss over the same views (the
    same float residuals; only the double sum's order differs: 1e-12)."""
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem, LossEvaluator
    from gslm.model import synthetic_gaussians
    m = synthetic_gaussians(3000, 2, seed=0, s0=0.03).to("cuda")
    gts = [torch.rand(3, 40, 56, generator=torch.Generator().manual_seed(20 + i)) for i in range(5)]
    cams = orbit_cameras(5, 56, 40, seed=7, images=gts)
    for c in cams:
        c.to("cuda")
    def close(a, b):
        return abs(float(a) - float(b)) <= 1e-12 * abs(float(b))

    ref = float(LMProblem(m, cams, torch.zeros(3)).evaluate())
    for batch in (1, 2, 8):
        ev = LossEvaluator(m, cams, torch.zeros(3), batch=batch)
        first = float(ev.evaluate())
        assert close(first, ref)
        assert float(ev.evaluate()) == first  # reused workspaces and the cached depth orders (gslm_preprocess_ordered)
    # a line-search-like step on everything but xyz: the cached orders stay valid (same point lists, bitwise)
    with torch.no_grad():
        m._opacity.add_(0.7 * torch.randn(m._opacity.shape, generator=torch.Generator().manual_seed(5)).cuda())
        m._scaling.add_(0.3 * torch.randn(m._scaling.shape, generator=torch.Generator().manual_seed(6)).cuda())
    assert close(ev.evaluate(), LMProblem(m, cams, torch.zeros(3)).evaluate())
    # xyz moves: the evaluator notices (tensor version) and sorts again
    with torch.no_grad():
        m._xyz.add_(0.05 * torch.randn(m._xyz.shape, generator=torch.Generator().manual_seed(7)).cuda())
    assert close(ev.evaluate(), LMProblem(m, cams, torch.zeros(3)).evaluate())


@pytest.mark.parametrize("check_every", [True, False])
def test_lm_step_nan_raises_before_update(check_every):
    """The reference's NaN asserts (solver/solver_functions.py:125-130): a NaN in one SH coefficient must make lm_step
    raise -- from the device stopping tests (gslm_cg_monitor stop 4, naming the group as the reference does) or, with
    the tests off, from the check of the step -- before update_params, leaving every parameter bitwise unchanged."""
    from gslm.lm import NonFiniteError, lm_step
    d, L, m, cams, val = _setup()
    with torch.no_grad():
        m._features_rest[11, 2, 0] = float("nan")
    before = [t.detach().clone() for t in m.params()]
    with pytest.raises(NonFiniteError) as ei:
        lm_step(m, cams, val, torch.zeros(3), max_iter=2, restart_iter=1, check_every=check_every)
    assert "NaN detected" in str(ei.value)
    if check_every:
        assert "gaussians._features_rest.grad" in str(ei.value) or "features_dc" in str(ei.value), str(ei.value)
    for a, b in zip(before, m.params()):
        assert torch.equal(a.view(torch.int32), b.detach().view(torch.int32))


def test_cg_monitor_nonfinite_stop_code():
    """gslm_cg_monitor: a non-finite delta / gamma / monitor dot sets stop = 4 (GSLM_CG_STOP_NONFINITE) and nothing
    else; finite scalars keep the reference's tests."""
    import ctypes
    import math
    from gslm import _lib
    lib = _lib.lib
    for bad in (2, 1, 0, 3, 4):
        sc = torch.tensor([1.0, 0.5, 2.0, 0.1, 0.1, 10.0], dtype=torch.float64, device="cuda")  # gam gamn del xg xs b2
        sc[bad] = math.nan if bad != 3 else math.inf
        ctl = torch.tensor([0.0, 0.0, math.inf, 0.0, 0.0, 0.0], dtype=torch.float64, device="cuda")
        p = lambda i: sc.data_ptr() + 8 * i
        _lib.check(lib.gslm_cg_monitor(p(0), p(1), p(2), p(3), p(4), p(5), 1e-10, 0.0, ctl.data_ptr(), 2,
                                       _lib.stream_handle()))
        torch.cuda.synchronize()
        assert ctl[0].item() == 4.0 and ctl[1].item() == 0.0 and ctl[3].item() == 0.0, (bad, ctl.tolist())
