"""CPU, world_size 2-4 (gloo): the view-sharded LM operator (gslm.parallel.ShardedOperator) equals the
single-process operator over the whole view batch -- loss, J^T b, (J^T J + D) v and a CG solve.
The per-rank operator is the oracle restatement (oracle.lm_ref), the sharding/reduction code is the
product's."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    from oracle import torch_raster as tr
    model = synthetic_gaussians(300, 1, seed=0, s0=0.06, n_cams=4)
    cams = orbit_cameras(4, 24, 20, seed=1)
    pert = synthetic_gaussians(300, 1, seed=0, s0=0.06, n_cams=4)
    with torch.no_grad():
        pert._opacity += 0.3
        for c in cams:
            c.original_image = tr.render_model(pert, c, torch.zeros(3))[0].detach().clone()
    return model, cams


def _lm_vector(layout, n):
    """A param-space direction as every LM iterate has it: xyz (masked) and exposure groups zero."""
    v = torch.randn(n, generator=torch.Generator().manual_seed(3))
    for grp in ("xyz", "exposure"):
        a, b = layout.offsets[grp]
        v[a:b] = 0
    return v


def _worker(rank, world, port, out_path, ssim=False, exchange="allreduce"):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gaussian-splatting-lm_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from gslm.parallel import GaussianShardedOperator, ShardedOperator, shard_views
    from oracle.lm_ref import OracleLMProblem, cgls_ref
    model, cams = _scene()
    mine = [cams[i] for i in shard_views(len(cams), rank, world)]
    local = OracleLMProblem(model, mine, torch.zeros(3), ssim=ssim)
    if exchange == "gaussian":
        # CG vectors sharded by Gaussian: the shard layout, shard <-> full maps and the all-reduced CG scalars
        op = GaussianShardedOperator(local)
        assert op.layout.P == op.hi - op.lo and op.layout.numel < local.layout.numel
        loss = op.evaluate()
        gs = op.rhs(op.zeros())
        g = op.gather_full(gs)
        v = _lm_vector(local.layout, g.numel())
        y = op.gather_full(op.matvec(op.shard(v), op.zeros()))
        x = op.gather_full(cgls_ref(op, gs, 4, 4))
    else:
        op = ShardedOperator(local)
        loss = op.evaluate()
        g = op.rhs(op.zeros())
        v = _lm_vector(op.layout, g.numel())
        y = op.matvec(v, op.zeros())
        x = cgls_ref(op, g, 4, 4)
    if rank == 0:
        torch.save({"loss": loss, "g": g, "y": y, "x": x}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ssim,exchange,world", [(False, "allreduce", 2), (True, "allreduce", 2), (False, "gaussian", 2),
                                               (False, "allreduce", 3), (False, "gaussian", 4)])
def test_sharded_operator_matches_single_process(tmp_path, ssim, exchange, world):
    """Both residuals: disable_ssim=True ([r; r]) and the SSIM residual ([r1; r2]); and the
    Gaussian-sharded vector layout (gslm.parallel.GaussianShardedOperator).  World sizes 3 (the 4 views
    split 2 + 1 + 1: the replicated-vector exchange, as the driver's uneven splits take it) and 4 (one view per rank,
    300 Gaussians in shards of 75: the Gaussian-sharded exchange as the n = 4 bench runs it)."""
    from oracle.lm_ref import OracleLMProblem, cgls_ref
    out = str(tmp_path / "r0.pt")
    mp.start_processes(_worker, args=(world, _free_port(), out, ssim, exchange), nprocs=world, start_method="spawn",
                       join=True)
    got = torch.load(out, weights_only=True)
    model, cams = _scene()
    op = OracleLMProblem(model, cams, torch.zeros(3), ssim=ssim)
    loss = op.evaluate()
    g = op.rhs()
    v = _lm_vector(op.layout, g.numel())
    y = op.matvec(v, op.zeros())
    x = cgls_ref(op, g, 4, 4)
    assert abs(float(got["loss"]) - float(loss)) <= 1e-9 * float(loss)
    assert torch.allclose(got["g"], g, rtol=1e-5, atol=1e-7)
    assert torch.allclose(got["y"], y, rtol=1e-4, atol=1e-5)
    assert (got["x"] - x).norm() <= 1e-4 * x.norm()


def test_shard_views_partition():
    from gslm.parallel import shard_views
    for n, w in [(8, 8), (8, 2), (32, 4), (5, 2), (3, 4)]:
        parts = [shard_views(n, r, w) for r in range(w)]
        flat = [i for p in parts for i in p]
        assert flat == list(range(n))


GROUPS = ("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure")


def _golden_scene():
    """The scene of tests/golden/lm_step_golden.npz (2 training views, 3 validation views, 400 Gaussians SH 1)."""
    import numpy as np
    from gslm.cameras import orbit_cameras
    from gslm.model import GaussianModel
    d = np.load(os.path.join(HERE, "golden", "solver_golden.npz"))
    L = np.load(os.path.join(HERE, "golden", "lm_step_golden.npz"))
    P, D, W, H, s0, nv = d["scene"]
    D, W, H, nv = int(D), int(W), int(H), int(nv)
    m = GaussianModel(D)
    m.set_params(*(torch.from_numpy(d[f"in_{k}"]) for k in GROUPS))
    m.active_sh_degree = D
    cams = orbit_cameras(nv, W, H, seed=1, images=[torch.from_numpy(d[f"gt{i}"]) for i in range(nv)])
    nval = sum(1 for k in L.files if k.startswith("val_gt"))
    val = orbit_cameras(nval, W, H, seed=4, images=[torch.from_numpy(L[f"val_gt{i}"]) for i in range(nval)])
    return L, m, cams, val


def _lm_step_worker(rank, world, port, out_path, tag, sched):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gaussian-splatting-lm_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from gslm.lm import lm_step
    from oracle.lm_ref import OracleLMProblem, OracleLossEvaluator, cgls_solver
    L, m, cams, val = _golden_scene()
    out = lm_step(m, cams, val, torch.zeros(3), max_iter=sched[0], restart_iter=sched[1], device="cpu",
                  backend=(OracleLMProblem, OracleLossEvaluator, cgls_solver))
    params = [t.detach().clone() for t in m.params()]
    torch.save({"out": {k: out[k] for k in ("start_loss", "final_val_loss", "best_alpha", "trace", "ranks")},
                "step": out["step"], "params": params}, out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("tag,sched,world", [("ref", (2, 1), 2), ("ten", (10, 10), 2), ("ten", (10, 10), 3)])
def test_sharded_lm_step_matches_reference_golden(tmp_path, tag, sched, world):
    """gslm.lm.lm_step across 2 ranks (train_jvp.py:237-279, SURVEY 8(e) 'Line search. Sharded the same way'): one
    training view per rank with Gaussian-sharded CG vectors, the 3 validation views split 2 + 1 with one all-reduced
    loss per line-search point, the step gathered whole and applied on both ranks.  Both ranks must end with
    bitwise identical parameters, and the step, best_alpha, search trace, final loss and parameters must match
    the reference's (lm_step_golden.npz) at the single-process GPU test's tolerances.  The per-rank problem is the
    oracle restatement; the driver, sharding and reductions are the product's.  At world size 3 the 2 training views
    leave one rank without a training view (the replicated-vector exchange) and the 3 validation views go 1 + 1 + 1."""
    import numpy as np
    out = str(tmp_path / "r")
    mp.start_processes(_lm_step_worker, args=(world, _free_port(), out, tag, sched), nprocs=world, start_method="spawn",
                       join=True)
    rs = [torch.load(out + f".{r}", weights_only=True) for r in range(world)]
    r0 = rs[0]
    for r1 in rs[1:]:
        for a, b in zip(r0["params"], r1["params"]):
            assert torch.equal(a, b)
        assert torch.equal(r0["step"], r1["step"])
    L = np.load(os.path.join(HERE, "golden", "lm_step_golden.npz"))
    o = r0["out"]
    assert o["ranks"] == world
    assert abs(o["start_loss"] - float(L[f"{tag}_start_loss"])) <= 1e-5 * float(L[f"{tag}_start_loss"])
    s_ref = L[f"{tag}_s"].astype(np.float64)
    s = r0["step"].numpy().astype(np.float64)
    assert np.linalg.norm(s - s_ref) <= 1e-4 * np.linalg.norm(s_ref)
    assert o["best_alpha"] == float(L[f"{tag}_best_alpha"])
    assert [a for a, _ in o["trace"]] == list(L[f"{tag}_trace_alpha"])
    ref = L[f"{tag}_trace_loss"]
    assert np.abs(np.array([v for _, v in o["trace"]]) - ref).max() <= 1e-4 * ref.max()
    assert abs(o["final_val_loss"] - float(L[f"{tag}_final_val_loss"])) <= 1e-4 * float(L[f"{tag}_final_val_loss"])
    scale = float(L[f"{tag}_best_alpha"]) * np.abs(s_ref).max()
    for k, t in zip(GROUPS, r0["params"]):
        err = np.abs(t.numpy().astype(np.float64) - L[f"{tag}_out_{k}"]).max()
        assert err <= 1e-4 * scale + 1e-6, (k, err, scale)


def _nan_worker(rank, world, port, out_path):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gaussian-splatting-lm_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from gslm.lm import NonFiniteError, lm_step
    from oracle.lm_ref import OracleLMProblem, OracleLossEvaluator, cgls_solver
    L, m, cams, val = _golden_scene()
    with torch.no_grad():
        m._features_rest[7, 1, 2] = float("nan")  # one SH coefficient of one Gaussian, on every rank's replica
    before = [t.detach().clone() for t in m.params()]
    err = None
    try:
        lm_step(m, cams, val, torch.zeros(3), max_iter=2, restart_iter=1, device="cpu",
                backend=(OracleLMProblem, OracleLossEvaluator, cgls_solver))
    except NonFiniteError as e:
        err = str(e)
    same = all(torch.equal(a.view(torch.int32), b.detach().view(torch.int32)) for a, b in zip(before, m.params()))
    torch.save({"err": err, "unchanged": same}, out_path + f".{rank}")
    dist.barrier()  # both ranks reach here: neither is left waiting in a collective of the step
    dist.destroy_process_group()


def test_sharded_lm_step_nan_raises_on_every_rank(tmp_path):
    """The reference's failure detection (solver/solver_functions.py:125-130 asserts no NaN in any gradient group)
    across 2 ranks: a NaN in one SH coefficient makes lm_step raise NonFiniteError (an AssertionError) on BOTH ranks,
    before update_params, so every replica of theta is bitwise unchanged and no rank hangs in a collective."""
    out = str(tmp_path / "n")
    mp.start_processes(_nan_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn", join=True)
    for r in (0, 1):
        got = torch.load(out + f".{r}", weights_only=True)
        assert got["err"] is not None and "NaN detected" in got["err"], got
        assert got["unchanged"]
