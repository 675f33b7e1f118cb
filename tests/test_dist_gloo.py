"""CPU, world_size 2 (gloo): the view-sharded LM operator (gslm.parallel.ShardedOperator) equals the
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


@pytest.mark.parametrize("ssim,exchange", [(False, "allreduce"), (True, "allreduce"), (False, "gaussian")])
def test_sharded_operator_matches_single_process(tmp_path, ssim, exchange):
    """Both residuals: disable_ssim=True ([r; r]) and the SSIM residual ([r1; r2]); and the
    Gaussian-sharded vector layout (gslm.parallel.GaussianShardedOperator)."""
    from oracle.lm_ref import OracleLMProblem, cgls_ref
    out = str(tmp_path / "r0.pt")
    mp.start_processes(_worker, args=(2, _free_port(), out, ssim, exchange), nprocs=2, start_method="spawn",
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
