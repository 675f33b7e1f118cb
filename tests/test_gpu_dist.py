"""GPU, world_size 2 (two processes sharing the one GPU, gloo with host-staged collectives): the
view-sharded LM operator -- both the screen-space exchange (gslm_gather_screen) and the param-space
all-reduce -- equals the single-process operator over the whole view batch: loss, J^T b,
(J^T J + D) v, and three CG iterations (device-resident, fused direction update)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
W, H, NV = 96, 72, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    model = synthetic_gaussians(6000, 3, seed=0, s0=0.03, n_cams=NV)
    gts = [torch.rand(3, H, W, generator=torch.Generator().manual_seed(10 + i)) for i in range(NV)]
    cams = orbit_cameras(NV, W, H, seed=1, images=gts)
    return model, cams


def _direction(layout, n):
    v = torch.randn(n, generator=torch.Generator().manual_seed(3))
    for grp in ("xyz", "exposure"):
        a, b = layout.offsets[grp]
        v[a:b] = 0
    return v


def _run(op, model_layout):
    from gslm.lm import cgls_fused
    loss = op.evaluate()
    g = op.rhs(op.zeros())
    v = _direction(model_layout, g.numel()).cuda()
    y = op.matvec(v, op.zeros())
    x, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=False)
    torch.cuda.synchronize()
    return {"loss": loss.cpu(), "g": g.cpu(), "y": y.cpu(), "x": x.cpu()}


def _worker(rank, world, port, mode, out_path, ssim=False):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gaussian-splatting-lm_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gslm.parallel import ShardedLMProblem, shard_views
    model, cams = _scene()
    model = model.to("cuda")
    for c in cams:
        c.to("cuda")
    mine = [cams[i] for i in shard_views(len(cams), rank, world)]
    op = ShardedLMProblem(model, mine, torch.zeros(3), all_cams=cams, exchange=mode, ssim=ssim)
    assert op.exchange == mode
    res = _run(op, op.layout)
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,ssim", [("screen", False), ("allreduce", False), ("allreduce", True)])
def test_sharded_gpu_operator_matches_single_process(tmp_path, mode, ssim):
    from gslm.lm import LMProblem
    out = str(tmp_path / "r0.pt")
    mp.start_processes(_worker, args=(2, _free_port(), mode, out, ssim), nprocs=2, start_method="spawn", join=True)
    got = torch.load(out, weights_only=True)
    model, cams = _scene()
    model = model.to("cuda")
    for c in cams:
        c.to("cuda")
    op = LMProblem(model, cams, torch.zeros(3), ssim=ssim)
    ref = _run(op, op.layout)
    assert abs(float(got["loss"]) - float(ref["loss"])) <= 1e-9 * float(ref["loss"])
    assert torch.allclose(got["g"], ref["g"], rtol=1e-5, atol=1e-7)
    scale = ref["y"].abs().max()
    assert (got["y"] - ref["y"]).abs().max() <= 1e-5 * scale
    assert (got["x"] - ref["x"]).norm() <= 1e-4 * ref["x"].norm()
