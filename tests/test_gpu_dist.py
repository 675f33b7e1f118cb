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


def _scene(nv=NV, P=6000):
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    model = synthetic_gaussians(P, 3, seed=0, s0=0.03, n_cams=nv)
    gts = [torch.rand(3, H, W, generator=torch.Generator().manual_seed(10 + i)) for i in range(nv)]
    cams = orbit_cameras(nv, W, H, seed=1, images=gts)
    return model, cams


def _direction(layout, n):
    v = torch.randn(n, generator=torch.Generator().manual_seed(3))
    for grp in ("xyz", "exposure"):
        a, b = layout.offsets[grp]
        v[a:b] = 0
    return v


def _run(op, model_layout, check_every=False, v=None):
    """v: the product's direction (default _direction); the Gaussian-sharded operator returns the one it used."""
    from gslm.lm import cgls_fused
    loss = op.evaluate()
    g = op.rhs(op.zeros())
    if getattr(op, "exchange", None) == "gaussian":  # shard-sized vectors: compare their gathered whole
        full = op.full_layout
        v = _direction(full, full.numel).cuda() if v is None else v.cuda()
        # SH-rest coordinates (op.rest_views): the direction's SH-rest group projected onto the views' span,
        # where every CG iterate lives (D v of a component off the span is not the product's)
        v = op.gather_full(op.shard(v))
        y = op.gather_full(op.matvec(op.shard(v), op.zeros()))
        x, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=check_every)
        res = {"loss": loss.cpu(), "g": op.gather_full(g).cpu(), "y": y.cpu(), "x": op.gather_full(x).cpu(),
               "v": v.cpu()}
        torch.cuda.synchronize()
        return res
    v = _direction(model_layout, g.numel()).cuda() if v is None else v.cuda()
    y = op.matvec(v, op.zeros())
    x, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=check_every)
    torch.cuda.synchronize()
    return {"loss": loss.cpu(), "g": g.cpu(), "y": y.cpu(), "x": x.cpu()}


def _worker(rank, world, port, mode, out_path, ssim=False, nv=NV, P=6000, check_every=False):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gaussian-splatting-lm_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gslm.parallel import ShardedLMProblem, shard_views
    model, cams = _scene(nv, P)
    model = model.to("cuda")
    for c in cams:
        c.to("cuda")
    mine = [cams[i] for i in shard_views(len(cams), rank, world)]
    op = ShardedLMProblem(model, mine, torch.zeros(3), all_cams=cams, exchange=mode, ssim=ssim)
    assert op.exchange == mode
    res = _run(op, op.layout, check_every)
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,ssim,nv,P,check_every", [
    ("screen", False, NV, 6000, False), ("allreduce", False, NV, 6000, False), ("allreduce", True, NV, 6000, False),
    # Gaussian-sharded exchange: 2 views per rank, a shard cut inside a 256-Gaussian block
    ("gaussian", False, 4, 6001, False), ("gaussian", False, NV, 6000, True)])
def test_sharded_gpu_operator_matches_single_process(tmp_path, mode, ssim, nv, P, check_every):
    from gslm.lm import LMProblem
    out = str(tmp_path / "r0.pt")
    mp.start_processes(_worker, args=(2, _free_port(), mode, out, ssim, nv, P, check_every), nprocs=2,
                       start_method="spawn", join=True)
    got = torch.load(out, weights_only=True)
    model, cams = _scene(nv, P)
    model = model.to("cuda")
    for c in cams:
        c.to("cuda")
    op = LMProblem(model, cams, torch.zeros(3), ssim=ssim)
    ref = _run(op, op.layout, check_every, v=got.get("v"))
    assert abs(float(got["loss"]) - float(ref["loss"])) <= 1e-9 * float(ref["loss"])
    if "v" in got:  # SH-rest coordinates: J^T b through projection -> expansion (double), rounding-level error
        assert (got["g"] - ref["g"]).abs().max() <= 1e-6 * ref["g"].abs().max()
    else:
        assert torch.allclose(got["g"], ref["g"], rtol=1e-5, atol=1e-7)
    scale = ref["y"].abs().max()
    assert (got["y"] - ref["y"]).abs().max() <= 1e-5 * scale
    assert (got["x"] - ref["x"]).norm() <= 1e-4 * ref["x"].norm()


def test_gaussian_sharded_single_rank_equals_lmproblem():
    """world_size 1: the Gaussian-sharded pipeline (tangent_views -> exchanged table -> RENDER | SCREEN ->
    gather_screen over the one shard) against the fused single-process product, in one process."""
    from gslm.lm import LMProblem
    from gslm.parallel import GaussianShardedOperator
    model, cams = _scene(3, 5000)
    model = model.to("cuda")
    for c in cams:
        c.to("cuda")
    op = GaussianShardedOperator(LMProblem(model, cams, torch.zeros(3)), all_cams=cams)
    assert op.rest_views == 3  # SH-rest coordinates: 9 floats per Gaussian instead of 45
    got = _run(op, op.layout)
    lp = LMProblem(model, cams, torch.zeros(3))
    ref = _run(lp, lp.layout, v=got["v"])
    assert abs(float(got["loss"]) - float(ref["loss"])) <= 1e-12 * float(ref["loss"])
    # J^T b is in the span: its SH-rest group survives the projection -> expansion (double) to float rounding
    assert (got["g"] - ref["g"]).abs().max() <= 1e-6 * ref["g"].abs().max()
    assert (got["y"] - ref["y"]).abs().max() <= 1e-5 * ref["y"].abs().max()
    assert (got["x"] - ref["x"]).norm() <= 1e-4 * ref["x"].norm()
