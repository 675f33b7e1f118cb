"""Worker of tests/test_gpu_rccl.py (run as its own process, not collected by pytest): one rank of a "nccl"
(RCCL) process group with GSLM_FORCE_COLLECTIVES=1, so the multi-GPU path's device-tensor collectives
(all_to_all_single, all_gather_into_tensor, all_reduce of CG scalars and vectors) run through RCCL on the one
GPU of the box.  Each exchange's loss, J^T b, product and 3 CG iterates are compared with the single-process
LMProblem; prints one JSON line with the backend, the exchanges run and their errors."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gaussian-splatting-lm_amd"), HERE]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    os.environ["GSLM_FORCE_COLLECTIVES"] = "1"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from gslm.lm import LMProblem
    from gslm.parallel import ShardedLMProblem
    from test_gpu_dist import _run, _scene
    out = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "exchanges": {}}
    for mode, nv in (("gaussian", 2), ("screen", 2), ("allreduce", 2)):
        model, cams = _scene(nv, 4001)
        model = model.to("cuda")
        for c in cams:
            c.to("cuda")
        op = ShardedLMProblem(model, cams, torch.zeros(3), all_cams=cams, exchange=mode)
        assert op.exchange == mode, (op.exchange, mode)
        got = _run(op, op.layout)
        # the Gaussian-sharded operator's direction (SH-rest group projected onto the views' span) for both
        ref_op = LMProblem(model, cams, torch.zeros(3))
        ref = _run(ref_op, ref_op.layout, v=got.get("v"))
        out["exchanges"][mode] = {
            "loss_rel": abs(float(got["loss"]) - float(ref["loss"])) / float(ref["loss"]),
            "g_max": float((got["g"] - ref["g"]).abs().max() / ref["g"].abs().max()),
            "y_max": float((got["y"] - ref["y"]).abs().max() / ref["y"].abs().max()),
            "x_rel": float((got["x"] - ref["x"]).norm() / ref["x"].norm()),
        }
        if mode == "gaussian":
            # two views per rank: the product ran pipelined (async all-to-alls per view group); the unpipelined
            # schedule must give the same product and iterates, bitwise
            from gslm.lm import cgls_fused
            out["exchanges"][mode]["pipelined"] = bool(op._overlap() and op.per > 1)
            vs = op.shard(got["v"].cuda())
            g = op.rhs(op.zeros())
            res = []
            for flag in ("1", "0"):
                os.environ["GSLM_OVERLAP"] = flag
                y = op.matvec(vs, op.zeros())
                x, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=False)
                torch.cuda.synchronize()
                res.append((y.clone(), x.clone()))
            del os.environ["GSLM_OVERLAP"]
            out["exchanges"][mode]["pipelined_bitwise"] = bool(torch.equal(res[0][0], res[1][0]) and
                                                               torch.equal(res[0][1], res[1][1]))
            # the same product and iterates with every collective through the C-ABI RCCL communicator
            # (GSLM_COMM=native: gslm_alltoall / gslm_allreduce_sum_*, pipelined on a side stream)
            os.environ["GSLM_COMM"] = "native"
            y = op.matvec(vs, op.zeros())
            x, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=True)
            torch.cuda.synchronize()
            del os.environ["GSLM_COMM"]
            x_t, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=True)
            torch.cuda.synchronize()
            from gslm.parallel import _NATIVE
            out["native"] = {"comm_made": len(_NATIVE) > 0, "y_bitwise": bool(torch.equal(y, res[0][0])),
                             "x_bitwise": bool(torch.equal(x, x_t))}
        if mode in ("screen", "allreduce"):
            # the screen exchange's all-gather (gslm_allgather) and the param-space all-reduce (gslm_allreduce_sum_f32)
            # through the C-ABI communicator: the same product, bitwise
            v = got.get("v")
            vv = (torch.randn(op.layout.numel, generator=torch.Generator().manual_seed(7)) if v is None else v).cuda()
            y_t = op.matvec(vv, op.zeros())
            os.environ["GSLM_COMM"] = "native"
            y_n = op.matvec(vv, op.zeros())
            torch.cuda.synchronize()
            del os.environ["GSLM_COMM"]
            out["exchanges"][mode]["native_bitwise"] = bool(torch.equal(y_t, y_n))
    # the C-ABI collectives on their own (one rank): sums and the all-to-all are identities / copies
    from gslm.comm import NativeComm
    nc = NativeComm(device="cuda")
    a = torch.randn(1000, device="cuda")
    a0 = a.clone()
    nc.all_reduce_(a)
    d64 = torch.randn(3, dtype=torch.float64, device="cuda")
    d0 = d64.clone()
    nc.all_reduce_(d64)
    src = torch.arange(4096, dtype=torch.int32, device="cuda")
    dst = torch.zeros_like(src)
    nc.all_to_all_async(dst, src).wait()
    gat = torch.zeros_like(src)
    nc.all_gather(gat, src)
    torch.cuda.synchronize()
    out["native"]["primitives"] = bool(torch.equal(a, a0) and torch.equal(d64, d0) and torch.equal(dst, src) and
                                       torch.equal(gat, src))
    nc.close()
    # the whole LM step (train_jvp.py:237-279) on the sharded path: Gaussian-sharded CG + all-reduced line search
    import numpy as np
    from gslm.lm import lm_step
    from test_gpu_lm_step import _setup
    d, L, m, cams, val = _setup()
    r = lm_step(m, cams, val, torch.zeros(3), max_iter=10, restart_iter=10, exchange="gaussian")
    s_ref = L["ten_s"].astype(np.float64)
    out["lm_step"] = {
        "ranks": r["ranks"], "best_alpha": r["best_alpha"], "best_alpha_ref": float(L["ten_best_alpha"]),
        "step_rel": float(np.linalg.norm(r["step"].cpu().numpy() - s_ref) / np.linalg.norm(s_ref)),
        "final_rel": abs(r["final_val_loss"] - float(L["ten_final_val_loss"])) / float(L["ten_final_val_loss"])}
    dist.barrier()
    from gslm.parallel import close_native_comms
    close_native_comms()  # the exchanges' cached GSLM_COMM=native communicator, before the process group
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
