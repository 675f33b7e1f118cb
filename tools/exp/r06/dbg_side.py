import os, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd"), os.path.join(ROOT, "tests")]
import torch
from test_gpu_dist import _scene
from gslm.lm import LMProblem, cgls_fused
print("current stream", torch.cuda.current_stream().cuda_stream, flush=True)
for nv, P in ((4, 6000), (2, 6001), (2, 6000)):
    model, cams = _scene(nv, P)
    model = model.to("cuda")
    for c in cams:
        c.to("cuda")
    op = LMProblem(model, cams, torch.zeros(3))
    op.evaluate()
    g = op.rhs(op.zeros())
    print("prob stream", op.stream, flush=True)
    os.environ["GSLM_CG_SIDE_X"] = "0"
    x0, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=False)
    res = []
    for same in ("0", "1", "0", "1", "0"):
        os.environ["GSLM_CG_SIDE_X"] = "1"
        os.environ["GSLM_CG_SIDE_SAME"] = same
        x1, _ = cgls_fused(op, g, max_iter=3, restart_iter=3, check_every=False)
        torch.cuda.synchronize()
        res.append((same, torch.equal(x1, x0), float((x1 - x0).norm()), float(x0.norm())))
    print(nv, P, res, flush=True)
