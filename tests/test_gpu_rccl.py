"""The multi-GPU path's collectives through RCCL on the one GPU of a gpurun box: a one-rank "nccl" process
group with GSLM_FORCE_COLLECTIVES=1 (gslm.parallel.collectives_on) runs the Gaussian-sharded, screen and
all-reduce exchanges with every device-tensor collective issued to RCCL (all_to_all_single,
all_gather_into_tensor, all_reduce), and each equals the single-process LMProblem.  Two RCCL ranks cannot
share one GPU (RCCL refuses the communicator: "Duplicate GPU detected"), so the cross-rank data movement itself
is first exercised on the driver's 8-GPU node; the gloo two-process tests (test_gpu_dist.py) cover the
sharding arithmetic with two ranks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_exchanges_through_rccl_one_rank():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29517 + os.getpid() % 1000),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py")], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl" and res["world_size"] == 1
    assert set(res["exchanges"]) == {"gaussian", "screen", "allreduce"}
    for mode, e in res["exchanges"].items():
        assert e["loss_rel"] <= 1e-9, (mode, e)
        assert e["g_max"] <= 1e-5, (mode, e)
        assert e["y_max"] <= 1e-5, (mode, e)
        assert e["x_rel"] <= 1e-4, (mode, e)
    # two views per rank: the product ran pipelined (async all-to-alls per view group), bitwise the synchronous one
    assert res["exchanges"]["gaussian"]["pipelined"], res["exchanges"]["gaussian"]
    assert res["exchanges"]["gaussian"]["pipelined_bitwise"], res["exchanges"]["gaussian"]
    # the C-ABI RCCL communicator (gslm_comm_*, GSLM_COMM=native) gives the torch.distributed path's product and
    # CG iterates bitwise, and its collectives alone are identities at one rank
    nat = res["native"]
    assert nat["comm_made"] and nat["y_bitwise"] and nat["x_bitwise"] and nat["primitives"], nat
    assert res["exchanges"]["screen"]["native_bitwise"] and res["exchanges"]["allreduce"]["native_bitwise"], res
    lm = res["lm_step"]  # the sharded LM step through RCCL against the reference's (lm_step_golden.npz)
    assert lm["ranks"] == 1 and lm["best_alpha"] == lm["best_alpha_ref"], lm
    assert lm["step_rel"] <= 1e-4 and lm["final_rel"] <= 1e-4, lm
