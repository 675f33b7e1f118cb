"""Native RCCL communicator over the C ABI (gslm_comm_*, gslm_allreduce_sum_*, gslm_alltoall, gslm_allgather;
csrc/comm.hip).

gslm.parallel moves the multi-GPU LM product's data with torch.distributed ("nccl" = RCCL on ROCm) by default;
with GSLM_COMM=native its device collectives go through this communicator instead -- the C-ABI collectives a host
without torch would bind (SURVEY §8(b) "gslm_allreduce*", comm handle passed in).  torch.distributed is used once,
to broadcast rank 0's RCCL unique id (the bootstrap any host needs some channel for).

Semantics match the torch calls they replace (in-place sum all-reduce, all_to_all_single over equal dim-0 blocks,
all_gather_into_tensor), enqueued on the caller's current stream.  `all_to_all_async` issues the collective on a
side stream ordered after the current stream's work and returns a handle whose wait() orders the current stream
after it (Work.wait()).
"""
import ctypes
import os
import sys

import torch
import torch.distributed as dist

from gslm import _lib
from gslm._lib import check, lib


def enabled():
    return os.environ.get("GSLM_COMM", "torch") == "native"


class _Pending:
    def __init__(self, side):
        self.ev = torch.cuda.Event()
        self.ev.record(side)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class NativeComm:
    def __init__(self, group=None, device=None):
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world_size = dist.get_world_size(group) if dist.is_initialized() else 1
        nb = int(lib.gslm_comm_id_bytes())
        uid = torch.zeros(nb, dtype=torch.uint8)
        if self.rank == 0:
            check(lib.gslm_comm_unique_id(uid.data_ptr()), "gslm_comm_unique_id")
        if self.world_size > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            if dist.get_backend(group) == "nccl":
                dev_uid = uid.to(self.device)
                dist.broadcast(dev_uid, src=src, group=group)
                uid = dev_uid.cpu()
            else:
                dist.broadcast(uid, src=src, group=group)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.gslm_comm_init(uid.data_ptr(), self.world_size, self.rank, ctypes.byref(handle)),
                  "gslm_comm_init")
        self.handle = handle
        self._side = None

    def close(self):
        if self.handle:
            check(lib.gslm_comm_destroy(self.handle), "gslm_comm_destroy")
            self.handle = None

    def __del__(self):
        # never at interpreter teardown: ranks reach it in no set order and the HIP runtime may already be gone, so a
        # communicator the program did not close() is left to process exit (the driver frees its resources); an
        # orderly shutdown calls close() on every rank before destroying the process group
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    def all_reduce_(self, t):
        """In-place sum over the ranks of a contiguous float32 / float64 device tensor."""
        if not (t.is_cuda and t.is_contiguous()):
            raise ValueError("NativeComm.all_reduce_: contiguous device tensor")
        if t.dtype == torch.float32:
            fn = lib.gslm_allreduce_sum_f32
        elif t.dtype == torch.float64:
            fn = lib.gslm_allreduce_sum_f64
        else:
            raise ValueError(f"NativeComm.all_reduce_: float32 / float64, got {t.dtype}")
        check(fn(self.handle, t.data_ptr(), t.numel(), _lib.stream_handle(t.device)), "gslm_allreduce_sum")
        return t

    def all_to_all(self, out, inp, stream=None):
        """out's r-th dim-0 block <- rank r's block `rank` of inp (torch's all_to_all_single, equal splits)."""
        if not (out.is_cuda and inp.is_cuda and out.is_contiguous() and inp.is_contiguous()):
            raise ValueError("NativeComm.all_to_all: contiguous device tensors")
        nbytes = inp.numel() * inp.element_size()
        if out.numel() * out.element_size() != nbytes or nbytes % self.world_size:
            raise ValueError("NativeComm.all_to_all: equal-size buffers divisible by the world size")
        s = stream.cuda_stream if stream is not None else _lib.stream_handle(out.device)
        check(lib.gslm_alltoall(self.handle, inp.data_ptr(), out.data_ptr(), nbytes // self.world_size, s),
              "gslm_alltoall")

    def all_gather(self, out, inp):
        """out's r-th dim-0 block <- rank r's inp (torch's all_gather_into_tensor)."""
        if not (out.is_cuda and inp.is_cuda and out.is_contiguous() and inp.is_contiguous()):
            raise ValueError("NativeComm.all_gather: contiguous device tensors")
        nbytes = inp.numel() * inp.element_size()
        if out.numel() * out.element_size() != nbytes * self.world_size:
            raise ValueError("NativeComm.all_gather: out must hold world_size copies of inp")
        check(lib.gslm_allgather(self.handle, inp.data_ptr(), out.data_ptr(), nbytes, _lib.stream_handle(out.device)),
              "gslm_allgather")

    def all_to_all_async(self, out, inp):
        """all_to_all on a side stream after the current stream's work; wait() orders the current stream after it."""
        if self._side is None:
            self._side = torch.cuda.Stream(device=out.device)
        cur = torch.cuda.current_stream(out.device)
        self._side.wait_stream(cur)
        self.all_to_all(out, inp, stream=self._side)
        # the buffers belong to the caller's stream again once the collective is done (caching-allocator safety)
        out.record_stream(self._side)
        inp.record_stream(self._side)
        return _Pending(self._side)
