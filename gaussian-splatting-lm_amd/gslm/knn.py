"""`simple_knn._C.distCUDA2` on the MI355X (csrc/knn.hip): per point, the mean squared distance to its
3 nearest other points.  Same call shape as the reference's (scene/gaussian_model.py:22, :249):

    dist2 = torch.clamp_min(distCUDA2(points.float().cuda()), 0.0000001)
"""
import torch

from gslm import _lib
from gslm._lib import check, lib


def distCUDA2(points):
    if points.dim() != 2 or points.shape[1] != 3:
        raise ValueError(f"distCUDA2 expects [N, 3] points, got {tuple(points.shape)}")
    if not points.is_cuda:
        raise ValueError("distCUDA2 expects a GPU tensor")
    pts = points.to(torch.float32).contiguous()
    n = pts.shape[0]
    out = torch.empty(n, dtype=torch.float32, device=pts.device)
    scratch = _lib.u8(lib.gslm_knn_scratch_bytes(n), pts.device)
    check(lib.gslm_knn3_mean_dist(n, pts.data_ptr(), out.data_ptr(), scratch.data_ptr(), scratch.numel(),
                                  _lib.stream_handle(pts.device)), "gslm_knn3_mean_dist")
    return out
