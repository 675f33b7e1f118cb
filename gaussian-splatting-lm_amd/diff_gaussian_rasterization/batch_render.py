"""`diff_gaussian_rasterization.batch_render` (imported at gaussian_renderer/batch_render.py:3).

BatchGaussianRasterizationSettings / BatchGaussianRasterizer with the fork's call shape
(batch_render.py:33-50, 100-108): per-view lists of sizes, fovs and matrices; output
color [B,3,maxH,maxW], radii [B,P] int32, invdepth [B,1,maxH,maxW], zero padded.  Each view runs
the single-view HIP pipeline, so every slice equals the single-view render exactly
(tests/test_batch_render.py:83 requires 1e-6).  Multi-view scaling is done by sharding views over
GPUs (gslm.parallel), not by a batched kernel.
"""
from typing import List, NamedTuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import GaussianRasterizationSettings, GaussianRasterizer

__all__ = ["BatchGaussianRasterizationSettings", "BatchGaussianRasterizer"]


class BatchGaussianRasterizationSettings(NamedTuple):
    batch_size: int
    image_heights: List[int]
    image_widths: List[int]
    tanfovxs: List[float]
    tanfovys: List[float]
    bg: torch.Tensor
    scale_modifier: float
    viewmatrices: List[torch.Tensor]
    projmatrices: List[torch.Tensor]
    sh_degree: int
    camposes: List[torch.Tensor]
    prefiltered: bool
    debug: bool
    antialiasing: bool = False

    def view(self, b):
        return GaussianRasterizationSettings(
            image_height=int(self.image_heights[b]), image_width=int(self.image_widths[b]),
            tanfovx=self.tanfovxs[b], tanfovy=self.tanfovys[b], bg=self.bg, scale_modifier=self.scale_modifier,
            viewmatrix=self.viewmatrices[b], projmatrix=self.projmatrices[b], sh_degree=self.sh_degree,
            campos=self.camposes[b], prefiltered=self.prefiltered, debug=self.debug, antialiasing=self.antialiasing)


class BatchGaussianRasterizer(nn.Module):
    def __init__(self, batch_raster_settings):
        super().__init__()
        self.batch_raster_settings = batch_raster_settings

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None, dc=None):
        s = self.batch_raster_settings
        maxH, maxW = max(int(h) for h in s.image_heights), max(int(w) for w in s.image_widths)
        colors, radii, depths = [], [], []
        for b in range(s.batch_size):
            c, r, d = GaussianRasterizer(s.view(b))(means3D=means3D, means2D=means2D, opacities=opacities, shs=shs,
                                                    colors_precomp=colors_precomp, scales=scales,
                                                    rotations=rotations, cov3D_precomp=cov3D_precomp, dc=dc)
            H, W = c.shape[1], c.shape[2]
            if H != maxH or W != maxW:
                c = F.pad(c, (0, maxW - W, 0, maxH - H))
                d = F.pad(d, (0, maxW - W, 0, maxH - H))
            colors.append(c)
            radii.append(r)
            depths.append(d)
        return torch.stack(colors), torch.stack(radii), torch.stack(depths)
