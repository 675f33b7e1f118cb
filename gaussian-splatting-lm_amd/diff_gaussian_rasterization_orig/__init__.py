"""`diff_gaussian_rasterization_orig` (imported at gaussian_renderer/reference_render.py:14 and
tests/test_rasterizer.py:4): the original, non-JVP upstream rasterizer.  Its primal forward is the
same computation, so the alias re-exports the same HIP-backed classes."""
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: F401

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer"]
