"""`simple_knn._C` (the upstream pybind11 extension's name): distCUDA2(points[N,3] float32 cuda) -> [N] float32, the
mean squared distance of each point to its 3 nearest other points (gslm.knn, csrc/knn.hip)."""
from gslm.knn import distCUDA2

__all__ = ["distCUDA2"]
