"""`simple_knn` for the MI355X build: the module the reference imports unconditionally at
scene/gaussian_model.py:22 (`from simple_knn._C import distCUDA2`) and calls in create_from_pcd
(gaussian_model.py:249).  `_C.distCUDA2` runs the HIP kernel of csrc/knn.hip (gslm_knn3_mean_dist) through
libgslm.so; there is no CPU fallback."""
