// residual.hip -- the LM residual epilogue of one view in one pass.
//
// Reference (disable_ssim=True, train_jvp.py:212): batch_render clamps the render to [0, 1]
// (gaussian_renderer/batch_render.py:118), compute_batch_loss_block multiplies by the alpha mask and
// subtracts the ground truth (solver/batch_training_loss.py:10-17, 56-67), the "ssim" slot aliases
// the L1 slot, and loss_scalar = ||r||^2 + ||r||^2 (solver/loss_image_state.py:16-19).  The
// reference pads every view to the batch's max H x W; padded pixels carry r = 0 and contribute
// nothing, so each view is processed at its own size here.
//
// Per pixel p and channel c, R = color, m = alpha mask (1 when absent), g = ground truth:
//   r      = m clamp(R, 0, 1) - g                      residual
//   w      = m m 1[0 <= R <= 1]                       weight of J^T J (d r / d R squared)
//   seed   = -2 m 1[0 <= R <= 1] r                    dL/dR of J^T b, b = -[r; r]  (the rhs backward input)
//   loss  += 2 sum r^2                                 (double, block partials + one final pass)
// The float expressions follow the torch ones in gslm/lm.py's reference restatement operation by
// operation, so r, w and seed are bit-identical to it.
#include <algorithm>

#include "gslm_internal.hpp"

namespace gslm {

constexpr int RES_THREADS = 256;

__global__ __launch_bounds__(RES_THREADS) void k_lm_residual(int64_t HW, const float* __restrict__ color,
                                                             const float* __restrict__ gt,
                                                             const float* __restrict__ mask,
                                                             float* __restrict__ residual, float* __restrict__ weight,
                                                             float* __restrict__ seed, double* __restrict__ part) {
  __shared__ double s[RES_THREADS / 64];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * RES_THREADS;
  for (int64_t p = (int64_t)blockIdx.x * RES_THREADS + threadIdx.x; p < HW; p += stride) {
    const float m = mask ? mask[p] : 1.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int64_t k = c * HW + p;
      const float R = color[k];
      const float inside = (R >= 0.0f && R <= 1.0f) ? 1.0f : 0.0f;
      const float r = m * clamp01(R) - gt[k];
      if (residual) residual[k] = r;
      if (weight) weight[k] = (m * m) * inside;
      if (seed) seed[k] = ((-2.0f * m) * inside) * r;
      acc += (double)r * (double)r;
    }
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if (lane == 0) s[w] = acc;
  __syncthreads();
  if (tid == 0) part[blockIdx.x] = ((s[0] + s[1]) + s[2]) + s[3];
}

__global__ __launch_bounds__(RES_THREADS) void k_lm_loss_final(const double* __restrict__ part, int np, int accumulate,
                                                               double* __restrict__ loss) {
  __shared__ double s[RES_THREADS / 64];
  double acc = strided_sum_in_order(part, np);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if (lane == 0) s[w] = acc;
  __syncthreads();
  if (tid == 0) {
    const double l = 2.0 * (((s[0] + s[1]) + s[2]) + s[3]);  // [r; r] aliasing
    *loss = accumulate ? *loss + l : l;
  }
}

}  // namespace gslm

using namespace gslm;

extern "C" {

size_t gslm_residual_scratch_bytes(int32_t H, int32_t W) {
  (void)H;
  (void)W;
  return (size_t)1024 * sizeof(double);
}

int gslm_lm_residual(int32_t H, int32_t W, const float* color, const float* gt, const float* alpha_mask,
                     float* residual, float* weight, float* seed, void* scratch, size_t scratch_bytes,
                     double* loss_dev, int32_t accumulate, void* stream) {
  if (H < 0 || W < 0) { set_error("lm_residual: negative image size"); return GSLM_ERR_INVALID; }
  const int64_t HW = (int64_t)H * W;
  if (HW > 0 && (!color || !gt)) { set_error("lm_residual: NULL color / gt"); return GSLM_ERR_INVALID; }
  if (!loss_dev || !scratch) { set_error("lm_residual: NULL loss or scratch"); return GSLM_ERR_INVALID; }
  if (scratch_bytes < gslm_residual_scratch_bytes(H, W)) { set_error("lm_residual: scratch too small"); return GSLM_ERR_CAPACITY; }
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (HW + RES_THREADS - 1) / RES_THREADS));
  double* part = (double*)scratch;
  hipLaunchKernelGGL(k_lm_residual, dim3(nb), dim3(RES_THREADS), 0, s, HW, color, gt, alpha_mask, residual, weight,
                     seed, part);
  GSLM_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_lm_loss_final, dim3(1), dim3(RES_THREADS), 0, s, part, nb, accumulate ? 1 : 0, loss_dev);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // extern "C"
