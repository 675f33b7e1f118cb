// ssim.hip -- the SSIM residual of the LM step and its image-space Jacobian.
//
// Reference: solver/batch_training_loss.py:18-30 (disable_ssim=False, FUSED_SSIM_AVAILABLE=False) on
// utils/loss_utils.py:91-122 ssim_per_pixel.  Per view, channel c and pixel p, with
//   x = m clamp(R, 0, 1) (batch_render.py:118, batch_training_loss.py:56-67), y = ground truth,
//   K = the 11-tap Gaussian window (sigma 1.5, utils/loss_utils.py:49-57), zero padding 5, per channel,
//   mu_x = K*x, P = K*(x x), Q = K*(x y) (and mu_y, K*(y y) for the fixed ground truth),
//   S = (2 mu_x mu_y + C1)(2 s_xy + C2) / ((mu_x^2 + mu_y^2 + C1)(s_x + s_y + C2)),
//   r1 = a sqrt(|x - y| + 1e-6),  r2 = b sqrt(|1 - S| + 1e-6),  a = sqrt((1 - l) / 3HW), b = sqrt(l / 3HW);
// the residual vector is [r1; r2] and loss = ||r1||^2 + ||r2||^2.
//
// Linearisation in x (what J^T J needs besides the render Jacobian G and M = m 1[0 <= R <= 1]):
//   dr1 = d1 dx,                           d1 = a sign(x - y) / (2 sqrt(|x - y| + 1e-6))
//   dr2 = c2 dS,                           c2 = -b sign(1 - S) / (2 sqrt(|1 - S| + 1e-6))
//   dS  = a1 K*dx + a2 K*(2 x dx) + a3 K*(y dx)   (chain through mu_x, P, Q):
//         a1 = 2 mu_y (B - A) / (C D) - 2 S mu_x (1/C - 1/D),  a2 = -S / D,  a3 = 2 A / (C D)
//   and its transpose  S^T w = K*(a1 w) + 2 x K*(a2 w) + y K*(a3 w)   (K symmetric, zero padding).
// So  J^T J v = G^T M [d1^2 + S^T c2^2 S] M G v   and   J^T b = -G^T M [d1 r1 + S^T (c2 r2)].
//
// Every convolution is the separable 11 + 11-tap form, one 32x16 output tile per 256-thread block with
// its 42x26 halo staged in LDS (zero outside the image, as conv2d's padding), horizontal pass into
// LDS, vertical pass into registers, then a per-pixel epilogue; up to 5 derived inputs share the tile.
#include <algorithm>
#include <cmath>

#include "gslm_internal.hpp"

namespace gslm {

constexpr int SS_TW = 32, SS_TH = 16, SS_R = 5, SS_K = 11;
constexpr int SS_IW = SS_TW + 2 * SS_R, SS_IH = SS_TH + 2 * SS_R;  // 42 x 26 halo tile
constexpr float SS_C1 = 0.01f * 0.01f, SS_C2 = 0.03f * 0.03f;

struct SsimWin {
  float g[SS_K];
};

// Per-view state laid out as planes of [3, H, W] floats.
enum SsimPlane { SP_A1 = 0, SP_A2, SP_A3, SP_C2, SP_D1, SP_M, SP_X, SP_V2, SP_E1, SP_NPLANES };
constexpr int SS_PARTIALS = 1024;

// Separable convolution of NIN derived inputs over one tile of channel blockIdx.z.
//   src(c, yy, xx, in[NIN])   fills the derived inputs of an in-image pixel
//   epi(c, yy, xx, k, conv[NIN])  consumes the convolved values of output pixel (yy, xx), k = c HW + yy W + xx
template <int NIN, class Src, class Epi>
__device__ __forceinline__ void sep_conv_tile(const SsimWin& w, int H, int W, float* lds, Src src, Epi epi) {
  float* s_in = lds;                              // [NIN][SS_IH][SS_IW]
  float* s_h = lds + NIN * SS_IH * SS_IW;         // [NIN][SS_IH][SS_TW]
  const int c = blockIdx.z;
  const int x0 = blockIdx.x * SS_TW, y0 = blockIdx.y * SS_TH;
  const int tid = threadIdx.x;
  for (int idx = tid; idx < SS_IH * SS_IW; idx += blockDim.x) {
    const int ry = idx / SS_IW, rx = idx - ry * SS_IW;
    const int yy = y0 - SS_R + ry, xx = x0 - SS_R + rx;
    float v[NIN];
#pragma unroll
    for (int k = 0; k < NIN; ++k) v[k] = 0.f;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) src(c, yy, xx, v);
#pragma unroll
    for (int k = 0; k < NIN; ++k) s_in[(k * SS_IH + ry) * SS_IW + rx] = v[k];
  }
  __syncthreads();
  for (int idx = tid; idx < SS_IH * SS_TW; idx += blockDim.x) {
    const int ry = idx / SS_TW, cx = idx - ry * SS_TW;
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      const float* row = s_in + (k * SS_IH + ry) * SS_IW + cx;
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < SS_K; ++j) a += w.g[j] * row[j];
      s_h[(k * SS_IH + ry) * SS_TW + cx] = a;
    }
  }
  __syncthreads();
  const int64_t HW = (int64_t)H * W;
  for (int idx = tid; idx < SS_TH * SS_TW; idx += blockDim.x) {
    const int oy = idx / SS_TW, ox = idx - oy * SS_TW;
    const int yy = y0 + oy, xx = x0 + ox;
    if (yy >= H || xx >= W) continue;
    float v[NIN];
#pragma unroll
    for (int k = 0; k < NIN; ++k) {
      const float* col = s_h + (k * SS_IH + oy) * SS_TW + ox;
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < SS_K; ++i) a += w.g[i] * col[i * SS_TW];
      v[k] = a;
    }
    epi(c, yy, xx, (int64_t)c * HW + (int64_t)yy * W + xx, v);
  }
}

template <int NIN>
constexpr size_t sep_conv_lds() { return (size_t)NIN * (SS_IH * SS_IW + SS_IH * SS_TW) * sizeof(float); }

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

__device__ __forceinline__ double block_sum_256(double acc, double* s) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if (lane == 0) s[w] = acc;
  __syncthreads();
  return ((s[0] + s[1]) + s[2]) + s[3];
}

// Residual evaluation: the SSIM map, r1 / r2, the linearisation planes, the J^T b inputs e1 = d1 r1
// and v2 = c2 r2, and this block's partial of ||r1||^2 + ||r2||^2.
__global__ __launch_bounds__(256) void k_ssim_eval(SsimWin w, int H, int W, float aw, float bw,
                                                   const float* __restrict__ color, const float* __restrict__ gt,
                                                   const float* __restrict__ mask, float* __restrict__ st,
                                                   float* __restrict__ r1o, float* __restrict__ r2o,
                                                   double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double s_red[4];
  const int64_t HW = (int64_t)H * W, N3 = 3 * HW;
  double acc = 0.0;
  auto xval = [&](int c, int yy, int xx) {
    const int64_t p = (int64_t)yy * W + xx;
    const float m = mask ? mask[p] : 1.0f;
    return m * clamp01(color[c * HW + p]);
  };
  auto src = [&](int c, int yy, int xx, float v[5]) {
    const float x = xval(c, yy, xx), y = gt[c * HW + (int64_t)yy * W + xx];
    v[0] = x; v[1] = y; v[2] = x * x; v[3] = y * y; v[4] = x * y;
  };
  auto epi = [&](int c, int yy, int xx, int64_t k, const float v[5]) {
    const int64_t p = (int64_t)yy * W + xx;
    const float m = mask ? mask[p] : 1.0f;
    const float R = color[k];
    const float x = m * clamp01(R), y = gt[k];
    const float mu1 = v[0], mu2 = v[1];
    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
    const float s1 = v[2] - mu1_sq, s2 = v[3] - mu2_sq, s12 = v[4] - mu1_mu2;
    const float A = 2.f * mu1_mu2 + SS_C1, B = 2.f * s12 + SS_C2;
    const float C = (mu1_sq + mu2_sq) + SS_C1, D = (s1 + s2) + SS_C2;
    const float S = (A * B) / (C * D);
    const float l1 = fabsf(x - y), ls = fabsf(1.0f - S);
    const float q1 = sqrtf(l1 + 1e-6f), q2 = sqrtf(ls + 1e-6f);
    const float r1 = aw * q1, r2 = bw * q2;
    const float d1 = aw * sgnf(x - y) / (2.f * q1);
    const float c2 = -bw * sgnf(1.0f - S) / (2.f * q2);
    const float CD = C * D;
    st[SP_A1 * N3 + k] = 2.f * mu2 * (B - A) / CD - 2.f * S * mu1 * (1.f / C - 1.f / D);
    st[SP_A2 * N3 + k] = -S / D;
    st[SP_A3 * N3 + k] = 2.f * A / CD;
    st[SP_C2 * N3 + k] = c2;
    st[SP_D1 * N3 + k] = d1;
    st[SP_M * N3 + k] = (R >= 0.0f && R <= 1.0f) ? m : 0.0f;
    st[SP_X * N3 + k] = x;
    st[SP_E1 * N3 + k] = d1 * r1;  // J^T b inputs
    st[SP_V2 * N3 + k] = c2 * r2;
    if (r1o) r1o[k] = r1;
    if (r2o) r2o[k] = r2;
    acc += (double)r1 * (double)r1 + (double)r2 * (double)r2;
  };
  sep_conv_tile<5>(w, H, W, lds, src, epi);
  const double t = block_sum_256(acc, s_red);
  if (threadIdx.x == 0)
    part[((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_ssim_loss_final(const double* __restrict__ part, int np, int accumulate,
                                                         double* __restrict__ loss) {
  __shared__ double s[4];
  double acc = strided_sum_in_order(part, np);
  const double t = block_sum_256(acc, s);
  if (threadIdx.x == 0) *loss = accumulate ? *loss + t : t;
}

// Forward half of the image operator: v2 = c2^2 S t with t = M jv.
__global__ __launch_bounds__(256) void k_ssim_fwd(SsimWin w, int H, int W, const float* __restrict__ gt,
                                                  float* __restrict__ st, const float* __restrict__ jv) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int64_t HW = (int64_t)H * W, N3 = 3 * HW;
  auto src = [&](int c, int yy, int xx, float v[3]) {
    const int64_t k = c * HW + (int64_t)yy * W + xx;
    const float t = st[SP_M * N3 + k] * jv[k];
    v[0] = t; v[1] = (2.f * st[SP_X * N3 + k]) * t; v[2] = gt[k] * t;
  };
  auto epi = [&](int c, int yy, int xx, int64_t k, const float v[3]) {
    const float s = (st[SP_A1 * N3 + k] * v[0] + st[SP_A2 * N3 + k] * v[1]) + st[SP_A3 * N3 + k] * v[2];
    const float c2 = st[SP_C2 * N3 + k];
    st[SP_V2 * N3 + k] = (c2 * c2) * s;
  };
  sep_conv_tile<3>(w, H, W, lds, src, epi);
}

// Transpose half: u = sign M (e1 + S^T v2), e1 = d1^2 t (matvec, from jv) or the stored d1 r1 (J^T b,
// jv == NULL, sign = -1).
__global__ __launch_bounds__(256) void k_ssim_bwd(SsimWin w, int H, int W, const float* __restrict__ gt,
                                                  const float* __restrict__ st, const float* __restrict__ jv,
                                                  float sign, float* __restrict__ u) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int64_t HW = (int64_t)H * W, N3 = 3 * HW;
  auto src = [&](int c, int yy, int xx, float v[3]) {
    const int64_t k = c * HW + (int64_t)yy * W + xx;
    const float v2 = st[SP_V2 * N3 + k];
    v[0] = st[SP_A1 * N3 + k] * v2; v[1] = st[SP_A2 * N3 + k] * v2; v[2] = st[SP_A3 * N3 + k] * v2;
  };
  auto epi = [&](int c, int yy, int xx, int64_t k, const float v[3]) {
    const float stv = (v[0] + (2.f * st[SP_X * N3 + k]) * v[1]) + gt[k] * v[2];
    const float M = st[SP_M * N3 + k];
    float e1;
    if (jv) {
      const float d1 = st[SP_D1 * N3 + k];
      e1 = (d1 * d1) * (M * jv[k]);
    } else {
      e1 = st[SP_E1 * N3 + k];
    }
    u[k] = sign * (M * (e1 + stv));
  };
  sep_conv_tile<3>(w, H, W, lds, src, epi);
}

// ---- the first-order training loss's SSIM term (train.py:121-125, utils/loss_utils.py:59-89 `ssim`, the
// role upstream's optional fused_ssim plays): mean SSIM of C channel planes and its gradient.
//   dmean(S)/dx = (1/n) [K*(a1) + 2 x K*(a2) + y K*(a3)]   (the S^T w of the LM path with w = 1).
// The forward stores a1, a2, a3 ([3][C H W] floats) for the backward.
__global__ __launch_bounds__(256) void k_ssim_mean(SsimWin w, int H, int W, int C, const float* __restrict__ x,
                                                   const float* __restrict__ y, float* __restrict__ planes,
                                                   double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double s_red[4];
  const int64_t NC = (int64_t)C * H * W;
  const int64_t HW = (int64_t)H * W;
  double acc = 0.0;
  auto src = [&](int c, int yy, int xx, float v[5]) {
    const int64_t k = c * HW + (int64_t)yy * W + xx;
    const float a = x[k], b = y[k];
    v[0] = a; v[1] = b; v[2] = a * a; v[3] = b * b; v[4] = a * b;
  };
  auto epi = [&](int c, int yy, int xx, int64_t k, const float v[5]) {
    // utils/loss_utils.py:70-84 operation order
    const float mu1 = v[0], mu2 = v[1];
    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
    const float s1 = v[2] - mu1_sq, s2 = v[3] - mu2_sq, s12 = v[4] - mu1_mu2;
    const float A = 2.f * mu1_mu2 + SS_C1, B = 2.f * s12 + SS_C2;
    const float Cc = (mu1_sq + mu2_sq) + SS_C1, D = (s1 + s2) + SS_C2;
    const float S = (A * B) / (Cc * D);
    const float CD = Cc * D;
    planes[0 * NC + k] = 2.f * mu2 * (B - A) / CD - 2.f * S * mu1 * (1.f / Cc - 1.f / D);
    planes[1 * NC + k] = -S / D;
    planes[2 * NC + k] = 2.f * A / CD;
    acc += (double)S;
  };
  sep_conv_tile<5>(w, H, W, lds, src, epi);
  const double t = block_sum_256(acc, s_red);
  if (threadIdx.x == 0)
    part[((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_ssim_mean_final(const double* __restrict__ part, int np, double inv_n,
                                                         float* __restrict__ out) {
  __shared__ double s[4];
  double acc = strided_sum_in_order(part, np);
  const double t = block_sum_256(acc, s);
  if (threadIdx.x == 0) *out = (float)(t * inv_n);
}

// grad = (*gscale / n) [K*(a1) + 2 x K*(a2) + y K*(a3)]
__global__ __launch_bounds__(256) void k_ssim_mean_bwd(SsimWin w, int H, int W, int C, const float* __restrict__ x,
                                                       const float* __restrict__ y, const float* __restrict__ planes,
                                                       const float* __restrict__ gscale, float inv_n,
                                                       float* __restrict__ grad) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int64_t NC = (int64_t)C * H * W;
  const int64_t HW = (int64_t)H * W;
  const float sc = *gscale * inv_n;
  auto src = [&](int c, int yy, int xx, float v[3]) {
    const int64_t k = c * HW + (int64_t)yy * W + xx;
    v[0] = planes[k]; v[1] = planes[NC + k]; v[2] = planes[2 * NC + k];
  };
  auto epi = [&](int c, int yy, int xx, int64_t k, const float v[3]) {
    grad[k] = sc * ((v[0] + (2.f * x[k]) * v[1]) + y[k] * v[2]);
  };
  sep_conv_tile<3>(w, H, W, lds, src, epi);
}

static SsimWin make_window() {
  // utils/loss_utils.py:49-51: exp in double, a float32 tensor, normalised by its float32 sum
  SsimWin w;
  float f[SS_K], sum = 0.f;
  for (int x = 0; x < SS_K; ++x) {
    f[x] = (float)std::exp(-(double)((x - SS_K / 2) * (x - SS_K / 2)) / (2.0 * 1.5 * 1.5));
    sum += f[x];
  }
  for (int x = 0; x < SS_K; ++x) w.g[x] = f[x] / sum;
  return w;
}

static dim3 ssim_grid(int H, int W, int C = 3) {
  return dim3((unsigned)((W + SS_TW - 1) / SS_TW), (unsigned)((H + SS_TH - 1) / SS_TH), (unsigned)C);
}

}  // namespace gslm

using namespace gslm;

extern "C" {

size_t gslm_ssim_state_bytes(int32_t H, int32_t W) {
  const size_t n3 = (size_t)3 * (size_t)(H > 0 ? H : 0) * (size_t)(W > 0 ? W : 0);
  const dim3 g = ssim_grid(H > 0 ? H : 1, W > 0 ? W : 1);
  const size_t parts = (size_t)g.x * g.y * g.z;
  return (size_t)SP_NPLANES * n3 * sizeof(float) + (parts + 16) * sizeof(double);
}

static double* ssim_partials(void* state, int32_t H, int32_t W) {
  const size_t n3 = (size_t)3 * H * W;
  size_t off = (size_t)SP_NPLANES * n3 * sizeof(float);
  off = (off + 15) & ~(size_t)15;
  return (double*)((char*)state + off);
}

int gslm_ssim_residual(int32_t H, int32_t W, const float* color, const float* gt, const float* alpha_mask,
                       float lambda_dssim, void* state, size_t state_bytes, float* r1, float* r2, float* seed,
                       double* loss_dev, int32_t accumulate, void* stream) {
  if (H <= 0 || W <= 0) { set_error("ssim_residual: empty image"); return GSLM_ERR_INVALID; }
  if (!color || !gt || !state || !loss_dev) { set_error("ssim_residual: NULL argument"); return GSLM_ERR_INVALID; }
  if (state_bytes < gslm_ssim_state_bytes(H, W)) { set_error("ssim_residual: state too small"); return GSLM_ERR_CAPACITY; }
  if (!(lambda_dssim >= 0.f && lambda_dssim <= 1.f)) { set_error("ssim_residual: lambda_dssim outside [0, 1]"); return GSLM_ERR_INVALID; }
  hipStream_t s = (hipStream_t)stream;
  const double n = 3.0 * (double)H * (double)W;
  const float aw = (float)std::sqrt((1.0 - (double)lambda_dssim) / n), bw = (float)std::sqrt((double)lambda_dssim / n);
  const SsimWin w = make_window();
  const dim3 grid = ssim_grid(H, W);
  double* part = ssim_partials(state, H, W);
  hipLaunchKernelGGL(k_ssim_eval, grid, dim3(256), sep_conv_lds<5>(), s, w, H, W, aw, bw, color, gt, alpha_mask,
                     (float*)state, r1, r2, part);
  GSLM_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_ssim_loss_final, dim3(1), dim3(256), 0, s, part, (int)(grid.x * grid.y * grid.z),
                     accumulate ? 1 : 0, loss_dev);
  GSLM_LAUNCH_CHECK();
  if (seed) {
    hipLaunchKernelGGL(k_ssim_bwd, grid, dim3(256), sep_conv_lds<3>(), s, w, H, W, gt, (const float*)state,
                       (const float*)nullptr, -1.0f, seed);
    GSLM_LAUNCH_CHECK();
  }
  return GSLM_OK;
}

int gslm_ssim_normal(int32_t H, int32_t W, const float* gt, void* state, const float* jv, float* u, void* stream) {
  if (H <= 0 || W <= 0) { set_error("ssim_normal: empty image"); return GSLM_ERR_INVALID; }
  if (!gt || !state || !jv || !u) { set_error("ssim_normal: NULL argument"); return GSLM_ERR_INVALID; }
  hipStream_t s = (hipStream_t)stream;
  const SsimWin w = make_window();
  const dim3 grid = ssim_grid(H, W);
  hipLaunchKernelGGL(k_ssim_fwd, grid, dim3(256), sep_conv_lds<3>(), s, w, H, W, gt, (float*)state, jv);
  GSLM_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_ssim_bwd, grid, dim3(256), sep_conv_lds<3>(), s, w, H, W, gt, (const float*)state, jv, 1.0f, u);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

size_t gslm_ssim_mean_state_bytes(int32_t C, int32_t H, int32_t W) {
  const size_t n = (size_t)(C > 0 ? C : 0) * (size_t)(H > 0 ? H : 0) * (size_t)(W > 0 ? W : 0);
  const dim3 g = ssim_grid(H > 0 ? H : 1, W > 0 ? W : 1, C > 0 ? C : 1);
  return align_up(3 * n * sizeof(float), 16) + ((size_t)g.x * g.y * g.z + 16) * sizeof(double);
}

int gslm_ssim_mean(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, void* state,
                   size_t state_bytes, float* ssim_out, void* stream) {
  if (C <= 0 || H <= 0 || W <= 0) { set_error("ssim_mean: empty image"); return GSLM_ERR_INVALID; }
  if (!img || !gt || !state || !ssim_out) { set_error("ssim_mean: NULL argument"); return GSLM_ERR_INVALID; }
  if (state_bytes < gslm_ssim_mean_state_bytes(C, H, W)) { set_error("ssim_mean: state too small"); return GSLM_ERR_CAPACITY; }
  hipStream_t s = (hipStream_t)stream;
  const SsimWin w = make_window();
  const dim3 grid = ssim_grid(H, W, C);
  const size_t n = (size_t)C * H * W;
  double* part = (double*)((char*)state + align_up(3 * n * sizeof(float), 16));
  hipLaunchKernelGGL(k_ssim_mean, grid, dim3(256), sep_conv_lds<5>(), s, w, H, W, C, img, gt, (float*)state, part);
  GSLM_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_ssim_mean_final, dim3(1), dim3(256), 0, s, part, (int)(grid.x * grid.y * grid.z),
                     1.0 / (double)n, ssim_out);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_ssim_mean_backward(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, const void* state,
                            const float* grad_out, float* grad_img, void* stream) {
  if (C <= 0 || H <= 0 || W <= 0) { set_error("ssim_mean_backward: empty image"); return GSLM_ERR_INVALID; }
  if (!img || !gt || !state || !grad_out || !grad_img) { set_error("ssim_mean_backward: NULL argument"); return GSLM_ERR_INVALID; }
  hipStream_t s = (hipStream_t)stream;
  const SsimWin w = make_window();
  const dim3 grid = ssim_grid(H, W, C);
  const float inv_n = (float)(1.0 / ((double)C * H * W));
  hipLaunchKernelGGL(k_ssim_mean_bwd, grid, dim3(256), sep_conv_lds<3>(), s, w, H, W, C, img, gt,
                     (const float*)state, grad_out, inv_n, grad_img);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // extern "C"
