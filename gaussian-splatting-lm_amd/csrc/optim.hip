// optim.hip -- the first-order training step's per-Gaussian passes:
//
//   gslm_adam_step       one launch for every parameter group of GaussianModel.training_setup
//                        (scene/gaussian_model.py:268-291):
//                          dense  = torch.optim.Adam(lr, eps=1e-15) with bias correction, the optimizer
//                                   train.py:184-186 steps (torch's foreach op sequence, opmath f32);
//                          sparse = SparseGaussianAdam.step(visible, N) (train.py:180-183): rows of
//                                   Gaussians with visible[g] == 0 are left untouched (param, moments),
//                                   no bias correction -- the upstream 3dgs_accel adamUpdate kernel that
//                                   gaussian_model.py:29,286 imports (absent here; semantics restated).
//   gslm_densify_stats   train.py:166-167 fused: max_radii2D[vis] = max(max_radii2D, radii),
//                        xyz_gradient_accum[vis] += ||means2D.grad[vis, :2]||, denom[vis] += 1,
//                        vis = radii > 0 (render()'s visibility_filter, gaussian_renderer/__init__.py:121).
//
// Both are HBM streams (no reuse): Adam moves 28 B per float (read p g m v, write p m v), ~1.65 GB for
// 1M Gaussians at SH 3 -- torch's foreach Adam makes ~7 passes over the same tensors.  float4 chunks,
// one grid over all groups (the group of a chunk from a prefix table in kernel arguments).
#include <algorithm>
#include <cmath>

#include "gslm_internal.hpp"

namespace gslm {

constexpr int ADAM_THREADS = 256;

struct AdamGroupK {
  float* param;
  const float* grad;
  float* m;
  float* v;
  int64_t n;           // floats
  int64_t chunk0;      // first float4 chunk of this group in the flattened chunk space
  int32_t per_gauss;   // floats per Gaussian (sparse visibility index = i / per_gauss)
  int32_t vec4;        // all four pointers 16-B aligned
  float step_size;     // dense: -lr / (1 - b1^t)    sparse: lr
  float bc2_sqrt;      // dense: sqrt(1 - b2^t)      sparse: unused
};

struct AdamArgsK {
  AdamGroupK grp[GSLM_ADAM_MAX_GROUPS];
  int32_t ngroups;
  int32_t sparse;
  float b1, b2, eps;
  float w1, w2;  // 1 - b1, 1 - b2: dense in double then rounded (torch's Python scalars), sparse in f32
  const uint8_t* visible;
  int64_t nchunks;
};

// torch: exp_avg.lerp_(g, 1 - b1) (weight < 0.5: m + w (g - m)); exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2);
// denom = sqrt(v) / bc2_sqrt + eps; param.addcdiv_(m, denom, step_size).
__device__ __forceinline__ void adam_dense(float& p, float g, float& m, float& v, const AdamArgsK& a,
                                           const AdamGroupK& G) {
  m = m + a.w1 * (g - m);
  v = v * a.b2;
  v = v + a.w2 * g * g;
  const float denom = sqrtf(v) / G.bc2_sqrt + a.eps;
  p = p + G.step_size * (m / denom);
}

// upstream adamUpdate: m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2; p += -lr m / (sqrt(v) + eps)
__device__ __forceinline__ void adam_sparse(float& p, float g, float& m, float& v, const AdamArgsK& a,
                                            const AdamGroupK& G) {
  m = a.b1 * m + a.w1 * g;
  v = a.b2 * v + a.w2 * g * g;
  p += -G.step_size * m / (sqrtf(v) + a.eps);
}

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamArgsK& a,
                                         const AdamGroupK& G) {
  if (a.sparse) adam_sparse(p, g, m, v, a, G);
  else adam_dense(p, g, m, v, a, G);
}

__global__ __launch_bounds__(ADAM_THREADS) void k_adam(AdamArgsK a) {
  for (int64_t c = (int64_t)blockIdx.x * ADAM_THREADS + threadIdx.x; c < a.nchunks;
       c += (int64_t)gridDim.x * ADAM_THREADS) {
    int gi = 0;
#pragma unroll
    for (int k = 1; k < GSLM_ADAM_MAX_GROUPS; ++k)
      if (k < a.ngroups && c >= a.grp[k].chunk0) gi = k;
    const AdamGroupK& G = a.grp[gi];
    const int64_t i0 = 4 * (c - G.chunk0);
    const int cnt = (int)min<int64_t>(4, G.n - i0);
    bool vis[4] = {true, true, true, true};
    if (a.sparse) {
      bool any = false;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        vis[e] = e < cnt && a.visible[(i0 + e) / G.per_gauss] != 0;
        any |= vis[e];
      }
      if (!any) continue;  // no reads at all for a chunk of culled Gaussians
    }
    if (G.vec4 && cnt == 4) {
      float4 p = *reinterpret_cast<const float4*>(G.param + i0);
      const float4 g = *reinterpret_cast<const float4*>(G.grad + i0);
      float4 m = *reinterpret_cast<const float4*>(G.m + i0);
      float4 v = *reinterpret_cast<const float4*>(G.v + i0);
      // invisible lanes keep the values just loaded (written back unchanged)
      if (vis[0]) adam_one(p.x, g.x, m.x, v.x, a, G);
      if (vis[1]) adam_one(p.y, g.y, m.y, v.y, a, G);
      if (vis[2]) adam_one(p.z, g.z, m.z, v.z, a, G);
      if (vis[3]) adam_one(p.w, g.w, m.w, v.w, a, G);
      *reinterpret_cast<float4*>(G.param + i0) = p;
      *reinterpret_cast<float4*>(G.m + i0) = m;
      *reinterpret_cast<float4*>(G.v + i0) = v;
    } else {
      for (int e = 0; e < cnt; ++e) {
        if (!vis[e]) continue;
        float p = G.param[i0 + e], m = G.m[i0 + e], v = G.v[i0 + e];
        adam_one(p, G.grad[i0 + e], m, v, a, G);
        G.param[i0 + e] = p;
        G.m[i0 + e] = m;
        G.v[i0 + e] = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_densify_stats(int64_t P, const float* __restrict__ grad2d,
                                                       int64_t grad_stride, const int32_t* __restrict__ radii,
                                                       float* __restrict__ max_radii, float* __restrict__ accum,
                                                       float* __restrict__ denom) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  const int32_t r = radii[i];
  if (r <= 0) return;
  if (max_radii) max_radii[i] = fmaxf(max_radii[i], (float)r);
  const float gx = grad2d[i * grad_stride], gy = grad2d[i * grad_stride + 1];
  accum[i] = accum[i] + sqrtf(gx * gx + gy * gy);
  denom[i] = denom[i] + 1.0f;
}

}  // namespace gslm

using namespace gslm;

extern "C" {

int gslm_adam_step(const gslm_adam_group* groups, int32_t ngroups, double beta1, double beta2, double eps,
                   const uint8_t* visible, int64_t num_gaussians, int32_t sparse, void* stream) {
  if (ngroups < 0 || ngroups > GSLM_ADAM_MAX_GROUPS || (ngroups > 0 && !groups)) {
    set_error("adam: ngroups must be in [0, GSLM_ADAM_MAX_GROUPS]");
    return GSLM_ERR_INVALID;
  }
  if (sparse && (!visible || num_gaussians < 0)) {
    set_error("adam: the sparse step needs the visibility mask");
    return GSLM_ERR_INVALID;
  }
  AdamArgsK a{};
  a.sparse = sparse ? 1 : 0;
  a.b1 = (float)beta1;
  a.b2 = (float)beta2;
  a.eps = (float)eps;
  if (sparse) {  // upstream adamUpdate takes float b1, b2 and forms 1.0f - b1 in f32
    a.w1 = 1.0f - a.b1;
    a.w2 = 1.0f - a.b2;
  } else {       // torch: lerp weight 1 - beta1 and addcmul value 1 - beta2 are Python floats
    a.w1 = (float)(1.0 - beta1);
    a.w2 = (float)(1.0 - beta2);
  }
  a.visible = visible;
  int64_t chunks = 0;
  int k = 0;
  for (int i = 0; i < ngroups; ++i) {
    const gslm_adam_group& s = groups[i];
    if (s.n < 0) { set_error("adam: negative group size"); return GSLM_ERR_INVALID; }
    if (s.n == 0 || !s.grad) continue;  // torch skips parameters without .grad
    if (!s.param || !s.exp_avg || !s.exp_avg_sq) { set_error("adam: NULL parameter / moment"); return GSLM_ERR_INVALID; }
    if (sparse) {
      if (s.floats_per_gaussian <= 0 || s.n != (int64_t)s.floats_per_gaussian * num_gaussians) {
        set_error("adam: sparse group size is not floats_per_gaussian * num_gaussians");
        return GSLM_ERR_INVALID;
      }
    }
    AdamGroupK& G = a.grp[k++];
    G.param = s.param;
    G.grad = s.grad;
    G.m = s.exp_avg;
    G.v = s.exp_avg_sq;
    G.n = s.n;
    G.chunk0 = chunks;
    G.per_gauss = sparse ? s.floats_per_gaussian : 1;
    const uintptr_t any = (uintptr_t)s.param | (uintptr_t)s.grad | (uintptr_t)s.exp_avg | (uintptr_t)s.exp_avg_sq;
    G.vec4 = (any & 15u) == 0 ? 1 : 0;
    if (sparse) {
      G.step_size = (float)s.lr;
      G.bc2_sqrt = 1.f;
    } else {
      if (s.step < 1) { set_error("adam: step count must be >= 1 (incremented before the update)"); return GSLM_ERR_INVALID; }
      const double bc1 = 1.0 - std::pow(beta1, (double)s.step);
      const double bc2 = 1.0 - std::pow(beta2, (double)s.step);
      G.step_size = (float)(-(s.lr / bc1));
      G.bc2_sqrt = (float)std::sqrt(bc2);
    }
    chunks += (s.n + 3) / 4;
  }
  a.ngroups = k;
  a.nchunks = chunks;
  if (chunks == 0) return GSLM_OK;
  const int64_t blocks = std::min<int64_t>((chunks + ADAM_THREADS - 1) / ADAM_THREADS, 8192);
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(ADAM_THREADS), 0, (hipStream_t)stream, a);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_densify_stats(int64_t P, const float* means2D_grad, int64_t grad_stride, const int32_t* radii,
                       float* max_radii2D, float* xyz_gradient_accum, float* denom, void* stream) {
  if (P < 0 || (P > 0 && (!means2D_grad || !radii || !xyz_gradient_accum || !denom)) || grad_stride < 2) {
    set_error("densify_stats: NULL buffer or grad_stride < 2");
    return GSLM_ERR_INVALID;
  }
  if (P == 0) return GSLM_OK;
  hipLaunchKernelGGL(k_densify_stats, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, (hipStream_t)stream, P,
                     means2D_grad, grad_stride, radii, max_radii2D, xyz_gradient_accum, denom);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // extern "C"
