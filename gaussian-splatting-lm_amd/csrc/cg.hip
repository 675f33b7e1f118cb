// cg.hip -- device-resident vector algebra for the CG / CGLS drivers on flat param-space vectors.
//
// Replaces GaussianModelState.dot / __add__ / __mul__ (solver/gaussian_model_state.py:197-273),
// whose every dot ends in `.item()` (a host sync per dot).  Here scalars stay in device memory
// (double) and the step sizes alpha = gamma / delta, beta = gamma' / gamma are read by the update
// kernels directly, so a CG iteration issues no host synchronisation.  Reductions are two-pass
// with a fixed block/thread assignment: deterministic.
#include "gslm_internal.hpp"

namespace gslm {

constexpr int MAXG = 8;
struct Groups {
  int64_t bound[MAXG + 1];
  double damp[MAXG];
  int n;
};

constexpr int DOT_THREADS = 256;
constexpr int DOT_BLOCKS = 1024;

__device__ __forceinline__ double group_w(const Groups& g, int64_t i) {
  double w = 1.0;
  if (g.n > 0) {
    w = 0.0;
#pragma unroll
    for (int k = 0; k < MAXG; ++k)
      if (k < g.n && i >= g.bound[k] && i < g.bound[k + 1]) w = g.damp[k];
  }
  return w;
}

__device__ __forceinline__ double block_sum_d(double x, double* s) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
  if (lane == 0) s[w] = x;
  __syncthreads();
  double t = 0.0;
  if (tid == 0)
    for (int k = 0; k < DOT_THREADS / 64; ++k) t += s[k];
  return t;
}

__global__ __launch_bounds__(DOT_THREADS) void k_dot_partial(const float* __restrict__ a, const float* __restrict__ b,
                                                             Groups g, int64_t n, double* __restrict__ part) {
  __shared__ double s[DOT_THREADS / 64];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * DOT_THREADS;
  if (g.n == 0) {
    for (int64_t i = (int64_t)blockIdx.x * DOT_THREADS + threadIdx.x; i < n; i += stride)
      acc += (double)a[i] * (double)b[i];
  } else {
    for (int k = 0; k < g.n; ++k) {
      double gacc = 0.0;
      const int64_t lo = g.bound[k], hi = min(g.bound[k + 1], n);
      // align the group start to the grid so each element is visited by exactly one thread
      for (int64_t i = lo + (int64_t)blockIdx.x * DOT_THREADS + threadIdx.x; i < hi; i += stride)
        gacc += (double)a[i] * (double)b[i];
      acc += g.damp[k] * gacc;
    }
  }
  const double t = block_sum_d(acc, s);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ __launch_bounds__(DOT_THREADS) void k_dot_final(const double* __restrict__ part, int np,
                                                           double* __restrict__ out) {
  __shared__ double s[DOT_THREADS / 64];
  const double acc = strided_sum_in_order(part, np);
  const double t = block_sum_d(acc, s);
  if (threadIdx.x == 0) *out = t;
}

// The monitor's three finalisations (γ', <x, g>, <x, s>) in one launch: block b sums part + b np into its output,
// bitwise as three k_dot_final launches.
__global__ __launch_bounds__(DOT_THREADS) void k_dot_final3(const double* __restrict__ part, int np,
                                                            double* __restrict__ o0, double* __restrict__ o1,
                                                            double* __restrict__ o2) {
  __shared__ double s[DOT_THREADS / 64];
  const int b = blockIdx.x;
  const double acc = strided_sum_in_order(part + (int64_t)b * np, np);
  const double t = block_sum_d(acc, s);
  if (threadIdx.x == 0) *(b == 0 ? o0 : (b == 1 ? o1 : o2)) = t;
}

__global__ __launch_bounds__(256) void k_axpy_dev(int64_t n, const double* __restrict__ num,
                                                  const double* __restrict__ den, float sign,
                                                  const float* __restrict__ x, float* __restrict__ y) {
  const double a = den ? (*num) / (*den) : (*num);
  const float af = (float)(a * (double)sign);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = y[i] + af * x[i];
}

__global__ __launch_bounds__(256) void k_xpby_dev(int64_t n, const float* __restrict__ s, const double* __restrict__ num,
                                                  const double* __restrict__ den, float* __restrict__ p) {
  const float b = (float)((*num) / (*den));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = s[i] + b * p[i];
}

// One CG step on flat vectors, a = gam / del (device scalars):
//   x += a p ;  s -= a q ;  part[block] = sum s_new^2     (then k_dot_final -> gamma')
// MONITOR also accumulates <x_new, g> and <x_new, s_new> (partials at part + nb, part + 2 nb): the
// residual monitor of conjugate_gradient.py:103-104, b^2 - <x, J^T b> - <x, s>, without two more
// passes over x.
// ctl (or NULL): the device CG control block of k_cg_monitor -- a stopped solve, or delta < 1e-20 (the
// reference's early termination, conjugate_gradient.py:88-91, before x moves), leaves x and s untouched.
template <bool MONITOR>
__global__ __launch_bounds__(DOT_THREADS) void k_cg_update(int64_t n, const double* __restrict__ gam,
                                                           const double* __restrict__ del,
                                                           const float* __restrict__ p, const float* __restrict__ q,
                                                           float* __restrict__ x, float* __restrict__ s,
                                                           const float* __restrict__ g, double* __restrict__ part,
                                                           const double* __restrict__ ctl) {
  __shared__ double sm[DOT_THREADS / 64];
  if (ctl && (ctl[0] != 0.0 || *del < 1e-20 || !isfinite(*del))) return;  // a NaN delta: x kept (stop 4 below)
  const float a = (float)((*gam) / (*del));
  double acc = 0.0, axg = 0.0, axs = 0.0;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * DOT_THREADS;
  const float4* p4 = reinterpret_cast<const float4*>(p);
  const float4* q4 = reinterpret_cast<const float4*>(q);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* x4 = reinterpret_cast<float4*>(x);
  float4* s4 = reinterpret_cast<float4*>(s);
  const bool do_x = x != nullptr;  // x == NULL: the x update is deferred into the next xpby
  for (int64_t i = (int64_t)blockIdx.x * DOT_THREADS + threadIdx.x; i < n4; i += stride) {
    const float4 qv = q4[i];
    float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), sv = s4[i];
    float4 gv;
    if (MONITOR) gv = g4[i];
    if (do_x) {
      const float4 pv = p4[i];
      xv = x4[i];
      xv.x += a * pv.x; xv.y += a * pv.y; xv.z += a * pv.z; xv.w += a * pv.w;
      x4[i] = xv;
    }
    sv.x -= a * qv.x; sv.y -= a * qv.y; sv.z -= a * qv.z; sv.w -= a * qv.w;
    s4[i] = sv;
    acc += (double)sv.x * sv.x + (double)sv.y * sv.y + (double)sv.z * sv.z + (double)sv.w * sv.w;
    if (MONITOR) {
      axg += (double)xv.x * gv.x + (double)xv.y * gv.y + (double)xv.z * gv.z + (double)xv.w * gv.w;
      axs += (double)xv.x * sv.x + (double)xv.y * sv.y + (double)xv.z * sv.z + (double)xv.w * sv.w;
    }
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * DOT_THREADS + threadIdx.x; i < n; i += stride) {
    float xv = 0.f;
    if (do_x) {
      xv = x[i] + a * p[i];
      x[i] = xv;
    }
    const float sv = s[i] - a * q[i];
    s[i] = sv;
    acc += (double)sv * sv;
    if (MONITOR) {
      axg += (double)xv * g[i];
      axs += (double)xv * sv;
    }
  }
  const double t = block_sum_d(acc, sm);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
  if (MONITOR) {
    __syncthreads();
    const double t1 = block_sum_d(axg, sm);
    if (threadIdx.x == 0) part[gridDim.x + blockIdx.x] = t1;
    __syncthreads();
    const double t2 = block_sum_d(axs, sm);
    if (threadIdx.x == 0) part[2 * gridDim.x + blockIdx.x] = t2;
  }
}

// The stopping tests of conjugate_gradient.py:88-117 on the device, once per inner iteration after the update
// (and the cross-rank sums of its scalars): ctl = [stop, iters, last_res, n_hist, history...] (doubles).
//   delta < 1e-20                       -> stop = 1 (x not moved: k_cg_update skipped it)
//   res = b^2 - <x, g> - <x, s> (the residual monitor of :103-104) appended to the history;
//   res > last_res                      -> stop = 2 (after the step, as the reference breaks after x += alpha p)
//   gamma' < max(tol sqrt(gamma), atol) -> stop = 3
//   otherwise iters += 1 (iter_total).  A stopped solve's later kernels return at once (ViewK::stop, k_cg_update).
// Failure detection first (the NaN asserts of matvec_T, solver_functions.py:125-130): a non-finite gamma, gamma',
// delta, <x, g> or <x, s> -- a NaN or Inf anywhere in J^T b, in a product (J^T J + D) p or in the iterate reaches
// these dots -- sets stop = 4 (GSLM_CG_STOP_NONFINITE) and nothing else; the host raises before the step is used.
// Same double arithmetic as the host-side tests of gslm.lm.cgls_fused.
__global__ void k_cg_monitor(const double* __restrict__ gam, const double* __restrict__ gamn,
                             const double* __restrict__ del, const double* __restrict__ xg,
                             const double* __restrict__ xs, const double* __restrict__ b2, double tol, double atol,
                             double* __restrict__ ctl, int max_hist) {
  if (threadIdx.x != 0 || ctl[0] != 0.0) return;
  if (!(isfinite(*gam) && isfinite(*gamn) && isfinite(*del) && isfinite(*xg) && isfinite(*xs))) {
    ctl[0] = 4.0;
    return;
  }
  if (*del < 1e-20) {
    ctl[0] = 1.0;
    return;
  }
  const double res = (*b2 - *xg) - *xs;
  const int nh = (int)ctl[3];
  if (nh < max_hist) ctl[4 + nh] = res;
  ctl[3] = (double)(nh + 1);
  if (res > ctl[2]) {
    ctl[0] = 2.0;
    return;
  }
  ctl[2] = res;
  if (*gamn < fmax(tol * sqrt(*gam), atol)) {
    ctl[0] = 3.0;
    return;
  }
  ctl[1] += 1.0;
}

__global__ __launch_bounds__(256) void k_damp_add(int64_t n, const float* __restrict__ x, Groups g,
                                                  float* __restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = y[i] + (float)group_w(g, i) * x[i];
}

static int make_groups(const int64_t* bounds, const double* damp, int ng, Groups* g) {
  if (ng < 0 || ng > MAXG) {
    set_error("at most 8 damping groups");
    return GSLM_ERR_INVALID;
  }
  g->n = ng;
  for (int k = 0; k <= MAXG; ++k) g->bound[k] = (k <= ng && bounds) ? bounds[k] : 0;
  for (int k = 0; k < MAXG; ++k) g->damp[k] = (k < ng && damp) ? damp[k] : 0.0;
  return GSLM_OK;
}

static unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace gslm

using namespace gslm;

extern "C" {

size_t gslm_dot_scratch_bytes(int64_t n) {
  const int64_t per_block = (n + 255) / 256 + 16;  // partials of a per-Gaussian fused dot
  return (size_t)(per_block > DOT_BLOCKS ? per_block : DOT_BLOCKS) * sizeof(double);
}

int gslm_cg_update(int64_t n, const double* gam_dev, const double* del_dev, const float* p, const float* q, float* x,
                   float* s, void* scratch, double* gam_new_dev, void* stream) {
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(x) |
       reinterpret_cast<uintptr_t>(s)) & 15) {
    set_error("gslm_cg_update: vectors must be 16-byte aligned");
    return GSLM_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_cg_update<false>, dim3(DOT_BLOCKS), dim3(DOT_THREADS), 0, st, n, gam_dev, del_dev, p, q, x, s,
                     nullptr, (double*)scratch, (const double*)nullptr);
  hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(DOT_THREADS), 0, st, (const double*)scratch, DOT_BLOCKS, gam_new_dev);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_cg_update_monitor(int64_t n, const double* gam_dev, const double* del_dev, const float* p, const float* q,
                           float* x, float* s, const float* g, void* scratch, size_t scratch_bytes,
                           double* gam_new_dev, double* xg_dev, double* xs_dev, const double* cg_ctl, void* stream) {
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(x) |
       reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(g)) & 15) {
    set_error("gslm_cg_update_monitor: vectors must be 16-byte aligned");
    return GSLM_ERR_INVALID;
  }
  if (scratch_bytes < (size_t)3 * DOT_BLOCKS * sizeof(double)) {
    set_error("gslm_cg_update_monitor: scratch < 3 * 1024 doubles");
    return GSLM_ERR_CAPACITY;
  }
  hipStream_t st = (hipStream_t)stream;
  const double* part = (const double*)scratch;
  hipLaunchKernelGGL(k_cg_update<true>, dim3(DOT_BLOCKS), dim3(DOT_THREADS), 0, st, n, gam_dev, del_dev, p, q, x, s, g,
                     (double*)scratch, cg_ctl);
  hipLaunchKernelGGL(k_dot_final3, dim3(3), dim3(DOT_THREADS), 0, st, part, DOT_BLOCKS, gam_new_dev, xg_dev, xs_dev);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_cg_monitor(const double* gam_dev, const double* gam_new_dev, const double* del_dev, const double* xg_dev,
                    const double* xs_dev, const double* b2_dev, double tol, double atol, double* cg_ctl,
                    int32_t max_hist, void* stream) {
  if (!gam_dev || !gam_new_dev || !del_dev || !xg_dev || !xs_dev || !b2_dev || !cg_ctl || max_hist < 0) {
    set_error("gslm_cg_monitor: NULL scalar / control block or negative max_hist");
    return GSLM_ERR_INVALID;
  }
  hipLaunchKernelGGL(k_cg_monitor, dim3(1), dim3(64), 0, (hipStream_t)stream, gam_dev, gam_new_dev, del_dev, xg_dev,
                     xs_dev, b2_dev, tol, atol, cg_ctl, max_hist);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_dot_finalize(const void* partials, int32_t np, double* out_dev, void* stream) {
  hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(DOT_THREADS), 0, (hipStream_t)stream, (const double*)partials, np,
                     out_dev);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_dot(const float* a, const float* b, const int64_t* group_bounds, const double* group_damp, int32_t ngroups,
             int64_t n, void* scratch, double* out_dev, void* stream) {
  Groups g;
  int st = make_groups(group_bounds, group_damp, ngroups, &g);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_dot_partial, dim3(DOT_BLOCKS), dim3(DOT_THREADS), 0, s, a, b, g, n, (double*)scratch);
  hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(DOT_THREADS), 0, s, (const double*)scratch, DOT_BLOCKS, out_dev);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_axpy_dev(int64_t n, const double* num_dev, const double* den_dev, float sign, const float* x, float* y,
                  void* stream) {
  if (n <= 0) return GSLM_OK;
  hipLaunchKernelGGL(k_axpy_dev, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, num_dev, den_dev, sign, x, y);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_xpby_dev(int64_t n, const float* s_, const double* num_dev, const double* den_dev, float* p, void* stream) {
  if (n <= 0) return GSLM_OK;
  hipLaunchKernelGGL(k_xpby_dev, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, s_, num_dev, den_dev, p);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int gslm_damp_add(int64_t n, const float* x, const int64_t* group_bounds, const double* group_damp, int32_t ngroups,
                  float* y, void* stream) {
  Groups g;
  int st = make_groups(group_bounds, group_damp, ngroups, &g);
  if (st) return st;
  if (n <= 0) return GSLM_OK;
  hipLaunchKernelGGL(k_damp_add, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, x, g, y);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // extern "C"
