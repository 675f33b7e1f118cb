/*
 * gslm.h -- C ABI of the MI355X-native Gaussian-splat rasterizer + LM normal-equations matvec.
 *
 * Drop-in boundary.  The reference binds its rasterizer through pybind11
 * (`diff_gaussian_rasterization._C`, absent submodule) from the Python call sites below; every
 * entry point here replaces one of those calls:
 *
 *   gslm_preprocess + gslm_rasterize (= gslm_forward)
 *        <- GaussianRasterizer.forward, called at gaussian_renderer/__init__.py:102-110,
 *           gaussian_renderer/batch_render.py:100-108, gaussian_renderer/reference_render.py:102
 *   gslm_backward   <- autograd backward of the rasterizer, driven by loss_image_state.py:93-97
 *                      from solver/solver_functions.py:119 (matvec_T)
 *   gslm_jvp        <- forward-mode tangent of the rasterizer (fork), driven by fwAD at
 *                      solver/solver_functions.py:86-92 (matvec)
 *   gslm_matvec_view<- fused (J^T W J) v of one view: solver_functions.py:83-132 matvec followed
 *                      by matvec_T with the disable_ssim residual of batch_training_loss.py:10-17
 *   gslm_cg_*       <- GaussianModelState dot / saxpy (solver/gaussian_model_state.py:197-273)
 *                      used by cgls_damped (solver/conjugate_gradient.py:51-127), device resident
 *
 * Conventions: raw device pointers, sizes, a settings POD and a hipStream_t (passed as void*).
 * Every function returns GSLM_OK (0) or a negative status; gslm_last_error() describes the last
 * failure.  No internal threads, no allocation (the caller allocates workspaces sized by the
 * *_bytes queries), stream ordered, not re-entrant on one workspace.  Only gslm_num_rendered(_many) and
 * gslm_forward (which calls it) synchronise the stream (the upstream forward does the same to
 * size its binning buffers); the *_dev rasterize forms do not.
 */
#ifndef GSLM_H
#define GSLM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSLM_OK 0
#define GSLM_ERR_INVALID (-1)
#define GSLM_ERR_HIP (-2)
#define GSLM_ERR_CAPACITY (-3) /* a workspace is too small; the required size is reported */

#define GSLM_ABI_VERSION 9

/* GaussianRasterizationSettings (gaussian_renderer/__init__.py:36-50) as a POD. */
typedef struct gslm_view {
  int32_t image_height;
  int32_t image_width;
  double tanfovx;
  double tanfovy;
  double scale_modifier;
  float viewmatrix[16]; /* world_view_transform, row-major torch storage (= column-major for the kernel) */
  float projmatrix[16]; /* full_proj_transform */
  float campos[3];
  float bg[3];
  int32_t sh_degree;    /* active SH degree D */
  int32_t prefiltered;
  int32_t antialiasing;
  int32_t debug;        /* nonzero (the settings' `debug`, arguments/__init__.py:70): upstream's debug mode --
                           gslm_preprocess / _rasterize(_dev) / _forward / _backward / _jvp / _matvec_view_ex
                           synchronise their stream after every kernel and fail at the launch that faulted
                           (gslm_last_error names its source line) -- and the exhaustive tile traversal: every
                           wave visits every list entry, as upstream does (the quadrant cull is off; results are
                           bit-identical either way) */
} gslm_view;

/* Per-Gaussian inputs.  With raw = 0 they are the activated tensors the rasterizer receives
 * (means3D, opacities = sigmoid, scales = exp, rotations = normalize, shs = cat(dc, rest));
 * with raw = 1 they are the GaussianModel leaves (_xyz, _opacity, _scaling, _rotation,
 * _features_dc, _features_rest, scene/gaussian_model.py:53-69) and the activations of
 * gaussian_model.py:192-220 are fused into the kernels.  SH coefficient k of Gaussian i,
 * channel c is sh_dc[i*sh_dc_stride + c] for k = 0 and sh_rest[i*sh_rest_stride + 3*(k-1) + c]
 * otherwise.  For tangents (gslm_jvp) the same struct carries the tangent tensors; a NULL pointer
 * means a zero tangent. */
typedef struct gslm_gaussians {
  int64_t P;
  int32_t max_coeffs; /* K: coefficients stored per Gaussian (dc + rest) */
  int32_t raw;
  const float* means3D;       /* [P,3] */
  const float* opacities;     /* [P]   */
  const float* scales;        /* [P,3] or NULL when cov3D_precomp is given */
  const float* rotations;     /* [P,4] (w,x,y,z) */
  const float* cov3D_precomp; /* [P,6] or NULL */
  const float* sh_dc;         /* or NULL when colors_precomp is given */
  int64_t sh_dc_stride;
  const float* sh_rest;
  int64_t sh_rest_stride;
  const float* colors_precomp; /* [P,3] or NULL */
} gslm_gaussians;

/* Gradients / param-space vectors, one pointer per GaussianModelState group
 * (solver/gaussian_model_state.py:52-62).  NULL = not requested.  Strides as in gslm_gaussians. */
typedef struct gslm_grads {
  float* means2D;   /* [P,3] NDC-space screen gradient (means2D.grad, gaussian_model.py:561-563) */
  float* means3D;   /* [P,3] */
  float* opacities; /* [P]   */
  float* scales;    /* [P,3] */
  float* rotations; /* [P,4] */
  float* cov3D;     /* [P,6] (only when cov3D_precomp was the input) */
  float* sh_dc;
  int64_t sh_dc_stride;
  float* sh_rest;
  int64_t sh_rest_stride;
  float* colors;    /* [P,3] (only when colors_precomp was the input) */
  int32_t accumulate; /* 1: add into the outputs, 0: overwrite */
} gslm_grads;

/* ---- workspace sizing (two-call protocol: query, allocate with the caller's allocator, call) ---- */
size_t gslm_geom_bytes(int64_t P);
size_t gslm_image_bytes(int32_t H, int32_t W);
size_t gslm_binning_bytes(int64_t num_rendered, int32_t H, int32_t W);
size_t gslm_scratch_bytes(int64_t P, int64_t num_rendered); /* backward / jvp / matvec scratch */

/* ---- forward (rasterizer_impl forward: preprocess -> scan -> duplicateWithKeys -> sort -> ranges -> render) ---- */
/* Per-Gaussian preprocess, depth sort and tile-count scan.  Writes radii (int32 [P]) if non-NULL. */
int gslm_preprocess(const gslm_view* view, const gslm_gaussians* g, void* geom, size_t geom_bytes,
                    int32_t* out_radii, void* stream);
/* gslm_preprocess with a reusable depth order.  The depth order (the stable sort of every Gaussian in front of the
 * near plane by view-space depth, index order on ties; Gaussians culled later by their footprint emit no tile, so
 * the point list is the same whatever their place) depends on means3D and the view alone.
 *   order_mode 0: as gslm_preprocess;  1: also copy the order to depth_order[P];
 *   2: take the order from depth_order[P] -- written by a mode-1 call on the same view with the same means3D --
 *      instead of sorting (the LM line search renders each validation view at 7 step sizes with xyz frozen,
 *      train_jvp.py:221-227,262-279: the same point list, bitwise, without the four depth-sort passes). */
int gslm_preprocess_ordered(const gslm_view* view, const gslm_gaussians* g, void* geom, size_t geom_bytes,
                            int32_t* out_radii, uint32_t* depth_order, int32_t order_mode, void* stream);
/* The per-Gaussian stage of gslm_preprocess for nviews <= 8 views in one pass over the Gaussians (ABI 8): each view's
 * render records, depth keys, tile counts and rects into geoms[b] (each >= gslm_geom_bytes(P)), bitwise as
 * gslm_preprocess writes them, with no depth sort and no tile-count scan.  A Gaussian's 236 B of inputs (SH 3) are
 * read once for the views.  depth_pos (or NULL): per view the Gaussians' depth positions (gslm_depth_positions of the
 * view's depth order); then only the render records are written, each at its Gaussian's depth position, the rect
 * slot zero when culled -- the DEPTH SPACE the line search's union binning reads (below) -- and each geoms[b] needs
 * only gslm_depth_records_bytes(P) (64 B per Gaussian; ABI 9).  Every layout and SH degree (ABI 9: degree 0 too). */
size_t gslm_depth_records_bytes(int64_t P);
int gslm_preprocess_views(const gslm_view* views, int32_t nviews, const gslm_gaussians* g, void* const* geoms,
                          size_t geom_bytes, const uint32_t* const* depth_pos, void* stream);
/* depth_pos[depth_order[s]] = s for s < P (the inverse of a gslm_preprocess_ordered depth order). */
int gslm_depth_positions(const uint32_t* depth_order, int64_t P, uint32_t* depth_pos, void* stream);
/* Synchronous read of the number of (tile, Gaussian) pairs produced by gslm_preprocess. */
int gslm_num_rendered(const void* geom, int64_t P, int64_t* out_num_rendered, void* stream);
/* The same for n preprocessed geometries (geoms[k] over Ps[k] Gaussians) with ONE stream synchronisation:
 * a batch of views (the line search's validation renders, gslm.lm.LossEvaluator) preprocesses every view first,
 * then sizes every view's binning from one read-back instead of one round trip per view. */
int gslm_num_rendered_many(const void* const* geoms, const int64_t* Ps, int32_t n, int64_t* out_num_rendered,
                           void* stream);
/* Binning + tile sort + ranges + per-tile blend.  out_color [3,H,W], out_invdepth [1,H,W] (nullable). */
int gslm_rasterize(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes,
                   int64_t num_rendered, void* image, size_t image_bytes, float* out_color,
                   float* out_invdepth, void* stream);
/* The LM line search's validation loss of one view with no image written (gslm.lm.LossEvaluator; train_jvp.py:258,
 * 268,279 val_loss_func().loss_scalar with disable_ssim=True): gslm_rasterize's binning and blend, the blend's
 * epilogue computing r = m clamp(color, 0, 1) - gt per pixel and channel (gslm_lm_residual's arithmetic; gt [3,H,W],
 * alpha_mask [H,W] or NULL) and summing r^2 in double per tile, then *loss_dev = [*loss_dev if accumulate] +
 * 2 sum over tiles in tile order (deterministic).  No colour, inverse depth, final_T or n_contrib is written.
 * scratch >= gslm_loss_scratch_bytes(H, W). */
size_t gslm_loss_scratch_bytes(int32_t H, int32_t W);
int gslm_rasterize_loss(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes,
                        int64_t num_rendered, const float* gt, const float* alpha_mask, void* scratch,
                        size_t scratch_bytes, double* loss_dev, int32_t accumulate, void* stream);
/* Device-count forms (ABI 7): no host read-back of the pair count between gslm_preprocess and the binning.  The
 * binning workspace is used as a list of gslm_binning_capacity(binning_bytes, H, W) pairs; the count stays in the
 * geometry workspace and the kernels read it there.  n_out (device or host-pinned uint32, nullable) receives the count
 * in stream order: when it exceeds the capacity the pairs past it were dropped and the image / loss is invalid -- render
 * the view again with gslm_rasterize and a buffer of gslm_binning_bytes(count).  The binning written here serves this
 * render only (gslm_backward / gslm_jvp / gslm_matvec_* take the layout of the exact count: use gslm_rasterize for
 * those).  Same pairs, order, image and loss as gslm_rasterize / gslm_rasterize_loss whenever the count fits. */
int64_t gslm_binning_capacity(size_t binning_bytes, int32_t H, int32_t W);
int gslm_rasterize_dev(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes,
                       void* image, size_t image_bytes, float* out_color, float* out_invdepth, uint32_t* n_out,
                       void* stream);
int gslm_rasterize_loss_dev(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes,
                            const float* gt, const float* alpha_mask, void* scratch, size_t scratch_bytes,
                            double* loss_dev, int32_t accumulate, uint32_t* n_out, void* stream);
/* Stream-ordered 4-byte copy of gslm_preprocess' pair count to dst (device or host-pinned); no synchronisation. */
int gslm_num_rendered_copy(const void* geom, int64_t P, uint32_t* dst, void* stream);

/* ---- The line search's shared binning (ABI 8; ABI 9: the per-set workspaces' size set_bytes, each
 * >= gslm_depth_records_bytes(P), and n_sets for gslm_rasterize_loss_slot, checked against slot and against the set
 * count gslm_union_binning recorded in the binning workspace -- a slot past it renders a NaN loss instead of a
 * plausible background-only one) ----
 * train_jvp.py:262-277 renders every validation view at six points theta + alpha s (alpha = 2, 1, .., 1/16) of one step
 * s whose xyz group is masked (:221-227).  A view's Gaussians then keep their screen centre and depth order at every
 * point, and each point's exact point list is the subsequence of one list binned over the union of the points' rects:
 * the entries whose tile lies in that point's rect, in the same (tile, depth, index) order.  So a view is binned once
 * for the six points instead of once per point (gslm.lm.LossEvaluator.evaluate_points):
 *   1. each point's render records in depth space, in its own geometry workspace (geoms[a]: gslm_preprocess_views
 *      with the view's depth positions; the depth order from one gslm_preprocess_ordered, order_mode 1);
 *   2. gslm_union_geometry: the union of the n <= 8 points' rects per depth position into union_geom, the tile counts
 *      scanned -- gslm_num_rendered(union_geom) is the union list's length N;
 *   3. gslm_union_binning (workspace >= gslm_union_binning_bytes(N, H, W)): duplicate + tile sort + ranges of the union
 *      list, each entry carrying 4 bits per point through the sort (slot a: the point's quadrant mask of the entry --
 *      the bits its own binning would give it -- and 0 when its tile is outside the point's rect or the Gaussian is
 *      culled there);
 *   4. gslm_rasterize_loss_slot(geom = geoms[a], slot = a): gslm_rasterize_loss's blend + loss over the entries of
 *      slot a -- the same visits in the same order with the same records as the exact render: the same loss, bitwise.
 * The union list's values are depth positions (every pass reads the points' records coalesced in depth order). */
size_t gslm_union_binning_bytes(int64_t num_rendered, int32_t H, int32_t W);
int gslm_union_geometry(const gslm_view* view, int64_t P, const void* const* geoms, int32_t n, size_t set_bytes,
                        void* union_geom, size_t union_geom_bytes, void* stream);
int gslm_union_binning(const gslm_view* view, int64_t P, const void* union_geom, void* binning, size_t binning_bytes,
                       int64_t num_rendered, const void* const* geoms, int32_t n, size_t set_bytes, void* stream);
int gslm_rasterize_loss_slot(const gslm_view* view, int64_t P, const void* geom, size_t set_bytes, const void* binning,
                             size_t binning_bytes, int64_t num_rendered, int32_t slot, int32_t n_sets, const float* gt,
                             const float* alpha_mask, void* scratch, size_t scratch_bytes, double* loss_dev,
                             int32_t accumulate, void* stream);
/* Step 4 for n sets in one pass over the union list (the list walked once; set a + 1's records loaded while set a's
 * hits are visited): geoms[a] / loss_dev[a] are slot first_set + a's (ABI 9: a group of the binning's sets);
 * *loss_dev[a] = [*loss_dev[a] if accumulate] + that set's loss, bitwise gslm_rasterize_loss_slot(geoms[a],
 * first_set + a).  scratch >= gslm_loss_sets_scratch_bytes(n, H, W). */
size_t gslm_loss_sets_scratch_bytes(int32_t n, int32_t H, int32_t W);
int gslm_rasterize_loss_sets(const gslm_view* view, int64_t P, const void* const* geoms, int32_t n, int32_t first_set,
                             size_t set_bytes, const void* binning, size_t binning_bytes, int64_t num_rendered,
                             const float* gt, const float* alpha_mask, void* scratch, size_t scratch_bytes,
                             double* const* loss_dev, int32_t accumulate, void* stream);
/* Convenience: gslm_preprocess + gslm_num_rendered + gslm_rasterize.  If binning_bytes is too
 * small returns GSLM_ERR_CAPACITY with *out_num_rendered set (geometry is valid: call
 * gslm_rasterize with a larger buffer). */
int gslm_forward(const gslm_view* view, const gslm_gaussians* g, void* geom, size_t geom_bytes,
                 void* binning, size_t binning_bytes, void* image, size_t image_bytes,
                 float* out_color, float* out_invdepth, int32_t* out_radii,
                 int64_t* out_num_rendered, void* stream);

/* ---- backward (VJP) of gslm_forward.  dL_dinvdepth may be NULL. ---- */
int gslm_backward(const gslm_view* view, const gslm_gaussians* g, const void* geom, const void* binning,
                  int64_t num_rendered, const void* image, const float* dL_dcolor,
                  const float* dL_dinvdepth, void* scratch, size_t scratch_bytes,
                  const gslm_grads* out, void* stream);

/* ---- forward-mode tangent (JVP) of gslm_forward; reuses the forward's sorted lists.
 * means2D_tangent [P,3] may be NULL. ---- */
int gslm_jvp(const gslm_view* view, const gslm_gaussians* g, const gslm_gaussians* tangent,
             const float* means2D_tangent, const void* geom, const void* binning, int64_t num_rendered,
             const void* image, void* scratch, size_t scratch_bytes, float* out_color_t,
             float* out_invdepth_t, void* stream);

/* ---- fused LM normal-equations product of one view:
 *   y += 2 * J^T ( w (.) (J v) )     (J: d clamp-free render / d raw params, g->raw must be 1)
 * w [3,H,W] is the per-pixel weight m^2 * 1[0 <= R <= 1] of the disable_ssim residual
 * (batch_training_loss.py:10-17; the factor 2 is the [r; r] aliasing).
 * mask_xyz = 1 freezes the xyz group (train_jvp.py:221-227): v.xyz is ignored, y.xyz untouched. ---- */
int gslm_matvec_view(const gslm_view* view, const gslm_gaussians* g, const gslm_grads* v,
                     const float* pixel_weight, int32_t mask_xyz, const void* geom, const void* binning,
                     int64_t num_rendered, const void* image, void* scratch, size_t scratch_bytes,
                     const gslm_grads* y, void* stream);

/* The three stages of gslm_matvec_view, separately launchable (profiling, overlap):
 * TANGENT: per-Gaussian tangent records from v; RENDER: fused JVP->VJP tile pass writing one row per
 * (tile, Gaussian); GATHER: per-Gaussian gather-sum + chain rule, y += ... */
#define GSLM_STAGE_TANGENT 1
#define GSLM_STAGE_RENDER 2
#define GSLM_STAGE_GATHER 4
#define GSLM_STAGE_ALL 7
#define GSLM_STAGE_OVERWRITE 8 /* GATHER writes y instead of accumulating into it */
#define GSLM_STAGE_SCREEN 16   /* view-sharded exchange: write this view's per-Gaussian screen-space sums to
                                  opts->screen_out (see gslm_gather_screen) instead of gathering into y */
/* opts->flags: GSLM_MV_TAIL_CLEAN -- the caller guarantees that the LM row map an earlier RENDER stage built
 * for this same geometry / binning is intact (no forward or drop-in backward, no other use of the scratch's map
 * or of the binning buffer since).  The row map gives gradient rows only to HEAD list entries (positions below
 * the largest n_contrib of their tile: every later entry's row would be zero), packed per Gaussian; it holds
 * each sorted entry's row slot (in the binning buffer's free sort ping-pong half) and the per-Gaussian row
 * offsets (in the scratch).  It depends on the geometry only, so an LM step's CG loop builds it once; without
 * the flag RENDER rebuilds it. */
#define GSLM_MV_TAIL_CLEAN 1
/* opts->flags: GSLM_MV_SH_REST_PROJECTED -- single-view Krylov space of the SH-rest group.  With one view,
 * Gaussian i's SH-rest columns of J are B_rest(dir_i) (x) d rgb, so J^T W J + D (D a scalar on the group)
 * maps span{B_rest(dir_i) (x) e_c} to itself and every CG iterate started from J^T b lies in it.  With this
 * flag the SH-rest group of v, y and xpby_s holds 3 floats per Gaussian (sh_rest_stride 3): the coordinates
 * along Bh = B_rest / |B_rest| (the same operator on the 3(M-1) -> 3 coordinates of that span; convert with
 * gslm_sh_rest_project).  Not for the SCREEN stage (multi-view). */
#define GSLM_MV_SH_REST_PROJECTED 2
typedef struct gslm_matvec_opts {
  int32_t stages;         /* GSLM_STAGE_* bits; 0 means GSLM_STAGE_ALL (accumulate) */
  int32_t flags;          /* GSLM_MV_* bits */
  const double* damp7;    /* host array (GaussianModelDampMatrix order: xyz, dc, rest, scaling, rotation,
                             opacity, exposure) or NULL; when set GATHER also adds D v (exposure untouched) */
  double* dot_vy;         /* device double or NULL: receives <v, y> over the gathered groups after GATHER */
  void* dot_scratch;      /* device scratch for dot_vy, >= gslm_dot_scratch_bytes(P) bytes */
  size_t dot_scratch_bytes;
  /* Fused CG direction update (the p = s + beta p of conjugate_gradient.py:121-123, deferred into the
   * next product): when xpby_s is set, before the TANGENT stage every group of v becomes
   * s + beta v, beta = *beta_num / *beta_den (device doubles), and so does the flat tail
   * xpby_tail_v[0..xpby_tail_n) (the exposure group) from xpby_tail_s.  v's groups must be
   * contiguous per Gaussian (sh_dc_stride 3, sh_rest_stride 3(M-1)) and writable.  Same arithmetic
   * as gslm_xpby_dev.  With mask_xyz the xyz group is not touched (zero in every LM iterate). */
  const gslm_grads* xpby_s;
  const double* beta_num;
  const double* beta_den;
  float* xpby_tail_v;
  const float* xpby_tail_s;
  int64_t xpby_tail_n;
  float* screen_out;      /* GSLM_STAGE_SCREEN output, P x 8 floats */
  /* J^T seed instead of J^T W J v: when set, RENDER runs only the back-to-front pass with dL/dcolor =
   * pixel_seed ([3,H,W], e.g. gslm_lm_residual's seed) into the LM rows, and GATHER sums them as usual
   * (v is then only read for D v / dot_vy).  Needs mask_xyz; excludes TANGENT, SCREEN and xpby.  This
   * is the J^T b of an LM step (train_jvp.py:243, solver_functions.py:101-132) on the fused path. */
  const float* pixel_seed;
  /* J v only: when set, RENDER runs the front-to-back tangent pass alone and writes the colour tangent
   * J v ([3,H,W], before the clamp / mask) to jv_out; no rows are written, so GATHER must not be in the
   * same call.  The SSIM residual's product uses it: J v -> gslm_ssim_normal -> pixel_seed. */
  float* jv_out;
  /* Deferred x update of the previous CG step (conjugate_gradient.py:95 x += alpha p), fused with xpby:
   * when alpha_num is set, every element of v (groups and tail) first adds (alpha_num / alpha_den) v into
   * x, where x lives xpby_x_offset bytes from v (x and v two flat vectors of the same layout).  Same
   * arithmetic as gslm_cg_update's x update, so the iterates are bitwise those of the undeferred loop. */
  const double* alpha_num;
  const double* alpha_den;
  int64_t xpby_x_offset;
  /* Gaussian-sharded exchange (gslm_tangent_views below): when set, RENDER reads this view's tangent render
   * records (gslm_tangent_views' output once exchanged: [>= P][8] floats with mask_xyz, [>= P][12] without)
   * instead of the TANGENT stage's (TANGENT must be off). */
  const float* trec_in;
  /* gslm_gather_screen only: Gaussians between consecutive views' blocks of screen (0 means P). */
  int64_t screen_stride;
  /* Device CG control block of gslm_cg_monitor, or NULL: when cg_ctl[0] != 0 (the solve's stopping tests have
   * fired) the TANGENT, RENDER and GATHER kernels of this call return without work (and without writing y,
   * the dot or the direction update), so a host can enqueue a whole CGLS schedule without reading the tests
   * back each iteration.  gslm_matvec_view_ex, gslm_tangent_views and gslm_gather_screen (the Gaussian-sharded
   * exchange's stages) all honour it. */
  const double* cg_ctl;
  /* gslm_tangent_views / gslm_gather_screen only (ABI 6): SH-rest coordinates of the Gaussian-sharded exchange.
   * When rest_basis is set, the SH-rest group of v, y (and of the fused direction update's s) holds 3 rest_views
   * floats per Gaussian -- the coordinates of the SH-rest vector in an orthonormal basis of span{B_rest(dir_b)}
   * over the job's rest_views views b -- and rest_basis is gslm_rest_basis' per-Gaussian factor R of those
   * views; view k of this call is column view_base + k of R.  See gslm_rest_basis. */
  const float* rest_basis;
  int32_t rest_views;
  int32_t view_base;
} gslm_matvec_opts;
int gslm_matvec_view_ex(const gslm_view* view, const gslm_gaussians* g, const gslm_grads* v,
                        const float* pixel_weight, int32_t mask_xyz, const void* geom, const void* binning,
                        int64_t num_rendered, const void* image, void* scratch, size_t scratch_bytes,
                        const gslm_grads* y, const gslm_matvec_opts* opts, void* stream);

/* SH-rest coordinates of GSLM_MV_SH_REST_PROJECTED for this view (gaussians: the raw leaves; means3D and
 * max_coeffs are used).  mode 0 (expand): out[i*out_stride + 3(k-1) + c] = Bh_k(dir_i) in[i*in_stride + c];
 * mode 1 (project): out[i*out_stride + c] = sum_k Bh_k(dir_i) in[i*in_stride + 3(k-1) + c]; Bh = B_rest/|B_rest|
 * over the view's active degree (inactive coefficients expand to 0). */
int gslm_sh_rest_project(const gslm_view* view, const gslm_gaussians* g, int32_t mode, const float* in,
                         int64_t in_stride, float* out, int64_t out_stride, void* stream);

/* ---- view-sharded exchange (multi-GPU LM product), SURVEY 8(e) ----
 * Instead of all-reducing the param-space partial J^T W J v (F = 59 floats per Gaussian at SH 3),
 * every rank all-gathers per-view screen-space sums (8 floats per Gaussian per view) and applies the
 * per-view chains itself.  GSLM_STAGE_SCREEN of gslm_matvec_view_ex writes, for Gaussian i of the
 * view, screen[8 i .. 8 i + 7] = (dL/dconic a, b, c, dL/dopacity_eff, dL/dr, dL/dg, dL/db, flags),
 * flags = bit 31 visible | bits 0-2 SH clamp mask (as float bits); xyz must be masked.
 * gslm_gather_screen(views[0..nviews), screen[nviews][P][8]) then writes
 *   y = sum_b J_b^T screen_b [+ D v]   (views summed in index order: identical on every rank),
 * with opts->stages' OVERWRITE bit, damp7 and dot_vy as in gslm_matvec_view_ex.  nviews <= 16 per
 * call (accumulate further calls).  Replaces the reduction of solver_functions.py:110-121. */
int gslm_gather_screen(const gslm_view* views, int32_t nviews, const gslm_gaussians* g, const float* screen,
                       const gslm_grads* v, const gslm_grads* y, const gslm_matvec_opts* opts, void* stream);

/* ---- Gaussian-sharded exchange (multi-GPU LM product; gslm.parallel.GaussianShardedOperator, exchange
 * "gaussian", the default of gslm.parallel.ShardedLMProblem when every rank renders the same number of views) ----
 * Rank r owns Gaussians [r S, (r + 1) S) of every CG vector and the vector algebra on them.  Per product:
 *   gslm_tangent_views   this shard's tangent render records for EVERY view b (chain_jvp, the TANGENT stage
 *                        of gslm_matvec_view_ex for a Gaussian range) -> all-to-all -> each rank holds its
 *                        own view's [P][8] table (mask_xyz; [P][12] without) for opts->trec_in;
 *   RENDER | SCREEN      with opts->trec_in -> [P][8] screen sums -> all-to-all -> each rank holds
 *                        screen[b][S][8] of its shard for every view;
 *   gslm_gather_screen   over the shard (g = the shard's slice of the leaves, opts->screen_stride = S).
 * A rank receives (32 + 32) (n - 1) / n bytes per Gaussian per view it renders instead of the screen
 * all-gather's 32 (n - 1), and runs 1/n of the chains and vector algebra.
 * gslm_view_flags: out[i] = 0 if Gaussian i touches no tile of the preprocessed view, else
 * 0x80000000 | its 3 SH-clamp bits (the flags word of the SCREEN rows); exchanged once per geometry. */
int gslm_view_flags(const void* geom, int64_t P, uint32_t* out, void* stream);
/* trec_out[(b trec_stride + i) * R ..] = tangent render record of shard Gaussian i in view b where
 * vflags[b flags_stride + i] is visible (other records untouched), R = 8 floats with mask_xyz (the LM rows:
 * [da db dc dop | dr dg db 0], the conic / opacity / colour tangents) or 12 without
 * ([dx dy da db | dc dop dr dg | db dinv 0 0]), b < nviews (<= 16).  g / v: the shard's
 * leaves and direction (P = shard size, SH-rest stride 3(M-1)); opts (or NULL): only the fused direction
 * update (xpby_s, beta_*, alpha_*, xpby_x_offset, xpby_tail_*) of gslm_matvec_view_ex, applied once before
 * the views' tangents.  The flat tail (xpby_tail_*) is updated once per call, so it must be this rank's
 * private copy and be passed to one call per product (several calls of one product: only the first gets
 * opts); an empty shard (P = 0) with a tail still applies the tail's update.
 * The trec_in table a RENDER stage reads must hold the records of every Gaussian the vflags of that same
 * geometry (gslm_view_flags of this view's current preprocess) mark visible: the kernel cannot check it. */
int gslm_tangent_views(const gslm_view* views, int32_t nviews, const gslm_gaussians* g, const gslm_grads* v,
                       int32_t mask_xyz, const uint32_t* vflags, int64_t flags_stride, float* trec_out,
                       int64_t trec_stride, const gslm_matvec_opts* opts, void* stream);

/* ---- SH-rest coordinates of the Gaussian-sharded exchange (ABI 6) ----
 * The SH-rest column of J for view b is B_rest(dir_b) (x) (d rgb), B_rest the view's SH basis over
 * coefficients 1..nc-1.  So with V views every CGLS iterate started from J^T b keeps each Gaussian's SH-rest
 * group in span{B_rest(dir_b) : b < V} (x) R^3, which (J^T J + D) maps into itself (D is a scalar on the group):
 * 3 V coordinates per Gaussian in an orthonormal basis Q of that span replace 3(M-1) floats (V = 1 is
 * GSLM_MV_SH_REST_PROJECTED).  With B = Q R (Gram-Schmidt in view order; R upper triangular, the Cholesky
 * factor of the Gram matrix B^T B, computed in double), view b's colour tangent is sum_{j<=b} R[j][b] c_j and
 * its gradient adds R[j][b] dL/drgb_b to coordinate j: the per-Gaussian kernels need R only.  A view whose
 * direction adds less than 1e-6 of its norm to the span of the earlier ones (R[b][b]^2 <= 1e-12 G[b][b]) gets
 * row b of R zeroed: its coordinate stays 0.
 *   gslm_rest_basis   R_out[i * V(V+1)/2 + b(b+1)/2 + j] = R[j][b] (j <= b), float, for the V = nviews views
 *                     (1..GSLM_MAX_REST_VIEWS) and the Gaussians of g (means3D and max_coeffs used; the SH
 *                     degree of views[0]).
 *   gslm_rest_coords  mode 0 (expand): out[i*out_stride + 3(k-1) + c] = (Q c_i)[k][c] (0 for k >= nc);
 *                     mode 1 (project): out[i*out_stride + 3j + c] = (Q^T t_i)[j][c], t_i = in[i*in_stride ..]
 *                     in the [M-1][3] layout (the orthogonal projection onto the span). */
#define GSLM_MAX_REST_VIEWS 8
int gslm_rest_basis(const gslm_view* views, int32_t nviews, const gslm_gaussians* g, float* R_out, void* stream);
int gslm_rest_coords(const gslm_view* views, int32_t nviews, const gslm_gaussians* g, const float* R, int32_t mode,
                     const float* in, int64_t in_stride, float* out, int64_t out_stride, void* stream);

/* ---- device-resident CG vector algebra on flat fp32 vectors (param-space, n floats) ----
 * damp_groups: per-element damping is d[group(i)] with group boundaries bounds[0..ngroups]. */
size_t gslm_dot_scratch_bytes(int64_t n);
/* out (double, device) = sum_i a_i b_i d_i  (d = NULL means 1).  Deterministic. */
int gslm_dot(const float* a, const float* b, const int64_t* group_bounds, const double* group_damp,
             int32_t ngroups, int64_t n, void* scratch, double* out_dev, void* stream);
/* y = alpha * x + y, alpha read from device memory as num/den (den==NULL -> 1), times sign. */
int gslm_axpy_dev(int64_t n, const double* num_dev, const double* den_dev, float sign, const float* x,
                  float* y, void* stream);
/* p = s + beta p, beta = num/den from device memory */
int gslm_xpby_dev(int64_t n, const float* s, const double* num_dev, const double* den_dev, float* p,
                  void* stream);
/* One CG step, a = gam / del read from device memory:  x += a p;  s -= a q;
 * *gam_new_dev = <s, s> (scratch >= gslm_dot_scratch_bytes(n)).  Vectors 16-byte aligned.
 * x == NULL: only s -= a q and <s, s> (the x update deferred into the next product's xpby, see
 * gslm_matvec_opts.alpha_num; p is then not read). */
int gslm_cg_update(int64_t n, const double* gam_dev, const double* del_dev, const float* p, const float* q,
                   float* x, float* s, void* scratch, double* gam_new_dev, void* stream);
/* gslm_cg_update plus the residual monitor of conjugate_gradient.py:103-104 in the same pass:
 * *xg_dev = <x_new, g>, *xs_dev = <x_new, s_new> (g = J^T b).  scratch >= 3 * 1024 doubles.
 * cg_ctl (or NULL): gslm_cg_monitor's control block; with cg_ctl[0] != 0, *del_dev < 1e-20 (the early
 * termination of conjugate_gradient.py:88-91) or a non-finite *del_dev, x and s are left untouched. */
int gslm_cg_update_monitor(int64_t n, const double* gam_dev, const double* del_dev, const float* p, const float* q,
                           float* x, float* s, const float* g, void* scratch, size_t scratch_bytes,
                           double* gam_new_dev, double* xg_dev, double* xs_dev, const double* cg_ctl, void* stream);
/* The stopping tests of cgls_damped (conjugate_gradient.py:88-117) on the device, one launch per inner iteration
 * after gslm_cg_update_monitor (and after any cross-rank sums of its scalars).  cg_ctl = doubles
 * [stop, iters, last_res, n_hist, history[max_hist]], initialised by the caller to [0, 0, +inf, 0, ...]:
 *   *del < 1e-20 -> stop = 1;  res = (*b2 - *xg) - *xs is appended to history;  res > last_res -> stop = 2;
 *   *gam_new < max(tol sqrt(*gam), atol) -> stop = 3;  otherwise iters += 1.
 * Checked before those: any of *gam, *gam_new, *del, *xg, *xs not finite -> stop = 4 (GSLM_CG_STOP_NONFINITE; the
 * reference's NaN asserts, solver/solver_functions.py:125-130) -- the caller must not use the iterate.
 * Once stop != 0 every later gslm_cg_monitor / gslm_cg_update_monitor / product with opts->cg_ctl is a no-op. */
#define GSLM_CG_STOP_NONFINITE 4
int gslm_cg_monitor(const double* gam_dev, const double* gam_new_dev, const double* del_dev, const double* xg_dev,
                    const double* xs_dev, const double* b2_dev, double tol, double atol, double* cg_ctl,
                    int32_t max_hist, void* stream);
/* *out_dev = sum of np per-block partials (second pass of the fused dots) */
int gslm_dot_finalize(const void* partials, int32_t np, double* out_dev, void* stream);
/* y += d[group] * x (the damping term D x) */
int gslm_damp_add(int64_t n, const float* x, const int64_t* group_bounds, const double* group_damp,
                  int32_t ngroups, float* y, void* stream);

/* ---- RCCL collectives over xGMI, communicator handle passed in (SURVEY 8(b) "gslm_allreduce*", 8(e)) ----
 * The reference has no multi-GPU code (its LinearSolverFunctions renders a view batch serially on one GPU,
 * solver/solver_functions.py:88-93,110-121); these replace the all-reduce of J^T r / J^T J v and of the CG scalars
 * that SURVEY 8(e) adds, and carry the Gaussian-sharded exchange's all-to-alls, for a host that does not go through
 * torch.distributed (gslm.parallel uses them with GSLM_COMM=native; its default is torch.distributed's "nccl"
 * backend, the same RCCL).  One rank calls gslm_comm_unique_id and the host broadcasts the gslm_comm_id_bytes()
 * bytes; every rank then calls gslm_comm_init with its HIP device current (blocks until all ranks joined).  The
 * collectives are enqueued on `stream` (RCCL stream semantics: ordered after the kernels enqueued on it before, and
 * before those after) and never synchronise the host.  librccl is loaded on the first call (GSLM_ERR_HIP if absent). */
int32_t gslm_comm_id_bytes(void);
int gslm_comm_unique_id(void* id_out);
int gslm_comm_init(const void* id, int32_t nranks, int32_t rank, void** comm_out);
int gslm_comm_destroy(void* comm);
/* in-place sums over the ranks: param-space partial products (f32), CG scalars / losses (f64) */
int gslm_allreduce_sum_f32(void* comm, float* buf, int64_t n, void* stream);
int gslm_allreduce_sum_f64(void* comm, double* buf, int64_t n, void* stream);
/* recv[r * bytes_per_rank ...] = rank r's send[rank * bytes_per_rank ...] (the Gaussian-sharded exchange's records
 * and screen sums, gslm_tangent_views / GSLM_STAGE_SCREEN) */
int gslm_alltoall(void* comm, const void* send, void* recv, int64_t bytes_per_rank, void* stream);
/* recv[r * bytes_per_rank ...] = rank r's send[0 .. bytes_per_rank) (the screen exchange's per-view sums,
 * gslm_gather_screen) */
int gslm_allgather(void* comm, const void* send, void* recv, int64_t bytes_per_rank, void* stream);

/* ---- LM residual epilogue of one view (replaces the render clamp
 * gaussian_renderer/batch_render.py:118 + compute_batch_loss_block, solver/batch_training_loss.py:10-17,
 * 56-67, disable_ssim=True, and loss_scalar, solver/loss_image_state.py:16-19) ----
 * color / gt / residual / weight / seed are [3,H,W]; alpha_mask [H,W] or NULL (= 1).  Writes
 *   residual = m clamp(color, 0, 1) - gt          (NULL: not written)
 *   weight   = m^2 1[0 <= color <= 1]             (the per-pixel weight of gslm_matvec_view_ex; NULL: not
 *                                                  written -- with residual and seed NULL too, the loss alone:
 *                                                  the line search's validation loss)
 *   seed     = -2 m 1[0 <= color <= 1] residual   (NULL: not written; gslm_backward's dL/dcolor for J^T b)
 * and *loss_dev (device double) = [*loss_dev if accumulate] + 2 sum residual^2 ([r; r] aliasing).
 * Deterministic (fixed two-pass reduction); scratch >= gslm_residual_scratch_bytes(H, W). */
size_t gslm_residual_scratch_bytes(int32_t H, int32_t W);
int gslm_lm_residual(int32_t H, int32_t W, const float* color, const float* gt, const float* alpha_mask,
                     float* residual, float* weight, float* seed, void* scratch, size_t scratch_bytes,
                     double* loss_dev, int32_t accumulate, void* stream);

/* ---- SSIM residual of the LM step (solver/batch_training_loss.py:18-30 with
 * disable_ssim=False, FUSED_SSIM_AVAILABLE=False, on utils/loss_utils.py:91-122 ssim_per_pixel) ----
 * Per view: r1 = a sqrt(|x - gt| + 1e-6), r2 = b sqrt(|1 - SSIM(x, gt)| + 1e-6) with x = m clamp(color, 0, 1),
 * a = sqrt((1 - lambda) / 3HW), b = sqrt(lambda / 3HW) (batch_training_loss.py:69-77); residual vector
 * [r1; r2], loss = ||r1||^2 + ||r2||^2.  `state` (gslm_ssim_state_bytes) keeps the linearisation at x.
 * gslm_ssim_residual: *loss_dev = [*loss_dev if accumulate] + loss; r1 / r2 / seed optional; seed =
 *   dL/dcolor of J^T b = -M (d1 r1 + S^T c2 r2) (feed it to gslm_matvec_view_ex's pixel_seed).
 * gslm_ssim_normal: u = M (d1^2 + S^T c2^2 S) M jv, the image-space factor of J^T J: with jv = J v
 *   (gslm_matvec_opts.jv_out), pixel_seed = u gives J^T J v.  Overwrites the state's scratch plane, so
 *   call gslm_ssim_residual with seed != NULL before the first gslm_ssim_normal of a geometry. */
size_t gslm_ssim_state_bytes(int32_t H, int32_t W);
int gslm_ssim_residual(int32_t H, int32_t W, const float* color, const float* gt, const float* alpha_mask,
                       float lambda_dssim, void* state, size_t state_bytes, float* r1, float* r2, float* seed,
                       double* loss_dev, int32_t accumulate, void* stream);
int gslm_ssim_normal(int32_t H, int32_t W, const float* gt, void* state, const float* jv, float* u, void* stream);

/* ---- the first-order loss's SSIM term (train.py:121-125 ssim(image, gt) = utils/loss_utils.py:59-89 with
 * size_average; upstream's optional fused_ssim plays this role) ----
 * img, gt [C,H,W] f32.  gslm_ssim_mean: *ssim_out (device f32) = mean of the SSIM map (11-tap Gaussian
 * window, sigma 1.5, zero padding), and `state` keeps the map's linearisation for the backward.
 * gslm_ssim_mean_backward: grad_img = *grad_out * d mean(SSIM) / d img (grad_out: device f32 scalar). */
size_t gslm_ssim_mean_state_bytes(int32_t C, int32_t H, int32_t W);
int gslm_ssim_mean(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, void* state,
                   size_t state_bytes, float* ssim_out, void* stream);
int gslm_ssim_mean_backward(int32_t C, int32_t H, int32_t W, const float* img, const float* gt, const void* state,
                            const float* grad_out, float* grad_img, void* stream);

/* ---- distCUDA2 (simple-knn, called at scene/gaussian_model.py:249 to initialise scales) ----
 * out[i] = mean of the squared distances from point i to its 3 nearest other points (exact; FLT_MAX
 * for missing neighbours when n < 4).  xyz [n,3] f32.  Synchronises once (bounding box -> grid size).
 * scratch >= gslm_knn_scratch_bytes(n). */
size_t gslm_knn_scratch_bytes(int64_t n);
int gslm_knn3_mean_dist(int64_t n, const float* xyz, float* out, void* scratch, size_t scratch_bytes, void* stream);

/* ---- first-order training step ----
 * One parameter group of GaussianModel.training_setup (scene/gaussian_model.py:273-280: xyz, f_dc, f_rest,
 * opacity, scaling, rotation; the exposure optimizer of :291 is one more group).  grad == NULL skips the
 * group (torch.optim skips parameters whose .grad is None). */
#define GSLM_ADAM_MAX_GROUPS 8
typedef struct gslm_adam_group {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;                   /* floats in the group */
  int32_t floats_per_gaussian; /* sparse: n == floats_per_gaussian * num_gaussians */
  int32_t _pad;
  double lr;                   /* param_group["lr"] */
  int64_t step;                /* dense: state["step"] after its increment (bias correction 1 - beta^step) */
} gslm_adam_group;
/* sparse == 0: torch.optim.Adam(params, lr, eps) step (train.py:184-186) -- its foreach arithmetic in f32:
 *   m += (1-b1)(g-m); v = v b2 + (1-b2) g g; p += (-lr/(1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps).
 * sparse != 0: SparseGaussianAdam.step(visible, num_gaussians) (train.py:180-183; gaussian_model.py:29,286,
 *   upstream 3dgs_accel rasterizer, absent): elements of Gaussians with visible[g] == 0 untouched, others
 *   m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p += -lr m / (sqrt(v) + eps)  (no bias correction).
 * One launch for all groups. */
int gslm_adam_step(const gslm_adam_group* groups, int32_t ngroups, double beta1, double beta2, double eps,
                   const uint8_t* visible, int64_t num_gaussians, int32_t sparse, void* stream);
/* train.py:166-167 (gaussian_model.py:561-563) fused, for the Gaussians with radii > 0 (render()'s
 * visibility_filter): max_radii2D = max(max_radii2D, radii) (skipped when max_radii2D is NULL),
 * xyz_gradient_accum += ||means2D_grad[i, 0:2]||, denom += 1.  means2D_grad rows are grad_stride floats. */
int gslm_densify_stats(int64_t P, const float* means2D_grad, int64_t grad_stride, const int32_t* radii,
                       float* max_radii2D, float* xyz_gradient_accum, float* denom, void* stream);

/* ---- diagnostics: device-to-device copies of internal buffers (any output may be NULL) ----
 * point_list [N] u32 (Gaussian id per sorted slot), ranges [ntiles*2] u32, tiles_touched [P] u32,
 * final_T [H*W] f32, n_contrib [H*W] u32, render records [P*12] f32. */
int gslm_inspect(const void* geom, int64_t P, const void* binning, int64_t num_rendered, int32_t H, int32_t W,
                 const void* image, uint32_t* point_list, uint32_t* ranges, uint32_t* tiles_touched,
                 float* final_T, uint32_t* n_contrib, float* records, void* stream);

/* Device self-test of the wave primitives (one 64-lane wave).  in: [64][8] floats, out: [64].
 * which = 0: transposed 8-value reduction (lane l returns the sum of value (l >> 3) & 7);
 * which = 1: DPP sum of in[l*8] (lane 63 returns the total). */
int gslm_selftest(int32_t which, const float* in, float* out, void* stream);
/* Device self-test of the library's exclusive u32 scan (the tile-count and LM row-map scans): out[i] = sum_{j<i} in[j],
 * *total = the sum (both device).  force_top != 0 takes the long-scan form (a scan of the block sums in a launch of
 * its own, used above 4096 blocks of 2048) at any n.  tmp: >= 8 ceil(n / 2048) + 64 bytes of device scratch, rounded
 * up to a multiple of 256. */
int gslm_selftest_scan(const uint32_t* in, uint32_t* out, int64_t n, int32_t force_top, void* tmp, size_t tmp_bytes,
                       uint32_t* total, void* stream);

const char* gslm_last_error(void);
int gslm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GSLM_H */
