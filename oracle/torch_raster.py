"""ORACLE -- test infrastructure only (never imported by the product path).

A CPU restatement, in PyTorch, of the tile rasterizer that the reference calls through
`diff_gaussian_rasterization` (absent submodule).  Call sites pinning the interface:
`gaussian_renderer/__init__.py:36-52,90-110`, `gaussian_renderer/batch_render.py:33-50,89-108`,
`gaussian_renderer/reference_render.py:102`.  Semantics follow SURVEY Appendix A (upstream
graphdeco forward) step by step; every step cites the in-repo Python it agrees with where one exists:

  * camera transforms ........ utils/graphics_utils.py:38-71, scene/cameras.py:86-89
  * cov3D = L L^T ............ scene/gaussian_model.py:36-40, utils/general_utils.py:79-111
  * SH -> RGB ................ utils/sh_utils.py:57-112 and gaussian_renderer/__init__.py:75-80
  * blend / binning .......... SURVEY App. A steps 10-11 (upstream forward.cu renderCUDA)

Differentiation: the forward is written so that torch reverse-mode autograd reproduces the
upstream backward and torch forward-AD gives its transpose, i.e. the JVP:
  - alpha = min(0.99, o*G) is straight-through (upstream: dL/dopacity = G*dL/dalpha, no clamp mask);
  - the +-1.3 tan-FoV clamp of t.x/t.z gives zero derivative outside and no t.z cross term
    (upstream computeCov2D backward: x_grad_mul / y_grad_mul);
  - SH colour clamp: gradient masked where result+0.5 < 0 (torch.clamp_min semantics);
  - skip / stop decisions (power > 0, alpha < 1/255, T < 1e-4) are frozen at the primal.

Rasterizer numerics are "parity unpinned" against the (absent) CUDA binary: this restatement is
pinned by the reference's importable Python (SH, covariance, cameras, solver; tests/golden/) and by
finite differences / the adjoint identity (tests/test_oracle.py).
"""
import math

import numpy as np
import torch

BLOCK_X = 16
BLOCK_Y = 16

# utils/sh_utils.py:26-55
SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]


def sqrt_ieee(x):
    """sqrt whose VALUE is the correctly rounded float32 sqrt (IEEE 754, as the GPU's sqrtf and
    upstream's CUDA sqrtf), with torch's derivative (straight-through, also under forward-AD).
    torch's CPU Vectorized sqrt is not correctly rounded and its result depends on the host's
    vector ISA (measured: 0.6% of random inputs on one AVX-512 host, 17% on another), which made
    the restatement's radii host-dependent at the 1M-Gaussian scale."""
    s = torch.sqrt(x)
    base = s.detach()
    exact = torch.from_numpy(np.sqrt(x.detach().cpu().numpy())).to(x.device)
    return s + (exact - base)


def eval_sh(deg, sh, dirs):
    """`utils/sh_utils.py:57-112` with sh laid out [P, K, 3] (reference `get_features` layout)."""
    result = SH_C0 * sh[:, 0]
    if deg > 0:
        x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
        result = result - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz = x * x, y * y, z * z
            xy, yz, xz = x * y, y * z, x * z
            result = (result + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5]
                      + SH_C2[2] * (2.0 * zz - xx - yy) * sh[:, 6]
                      + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                result = (result + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9]
                          + SH_C3[1] * xy * z * sh[:, 10]
                          + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11]
                          + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
                          + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13]
                          + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                          + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return result


def quat_to_rotmat(q):
    """Rotation matrix of an (un-renormalised) wxyz quaternion, `utils/general_utils.py:91-99`
    (the kernel does not renormalise: normalisation happens in Python, gaussian_model.py:50)."""
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], dim=1).view(-1, 3, 3)


def compute_cov3d(scales, scale_modifier, rotations):
    """Upper triangle [s00,s01,s02,s11,s12,s22] of R diag(s)^2 R^T (gaussian_model.py:36-40)."""
    R = quat_to_rotmat(rotations)
    s = scale_modifier * scales
    L = R * s[:, None, :]
    # S = L L^T with every product and sum an explicit float32 elementwise op in a fixed association:
    # a batched matmul (`L @ L.transpose`) is host-dependent (BLAS kernels may fuse multiply-adds or
    # reorder on AVX-512 hosts), which made the restatement itself differ by ulps between machines.

    def row_dot(i, j):
        return (L[:, i, 0] * L[:, j, 0] + L[:, i, 1] * L[:, j, 1]) + L[:, i, 2] * L[:, j, 2]

    return torch.stack([row_dot(0, 0), row_dot(0, 1), row_dot(0, 2), row_dot(1, 1), row_dot(1, 2), row_dot(2, 2)],
                       dim=1)


def _tp43(M, x, y, z, r):
    # transformPoint4x3 / 4x4 row r of a column-major 4x4
    return x * M[r] + y * M[4 + r] + z * M[8 + r] + M[12 + r]


def preprocess(means3D, means2D, opacities, shs, colors_precomp, scales, rotations, cov3D_precomp, st):
    """Per-Gaussian stage.  Returns a dict of per-Gaussian tensors."""
    H, W = int(st.image_height), int(st.image_width)
    gx = (W + BLOCK_X - 1) // BLOCK_X
    gy = (H + BLOCK_Y - 1) // BLOCK_Y
    V = st.viewmatrix.reshape(-1).to(means3D.dtype)
    Pm = st.projmatrix.reshape(-1).to(means3D.dtype)
    x, y, z = means3D[:, 0], means3D[:, 1], means3D[:, 2]

    # 1. cull (in_frustum): p_view.z <= 0.2
    tx, ty, tz = _tp43(V, x, y, z, 0), _tp43(V, x, y, z, 1), _tp43(V, x, y, z, 2)
    # 2. project; p_proj = p_hom * (1 / (w + 1e-7))
    hx, hy, hw = _tp43(Pm, x, y, z, 0), _tp43(Pm, x, y, z, 1), _tp43(Pm, x, y, z, 3)
    p_w = 1.0 / (hw + 1e-7)
    px = hx * p_w + means2D[:, 0]
    py = hy * p_w + means2D[:, 1]

    # 3. cov3D
    if cov3D_precomp is not None:
        cov3D = cov3D_precomp
    else:
        cov3D = compute_cov3d(scales, st.scale_modifier, rotations)

    # 4. cov2D (EWA) with the +-1.3 tan-FoV clamp
    fx = W / (2.0 * st.tanfovx)
    fy = H / (2.0 * st.tanfovy)
    limx = 1.3 * st.tanfovx
    limy = 1.3 * st.tanfovy
    txtz = tx / tz
    tytz = ty / tz
    inx = ((txtz >= -limx) & (txtz <= limx)).detach()
    iny = ((tytz >= -limy) & (tytz <= limy)).detach()
    tcx = torch.where(inx, txtz * tz, (txtz.clamp(-limx, limx) * tz).detach())
    tcy = torch.where(iny, tytz * tz, (tytz.clamp(-limy, limy) * tz).detach())
    # fx / tz as a tensor division: torch evaluates `python_scalar / tensor` as reciprocal(tensor) *
    # scalar (two roundings), upstream divides once (computeCov2D); that differed in 26% of the J00s
    J00 = torch.full_like(tz, fx) / tz
    J02 = -(fx * tcx) / (tz * tz)
    J11 = torch.full_like(tz, fy) / tz
    J12 = -(fy * tcy) / (tz * tz)
    # A = J * W2C  (2x3); W2C[j][k] = V[4k + j]
    A0 = [J00 * V[4 * k + 0] + J02 * V[4 * k + 2] for k in range(3)]
    A1 = [J11 * V[4 * k + 1] + J12 * V[4 * k + 2] for k in range(3)]
    s00, s01, s02, s11, s12, s22 = [cov3D[:, i] for i in range(6)]
    Sg = [[s00, s01, s02], [s01, s11, s12], [s02, s12, s22]]

    def quad(a, b):
        return sum(a[k] * sum(Sg[k][l] * b[l] for l in range(3)) for k in range(3))

    c00 = quad(A0, A0)
    c01 = quad(A0, A1)
    c11 = quad(A1, A1)

    # 5. low-pass + antialiasing
    det0 = c00 * c11 - c01 * c01
    c00 = c00 + 0.3
    c11 = c11 + 0.3
    det = c00 * c11 - c01 * c01
    if st.antialiasing:
        h = sqrt_ieee(torch.clamp_min(det0 / det, 0.000025))
    else:
        h = torch.ones_like(det)
    det_ok = (det != 0).detach()
    det_safe = torch.where(det_ok, det, torch.ones_like(det))
    det_inv = 1.0 / det_safe
    conic = torch.stack([c11 * det_inv, -c01 * det_inv, c00 * det_inv], dim=1)

    # 6. radius
    with torch.no_grad():
        mid = 0.5 * (c00 + c11)
        lam1 = mid + sqrt_ieee(torch.clamp_min(mid * mid - det, 0.1))
        radius = torch.ceil(3.0 * sqrt_ieee(lam1))

    # 7. screen position and rect
    # ndc2Pix is evaluated in double upstream (`((v + 1.0) * S - 1.0) * 0.5` with double literals)
    xy = torch.stack([(((px.double() + 1.0) * W - 1.0) * 0.5).to(px.dtype),
                      (((py.double() + 1.0) * H - 1.0) * 0.5).to(py.dtype)], dim=1)
    with torch.no_grad():
        def trunc_i(v):
            return v.clamp(-2.0 ** 30, 2.0 ** 30).to(torch.int64)  # C (int) cast truncates toward 0
        xyd = xy.detach()
        rmin_x = trunc_i((xyd[:, 0] - radius) / BLOCK_X).clamp(0, gx)
        rmin_y = trunc_i((xyd[:, 1] - radius) / BLOCK_Y).clamp(0, gy)
        rmax_x = trunc_i((xyd[:, 0] + radius + BLOCK_X - 1) / BLOCK_X).clamp(0, gx)
        rmax_y = trunc_i((xyd[:, 1] + radius + BLOCK_Y - 1) / BLOCK_Y).clamp(0, gy)
        area = (rmax_x - rmin_x) * (rmax_y - rmin_y)
        visible = (tz > 0.2) & det_ok & (area > 0)

    # 8. colour
    if colors_precomp is None:
        campos = st.campos.reshape(-1).to(means3D.dtype)
        d = means3D - campos[None, :]
        d = d / sqrt_ieee((d[:, 0:1] * d[:, 0:1] + d[:, 1:2] * d[:, 1:2]) + d[:, 2:3] * d[:, 2:3])
        res = eval_sh(st.sh_degree, shs, d) + 0.5
        clamped = (res < 0).detach()
        rgb = torch.clamp_min(res, 0.0)
    else:
        rgb = colors_precomp
        clamped = torch.zeros_like(rgb, dtype=torch.bool)

    radii = torch.where(visible, radius, torch.zeros_like(radius)).to(torch.int32)
    tiles = torch.where(visible, area, torch.zeros_like(area))
    return dict(xy=xy, depth=tz, conic=conic, cov2d=torch.stack([c00, c01, c11], dim=1), opacity=opacities[:, 0] * h, rgb=rgb, clamped=clamped,
                radii=radii, tiles_touched=tiles, visible=visible,
                rect=torch.stack([rmin_x, rmin_y, rmax_x, rmax_y], dim=1), grid=(gx, gy))


def binning(pre):
    """Duplicate-with-keys + stable sort on (tile << 32 | depth bits) + tile ranges (App. A step 10).
    Returns (point_list[int64], tile_of_entry[int64], ranges[num_tiles, 2])."""
    gx, gy = pre["grid"]
    vis = np.nonzero(pre["visible"].numpy())[0]
    rect = pre["rect"].numpy()[vis]
    depth_bits = pre["depth"].detach().to(torch.float32).numpy().view(np.uint32)
    x0, y0, x1, y1 = rect[:, 0], rect[:, 1], rect[:, 2], rect[:, 3]
    nx = x1 - x0
    cnt = nx * (y1 - y0)
    total = int(cnt.sum())
    # duplicateWithKeys in row-major rect order (vectorised)
    gids = np.repeat(vis.astype(np.int64), cnt)
    start = np.repeat(np.cumsum(cnt) - cnt, cnt)
    local = np.arange(total, dtype=np.int64) - start
    nxr = np.repeat(nx, cnt)
    tiles = (np.repeat(y0, cnt) + local // np.maximum(nxr, 1)) * gx + np.repeat(x0, cnt) + local % np.maximum(nxr, 1)
    dkeys = depth_bits[gids].astype(np.uint64)
    # stable radix sort of the 64-bit key with input in Gaussian-index order == lexsort by (tile, depth, index)
    order = np.lexsort((gids, dkeys, tiles)) if len(tiles) else np.zeros(0, dtype=np.int64)
    point_list = gids[order]
    tile_sorted = tiles[order]
    ntiles = gx * gy
    starts = np.searchsorted(tile_sorted, np.arange(ntiles), side="left")
    ends = np.searchsorted(tile_sorted, np.arange(ntiles), side="right")
    ranges = np.stack([starts, ends], axis=1)
    ranges[starts == ends] = 0  # upstream zero-fills the range buffer: empty tiles are [0, 0)
    return torch.from_numpy(point_list), torch.from_numpy(tile_sorted), torch.from_numpy(ranges)


def _tile_pixels(t, gx, H, W):
    ty, tx = divmod(t, gx)
    ys = torch.arange(ty * BLOCK_Y, min((ty + 1) * BLOCK_Y, H))
    xs = torch.arange(tx * BLOCK_X, min((tx + 1) * BLOCK_X, W))
    py, px = torch.meshgrid(ys, xs, indexing="ij")
    return py.reshape(-1), px.reshape(-1)


def _blend_tile(xy, conic, opac, rgb, invd, L, px, py, bg):
    """Front-to-back blend of one tile's pixels over its sorted list L (upstream renderCUDA semantics).
    Returns (color[npx,3], invdepth[npx], final_T[npx], n_contrib[npx] int32)."""
    dtype = xy.dtype
    npx = py.numel()
    pxf = px.to(dtype)[:, None]
    pyf = py.to(dtype)[:, None]
    dx = xy[L, 0][None, :] - pxf
    dy = xy[L, 1][None, :] - pyf
    a, b, c = conic[L, 0][None, :], conic[L, 1][None, :], conic[L, 2][None, :]
    power = -0.5 * (a * dx * dx + c * dy * dy) - b * dx * dy
    G = torch.exp(power)
    araw = opac[L][None, :] * G
    alpha = araw + (torch.clamp_max(araw, 0.99) - araw).detach()
    with torch.no_grad():
        ac = torch.clamp_max(araw.detach(), 0.99)
        valid = (power.detach() <= 0) & (ac >= 1.0 / 255.0)
        om = torch.where(valid, 1 - ac, torch.ones_like(ac))
        Tincl = torch.cumprod(om, dim=1)
        stop = valid & (Tincl < 0.0001)
        n = L.numel()
        idx = torch.arange(n)[None, :].expand_as(stop)
        first_stop = torch.where(stop, idx, torch.full_like(idx, n)).min(dim=1).values
        contrib = valid & (idx < first_stop[:, None])
        last = torch.where(contrib, idx + 1, torch.zeros_like(idx)).max(dim=1).values
    m = contrib.to(dtype)
    one_m = 1 - m * alpha
    Tin = torch.cumprod(one_m, dim=1)
    Tex = torch.cat([torch.ones(npx, 1, dtype=dtype), Tin[:, :-1]], dim=1)
    wgt = m * alpha * Tex
    Tfin = Tin[:, -1]
    return wgt @ rgb[L] + Tfin[:, None] * bg[None, :], wgt @ invd[L], Tfin, last.to(torch.int32)


def blend(pre, point_list, ranges, H, W, bg, tile_subset=None):
    """Per-tile front-to-back alpha blending (App. A step 11), dense per tile.
    Returns color[3,H,W], invdepth[1,H,W], final_T[H,W], n_contrib[H,W] (int32)."""
    gx, gy = pre["grid"]
    xy, conic, opac, rgb = pre["xy"], pre["conic"], pre["opacity"], pre["rgb"]
    invd = 1.0 / pre["depth"]
    dtype = xy.dtype
    bg = bg.to(dtype).reshape(3)
    pix_chunks, col_chunks, dep_chunks, T_chunks, nc_chunks = [], [], [], [], []
    for t in range(gx * gy):
        py, px = _tile_pixels(t, gx, H, W)
        pix_chunks.append(py * W + px)
        s, e = int(ranges[t, 0]), int(ranges[t, 1])
        npx = py.numel()
        if e <= s or (tile_subset is not None and t not in tile_subset):
            col_chunks.append(bg[None, :].expand(npx, 3) * torch.ones(npx, 1, dtype=dtype))
            dep_chunks.append(torch.zeros(npx, dtype=dtype))
            T_chunks.append(torch.ones(npx, dtype=dtype))
            nc_chunks.append(torch.zeros(npx, dtype=torch.int32))
            continue
        col, dep, Tfin, last = _blend_tile(xy, conic, opac, rgb, invd, point_list[s:e], px, py, bg)
        col_chunks.append(col)
        dep_chunks.append(dep)
        T_chunks.append(Tfin)
        nc_chunks.append(last)
    pix = torch.cat(pix_chunks)
    inv = torch.empty_like(pix)
    inv[pix] = torch.arange(pix.numel())
    color = torch.cat(col_chunks, dim=0).index_select(0, inv).t().reshape(3, H, W)
    invdepth = torch.cat(dep_chunks).index_select(0, inv).reshape(1, H, W)
    final_T = torch.cat(T_chunks).index_select(0, inv).reshape(H, W)
    n_contrib = torch.cat(nc_chunks).index_select(0, inv).reshape(H, W)
    return color, invdepth, final_T, n_contrib


def blend_tiles(pre, point_list, ranges, H, W, bg, tiles):
    """The colours of the listed tiles only (nothing is done for the others): [sum of their pixels, 3], the
    per-tile arithmetic of blend() -- the bounded sample of the CPU baseline (oracle/cpu_baseline.py)."""
    gx, _ = pre["grid"]
    xy, conic, opac, rgb = pre["xy"], pre["conic"], pre["opacity"], pre["rgb"]
    invd = 1.0 / pre["depth"]
    bg = bg.to(xy.dtype).reshape(3)
    out = []
    for t in tiles:
        s, e = int(ranges[t, 0]), int(ranges[t, 1])
        if e <= s:
            continue
        py, px = _tile_pixels(t, gx, H, W)
        out.append(_blend_tile(xy, conic, opac, rgb, invd, point_list[s:e], px, py, bg)[0])
    return torch.cat(out, dim=0) if out else torch.zeros(0, 3, dtype=xy.dtype) + 0.0 * xy.sum()


def rasterize(means3D, means2D, opacities, st, shs=None, colors_precomp=None, scales=None,
              rotations=None, cov3D_precomp=None, return_internals=False):
    """GaussianRasterizer(...)(...) semantics: -> (color[3,H,W], radii[P] int32, invdepth[1,H,W])."""
    H, W = int(st.image_height), int(st.image_width)
    pre = preprocess(means3D, means2D, opacities, shs, colors_precomp, scales, rotations, cov3D_precomp, st)
    point_list, tile_sorted, ranges = binning(pre)
    color, invdepth, final_T, n_contrib = blend(pre, point_list, ranges, H, W, st.bg)
    if return_internals:
        return color, pre["radii"], invdepth, dict(pre=pre, point_list=point_list, tile_sorted=tile_sorted,
                                                    ranges=ranges, final_T=final_T, n_contrib=n_contrib)
    return color, pre["radii"], invdepth


class Settings:
    """Duck-typed stand-in for GaussianRasterizationSettings (gaussian_renderer/__init__.py:36-50)."""

    def __init__(self, image_height, image_width, tanfovx, tanfovy, bg, scale_modifier, viewmatrix,
                 projmatrix, sh_degree, campos, prefiltered=False, debug=False, antialiasing=False):
        self.image_height, self.image_width = image_height, image_width
        self.tanfovx, self.tanfovy = tanfovx, tanfovy
        self.bg, self.scale_modifier = bg, scale_modifier
        self.viewmatrix, self.projmatrix = viewmatrix, projmatrix
        self.sh_degree, self.campos = sh_degree, campos
        self.prefiltered, self.debug, self.antialiasing = prefiltered, debug, antialiasing


def settings_from_camera(cam, bg, sh_degree, scale_modifier=1.0, antialiasing=False):
    """The settings `render()` builds from a camera (gaussian_renderer/__init__.py:33-50)."""
    return Settings(int(cam.image_height), int(cam.image_width), math.tan(cam.FoVx * 0.5),
                    math.tan(cam.FoVy * 0.5), bg, scale_modifier, cam.world_view_transform,
                    cam.full_proj_transform, sh_degree, cam.camera_center, antialiasing=antialiasing)


def render_model(model, cam, bg, raw=True, antialiasing=False):
    """Activations as `render()` applies them (gaussian_renderer/__init__.py:54-73, gaussian_model.py:192-220)
    followed by `rasterize` and the [0,1] clamp (:119).  Returns (clamped image, radii, invdepth, raw image)."""
    st = settings_from_camera(cam, bg, model.active_sh_degree, antialiasing=antialiasing)
    means2D = torch.zeros_like(model.get_xyz)
    color, radii, invd = rasterize(model.get_xyz, means2D, model.get_opacity, st, shs=model.get_features,
                                   scales=model.get_scaling, rotations=model.get_rotation)
    return color.clamp(0, 1), radii, invd, color
