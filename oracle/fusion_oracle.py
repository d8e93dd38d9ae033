"""numpy restatement of the reference fusion hot path — TEST INFRASTRUCTURE ONLY.

Every function cites the reference lines it follows. dtype flow is reproduced
deliberately (numba/numpy promotion rules of the reference):
float32 where the reference stores float32, float64 where numba/numpy promote.

Parity unpinned against reference *outputs* for integrate/warp (the reference
Python cannot be imported in this container); pinned by closed-form KATs in
tests/test_oracle_kat.py. Skinning k-NN is pinned against the compiled
reference csrc (oracle/build_ref.py).
"""
import math

import numpy as np

F32 = np.float32
F64 = np.float64
TRUNC_MARGIN = 0.04          # tsdf.py:127 (fixed, independent of voxel size)
COLOR_CONST = 256 * 256      # tsdf.py:90


# ----------------------------------------------------------------------------
# a1: volume geometry  (tsdf.py:55-59, 75-129)
# ----------------------------------------------------------------------------
def volume_geometry(bbox, max_depth, cam_intr, voxel_dim=None, voxel_size=None):
    """Returns (vol_bnds (3,2) f64, vol_dim (3,) int, voxel_size float, origin (3,) f32, trunc).

    bbox = (w_min, h_min, w_max, h_max); cam_intr = (fx, fy, cx, cy).
    voxel_dim wins over voxel_size, as `hasattr(fopt,"voxel_dim")` is tested first (tsdf.py:95).
    """
    K = np.eye(3)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = cam_intr[0], cam_intr[1], cam_intr[2], cam_intr[3]
    w_min, h_min, w_max, h_max = bbox
    md = np.array([0, max_depth, max_depth, max_depth, max_depth])
    view_frust_pts = np.array([
        (np.array([0, w_min, w_min, w_max, w_max]) - K[0, 2]) * md / K[0, 0],
        (np.array([0, h_min, h_max, h_min, h_max]) - K[1, 2]) * md / K[1, 1],
        md,
    ])
    vol_bnds = np.asarray([np.min(view_frust_pts, axis=1), np.max(view_frust_pts, axis=1)]).T
    if voxel_dim is not None:
        if isinstance(voxel_dim, int):
            vol_dim = np.array([voxel_dim] * 3)
        else:
            vol_dim = np.asarray(voxel_dim)
        vs = ((vol_bnds[:, 1] - vol_bnds[:, 0]) / vol_dim).max()
    elif voxel_size is not None:
        vs = float(voxel_size)
        vol_dim = np.ceil((vol_bnds[:, 1] - vol_bnds[:, 0]) / vs).copy(order='C').astype(int)
    else:
        raise ValueError("need voxel_dim or voxel_size")
    vol_bnds[:, 1] = vol_bnds[:, 0] + vol_dim * vs
    origin = vol_bnds[:, 0].copy(order='C').astype(F32)
    return vol_bnds, vol_dim.astype(np.int64), float(vs), origin, TRUNC_MARGIN


def world_points(origin, vol_dim, voxel_size):
    """vox2world over the C-order meshgrid (tsdf.py:294-307, 338-349).

    numba: f32 origin + (f64 voxel_size * f32 coord) computed in f64, stored f32.
    """
    Dx, Dy, Dz = (int(d) for d in vol_dim)
    o = np.asarray(origin, F32).astype(F64)
    vs = F64(voxel_size)
    ax = [(o[j] + vs * np.arange(n, dtype=F32).astype(F64)).astype(F32) for j, n in enumerate((Dx, Dy, Dz))]
    pts = np.empty((Dx, Dy, Dz, 3), F32)
    pts[..., 0] = ax[0][:, None, None]
    pts[..., 1] = ax[1][None, :, None]
    pts[..., 2] = ax[2][None, None, :]
    return pts.reshape(-1, 3)


# ----------------------------------------------------------------------------
# a2: frame unpack (tsdf.py:545-566)
# ----------------------------------------------------------------------------
def pack_color(im):
    """im (6,H,W) f32 -> packed color (H,W) f32 = floor(b*65536 + g*256 + r) of 255*rgb."""
    c = 255 * np.moveaxis(np.asarray(im)[:3], 0, -1).astype(F32)
    return np.floor(c[..., 2] * COLOR_CONST + c[..., 1] * 256 + c[..., 0])


def depth_of(im):
    return np.asarray(im)[-1]


# ----------------------------------------------------------------------------
# a3: skinning (warpfield.py:83-129)
# ----------------------------------------------------------------------------
def exp_f32(x):
    """Canonical f32 exp of the oracle: f64 exp rounded to f32.

    The reference uses numpy's float32 SIMD exp (warpfield.py:114) whose last bit
    is platform dependent; the oracle and the HIP kernel both use this
    correctly-rounded form (documented deviation).
    """
    return np.exp(np.asarray(x, F32).astype(F64)).astype(F32)


def knn_sqdist(points, nodes, k, chunk=1 << 14):
    """Exact k nearest nodes by f32 squared distance ((dx²+dy²)+dz², pykdtree calc_dist order),
    ties broken by lower node index. Returns (sqdist (P,k) f32, idx (P,k) int64)."""
    points = np.asarray(points, F32)
    nodes = np.asarray(nodes, F32)
    P = points.shape[0]
    out_d = np.empty((P, k), F32)
    out_i = np.empty((P, k), np.int64)
    for s in range(0, P, chunk):
        p = points[s:s + chunk]
        dx = p[:, None, 0] - nodes[None, :, 0]
        dy = p[:, None, 1] - nodes[None, :, 1]
        dz = p[:, None, 2] - nodes[None, :, 2]
        d2 = (dx * dx + dy * dy) + dz * dz                      # f32, no FMA
        if k < nodes.shape[0]:
            part = np.argpartition(d2, k - 1, axis=1)[:, :k]
            cand_d = np.take_along_axis(d2, part, axis=1)
            o = np.lexsort((part, cand_d), axis=-1)              # order by (d2, idx)
            sel = np.take_along_axis(part, o, axis=1)
            kth = np.take_along_axis(d2, sel[:, -1:], axis=1)
            tie = (d2 <= kth).sum(axis=1) > k                    # tie straddles the k-th slot
            for r in np.nonzero(tie)[0]:
                sel[r] = np.argsort(d2[r], kind='stable')[:k]
        else:
            sel = np.argsort(d2, axis=1, kind='stable')
        out_i[s:s + chunk] = sel
        out_d[s:s + chunk] = np.take_along_axis(d2, sel, axis=1)
    return out_d, out_i


def skin(points, nodes, node_coverage, k=None):
    """WarpField.skin (warpfield.py:83-129). Returns (anchors i32 (P,K), weights f32 (P,K), valid bool (P,)).

    K = min(N, 4) (warpfield.py:60). dist = sqrt(sqdist) in f32 (pykdtree), cut-off
    `dist > 4*node_coverage` strict (:109), w = exp(-dist**2/(2σ²)) in f32 (:114),
    valid = all K anchors >= 0 (:120), w /= (Σw + 1e-6) (:121).
    """
    nodes = np.asarray(nodes, F32)
    K = min(nodes.shape[0], 4) if k is None else k
    sq, idx = knn_sqdist(points, nodes, K)
    dist = np.sqrt(sq)                                           # f32
    dist[dist > F32(4 * node_coverage)] = np.inf
    anchors = idx.astype(np.int32)
    anchors[dist == np.inf] = -1
    denom = F32(2.0 * (node_coverage ** 2))
    weights = exp_f32(-(dist ** 2) / denom)
    valid = np.sum(anchors >= 0, axis=-1) == K
    wsum = weights[:, 0].copy()
    for j in range(1, K):
        wsum = wsum + weights[:, j]                              # ((w0+w1)+w2)+w3, f32
    weights = weights / (wsum[:, None] + F32(1e-6))
    return anchors, weights.astype(F32), valid


# ----------------------------------------------------------------------------
# a4: ED warp (geometry.py:9-25 via registration_fusion.py:157-184)
# ----------------------------------------------------------------------------
def ed_warp(points, anchors, weights, valid, node_R, node_T, nodes):
    """y = Σ_k w_k (R_k (x - g_k) + g_k + t_k) in f32, per-op rounding, summed k=0..3 in order.

    Invalid points keep x (deform_ED returns a copy of `points` with only valid rows replaced).
    R is applied as a 3x3 matrix, row i = ((R_i0 d0 + R_i1 d1) + R_i2 d2).
    """
    x = np.asarray(points, F32)
    out = x.copy()
    v = np.asarray(valid, bool)
    if not v.any():
        return out
    xv = x[v]
    a = np.asarray(anchors)[v]
    w = np.asarray(weights, F32)[v]
    R = np.asarray(node_R, F32)
    T = np.asarray(node_T, F32)
    g = np.asarray(nodes, F32)
    acc = None
    for k in range(a.shape[1]):
        ak = a[:, k]
        gk, Rk, tk = g[ak], R[ak], T[ak]
        d = xv - gk
        r = np.stack([(Rk[:, i, 0] * d[:, 0] + Rk[:, i, 1] * d[:, 1]) + Rk[:, i, 2] * d[:, 2] for i in range(3)], 1)
        y = ((r + gk) + tk) * w[:, k:k + 1]
        acc = y if acc is None else acc + y
    out[v] = acc
    return out


def deform_lbs(node_rotations, node_translations, world_pts, world_anchors, world_weights, valid_pts):
    """warpfield.py:208-231 (numba): origin-form y = Σ_{k: w_k != 0} w_k (R_k x + t_k), accumulated from
    zero in anchor order, f32; np.dot(R, x) taken as ((R0 x + R1 y) + R2 z) — numba's BLAS gemv order
    is implementation-defined (last-bit parity with the reference unpinned). Invalid points keep x."""
    x = np.asarray(world_pts, F32)
    out = x.copy()
    v = np.asarray(valid_pts, bool)
    R = np.asarray(node_rotations, F32).reshape(-1, 3, 3)
    T = np.asarray(node_translations, F32).reshape(-1, 3)
    a = np.asarray(world_anchors)
    w = np.asarray(world_weights, F32)
    acc = np.zeros((int(v.sum()), 3), F32)
    xv, av, wv = x[v], a[v], w[v]
    for k in range(a.shape[1]):
        use = wv[:, k] != 0
        ak = np.where(use, av[:, k], 0)
        Rk, tk = R[ak], T[ak]
        y = np.stack([((Rk[:, i, 0] * xv[:, 0] + Rk[:, i, 1] * xv[:, 1]) + Rk[:, i, 2] * xv[:, 2]) + tk[:, i]
                      for i in range(3)], 1)
        acc = np.where(use[:, None], acc + wv[:, k:k + 1] * y, acc)
    out[v] = acc
    return out


# ----------------------------------------------------------------------------
# a7: CPU integrate (tsdf.py:378-494 with 329-376, 576-612)
# ----------------------------------------------------------------------------
def cam2pix(cam_pts_f64, intr):
    """tsdf.py:351-364: (x*fx)/z + cx in f64 with f32 intrinsics, np.round (half-even), int().
    Returns float64 rounded pixel coordinates (int() of them is taken by the caller's range test)."""
    fx, fy, cx, cy = (F64(F32(v)) for v in intr)
    with np.errstate(divide='ignore', invalid='ignore'):
        px = np.rint((cam_pts_f64[:, 0] * fx) / cam_pts_f64[:, 2] + cx)
        py = np.rint((cam_pts_f64[:, 1] * fy) / cam_pts_f64[:, 2] + cy)
    return px, py


def check_visibility(cam_pts_f64, depth_im, intr, trunc=TRUNC_MARGIN):
    """tsdf.py:576-612. Returns (valid_pts, depth_diff f64, px int64, py int64)."""
    H, W = depth_im.shape
    px, py = cam2pix(cam_pts_f64, intr)
    z = cam_pts_f64[:, 2]
    valid_pix = (px >= 0) & (px < W) & (py >= 0) & (py < H) & (z > 0)
    pxi = np.where(valid_pix, px, 0).astype(np.int64)
    pyi = np.where(valid_pix, py, 0).astype(np.int64)
    depth_val = np.zeros(px.shape, F64)
    depth_val[valid_pix] = depth_im[pyi[valid_pix], pxi[valid_pix]]
    depth_diff = depth_val - z
    valid_pts = (depth_val > 0) & (depth_diff >= -trunc)
    return valid_pts, depth_diff, pxi, pyi


def check_visibility_f32(points_f32, depth_im, intr, trunc=TRUNC_MARGIN):
    """tsdf.py:599-612 on an f32 point array (get_visible_nodes, tsdf.py:614-638): numba types cam2pix
    (tsdf.py:351-364) in f32 — (x·fx)/z + cx with f32 intrinsics, np.round half-even in f32, int() — while
    get_depth_from_image's depth array is f64 (np.zeros), so depth_diff = f64(depth) - f32 z. -> (valid, depth_diff)."""
    p = np.asarray(points_f32, F32)
    fx, fy, cx, cy = (F32(v) for v in intr)
    H, W = depth_im.shape
    with np.errstate(divide='ignore', invalid='ignore', over='ignore'):
        su = ((p[:, 0] * fx) / p[:, 2] + cx).astype(F32)
        sv = ((p[:, 1] * fy) / p[:, 2] + cy).astype(F32)
        u, v = np.rint(su), np.rint(sv)
    z = p[:, 2]
    valid_pix = (u >= 0) & (u < W) & (v >= 0) & (v < H) & (z > 0)
    ui = np.where(valid_pix, u, 0).astype(np.int64)
    vi = np.where(valid_pix, v, 0).astype(np.int64)
    depth_val = np.zeros(p.shape[0], F64)
    depth_val[valid_pix] = depth_im[vi[valid_pix], ui[valid_pix]]
    depth_diff = depth_val - z
    return (depth_val > 0) & (depth_diff >= -trunc), depth_diff


def integrate(tsdf, weight, color, pts, valid_points, depth_im, color_im, intr,
              obs_weight=1.0, trunc=TRUNC_MARGIN, with_color=True):
    """In-place CPU integrate over flat f32 volumes (V,). Returns number of updated voxels.

    pts (V,3) f32 (world or warped), valid_points (V,) bool.
    """
    cam = np.asarray(pts, F32).astype(F64)                    # rigid_transform(inv(I)) -> exact f64
    valid_pts, depth_diff, pxi, pyi = check_visibility(cam, np.asarray(depth_im, F32), intr, trunc)
    valid_pts &= np.asarray(valid_points, bool)
    dist = np.minimum(1, depth_diff / trunc)
    idx = np.nonzero(valid_pts)[0]
    w_old = weight[idx]
    tsdf_vals = tsdf[idx]
    vd = dist[idx]
    ow = F64(obs_weight)
    w_new = (w_old.astype(F64) + ow).astype(F32)
    prod = (w_old * tsdf_vals).astype(F32)                    # numba f32*f32 -> f32
    tsdf_new = ((prod.astype(F64) + ow * vd) / w_new.astype(F64)).astype(F32)
    weight[idx] = w_new
    tsdf[idx] = tsdf_new
    if with_color:
        old_color = color[idx]
        old_b = np.floor(old_color / F32(COLOR_CONST))
        old_g = np.floor((old_color - old_b * F32(COLOR_CONST)) / F32(256))
        old_r = old_color - old_b * F32(COLOR_CONST) - old_g * F32(256)
        new_color = np.asarray(color_im, F32)[pyi[idx], pxi[idx]]
        new_b = np.floor(new_color / F32(COLOR_CONST))
        new_g = np.floor((new_color - new_b * F32(COLOR_CONST)) / F32(256))
        new_r = new_color - new_b * F32(COLOR_CONST) - new_g * F32(256)
        owf = F32(obs_weight)
        nb = np.minimum(F32(255.), np.rint((w_old * old_b + owf * new_b) / w_new))
        ng = np.minimum(F32(255.), np.rint((w_old * old_g + owf * new_g) / w_new))
        nr = np.minimum(F32(255.), np.rint((w_old * old_r + owf * new_r) / w_new))
        color[idx] = nb * F32(COLOR_CONST) + ng * F32(256) + nr
    return int(idx.size)


# ----------------------------------------------------------------------------
# a8: pycuda integrate kernel (tsdf.py:192-288) — the reference's GPU-mode arithmetic
# ----------------------------------------------------------------------------
def _roundf(v):
    """CUDA roundf (half away from zero) of f32 values, formed exactly in f64."""
    a = np.floor(np.abs(v.astype(F64)) + 0.5)
    return np.copysign(a, v).astype(F32)


def _cvt_sat_i32(v):
    """(int) of f32 with the saturating GPU conversion: NaN -> 0, clamp to the int32 range."""
    v64 = v.astype(F64)
    out = np.where(np.isnan(v64), 0.0, np.clip(np.trunc(np.nan_to_num(v64, nan=0.0)), -2147483648.0, 2147483647.0))
    return out.astype(np.int64)


def integrate_pycuda(tsdf, weight, color, pts, valid_points, depth_im, color_im, intr, obs_weight=1.0,
                     trunc=TRUNC_MARGIN, with_color=True):
    """In-place restatement of the pycuda `integrate` kernel (tsdf.py:192-288) over flat f32 volumes.

    f32 arithmetic, identity cam_pose applied literally (tsdf.py:236-241); pixel =
    (int)roundf(f32(f64(f·(x/z)+c) + 0.5)) (:243-244: the 0.5 literal is a double); skip if outside the
    image or z < 0 (:248) or depth == 0 (:252); depth difference times sqrt(1+mx²+my²) of the integer
    pixel (:261-264); dist = fminf(1, dd/trunc); roundf colours (:282-284). nvcc's default FMA
    contraction is not modelled (each product is rounded): parity unpinned at the last-bit level.
    Returns the number of updated voxels."""
    one, zero = F32(1), F32(0)
    P = np.asarray(pts, F32)
    sel = np.nonzero(np.asarray(valid_points, bool))[0]
    x, y, z = P[sel, 0] - zero, P[sel, 1] - zero, P[sel, 2] - zero
    with np.errstate(all="ignore"):
        cxp = (one * x + zero * y) + zero * z
        cyp = (zero * x + one * y) + zero * z
        czp = (zero * x + zero * y) + one * z
        fx, fy, cx, cy = (F32(v) for v in intr)
        sx = fx * (cxp / czp) + cx
        sy = fy * (cyp / czp) + cy
        u = _cvt_sat_i32(_roundf((sx.astype(F64) + 0.5).astype(F32)))
        v = _cvt_sat_i32(_roundf((sy.astype(F64) + 0.5).astype(F32)))
        H, W = depth_im.shape
        ok = (u >= 0) & (u < W) & (v >= 0) & (v < H) & ~(czp < 0)
        sel, u, v, czp = sel[ok], u[ok], v[ok], czp[ok]
        d = np.asarray(depth_im, F32)[v, u]
        ok = d != 0
        sel, u, v, czp, d = sel[ok], u[ok], v[ok], czp[ok], d[ok]
        dd = d - czp
        mx = (u.astype(F32) - cx) / fx
        my = (v.astype(F32) - cy) / fy
        dd = dd * np.sqrt((one + mx * mx) + my * my)
        tr = F32(trunc)
        ok = ~(dd < -tr)
        sel, u, v, dd = sel[ok], u[ok], v[ok], dd[ok]
        dist = np.fmin(one, dd / tr)
        ow = F32(obs_weight)
        w_old = weight[sel]
        w_new = w_old + ow
        weight[sel] = w_new
        tsdf[sel] = (tsdf[sel] * w_old + ow * dist) / w_new
        if with_color:
            C, c256 = F32(65536), F32(256)
            oc = color[sel]
            ob = np.floor(oc / C)
            og = np.floor((oc - ob * c256 * c256) / c256)
            orr = (oc - ob * c256 * c256) - og * c256
            nc = np.asarray(color_im, F32)[v, u]
            nb = np.floor(nc / C)
            ng = np.floor((nc - nb * c256 * c256) / c256)
            nr = (nc - nb * c256 * c256) - ng * c256
            b2 = np.fmin(_roundf((ob * w_old + ow * nb) / w_new), F32(255))
            g2 = np.fmin(_roundf((og * w_old + ow * ng) / w_new), F32(255))
            r2 = np.fmin(_roundf((orr * w_old + ow * nr) / w_new), F32(255))
            color[sel] = (b2 * c256 * c256 + g2 * c256) + r2
    return int(sel.size)


# ----------------------------------------------------------------------------
# a9: transform conventions (warpfield.py:389-449)
# ----------------------------------------------------------------------------
def to_origin_form(R, T, nodes):
    """t_origin = -R g + g + T (warpfield.py:407-408)."""
    return -np.einsum('nij,nj->ni', R, nodes) + nodes + T


# ----------------------------------------------------------------------------
# a10: Gauss-Newton (model/model.py:222-859), dense float64 restatement
# ----------------------------------------------------------------------------
def angle_axis_to_rotation_matrix(aa):
    """kornia 0.7.0 angle_axis_to_rotation_matrix (called at model.py:744).

    θ² > 1e-6: Rodrigues with axis = ω/(θ+1e-6); else first-order I + [ω]×.
    """
    aa = np.asarray(aa, F64)
    theta2 = np.sum(aa * aa, axis=1)
    theta = np.sqrt(theta2)
    w = aa / (theta + 1e-6)[:, None]
    wx, wy, wz = w[:, 0], w[:, 1], w[:, 2]
    c, s = np.cos(theta), np.sin(theta)
    oc = 1.0 - c
    Rn = np.stack([
        c + wx * wx * oc, wx * wy * oc - wz * s, wy * s + wx * wz * oc,
        wz * s + wx * wy * oc, c + wy * wy * oc, -wx * s + wy * wz * oc,
        -wy * s + wx * wz * oc, wx * s + wy * wz * oc, c + wz * wz * oc], 1).reshape(-1, 3, 3)
    rx, ry, rz = aa[:, 0], aa[:, 1], aa[:, 2]
    one = np.ones_like(rx)
    Rt = np.stack([one, -rz, ry, rz, one, -rx, -ry, rx, one], 1).reshape(-1, 3, 3)
    mask = (theta2 > 1e-6)[:, None, None]
    return np.where(mask, Rn, Rt)


def skew(v):
    """vec_to_skew_mat @ v (model.py:133-144): [[0,-z,y],[z,0,-x],[-y,x,0]]."""
    z = np.zeros(v.shape[0])
    return np.stack([z, -v[:, 2], v[:, 1], v[:, 2], z, -v[:, 0], -v[:, 1], v[:, 0], z], 1).reshape(-1, 3, 3)


GN_DEFAULTS = dict(num_iter=10, lambda_flow=0.0, lambda_depth=1.0, lambda_arap=0.5,
                   lambda_motion=1.0, lm_factor=1e-7, stop_loss_diff=1.0, use_edge_weighting=False)


def gn_edges(graph_edges):
    """Valid directed edges in (node, slot) order (model.py:356-364)."""
    ge = np.asarray(graph_edges)
    ii, kk = np.nonzero(ge >= 0)
    return np.stack([ii, ge[ii, kk]], 1).astype(np.int64), (ii, kk)


def gn_optimize(graph_nodes, graph_edges, graph_edges_weights, target_node_position, node_confidence,
                source_points, anchors, weights, target_points, intrinsics,
                target_px=None, target_py=None, prev_rot=None, prev_trans=None, **params):
    """One DeformNet.optimize solve (model.py:222-859) for a single batch item, dense float64.

    Reproduces: LM schedule (:418-419), data rows with the flow-rotation operator-precedence
    quirk (:505-510), ARAP rows (:554-601), motion rows (:604-612), A = JᵀJ + λI, b = -Jᵀr
    (:641-662), LU solve (:694-709), loss-based early stop (:726-732), R ← exp(x_rot)·R,
    t += x_trans (:744-748). Returns dict(node_rotations, node_translations, valid_solve,
    convergence_info).
    """
    p = dict(GN_DEFAULTS)
    p.update(params)
    from scipy.linalg import lu_factor, lu_solve
    g = np.asarray(graph_nodes, F64)
    N = g.shape[0]
    src = np.asarray(source_points, F64)
    M = src.shape[0]
    anc = np.asarray(anchors, np.int64)
    wts = np.asarray(weights, F64)
    tgt = np.asarray(target_points, F64)
    tpos = np.asarray(target_node_position, F64)
    conf = np.asarray(node_confidence, F64).reshape(-1)
    fx, fy, cx, cy = (float(v) for v in intrinsics)
    tpx = np.zeros(M) if target_px is None else np.asarray(target_px, F64).reshape(-1)
    tpy = np.zeros(M) if target_py is None else np.asarray(target_py, F64).reshape(-1)
    edges, (ei, ek) = gn_edges(graph_edges)
    E = edges.shape[0]
    n_nb = np.asarray(graph_edges).shape[1]
    ew = np.ones(E)
    if p['use_edge_weighting']:
        ew = float(n_nb) * np.asarray(graph_edges_weights, F64)[ei, ek]

    lf, ld = math.sqrt(p['lambda_flow']), math.sqrt(p['lambda_depth'])
    lm_, la = math.sqrt(p['lambda_motion']), math.sqrt(p['lambda_arap'])
    lm_factor = p['lm_factor']
    R = np.tile(np.eye(3), (N, 1, 1)) if prev_rot is None else np.asarray(prev_rot, F64).reshape(N, 3, 3).copy()
    t = np.zeros((N, 3)) if prev_trans is None else np.asarray(prev_trans, F64).reshape(N, 3).copy()
    conv = dict(total=[], data=[], arap=[], motion=[], errors=[])
    ill_posed = False
    rowsM = np.arange(M) * 3
    res = None
    for gn_i in range(p['num_iter']):
        if gn_i % 3 == 2:
            lm_factor /= 2
        J = np.zeros((M * 3, N * 6))
        defp = np.zeros((M, 3))
        for k in range(4):
            nk = anc[:, k]
            rot = np.einsum('mij,mj->mi', R[nk], src - g[nk])
            defp += wts[:, k:k + 1] * (rot + g[nk] + t[nk])
        zinv = 1.0 / (defp[:, 2] + 1e-7)
        fx_mul_x, fy_mul_y = fx * defp[:, 0], fy * defp[:, 1]
        fx_div_z, fy_div_z = fx * zinv, fy * zinv
        fx_mul_x_div_z, fy_mul_y_div_z = fx_mul_x * zinv, fy_mul_y * zinv
        mfx = -fx_mul_x_div_z * zinv
        mfy = -fy_mul_y_div_z * zinv
        for k in range(4):
            nk = anc[:, k]
            wk = wts[:, k]
            rot = np.einsum('mij,mj->mi', R[nk], src - g[nk])
            S = -skew(wk[:, None] * rot)
            ct = 3 * N + 3 * nk
            J[rowsM, ct + 0] += lf * wk * fx_div_z
            J[rowsM, ct + 2] += lf * wk * mfx
            J[rowsM + 1, ct + 1] += lf * wk * fy_div_z
            J[rowsM + 1, ct + 2] += lf * wk * mfy
            J[rowsM, ct + 0] += ld * wk
            J[rowsM + 1, ct + 1] += ld * wk
            J[rowsM + 2, ct + 2] += ld * wk
            cr = 3 * nk
            for j in range(3):      # flow part with the reference's precedence quirk (model.py:505-510)
                J[rowsM, cr + j] += lf * fx_div_z * S[:, 0, j] + mfx * S[:, 2, j]
                J[rowsM + 1, cr + j] += lf * fy_div_z * S[:, 1, j] + mfy * S[:, 2, j]
            for i in range(3):
                for j in range(3):
                    J[rowsM + i, cr + j] += ld * S[:, i, j]
        rd = np.zeros(M * 3)
        rd[rowsM] = lf * (fx_mul_x_div_z + cx - tpx)
        rd[rowsM + 1] = lf * (fy_mul_y_div_z + cy - tpy)
        rd[rowsM] += ld * (defp[:, 0] - tgt[:, 0])
        rd[rowsM + 1] += ld * (defp[:, 1] - tgt[:, 1])
        rd[rowsM + 2] += ld * (defp[:, 2] - tgt[:, 2])
        blocks_J, blocks_r = [J], [rd]
        ra = None
        if E > 0:
            Ja = np.zeros((E * 3, N * 6))
            i0, i1 = edges[:, 0], edges[:, 1]
            rowsE = np.arange(E) * 3
            delta = np.einsum('eij,ej->ei', R[i0], g[i1] - g[i0])
            ra = (la * ew[:, None] * (delta + g[i0] + t[i0] - (g[i1] + t[i1]))).reshape(-1)
            for c in range(3):
                Ja[rowsE + c, 3 * N + 3 * i0 + c] += la * ew
                Ja[rowsE + c, 3 * N + 3 * i1 + c] += -la * ew
            Sa = -la * ew[:, None, None] * skew(delta)
            for i in range(3):
                for j in range(3):
                    Ja[rowsE + i, 3 * i0 + j] += Sa[:, i, j]
            blocks_J.append(Ja)
            blocks_r.append(ra)
        Jm = np.zeros((N * 3, N * 6))
        ids = np.arange(N)
        for c in range(3):
            Jm[ids * 3 + c, 3 * N + 3 * ids + c] += lm_ * conf
        rm = (lm_ * conf[:, None] * (t + g - tpos)).reshape(-1)
        blocks_J.append(Jm)
        blocks_r.append(rm)
        Jall = np.concatenate(blocks_J, 0)
        res = np.concatenate(blocks_r, 0)
        A = Jall.T @ Jall + np.eye(6 * N) * lm_factor
        b = -(Jall.T @ res)
        try:
            x = lu_solve(lu_factor(A), b)
        except Exception:
            ill_posed = True
            conv['errors'].append("Solver failed: Ill-posed system!")
            break
        if not np.all(np.isfinite(x)):
            ill_posed = True
            conv['errors'].append("Solver failed: Non-finite solution x!")
            break
        loss_total = float(np.linalg.norm(res))
        if len(conv['total']):
            if loss_total - conv['total'][-1] > p['stop_loss_diff']:
                break
            if loss_total == conv['total'][-1]:
                break
        conv['data'].append(float(np.linalg.norm(rd)))
        conv['total'].append(loss_total)
        R_inc = angle_axis_to_rotation_matrix(x[:3 * N].reshape(N, 3))
        R = R_inc @ R
        t = t + x[3 * N:].reshape(N, 3)
        if ra is not None:
            conv['arap'].append(float(np.linalg.norm(ra)))
        conv['motion'].append(float(np.linalg.norm(rm)))
    valid = (not ill_posed) and res is not None and bool(np.all(np.isfinite(res)))
    if not valid:
        R = np.tile(np.eye(3), (N, 1, 1))
        t = np.zeros((N, 3))
    conv['valid'] = int(valid)
    return dict(node_rotations=R, node_translations=t, valid_solve=int(valid), convergence_info=conv)


def gn_optimize_sparse(graph_nodes, graph_edges, graph_edges_weights, target_node_position, node_confidence,
                       source_points, anchors, weights, target_points, intrinsics,
                       target_px=None, target_py=None, prev_rot=None, prev_trans=None, **params):
    """gn_optimize (model.py:222-859) with the same Jacobian entries held as a sparse f64 matrix: JᵀJ and Jᵀr by
    sparse products, then the reference's dense LU of the 6N x 6N system (model.py:59-86,694-709). Identical rows,
    columns, LM schedule, early stop and update; only the f64 summation order of JᵀJ differs from the dense J
    (tests/test_oracle.py checks the two against each other). For graphs whose dense J does not fit (2k-4k
    nodes: J is (3M+3E+3N) x 6N, 8.5 GB at 2k nodes)."""
    import scipy.sparse as sp
    from scipy.linalg import lu_factor, lu_solve
    p = dict(GN_DEFAULTS)
    p.update(params)
    g = np.asarray(graph_nodes, F64)
    N = g.shape[0]
    src = np.asarray(source_points, F64)
    M = src.shape[0]
    anc = np.asarray(anchors, np.int64)
    wts = np.asarray(weights, F64)
    tgt = np.asarray(target_points, F64)
    tpos = np.asarray(target_node_position, F64)
    conf = np.asarray(node_confidence, F64).reshape(-1)
    fx, fy, cx, cy = (float(v) for v in intrinsics)
    tpx = np.zeros(M) if target_px is None else np.asarray(target_px, F64).reshape(-1)
    tpy = np.zeros(M) if target_py is None else np.asarray(target_py, F64).reshape(-1)
    edges, (ei, ek) = gn_edges(graph_edges)
    E = edges.shape[0]
    n_nb = np.asarray(graph_edges).shape[1]
    ew = np.ones(E)
    if p['use_edge_weighting']:
        ew = float(n_nb) * np.asarray(graph_edges_weights, F64)[ei, ek]
    lf, ld = math.sqrt(p['lambda_flow']), math.sqrt(p['lambda_depth'])
    lm_, la = math.sqrt(p['lambda_motion']), math.sqrt(p['lambda_arap'])
    lm_factor = p['lm_factor']
    R = np.tile(np.eye(3), (N, 1, 1)) if prev_rot is None else np.asarray(prev_rot, F64).reshape(N, 3, 3).copy()
    t = np.zeros((N, 3)) if prev_trans is None else np.asarray(prev_trans, F64).reshape(N, 3).copy()
    conv = dict(total=[], data=[], arap=[], motion=[], errors=[])
    ill_posed = False
    rowsM = np.arange(M) * 3
    nrow = 3 * M + 3 * E + 3 * N
    res = None
    for gn_i in range(p['num_iter']):
        if gn_i % 3 == 2:
            lm_factor /= 2
        rr, cc, vv = [], [], []

        def put(r, c, v):
            rr.append(np.asarray(r, np.int64).reshape(-1))
            cc.append(np.asarray(c, np.int64).reshape(-1))
            vv.append(np.broadcast_to(np.asarray(v, F64), np.shape(r)).reshape(-1))
        defp = np.zeros((M, 3))
        for k in range(4):
            nk = anc[:, k]
            rot = np.einsum('mij,mj->mi', R[nk], src - g[nk])
            defp += wts[:, k:k + 1] * (rot + g[nk] + t[nk])
        zinv = 1.0 / (defp[:, 2] + 1e-7)
        fx_mul_x, fy_mul_y = fx * defp[:, 0], fy * defp[:, 1]
        fx_div_z, fy_div_z = fx * zinv, fy * zinv
        fx_mul_x_div_z, fy_mul_y_div_z = fx_mul_x * zinv, fy_mul_y * zinv
        mfx = -fx_mul_x_div_z * zinv
        mfy = -fy_mul_y_div_z * zinv
        for k in range(4):
            nk = anc[:, k]
            wk = wts[:, k]
            rot = np.einsum('mij,mj->mi', R[nk], src - g[nk])
            S = -skew(wk[:, None] * rot)
            ct = 3 * N + 3 * nk
            put(rowsM, ct + 0, lf * wk * fx_div_z)
            put(rowsM, ct + 2, lf * wk * mfx)
            put(rowsM + 1, ct + 1, lf * wk * fy_div_z)
            put(rowsM + 1, ct + 2, lf * wk * mfy)
            put(rowsM, ct + 0, ld * wk)
            put(rowsM + 1, ct + 1, ld * wk)
            put(rowsM + 2, ct + 2, ld * wk)
            cr = 3 * nk
            for j in range(3):      # flow part with the reference's precedence quirk (model.py:505-510)
                put(rowsM, cr + j, lf * fx_div_z * S[:, 0, j] + mfx * S[:, 2, j])
                put(rowsM + 1, cr + j, lf * fy_div_z * S[:, 1, j] + mfy * S[:, 2, j])
            for i in range(3):
                for j in range(3):
                    put(rowsM + i, cr + j, ld * S[:, i, j])
        rd = np.zeros(M * 3)
        rd[rowsM] = lf * (fx_mul_x_div_z + cx - tpx)
        rd[rowsM + 1] = lf * (fy_mul_y_div_z + cy - tpy)
        rd[rowsM] += ld * (defp[:, 0] - tgt[:, 0])
        rd[rowsM + 1] += ld * (defp[:, 1] - tgt[:, 1])
        rd[rowsM + 2] += ld * (defp[:, 2] - tgt[:, 2])
        blocks_r = [rd]
        ra = None
        if E > 0:
            i0, i1 = edges[:, 0], edges[:, 1]
            rowsE = 3 * M + np.arange(E) * 3
            delta = np.einsum('eij,ej->ei', R[i0], g[i1] - g[i0])
            ra = (la * ew[:, None] * (delta + g[i0] + t[i0] - (g[i1] + t[i1]))).reshape(-1)
            for c in range(3):
                put(rowsE + c, 3 * N + 3 * i0 + c, la * ew)
                put(rowsE + c, 3 * N + 3 * i1 + c, -la * ew)
            Sa = -la * ew[:, None, None] * skew(delta)
            for i in range(3):
                for j in range(3):
                    put(rowsE + i, 3 * i0 + j, Sa[:, i, j])
            blocks_r.append(ra)
        ids = np.arange(N)
        for c in range(3):
            put(3 * M + 3 * E + ids * 3 + c, 3 * N + 3 * ids + c, lm_ * conf)
        rm = (lm_ * conf[:, None] * (t + g - tpos)).reshape(-1)
        blocks_r.append(rm)
        J = sp.csr_matrix((np.concatenate(vv), (np.concatenate(rr), np.concatenate(cc))), shape=(nrow, 6 * N))
        res = np.concatenate(blocks_r, 0)
        JT = J.T.tocsr()
        A = (JT @ J).toarray()
        A[np.diag_indices(6 * N)] += lm_factor
        b = -(JT @ res)
        try:
            x = lu_solve(lu_factor(A, overwrite_a=True), b)
        except Exception:
            ill_posed = True
            conv['errors'].append("Solver failed: Ill-posed system!")
            break
        del A
        if not np.all(np.isfinite(x)):
            ill_posed = True
            conv['errors'].append("Solver failed: Non-finite solution x!")
            break
        loss_total = float(np.linalg.norm(res))
        if len(conv['total']):
            if loss_total - conv['total'][-1] > p['stop_loss_diff']:
                break
            if loss_total == conv['total'][-1]:
                break
        conv['data'].append(float(np.linalg.norm(rd)))
        conv['total'].append(loss_total)
        R_inc = angle_axis_to_rotation_matrix(x[:3 * N].reshape(N, 3))
        R = R_inc @ R
        t = t + x[3 * N:].reshape(N, 3)
        if ra is not None:
            conv['arap'].append(float(np.linalg.norm(ra)))
        conv['motion'].append(float(np.linalg.norm(rm)))
    valid = (not ill_posed) and res is not None and bool(np.all(np.isfinite(res)))
    if not valid:
        R = np.tile(np.eye(3), (N, 1, 1))
        t = np.zeros((N, 3))
    conv['valid'] = int(valid)
    return dict(node_rotations=R, node_translations=t, valid_solve=int(valid), convergence_info=conv)


def gn_arap(graph_nodes, source_node_position, target_node_position, valid_nodes_mask, original_graph_nodes,
            graph_edges, graph_edges_weights, R_current, t_current, **params):
    """DeformNet.arap (model/model.py:1639-1986), dense float64: data rows per valid node with the
    residual as its own translation Jacobian (:1766-1784), ARAP rows on original_graph_nodes
    (:1796-1840), A = JᵀJ + λI, b = -Jᵀr, LU, early stop (:1915-1926), update of the invalid nodes
    only (:1935-1943). Returns dict(node_rotations, node_translations, deformed_nodes_to_target,
    valid_solve, convergence_info)."""
    p = dict(GN_DEFAULTS)
    p.update(params)
    from scipy.linalg import lu_factor, lu_solve
    g = np.asarray(graph_nodes, F64)
    go = np.asarray(original_graph_nodes, F64)
    N = g.shape[0]
    valid = np.asarray(valid_nodes_mask, bool).reshape(N)
    vidx = np.nonzero(valid)[0]
    M = vidx.size
    src = np.asarray(source_node_position, F64).reshape(M, 3)
    tgt = np.asarray(target_node_position, F64).reshape(M, 3)
    R = np.asarray(R_current, F64).reshape(N, 3, 3).copy()
    t = np.asarray(t_current, F64).reshape(N, 3).copy()
    edges, (ei, ek) = gn_edges(graph_edges)
    E = edges.shape[0]
    n_nb = np.asarray(graph_edges).shape[1]
    ew = np.ones(E)
    if p['use_edge_weighting']:
        ew = float(n_nb) * np.asarray(graph_edges_weights, F64)[ei, ek]
    lf, la = math.sqrt(p['lambda_flow']), math.sqrt(p['lambda_arap'])
    lm_factor = p['lm_factor']
    conv = dict(total=[], arap=[], data=[], condition_numbers=[], valid=0, errors=[])
    inv = ~valid
    ill_posed = False
    res = None
    deformed = None
    for gn_i in range(p['num_iter']):
        if gn_i % 3 == 2:
            lm_factor /= 2
        deformed = src + t[vidx]
        J = np.zeros((M * 3, N * 6))
        rd = (lf * (deformed - tgt)).reshape(-1)
        for c in range(3):
            J[np.arange(M) * 3 + c, 3 * N + 3 * vidx + c] += rd[c::3]
        blocks_J, blocks_r = [J], [rd]
        ra = None
        if E > 0:
            Ja = np.zeros((E * 3, N * 6))
            i0, i1 = edges[:, 0], edges[:, 1]
            rowsE = np.arange(E) * 3
            delta = np.einsum('eij,ej->ei', R[i0], go[i1] - go[i0])
            ra = (la * ew[:, None] * (delta + go[i0] + t[i0] - (go[i1] + t[i1]))).reshape(-1)
            for c in range(3):
                Ja[rowsE + c, 3 * N + 3 * i0 + c] += la * ew
                Ja[rowsE + c, 3 * N + 3 * i1 + c] += -la * ew
            Sa = -la * ew[:, None, None] * skew(delta)
            for i in range(3):
                for j in range(3):
                    Ja[rowsE + i, 3 * i0 + j] += Sa[:, i, j]
            blocks_J.append(Ja)
            blocks_r.append(ra)
        Jall = np.concatenate(blocks_J, 0)
        res = np.concatenate(blocks_r, 0)
        A = Jall.T @ Jall + np.eye(6 * N) * lm_factor
        b = -(Jall.T @ res)
        try:
            x = lu_solve(lu_factor(A), b)
        except Exception:
            ill_posed = True
            conv['errors'].append("Solver failed: Ill-posed system!")
            break
        if not np.all(np.isfinite(x)):
            ill_posed = True
            conv['errors'].append("Solver failed: Non-finite solution x!")
            break
        loss_data, loss_total = float(np.linalg.norm(rd)), float(np.linalg.norm(res))
        if len(conv['total']):
            if loss_total - conv['total'][-1] > p['stop_loss_diff']:
                break
            if loss_total == conv['total'][-1]:
                break
        conv['data'].append(loss_data)
        conv['total'].append(loss_total)
        R_inc = angle_axis_to_rotation_matrix(x[:3 * N].reshape(N, 3))
        R[inv] = R_inc[inv] @ R[inv]
        t[inv] = t[inv] + x[3 * N:].reshape(N, 3)[inv]
        if ra is not None:
            conv['arap'].append(float(np.linalg.norm(ra)))
    valid_solve = (not ill_posed) and res is not None and bool(np.all(np.isfinite(res)))
    conv['valid'] = int(valid_solve)
    return dict(node_rotations=R, node_translations=t, deformed_nodes_to_target=deformed,
                valid_solve=int(valid_solve), convergence_info=conv)


def gn_system(graph_nodes, graph_edges, target_node_position, node_confidence, source_points, anchors,
              weights, target_points, intrinsics, R, t, lm_factor=1e-7, include_data=True, include_reg=True,
              **params):
    """A, b, ||res|| of one GN linearisation at (R, t) — dense, for block-level and sharding tests.
    include_data / include_reg select the data rows / the ARAP+motion rows (a match shard's share)."""
    out = {}
    p = dict(GN_DEFAULTS)
    p.update(params)
    p['num_iter'] = 1
    p['lm_factor'] = lm_factor
    # reuse gn_optimize's assembly by a single-iteration call would update R,t; rebuild here instead
    g = np.asarray(graph_nodes, F64)
    N = g.shape[0]
    src = np.asarray(source_points, F64)
    M = src.shape[0]
    anc = np.asarray(anchors, np.int64)
    wts = np.asarray(weights, F64)
    tgt = np.asarray(target_points, F64)
    conf = np.asarray(node_confidence, F64).reshape(-1)
    tpos = np.asarray(target_node_position, F64)
    fx, fy, cx, cy = (float(v) for v in intrinsics)
    R = np.asarray(R, F64)
    t = np.asarray(t, F64)
    ld, la, lmo = math.sqrt(p['lambda_depth']), math.sqrt(p['lambda_arap']), math.sqrt(p['lambda_motion'])
    defp = np.zeros((M, 3))
    for k in range(4):
        nk = anc[:, k]
        defp += wts[:, k:k + 1] * (np.einsum('mij,mj->mi', R[nk], src - g[nk]) + g[nk] + t[nk])
    zinv = 1.0 / (defp[:, 2] + 1e-7)
    mfx = -(fx * defp[:, 0] * zinv) * zinv
    mfy = -(fy * defp[:, 1] * zinv) * zinv
    rowsM = np.arange(M) * 3
    J = np.zeros((M * 3, N * 6))
    for k in range(4):
        nk = anc[:, k]
        wk = wts[:, k]
        S = -skew(wk[:, None] * np.einsum('mij,mj->mi', R[nk], src - g[nk]))
        for c in range(3):
            J[rowsM + c, 3 * N + 3 * nk + c] += ld * wk
        for j in range(3):
            J[rowsM, 3 * nk + j] += mfx * S[:, 2, j]
            J[rowsM + 1, 3 * nk + j] += mfy * S[:, 2, j]
        for i in range(3):
            for j in range(3):
                J[rowsM + i, 3 * nk + j] += ld * S[:, i, j]
    rd = (ld * (defp - tgt)).reshape(-1)
    edges, _ = gn_edges(graph_edges)
    E = edges.shape[0] if include_reg else 0
    Js, rs = ([J], [rd]) if include_data else ([], [])
    if E:
        i0, i1 = edges[:, 0], edges[:, 1]
        delta = np.einsum('eij,ej->ei', R[i0], g[i1] - g[i0])
        rs.append((la * (delta + g[i0] + t[i0] - (g[i1] + t[i1]))).reshape(-1))
        Ja = np.zeros((E * 3, N * 6))
        rowsE = np.arange(E) * 3
        for c in range(3):
            Ja[rowsE + c, 3 * N + 3 * i0 + c] += la
            Ja[rowsE + c, 3 * N + 3 * i1 + c] += -la
        Sa = -la * skew(delta)
        for i in range(3):
            for j in range(3):
                Ja[rowsE + i, 3 * i0 + j] += Sa[:, i, j]
        Js.append(Ja)
    if include_reg:
        Jm = np.zeros((N * 3, N * 6))
        ids = np.arange(N)
        for c in range(3):
            Jm[ids * 3 + c, 3 * N + 3 * ids + c] += lmo * conf
        Js.append(Jm)
        rs.append((lmo * conf[:, None] * (t + g - tpos)).reshape(-1))
    if not Js:
        Js, rs = [np.zeros((0, 6 * N))], [np.zeros(0)]
    Jall = np.concatenate(Js, 0)
    res = np.concatenate(rs, 0)
    out['A'] = Jall.T @ Jall + np.eye(6 * N) * lm_factor
    out['b'] = -(Jall.T @ res)
    out['loss'] = float(np.linalg.norm(res))
    out['loss2'] = float(res @ res)
    return out


def node_major_perm(N):
    """Permutation from the reference's [rot(3N) | trans(3N)] unknown order to [node: rot3, trans3]."""
    return np.concatenate([[3 * i, 3 * i + 1, 3 * i + 2, 3 * N + 3 * i, 3 * N + 3 * i + 1, 3 * N + 3 * i + 2]
                           for i in range(N)])


# ----------------------------------------------------------------------------
# f1: surface extraction — compute_truncated_region (tsdf.py:704-745) + marching cubes (skimage 0.22
#     measure.marching_cubes as called at tsdf.py:755,794) + get_mesh colours (tsdf.py:770-809)
# ----------------------------------------------------------------------------
def compute_truncated_region(tsdf_vol, max_diff):
    """tsdf.py:704-745 (numba prange): True where |t| <= 0.9, not on the volume boundary, and every one of
    the 27 neighbours (itself included) differs from t by at most max_diff. The neighbour writes inside
    the loop (`if abs(tsdf_vol[w,h,d]) > 0.9`, :738-739) are dead code (that case `continue`d at :727),
    so the result is race-free. Comparisons: f32 |t| and f32 |t_n - t| against f64 literals."""
    t = np.asarray(tsdf_vol, F32)
    W, H, D = t.shape
    out = ~(np.abs(t).astype(F64) > 0.9)
    inner = np.zeros_like(out)
    inner[1:-1, 1:-1, 1:-1] = True
    out &= inner
    if W < 3 or H < 3 or D < 3:
        return out
    c = t[1:-1, 1:-1, 1:-1]
    ok = np.ones(c.shape, bool)
    for dw in (-1, 0, 1):
        for dh in (-1, 0, 1):
            for dd in (-1, 0, 1):
                n = t[1 + dw:W - 1 + dw, 1 + dh:H - 1 + dh, 1 + dd:D - 1 + dd]
                ok &= ~(np.abs(n - c).astype(F64) > max_diff)
    out[1:-1, 1:-1, 1:-1] &= ok
    return out


FLT_EPSILON = float(np.finfo(np.float32).eps)
MC_EDGES = []          # 12 cube edges: (start corner, end corner); corner c = (c&1, c>>1&1, c>>2&1)
for _a in range(3):
    _b, _c = [x for x in range(3) if x != _a]
    for _oc in range(2):
        for _ob in range(2):
            _s = [0, 0, 0]
            _s[_b], _s[_c] = _ob, _oc
            _e = list(_s)
            _e[_a] = 1
            MC_EDGES.append((_s[0] + 2 * _s[1] + 4 * _s[2], _e[0] + 2 * _e[1] + 4 * _e[2]))


def mc_tables():
    """Triangle table of the 256 cube configurations (corner inside iff value < level), generated by rule
    rather than transcribed: on each cube face the cut edges pair up so that every run of inside corners
    is cut off on its own (ambiguous faces separate the inside corners — a rule that depends on the
    face's corner signs only, so neighbouring cells agree and the surface is closed); the face segments,
    directed exit -> entry with the inside on the left seen from outside the cube, chain into loops;
    each loop is fanned from its lowest edge id, wound so the right-hand normal points to the outside
    (values >= level). Returns list of 256 lists of (e0, e1, e2). Same rule as csrc/mc.hip."""
    edge_id = {}
    for k, (p, q) in enumerate(MC_EDGES):
        edge_id[(p, q)] = edge_id[(q, p)] = k
    faces = []
    for a in range(3):
        b, c = [x for x in range(3) if x != a]
        for s in range(2):
            cs = []
            for ub, uc in ((0, 0), (1, 0), (1, 1), (0, 1)):
                v = [0, 0, 0]
                v[a], v[b], v[c] = s, ub, uc
                cs.append(v[0] + 2 * v[1] + 4 * v[2])
            n = np.zeros(3)
            n[a] = 2 * s - 1
            if np.dot(np.cross(np.eye(3)[b], np.eye(3)[c]), n) < 0:
                cs = cs[::-1]
            faces.append(cs)
    tables = []
    for cfg in range(256):
        inside = [(cfg >> c) & 1 for c in range(8)]
        nxt = {}
        for cs in faces:
            ins = [inside[c] for c in cs]
            for i in range(4):
                if ins[i] and not ins[(i + 1) % 4]:
                    j = i
                    while ins[(j - 1) % 4]:
                        j -= 1
                    nxt[edge_id[(cs[i], cs[(i + 1) % 4])]] = edge_id[(cs[(j - 1) % 4], cs[j % 4])]
        tris, used = [], set()
        for s0 in sorted(nxt):
            if s0 in used:
                continue
            loop = [s0]
            used.add(s0)
            while nxt[loop[-1]] != s0:
                loop.append(nxt[loop[-1]])
                used.add(loop[-1])
            m = loop.index(min(loop))
            loop = loop[m:] + loop[:m]
            tris += [(loop[0], loop[i + 1], loop[i]) for i in range(1, len(loop) - 1)]
        tables.append(tris)
    return tables


def _grad(v, p, axis):
    """Central difference along axis at integer points p (n,3), one-sided on the volume boundary."""
    D = v.shape[axis]
    lo, hi = p.copy(), p.copy()
    lo[:, axis] = np.maximum(p[:, axis] - 1, 0)
    hi[:, axis] = np.minimum(p[:, axis] + 1, D - 1)
    num = v[tuple(hi.T)].astype(F64) - v[tuple(lo.T)].astype(F64)
    return num / (hi[:, axis] - lo[:, axis]).astype(F64)


def marching_cubes(volume, level=0.0, mask=None):
    """Marching cubes over a dense (X,Y,Z) f32 volume in voxel-index coordinates (the skimage convention,
    tsdf.py:755,794). Cell c = [c, c+1]³ is processed iff mask[c+1] (the cell's far corner) when a mask
    is given. One vertex per cut edge used by a processed cell: along the edge from p (value va) to
    p+e_a (vb), w = 1/(FLT_EPSILON+|v-level|) per end, offset = wb/(wa+wb), coordinate f32(p_a + offset);
    normal = normalised (wa·∇v(p) + wb·∇v(p+e_a))/(wa+wb) (central differences), pointing to increasing
    values; value = (wa·va + wb·vb)/(wa+wb). Vertices ordered by edge key = C-index(p)·3 + a.
    Returns (verts f32 (V,3), faces int64 (F,3), normals f32 (V,3), values f32 (V,), keys int64 (V,)).
    skimage's Lewiner tables and its vertex order are not available here (skimage is not installed):
    the triangulation is this module's rule (mc_tables), vertex positions follow the interpolation
    above — parity with skimage unpinned."""
    v = np.asarray(volume, F32)
    X, Y, Z = v.shape
    tabs = mc_tables()
    if X < 2 or Y < 2 or Z < 2:
        return (np.zeros((0, 3), F32), np.zeros((0, 3), np.int64), np.zeros((0, 3), F32), np.zeros(0, F32),
                np.zeros(0, np.int64))
    below = v < F32(level)
    idx = np.zeros((X - 1, Y - 1, Z - 1), np.int64)
    for c in range(8):
        dx, dy, dz = c & 1, (c >> 1) & 1, (c >> 2) & 1
        idx |= below[dx:X - 1 + dx, dy:Y - 1 + dy, dz:Z - 1 + dz].astype(np.int64) << c
    emit = (idx != 0) & (idx != 255)
    if mask is not None:
        emit &= np.asarray(mask, bool)[1:, 1:, 1:]
    cells = np.argwhere(emit)
    cfg = idx[emit]
    keys_t = []
    corner_off = np.array([[c & 1, (c >> 1) & 1, (c >> 2) & 1] for c in range(8)])
    edge_start = np.array([corner_off[p] for p, q in MC_EDGES])
    edge_axis = np.array([k // 4 for k in range(12)])
    tri_cell, tri_edges = [], []
    for ci, cf in zip(range(len(cells)), cfg):
        for tr in tabs[cf]:
            tri_cell.append(ci)
            tri_edges.append(tr)
    if not tri_cell:
        return (np.zeros((0, 3), F32), np.zeros((0, 3), np.int64), np.zeros((0, 3), F32), np.zeros(0, F32),
                np.zeros(0, np.int64))
    tri_cell = np.array(tri_cell)
    tri_edges = np.array(tri_edges)
    st = cells[tri_cell][:, None, :] + edge_start[tri_edges]                  # (F,3,3) start voxels
    keys_t = ((st[..., 0] * Y + st[..., 1]) * Z + st[..., 2]) * 3 + edge_axis[tri_edges]
    keys, faces = np.unique(keys_t.reshape(-1), return_inverse=True)
    faces = faces.reshape(-1, 3).astype(np.int64)
    a = keys % 3
    flat = keys // 3
    p = np.stack([flat // (Y * Z), (flat // Z) % Y, flat % Z], 1)
    q = p.copy()
    q[np.arange(len(q)), a] += 1
    va, vb = v[tuple(p.T)].astype(F64), v[tuple(q.T)].astype(F64)
    wa = 1.0 / (FLT_EPSILON + np.abs(va - level))
    wb = 1.0 / (FLT_EPSILON + np.abs(vb - level))
    off = wb / (wa + wb)
    verts = p.astype(F64)
    verts[np.arange(len(p)), a] += off
    g = np.zeros((len(p), 3))
    for ax in range(3):
        g[:, ax] = (wa * _grad(v, p, ax) + wb * _grad(v, q, ax)) / (wa + wb)
    nrm = np.sqrt((g[:, 0] * g[:, 0] + g[:, 1] * g[:, 1]) + g[:, 2] * g[:, 2])
    normals = g / np.where(nrm > 0, nrm, 1.0)[:, None]
    values = (wa * va + wb * vb) / (wa + wb)
    return verts.astype(F32), faces, normals.astype(F32), values.astype(F32), keys


def mesh_colors(verts, color_vol):
    """tsdf.py:759-767 / 800-807: colour of the voxel nearest each vertex (np.round half-even), unpacked
    from the b·65536 + g·256 + r float encoding in f32, as uint8 (N,3) [r, g, b]."""
    vi = np.rint(np.asarray(verts, F32)).astype(np.int64)
    rgb = np.asarray(color_vol, F32)[vi[:, 0], vi[:, 1], vi[:, 2]]
    b = np.floor(rgb / F32(COLOR_CONST))
    g = np.floor((rgb - b * F32(COLOR_CONST)) / F32(256))
    r = rgb - b * F32(COLOR_CONST) - g * F32(256)
    return np.floor(np.asarray([r, g, b])).T.astype(np.uint8)


def get_mesh(tsdf_vol, color_vol, voxel_size, origin, max_diff=1.2):
    """tsdf.py:770-809: masked marching cubes of the truncated region; voxel -> world as
    verts·f32(voxel_size) + origin in f32 (numpy-1.26 value-based casting); (verts, faces, norms, colors)."""
    mask = compute_truncated_region(tsdf_vol, max_diff)
    verts, faces, norms, _, _ = marching_cubes(tsdf_vol, 0.0, mask)
    colors = mesh_colors(verts, color_vol)
    world = verts * F32(voxel_size) + np.asarray(origin, F32)
    return world, faces, norms, colors


# ----------------------------------------------------------------------------
# f3: correspondence front-end — csrc image_proc.cpp:351-545 (backproject, pixel-grid mesh),
#     depth_2_pc (NonRigidICP/model/geometry.py:44-59), target cloud + pixel map
#     (registration_fusion.py:104-109, 388-395)
# ----------------------------------------------------------------------------
def backproject_depth(depth_image, fx, fy, cx, cy, normalizer=1000.0):
    """image_proc.cpp:351-401 via utils/image_proc.py:335-349: f32 arithmetic d*(x-cx)/fx, zeros where d <= 0.
    A float32 image is metres; any other dtype is read as uint16 and divided by f32(normalizer)."""
    f32 = np.float32
    if depth_image.dtype == np.float32:
        d = depth_image
    else:
        d = depth_image.astype(np.uint16).astype(f32) / f32(normalizer)
    H, W = d.shape
    xs = np.arange(W, dtype=f32)[None, :]
    ys = np.arange(H, dtype=f32)[:, None]
    out = np.zeros((3, H, W), f32)
    ok = d > 0
    px = (d * (xs - f32(cx))) / f32(fx)
    py = (d * (ys - f32(cy))) / f32(fy)
    out[0][ok] = px[ok]
    out[1][ok] = py[ok]
    out[2][ok] = d[ok]
    return out


def _edge_len_f32(a, b):
    """Eigen 3.3.7 (a-b).norm() for Vector3f: the unrolled redux sums x0 + (x1 + x2) (Redux.h:92-104)."""
    f32 = np.float32
    d = (a - b).astype(f32)
    s = d * d
    return np.sqrt(f32(s[0] + f32(s[1] + s[2])))


def compute_mesh_from_depth(point_image, max_dist):
    """image_proc.cpp:405-545, sequentially: quads row-major, triangle A (00, 01, 10) then B (11, 10, 01),
    vertices numbered on first use. Returns (vertices f32 (V,3), vertex_pixels i32 (V,2) [x,y],
    faces i32 (F,3)). Pure-Python loop: small images only."""
    f32 = np.float32
    P = np.asarray(point_image, f32)
    _, H, W = P.shape
    md = f32(max_dist)
    vmap = -np.ones(H * W, np.int64)
    verts, pix, faces = [], [], []

    def vid(x, y):
        i = y * W + x
        if vmap[i] < 0:
            vmap[i] = len(verts)
            verts.append(P[:, y, x])
            pix.append((x, y))
        return int(vmap[i])

    for y in range(H - 1):
        for x in range(W - 1):
            o00, o01, o10, o11 = P[:, y, x], P[:, y + 1, x], P[:, y, x + 1], P[:, y + 1, x + 1]
            if o00[2] > 0 and o01[2] > 0 and o10[2] > 0:
                if (_edge_len_f32(o00, o01) <= md and _edge_len_f32(o00, o10) <= md
                        and _edge_len_f32(o01, o10) <= md):
                    faces.append((vid(x, y), vid(x, y + 1), vid(x + 1, y)))
            if o01[2] > 0 and o10[2] > 0 and o11[2] > 0:
                if (_edge_len_f32(o10, o01) <= md and _edge_len_f32(o10, o11) <= md
                        and _edge_len_f32(o01, o11) <= md):
                    faces.append((vid(x + 1, y + 1), vid(x + 1, y), vid(x, y + 1)))
    V = np.array(verts, f32).reshape(-1, 3)
    return V, np.array(pix, np.int32).reshape(-1, 2), np.array(faces, np.int32).reshape(-1, 3)


def depth_2_pc(depth, intrin):
    """geometry.py:44-59: float64 (3,H,W) with X = ((u - cx)·d)/fx, Y = ((v - cy)·d)/fy, Z = d."""
    K = np.asarray(intrin, np.float64)
    H, W = depth.shape
    u = np.broadcast_to(np.arange(W, dtype=np.float64)[None, :], (H, W))
    v = np.broadcast_to(np.arange(H, dtype=np.float64)[:, None], (H, W))
    d = depth.astype(np.float64)
    return np.stack([(u - K[0, 2]) * d / K[0, 0], (v - K[1, 2]) * d / K[1, 1], d])


def xyz_2_uv(pcd, intrin):
    """NonRigidICP/model/geometry.py:30-41: pixel (u, v) of camera points, truncated toward zero by astype(int).
    Under the reference's numpy 1.x value-based casting the f64 intrinsic scalars meet the f32 point arrays as
    f32, so every step rounds to f32."""
    K = np.asarray(intrin, np.float64)
    f32 = np.float32
    X, Y, Z = (np.asarray(pcd[:, q], f32) for q in range(3))
    u = ((f32(K[0, 0]) * X) / Z + f32(K[0, 2])).astype(np.int64)
    v = ((f32(K[1, 1]) * Y) / Z + f32(K[1, 2])).astype(np.int64)
    return np.stack([u, v], -1)


def target_point_cloud(depth, intrin):
    """registration_fusion.py:104-109 + map_pixel_to_pcd (:388-395): the f32 cloud of pixels with depth > 0
    (row-major) and the pixel -> point index map (int64, -1 where invalid)."""
    ok = depth > 0
    pc = depth_2_pc(depth, intrin).transpose(1, 2, 0)[ok].astype(np.float32)
    pmap = np.cumsum(ok.reshape(-1)).reshape(ok.shape).astype(np.int64) - 1
    pmap[~ok] = -1
    return pc, pmap


# ----------------------------------------------------------------------------
# f2: standalone skinning / anchors — csrc graph_proc.cpp:483-709,934-961; KDTree.query in
#     WarpField.find_unreachable_nodes (warpfield.py:462-485); skin_image (warpfield.py:143-199)
# ----------------------------------------------------------------------------
GRAPH_K = 4   # csrc/cpu/graph_proc.h:8


def _csrc_weights(d2, cov):
    """graph_proc.cpp:147-153 + the normalisation at :672-696 / :583-597 for one anchor list (f32)."""
    f32 = np.float32
    two_c2 = f32(f32(2.0 * f32(cov)) * f32(cov))
    w = np.array([exp_f32(np.array([f32(-d) / two_c2], f32))[0] for d in d2], f32)
    s = f32(0)
    for x in w:
        s = f32(s + x)
    if s > 0:
        return (w / s).astype(f32)
    if len(w):
        return np.full(len(w), f32(1) / f32(len(w)), f32)
    return w


def pixel_anchors_euclidean(nodes, point_image, node_coverage):
    """compute_pixel_anchors_euclidean (graph_proc.cpp:610-709): brute-force 4-NN per pixel with z > 0, no
    cut-off; squared distance summed x0 + (x1 + x2) (Eigen); equal distances: the later node id first."""
    f32 = np.float32
    nodes = np.asarray(nodes, f32)
    P = np.asarray(point_image, f32)
    _, H, W = P.shape
    A = -np.ones((H, W, GRAPH_K), np.int32)
    Wt = np.zeros((H, W, GRAPH_K), f32)
    ys, xs = np.nonzero(P[2] > 0)
    pts = P[:, ys, xs].T
    if pts.shape[0] == 0 or nodes.shape[0] == 0:
        return A, Wt
    d = (pts[:, None, :] - nodes[None, :, :]).astype(f32)
    s = d * d
    d2 = (s[..., 0] + (s[..., 1] + s[..., 2])).astype(f32)
    ids = np.arange(nodes.shape[0])
    for r in range(pts.shape[0]):
        o = np.lexsort((-ids, d2[r]))[:GRAPH_K]
        A[ys[r], xs[r], :len(o)] = o
        Wt[ys[r], xs[r], :len(o)] = _csrc_weights(d2[r][o], node_coverage)
    return A, Wt


def pixel_anchors_geodesic(node_to_vertex_distance, valid_nodes_mask, vertex_pixels, width, height, node_coverage):
    """compute_pixel_anchors_geodesic (graph_proc.cpp:483-608): per vertex the valid nodes with distance >= 0
    in a set ordered by distance alone (the lowest node id of each distinct distance survives), first 4."""
    f32 = np.float32
    D = np.asarray(node_to_vertex_distance, f32)
    valid = np.asarray(valid_nodes_mask).reshape(-1) != 0
    A = -np.ones((height, width, GRAPH_K), np.int32)
    Wt = np.zeros((height, width, GRAPH_K), f32)
    for v in range(D.shape[1]):
        col = D[:, v]
        cand = np.nonzero(valid & (col >= 0))[0]
        if cand.size == 0:
            continue
        uq, first = np.unique(col[cand], return_index=True)
        sel = cand[first][:GRAPH_K]
        u, y = vertex_pixels[v]
        A[y, u, :len(sel)] = sel
        dd = col[sel]
        Wt[y, u, :len(sel)] = _csrc_weights((dd * dd).astype(f32), node_coverage)
    return A, Wt


def remap_anchors(anchors, node_id_mapping):
    """update_pixel_anchors (graph_proc.cpp:934-961): every anchor != -1 through the (old -> new) map."""
    out = np.array(anchors, np.int32, copy=True)
    flat = out.reshape(-1)
    for i, a in enumerate(flat):
        if a != -1:
            flat[i] = node_id_mapping[int(a)]
    return out


def knn(points, nodes, k):
    """k nearest nodes ascending by (f32 squared distance (dx²+dy²)+dz², node id) -> (idx, sq_dist)."""
    f32 = np.float32
    d = (np.asarray(points, f32)[:, None, :] - np.asarray(nodes, f32)[None, :, :]).astype(f32)
    s = d * d
    d2 = ((s[..., 0] + s[..., 1]) + s[..., 2]).astype(f32)
    o = np.argsort(d2, axis=1, kind="stable")[:, :k]
    return o.astype(np.int32), np.take_along_axis(d2, o, 1)


def find_unreachable_nodes(points, nodes, node_coverage):
    """warpfield.py:462-485: indices of points whose nearest node is farther than 2·coverage, sorted by that
    distance descending (argsort(...)[::-1]: among equal distances the later index first)."""
    _, d2 = knn(points, nodes, 1)
    dist = np.sqrt(d2.reshape(-1))
    un = np.where(dist > np.float32(2 * node_coverage))[0]
    if un.size == 0:
        return []
    return un[np.argsort(dist[un], kind="stable")[::-1]]


# ----------------------------------------------------------------------------
# f4: graph construction — csrc graph_proc.cpp:17-481 (erode_mesh, sample_nodes, compute_edges_geodesic,
#     compute_edges_euclidean, node_and_edge_clean_up, compute_clusters) as called by EDGraph
#     (embedded_deformation_graph.py:153-380); get_reduced_graph (:382-477)
# ----------------------------------------------------------------------------
def _eigen_sqnorm(d):
    """Eigen 3.3.7 squaredNorm of Vector3f rows: x0 + (x1 + x2) in f32."""
    s = (d * d).astype(np.float32)
    return (s[..., 0] + (s[..., 1] + s[..., 2])).astype(np.float32)


def erode_mesh(vertices, faces, n_iterations, min_neighbors):
    """graph_proc.cpp:17-77 -> non-eroded mask (V,1) bool."""
    V = np.asarray(vertices).shape[0]
    F = np.asarray(faces, np.int64).reshape(-1, 3)
    for _ in range(n_iterations):
        cnt = np.bincount(F.reshape(-1), minlength=V)
        F = F[(cnt[F] >= min_neighbors).all(1)]
    m = np.zeros(V, bool)
    m[F.reshape(-1)] = True
    return m.reshape(V, 1)


def sample_nodes(vertices, non_eroded, node_coverage, use_only_non_eroded=True):
    """graph_proc.cpp:79-136 with randomShuffle = False (EDGraph's SAMPLE_RANDOM_SHUFFLE,
    embedded_deformation_graph.py:195): vertices in index order, a vertex becomes a node iff no earlier node
    lies within squaredNorm <= coverage² (f32). -> (node positions (n,3) f32, node vertex indices (n,1) i32)."""
    f32 = np.float32
    P = np.asarray(vertices, f32)
    valid = np.asarray(non_eroded).reshape(-1).astype(bool)
    cov2 = f32(f32(node_coverage) * f32(node_coverage))
    nodes = np.zeros((0, 3), f32)
    idx = []
    for v in range(P.shape[0]):
        if use_only_non_eroded and not valid[v]:
            continue
        if nodes.shape[0] and (_eigen_sqnorm(P[v][None, :] - nodes) <= cov2).any():
            continue
        nodes = np.concatenate([nodes, P[v][None, :]])
        idx.append(v)
    return nodes, np.array(idx, np.int32).reshape(-1, 1)


def graph_downsample(old_nodes, node_coverage):
    """embedded_deformation_graph.py:278-299 (one level of create_graph_pyramid): nodes in order; the first is
    kept; every later node appends argmin (first minimum) of its f32 np.linalg.norm distances to the kept
    nodes (an index INTO the kept list, as the reference) to up_sample_idx, and is kept iff that minimum is
    not < node_coverage (f32 distance vs Python float: compared in f64 under the reference's numpy 1.26). -> (down_sample_idx, up_sample_idx) int lists."""
    P = np.asarray(old_nodes, np.float32)
    down, up = [], []
    for i in range(P.shape[0]):
        if not down:
            up.append(i)
            down.append(i)
            continue
        d = np.linalg.norm(P[down] - P[i], axis=1)
        j = int(np.argmin(d))
        up.append(j)
        if float(d[j]) < node_coverage:   # numpy 1.26 (environment.yml:94): f32 scalar vs Python float in f64
            continue
        down.append(i)
    return down, up


def _lt_push(h, hole, top, val):
    """libstdc++ std::__push_heap with CustomCompare (a.dist > b.dist: a min-heap on distance)."""
    parent = (hole - 1) // 2
    while hole > top and h[parent][1] > val[1]:
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = val


def _heap_push(h, val):
    h.append(val)
    _lt_push(h, len(h) - 1, 0, val)


def _heap_pop(h):
    """std::pop_heap + pop_back (libstdc++ __pop_heap / __adjust_heap)."""
    top = h[0]
    n = len(h) - 1
    if n > 0:
        val = h[n]
        h[n] = h[0]
        hole, second = 0, 0
        while second < (n - 1) // 2:
            second = 2 * (second + 1)
            if h[second][1] > h[second - 1][1]:
                second -= 1
            h[hole] = h[second]
            hole = second
        if (n & 1) == 0 and second == (n - 2) // 2:
            second = 2 * (second + 1)
            h[hole] = h[second - 1]
            hole = second - 1
        _lt_push(h, hole, 0, val)
    h.pop()
    return top


def vertex_neighbors(faces, V):
    nb = [set() for _ in range(V)]
    for f in np.asarray(faces).reshape(-1, 3):
        a, b, c = (int(x) for x in f)
        nb[a].update((b, c)); nb[b].update((a, c)); nb[c].update((a, b))
    for i in range(V):
        nb[i].discard(i)
    return [sorted(s) for s in nb]


def compute_edges_geodesic(vertices, valid_vertices, faces, node_indices, n_max_neighbors, node_coverage,
                           allow_only_valid_vertices=True, enforce_total_num_neighbors=True):
    """graph_proc.cpp:155-300: per node a Dijkstra over the mesh (std::priority_queue semantics restated
    exactly, neighbours in ascending id) collecting the first n_max_neighbors other nodes reached.
    -> (edges (N,K) i32 -1-padded, weights (N,K) f32, distances (N,K) f32, node_to_vertex (N,V) f32 -1)."""
    f32 = np.float32
    P = np.asarray(vertices, f32)
    V = P.shape[0]
    valid = np.asarray(valid_vertices).reshape(V, -1)[:, 0].astype(bool)
    ni = np.asarray(node_indices).reshape(-1)
    N = ni.shape[0]
    K = n_max_neighbors
    nb = vertex_neighbors(faces, V)
    v2n = -np.ones(V, np.int64)
    for n in range(N):
        if ni[n] >= 0:
            v2n[ni[n]] = n
    max_inf = f32(2.0 * f32(node_coverage))
    E = -np.ones((N, K), np.int32)
    EW = np.zeros((N, K), f32)
    ED = np.zeros((N, K), f32)
    D = -np.ones((N, V), f32)
    for n in range(N):
        s = int(ni[n])
        if s < 0:
            continue
        h = [(s, f32(0))]
        visited = set()
        ids, ds = [], []
        while h:
            v, d = _heap_pop(h)
            if v in visited:
                continue
            if allow_only_valid_vertices and not valid[v]:
                raise RuntimeError("compute_edges_geodesic: visited an invalid vertex (the C++ calls exit(0))")
            m = v2n[v]
            if m >= 0 and m != n:
                ids.append(int(m)); ds.append(d)
                if len(ids) >= K:
                    break
            D[n, v] = d
            visited.add(v)
            for u in nb[v]:
                if allow_only_valid_vertices and not valid[u]:
                    continue
                dist = f32(d + np.sqrt(_eigen_sqnorm((P[v] - P[u])[None, :])[0]))
                if enforce_total_num_neighbors or dist <= max_inf:
                    _heap_push(h, (u, dist))
        if ids:
            dd = np.array(ds, f32)
            two_c2 = f32(f32(2.0 * f32(node_coverage)) * f32(node_coverage))
            w = exp_f32(-(dd * dd) / two_c2)
            tot = f32(0)
            for x in w:
                tot = f32(tot + x)
            w = w / tot if tot > 0 else w / f32(len(ids))      # graph_proc.cpp:270-281 (w / n, not 1 / n)
            E[n, :len(ids)] = ids
            EW[n, :len(ids)] = w
            ED[n, :len(ids)] = ds
    return E, EW, ED, D


def compute_edges_euclidean(nodes, n_max_neighbors):
    """graph_proc.cpp:302-356: K nearest other nodes, csrc list semantics (ties: later id first), -1 padded."""
    f32 = np.float32
    X = np.asarray(nodes, f32)
    N = X.shape[0]
    E = -np.ones((N, n_max_neighbors), np.int32)
    ids = np.arange(N)
    for n in range(N):
        d2 = _eigen_sqnorm(X[n][None, :] - X)
        o = [i for i in np.lexsort((-ids, d2)) if i != n][:n_max_neighbors]
        E[n, :len(o)] = o
    return E


def node_and_edge_clean_up(graph_edges, valid_nodes_mask):
    """graph_proc.cpp:388-438 (in place on a copy): sweeps in node order until no removal; a node with <= 1
    neighbour not removed BY THIS CALL is removed (neighbours invalid on entry still count)."""
    E = np.asarray(graph_edges)
    valid = np.array(valid_nodes_mask, bool).reshape(-1, 1).copy()
    removed = set()
    while True:
        k = 0
        for n in range(E.shape[0]):
            if not valid[n, 0]:
                continue
            c = 0
            for j in E[n]:
                if j == -1:
                    break
                if int(j) in removed:
                    continue
                c += 1
            if c <= 1:
                valid[n, 0] = False
                removed.add(n)
                k += 1
        if k == 0:
            return valid


def compute_clusters(graph_edges):
    """graph_proc.cpp:440-481: connected components of the symmetrised edge graph, numbered by their lowest
    node id -> (clusters (N,1) i32, sizes list)."""
    E = np.asarray(graph_edges)
    N = E.shape[0]
    nb = [set() for _ in range(N)]
    for n in range(N):
        for j in E[n]:
            if j == -1:
                break
            nb[n].add(int(j)); nb[int(j)].add(n)
    cl = -np.ones(N, np.int32)
    sizes = []
    for s in range(N):
        if cl[s] != -1:
            continue
        stack, size = [s], 0
        cl[s] = len(sizes)
        while stack:
            a = stack.pop()
            size += 1
            for b in nb[a]:
                if cl[b] == -1:
                    cl[b] = len(sizes)
                    stack.append(b)
        sizes.append(size)
    return cl.reshape(N, 1), sizes


def reduced_graph(nodes, edges, edges_weights, edges_distances, clusters, valid_nodes_mask):
    """EDGraph.get_reduced_graph (embedded_deformation_graph.py:382-477): keep valid nodes, drop edges to
    removed nodes (compacted left, ids remapped) and renormalise the weights by (sum + 1e-6) in f32."""
    m = np.asarray(valid_nodes_mask).reshape(-1).astype(bool)
    nodes_r, E = nodes[m].copy(), edges[m].copy()
    W, Dd, C = edges_weights[m].copy(), edges_distances[m].copy(), clusters[m].copy()
    black = np.nonzero(~m)[0]
    if black.size:
        new_id = np.cumsum(m) - 1
        for r in range(E.shape[0]):
            e, w, d = E[r].copy(), W[r].copy(), Dd[r].copy()
            keep = ~np.isin(e, black)
            E[r], W[r], Dd[r] = -1, 0, 0
            c = 0
            for j in np.nonzero(keep)[0]:
                E[r, c] = -1 if e[j] == -1 else new_id[e[j]]
                W[r, c], Dd[r, c] = w[j], d[j]
                c += 1
            s = _np_sum_f32(W[r])
            if s > 0:        # numpy 1.26 (environment.yml:94): f32 scalar + 1e-6 is f64, cast back for the division
                W[r] /= np.float32(np.float64(s) + 1e-6)
    return nodes_r, E, W, Dd, C


def _np_sum_f32(a):
    """numpy's pairwise float32 sum of a short contiguous row (< 8: in order; 8..128: 8 partial sums)."""
    a = np.asarray(a, np.float32)
    f32 = np.float32
    n = a.shape[0]
    if n < 8:
        s = f32(0)
        for x in a:
            s = f32(s + x)
        return s
    r = [f32(x) for x in a[:8]]
    i = 8
    while i + 8 <= n:
        for j in range(8):
            r[j] = f32(r[j] + a[i + j])
        i += 8
    s = f32(f32(f32(r[0] + r[1]) + f32(r[2] + r[3])) + f32(f32(r[4] + r[5]) + f32(r[6] + r[7])))
    for x in a[i:]:
        s = f32(s + x)
    return s


# ----------------------------------------------------------------------------
# (new capability) TSDF raycast — no reference twin: the restatement of csrc/raycast.hip op for op (f32,
# un-contracted), so the GPU kernel can be checked bit for bit. Parity against the reference is unpinned.
# ----------------------------------------------------------------------------
def raycast(tsdf, weight, color, origin, voxel_size, intr, height, width, z_near=0.1, z_far=10.0,
            trunc=TRUNC_MARGIN, rows=None):
    """Depth (H,W), normals (H,W,3), colours (H,W) of dense C-order volumes (Dx,Dy,Dz) seen from the identity
    camera: trilinear tsdf march (unobserved / outside = +1), coarse steps 0.8·trunc while >= 0.999, else one
    voxel; first + -> - change refined linearly; central-difference normals; nearest-voxel colour.
    rows: optional subset of image rows (the other rows stay 0)."""
    tsdf = np.asarray(tsdf, F32)
    weight = np.asarray(weight, F32)
    D = tsdf.shape
    lo = np.asarray(origin, F32)
    hi = np.array([F32(float(origin[a]) + float(voxel_size) * D[a]) for a in range(3)], F32)
    inv_vs = F32(1.0 / float(voxel_size))
    step_c, step_f = F32(0.8 * trunc), F32(float(voxel_size))
    fx, fy, cx, cy = (F32(v) for v in intr)
    rows = np.arange(height) if rows is None else np.asarray(rows)
    vv, uu = np.meshgrid(rows, np.arange(width), indexing="ij")
    u, v = uu.reshape(-1), vv.reshape(-1)
    dx = (u.astype(F32) - cx) / fx
    dy = (v.astype(F32) - cy) / fy
    n = u.size
    z0 = np.full(n, F32(z_near), F32)
    z1 = np.full(n, F32(z_far), F32)
    miss = np.zeros(n, bool)
    for a, d in enumerate((dx, dy, np.ones(n, F32))):
        zero = d == 0
        miss |= zero & ~((F32(0) >= lo[a]) & (F32(0) <= hi[a]))
        with np.errstate(divide="ignore", invalid="ignore"):
            ta = np.where(zero, F32(0), lo[a] / np.where(zero, F32(1), d)).astype(F32)
            tb = np.where(zero, F32(0), hi[a] / np.where(zero, F32(1), d)).astype(F32)
        z0 = np.where(zero, z0, np.maximum(z0, np.minimum(ta, tb)))
        z1 = np.where(zero, z1, np.minimum(z1, np.maximum(ta, tb)))

    def voxel(i, j, k):
        ok = (i >= 0) & (j >= 0) & (k >= 0) & (i < D[0]) & (j < D[1]) & (k < D[2])
        ic, jc, kc = (np.clip(x, 0, D[q] - 1) for q, x in enumerate((i, j, k)))
        t = tsdf[ic, jc, kc]
        w = weight[ic, jc, kc]
        return np.where(ok & (w > 0), t, F32(1)).astype(F32)

    def trilinear(qx, qy, qz):
        f0 = [np.floor(q) for q in (qx, qy, qz)]
        ax, ay, az = (q - f for q, f in zip((qx, qy, qz), f0))
        i, j, k = (f.astype(np.int64) for f in f0)
        t000, t100, t010, t110 = voxel(i, j, k), voxel(i + 1, j, k), voxel(i, j + 1, k), voxel(i + 1, j + 1, k)
        t001, t101, t011, t111 = (voxel(i, j, k + 1), voxel(i + 1, j, k + 1), voxel(i, j + 1, k + 1),
                                  voxel(i + 1, j + 1, k + 1))
        bx, by, bz = F32(1) - ax, F32(1) - ay, F32(1) - az
        c00, c10 = t000 * bx + t100 * ax, t010 * bx + t110 * ax
        c01, c11 = t001 * bx + t101 * ax, t011 * bx + t111 * ax
        c0, c1 = c00 * by + c10 * ay, c01 * by + c11 * ay
        return (c0 * bz + c1 * az).astype(F32)

    hit = np.zeros(n, F32)
    act = np.nonzero(~miss & (z0 <= z1))[0]
    z, zp, sp = z0[act].copy(), z0[act].copy(), np.ones(act.size, F32)
    have = np.zeros(act.size, bool)   # a sign change needs a real sample before it (no hit at the entry plane)
    while act.size:
        run = z <= z1[act]
        act, z, zp, sp, have = act[run], z[run], zp[run], sp[run], have[run]
        if not act.size:
            break
        s = trilinear((z * dx[act] - lo[0]) * inv_vs, (z * dy[act] - lo[1]) * inv_vs, (z - lo[2]) * inv_vs)
        h = have & (sp > 0) & (s < 0)
        hit[act[h]] = zp[h] + (z[h] - zp[h]) * (sp[h] / (sp[h] - s[h]))
        keep = ~h
        act, z, s = act[keep], z[keep], s[keep]
        zp, sp, have = z.copy(), s, np.ones(act.size, bool)
        z = (z + np.where(s >= F32(0.999), step_c, step_f)).astype(F32)
    nrm = np.zeros((n, 3), F32)
    col = np.zeros(n, F32)
    hh = np.nonzero(hit > 0)[0]
    if hh.size:
        zh = hit[hh]
        qx, qy, qz = (zh * dx[hh] - lo[0]) * inv_vs, (zh * dy[hh] - lo[1]) * inv_vs, (zh - lo[2]) * inv_vs
        one = F32(1)
        g = np.stack([trilinear(qx + one, qy, qz) - trilinear(qx - one, qy, qz),
                      trilinear(qx, qy + one, qz) - trilinear(qx, qy - one, qz),
                      trilinear(qx, qy, qz + one) - trilinear(qx, qy, qz - one)], 1).astype(F32)
        ln = np.sqrt((g[:, 0] * g[:, 0] + g[:, 1] * g[:, 1]) + g[:, 2] * g[:, 2])
        with np.errstate(divide="ignore", invalid="ignore"):
            nrm[hh] = np.where((ln > 0)[:, None], g / np.where(ln > 0, ln, one)[:, None], F32(0))
        if color is not None:
            ii, jj, kk = (np.floor(q + F32(0.5)).astype(np.int64) for q in (qx, qy, qz))
            ok = (ii >= 0) & (jj >= 0) & (kk >= 0) & (ii < D[0]) & (jj < D[1]) & (kk < D[2])
            cv = np.asarray(color, F32)[np.clip(ii, 0, D[0] - 1), np.clip(jj, 0, D[1] - 1), np.clip(kk, 0, D[2] - 1)]
            col[hh] = np.where(ok, cv, F32(0))
    out_d = np.zeros((height, width), F32)
    out_n = np.zeros((height, width, 3), F32)
    out_c = np.zeros((height, width), F32)
    out_d[rows] = hit.reshape(rows.size, width)
    out_n[rows] = nrm.reshape(rows.size, width, 3)
    out_c[rows] = col.reshape(rows.size, width)
    return out_d, out_n, out_c
