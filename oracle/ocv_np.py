"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product package).

NumPy restatement of the OpenCV 4.x primitives on the reference hot path, written
independently of ``ocv_ref.c`` so the two restatements cross-check each other, and a
restatement of ``bev_transform_tools.create_occupancy_grid`` that follows the reference's
own array flow (full warped image, then the crop/pad slicing of bev.py:183-195) rather than
the coordinate-shift form the C oracle and the HIP kernel use.

Parity status: UNPINNED against OpenCV/TensorFlow (neither is installed, the reference holds
no fixtures). Semantics pinned to the classic OpenCV 4.x fixed-point paths,
see ocv_ref.c's header.
"""
from __future__ import annotations

import numpy as np

INTER_BITS = 5
INTER_TAB_SIZE = 1 << INTER_BITS


def invert3x3(M: np.ndarray) -> np.ndarray:
    """cv::invert DECOMP_LU closed-form 3x3 branch (used by warpPerspective, bev.py:182)."""
    S = np.asarray(M, dtype=np.float64).reshape(3, 3)
    d = (S[0, 0] * (S[1, 1] * S[2, 2] - S[1, 2] * S[2, 1])
         - S[0, 1] * (S[1, 0] * S[2, 2] - S[1, 2] * S[2, 0])
         + S[0, 2] * (S[1, 0] * S[2, 1] - S[1, 1] * S[2, 0]))
    if d == 0.0:
        return np.zeros((3, 3))
    d = 1.0 / d
    t = np.empty(9)
    t[0] = (S[1, 1] * S[2, 2] - S[1, 2] * S[2, 1]) * d
    t[1] = (S[0, 2] * S[2, 1] - S[0, 1] * S[2, 2]) * d
    t[2] = (S[0, 1] * S[1, 2] - S[0, 2] * S[1, 1]) * d
    t[3] = (S[1, 2] * S[2, 0] - S[1, 0] * S[2, 2]) * d
    t[4] = (S[0, 0] * S[2, 2] - S[0, 2] * S[2, 0]) * d
    t[5] = (S[0, 2] * S[1, 0] - S[0, 0] * S[1, 2]) * d
    t[6] = (S[1, 0] * S[2, 1] - S[1, 1] * S[2, 0]) * d
    t[7] = (S[0, 1] * S[2, 0] - S[0, 0] * S[2, 1]) * d
    t[8] = (S[0, 0] * S[1, 1] - S[0, 1] * S[1, 0]) * d
    return t.reshape(3, 3)


def warp_perspective(src: np.ndarray, M: np.ndarray, dsize: tuple[int, int]) -> np.ndarray:
    """cv2.warpPerspective(src u8 1ch, M, dsize=(w, h)), INTER_LINEAR, BORDER_CONSTANT 0.

    WarpPerspectiveInvoker forms X0/Y0/W0 at each block start xb (block width
    bw0 = min(1024 // min(16, h), w)) and adds M0*x1 inside the block; remapBilinear
    interpolates with the Q15 table indexed by the 5-bit fractions."""
    dw, dh = dsize
    sh, sw = src.shape
    Mi = invert3x3(M).ravel()
    bh0 = min(16, dh)
    bw0 = min(1024 // bh0, dw)
    ys, xs = np.meshgrid(np.arange(dh), np.arange(dw), indexing="ij")
    xb = (xs // bw0) * bw0
    x1 = (xs - xb).astype(np.float64)
    xb = xb.astype(np.float64)
    yd = ys.astype(np.float64)
    X0 = Mi[0] * xb + Mi[1] * yd + Mi[2]
    Y0 = Mi[3] * xb + Mi[4] * yd + Mi[5]
    W0 = Mi[6] * xb + Mi[7] * yd + Mi[8]
    W = W0 + Mi[6] * x1
    with np.errstate(divide="ignore"):
        W = np.where(W != 0.0, INTER_TAB_SIZE / np.where(W != 0.0, W, 1.0), 0.0)
    fX = np.clip((X0 + Mi[0] * x1) * W, -2147483648.0, 2147483647.0)
    fY = np.clip((Y0 + Mi[3] * x1) * W, -2147483648.0, 2147483647.0)
    X = np.rint(fX).astype(np.int64)          # np.rint: round half to even == cvRound
    Y = np.rint(fY).astype(np.int64)
    sx = np.clip(X >> INTER_BITS, -32768, 32767)
    sy = np.clip(Y >> INTER_BITS, -32768, 32767)
    ax = X & (INTER_TAB_SIZE - 1)
    ay = Y & (INTER_TAB_SIZE - 1)
    src_i = src.astype(np.int64)

    def tap(yy, xx):
        ok = (yy >= 0) & (yy < sh) & (xx >= 0) & (xx < sw)
        return np.where(ok, src_i[np.clip(yy, 0, sh - 1), np.clip(xx, 0, sw - 1)], 0)

    acc = (tap(sy, sx) * (32 - ax) * (32 - ay) + tap(sy, sx + 1) * ax * (32 - ay)
           + tap(sy + 1, sx) * (32 - ax) * ay + tap(sy + 1, sx + 1) * ax * ay) * 32
    return np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)


def resize_nearest(src: np.ndarray, dsize: tuple[int, int]) -> np.ndarray:
    """cv2.resize(..., INTER_NEAREST) (resizeNN): floor(d * (1/(dw/sw))), clamped."""
    dw, dh = dsize
    sh, sw = src.shape[:2]
    ifx = 1.0 / (dw / sw)
    ify = 1.0 / (dh / sh)
    sx = np.minimum(np.floor(np.arange(dw) * ifx).astype(np.int64), sw - 1)
    sy = np.minimum(np.floor(np.arange(dh) * ify).astype(np.int64), sh - 1)
    return src[sy][:, sx]


def morph_open3x3(src: np.ndarray) -> np.ndarray:
    """cv2.morphologyEx(src, MORPH_OPEN, ones((3,3))) with the default border values."""
    h, w = src.shape
    big = np.full((h + 2, w + 2), 255, dtype=np.uint8)
    big[1:-1, 1:-1] = src
    er = np.full((h, w), 255, dtype=np.uint8)
    for dy in range(3):
        for dx in range(3):
            er = np.minimum(er, big[dy:dy + h, dx:dx + w])
    big = np.zeros((h + 2, w + 2), dtype=np.uint8)
    big[1:-1, 1:-1] = er
    di = np.zeros((h, w), dtype=np.uint8)
    for dy in range(3):
        for dx in range(3):
            di = np.maximum(di, big[dy:dy + h, dx:dx + w])
    return di


def _linear_coeffs(dsize: int, ssize: int, scale: float):
    d = np.arange(dsize)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo] = 0.0
    s[lo] = 0
    hi = s >= ssize - 1
    f[hi] = 0.0
    s[hi] = ssize - 1
    a0 = np.clip(np.rint((np.float32(1.0) - f) * np.float32(2048.0)), -32768, 32767).astype(np.int64)
    a1 = np.clip(np.rint(f * np.float32(2048.0)), -32768, 32767).astype(np.int64)
    return s, a0, a1


def resize_linear(src: np.ndarray, dsize: tuple[int, int]) -> np.ndarray:
    """cv2.resize(src u8 HxWxC, dsize) default INTER_LINEAR, classic fixed point (see ocv_ref.c)."""
    dw, dh = dsize
    sh, sw = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    if (sh, sw) == (dh, dw):
        return src.copy()
    s3 = src.reshape(sh, sw, cn).astype(np.int64)
    scale_x = 1.0 / (dw / sw)
    scale_y = 1.0 / (dh / sh)
    isx, isy = int(np.rint(scale_x)), int(np.rint(scale_y))
    eps = np.finfo(np.float64).eps
    if abs(scale_x - isx) < eps and abs(scale_y - isy) < eps and isx == 2 and isy == 2:
        v = s3[0:2 * dh:2, 0:2 * dw:2] + s3[0:2 * dh:2, 1:2 * dw:2] + s3[1:2 * dh:2, 0:2 * dw:2] + s3[1:2 * dh:2, 1:2 * dw:2]
        out = ((v + 2) >> 2).astype(np.uint8)
        return out[..., 0] if src.ndim == 2 else out
    xo, xa0, xa1 = _linear_coeffs(dw, sw, scale_x)
    yo, yb0, yb1 = _linear_coeffs(dh, sh, scale_y)
    xo1 = np.minimum(xo + 1, sw - 1)
    hrow = s3[:, xo, :] * xa0[None, :, None] + s3[:, xo1, :] * xa1[None, :, None]   # (sh, dw, cn)
    r0 = hrow[yo].reshape(dh, dw * cn)
    r1 = hrow[np.minimum(yo + 1, sh - 1)].reshape(dh, dw * cn)
    b0 = yb0[:, None]
    b1 = yb1[:, None]
    width = dw * cn
    vec_end = width - (width % 8)
    s0 = np.clip(r0 >> 4, -32768, 32767)
    s1 = np.clip(r1 >> 4, -32768, 32767)
    vec = (((s0 * b0) >> 16) + ((s1 * b1) >> 16) + 2) >> 2
    sca = (r0 * b0 + r1 * b1 + (1 << 21)) >> 22
    out = np.where(np.arange(width)[None, :] < vec_end, vec, sca)
    out = np.clip(out, 0, 255).astype(np.uint8).reshape(dh, dw, cn)
    return out[..., 0] if src.ndim == 2 else out


def create_occupancy_grid(segmap: np.ndarray, M: np.ndarray, after_warp_w: int, after_warp_h: int,
                          cm_per_px: float, grid_w_m: float, grid_h_m: float, cell_m: float) -> np.ndarray:
    """Restates bev.py:166-246 (non-laserscan branch) step by step on the arrays it builds."""
    cell_px = cell_m * 100 / cm_per_px                                   # bev.py:172
    occ_w = int(grid_w_m / cell_m)                                       # bev.py:173
    occ_w_px = int(occ_w * cell_px)                                      # bev.py:174
    occ_h = int(grid_h_m / cell_m)                                       # bev.py:175
    occ_h_px = int(occ_h * cell_px)                                      # bev.py:176
    lifted = np.add(segmap, 1).astype(np.uint8)                          # bev.py:177
    warped = warp_perspective(lifted, M, (after_warp_w, after_warp_h))   # bev.py:182
    left_x = int((after_warp_w - occ_w_px) / 2)                          # bev.py:183
    top_y = after_warp_h - occ_h_px                                      # bev.py:184
    wlx = int(np.clip(left_x, 0, np.inf))                                # bev.py:185
    warped = warped[int(np.clip(top_y, 0, np.inf)):after_warp_h, wlx:wlx + occ_w_px]   # bev.py:186
    glx = int(np.clip(-left_x, 0, np.inf))                               # bev.py:188
    gty = int(np.clip(-top_y, 0, np.inf))                                # bev.py:189
    tmpl = np.zeros((occ_h_px, occ_w_px))                                # bev.py:190
    tmpl[gty:occ_h_px, glx:glx + warped.shape[1]] = warped               # bev.py:192
    tmpl = tmpl.astype(np.uint8)                                         # bev.py:195
    occ = np.logical_or(tmpl == 1, tmpl == 3).astype(np.uint8)           # bev.py:196
    opened = morph_open3x3(occ)                                          # bev.py:198
    mask1 = (opened > 0).astype(np.uint8)                                # bev.py:203
    sub = np.clip(occ.astype(np.int16) - mask1, 0, 255)                  # bev.py:204 cv2.subtract saturates
    tmpl = np.where(sub > 0, 2, tmpl).astype(np.uint8)                   # bev.py:205
    tmpl = resize_nearest(tmpl, (occ_w, occ_h))                          # bev.py:209
    new = np.where(tmpl == 3, 1, tmpl)                                   # bev.py:242
    return np.where(new == 0, -1, 200 - new.astype(np.int64) * 100).astype(np.int8)   # bev.py:244


def create_occupancy_grid_binary(segmap: np.ndarray, M: np.ndarray, after_warp_w: int, after_warp_h: int,
                                 cm_per_px: float, grid_w_m: float, grid_h_m: float, cell_m: float) -> np.ndarray:
    """Restates bev.py:97-165 (legacy binary variant, non-laserscan branch) on the arrays it builds.
    Its uint8 arithmetic is NumPy 1.x's (value-based casting, wrap-around), emulated explicitly."""
    cell_px = cell_m * 100 / cm_per_px                                   # bev.py:103
    occ_w = int(grid_w_m / cell_m)                                       # bev.py:104
    occ_w_px = int(occ_w * cell_px)                                      # bev.py:105
    occ_h = int(grid_h_m / cell_m)                                       # bev.py:106
    occ_h_px = int(occ_h * cell_px)                                      # bev.py:107
    lifted = np.add(segmap, 1).astype(np.uint8)                          # bev.py:108
    warped = warp_perspective(lifted, M, (after_warp_w, after_warp_h))   # bev.py:114
    left_x = int((after_warp_w - occ_w_px) / 2)                          # bev.py:115
    top_y = after_warp_h - occ_h_px                                      # bev.py:116
    wlx = int(np.clip(left_x, 0, np.inf))                                # bev.py:117
    warped = warped[int(np.clip(top_y, 0, np.inf)):after_warp_h, wlx:wlx + occ_w_px]   # bev.py:118-119
    glx = int(np.clip(-left_x, 0, np.inf))                               # bev.py:120
    gty = int(np.clip(-top_y, 0, np.inf))                                # bev.py:121
    tmpl = np.zeros((occ_h_px, occ_w_px))                                # bev.py:122
    tmpl[gty:occ_h_px, glx:glx + warped.shape[1]] = warped               # bev.py:124-126
    tmpl = tmpl.astype(np.uint8)                                         # bev.py:127
    occ = (tmpl == 1).astype(np.uint8)                                   # bev.py:128
    opened = morph_open3x3(occ)                                          # bev.py:130-131
    mask1 = (opened > 0).astype(np.uint8)                                # bev.py:133
    sub = np.clip(occ.astype(np.int16) - mask1, 0, 255)                  # bev.py:134 cv2.subtract saturates
    tmpl = np.where(sub > 0, 2, tmpl).astype(np.uint8)                   # bev.py:135
    og = (resize_nearest(tmpl, (occ_w, occ_h)).astype(np.int64) * 100) % 256   # bev.py:139-142: uint8 * 100 wraps
    r = np.where(og == 0, -1, (200 - og) % 256)                          # bev.py:143-144 (uint8 200 - og)
    return (r % 256).astype(np.uint8).astype(np.int8)                    # bev.py:144, :165


def ros_layout(grid: np.ndarray) -> np.ndarray:
    """cv2.flip(g, 0) then cv2.rotate(ROTATE_90_COUNTERCLOCKWISE) (occgrid_to_ros.py:18,21)."""
    flipped = grid[::-1, :]
    return np.ascontiguousarray(np.rot90(flipped, 1))


# ---- laserscan-like occupancy (bev.py:216-240, binary variant bev.py:143-164) -----------------------

CV_PI = 3.1415926535897932384626433832795
_F = np.float32
_ATAN_P = [_F(c) * _F(180 / CV_PI) for c in (0.9997878412794807, -0.3258083974640975, 0.1555786518463281,
                                              -0.04432655554792128)]   # p1, p3, p5, p7 (float products)


def _fma32(a, b, c):
    """float32 fused multiply-add (one rounding) via 80-bit long double: a*b of two floats is exact
    there and the sum rounds once before the float32 rounding."""
    ld = np.longdouble
    return (np.asarray(a, ld) * np.asarray(b, ld) + np.asarray(c, ld)).astype(_F)


def fast_atan_rad(y: np.ndarray, x: np.ndarray) -> np.ndarray:
    """cv::hal::fastAtan32f (AVX2 dispatch, v_fma polynomial), angle in radians, float32."""
    x = np.asarray(x, _F)
    y = np.asarray(y, _F)
    ax, ay = np.abs(x), np.abs(y)
    c = np.minimum(ax, ay) / (np.maximum(ax, ay) + _F(2.220446049250313e-16))
    cc = c * c
    p1, p3, p5, p7 = _ATAN_P
    a = _fma32(_fma32(_fma32(cc, p7, p5), cc, p3), cc, p1) * c
    a = np.where(ax >= ay, a, _F(90) - a)
    a = np.where(x < 0, _F(180) - a, a)
    a = np.where(y < 0, _F(360) - a, a)
    return (a * _F(CV_PI / 180)).astype(_F)


def _remap_nearest(src: np.ndarray, mx: np.ndarray, my: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """remap(INTER_NEAREST, BORDER_TRANSPARENT) with float maps: coordinates round half-to-even to
    short; pixels mapping outside src keep dst's value."""
    sx = np.clip(np.rint(mx), -32768, 32767).astype(np.int64)
    sy = np.clip(np.rint(my), -32768, 32767).astype(np.int64)
    ok = (sx >= 0) & (sx < src.shape[1]) & (sy >= 0) & (sy < src.shape[0])
    dst[ok] = src[sy[ok], sx[ok]]
    return dst


def warp_polar(src: np.ndarray, dsize, center, max_radius: float, inverse: bool = False) -> np.ndarray:
    """cv2.warpPolar(src, dsize, center, maxRadius, WARP_POLAR_LINEAR [| WARP_INVERSE_MAP]) with
    INTER_NEAREST and BORDER_TRANSPARENT (imgwarp.cpp 4.x). The destination starts zeroed (the
    reference's is an uninitialised array: pixels mapping outside the source are unspecified there)."""
    dw, dh = dsize
    cx, cy = _F(center[0]), _F(center[1])
    if not inverse:
        if dw <= 0 and dh <= 0:
            dw, dh = int(np.rint(max_radius)), int(np.rint(max_radius * CV_PI))
        elif dh <= 0:
            dh = int(np.rint(dw * CV_PI))
        Kangle = 2 * CV_PI / dh
        Kmag = max_radius / dw
        rhos = (np.arange(dw) * Kmag).astype(_F).astype(np.float64)
        kky = Kangle * np.arange(dh)
        cp, sp = np.cos(kky)[:, None], np.sin(kky)[:, None]
        mx = (rhos[None, :] * cp + np.float64(cx)).astype(_F)
        my = (rhos[None, :] * sp + np.float64(cy)).astype(_F)
        return _remap_nearest(src, mx, my, np.zeros((dh, dw), src.dtype))
    ph, pw = src.shape[:2]
    bordered = np.concatenate([src[-1:], src, src[:1]], 0)      # copyMakeBorder(1, 1, 0, 0, BORDER_WRAP)
    Kangle = 2 * CV_PI / ph
    Kmag = max_radius / pw
    bx = (np.arange(dw, dtype=_F) - cx)[None, :].repeat(dh, 0)
    by = (np.arange(dh, dtype=_F) - cy)[:, None].repeat(dw, 1)
    mag = np.sqrt(_fma32(bx, bx, by * by)).astype(_F)           # hal::magnitude32f (v_muladd)
    ang = fast_atan_rad(by, bx)
    mx = (mag.astype(np.float64) / Kmag).astype(_F)
    my = ((ang.astype(np.float64) / Kangle).astype(_F) + _F(1)).astype(_F)
    return _remap_nearest(bordered, mx, my, np.zeros((dh, dw), src.dtype))


def circle_filled_r1(img: np.ndarray, center, color) -> np.ndarray:
    """cv2.circle(img, center, 1, color, -1): drawing.cpp Circle() with radius 1 fills the plus
    {(x-1..x+1, y), (x, y-1), (x, y+1)}, clipped to the image."""
    x, y = int(center[0]), int(center[1])
    h, w = img.shape[:2]
    if 0 <= y < h:
        img[y, max(x - 1, 0):min(x + 1, w - 1) + 1] = color
    for yy in (y - 1, y + 1):
        if 0 <= yy < h and 0 <= x < w:
            img[yy, x] = color
    return img


def _group_min(rows: np.ndarray, cols: np.ndarray):
    """npi.group_by(rows).min(cols) -> (sorted unique rows, min col per row)."""
    if rows.size == 0:
        return rows, cols
    keys = np.unique(rows)
    mins = np.full(keys.size, np.iinfo(np.int64).max)
    np.minimum.at(mins, np.searchsorted(keys, rows), cols)
    return keys, mins


def _template_cells(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m, binary):
    """The array flow of bev.py:166-212 (or :97-138 binary) up to the NN resize."""
    cell_px = cell_m * 100 / cm_per_px
    occ_w = int(grid_w_m / cell_m)
    occ_w_px = int(occ_w * cell_px)
    occ_h = int(grid_h_m / cell_m)
    occ_h_px = int(occ_h * cell_px)
    lifted = np.add(segmap, 1).astype(np.uint8)
    warped = warp_perspective(lifted, M, (after_warp_w, after_warp_h))
    left_x = int((after_warp_w - occ_w_px) / 2)
    top_y = after_warp_h - occ_h_px
    wlx = int(np.clip(left_x, 0, np.inf))
    warped = warped[int(np.clip(top_y, 0, np.inf)):after_warp_h, wlx:wlx + occ_w_px]
    glx = int(np.clip(-left_x, 0, np.inf))
    gty = int(np.clip(-top_y, 0, np.inf))
    tmpl = np.zeros((occ_h_px, occ_w_px))
    tmpl[gty:occ_h_px, glx:glx + warped.shape[1]] = warped
    tmpl = tmpl.astype(np.uint8)
    occ = ((tmpl == 1) if binary else np.logical_or(tmpl == 1, tmpl == 3)).astype(np.uint8)
    mask1 = (morph_open3x3(occ) > 0).astype(np.uint8)
    sub = np.clip(occ.astype(np.int16) - mask1, 0, 255)
    tmpl = np.where(sub > 0, 2, tmpl).astype(np.uint8)
    return resize_nearest(tmpl, (occ_w, occ_h))


def create_occupancy_grid_laserscan(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m):
    """Restates bev.py:166-246 with is_laserscan (the polar branch, bev.py:216-240)."""
    t = _template_cells(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m, False)
    shape = (t.shape[1], t.shape[0])                                                # bev.py:217
    longer = max(shape[0], shape[1])                                                # bev.py:218
    center = (shape[0] / 2 - 1, shape[1])
    polar = warp_polar(t, (-1, -1), center, longer)                                 # bev.py:219
    empty = np.zeros(polar.shape)                                                   # bev.py:224
    pts = np.where(polar == 3)                                                      # bev.py:227
    keys, mins = _group_min(pts[0], pts[1])                                         # bev.py:229
    for i, mx in enumerate(mins):                                                   # bev.py:232-233
        empty = circle_filled_r1(empty, (mx, keys[i]), 1)
    new = warp_polar(empty, shape, center, longer, inverse=True)                    # bev.py:235
    new = np.where(t != 3, t, new)                                                  # bev.py:236
    return np.where(new == 0, -1, 200 - new * 100).astype(np.int8)                  # bev.py:244


def create_occupancy_grid_binary_laserscan(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m,
                                           cell_m):
    """Restates bev.py:97-165 with is_laserscan (bev.py:143-164) -> (grid int8, new int8)."""
    t = _template_cells(segmap, M, after_warp_w, after_warp_h, cm_per_px, grid_w_m, grid_h_m, cell_m, True)
    og = (t.astype(np.int64) * 100) % 256                                           # bev.py:139-142 (uint8)
    og = ((np.where(og == 0, -1, (200 - og) % 256)) % 256).astype(np.uint8)          # bev.py:143-144
    shape = (og.shape[1], og.shape[0])                                              # bev.py:146
    longer = max(shape[0], shape[1])                                                # bev.py:147
    center = (og.shape[1] / 2 - 1, og.shape[0])
    polar = warp_polar(og, shape, center, longer)                                   # bev.py:148
    empty = np.zeros(polar.shape)                                                   # bev.py:152
    vc = np.where(polar == 100)                                                     # bev.py:154
    keys, mins = _group_min(vc[0], vc[1])                                           # bev.py:155-156
    for i, mx in enumerate(mins):                                                   # bev.py:157-158
        empty = circle_filled_r1(empty, (mx, keys[i]), 100)
    new = warp_polar(empty, shape, center, longer, inverse=True).astype(np.int8)   # bev.py:160-161
    new[og == 255] = -1                                                             # bev.py:163
    return og.astype(np.int8), new                                                  # bev.py:164
