/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the OpenCV 4.x primitives the reference's hot path calls, plus the
 * reference's occupancy-grid rasteriser built on them. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the checker / CPU
 * baseline. The product path (bugcar_image_segmentation_amd) never links or calls it.
 *
 * Parity status: UNPINNED against the real reference. OpenCV is absent from this image and
 * the reference ships no golden vectors. The semantics restated here are
 * the classic OpenCV 4.x fixed-point paths (imgwarp.cpp / resize.cpp / morph.cpp of the
 * 4.2-4.10 series, the opencv-python wheels that accompanied TF 2.2; requirements.txt:1
 * leaves opencv-python unpinned). OpenCV >= 4.11 replaced warpPerspective with a float
 * implementation and is NOT what this pins.
 *
 * Build: cc -O2 -ffp-contract=off -fPIC -shared (x86-64 SSE2 doubles, no FMA contraction),
 * so the double arithmetic is the IEEE evaluation order written below.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <limits.h>
#include <stdlib.h>

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int cv_round(double v) { return (int)lrint(v); }          /* round half to even */
static inline int sat_short(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

/* cv::invert(M, M) with the default DECOMP_LU: the closed-form 3x3 double branch of
 * lapack.cpp (det3 + cofactors * 1/det). Used by warpPerspective without WARP_INVERSE_MAP
 * (bev.py:182 passes the forward bev matrix). Returns 0 when det == 0 (OpenCV zeroes M). */
int ocv_invert3x3(const double *S, double *t)
{
#define m(i, j) S[(i) * 3 + (j)]
    double d = m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) -
               m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
               m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
    if (d == 0.0) {
        memset(t, 0, 9 * sizeof(double));
        return 0;
    }
    d = 1.0 / d;
    t[0] = (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) * d;
    t[1] = (m(0, 2) * m(2, 1) - m(0, 1) * m(2, 2)) * d;
    t[2] = (m(0, 1) * m(1, 2) - m(0, 2) * m(1, 1)) * d;
    t[3] = (m(1, 2) * m(2, 0) - m(1, 0) * m(2, 2)) * d;
    t[4] = (m(0, 0) * m(2, 2) - m(0, 2) * m(2, 0)) * d;
    t[5] = (m(0, 2) * m(1, 0) - m(0, 0) * m(1, 2)) * d;
    t[6] = (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0)) * d;
    t[7] = (m(0, 1) * m(2, 0) - m(0, 0) * m(2, 1)) * d;
    t[8] = (m(0, 0) * m(1, 1) - m(0, 1) * m(1, 0)) * d;
#undef m
    return 1;
}

/* One destination pixel of warpPerspective(INTER_LINEAR, BORDER_CONSTANT 0) on a 1-channel
 * u8 image. Mi is the INVERSE map. The x coordinate is evaluated relative to the start of
 * its 32x32-pixel-budget block (WarpPerspectiveInvoker: bh0 = min(16,H), bw0 = min(1024/bh0,W)),
 * because OpenCV forms X0 = M0*xb + M1*y + M2 once per block row and then adds M0*x1; the
 * rounding of that split is part of the result. Coordinates: saturate_cast<int>(fX*32/W)
 * (cvRound, half-even), integer part X>>5 saturated to short, 5-bit fraction indexes the
 * Q15 bilinear table; taps outside the source read the border value 0 (remapBilinear). */
static inline uint8_t warp_px(const uint8_t *src, int sh, int sw, const double *Mi, int x, int y, int bw0)
{
    int xb = (x / bw0) * bw0, x1 = x - xb;
    double X0 = Mi[0] * xb + Mi[1] * y + Mi[2];
    double Y0 = Mi[3] * xb + Mi[4] * y + Mi[5];
    double W0 = Mi[6] * xb + Mi[7] * y + Mi[8];
    double W = W0 + Mi[6] * x1;
    W = W != 0.0 ? 32.0 / W : 0.0;
    double fX = (X0 + Mi[0] * x1) * W;
    double fY = (Y0 + Mi[3] * x1) * W;
    fX = fX < (double)INT_MIN ? (double)INT_MIN : (fX > (double)INT_MAX ? (double)INT_MAX : fX);
    fY = fY < (double)INT_MIN ? (double)INT_MIN : (fY > (double)INT_MAX ? (double)INT_MAX : fY);
    int X = cv_round(fX), Y = cv_round(fY);
    int sx = sat_short(X >> 5), sy = sat_short(Y >> 5);
    int ax = X & 31, ay = Y & 31;
    int w0 = (32 - ax) * (32 - ay), w1 = ax * (32 - ay), w2 = (32 - ax) * ay, w3 = ax * ay;
    int v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    int x0ok = (unsigned)sx < (unsigned)sw, x1ok = (unsigned)(sx + 1) < (unsigned)sw;
    int y0ok = (unsigned)sy < (unsigned)sh, y1ok = (unsigned)(sy + 1) < (unsigned)sh;
    if (y0ok) {
        if (x0ok) v0 = src[(size_t)sy * sw + sx];
        if (x1ok) v1 = src[(size_t)sy * sw + sx + 1];
    }
    if (y1ok) {
        if (x0ok) v2 = src[(size_t)(sy + 1) * sw + sx];
        if (x1ok) v3 = src[(size_t)(sy + 1) * sw + sx + 1];
    }
    int acc = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3) * 32;   /* weights in Q15 sum to 32768 */
    return sat_u8((acc + (1 << 14)) >> 15);
}

static inline int warp_bw0(int dh, int dw)
{
    int bh0 = imin(16, dh);
    return imin(1024 / bh0, dw);
}

/* cv2.warpPerspective(src, M, (dw, dh)) with default flags; M is the FORWARD matrix. */
int ocv_warp_perspective_u8(const uint8_t *src, int sh, int sw, uint8_t *dst, int dh, int dw, const double *M)
{
    double Mi[9];
    ocv_invert3x3(M, Mi);
    int bw0 = warp_bw0(dh, dw);
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++)
            dst[(size_t)y * dw + x] = warp_px(src, sh, sw, Mi, x, y, bw0);
    return 0;
}

/* cv2.resize(src, (dw, dh), interpolation=INTER_NEAREST) (resizeNN): sx = min(floor(x*ifx), sw-1)
 * with ifx = 1/(dw/sw) in double. */
int ocv_resize_nearest_u8(const uint8_t *src, int sh, int sw, int cn, uint8_t *dst, int dh, int dw)
{
    double ifx = 1.0 / ((double)dw / sw), ify = 1.0 / ((double)dh / sh);
    for (int y = 0; y < dh; y++) {
        int sy = imin((int)floor(y * ify), sh - 1);
        for (int x = 0; x < dw; x++) {
            int sx = imin((int)floor(x * ifx), sw - 1);
            for (int c = 0; c < cn; c++)
                dst[((size_t)y * dw + x) * cn + c] = src[((size_t)sy * sw + sx) * cn + c];
        }
    }
    return 0;
}

/* cv2.morphologyEx(src, MORPH_OPEN, ones(3,3)): erode then dilate, each with the default
 * morphology border (+inf for erode, -inf for dilate), i.e. out-of-image taps are ignored. */
int ocv_morph_open3x3_u8(const uint8_t *src, int h, int w, uint8_t *dst)
{
    uint8_t *tmp = (uint8_t *)malloc((size_t)h * w);
    if (!tmp) return -1;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int v = 255;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int yy = y + dy, xx = x + dx;
                    if (yy >= 0 && yy < h && xx >= 0 && xx < w) v = imin(v, src[(size_t)yy * w + xx]);
                }
            tmp[(size_t)y * w + x] = (uint8_t)v;
        }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int v = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int yy = y + dy, xx = x + dx;
                    if (yy >= 0 && yy < h && xx >= 0 && xx < w) v = imax(v, tmp[(size_t)yy * w + xx]);
                }
            dst[(size_t)y * w + x] = (uint8_t)v;
        }
    free(tmp);
    return 0;
}

/* cv2.resize(src, (dw, dh)) with the default INTER_LINEAR on u8 (models.py:87), classic
 * resizeGeneric_ fixed point: per-axis float coefficients fx = (float)((d+0.5)*scale-0.5),
 * clamped at both edges, quantised to Q11 (saturate_cast<short>(c*2048)); horizontal pass
 * exact in int; vertical pass as VResizeLinearVec_32s8u (128-bit universal intrinsics):
 * ((S0>>4)*b0>>16) + ((S1>>4)*b1>>16), then (v+2)>>2 saturated — applied to every element
 * of the row except a tail of fewer than 8 elements, which takes the scalar
 * FixedPtCast<int,uchar,22> ((v + 2^21) >> 22). Exact 2x downscale is routed to INTER_AREA
 * (resize.cpp: "INTER_AREA (fast) also is equal to INTER_LINEAR"), equal size is a copy. */
static void linear_coeffs(int dsize, int ssize, double scale, int *ofs, short *a0, short *a1)
{
    for (int d = 0; d < dsize; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)floorf(f);
        f -= (float)s;
        if (s < 0) { f = 0.f; s = 0; }
        if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
        ofs[d] = s;
        a0[d] = (short)sat_short((int)lrintf((1.f - f) * 2048.f));
        a1[d] = (short)sat_short((int)lrintf(f * 2048.f));
    }
}

int ocv_resize_linear_u8(const uint8_t *src, int sh, int sw, int cn, uint8_t *dst, int dh, int dw)
{
    if (sh == dh && sw == dw) {
        memcpy(dst, src, (size_t)sh * sw * cn);
        return 0;
    }
    double inv_x = (double)dw / sw, inv_y = (double)dh / sh;
    double scale_x = 1.0 / inv_x, scale_y = 1.0 / inv_y;
    int isx = cv_round(scale_x), isy = cv_round(scale_y);
    int area_fast = fabs(scale_x - isx) < 2.220446049250313e-16 && fabs(scale_y - isy) < 2.220446049250313e-16;
    if (area_fast && isx == 2 && isy == 2) {
        for (int y = 0; y < dh; y++)
            for (int x = 0; x < dw; x++)
                for (int c = 0; c < cn; c++) {
                    const uint8_t *s = src + ((size_t)(2 * y) * sw + 2 * x) * cn + c;
                    int v = s[0] + s[cn] + s[(size_t)sw * cn] + s[(size_t)sw * cn + cn];
                    dst[((size_t)y * dw + x) * cn + c] = (uint8_t)((v + 2) >> 2);
                }
        return 0;
    }
    int *xo = (int *)malloc(sizeof(int) * dw), *yo = (int *)malloc(sizeof(int) * dh);
    short *xa0 = (short *)malloc(sizeof(short) * dw), *xa1 = (short *)malloc(sizeof(short) * dw);
    short *yb0 = (short *)malloc(sizeof(short) * dh), *yb1 = (short *)malloc(sizeof(short) * dh);
    int *r0 = (int *)malloc(sizeof(int) * dw * cn), *r1 = (int *)malloc(sizeof(int) * dw * cn);
    if (!xo || !yo || !xa0 || !xa1 || !yb0 || !yb1 || !r0 || !r1) return -1;
    linear_coeffs(dw, sw, scale_x, xo, xa0, xa1);
    linear_coeffs(dh, sh, scale_y, yo, yb0, yb1);
    int width = dw * cn, vec_end = width - (width % 8);
    for (int y = 0; y < dh; y++) {
        int sy0 = yo[y], sy1 = imin(yo[y] + 1, sh - 1);
        for (int k = 0; k < 2; k++) {
            const uint8_t *row = src + (size_t)(k ? sy1 : sy0) * sw * cn;
            int *r = k ? r1 : r0;
            for (int x = 0; x < dw; x++)
                for (int c = 0; c < cn; c++) {
                    int sx = xo[x];
                    int v = row[sx * cn + c] * xa0[x];
                    if (xa1[x]) v += row[(sx + 1) * cn + c] * xa1[x];
                    r[x * cn + c] = v;
                }
        }
        int b0 = yb0[y], b1 = yb1[y];
        uint8_t *d = dst + (size_t)y * width;
        for (int x = 0; x < width; x++) {
            if (x < vec_end) {
                int s0 = sat_short(r0[x] >> 4), s1 = sat_short(r1[x] >> 4);
                int v = ((s0 * b0) >> 16) + ((s1 * b1) >> 16);
                d[x] = sat_u8((v + 2) >> 2);
            } else {
                d[x] = sat_u8((r0[x] * b0 + r1[x] * b1 + (1 << 21)) >> 22);
            }
        }
    }
    free(xo); free(yo); free(xa0); free(xa1); free(yb0); free(yb1); free(r0); free(r1);
    return 0;
}

/* bev_transform_tools.create_occupancy_grid, non-laserscan branch (bev.py:166-246):
 *   t  = warpPerspective(segmap + 1, M, (Wb, Hb))                     bev.py:177,182
 *   template[ty][tx] = t[ty+top_y][tx+left_x] (0 outside)             bev.py:183-195
 *   occ = (template==1)|(template==3); open 3x3; template[occ&!open]=2 bev.py:196-205
 *   g = resize_nearest(template, (occ_w, occ_h))                      bev.py:209-212
 *   g = where(g==3, 1, g); out = where(g==0, -1, 200-100*g) as int8    bev.py:242-245
 * The crop/pad of bev.py:183-195 is restated as the equivalent coordinate shift.
 * segmap is (hin, win) u8 class ids {0,1,2}; M is the forward bev matrix. */
/* The template cells both rasterisers share: warp + crop/pad + opening + NN resize, before the
 * encoding. binary = 0: occupied set {1, 3} (bev.py:196-205); 1: {1} (bev.py:128). */
int bev_template_cells_ref(const uint8_t *segmap, int hin, int win, const double *M, int Wb, int Hb,
                           int occ_w_px, int occ_h_px, int occ_w, int occ_h, int left_x, int top_y, int binary,
                           uint8_t *cells)
{
    size_t n = (size_t)hin * win;
    uint8_t *lifted = (uint8_t *)malloc(n);
    uint8_t *tmpl = (uint8_t *)malloc((size_t)occ_h_px * occ_w_px);
    uint8_t *occ = (uint8_t *)malloc((size_t)occ_h_px * occ_w_px);
    uint8_t *opened = (uint8_t *)malloc((size_t)occ_h_px * occ_w_px);
    if (!lifted || !tmpl || !occ || !opened) return -1;
    for (size_t i = 0; i < n; i++) lifted[i] = (uint8_t)(segmap[i] + 1);                      /* bev.py:177 / :108 */
    double Mi[9];
    ocv_invert3x3(M, Mi);
    int bw0 = warp_bw0(Hb, Wb);
    for (int ty = 0; ty < occ_h_px; ty++)
        for (int tx = 0; tx < occ_w_px; tx++) {
            int wy = ty + top_y, wx = tx + left_x;                                                /* bev.py:183-195 */
            uint8_t v = 0;
            if (wy >= 0 && wy < Hb && wx >= 0 && wx < Wb) v = warp_px(lifted, hin, win, Mi, wx, wy, bw0);
            tmpl[(size_t)ty * occ_w_px + tx] = v;
            occ[(size_t)ty * occ_w_px + tx] = (uint8_t)(binary ? v == 1 : (v == 1 || v == 3));
        }
    ocv_morph_open3x3_u8(occ, occ_h_px, occ_w_px, opened);                                        /* bev.py:198 / :130 */
    for (size_t i = 0; i < (size_t)occ_h_px * occ_w_px; i++)
        if (occ[i] && !opened[i]) tmpl[i] = 2;
    ocv_resize_nearest_u8(tmpl, occ_h_px, occ_w_px, 1, cells, occ_h, occ_w);                      /* bev.py:209 / :139 */
    free(lifted); free(tmpl); free(occ); free(opened);
    return 0;
}

int bev_occgrid_ref(const uint8_t *segmap, int hin, int win, const double *M, int Wb, int Hb,
                    int occ_w_px, int occ_h_px, int occ_w, int occ_h, int left_x, int top_y, int8_t *out)
{
    uint8_t *cells = (uint8_t *)malloc((size_t)occ_h * occ_w);
    if (!cells) return -1;
    if (bev_template_cells_ref(segmap, hin, win, M, Wb, Hb, occ_w_px, occ_h_px, occ_w, occ_h, left_x, top_y, 0, cells))
        return -1;
    for (size_t i = 0; i < (size_t)occ_h * occ_w; i++) {
        int g = cells[i] == 3 ? 1 : cells[i];                                                     /* bev.py:242-245 */
        out[i] = (int8_t)(g == 0 ? -1 : 200 - 100 * g);
    }
    free(cells);
    return 0;
}

/* bev_transform_tools.create_occupancy_grid_binary (bev.py:97-165, non-laserscan branch; the legacy
 * variant for predict_binary maps). Same warp / crop-pad / opening / NN resize as above, but the
 * occupied set is {1} only (bev.py:128) and the encoding is the reference's uint8 arithmetic under
 * NumPy 1.x casting: g = uint8(cell * 100) (bev.py:139-142), r = g == 0 ? -1 : uint8(200 - g)
 * (bev.py:143-144), out = int8(uint8(r)) (bev.py:144, :165) -> {0:-1, 1:100, 2:0, 3:-100}. */
int bev_occgrid_binary_ref(const uint8_t *segmap, int hin, int win, const double *M, int Wb, int Hb,
                           int occ_w_px, int occ_h_px, int occ_w, int occ_h, int left_x, int top_y, int8_t *out)
{
    uint8_t *cells = (uint8_t *)malloc((size_t)occ_h * occ_w);
    if (!cells) return -1;
    if (bev_template_cells_ref(segmap, hin, win, M, Wb, Hb, occ_w_px, occ_h_px, occ_w, occ_h, left_x, top_y, 1, cells))
        return -1;
    for (size_t i = 0; i < (size_t)occ_h * occ_w; i++) {
        uint8_t g = (uint8_t)(cells[i] * 100);
        int r = g == 0 ? -1 : (int)(uint8_t)(200 - g);
        out[i] = (int8_t)(uint8_t)r;
    }
    free(cells);
    return 0;
}

/* ---- laserscan-like occupancy (bev.py:216-240; binary variant bev.py:143-164) -------------------
 *
 * cv::warpPolar(WARP_POLAR_LINEAR, INTER_NEAREST, no WARP_FILL_OUTLIERS -> BORDER_TRANSPARENT) as
 * imgwarp.cpp (4.x) builds it: float remap tables, then remap() with INTER_NEAREST, which rounds
 * each float coordinate half-to-even to a short (v_round / saturate_cast<short>) and leaves a
 * destination pixel UNTOUCHED when it maps outside the source. The reference's destinations are
 * fresh, uninitialised NumPy arrays, so those pixels are unspecified there; this restatement (and
 * the kernel) writes 0 — what fresh zeroed pages give. */

#define CV_PI 3.1415926535897932384626433832795

/* cv::hal::fastAtan32f (mathfuncs_core.simd.hpp, the AVX2 dispatch: v_fma polynomial), radians */
static const float ATAN_P1 = 0.9997878412794807f * (float)(180 / CV_PI);
static const float ATAN_P3 = -0.3258083974640975f * (float)(180 / CV_PI);
static const float ATAN_P5 = 0.1555786518463281f * (float)(180 / CV_PI);
static const float ATAN_P7 = -0.04432655554792128f * (float)(180 / CV_PI);

float ocv_fast_atan_rad(float y, float x)
{
    float ax = fabsf(x), ay = fabsf(y);
    float c = (ax < ay ? ax : ay) / ((ax > ay ? ax : ay) + (float)2.220446049250313e-16);
    float cc = c * c;
    float a = fmaf(fmaf(fmaf(cc, ATAN_P7, ATAN_P5), cc, ATAN_P3), cc, ATAN_P1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a * (float)(CV_PI / 180);
}

static inline int round_short(float v) { return sat_short((int)lrintf(v)); }

/* Forward polar table of warpPolar(src (sw x sh), dsize (pw x ph), center, maxRadius):
 * fmap[phi*pw + rho] = sx | sy << 16 (source pixel), or -1 outside the source. */
void ocv_polar_forward_map(int pw, int ph, double max_radius, float cx, float cy, int sw, int sh, int32_t *fmap)
{
    double Kangle = 2 * CV_PI / ph, Kmag = max_radius / pw;
    for (int phi = 0; phi < ph; phi++) {
        double KKy = Kangle * phi, cp = cos(KKy), sp = sin(KKy);
        for (int rho = 0; rho < pw; rho++) {
            float r = (float)(rho * Kmag);
            float mx = (float)(r * cp + cx), my = (float)(r * sp + cy);
            int sx = round_short(mx), sy = round_short(my);
            fmap[(size_t)phi * pw + rho] = ((unsigned)sx < (unsigned)sw && (unsigned)sy < (unsigned)sh) ? (sx | (sy << 16)) : -1;
        }
    }
}

/* Inverse table of warpPolar(polar (pw x ph), dsize (dw x dh), center, maxRadius, WARP_INVERSE_MAP):
 * the source is the polar image with one BORDER_WRAP row above and below; imap[y*dw + x] =
 * rho | row << 16 (row already unwrapped into 0..ph-1), or -1 when rho falls outside. */
void ocv_polar_inverse_map(int pw, int ph, double max_radius, float cx, float cy, int dw, int dh, int32_t *imap)
{
    double Kangle = 2 * CV_PI / ph, Kmag = max_radius / pw;
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            float bx = (float)x - cx, by = (float)y - cy;
            float mag = sqrtf(fmaf(bx, bx, by * by));        /* hal::magnitude32f (v_muladd) */
            float ang = ocv_fast_atan_rad(by, bx);
            double rho = mag / Kmag, phi = ang / Kangle;
            float mx = (float)rho, my = (float)phi + 1;       /* ANGLE_BORDER = 1 */
            int X = round_short(mx), Y = round_short(my);
            int32_t v = -1;
            if ((unsigned)X < (unsigned)pw && (unsigned)Y < (unsigned)(ph + 2)) {
                int row = Y == 0 ? ph - 1 : (Y == ph + 1 ? 0 : Y - 1);
                v = X | (row << 16);
            }
            imap[(size_t)y * dw + x] = v;
        }
}

/* The laserscan step on a (h x w) grid `g`: polar-warp it (fmap), take per polar row the smallest
 * rho whose value is `hit` (npi.group_by(rows).min(cols)), stamp a radius-1 filled cv2.circle there
 * (Circle(): the plus {(r-1..r+1, phi), (r, phi-1), (r, phi+1)}, clipped, no angular wrap), and
 * sample the stamps back per grid pixel (imap) -> s[y*w+x] in {0, 1}. */
static int polar_stamps(const uint8_t *g, int w, int h, int pw, int ph, const int32_t *fmap, const int32_t *imap,
                        uint8_t hit, uint8_t *s)
{
    int *rmin = (int *)malloc(sizeof(int) * ph);
    uint8_t *stamp = (uint8_t *)calloc((size_t)ph * pw, 1);
    if (!rmin || !stamp) return -1;
    for (int phi = 0; phi < ph; phi++) {
        rmin[phi] = -1;
        for (int rho = 0; rho < pw; rho++) {
            int32_t m = fmap[(size_t)phi * pw + rho];
            uint8_t v = m < 0 ? 0 : g[(size_t)(m >> 16) * w + (m & 0xffff)];
            if (v == hit) { rmin[phi] = rho; break; }
        }
    }
    for (int phi = 0; phi < ph; phi++) {
        int r = rmin[phi];
        if (r < 0) continue;
        for (int c = imax(r - 1, 0); c <= imin(r + 1, pw - 1); c++) stamp[(size_t)phi * pw + c] = 1;
        if (phi > 0) stamp[(size_t)(phi - 1) * pw + r] = 1;
        if (phi + 1 < ph) stamp[(size_t)(phi + 1) * pw + r] = 1;
    }
    for (size_t i = 0; i < (size_t)w * h; i++) {
        int32_t m = imap[i];
        s[i] = m < 0 ? 0 : stamp[(size_t)(m >> 16) * pw + (m & 0xffff)];
    }
    free(rmin); free(stamp);
    return 0;
}

/* create_occupancy_grid with is_laserscan (bev.py:166-246): the template cells of bev_occgrid_ref,
 * then warpPolar(cells, (-1,-1), (w/2-1, h), L = max(w, h)) -> (round(L), round(L*pi)) polar image;
 * obstacle value 3; new = cells != 3 ? cells : stamp; out = new == 0 ? -1 : 200 - 100*new. */
int bev_occgrid_laserscan_ref(const uint8_t *segmap, int hin, int win, const double *M, int Wb, int Hb,
                              int occ_w_px, int occ_h_px, int occ_w, int occ_h, int left_x, int top_y, int8_t *out)
{
    size_t n = (size_t)occ_h * occ_w;
    uint8_t *cells = (uint8_t *)malloc(n), *s = (uint8_t *)malloc(n);
    int L = occ_w > occ_h ? occ_w : occ_h;
    int pw = cv_round((double)L), ph = cv_round((double)L * CV_PI);
    int32_t *fmap = (int32_t *)malloc(sizeof(int32_t) * (size_t)pw * ph), *imap = (int32_t *)malloc(sizeof(int32_t) * n);
    if (!cells || !s || !fmap || !imap) return -1;
    bev_template_cells_ref(segmap, hin, win, M, Wb, Hb, occ_w_px, occ_h_px, occ_w, occ_h, left_x, top_y, 0, cells);
    float cx = (float)(occ_w / 2.0 - 1), cy = (float)occ_h;
    ocv_polar_forward_map(pw, ph, (double)L, cx, cy, occ_w, occ_h, fmap);
    ocv_polar_inverse_map(pw, ph, (double)L, cx, cy, occ_w, occ_h, imap);
    if (polar_stamps(cells, occ_w, occ_h, pw, ph, fmap, imap, 3, s)) return -1;
    for (size_t i = 0; i < n; i++) {
        int g = cells[i] != 3 ? cells[i] : s[i];
        out[i] = (int8_t)(g == 0 ? -1 : 200 - 100 * g);
    }
    free(cells); free(s); free(fmap); free(imap);
    return 0;
}

/* create_occupancy_grid_binary with is_laserscan (bev.py:143-164): the encoded binary grid G (as
 * bev_occgrid_binary_ref, kept as uint8: 255 = -1), warpPolar(G, (w, h), (w/2-1, h), L) — an
 * explicit dsize, so the polar image is w x h; obstacle value 100; stamps of 100 sampled back;
 * new = int8(stamp * 100), -1 where G == 255. Returns G in out and new in out2. */
int bev_occgrid_binary_laserscan_ref(const uint8_t *segmap, int hin, int win, const double *M, int Wb, int Hb,
                                     int occ_w_px, int occ_h_px, int occ_w, int occ_h, int left_x, int top_y,
                                     int8_t *out, int8_t *out2)
{
    size_t n = (size_t)occ_h * occ_w;
    uint8_t *s = (uint8_t *)malloc(n);
    int L = occ_w > occ_h ? occ_w : occ_h;
    int pw = occ_w, ph = occ_h;
    int32_t *fmap = (int32_t *)malloc(sizeof(int32_t) * (size_t)pw * ph), *imap = (int32_t *)malloc(sizeof(int32_t) * n);
    if (!s || !fmap || !imap) return -1;
    if (bev_occgrid_binary_ref(segmap, hin, win, M, Wb, Hb, occ_w_px, occ_h_px, occ_w, occ_h, left_x, top_y, out)) return -1;
    float cx = (float)(occ_w / 2.0 - 1), cy = (float)occ_h;
    ocv_polar_forward_map(pw, ph, (double)L, cx, cy, occ_w, occ_h, fmap);
    ocv_polar_inverse_map(pw, ph, (double)L, cx, cy, occ_w, occ_h, imap);
    if (polar_stamps((const uint8_t *)out, occ_w, occ_h, pw, ph, fmap, imap, 100, s)) return -1;
    for (size_t i = 0; i < n; i++) out2[i] = (uint8_t)out[i] == 255 ? -1 : (int8_t)(s[i] * 100);
    free(s); free(fmap); free(imap);
    return 0;
}
