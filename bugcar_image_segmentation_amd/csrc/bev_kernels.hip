// Fused BEV occupancy-grid rasteriser: bev_transform_tools.create_occupancy_grid, non-laserscan
// branch (bev.py:166-246), for a batch of class maps in one launch.
//
// The reference materialises segmap+1 (bev.py:177), a full warped image (bev.py:182, e.g. 1000x1000),
// a cropped/padded template (bev.py:183-195), an occupancy mask, its 3x3 opening (bev.py:196-205)
// and the INTER_NEAREST-downsampled grid (bev.py:209). Here one thread produces one output cell:
//   * the cell samples ONE template pixel p = (min(floor(cy*ify), h_px-1), min(floor(cx*ifx), w_px-1))
//     (resizeNN), so only the template values that p depends on are ever computed;
//   * template(t) = warp(t + (left_x, top_y)) when inside the warped image, else 0 — the crop/pad of
//     bev.py:183-195 is exactly this shift;
//   * warp() is cv2.warpPerspective INTER_LINEAR/BORDER_CONSTANT on segmap+1: double-precision
//     inverse mapping with OpenCV's per-32x32-block split X0 + M0*x1 (FP contraction OFF so the
//     IEEE order matches), cvRound to 1/32 pixel, Q15 bilinear weights, (sum + 2^14) >> 15;
//   * if p is occupied ({1,3}) it is a speckle unless some 3x3-neighbour q of p has an all-occupied
//     3x3 neighbourhood (erode then dilate, out-of-template taps ignored = OpenCV's default morphology
//     border): the 5x5 occupancy window around p is evaluated lazily;
//   * encode: speckle -> 2, 3 -> 1, then {0:-1, 1:100, 2:0} as int8 (bev.py:242-245), written in the
//     reference (h, w) layout or directly in the ROS data order flip(0)+rot90ccw (occgrid_to_ros.py:18-25).
// Algorithmic traffic per frame: the class map read once (in_rows*in_cols B, gathered; L2-resident)
// + occ_h*occ_w B written — latency/gather-bound, far below the HBM roof.
#include "bugseg_internal.h"

namespace bugseg {

__device__ __forceinline__ int warp_value(const BevArgs &a, const uint8_t *seg, int x, int y) {
#pragma clang fp contract(off)
    const double *M = a.Mi;
    const int xb = (x / a.bw0) * a.bw0, x1 = x - xb;
    const double X0 = M[0] * (double)xb + M[1] * (double)y + M[2];
    const double Y0 = M[3] * (double)xb + M[4] * (double)y + M[5];
    const double W0 = M[6] * (double)xb + M[7] * (double)y + M[8];
    double W = W0 + M[6] * (double)x1;
    W = W != 0.0 ? 32.0 / W : 0.0;
    double fX = (X0 + M[0] * (double)x1) * W;
    double fY = (Y0 + M[3] * (double)x1) * W;
    fX = fmin(fmax(fX, -2147483648.0), 2147483647.0);
    fY = fmin(fmax(fY, -2147483648.0), 2147483647.0);
    const int X = (int)__builtin_rint(fX), Y = (int)__builtin_rint(fY);
    int sx = X >> 5, sy = Y >> 5;
    sx = sx < -32768 ? -32768 : (sx > 32767 ? 32767 : sx);
    sy = sy < -32768 ? -32768 : (sy > 32767 ? 32767 : sy);
    const int ax = X & 31, ay = Y & 31;
    const int w = a.in_cols, h = a.in_rows;
    // segmap + 1 (bev.py:177): taps inside the image read class+1, outside the border value 0
    const bool x0 = (unsigned)sx < (unsigned)w, x1ok = (unsigned)(sx + 1) < (unsigned)w;
    const bool y0 = (unsigned)sy < (unsigned)h, y1ok = (unsigned)(sy + 1) < (unsigned)h;
    int v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    if (y0) {
        const uint8_t *r = seg + (size_t)sy * w;
        if (x0) v0 = r[sx] + 1;
        if (x1ok) v1 = r[sx + 1] + 1;
    }
    if (y1ok) {
        const uint8_t *r = seg + (size_t)(sy + 1) * w;
        if (x0) v2 = r[sx] + 1;
        if (x1ok) v3 = r[sx + 1] + 1;
    }
    const int acc = (v0 * (32 - ax) * (32 - ay) + v1 * ax * (32 - ay) + v2 * (32 - ax) * ay + v3 * ax * ay) * 32;
    int v = (acc + (1 << 14)) >> 15;
    return v > 255 ? 255 : v;
}

// template value at template pixel (tx, ty) (caller guarantees it lies inside the template)
__device__ __forceinline__ int tmpl_value(const BevArgs &a, const uint8_t *seg, int tx, int ty) {
    const int wx = tx + a.left_x, wy = ty + a.top_y;
    if ((unsigned)wx >= (unsigned)a.warp_w || (unsigned)wy >= (unsigned)a.warp_h) return 0;
    return warp_value(a, seg, wx, wy);
}

// occupied template values: {1, 3} (bev.py:196), or {1} in the binary variant (bev.py:128)
__device__ __forceinline__ bool occupied(const BevArgs &a, int v) { return v == 1 || (v == 3 && !a.variant); }

// Occupancy bit of template pixel p + (dx, dy); pixels outside the template read 1 (neutral for the
// erode: OpenCV's default erode border is +inf).
__device__ __forceinline__ uint32_t occ_bit(const BevArgs &a, const uint8_t *seg, int tx, int ty, int dx, int dy) {
    const int x = tx + dx, y = ty + dy;
    if ((unsigned)x >= (unsigned)a.occ_w_px || (unsigned)y >= (unsigned)a.occ_h_px) return 1u;
    return occupied(a, tmpl_value(a, seg, x, y)) ? 1u : 0u;
}

// bit index of offset (dx, dy) in the 5x5 window around p
#define B5(dx, dy) (((dy) + 2) * 5 + ((dx) + 2))

__global__ void __launch_bounds__(256) bev_occgrid_kernel(const BevArgs a) {
    const long cells = (long)a.occ_h * a.occ_w, total = cells * a.B;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int b = (int)(i / cells);
        const int rem = (int)(i - (long)b * cells);
        const int cy = rem / a.occ_w, cx = rem - cy * a.occ_w;
        const uint8_t *seg = a.seg + (size_t)b * a.in_rows * a.in_cols;
        int ty = (int)floor((double)cy * a.ify);
        int tx = (int)floor((double)cx * a.ifx);
        ty = ty < a.occ_h_px - 1 ? ty : a.occ_h_px - 1;
        tx = tx < a.occ_w_px - 1 ? tx : a.occ_w_px - 1;
        int v = tmpl_value(a, seg, tx, ty);
        if (occupied(a, v)) {
            // Opening at p = OR over q in N3(p) (inside the template) of AND over N3(q) of occupancy.
            // Round 1: the 8 neighbours of p (independent gathers, issued together). If they are all
            // occupied, q = p already survives the erode. Round 2 only for the rest: the 16-pixel ring.
            uint32_t m = 1u << B5(0, 0);
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx)
                    if (dx || dy) m |= occ_bit(a, seg, tx, ty, dx, dy) << B5(dx, dy);
            const uint32_t inner = 0x739C0u;        // bits of the 3x3 around p: rows 1..3, cols 1..3
            bool opened = (m & inner) == inner;
            if (!opened) {
#pragma unroll
                for (int dy = -2; dy <= 2; ++dy)
#pragma unroll
                    for (int dx = -2; dx <= 2; ++dx)
                        if (dx == -2 || dx == 2 || dy == -2 || dy == 2) m |= occ_bit(a, seg, tx, ty, dx, dy) << B5(dx, dy);
#pragma unroll
                for (int qy = -1; qy <= 1; ++qy)
#pragma unroll
                    for (int qx = -1; qx <= 1; ++qx) {
                        const bool inside = (unsigned)(tx + qx) < (unsigned)a.occ_w_px && (unsigned)(ty + qy) < (unsigned)a.occ_h_px;
                        const int sh = qy * 5 + qx;
                        const uint32_t win = sh >= 0 ? inner << sh : inner >> -sh;   // 3x3 window centred at q
                        opened |= inside && (m & win) == win;
                    }
            }
            if (!opened) v = 2;                  // isolated occupied pixel -> free (bev.py:204-205)
        }
        int8_t o;
        if (!a.variant) {
            const int g = v == 3 ? 1 : v;        // bev.py:242
            o = (int8_t)(g == 0 ? -1 : 200 - 100 * g);   // bev.py:244-245
        } else {
            // bev.py:139-144, :165 in uint8 arithmetic: {0:-1, 1:100, 2:0, 3:-100}
            const uint8_t g = (uint8_t)(v * 100);
            o = (int8_t)(uint8_t)(g == 0 ? 0xff : (uint8_t)(200 - g));
        }
        if (a.laserscan) {
            // the polar warp's source: the cells (bev.py:219) or the encoded grid (bev.py:146)
            a.cells[i] = a.variant ? (uint8_t)o : (uint8_t)v;
            if (!a.variant) continue;            // the final laserscan kernel writes out
        }
        if (a.ros_layout) {
            // occgrid_to_ros.py:18-21: flip(0) then rot90ccw == G[::-1, ::-1].T, shape (occ_w, occ_h)
            a.out[(size_t)b * cells + (size_t)(a.occ_w - 1 - cx) * a.occ_h + (a.occ_h - 1 - cy)] = o;
        } else {
            a.out[i] = o;
        }
    }
}

// ---- laserscan-like occupancy (bev.py:216-240; binary variant bev.py:143-164) ----------------------
// The reference polar-warps the grid (cv2.warpPolar, nearest), finds per polar row (ray angle) the
// nearest obstacle (np.where + npi.group_by(...).min — a Python loop over rays follows), stamps a
// radius-1 cv2.circle there and warps the stamps back. Here:
//   polar_min_kernel   one wave per (frame, ray): the ray's cells are gathered through the host-built
//                      forward table (fmap) and the nearest hit is a ballot + find-first-set per 64
//                      radii — the polar image is never materialised;
//   laserscan_kernel   one thread per output cell: the inverse table (imap) gives its (rho, ray); it is
//                      stamped iff some circle covers it — Circle() radius 1 is the plus
//                      {(r-1..r+1, ray), (r, ray-1), (r, ray+1)} — i.e. |rho - rmin[ray]| <= 1 or
//                      rmin[ray -/+ 1] == rho; then the reference's merge and encoding.
// The tables hold the float -> short rounding of remap(INTER_NEAREST) exactly as OpenCV builds them
// (cos/sin and fastAtan32f on the host, once per geometry). Traffic per frame: the grid read a few
// times (L2) + the tables (L2-resident, shared by the batch) + the grid written once.

__global__ void __launch_bounds__(256) polar_min_kernel(const BevArgs a) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long rays = (long)a.B * a.ph;
    const long cells = (long)a.occ_h * a.occ_w;
    for (long r = blockIdx.x * 4L + wave; r < rays; r += (long)gridDim.x * 4) {
        const int b = (int)(r / a.ph), phi = (int)(r - (long)b * a.ph);
        const uint8_t *g = a.cells + (size_t)b * cells;
        const int32_t *fm = a.fmap + (size_t)phi * a.pw;
        int found = -1;
        for (int r0 = 0; r0 < a.pw; r0 += 64) {
            const int rho = r0 + lane;
            bool hit = false;
            if (rho < a.pw) {
                const int32_t m = fm[rho];
                hit = m >= 0 && g[(size_t)(m >> 16) * a.occ_w + (m & 0xffff)] == a.hit;
            }
            const unsigned long long bal = __ballot(hit);
            if (bal) { found = r0 + __ffsll((long long)bal) - 1; break; }
        }
        if (lane == 0) a.rmin[r] = found;
    }
}

__global__ void __launch_bounds__(256) laserscan_kernel(const BevArgs a) {
    const long cells = (long)a.occ_h * a.occ_w, total = cells * a.B;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int b = (int)(i / cells);
        const int rem = (int)(i - (long)b * cells);
        const int cy = rem / a.occ_w, cx = rem - cy * a.occ_w;
        const int v = a.cells[i];
        int s = 0;
        if (a.variant || v == 3) {
            const int32_t m = a.imap[rem];
            if (m >= 0) {
                const int rho = m & 0xffff, row = m >> 16;
                const int32_t *rm = a.rmin + (size_t)b * a.ph;
                const int r0 = rm[row];
                s = (r0 >= 0 && abs(rho - r0) <= 1) || (row > 0 && rm[row - 1] == rho) ||
                    (row + 1 < a.ph && rm[row + 1] == rho);
            }
        }
        int8_t o;
        if (!a.variant) {
            const int g = v != 3 ? v : s;        // bev.py:236
            o = (int8_t)(g == 0 ? -1 : 200 - 100 * g);   // bev.py:244
        } else {
            o = v == 255 ? (int8_t)-1 : (int8_t)(s * 100);  // bev.py:160-163
        }
        int8_t *out = a.variant ? a.out + (size_t)a.B * cells : a.out;   // binary: the second grid
        if (a.ros_layout) out[(size_t)b * cells + (size_t)(a.occ_w - 1 - cx) * a.occ_h + (a.occ_h - 1 - cy)] = o;
        else out[i] = o;
    }
}

hipError_t launch_bev(const BevArgs &a, hipStream_t s) {
    const long total = (long)a.occ_h * a.occ_w * a.B;
    long g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(bev_occgrid_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
    if (!a.laserscan) return hipGetLastError();
    const long rays = (long)a.B * a.ph;
    long gr = (rays + 3) / 4;
    if (gr > 8192) gr = 8192;
    hipLaunchKernelGGL(polar_min_kernel, dim3((unsigned)gr), dim3(256), 0, s, a);
    hipLaunchKernelGGL(laserscan_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace bugseg
