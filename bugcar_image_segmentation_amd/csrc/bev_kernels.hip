// Fused BEV occupancy-grid rasteriser: bev_transform_tools.create_occupancy_grid, non-laserscan
// branch (bev.py:166-246), for a batch of class maps in one launch.
//
// The reference materialises segmap+1 (bev.py:177), a full warped image (bev.py:182, e.g. 1000x1000),
// a cropped/padded template (bev.py:183-195), an occupancy mask, its 3x3 opening (bev.py:196-205)
// and the INTER_NEAREST-downsampled grid (bev.py:209). Here one thread produces one output cell.
// The geometry (which class-map taps, with which Q15 fractions, each template pixel blends) does not
// depend on the frame: bev_table_kernel evaluates the double-precision inverse mapping ONCE per
// calibration for the 5x5 window of template pixels around every cell's sample (a [25][cells] table,
// 8 B per entry, resident across calls), and bev_occgrid_kernel does per frame only byte gathers and
// integer arithmetic:
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
// + occ_h*occ_w B written, plus the table entries a cell reads (1, 9 or 25 x 8 B, shared by every
// frame: L2 / Infinity-Cache hits) — gather-bound, far below the HBM roof.
#include <cstdlib>
#include <type_traits>

#include "bugseg_internal.h"

namespace bugseg {

// warpPerspective's source taps of warped pixel (x, y): (sy, sx) of the top-left tap, the 1/32-pixel
// fractions (ax, ay) and which of the 4 taps lie inside the image — OpenCV's arithmetic exactly:
// double-precision inverse mapping with the per-block split X0 + M0*x1 (FP contraction OFF so the IEEE
// order matches), cvRound to 1/32 pixel.
struct WarpTap { int sx, sy, ax, ay; bool x0, x1, y0, y1; };
__device__ __forceinline__ WarpTap warp_tap(const BevArgs &a, int x, int y) {
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
    WarpTap t;
    t.sx = sx; t.sy = sy; t.ax = X & 31; t.ay = Y & 31;
    const int w = a.in_cols, h = a.in_rows;
    t.x0 = (unsigned)sx < (unsigned)w; t.x1 = (unsigned)(sx + 1) < (unsigned)w;
    t.y0 = (unsigned)sy < (unsigned)h; t.y1 = (unsigned)(sy + 1) < (unsigned)h;
    return t;
}

// Table entry of a template pixel (bits of .y): 0-4 ax, 5-9 ay, 10-13 which taps (top-left,
// top-right, bottom-left, bottom-right) are inside the class map, 14 = the pixel lies outside the
// template (a neutral 1 for the erode: OpenCV's default erode border is +inf), 15-31 = the top-left
// tap's byte offset in the band's LDS box (bev_bandbox_kernel; band-staged form only). .x = the top-left tap
// (sy << 16 | sx & 0xffff, both 16-bit signed). A pixel inside the template but outside the warped
// image has no valid tap: value 0 (the crop/pad of bev.py:183-195).
constexpr uint32_t TAB_OUT = 1u << 14;
__device__ __forceinline__ uint2 tab_entry(const BevArgs &a, int tx, int ty) {
    if ((unsigned)tx >= (unsigned)a.occ_w_px || (unsigned)ty >= (unsigned)a.occ_h_px) return make_uint2(0u, TAB_OUT);
    const int wx = tx + a.left_x, wy = ty + a.top_y;   // template(t) = warp(t + (left_x, top_y))
    if ((unsigned)wx >= (unsigned)a.warp_w || (unsigned)wy >= (unsigned)a.warp_h) return make_uint2(0u, 0u);
    const WarpTap t = warp_tap(a, wx, wy);
    const uint32_t valid = (uint32_t)(t.y0 && t.x0) | (uint32_t)(t.y0 && t.x1) << 1 | (uint32_t)(t.y1 && t.x0) << 2 |
                           (uint32_t)(t.y1 && t.x1) << 3;
    return make_uint2((uint32_t)t.sy << 16 | ((uint32_t)t.sx & 0xffffu), (uint32_t)t.ax | (uint32_t)t.ay << 5 | valid << 10);
}

// template pixel sampled by cell (cx, cy): resizeNN (bev.py:209), src = min(floor(d * inv_scale), size - 1)
__device__ __forceinline__ void cell_pixel(const BevArgs &a, int cx, int cy, int &tx, int &ty) {
    ty = (int)floor((double)cy * a.ify);
    tx = (int)floor((double)cx * a.ifx);
    ty = ty < a.occ_h_px - 1 ? ty : a.occ_h_px - 1;
    tx = tx < a.occ_w_px - 1 ? tx : a.occ_w_px - 1;
}

// bit index of offset (dx, dy) in the 5x5 window around p
#define B5(dx, dy) (((dy) + 2) * 5 + ((dx) + 2))

// Table order of the window positions B5(dx, dy): the sample itself and its 3x3 first (one round of
// 5 slots serves every cell), then the 16-pixel ring (8 more slots, read only when the 3x3 does not
// settle the opening); entry i lives in slot i / 2, half i % 2.
__device__ constexpr int BEV_ORDER[BEV_WIN] = {12, 6, 7, 8, 11, 13, 16, 17, 18,
                                               0, 1, 2, 3, 4, 5, 9, 10, 14, 15, 19, 20, 21, 22, 23, 24};
__device__ __forceinline__ uint2 slot_half(const uint4 &s, int h) { return h ? make_uint2(s.z, s.w) : make_uint2(s.x, s.y); }
// BEV_ORDER as a runtime-indexed table (the band kernel's rolled ring loop); entry 25 (the padding half
// of the last slot, TAB_OUT) sets bit 25, outside the 5x5 window bits every test reads
__device__ constexpr int BEV_ORDER_D[2 * BEV_SLOTS] = {12, 6, 7, 8, 11, 13, 16, 17, 18, 0, 1, 2, 3,
                                                       4, 5, 9, 10, 14, 15, 19, 20, 21, 22, 23, 24, 25};

// One thread per (cell, table slot): the geometry-only half of the rasteriser, run once per
// calibration. Everything per frame (bev_occgrid_kernel) is then integer gathers and Q15 arithmetic.
__global__ void __launch_bounds__(256) bev_table_kernel(const BevArgs a) {
    const long cells = (long)a.occ_h * a.occ_w, total = cells * BEV_SLOTS;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int j = (int)(i / cells), c = (int)(i - (long)j * cells);
        const int cy = c / a.occ_w, cx = c - cy * a.occ_w;
        int tx, ty;
        cell_pixel(a, cx, cy, tx, ty);
        const int k0 = BEV_ORDER[2 * j];
        const uint2 e0 = tab_entry(a, tx + k0 % 5 - 2, ty + k0 / 5 - 2);
        uint2 e1 = make_uint2(0u, TAB_OUT);
        if (2 * j + 1 < BEV_WIN) {
            const int k1 = BEV_ORDER[2 * j + 1];
            e1 = tab_entry(a, tx + k1 % 5 - 2, ty + k1 / 5 - 2);
        }
        a.wtab[i] = make_uint4(e0.x, e0.y, e1.x, e1.y);
    }
}

// the top-left tap of a table entry (.x = sy << 16 | sx & 0xffff)
__device__ __forceinline__ int tap_sy(uint2 e) { return (int)e.x >> 16; }
__device__ __forceinline__ int tap_sx(uint2 e) { return (int)(short)(e.x & 0xffffu); }

typedef unsigned short bev_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot2(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(bev_u16x2, a), __builtin_bit_cast(bev_u16x2, b), c, false);
}
// labels (segmap + 1, uint8 wrap-around as np.add on uint8) of the 4 taps, 0 outside the class map,
// blended in Q15 with three v_dot2_u32_u16: (32 - ax) | ax << 16 weights each row pair, then the rows.
// Each tap row is ONE 2-byte load (byte-aligned: gfx950 buffer loads need no alignment) of the pair
// (sx, sx + 1), shifted by one byte where one of the two lies outside the class map, so the load never
// leaves the tap's image row.
__device__ __forceinline__ uint32_t tap_pair(__amdgpu_buffer_rsrc_t seg, uint32_t b, bool v0, bool v1) {
    const uint32_t off = v0 ? (v1 ? b : b - 1) : (v1 ? b + 1 : 0x80000000u);
    const uint32_t r = __builtin_amdgcn_raw_buffer_load_b16(seg, (int)off, 0, 0);
    const uint32_t lo = v0 ? (((v1 ? r : r >> 8) + 1) & 255u) : 0u;              // byte sx  (+1)
    const uint32_t hi = v1 ? ((((v0 ? r >> 8 : r) & 255u) + 1) & 255u) : 0u;     // byte sx+1 (+1)
    return lo | hi << 16;
}
__device__ __forceinline__ int tab_value(__amdgpu_buffer_rsrc_t seg, int w, uint2 e) {
    const uint32_t m = e.y;
    const uint32_t b = (uint32_t)(__mul24(tap_sy(e), w) + tap_sx(e));
    const uint32_t t0 = tap_pair(seg, b, m & (1u << 10), m & (1u << 11));
    const uint32_t t1 = tap_pair(seg, b + w, m & (1u << 12), m & (1u << 13));
    const uint32_t ax = m & 31u, ay = (m >> 5) & 31u;
    const uint32_t wx = 32u + ax * 65535u, wy = 32u + ay * 65535u;
    const uint32_t top = dot2(t0, wx, 0u), bot = dot2(t1, wx, 0u);
    return (int)(dot2(top | bot << 16, wy, 512u) >> 10);
}

// occupied template values: {1, 3} (bev.py:196), or {1} in the binary variant (bev.py:128)
__device__ __forceinline__ bool occupied(const BevArgs &a, int v) {
    return (v == 1) | ((v == 3) & !a.variant);      // bitwise: no divergent branch per tap
}

// F frames per thread (the cell's table entries are loaded once and serve all F), the 3x3 around the
// sample evaluated eagerly (one round of 36 gathers per frame instead of a dependent centre-then-
// neighbours chain); the 16-pixel ring only for the frames whose 3x3 does not settle the opening.
// encode template value v of cell (cx, cy) of frame b and store it (or, in the laserscan mode, the
// polar warp's source)
__device__ __forceinline__ void bev_emit(const BevArgs &a, int b, int rem, int cx, int cy, long cells, int v) {
#ifdef BEV_ABL
    if constexpr (BEV_ABL & 2) { if (v == 12345) a.out[0] = 0; return; }
#endif
    const long o_i = (long)b * cells + rem;
    int8_t o;
    if (!a.variant) {
        const int gg = v == 3 ? 1 : v;               // bev.py:242
        o = (int8_t)(gg == 0 ? -1 : 200 - 100 * gg);   // bev.py:244-245
    } else {
        // bev.py:139-144, :165 in uint8 arithmetic: {0:-1, 1:100, 2:0, 3:-100}
        const uint8_t gg = (uint8_t)(v * 100);
        o = (int8_t)(uint8_t)(gg == 0 ? 0xff : (uint8_t)(200 - gg));
    }
    if (a.laserscan) {
        // the polar warp's source: the cells (bev.py:219) or the encoded grid (bev.py:146)
        a.cells[o_i] = a.variant ? (uint8_t)o : (uint8_t)v;
        if (!a.variant) return;                      // the final laserscan kernel writes out
    }
    if (a.ros_layout) {
        // occgrid_to_ros.py:18-21: flip(0) then rot90ccw == G[::-1, ::-1].T, shape (occ_w, occ_h)
        a.out[(size_t)b * cells + (size_t)(a.occ_w - 1 - cx) * a.occ_h + (a.occ_h - 1 - cy)] = o;
    } else {
        a.out[o_i] = o;
    }
}

// XCD-aware work split: the grid is a multiple of 8 and the blocks b with b % 8 == x (one XCD under
// round-robin dispatch; speed only, never correctness) take grid rows [x*rows, (x+1)*rows) of every
// frame. A band of grid rows is a band of distances, i.e. a band of class-map rows, so each XCD's L2
// holds 1/8 of the tap table and 1/8 of every class map instead of all of both.
template <int F>
__global__ void __launch_bounds__(256) bev_occgrid_kernel(const BevArgs a) {
    const long cells = (long)a.occ_h * a.occ_w;
    const int groups = (a.B + F - 1) / F;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
    const int rows = (a.occ_h + 7) >> 3, r0 = min(a.occ_h, xcd * rows), r1 = min(a.occ_h, r0 + rows);
    const long band = (long)(r1 - r0) * a.occ_w;
    const long total = band * groups;
    const uint32_t frame_bytes = (uint32_t)a.in_rows * (uint32_t)a.in_cols;
    for (long j = slot * 256L + threadIdx.x; j < total; j += (long)nslot * 256) {
        const int g = (int)(j / band);
        const int rem = (int)((long)r0 * a.occ_w + (j - (long)g * band));
        const int cy = rem / a.occ_w, cx = rem - cy * a.occ_w;
        const uint4 *tab = a.wtab + rem;
        // table entries 0..8: the sample and its 3x3 (slots 0..4; slot 4's second half is ring entry 9)
        uint4 s3[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) s3[q] = tab[(long)q * cells];
        __amdgpu_buffer_rsrc_t seg[F];
#pragma unroll
        for (int f = 0; f < F; ++f) {
            // a frame past the batch gets an empty descriptor: its loads read 0, its result is dropped
            const int b = g * F + f;
            seg[f] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.seg) + (size_t)(b < a.B ? b : 0) * frame_bytes,
                                                       (short)0, b < a.B ? (int)frame_bytes : 0, 0x00020000);
        }
        uint32_t m[F];
        int v[F];
#pragma unroll
        for (int f = 0; f < F; ++f) {
            m[f] = 0;
#pragma unroll
            for (int i = 0; i < 9; ++i) {
                const uint2 e = slot_half(s3[i >> 1], i & 1);
                const int t = tab_value(seg[f], a.in_cols, e);
                if (i == 0) v[f] = t;
                // outside the template: 1 (neutral for the erode: OpenCV's default erode border is +inf)
                const bool o = (e.y & TAB_OUT) || occupied(a, t);
                m[f] |= (uint32_t)o << BEV_ORDER[i];
            }
        }
        const uint32_t inner = 0x739C0u;            // bits of the 3x3 around p: rows 1..3, cols 1..3
        bool need_ring = false;
#pragma unroll
        for (int f = 0; f < F; ++f) need_ring |= occupied(a, v[f]) && (m[f] & inner) != inner;
        if (need_ring) {
            // Opening at p = OR over q in N3(p) (inside the template) of AND over N3(q) of occupancy:
            // the ring completes the 5x5 window for the frames whose centre is occupied but whose 3x3
            // is not (if it is, q = p already survives the erode)
            int tx, ty;
            cell_pixel(a, cx, cy, tx, ty);
            uint4 sr[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) sr[q] = tab[(long)(q + 5) * cells];
#pragma unroll
            for (int f = 0; f < F; ++f) {
                if (!(occupied(a, v[f]) && (m[f] & inner) != inner)) continue;
#pragma unroll
                for (int i = 9; i < BEV_WIN; ++i) {
                    const uint2 e = i == 9 ? slot_half(s3[4], 1) : slot_half(sr[(i >> 1) - 5], i & 1);
                    const bool o = (e.y & TAB_OUT) || occupied(a, tab_value(seg[f], a.in_cols, e));
                    m[f] |= (uint32_t)o << BEV_ORDER[i];
                }
                bool opened = false;
#pragma unroll
                for (int qy = -1; qy <= 1; ++qy)
#pragma unroll
                    for (int qx = -1; qx <= 1; ++qx) {
                        const bool inside = (unsigned)(tx + qx) < (unsigned)a.occ_w_px && (unsigned)(ty + qy) < (unsigned)a.occ_h_px;
                        const int sh = qy * 5 + qx;
                        const uint32_t win = sh >= 0 ? inner << sh : inner >> -sh;   // 3x3 window centred at q
                        opened |= inside && (m[f] & win) == win;
                    }
                if (!opened) v[f] = 2;           // isolated occupied pixel -> free (bev.py:204-205)
            }
        }
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const int b = g * F + f;
            if (b >= a.B) break;
            bev_emit(a, b, rem, cx, cy, cells, v[f]);
        }
    }
}

// ---- LDS-staged form (the default when in_cols % 16 == 0): a workgroup owns a 16 x 16 block of
// cells and a group of frames. The taps of every template pixel its cells need fall in one box of the
// class map (fixed by the geometry; found once per workgroup from the table). Each frame's box is read
// once with coalesced 16-B loads into LDS as segmap + 1 (bev.py:177, uint8 wrap-around), with a
// border of zeros where the box leaves the image — exactly warpPerspective's BORDER_CONSTANT taps — so
// every one of a cell's 25 x 4 taps is an unmasked LDS byte read and the Q15 blend is three
// v_dot2_u32_u16; the next frame's box is in flight in registers while the current one is evaluated.
// A block whose box exceeds BEV_BOX_CAP (or has no valid tap) gathers from global memory instead, with
// the same arithmetic.
constexpr int BEV_CB = 16, BEV_BOX_CAP = 32768, BEV_PF = BEV_BOX_CAP / 16 / 256;   // 16-B chunks per thread
// per-byte x + 1 mod 256 of 4 packed bytes (no carry between bytes)
__device__ __forceinline__ uint32_t inc4(uint32_t v) { return ((v & 0x7f7f7f7fu) + 0x01010101u) ^ (v & 0x80808080u); }

__global__ void __launch_bounds__(256, 4) bev_occgrid_lds_kernel(const BevArgs a, int fg) {
    __shared__ __attribute__((aligned(16))) uint8_t box[BEV_BOX_CAP];
    __shared__ int red[4];
    const int tid = threadIdx.x;
    const long cells = (long)a.occ_h * a.occ_w;
    const int nbx = (a.occ_w + BEV_CB - 1) / BEV_CB, nby = (a.occ_h + BEV_CB - 1) / BEV_CB, nblk = nbx * nby;
    const int blk = blockIdx.x % nblk, grp = blockIdx.x / nblk;
    const int cx = (blk % nbx) * BEV_CB + (tid & 15), cy = (blk / nbx) * BEV_CB + (tid >> 4);
    const bool cell_ok = cx < a.occ_w && cy < a.occ_h;
    const int rem = cell_ok ? cy * a.occ_w + cx : 0;
    const uint4 *tab = a.wtab + rem;
    auto ent = [&](int i) { return slot_half(tab[(long)(i >> 1) * cells], i & 1); };   // table entry i
    // the class-map box of every valid tap of the block: rows [ylo, yhi], columns [xlo, xhi]
    int ylo = 1 << 30, yhi = -(1 << 30), xlo = 1 << 30, xhi = -(1 << 30);
    uint32_t outm = 0;                              // window positions outside the template
    if (cell_ok) {
#pragma unroll
        for (int k = 0; k < BEV_WIN; ++k) {
            const uint2 e = ent(k);
            const uint32_t v = (e.y >> 10) & 15;
            const int sy = tap_sy(e), sx = tap_sx(e);
            if (v & 3) { ylo = min(ylo, sy); yhi = max(yhi, sy); }
            if (v & 12) { ylo = min(ylo, sy + 1); yhi = max(yhi, sy + 1); }
            if (v & 5) { xlo = min(xlo, sx); xhi = max(xhi, sx); }
            if (v & 10) { xlo = min(xlo, sx + 1); xhi = max(xhi, sx + 1); }
            outm |= (uint32_t)((e.y & TAB_OUT) != 0) << BEV_ORDER[k];
        }
    } else {
        outm = (1u << BEV_WIN) - 1;
    }
    if (tid < 4) red[tid] = tid & 1 ? -(1 << 30) : (1 << 30);
    __syncthreads();
    atomicMin(&red[0], ylo); atomicMax(&red[1], yhi); atomicMin(&red[2], xlo); atomicMax(&red[3], xhi);
    __syncthreads();
    // the box with a one-pixel border: rows [ylo - 1, yhi + 1], columns [xa, xb) in whole 16-B chunks,
    // then a 16-B-aligned zero pad that tap-less template pixels read
    const int y0 = red[0] - 1, bh = red[1] - red[0] + 3;
    const int xa = (red[2] - 1) & ~15, bw = ((red[3] + 17) & ~15) - xa;
    const int zpad = bh * bw;
    const bool lds = red[1] >= red[0] && (long)bh * bw + 2 * bw + 16 <= BEV_BOX_CAP;   // workgroup-uniform
    const int cpr = lds ? bw >> 4 : 1, nch = lds ? bh * cpr : 0;          // 16-B chunks per row / in all
    const uint32_t frame_bytes = (uint32_t)a.in_rows * (uint32_t)a.in_cols;
    // this thread's chunks q = tid + 256 i of the box: LDS offset 16 q (rows of bw bytes), global
    // offset, or OOB where the chunk lies outside the image (whole chunks: in_cols % 16 == 0)
    uint32_t goff[BEV_PF];
#pragma unroll
    for (int i = 0; i < BEV_PF; ++i) {
        const int q = tid + 256 * i;
        const int r = q / cpr, c = q - r * cpr;
        const int gy = y0 + r, gx = xa + c * 16;
        const bool in = q < nch && (unsigned)gy < (unsigned)a.in_rows && (unsigned)gx < (unsigned)a.in_cols;
        goff[i] = in ? (uint32_t)(gy * a.in_cols + gx) : 0x80000000u;
    }
    // per window position ONE register: the top-left tap's offset in the box (16 bits) | ax << 16 |
    // ay << 21; a template pixel with no tap inside the class map reads the zero pad
    uint32_t ek[BEV_WIN];
    if (lds) {
#pragma unroll
        for (int k = 0; k < BEV_WIN; ++k) {
            const uint2 e = cell_ok ? ent(k) : make_uint2(0u, TAB_OUT);
            const bool any = ((e.y >> 10) & 15) != 0;
            const int o = any ? (tap_sy(e) - y0) * bw + (tap_sx(e) - xa) : zpad;
            ek[k] = (uint32_t)o | (e.y & 1023u) << 16;
        }
    }
    auto frame_rsrc = [&](int b) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.seg) + (size_t)(b < a.B ? b : 0) * frame_bytes,
                                                 (short)0, b < a.B ? (int)frame_bytes : 0, 0x00020000);
    };
    uint4 pf[BEV_PF];
    auto fetch = [&](int b) {
        const auto r = frame_rsrc(b);
#pragma unroll
        for (int i = 0; i < BEV_PF; ++i) pf[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)goff[i], 0, 0));
    };
    const int b0 = grp * fg;
    if (lds) {
        fetch(b0);
        for (int i = tid; i < 2 * bw + 16; i += 256) box[zpad + i] = 0;
    }
    const uint32_t inner = 0x739C0u;                // bits of the 3x3 around p: rows 1..3, cols 1..3
    int tx = 0, ty = 0;
    cell_pixel(a, cx, cy, tx, ty);
    // windows of the 9 q in N3(p) that lie inside the template
    uint32_t wins[9];
#pragma unroll
    for (int qy = -1; qy <= 1; ++qy)
#pragma unroll
        for (int qx = -1; qx <= 1; ++qx) {
            const bool inside = (unsigned)(tx + qx) < (unsigned)a.occ_w_px && (unsigned)(ty + qy) < (unsigned)a.occ_h_px;
            const int sh = qy * 5 + qx;
            wins[(qy + 1) * 3 + qx + 1] = inside ? (sh >= 0 ? inner << sh : inner >> -sh) : 0xffffffffu;
        }
    for (int fi = 0; fi < fg; ++fi) {
        const int b = b0 + fi;
        if (b >= a.B) break;                        // workgroup-uniform
        uint32_t msk = 0;
        int v = 0;
        if (lds) {
            __syncthreads();                        // the previous frame's reads of the box are done
#pragma unroll
            for (int i = 0; i < BEV_PF; ++i)
                if (tid + 256 * i < nch)
                    *reinterpret_cast<uint4 *>(box + 16 * (tid + 256 * i)) =
                        goff[i] == 0x80000000u ? make_uint4(0u, 0u, 0u, 0u)
                                               : make_uint4(inc4(pf[i].x), inc4(pf[i].y), inc4(pf[i].z), inc4(pf[i].w));
            __syncthreads();
            if (fi + 1 < fg && b + 1 < a.B) fetch(b + 1);   // next frame's box flies during this frame
#pragma unroll 5
            for (int k = 0; k < BEV_WIN; ++k) {
                const uint32_t e = ek[k];
                const uint8_t *p = box + (e & 0xffffu);
                const uint32_t l0 = p[0], l1 = p[1], l2 = p[bw], l3 = p[bw + 1];
                const uint32_t ax = (e >> 16) & 31u, ay = (e >> 21) & 31u;
                const uint32_t wx = 32u + ax * 65535u, wy = 32u + ay * 65535u;   // (32 - a) | a << 16
                const uint32_t top = dot2(l0 | l1 << 16, wx, 0u), bot = dot2(l2 | l3 << 16, wx, 0u);
                const int t = (int)(dot2(top | bot << 16, wy, 512u) >> 10);      // (sum + 2^14) >> 15 of OpenCV
                if (k == 0) v = t;
                msk |= (uint32_t)occupied(a, t) << BEV_ORDER[k];
            }
        } else {
            const auto seg = frame_rsrc(b);
#pragma unroll 1
            for (int k = 0; k < BEV_WIN; ++k) {
                const uint2 e = cell_ok ? ent(k) : make_uint2(0u, TAB_OUT);
                const int t = tab_value(seg, a.in_cols, e);
                if (k == 0) v = t;
                msk |= (uint32_t)occupied(a, t) << BEV_ORDER[k];
            }
        }
        if (!cell_ok) continue;
        msk |= outm;                                // outside the template: the erode's +inf border
        if (occupied(a, v)) {
            // opening at p = OR over q in N3(p) (inside the template) of AND over N3(q) of occupancy
            bool opened = false;
#pragma unroll
            for (int q = 0; q < 9; ++q) opened |= (msk & wins[q]) == wins[q];
            if (!opened) v = 2;                     // isolated occupied pixel -> free (bev.py:204-205)
        }
        bev_emit(a, b, rem, cx, cy, cells, v);
    }
}

// ---- band-staged form (the default when in_cols % 16 == 0): a workgroup owns one frame and a band of
// BEV_BAND grid rows (all columns). A band of grid rows is a band of distances, so every tap its cells
// read lies in one class-map box that is a few rows deep and at most the image wide; the box is a
// property of the geometry (bev_bandbox_kernel, once per calibration, stored after the tap table).
// The box is read with coalesced 16-B loads into LDS as segmap + 1 (bev.py:177, uint8 wrap-around),
// with zeros where it leaves the image — exactly warpPerspective's BORDER_CONSTANT taps — and then
// every tap of the band's cells is an unmasked LDS byte read: no gathers from global memory. Bands
// whose box exceeds BEV_BAND_CAP gather from global memory (same arithmetic). XCD-aware: XCD x takes
// bands x, x + 8, ... of every frame, so each XCD's L2 holds only its bands' share of the tap table.
// 4 grid rows: ~1,600 workgroups at 32 frames, all resident at once (16 KB of LDS each); 8 rows (40 KB,
// 3 per CU) left a second round of workgroups: 58.5 vs 62 us for the gather kernel
constexpr int BEV_BAND_CAP = 16384, BEV_BAND_PF = BEV_BAND_CAP / 16 / 256;
// per band BEV_BOXREC int4 records: (P, rows per part, 0, 0), then the box of each of its P row parts.
// A band whose box would exceed BEV_BAND_CAP is split into 2 or 4 row parts (the nearest bands of a
// forward camera span many image rows), each staged and evaluated in turn by the same workgroup;
// only a part whose single-row box still exceeds the cap gathers from global memory.
static_assert(BEV_BOXREC == 1 + BEV_BAND, "band record: header + one box per row part");
#ifndef BEV_MINP
#define BEV_MINP 1                                   // fewest row parts per band (A/B knob: 1, 2, 4)
#endif
constexpr int BEV_WL = 448;                          // band kernel: ring work-list records per workgroup (LDS: 8 per CU)
static_assert(BEV_WL <= 2 * 256, "a thread takes at most two work-list records");
// The band kernel's compact table, after the band boxes: [BEV_WIN][cells] u32, entry i of every cell
// (BEV_ORDER_D order: the sample, its 3x3, then the ring) as the .y word alone — the tap's byte offset
// in the band's LDS box, the fractions, the valid-tap and outside-template bits: what the LDS form
// reads (4 B per entry instead of 8; no slot halves to pick). Filled by bev_bandbox_kernel for the
// bands that stage their box.
// (bev_ctab_offset: bugseg_internal.h)

// per band: the class-map box (y0, xa, bh, bw) every valid tap of its cells reads, with a one-pixel
// border, xa and bw whole 16-B chunks; bh = 0: no valid tap (every pixel reads the zero pad);
// bh = -1: the box (+ its zero pad) exceeds BEV_BAND_CAP
__global__ void __launch_bounds__(256) bev_bandbox_kernel(const BevArgs a, int4 *bbox) {
    __shared__ int red[BEV_BAND][4];
    __shared__ int4 pbox[BEV_BAND];
    __shared__ int np_rpp[2];
    const long cells = (long)a.occ_h * a.occ_w;
    const int band = blockIdx.x, r0 = band * BEV_BAND, r1 = min(a.occ_h, r0 + BEV_BAND);
    const int nr = r1 - r0, n = nr * a.occ_w;
    // per band row: the extent of every valid tap of its cells
    int ylo[BEV_BAND], yhi[BEV_BAND], xlo[BEV_BAND], xhi[BEV_BAND];
#pragma unroll
    for (int k = 0; k < BEV_BAND; ++k) { ylo[k] = xlo[k] = 1 << 30; yhi[k] = xhi[k] = -(1 << 30); }
    for (int i = threadIdx.x; i < n * BEV_WIN; i += 256) {
        const int c = i / BEV_WIN, k = i - c * BEV_WIN, ri = c / a.occ_w;
        const long rem = (long)r0 * a.occ_w + c;
        const uint2 e = slot_half(a.wtab[(long)(k >> 1) * cells + rem], k & 1);
        const uint32_t v = (e.y >> 10) & 15;
        const int sy = tap_sy(e), sx = tap_sx(e);
        int y_lo = 1 << 30, y_hi = -(1 << 30), x_lo = 1 << 30, x_hi = -(1 << 30);
        if (v & 3) { y_lo = min(y_lo, sy); y_hi = max(y_hi, sy); }
        if (v & 12) { y_lo = min(y_lo, sy + 1); y_hi = max(y_hi, sy + 1); }
        if (v & 5) { x_lo = min(x_lo, sx); x_hi = max(x_hi, sx); }
        if (v & 10) { x_lo = min(x_lo, sx + 1); x_hi = max(x_hi, sx + 1); }
#pragma unroll
        for (int q = 0; q < BEV_BAND; ++q)
            if (q == ri) { ylo[q] = min(ylo[q], y_lo); yhi[q] = max(yhi[q], y_hi); xlo[q] = min(xlo[q], x_lo); xhi[q] = max(xhi[q], x_hi); }
    }
    if (threadIdx.x < 4 * BEV_BAND) red[threadIdx.x >> 2][threadIdx.x & 3] = threadIdx.x & 1 ? -(1 << 30) : (1 << 30);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BEV_BAND; ++q) {
        atomicMin(&red[q][0], ylo[q]); atomicMax(&red[q][1], yhi[q]); atomicMin(&red[q][2], xlo[q]); atomicMax(&red[q][3], xhi[q]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // the box of rows [q0, q1) of the band: (y0, xa, bh, bw), bh = 0: no valid tap, -1: over the cap
        auto boxof = [&](int q0, int q1) {
            int yl = 1 << 30, yh = -(1 << 30), xl = 1 << 30, xh = -(1 << 30);
            for (int q = q0; q < q1 && q < nr; ++q) {
                yl = min(yl, red[q][0]); yh = max(yh, red[q][1]); xl = min(xl, red[q][2]); xh = max(xh, red[q][3]);
            }
            int4 bx = make_int4(0, 0, 0, 16);
            if (yh >= yl) {
                const int y0 = yl - 1, bh = yh - yl + 3;
                const int xa = (xl - 1) & ~15, bw = ((xh + 17) & ~15) - xa;
                bx = make_int4(y0, xa, (long)bh * bw + 2 * bw + 16 <= BEV_BAND_CAP ? bh : -1, bw);
            }
            return bx;
        };
        int P = BEV_MINP;
        for (; P < BEV_BAND; P *= 2) {                 // fewest row parts whose boxes all fit
            bool fit = true;
            for (int k = 0; k < P; ++k) fit = fit && boxof(k * (BEV_BAND / P), (k + 1) * (BEV_BAND / P)).z >= 0;
            if (fit) break;
        }
        int rpp = BEV_BAND / P;
        for (int k = 0; k < BEV_BAND; ++k) pbox[k] = k < P ? boxof(k * rpp, (k + 1) * rpp) : make_int4(0, 0, 0, 16);
        bool fit = true;
        for (int k = 0; k < P; ++k) fit = fit && pbox[k].z >= 0;
        if (!fit) {                                    // even one row is over the cap: the whole band gathers
            P = 1; rpp = BEV_BAND;
            pbox[0] = boxof(0, BEV_BAND);
            pbox[0].z = -1;
        }
        np_rpp[0] = P; np_rpp[1] = rpp;
        bbox[(size_t)band * BEV_BOXREC] = make_int4(P, rpp, 0, 0);
        for (int k = 0; k < BEV_BAND; ++k) bbox[(size_t)band * BEV_BOXREC + 1 + k] = pbox[k];
    }
    __syncthreads();
    const int rpp = np_rpp[1];
    // each entry's top-left tap as a byte offset in the band's LDS box, in the entry's free bits 15..31
    // (a template pixel without a valid tap: the zero pad after the box); the .y words also go to the
    // compact table (bev_ctab_offset)
    uint32_t *ctab = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(a.wtab) + bev_ctab_offset(a.occ_w, a.occ_h));
    for (int i = threadIdx.x; i < n * BEV_SLOTS; i += 256) {
        const int c = i / BEV_SLOTS, q = i - c * BEV_SLOTS;
        const int4 bx = pbox[(c / a.occ_w) / rpp];     // this cell's row part
        if (bx.z < 0) continue;                        // (an oversized part gathers from global memory)
        const long rem = (long)r0 * a.occ_w + c;
        uint4 *sp = a.wtab + (long)q * cells + rem;
        uint4 sv = *sp;
        auto put = [&](uint32_t x, uint32_t &y) {
            const uint2 e = make_uint2(x, y);
            const bool any = ((y >> 10) & 15) != 0;
            const int o = any ? (tap_sy(e) - bx.x) * bx.w + (tap_sx(e) - bx.y) : bx.z * bx.w;
            y = (y & 0x7fffu) | (uint32_t)o << 15;
        };
        put(sv.x, sv.y);
        put(sv.z, sv.w);
        *sp = sv;
        ctab[(long)(2 * q) * cells + rem] = sv.y;
        if (2 * q + 1 < BEV_WIN) ctab[(long)(2 * q + 1) * cells + rem] = sv.w;
    }
    // per cell: which of the 25 window positions lie outside the template (bit B5(dx, dy)), a geometry
    // fact the band kernel would otherwise re-derive from 9-25 entries (and the cell's pixel) per frame
    __syncthreads();
    uint32_t *omask = ctab + (size_t)BEV_WIN * cells;
    for (int c = threadIdx.x; c < n; c += 256) {
        if (pbox[(c / a.occ_w) / rpp].z < 0) continue;
        const long rem = (long)r0 * a.occ_w + c;
        uint32_t m = 0;
        for (int k = 0; k < BEV_WIN; ++k)
            m |= (uint32_t)((ctab[(long)k * cells + rem] & TAB_OUT) != 0) << BEV_ORDER[k];
        omask[rem] = m;
    }
}

// FB frames per workgroup (one box each): a cell's table slots and entry decoding serve all FB frames.
// Held to 8 waves per SIMD (FB = 1: 64 VGPRs, no spills; LDS 19.97 KB with a 448-record work list)
// so the 58 work items x 32 frames of a bench call (1,856 workgroups; the near bands' row parts add
// 8 items to the 50 bands) are one round of 2,048 slots — at 7 per CU, 64 of them took a second round.
// One cell of one frame from a band's LDS box (bev_band_kernel's compact-table form and
// bev_pipe_kernel): e9 = the cell's sample + 3x3 entries (offset in the box, Q5 fractions; BEV_ORDER),
// outm = its 25-bit outside-template mask, ring = its 16 ring entries (stride `cells`), read only when
// the opening needs them. Returns the template value after the speckle opening (bev.py:196-205).
// BEV_ABL (debug ablation builds, wrong grids; scripts/gpu_r4_abl.sh): 1 = no ring pass, 4 = no template
// values (the sample's entry bits stand in), 2 = no output stores (bev_emit), 8 = no box staging,
// 16 = no compact-table loads (the cell index stands in), 32 = every workgroup leaves at once
#ifndef BEV_ABL
#define BEV_ABL 0
#endif
__device__ __forceinline__ int bev_value_lds(const uint8_t *box, int bw, uint32_t ey) {
    const uint8_t *p = box + (ey >> 15);
    const uint32_t l0 = p[0], l1 = p[1], l2 = p[bw], l3 = p[bw + 1];
    const uint32_t ax = ey & 31u, ay = (ey >> 5) & 31u;
    const uint32_t wx = 32u + ax * 65535u, wy = 32u + ay * 65535u;   // (32 - a) | a << 16
    const uint32_t top = dot2(l0 | l1 << 16, wx, 0u), bot = dot2(l2 | l3 << 16, wx, 0u);
    return (int)(dot2(top | bot << 16, wy, 512u) >> 10);              // (sum + 2^14) >> 15 of OpenCV
}
constexpr uint32_t BEV_INNER = 0x739C0u;          // bits of the 3x3 around p: rows 1..3, cols 1..3
// First pass of a cell: v = the sample's template value, m = occupancy of the 3x3 (outside-template
// positions of the whole 5x5 counted occupied), and — when the opening is undecided by the 3x3 —
// cand = the neighbours q of p whose part of N3(q) inside the 3x3 is all occupied. Returns true when v
// is final (not occupied, the 3x3 all occupied, or no candidate: then v is already the speckle's 2).
// Opening at p (bev.py:196-205) = OR over the q in N3(p) inside the template of AND over N3(q); the
// centre fails whenever the 3x3 is not all occupied, so only the 8 neighbours can open p.
__device__ __forceinline__ bool bev_cell_pass1(const BevArgs &a, const uint8_t *box, int bw, const uint32_t (&e9)[9],
                                               uint32_t outm, int &v, uint32_t &m, uint32_t &cand) {
    int t9[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) t9[i] = bev_value_lds(box, bw, e9[i]);
    v = t9[0];
    m = outm;
#pragma unroll
    for (int i = 0; i < 9; ++i) m |= (uint32_t)occupied(a, t9[i]) << BEV_ORDER[i];
    cand = 0;
    if (!(occupied(a, v) && (m & BEV_INNER) != BEV_INNER)) return true;
#pragma unroll
    for (int qi = 0; qi < 9; ++qi) {
        if (qi == 4) continue;
        const int qx = qi % 3 - 1, qy = qi / 3 - 1, sh = qy * 5 + qx;
        const uint32_t win = sh >= 0 ? BEV_INNER << sh : BEV_INNER >> -sh, wi = win & BEV_INNER;
        cand |= (!((outm >> B5(qx, qy)) & 1u) && (m & wi) == wi) ? 1u << qi : 0u;
    }
    if (cand == 0) { v = 2; return true; }           // isolated occupied pixel -> free (bev.py:204-205)
    return false;
}
// Second pass: the candidates' ring pixels (the 16 ring entries in one round trip, only the needed
// ones evaluated), then the opening. ring = the cell's ring entries, stride `cells`.
__device__ __forceinline__ int bev_cell_pass2(const BevArgs &a, const uint8_t *box, int bw, int v, uint32_t m,
                                              uint32_t cand, uint32_t outm, const uint32_t *ring, long cells) {
    if constexpr (BEV_ABL & 1) return v;
    uint32_t rneed = 0;
#pragma unroll
    for (int qi = 0; qi < 9; ++qi) {
        const int qx = qi % 3 - 1, qy = qi / 3 - 1, sh = qy * 5 + qx;
        const uint32_t win = sh >= 0 ? BEV_INNER << sh : BEV_INNER >> -sh;
        rneed |= ((cand >> qi) & 1u) ? win & ~BEV_INNER & ~outm : 0u;
    }
    uint32_t er[BEV_WIN - 9];
#pragma unroll
    for (int k = 0; k < BEV_WIN - 9; ++k) er[k] = ring[(long)k * cells];
#pragma unroll
    for (int k = 0; k < BEV_WIN - 9; ++k) {
        const int bit = BEV_ORDER[9 + k];
        if ((rneed >> bit) & 1u) m |= (uint32_t)occupied(a, bev_value_lds(box, bw, er[k])) << bit;
    }
    bool opened = false;
#pragma unroll
    for (int qi = 0; qi < 9; ++qi) {
        if (qi == 4) continue;
        const int qx = qi % 3 - 1, qy = qi / 3 - 1, sh = qy * 5 + qx;
        const uint32_t win = sh >= 0 ? BEV_INNER << sh : BEV_INNER >> -sh;
        opened |= ((cand >> qi) & 1u) && (m & win) == win;
    }
    return opened ? v : 2;
}
// One cell of one frame from a band's LDS box, both passes (the FB = 2 form): e9 = the cell's sample +
// 3x3 entries (offset in the box, Q5 fractions; BEV_ORDER), outm = its 25-bit outside-template mask.
__device__ __forceinline__ int bev_cell_lds(const BevArgs &a, const uint8_t *box, int bw, const uint32_t (&e9)[9],
                                            uint32_t outm, const uint32_t *ring, long cells) {
    if constexpr (BEV_ABL & 4) return (int)(e9[0] & 3u) | (int)(outm & 1u);
    int v;
    uint32_t m, cand;
    if (bev_cell_pass1(a, box, bw, e9, outm, v, m, cand)) return v;
    return bev_cell_pass2(a, box, bw, v, m, cand, outm, ring, cells);
}

#ifndef BEV_CTAB
#define BEV_CTAB 1
#endif
// Debug build only (-DBUGSEG_STAMPS, scripts/bev_stamp_probe.py): thread 0 of each band workgroup
// records the constant 100 MHz clock at its phase boundaries, bugseg_bev_stamps[blockIdx.x * 8 + k]
#ifdef BUGSEG_STAMPS
__device__ unsigned long long *bugseg_bev_stamps;
#define BSTAMP(k) do { if (threadIdx.x == 0 && bugseg_bev_stamps) bugseg_bev_stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define BSTAMP(k) do {} while (0)
#endif
template <int FB>
__global__ void __launch_bounds__(256, FB == 1 ? 8 : 4) bev_band_kernel(const BevArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t box[FB][BEV_BAND_CAP];
    const int tid = threadIdx.x;
    const long cells = (long)a.occ_h * a.occ_w;
    // one work item (a band's row part) per workgroup: workgroup (x, y) = (frame group f * 8 + XCD x % 8,
    // item slot y) runs item 8 y + x % 8 of frames f FB .. Dispatch order is x fastest, so consecutive
    // workgroups of an XCD take the same item for successive frames and the item's compact-table words
    // are L2 hits for all but the first frames (item-major): 30.9 -> 26.3 us per 32 frames against the
    // frame-major order (all items of frame 0, then frame 1, ...), bit-identical (scripts/gpu_r4_im.sh).
    // (A 2-D grid, not a division of the linear index: the division cost the kernel 3 spilled VGPRs.)
    const int xcd = blockIdx.x & 7;
    const int item = (int)blockIdx.y * 8 + xcd, b0 = (int)(blockIdx.x >> 3) * FB;
    if (item >= a.nitems || b0 >= a.B || (BEV_ABL & 32)) return;  // workgroup-uniform
    BSTAMP(0);
    const int2 wi = reinterpret_cast<const int2 *>(reinterpret_cast<const unsigned char *>(a.wtab) +
                                                   bev_items_offset(a.occ_w, a.occ_h))[item];
    const int band = wi.x, part = wi.y;
    const int nf = min(FB, a.B - b0);                          // frames of this workgroup
    const uint32_t frame_bytes = (uint32_t)a.in_rows * (uint32_t)a.in_cols;
    __amdgpu_buffer_rsrc_t seg[FB];
#pragma unroll
    for (int f = 0; f < FB; ++f)
        seg[f] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.seg) + (size_t)(f < nf ? b0 + f : b0) * frame_bytes,
                                                   (short)0, (int)frame_bytes, 0x00020000);
    // the band's row parts (BEV_BOXREC), evaluated in turn: part k = rows r0 .. r0 + rpp - 1 of the band
    const int4 *rec = reinterpret_cast<const int4 *>(a.wtab + (size_t)BEV_SLOTS * cells) + (size_t)band * BEV_BOXREC;
    const int4 hdr = rec[0];
    (void)hdr;
    // rows r0 .. of the band (n cells) with box bb: from LDS, or (Lc false) gathered from global memory
    auto body = [&](const int4 bb, const int r0, const int n, auto Lc) {
    constexpr bool lds = decltype(Lc)::value;
    const int y0 = bb.x, xa = bb.y, bh = lds ? bb.z : 0, bw = bb.w, zpad = bh * bw;
    // the LDS form's compact table (BEV_WIN planes of 4-B entries) and per-cell outside-template mask;
    // the first cell's entries are requested before the box staging, so their latency overlaps it
    const uint32_t *ct = reinterpret_cast<const uint32_t *>(reinterpret_cast<const unsigned char *>(a.wtab) +
                                                            bev_ctab_offset(a.occ_w, a.occ_h)) + (size_t)r0 * a.occ_w;
    const uint32_t *om = ct + (size_t)BEV_WIN * cells;
    uint32_t c9n[9], omn = 0;
    auto load9 = [&](int c) {
        const uint32_t *t = ct + min(c, n - 1);
#pragma unroll
        for (int i = 0; i < 9; ++i) c9n[i] = (BEV_ABL & 16) ? (uint32_t)(c + i) : t[(long)i * cells];
        omn = (BEV_ABL & 16) ? (uint32_t)c : om[min(c, n - 1)];
    };
    if (lds && BEV_CTAB) load9(tid);
    if (lds && !(BEV_ABL & 8)) {
        // each frame's box: all of this thread's 16-B chunks in flight before the first LDS store
        const int cpr = bw >> 4, nch = bh * cpr;
#pragma unroll
        for (int f = 0; f < FB; ++f) {
            if (f >= nf) break;
            uint4 pf[BEV_BAND_PF];
            bool in[BEV_BAND_PF];
#pragma unroll
            for (int i = 0; i < BEV_BAND_PF; ++i) {
                const int q = tid + 256 * i;
                const int r = q / cpr, c = q - r * cpr;
                const int gy = y0 + r, gx = xa + c * 16;
                in[i] = q < nch && (unsigned)gy < (unsigned)a.in_rows && (unsigned)gx < (unsigned)a.in_cols;
                pf[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                    seg[f], in[i] ? (int)(gy * a.in_cols + gx) : (int)0x80000000, 0, 0));
            }
#pragma unroll
            for (int i = 0; i < BEV_BAND_PF; ++i)
                if (tid + 256 * i < nch)
                    *reinterpret_cast<uint4 *>(box[f] + 16 * (tid + 256 * i)) =
                        in[i] ? make_uint4(inc4(pf[i].x), inc4(pf[i].y), inc4(pf[i].z), inc4(pf[i].w)) : make_uint4(0u, 0u, 0u, 0u);
            for (int i = tid; i < 2 * bw + 16; i += 256) box[f][zpad + i] = 0;
        }
        __syncthreads();
    }
    BSTAMP(1);
    // value of template pixel e in frame f: its 4 taps from the box (L: the offset the bandbox kernel
    // stored in the entry) or, for an oversized band, from global memory. The two forms are separate
    // loops (a compile-time choice): no branch between the taps, so a cell's LDS reads fly together
    const uint32_t inner = 0x739C0u;                  // bits of the 3x3 around p: rows 1..3, cols 1..3
    // the next cell's 3x3 table slots are in flight while this cell is evaluated (always issued, at a
    // clamped index, so the waits count only the current cell's loads)
    uint4 s3n[5];
    auto load3 = [&](int c) {
        const uint4 *t = a.wtab + r0 * a.occ_w + min(c, n - 1);
#pragma unroll
        for (int q = 0; q < 5; ++q) s3n[q] = t[(long)q * cells];
    };
    auto cells_loop = [&](auto from_lds) {
        constexpr bool L = decltype(from_lds)::value;
        auto value = [&](uint2 e, int f) -> int {
            if constexpr (!L) {
                return tab_value(seg[f], a.in_cols, e);
            } else {
                const uint8_t *p = box[f] + (e.y >> 15);
                const uint32_t l0 = p[0], l1 = p[1], l2 = p[bw], l3 = p[bw + 1];
                const uint32_t ax = e.y & 31u, ay = (e.y >> 5) & 31u;
                const uint32_t wx = 32u + ax * 65535u, wy = 32u + ay * 65535u;   // (32 - a) | a << 16
                const uint32_t top = dot2(l0 | l1 << 16, wx, 0u), bot = dot2(l2 | l3 << 16, wx, 0u);
                return (int)(dot2(top | bot << 16, wy, 512u) >> 10);              // (sum + 2^14) >> 15 of OpenCV
            }
        };
        load3(tid);
        for (int c = tid; c < n; c += 256) {
            const int rem = r0 * a.occ_w + c;
            const int cy = rem / a.occ_w, cx = rem - cy * a.occ_w;
            const uint4 *tab = a.wtab + rem;
            uint4 s3[5];
#pragma unroll
            for (int q = 0; q < 5; ++q) s3[q] = s3n[q];
            load3(c + 256);
            uint32_t outm = 0;                        // window positions outside the template
#pragma unroll
            for (int i = 0; i < 9; ++i) outm |= (uint32_t)((slot_half(s3[i >> 1], i & 1).y & TAB_OUT) != 0) << BEV_ORDER[i];
            int v[FB];
            uint32_t m[FB];
            bool need = false;
#pragma unroll
            for (int f = 0; f < FB; ++f) {
                int t9[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) t9[i] = value(slot_half(s3[i >> 1], i & 1), f);
                v[f] = t9[0];
                m[f] = outm;
#pragma unroll
                for (int i = 0; i < 9; ++i) m[f] |= (uint32_t)occupied(a, t9[i]) << BEV_ORDER[i];
                need |= f < nf && occupied(a, v[f]) && (m[f] & inner) != inner;
            }
            if (need) {
                // the ring completes the 5x5 window (opening at p = OR over q in N3(p) inside the template
                // of AND over N3(q) of occupancy); if the 3x3 is all occupied, q = p already survives.
                // Ring entry 9 shares the 3x3's last slot; the other 16 a slot (two entries) at a time:
                // few cells need the ring, and holding all 8 slots would cost every cell's occupancy
                {
                    const uint2 e = slot_half(s3[4], 1);
#pragma unroll
                    for (int f = 0; f < FB; ++f)
                        m[f] |= (uint32_t)((e.y & TAB_OUT) || occupied(a, value(e, f))) << BEV_ORDER[9];
                }
#pragma unroll 1
                for (int q = 5; q < BEV_SLOTS; ++q) {
                    const uint4 sq = tab[(long)q * cells];
                    const int i0 = 2 * q;
#pragma unroll
                    for (int f = 0; f < FB; ++f) {
                        m[f] |= (uint32_t)((sq.y & TAB_OUT) || occupied(a, value(make_uint2(sq.x, sq.y), f))) << BEV_ORDER_D[i0];
                        m[f] |= (uint32_t)((sq.w & TAB_OUT) || occupied(a, value(make_uint2(sq.z, sq.w), f))) << BEV_ORDER_D[i0 + 1];
                    }
                }
                int tx, ty;
                cell_pixel(a, cx, cy, tx, ty);
#pragma unroll
                for (int f = 0; f < FB; ++f) {
                    if (!(occupied(a, v[f]) && (m[f] & inner) != inner)) continue;
                    bool opened = false;
#pragma unroll
                    for (int qy = -1; qy <= 1; ++qy)
#pragma unroll
                        for (int qx = -1; qx <= 1; ++qx) {
                            const bool inside = (unsigned)(tx + qx) < (unsigned)a.occ_w_px && (unsigned)(ty + qy) < (unsigned)a.occ_h_px;
                            const int sh = qy * 5 + qx;
                            const uint32_t win = sh >= 0 ? inner << sh : inner >> -sh;
                            opened |= inside && (m[f] & win) == win;
                        }
                    if (!opened) v[f] = 2;           // isolated occupied pixel -> free (bev.py:204-205)
                }
            }
#pragma unroll
            for (int f = 0; f < FB; ++f)
                if (f < nf) bev_emit(a, b0 + f, rem, cx, cy, cells, v[f]);
        }
    };
// (measured, round 3, 32 frames of 480x640, scripts/bev_sweep.py: 42.2-49.0 -> 35.6-39.2 us per launch,
// laserscan 52.6-55.8 -> 49.8-52.1; BEV_CTAB=0: the uint4-slot form)
    if (lds && BEV_CTAB && FB == 1) {
        // the LDS form on the compact table: 4-B entries, the 3x3's 9 (and the outside-template mask) of
        // the next cell in flight while one is evaluated. Two passes: every cell's 3x3 first (most are
        // decided there), the cells whose opening needs ring pixels appended to a work list in LDS; then
        // the list, so the ring work runs on full waves instead of as divergent branches of waves whose
        // other lanes are idle (with noisy class maps the ring pass took ~40 % of the kernel)
        __shared__ uint32_t wl_n;
        __shared__ uint2 wl[BEV_WL];                 // (cell | cand << 16 | v << 25, m)
        if (tid == 0) wl_n = 0;
        __syncthreads();
        // the grid stores wait until the end: a store ahead of the next cell's table loads would hold
        // them (vmcnt retires in order), so the first 4 cells' values stay in registers (bytes of pv)
        uint32_t pv = 0, pdone = 0;
        int it = 0;
        for (int c = tid; c < n; c += 256, ++it) {
            const int rem = r0 * a.occ_w + c;
            uint32_t e9[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) e9[i] = c9n[i];
            const uint32_t outm = omn;
            load9(c + 256);
            int v;
            uint32_t m, cand;
            bool done = true;
            if constexpr (BEV_ABL & 4) v = (int)(e9[0] & 3u) | (int)(outm & 1u);
            else done = bev_cell_pass1(a, box[0], bw, e9, outm, v, m, cand);
            if (!done) {
                const uint32_t slot = c < 65536 ? atomicAdd(&wl_n, 1u) : (uint32_t)BEV_WL;
                if (slot < (uint32_t)BEV_WL) {
                    wl[slot] = make_uint2((uint32_t)c | cand << 16 | (uint32_t)v << 25, m);
                    continue;
                }
                v = bev_cell_pass2(a, box[0], bw, v, m, cand, outm, ct + (size_t)9 * cells + c, cells);   // (list full)
            }
            if (it < 4) {
                pv |= (uint32_t)v << (8 * it);
                pdone |= 1u << it;
            } else {
                // (the cell's row and column only for the ROS layout: no division per store otherwise)
                const int cy = a.ros_layout ? rem / a.occ_w : 0, cx = rem - cy * a.occ_w;
                bev_emit(a, b0, rem, cx, cy, cells, v);
            }
        }
        __syncthreads();
        BSTAMP(2);
        const int nw = (int)min(wl_n, (uint32_t)BEV_WL);
        int qv[2] = {0, 0}, qc[2] = {-1, -1};        // this thread's (at most two) list results
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int i = tid + 256 * k;
            if (i >= nw) break;
            const uint2 r = wl[i];
            const int c = (int)(r.x & 0xffffu);
            const uint32_t outm = ct[(long)BEV_WIN * cells + c];        // (L2: read again rather than kept)
            qv[k] = bev_cell_pass2(a, box[0], bw, (int)(r.x >> 25), r.y, (r.x >> 16) & 0x1ffu, outm,
                                   ct + (size_t)9 * cells + c, cells);
            qc[k] = c;
        }
        BSTAMP(3);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if ((pdone >> k) & 1u) {
                const int rem = r0 * a.occ_w + tid + 256 * k, cy = a.ros_layout ? rem / a.occ_w : 0, cx = rem - cy * a.occ_w;
                bev_emit(a, b0, rem, cx, cy, cells, (int)((pv >> (8 * k)) & 0xffu));
            }
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (qc[k] >= 0) {
                const int rem = r0 * a.occ_w + qc[k], cy = a.ros_layout ? rem / a.occ_w : 0, cx = rem - cy * a.occ_w;
                bev_emit(a, b0, rem, cx, cy, cells, qv[k]);
            }
        BSTAMP(4);
#ifdef BUGSEG_STAMPS
        if (tid == 0 && bugseg_bev_stamps) bugseg_bev_stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + 6] = (unsigned long long)nw | (unsigned long long)band << 16 | (unsigned long long)n << 32;
#endif
    } else if (lds && BEV_CTAB) {
        // (FB = 2: each cell's both passes in place)
        for (int c = tid; c < n; c += 256) {
            const int rem = r0 * a.occ_w + c;
            const int cy = rem / a.occ_w, cx = rem - cy * a.occ_w;
            uint32_t e9[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) e9[i] = c9n[i];
            const uint32_t outm = omn;
            load9(c + 256);
#pragma unroll
            for (int f = 0; f < FB; ++f)
                if (f < nf) bev_emit(a, b0 + f, rem, cx, cy, cells, bev_cell_lds(a, box[f], bw, e9, outm, ct + (size_t)9 * cells + c, cells));
        }
    } else if (lds) {
        cells_loop(std::true_type());
    } else {
        cells_loop(std::false_type());
    }
    };
    const int r0 = band * BEV_BAND + part * hdr.y, n = (min(a.occ_h, r0 + hdr.y) - r0) * a.occ_w;
    if (n <= 0) return;                                        // (a partial last band)
    // (rec[1].z < 0: a band some single-row part of which exceeds BEV_BAND_CAP gathers as one part)
    if (rec[1 + part].z < 0) body(rec[1 + part], r0, n, std::false_type());
    else body(rec[1 + part], r0, n, std::true_type());
}

// (Round 4 measured a pipelined form — one band and 2 frames per workgroup, a loader wave staging the
// next frame's box by LDS-DMA while four waves evaluate the current one — at 35.3-39.5 us per 32
// frames against 35.3-36.4 for this kernel: the band kernel is not bound by its box staging latency.
// Removed.)

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

size_t bev_table_bytes(int occ_w, int occ_h) {
    return bev_items_offset(occ_w, occ_h) + (size_t)bev_bands(occ_h) * BEV_BAND * sizeof(int2);
}

hipError_t launch_bev_table(const BevArgs &a, hipStream_t s) {
    const long cells = (long)a.occ_h * a.occ_w, total = cells * BEV_SLOTS;
    long g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(bev_table_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
    // the band boxes of the band-staged form, after the tap table (same stream)
    hipLaunchKernelGGL(bev_bandbox_kernel, dim3((unsigned)bev_bands(a.occ_h)), dim3(256), 0, s, a,
                       reinterpret_cast<int4 *>(a.wtab + (size_t)BEV_SLOTS * cells));
    return hipGetLastError();
}

#ifdef BUGSEG_STAMPS
extern "C" int bugseg_debug_set_bev_stamps(void *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(bugseg_bev_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif
hipError_t launch_bev(const BevArgs &a, hipStream_t s) {
    // form (measured, scripts/bev_probe.py): the gather kernel, 1 frame per thread (BUGSEG_BEV_F = 2 / 4:
    // frames per thread; BUGSEG_BEV_FG = n > 0: the LDS-staged kernel with n frames per workgroup);
    // read per call so tests can exercise every form
    const char *fe = std::getenv("BUGSEG_BEV_F");
    const int F = fe ? std::atoi(fe) : 1;
    const long total = (long)a.occ_h * a.occ_w * a.B;
    const int f = F == 4 ? 4 : F == 1 ? 1 : 2;
    const long band = (long)((a.occ_h + 7) / 8) * a.occ_w * ((a.B + f - 1) / f);   // items of one XCD
    long gf = 8 * ((band + 255) / 256);
    if (gf > 8192) gf = 8192;
    if (gf < 8) gf = 8;
    const char *fge = std::getenv("BUGSEG_BEV_FG");
    const int FG = fge ? std::atoi(fge) : 0;
    // BUGSEG_BEV_BAND=0: the gather / block-staged forms (A/B and tests)
    const char *be = std::getenv("BUGSEG_BEV_BAND");
    const bool banded = (!be || std::atoi(be) != 0) && !fe && FG == 0 && a.in_cols % 16 == 0;
    if (banded) {
        // frames per workgroup (BUGSEG_BEV_FB = 1 or 2; read per call)
        const char *fbe = std::getenv("BUGSEG_BEV_FB");
        // (measured at 32 frames of 480x640: FB = 1 38.7-40.1 us, FB = 2 44.6-48.5 us)
        const int FB = fbe && std::atoi(fbe) == 2 ? 2 : 1;
        const dim3 grid(8u * (unsigned)((a.B + FB - 1) / FB), (unsigned)((a.nitems + 7) / 8));   // (frame group x XCD, item slot)
        if (FB == 1) hipLaunchKernelGGL(bev_band_kernel<1>, grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL(bev_band_kernel<2>, grid, dim3(256), 0, s, a);
    } else if (F != 0 && a.in_cols % 16 == 0 && FG > 0) {
        const long nblk = (long)((a.occ_w + BEV_CB - 1) / BEV_CB) * ((a.occ_h + BEV_CB - 1) / BEV_CB);
        const long grid = nblk * ((a.B + FG - 1) / FG);
        if (grid < (1L << 31)) hipLaunchKernelGGL(bev_occgrid_lds_kernel, dim3((unsigned)grid), dim3(256), 0, s, a, FG);
    } else if (f == 1) hipLaunchKernelGGL(bev_occgrid_kernel<1>, dim3((unsigned)gf), dim3(256), 0, s, a);
    else if (f == 2) hipLaunchKernelGGL(bev_occgrid_kernel<2>, dim3((unsigned)gf), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(bev_occgrid_kernel<4>, dim3((unsigned)gf), dim3(256), 0, s, a);
    long g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    if (!a.laserscan) return hipGetLastError();
    const long rays = (long)a.B * a.ph;
    long gr = (rays + 3) / 4;
    if (gr > 8192) gr = 8192;
    hipLaunchKernelGGL(polar_min_kernel, dim3((unsigned)gr), dim3(256), 0, s, a);
    hipLaunchKernelGGL(laserscan_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace bugseg
