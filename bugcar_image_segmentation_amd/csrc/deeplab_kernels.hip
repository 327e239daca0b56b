// DeepLabV3 (MobileNetV2 backbone + ASPP) kernels for gfx950 — SURVEY.md §8(f) row 3, config 4.
//
// The reference runs the frozen DeepLab export through TF sess.run (models.py:115-125:
// ImageTensor u8 -> SemanticPredictions int64). The graph is the standard TF DeepLab export
// (deeplab/export_model.py): pad to the crop size with the mean pixel, (2/255)x - 1, MobileNetV2
// (inverted residuals: 1x1 expand + ReLU6, 3x3 depthwise (strided / atrous) + ReLU6, linear 1x1
// projection, residual), ASPP (image pooling, 1x1, optional atrous 3x3 branches), concat
// projection, 1x1 logits, bilinear resize (align_corners) to the crop, argmax.
//
// Kernels (NHWC activations, channel stride a multiple of 8, T = float | __bf16):
//   dl_prep_kernel        u8 RGB -> padded, normalised (B, Hc, Wc, 8) engine input
//   dl_conv_kernel        implicit-GEMM dense conv (1x1, 3x3 strided / atrous) on MFMA 16x16x32 bf16
//                         (or 8x 16x16x4 f32): rows = output channels, columns = pixels, k = (tap, ci);
//                         epilogue bias (+ per-image bias) + ReLU / ReLU6 + residual, written at a
//                         channel offset of the destination (ASPP concat without a copy)
//   dl_dw_kernel          depthwise 3x3 (stride, dilation, SAME pad) + bias + ReLU6, 8 channels/thread
//   dl_gap_kernel         image-pooling partial sums (deterministic: fixed chunking, no atomics)
//   dl_pool_mean/gemv     image-pooling branch: mean -> 1x1 + ReLU -> its share of the concat
//                         projection, folded into a per-image bias of the projection conv (the
//                         branch is a broadcast 1x1 image, so it never has to exist at 65x65)
//   dl_resize_argmax_kernel  logits (h, w) -> bilinear (align_corners, TF's legacy lerp order) at the
//                         crop resolution -> argmax (lowest index on ties) -> int64 class map
#include "bugseg_internal.h"
#include "deeplab_internal.h"
#include "mfma_common.h"

#include <cstdlib>

namespace bugseg {

// XCD-aware block order: workgroup h goes to XCD h % 8 (round-robin dispatch), so neighbouring
// blockIdx values land on different XCDs and each of them pulls the tiles they share into its own L2.
// Remapped, XCD x walks the contiguous run of logical blocks [x q', (x + 1) q') (q' = G / 8, the first
// G % 8 XCDs one more): the N tiles of one pixel tile, and row-neighbouring pixel tiles, share an L2.
__device__ __forceinline__ int xcd_block(int h, int G) {
    const int q = G >> 3, r = G & 7, x = h & 7, s = h >> 3;
    return x < r ? x * (q + 1) + s : r * (q + 1) + (x - r) * q + s;
}

// ------------------------------------------------------------------ preprocess
// TF: pad_to_bounding_box(x - 127.5) + 127.5 (exact for integer x), then (2/255) * x - 1 in f32.
template <typename T>
__global__ void __launch_bounds__(256) dl_prep_kernel(const DlPrepArgs a) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = a.B * a.Hc * a.Wc;
    if (i >= n) return;
    const int x = i % a.Wc, t = i / a.Wc, y = t % a.Hc, b = t / a.Hc;
    const float scale = 2.0f / 255.0f;   // f32(2/255), as TF's constant
    float v[3];
    if (y < a.H && x < a.W) {
        const uint8_t *p = a.rgb + ((size_t)(b * a.H + y) * a.W + x) * 3;
        for (int c = 0; c < 3; ++c) v[c] = scale * (float)p[c] - 1.0f;
    } else {
        for (int c = 0; c < 3; ++c) v[c] = scale * 127.5f - 1.0f;
    }
    T *o = reinterpret_cast<T *>(a.out) + (size_t)i * 8;
    typename Tr<T>::Raw r;
    set3(r, v[0], v[1], v[2]);
    if constexpr (sizeof(T) == 2) *reinterpret_cast<uint4 *>(o) = r.v;
    else {
        reinterpret_cast<float4 *>(o)[0] = r.a;
        reinterpret_cast<float4 *>(o)[1] = r.b;
    }
}

// The engine input at crop pixel (iy, ix) of image b, formed from the raw RGB bytes exactly as
// dl_prep_kernel stores it (inside the image: f32(2/255) x - 1; padding: the mean pixel 127.5
// normalised), for the stem's fused-preprocessing operand loads. Caller: (iy, ix) inside the crop.
template <typename T>
__device__ __forceinline__ void prep_px(typename Tr<T>::Raw &r, const uint8_t *rgb, int b, int H, int W, int iy, int ix) {
#pragma clang fp contract(off)
    const float scale = 2.0f / 255.0f;
    float v[3];
    if (iy < H && ix < W) {
        const uint8_t *p = rgb + ((size_t)(b * H + iy) * W + ix) * 3;
        for (int c = 0; c < 3; ++c) v[c] = scale * (float)p[c] - 1.0f;
    } else {
        for (int c = 0; c < 3; ++c) v[c] = scale * 127.5f - 1.0f;
    }
    set3(r, v[0], v[1], v[2]);
}

// ------------------------------------------------------------------ dense conv (implicit GEMM)
// Workgroup = 4 waves = 128 pixels x 64 output channels; a wave owns 32 pixels (2 B fragments)
// x 64 channels (4 A fragments): 8 MFMAs per k-step of 32 (one tap, 32 input channels).
// A fragment (weights, packed [NP][taps][cinP], k contiguous): lane row = col, k = 8*kq .. +7.
// B fragment (pixels): lane column = col, channels 8*kq .. +7 of that pixel at that tap; taps
// outside the image and channels past the input's stride read 0 through the buffer descriptor.
constexpr int DL_STG_RS = 68;   // staging row stride (floats): 64 channels + 4 (bank spread)

__device__ __forceinline__ void raw4(const RawB &r, float4 &a, float4 &b) {
    a = unpack_bf16x4((u32x2_t){r.v.x, r.v.y});
    b = unpack_bf16x4((u32x2_t){r.v.z, r.v.w});
}
__device__ __forceinline__ void raw4(const RawF &r, float4 &a, float4 &b) { a = r.a; b = r.b; }

// Depthwise 3x3 of 8 channels [c, c+8) at one pixel from its 9 tap offsets (OOB = padding), in the
// dw kernel's exact order (taps (ky, kx), fmaf per channel, then bias, ReLU6), rounded to T.
template <typename T>
__device__ __forceinline__ void dw8(typename Tr<T>::Raw &out, __amdgpu_buffer_rsrc_t rin, const uint32_t (&tb)[9], int c,
                                    const T *dw_w, const float *dw_b, int C) {
    // branch-free (padding taps read 0 through the descriptor, as in dl_dw_kernel): 18 loads in flight
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    typename Tr<T>::Raw xr[9], wr[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        bld8(xr[t], rin, tb[t] == OOB ? OOB : (tb[t] + c) * (uint32_t)sizeof(T));
        ld8(wr[t], dw_w + t * C + c);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        float4 x0, x1, w0, w1;
        raw4(xr[t], x0, x1);
        raw4(wr[t], w0, w1);
        acc[0] = fmaf(x0.x, w0.x, acc[0]); acc[1] = fmaf(x0.y, w0.y, acc[1]);
        acc[2] = fmaf(x0.z, w0.z, acc[2]); acc[3] = fmaf(x0.w, w0.w, acc[3]);
        acc[4] = fmaf(x1.x, w1.x, acc[4]); acc[5] = fmaf(x1.y, w1.y, acc[5]);
        acc[6] = fmaf(x1.z, w1.z, acc[6]); acc[7] = fmaf(x1.w, w1.w, acc[7]);
    }
    const float4 b0 = ld4f(dw_b + c), b1 = ld4f(dw_b + c + 4);
    auto r6 = [](float v) { return fminf(fmaxf(v, 0.f), 6.f); };
    const T v[8] = {(T)r6(acc[0] + b0.x), (T)r6(acc[1] + b0.y), (T)r6(acc[2] + b0.z), (T)r6(acc[3] + b0.w),
                    (T)r6(acc[4] + b1.x), (T)r6(acc[5] + b1.y), (T)r6(acc[6] + b1.z), (T)r6(acc[7] + b1.w)};
    set8(out, v);
}

// Grid: 1-D, the N tiles of one pixel tile adjacent in logical order (they share the input tile), the
// logical order XCD-aware (xcd_block).
// NB = pixel fragments per wave (2: 128-px workgroup tiles, 4: 256 px, 8: 512 px (bf16 only); NB MFMAs per
// weight-fragment load).
template <typename T, bool OUTF32, bool DWF, int NB, int PD = 1>
__global__ void __launch_bounds__(256) dl_conv_kernel(const DlConvArgs a) {
    constexpr int WPX = NB * 16, TPX = 4 * WPX;   // pixels per wave / per workgroup
    using Raw = typename Tr<T>::Raw;
    const int lane = threadIdx.x & 63, col = lane & 15, kq = lane >> 4;
    const int wave = threadIdx.x >> 6;
    const int ntn = a.NP >> 6;
    const int bid = xcd_block(blockIdx.x, gridDim.x);
    const int n0 = (bid % ntn) * 64;
    const int mtile = bid / ntn;
    const __amdgpu_buffer_rsrc_t rin = mkbuf(a.in, a.in_bytes);
    const int esz = (int)sizeof(T);

    int pb[NB], piy[NB], pix[NB];
    bool pv[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        const int p = mtile * TPX + wave * WPX + j * 16 + col;
        pv[j] = p < a.M;
        const int pp = pv[j] ? p : 0;
        const int b = (int)fdiv((uint32_t)pp, a.mHW, a.sHW);
        const int r = pp - b * a.Hout * a.Wout;
        const int oy = (int)fdiv((uint32_t)r, a.mW, a.sW);
        const int ox = r - oy * a.Wout;
        pb[j] = b;
        piy[j] = oy * a.stride - a.pad_t;
        pix[j] = ox * a.stride - a.pad_l;
    }
    f32x4 acc[NB][4];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[j][r] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const int K = a.tap_packed ? ((a.taps + 3) >> 2) * 32 : a.taps * a.cinP;
    const T *wrow[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) wrow[r] = reinterpret_cast<const T *>(a.w) + (size_t)(n0 + r * 16 + col) * K + kq * 8;
    const int chunks = a.cinP >> 5;

    if constexpr (DWF) {
        // 1x1 projection of the depthwise output computed on load; pixel (oy, ox) of the dw output grid
        uint32_t tb[NB][9];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int iy0 = piy[j] * a.dw_stride - a.dw_pt, ix0 = pix[j] * a.dw_stride - a.dw_pl;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int iy = iy0 + (t / 3) * a.dw_dil, ix = ix0 + (t % 3) * a.dw_dil;
                const bool ok = pv[j] && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
                tb[j][t] = ok ? (uint32_t)(((pb[j] * a.Hin + iy) * a.Win + ix) * a.CS) : OOB;
            }
        }
        for (int ch = 0; ch < chunks; ++ch) {
            const int c = ch * 32 + kq * 8;
            Raw bx[NB], wa[4];
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                if (c < a.CS) dw8<T>(bx[j], rin, tb[j], c, reinterpret_cast<const T *>(a.dw_w), a.dw_b, a.CS);
                else zero(bx[j]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) ld8(wa[r], wrow[r] + ch * 32);
#pragma unroll
            for (int j = 0; j < NB; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) mma(acc[j][r], wa[r], bx[j]);
        }
    } else if (a.tap_packed) {
        // input of at most 8 channels (the stem): a k-step is 4 taps x 8 channels, lane group kq
        // takes tap 4 ks + kq (weights packed k = tap * 8 + c): 3 k-steps for a 3x3 instead of 9
        const int nks = (a.taps + 3) >> 2;
        for (int ks = 0; ks < nks; ++ks) {
            const int t = ks * 4 + kq;
            const int ky = t / a.kw, kx = t - (t / a.kw) * a.kw;
            Raw bx[NB], wa[4];
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const int iy = piy[j] + ky * a.dil, ix = pix[j] + kx * a.dil;
                const bool ok = t < a.taps && pv[j] && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
                if (a.rgb) {
                    if (ok) prep_px<T>(bx[j], a.rgb, pb[j], a.img_h, a.img_w, iy, ix);
                    else zero(bx[j]);
                } else {
                    bld8(bx[j], rin, ok ? (uint32_t)(((pb[j] * a.Hin + iy) * a.Win + ix) * a.CS) * esz : OOB);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) ld8(wa[r], wrow[r] + ks * 32);
#pragma unroll
            for (int j = 0; j < NB; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) mma(acc[j][r], wa[r], bx[j]);
        }
    } else {
        // k-steps (tap, 32-channel chunk) flattened; the fragments of the next PD steps are in flight
        // while the current step's MFMAs run (a ring of PD + 1 register slots, unrolled so every slot
        // index is a compile-time constant; loads are issued in step order by one cursor)
        const int nks = a.taps * chunks;
        int lt = 0, lch = 0;                    // load cursor: tap, chunk
        uint32_t base[NB];
        auto bases = [&](int t) {
            const int ky = t / a.kw, kx = t - (t / a.kw) * a.kw;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const int iy = piy[j] + ky * a.dil, ix = pix[j] + kx * a.dil;
                const bool ok = pv[j] && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
                base[j] = ok ? (uint32_t)(((pb[j] * a.Hin + iy) * a.Win + ix) * a.CS) : OOB;
            }
        };
        auto load = [&](Raw (&bx)[NB], Raw (&wa)[4]) {
            const int c = lch * 32 + kq * 8;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                const uint32_t off = (base[j] != OOB && c < a.CS) ? (base[j] + c) * esz : OOB;
                bld8(bx[j], rin, off);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) ld8(wa[r], wrow[r] + lt * a.cinP + lch * 32);
            if (++lch == chunks) {
                lch = 0;
                if (++lt < a.taps) bases(lt);
            }
        };
        bases(0);
        Raw bx[PD + 1][NB], wa[PD + 1][4];
#pragma unroll
        for (int u = 0; u < PD; ++u)
            if (u < nks) load(bx[u], wa[u]);
        for (int ks = 0; ks < nks; ks += PD + 1) {
#pragma unroll
            for (int u = 0; u <= PD; ++u) {
                if (ks + u < nks) {
                    if (ks + u + PD < nks) load(bx[(u + PD) % (PD + 1)], wa[(u + PD) % (PD + 1)]);
#pragma unroll
                    for (int j = 0; j < NB; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) mma(acc[j][r], wa[u][r], bx[u][j]);
                }
            }
        }
    }

    // epilogue: lane holds channels n0 + 16r + 4kq .. +3 of pixel column `col` of fragment j.
    // bias (+ per-image bias) and the activation in registers, then the wave's 32 px x 64 ch tile goes
    // through LDS (f32, so a residual add still rounds once) and comes back as 8 consecutive channels
    // per lane: each store / residual load instruction covers 8 pixels' contiguous 128-B channel runs.
    // staged 32 pixels (two fragments) at a time: 34 KB of LDS per workgroup at any NB
    __shared__ __attribute__((aligned(16))) float stg[4][32 * DL_STG_RS];
    float *st = stg[wave];
    const int c8 = (lane & 7) * 8;
    const bool cok = n0 + c8 < a.cout;          // cout is a multiple of 8
#pragma unroll
    for (int h = 0; h < NB / 2; ++h) {
        if (h) wave_lds_sync();                 // the previous half's reads are done
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * h + jj;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int nl = r * 16 + kq * 4, n = n0 + nl;
                float4 v = add4(f4(acc[j][r]), ld4f(a.bias + n));
                if (a.bias_img) v = add4(v, ld4f(a.bias_img + (size_t)pb[j] * a.bias_img_stride + n));
                if (a.act == 1 || a.act == 2) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
                if (a.act == 2) v = make_float4(fminf(v.x, 6.f), fminf(v.y, 6.f), fminf(v.z, 6.f), fminf(v.w, 6.f));
                *reinterpret_cast<float4 *>(st + (jj * 16 + col) * DL_STG_RS + nl) = v;
            }
        }
        wave_lds_sync();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int pl = it * 8 + (lane >> 3);
            const int p = mtile * TPX + wave * WPX + h * 32 + pl;
            if (p >= a.M || !cok) continue;
            float4 v0 = *reinterpret_cast<const float4 *>(st + pl * DL_STG_RS + c8);
            float4 v1 = *reinterpret_cast<const float4 *>(st + pl * DL_STG_RS + c8 + 4);
            const int n = n0 + c8;
            if (a.res) {
                const T *rp = reinterpret_cast<const T *>(a.res) + (size_t)p * a.res_cs + n;
                v0 = add4(v0, ld4(rp));
                v1 = add4(v1, ld4(rp + 4));
            }
            if (a.act == 3) {              // ReLU after the residual add (ResNet units)
                v0 = make_float4(fmaxf(v0.x, 0.f), fmaxf(v0.y, 0.f), fmaxf(v0.z, 0.f), fmaxf(v0.w, 0.f));
                v1 = make_float4(fmaxf(v1.x, 0.f), fmaxf(v1.y, 0.f), fmaxf(v1.z, 0.f), fmaxf(v1.w, 0.f));
            }
            if constexpr (OUTF32) {
                float *o = reinterpret_cast<float *>(a.out) + (size_t)p * a.out_cs + a.out_off + n;
                st4(o, v0);
                st4(o + 4, v1);
            } else {
                T *o = reinterpret_cast<T *>(a.out) + (size_t)p * a.out_cs + a.out_off + n;
                st4(o, v0);
                st4(o + 4, v1);
            }
        }
    }
}

// ------------------------------------------------------------------ 1x1 conv as an LDS-staged GEMM
// The expansions, projections and the ASPP / logits 1x1s (bf16): out[p][n] = act(sum_k in[p][k] w[n][k]
// + bias (+ per-image bias)) (+ residual). dl_conv_kernel feeds its MFMAs straight from global memory,
// every wave issuing 16-B loads that touch half-used lines and re-load the weights its neighbours
// load (the measured limit: vector-memory issue); here a workgroup tile of TM = 256 pixels
// x 64 output channels is staged through LDS in k-stages of 64 channels: the pixels' 128-B channel
// runs and the weight rows arrive as whole lines (8 lanes per line), once per workgroup, the next
// stage's loads are in flight in registers while the current stage's 32 MFMAs per wave run, and every
// wave reads its 16 x 16 fragments from LDS. The k-steps (32 channels) go through the MFMAs in the
// same order and with the same epilogue as dl_conv_kernel, so the results are bit-identical.
constexpr int GM_TM = 256, GM_TN = 64, GM_KT = 64, GM_RS = GM_KT + 16;   // LDS row: 80 elements (40 dwords)

// TM = pixels per workgroup tile: 256 (4 fragments per wave) or 128 (2 fragments per wave: a smaller
// LDS and register footprint, so more workgroups per CU keep more loads and stores in flight)
template <bool OUTF32, bool RPF, bool PD2 = false, int TM = GM_TM>
__global__ void __launch_bounds__(256, 2) dl_gemm_kernel(const DlConvArgs a) {
    constexpr int FJ = TM / 64, WPX = TM / 4, NBC = TM / 32;   // fragments / pixels per wave, B chunks per thread
    constexpr int SMB = (GM_TN + TM) * GM_RS * 2, STB = 4 * 32 * DL_STG_RS * 4;   // operand / staging bytes
    __shared__ __attribute__((aligned(16))) __bf16 sm[(SMB > STB ? SMB : STB) / 2];
    __bf16 *sA = sm, *sB = sm + GM_TN * GM_RS;
    const int tid = threadIdx.x, lane = tid & 63, col = lane & 15, kq = lane >> 4, wave = tid >> 6;
    const int ntn = a.NP >> 6;
    const int bid = xcd_block(blockIdx.x, gridDim.x);
    const int n0 = (bid % ntn) * GM_TN, p0 = (bid / ntn) * TM;
    const int K = a.cinP;
    const __amdgpu_buffer_rsrc_t rin = mkbuf(a.in, a.in_bytes);
    const __amdgpu_buffer_rsrc_t rw = mkbuf(a.w, (uint32_t)((size_t)a.NP * K * 2));
    // this thread's 16-B chunks of a stage: pixel rows q >> 3 (8 per thread), weight rows (2 per thread)
    uint32_t boff[NBC], woff[2];
    int bk[NBC], wk[2];
#pragma unroll
    for (int i = 0; i < NBC; ++i) {
        const int q = tid + 256 * i, px = q >> 3;
        bk[i] = (q & 7) * 8;
        boff[i] = p0 + px < a.M ? (uint32_t)((p0 + px) * a.CS + bk[i]) * 2u : OOB;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = tid + 256 * i, row = q >> 3;
        wk[i] = (q & 7) * 8;
        woff[i] = (uint32_t)((n0 + row) * K + wk[i]) * 2u;
    }
    uint4 pb[NBC], pw[2], qb[NBC], qw[2];   // qb / qw: PD2's second stage in flight
    auto fetch_to = [&](int k0, uint4 (&xb)[NBC], uint4 (&xw)[2]) {
#pragma unroll
        for (int i = 0; i < NBC; ++i) xb[i] = bld16(rin, boff[i] != OOB && k0 + bk[i] < a.CS ? boff[i] + k0 * 2 : OOB);
#pragma unroll
        for (int i = 0; i < 2; ++i) xw[i] = bld16(rw, k0 + wk[i] < K ? woff[i] + k0 * 2 : OOB);
    };
    auto fetch = [&](int k0) { fetch_to(k0, pb, pw); };
    f32x4 acc[FJ][4];
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[j][r] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int nst = (K + GM_KT - 1) / GM_KT;
    const int c8 = (lane & 7) * 8;
    const bool cok = n0 + c8 < a.cout;
    uint4 rres[FJ / 2][4];   // the epilogue's residual, loaded ahead of the k-loop (as dl_gemm128_kernel)
    if constexpr (RPF) {
#pragma unroll
        for (int h = 0; h < FJ / 2; ++h)
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int p = p0 + wave * WPX + h * 32 + it * 8 + (lane >> 3);
                rres[h][it] = cok && p < a.M ? *reinterpret_cast<const uint4 *>(reinterpret_cast<const __bf16 *>(a.res) +
                                                                                (size_t)p * a.res_cs + n0 + c8)
                                             : make_uint4(0, 0, 0, 0);
            }
    }
    auto put = [&](const uint4 (&xb)[NBC], const uint4 (&xw)[2]) {
        __syncthreads();                          // every wave is done reading the previous stage
#pragma unroll
        for (int i = 0; i < NBC; ++i) {
            const int q = tid + 256 * i;
            *reinterpret_cast<uint4 *>(sB + (q >> 3) * GM_RS + (q & 7) * 8) = xb[i];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = tid + 256 * i;
            *reinterpret_cast<uint4 *>(sA + (q >> 3) * GM_RS + (q & 7) * 8) = xw[i];
        }
        __syncthreads();
    };
    auto compute = [&](int st) {
#pragma unroll
        for (int s2 = 0; s2 < GM_KT / 32; ++s2) {
            if (st * GM_KT + s2 * 32 >= K) break;  // (uniform) a 32-channel tail stage: no empty k-step
            RawB wa[4], bx[FJ];
#pragma unroll
            for (int r = 0; r < 4; ++r) ld8(wa[r], sA + (r * 16 + col) * GM_RS + s2 * 32 + kq * 8);
#pragma unroll
            for (int j = 0; j < FJ; ++j) ld8(bx[j], sB + (wave * WPX + j * 16 + col) * GM_RS + s2 * 32 + kq * 8);
#pragma unroll
            for (int j = 0; j < FJ; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) mma(acc[j][r], wa[r], bx[j]);
        }
    };
    fetch(0);
    if constexpr (PD2) {
        // two stages in flight in registers (K > 64: a stage's 32 MFMAs per wave are too short to
        // cover one fetch's latency); the loop unrolled by two so each register set's role is static
        if (nst > 1) fetch_to(GM_KT, qb, qw);
        for (int st = 0; st < nst; st += 2) {
            put(pb, pw);
            if (st + 2 < nst) fetch_to((st + 2) * GM_KT, pb, pw);
            compute(st);
            if (st + 1 >= nst) break;
            put(qb, qw);
            if (st + 3 < nst) fetch_to((st + 3) * GM_KT, qb, qw);
            compute(st + 1);
        }
    } else {
        for (int st = 0; st < nst; ++st) {
            put(pb, pw);
            if (st + 1 < nst) fetch((st + 1) * GM_KT);
            compute(st);
        }
    }
    // epilogue (dl_conv_kernel's, 32 pixels at a time through the wave's share of the staging LDS)
    __syncthreads();
    float *st = reinterpret_cast<float *>(sm) + wave * 32 * DL_STG_RS;
#pragma unroll
    for (int h = 0; h < FJ / 2; ++h) {
        if (h) wave_lds_sync();
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * h + jj;
            const int p = p0 + wave * WPX + j * 16 + col;
            const int pimg = a.bias_img ? (int)fdiv((uint32_t)(p < a.M ? p : 0), a.mHW, a.sHW) : 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int nl = r * 16 + kq * 4, n = n0 + nl;
                float4 v = add4(f4(acc[j][r]), ld4f(a.bias + n));
                if (a.bias_img) v = add4(v, ld4f(a.bias_img + (size_t)pimg * a.bias_img_stride + n));
                if (a.act == 1 || a.act == 2) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
                if (a.act == 2) v = make_float4(fminf(v.x, 6.f), fminf(v.y, 6.f), fminf(v.z, 6.f), fminf(v.w, 6.f));
                *reinterpret_cast<float4 *>(st + (jj * 16 + col) * DL_STG_RS + nl) = v;
            }
        }
        wave_lds_sync();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int pl = it * 8 + (lane >> 3);
            const int p = p0 + wave * WPX + h * 32 + pl;
            if (p >= a.M || !cok) continue;
            float4 v0 = *reinterpret_cast<const float4 *>(st + pl * DL_STG_RS + c8);
            float4 v1 = *reinterpret_cast<const float4 *>(st + pl * DL_STG_RS + c8 + 4);
            const int n = n0 + c8;
            if (RPF) {
                const uint4 u = rres[h][it];
                v0 = add4(v0, make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                          __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)));
                v1 = add4(v1, make_float4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u),
                                          __uint_as_float(u.w << 16), __uint_as_float(u.w & 0xffff0000u)));
            }
            if (a.act == 3) {              // ReLU after the residual add (ResNet units)
                v0 = make_float4(fmaxf(v0.x, 0.f), fmaxf(v0.y, 0.f), fmaxf(v0.z, 0.f), fmaxf(v0.w, 0.f));
                v1 = make_float4(fmaxf(v1.x, 0.f), fmaxf(v1.y, 0.f), fmaxf(v1.z, 0.f), fmaxf(v1.w, 0.f));
            }
            if constexpr (OUTF32) {
                float *o = reinterpret_cast<float *>(a.out) + (size_t)p * a.out_cs + a.out_off + n;
                st4(o, v0);
                st4(o + 4, v1);
            } else {
                __bf16 *o = reinterpret_cast<__bf16 *>(a.out) + (size_t)p * a.out_cs + a.out_off + n;
                st4(o, v0);
                st4(o + 4, v1);
            }
        }
    }
}

// ------------------------------------------------------------------ 1x1 conv, MFMA-heavy shapes
// Deep 1x1 convolutions (K >= 256 input channels, >= 128 outputs: Xception's 728/1024/1536-channel
// pointwise layers, MobileNetV2's 576/960 -> N projections, the ASPP 1x1s) are MFMA-bound, and
// dl_gemm_kernel's 256 x 64 tile with register-staged k-stages is latency-bound on them (one stage in
// flight behind 32 MFMAs per wave). Here: a 128-pixel x 128-channel tile, four waves as 2 x 2 (each
// 64 x 64 = the same acc[4][4] fragment set), k-stages of 64 channels moved global -> LDS by
// global_load_lds (16 B per lane, no VGPR round trip) into two LDS buffers, so stage s + 1 is in
// flight while stage s's 32 MFMAs per wave run; one raw barrier after the counted vmcnt wait, one
// after the reads. LDS rows are 128 B (64 bf16) with the 16-B slots XOR-swizzled by row:
// slot = kchunk ^ ((row >> 1) & 7), so the 16 rows a ds_read_b128 lane group reads (one k-chunk)
// land on 16 distinct 16-B bank groups; glds writes lane-linear, so each lane fetches the chunk its
// slot holds (the swizzle is applied to the global source address). The k-steps go through the same
// MFMA in the same order as dl_conv_kernel / dl_gemm_kernel with the same epilogue: bit-identical.
// Tails: rows past M / NP re-read an in-range row (their products are never stored); activation
// chunks past the stored CS read the weights' zero padding (columns >= cin), so they add exact zeros.
constexpr int G2_T = 128, G2_KT = 64;

__device__ __forceinline__ void glds16(const void *g, void *lds) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}
// An LDS read the compiler does not see: its alias tracking of the in-flight glds otherwise puts a
// vmcnt(0) ahead of the reads and drains the next stage's prefetch. The data is waited for by
// lds_wait8, which takes the eight destination registers as operands so no MFMA can move above it.
__device__ __forceinline__ u32x4 lds_read16(const void *p) {
    u32x4 v;
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ void lds_wait8(u32x4 &a0, u32x4 &a1, u32x4 &a2, u32x4 &a3, u32x4 &b0, u32x4 &b1,
                                          u32x4 &b2, u32x4 &b3) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2),
                 "+v"(b3));
}

// Ablation builds (round 3, Xception-65 B = 32, the 63 pointwise launches per forward): 4,826 us as
// built, 4,454 us without the MFMAs, 3,479 us without the operand loads — the tile is bound by the
// operand delivery (global -> LDS, 64 B per CU-clock at the MFMA rate for a 128 x 128 tile), not by the
// matrix pipe. Reading both k-steps' fragments ahead of the first step's MFMAs (opaque asm reads with
// a counted lgkmcnt) gave wrong results: the register allocator copied a pending read's destination

//
// CONV = true: the same tile as an implicit-GEMM k x k convolution (ResNet's dense 3x3s, strided or
// atrous, and the ASPP atrous branches): K = taps * cinP with cinP = CS a multiple of 64, so each
// 64-channel k-stage lies inside one tap (ky, kx) and its pixel rows read the input pixel
// (y * stride - pad_t + ky * dil, x * stride - pad_l + kx * dil) — no im2col buffer. Taps outside the
// image read a 16-B zero chunk placed after the weight blob (a.zero). The k order is the packing's
// (tap-major, 32-channel steps), the order dl_conv_kernel walks, through the same MFMA: bit-identical.
// s_waitcnt vmcnt(N): all but the N most recent vector-memory loads of this wave have landed
template <int N> __device__ __forceinline__ void vm_wait_stage();
template <> __device__ __forceinline__ void vm_wait_stage<8>() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
template <> __device__ __forceinline__ void vm_wait_stage<10>() { asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); }

template <bool OUTF32, bool CONV, bool RPF, int TPX = G2_T>
__device__ __forceinline__ void g2_body(const DlConvArgs &a, const int bid) {
    // TPX = pixels per tile: 128 (the 128 x 128 tile, waves 2 x 2) or 256 (256 pixels x 64 channels,
    // waves 4 x 1: 64-channel outputs, ResNet's root and block-1 3x3s); each wave's 64 x 64 is the same
    constexpr int TN = G2_T * G2_T / TPX, WM = TPX / 64, NA = TN / 32, NBL = TPX / 32;   // glds per wave: NA + NBL
    // two LDS objects, one per buffer, and the k-loop unrolled by two so each buffer's role is static:
    // the compiler then sees that a stage's ds_reads cannot alias the glds filling the other buffer
    // and does not drain the prefetch (vmcnt(0)) ahead of them
    __shared__ __attribute__((aligned(16))) __bf16 sm0[(TN + TPX) * G2_KT];   // [A | B][rows][64]: 32 / 40 KB
    __shared__ __attribute__((aligned(16))) __bf16 sm1[(TN + TPX) * G2_KT];
    const int tid = threadIdx.x, lane = tid & 63, col = lane & 15, kq = lane >> 4, wave = tid >> 6;
    const int wm = wave % WM, wn = wave / WM;
    const int ntn = (a.NP + TN - 1) / TN;
    const int n0 = (bid % ntn) * TN, p0 = (bid / ntn) * TPX;
    const __bf16 *wg = reinterpret_cast<const __bf16 *>(a.w), *xg = reinterpret_cast<const __bf16 *>(a.in);
    // this lane's glds sources: A instruction i fills LDS rows wave * TN / 4 + i * 8 + (lane >> 3), B
    // instruction i rows wave * TPX / 4 + i * 8 + (lane >> 3); slot lane & 7
    const int K = CONV ? a.taps * a.cinP : a.cinP;
    const __bf16 *sa[NA], *sb[NBL];
    int ka[NA], kb[NBL], y0[NBL], x0[NBL];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int r = wave * (TN / 4) + i * 8 + (lane >> 3);
        ka[i] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
        sa[i] = wg + (size_t)min(n0 + r, a.NP - 1) * K;
    }
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
        const int r = wave * (TPX / 4) + i * 8 + (lane >> 3);
        kb[i] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
        const int p = min(p0 + r, a.M - 1);
        if constexpr (CONV) {   // this row's output pixel -> its top-left tap in the input image
            const int b = (int)fdiv((uint32_t)p, a.mHW, a.sHW), q = p - b * a.Hout * a.Wout;
            const int y = (int)fdiv((uint32_t)q, a.mW, a.sW), x = q - y * a.Wout;
            y0[i] = y * a.stride - a.pad_t;
            x0[i] = x * a.stride - a.pad_l;
            sb[i] = xg + (size_t)b * a.Hin * a.Win * a.CS + kb[i];
        } else {
            sb[i] = xg + (size_t)p * a.CS;
        }
    }
    auto stage = [&](int st, __bf16 *buf) {
        const int k0 = st * G2_KT;
        __bf16 *bA = buf + wave * (TN / 4) * G2_KT, *bB = buf + TN * G2_KT + wave * (TPX / 4) * G2_KT;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int k = k0 + ka[i];
            glds16(sa[i] + (k < K ? k : 0), bA + i * 8 * G2_KT);
        }
        if constexpr (CONV) {
            const int tap = k0 / a.cinP, c0 = k0 - tap * a.cinP;   // uniform
            const int ky = tap / a.kw, dy = ky * a.dil, dx = (tap - ky * a.kw) * a.dil;
#pragma unroll
            for (int i = 0; i < NBL; ++i) {
                const int iy = y0[i] + dy, ix = x0[i] + dx;
                const bool in = (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
                glds16(in ? sb[i] + ((size_t)iy * a.Win + ix) * a.CS + c0 : reinterpret_cast<const __bf16 *>(a.zero),
                       bB + i * 8 * G2_KT);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NBL; ++i) {
                const int k = k0 + kb[i];
                // channels past the stored CS (K padded up to the k-stage) read a zero chunk: the weight
                // row 0's own padding columns k >= CS >= cin, so a non-finite activation never meets them
                glds16(k < a.CS ? sb[i] + k : wg + k, bB + i * 8 * G2_KT);
            }
        }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[j][r] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // one 32-channel k-step's fragments: 4 weight rows, 4 pixel rows (ds_read_b128, swizzled slots)
    auto rd = [&](const __bf16 *bA, int s2, u32x4 (&ra)[4], u32x4 (&rb)[4]) {
        const __bf16 *bB = bA + TN * G2_KT;
        const int ch = s2 * 4 + kq;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = wn * 64 + r * 16 + col;
            ra[r] = lds_read16(bA + row * G2_KT + ((ch ^ ((row >> 1) & 7)) << 3));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = wm * 64 + j * 16 + col;
            rb[j] = lds_read16(bB + row * G2_KT + ((ch ^ ((row >> 1) & 7)) << 3));
        }
    };
    auto mm = [&](const u32x4 (&ra)[4], const u32x4 (&rb)[4]) {
        RawB wa[4], bx[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            wa[r].v = __builtin_bit_cast(uint4, ra[r]);
            bx[r].v = __builtin_bit_cast(uint4, rb[r]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) mma(acc[j][r], wa[r], bx[j]);
    };
    auto compute = [&](int st, const __bf16 *bA) {
        const bool two = st * G2_KT + 32 < K;                  // (uniform) 32-channel tail stage
#pragma unroll
        for (int s2 = 0; s2 < G2_KT / 32; ++s2) {
            if (s2 == 1 && !two) break;
            u32x4 ra[4], rb[4];
            rd(bA, s2, ra, rb);
            lds_wait8(ra[0], ra[1], ra[2], ra[3], rb[0], rb[1], rb[2], rb[3]);
            mm(ra, rb);
        }
    };
    const int nst = (K + G2_KT - 1) / G2_KT;
    // RPF (launches with a residual: the ResNet units' expansions): the epilogue's residual (64 pixels x
    // 64 channels per wave, 8 x 16 B per lane) is loaded ahead of the k-loop, so its latency hides behind
    // the MFMAs. Measured (ResNet-101, B = 16): expansions 1,200 -> 1,120 us per forward; an
    // instantiation of its own because the 32 extra VGPRs slow the launches without one by ~5%
    const int nb = n0 + wn * 64;
    const int c8 = (lane & 7) * 8;
    const bool cok = nb < a.NP && nb + c8 < a.cout;
    uint4 rres[2][4];
    if constexpr (RPF) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int p = p0 + wm * 64 + h * 32 + it * 8 + (lane >> 3);
                rres[h][it] = cok && p < a.M ? *reinterpret_cast<const uint4 *>(reinterpret_cast<const __bf16 *>(a.res) +
                                                                                (size_t)p * a.res_cs + nb + c8)
                                             : make_uint4(0, 0, 0, 0);
            }
    }
    stage(0, sm0);
    for (int st = 0; st < nst; st += 2) {
        if (st + 1 < nst) {
            stage(st + 1, sm1);
            vm_wait_stage<NA + NBL>();                         // this wave's loads of stage st landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();                          // ... and every other wave's
        compute(st, sm0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                          // sm0 may be refilled (stage st + 2)
        if (st + 1 >= nst) break;
        if (st + 2 < nst) {
            stage(st + 2, sm0);
            vm_wait_stage<NA + NBL>();
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        compute(st + 1, sm1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    // epilogue (dl_gemm_kernel's, per wave: its 64 pixels x 64 channels, 32 pixels at a time)
    if (nb >= a.NP) return;
    // two waves' 8.7 KB staging areas in each LDS object (each area lies inside one object)
    static_assert(2 * 32 * DL_STG_RS * sizeof(float) <= sizeof(sm0), "epilogue staging must fit one LDS object");
    float *stg = reinterpret_cast<float *>(wave < 2 ? sm0 : sm1) + (wave & 1) * 32 * DL_STG_RS;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h) wave_lds_sync();
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int j = 2 * h + jj;
            const int p = p0 + wm * 64 + j * 16 + col;
            const int pimg = a.bias_img ? (int)fdiv((uint32_t)(p < a.M ? p : 0), a.mHW, a.sHW) : 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int nl = r * 16 + kq * 4, n = nb + nl;
                float4 v = add4(f4(acc[j][r]), ld4f(a.bias + n));
                if (a.bias_img) v = add4(v, ld4f(a.bias_img + (size_t)pimg * a.bias_img_stride + n));
                if (a.act == 1 || a.act == 2) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
                if (a.act == 2) v = make_float4(fminf(v.x, 6.f), fminf(v.y, 6.f), fminf(v.z, 6.f), fminf(v.w, 6.f));
                *reinterpret_cast<float4 *>(stg + (jj * 16 + col) * DL_STG_RS + nl) = v;
            }
        }
        wave_lds_sync();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int pl = it * 8 + (lane >> 3);
            const int p = p0 + wm * 64 + h * 32 + pl;
            if (p >= a.M || !cok) continue;
            float4 v0 = *reinterpret_cast<const float4 *>(stg + pl * DL_STG_RS + c8);
            float4 v1 = *reinterpret_cast<const float4 *>(stg + pl * DL_STG_RS + c8 + 4);
            const int n = nb + c8;
            if (RPF) {
                const uint4 u = rres[h][it];
                v0 = add4(v0, make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                          __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)));
                v1 = add4(v1, make_float4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u),
                                          __uint_as_float(u.w << 16), __uint_as_float(u.w & 0xffff0000u)));
            }
            if (a.act == 3) {              // ReLU after the residual add (ResNet units)
                v0 = make_float4(fmaxf(v0.x, 0.f), fmaxf(v0.y, 0.f), fmaxf(v0.z, 0.f), fmaxf(v0.w, 0.f));
                v1 = make_float4(fmaxf(v1.x, 0.f), fmaxf(v1.y, 0.f), fmaxf(v1.z, 0.f), fmaxf(v1.w, 0.f));
            }
            if constexpr (OUTF32) {
                float *o = reinterpret_cast<float *>(a.out) + (size_t)p * a.out_cs + a.out_off + n;
                st4(o, v0);
                st4(o + 4, v1);
            } else {
                __bf16 *o = reinterpret_cast<__bf16 *>(a.out) + (size_t)p * a.out_cs + a.out_off + n;
                st4(o, v0);
                st4(o + 4, v1);
            }
        }
    }
}

template <bool OUTF32, bool CONV, bool RPF, int TPX = G2_T>
__global__ void __launch_bounds__(256, 2) dl_gemm128_kernel(const DlConvArgs a) {
    g2_body<OUTF32, CONV, RPF, TPX>(a, xcd_block(blockIdx.x, gridDim.x));
}

// Grouped launch: n convolutions of one shape (the ASPP's atrous branches: same input, same output
// buffer at their own channel offsets, their own rates and weights) as one grid, branch = logical
// block / tiles — 3 x 274 tiles at B = 16 fill the chip where each alone left half the slots idle.
template <bool CONV, int TPX>
__global__ void __launch_bounds__(256, 2) dl_gemm128_group_kernel(const DlConvGroup g) {
    const int L = xcd_block(blockIdx.x, gridDim.x), gi = L / g.tiles;
    g2_body<false, CONV, false, TPX>(g.a[gi], L - gi * g.tiles);
}

// (Round 3 measured three other tilings of these shapes, all bit-identical and all slower, and removed
// them: 3-5 stage buffers of 32 channels on the 128 x 128 tile, 4,863 -> 5,211-5,644 us per Xception-65
// forward at B = 32 (a 32-channel stage fetches every 128-B line as two 64-B halves, and more stages do
// not help a delivery-bound tile); a 256 x 128 tile two per CU, 4,797 -> 4,866 us; a 256 x 256 tile one
// per CU, 4.87 -> 5.27 ms (its barriers, epilogue and first-stage latency are no longer hidden by a
// co-resident workgroup, and 411 tiles on 256 CUs quantise to 2 rounds).)

// ------------------------------------------------------------------ depthwise 3x3
// One thread = one output pixel x 8 channels; threads with consecutive ids take consecutive channel
// groups of the same pixel (coalesced 16-B loads). Weights [9][C] f32 (already rounded to T's
// precision on the host), loaded per in-range tap; bias [C]. Sum in tap order (ky, kx), then bias,
// ReLU6. Measured variants (per 16-frame 513x513 forward, 17 launches): one pixel per thread with f32
// weights 1.09 ms (L1-bound: 48 B of loads per tap and lane, two thirds of them weights); all 72
// weights hoisted into registers 1.41 ms; 4 output pixels per thread sharing them 1.36 ms.
// 8 consecutive elements -> two float4, one 16-B load for bf16
__device__ __forceinline__ void ld8f(const __bf16 *p, float4 &a, float4 &b) {
    const uint4 u = *reinterpret_cast<const uint4 *>(p);
    a = unpack_bf16x4((u32x2_t){u.x, u.y});
    b = unpack_bf16x4((u32x2_t){u.z, u.w});
}
__device__ __forceinline__ void ld8f(const float *p, float4 &a, float4 &b) {
    a = ld4f(p);
    b = ld4f(p + 4);
}

// Two output rows per thread: rows r1 and r1 + ph where ph = the dilation for stride 1 (their taps
// share two of three input rows) and 1 for stride 2; each 16-B weight load (T, per tap) serves both.
// Row slots: slot yq -> block yq / ph, phase yq % ph, r1 = block * 2ph + phase; every row exactly once.
// The two rows' taps overlap in input rows (stride 1: rows r1 + {0,1,2} d and r1 + {1,2,3} d, two
// shared; stride 2: 2 r1 + {0,1,2} and 2 r1 + {2,3,4}, one shared), so each distinct input row-tap is
// loaded (and unpacked) once: 12 or 15 activation loads instead of 18. FMAs go two channels per
// v_pk_fma_f32 (each lane an IEEE fma, so the sums equal the scalar fmaf chain bit for bit).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 relu4(float4 v) {
    return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
}

// ACT: 0 none, 1 ReLU, 2 ReLU6; IRELU: ReLU on the loaded input (compile-time: a runtime switch
// pushed the R = 8 form from 246 VGPRs into scratch spills)
template <typename T, bool S1, int R, int ACT, bool IRELU>
__global__ void __launch_bounds__(256) dl_dw_kernel(const DlDwArgs a) {
    constexpr int NR = S1 ? R + 2 : 2 * R + 1;   // distinct input rows of the R output rows
    constexpr int RB = S1 ? 1 : 2;               // row index offset between consecutive output rows
    const int i = xcd_block(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
    const int groups = a.C >> 3;
    const int ph = S1 ? a.dil : 1;
    const int slots = (a.Hout + R * ph - 1) / (R * ph) * ph;
    if (i >= a.B * slots * a.Wout * groups) return;
    const int g = i % groups, q = i / groups;
    const int ox = q % a.Wout, t = q / a.Wout;
    const int yq = t % slots, b = t / slots;
    const int r1 = (yq / ph) * R * ph + yq % ph;  // output rows r1 + j ph, j < R
    if (r1 >= a.Hout) return;
    const int ix0 = ox * a.stride - a.pad_l;
    const int iy1 = r1 * a.stride - a.pad_t;
    const int rstep = S1 ? a.dil : 1;            // input-row distance between consecutive distinct rows
    const int rows_in = min(NR, S1 ? (a.Hout - r1 + ph - 1) / ph + 2 : 2 * ((a.Hout - r1 + ph - 1) / ph) + 1);
    const T *wt = reinterpret_cast<const T *>(a.w) + g * 8;
    f32x2_t acc[R][4];
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[j][c] = (f32x2_t){0.f, 0.f};
    auto fma8 = [](f32x2_t (&ac)[4], float4 x0, float4 x1, float4 w0, float4 w1) {
        ac[0] = __builtin_elementwise_fma((f32x2_t){x0.x, x0.y}, (f32x2_t){w0.x, w0.y}, ac[0]);
        ac[1] = __builtin_elementwise_fma((f32x2_t){x0.z, x0.w}, (f32x2_t){w0.z, w0.w}, ac[1]);
        ac[2] = __builtin_elementwise_fma((f32x2_t){x1.x, x1.y}, (f32x2_t){w1.x, w1.y}, ac[2]);
        ac[3] = __builtin_elementwise_fma((f32x2_t){x1.z, x1.w}, (f32x2_t){w1.z, w1.w}, ac[3]);
    };
    // branch-free: a padding tap's offset is out of the descriptor's range and reads 0; adding the
    // zero product leaves the sum unchanged (+0 + -0 = +0), so this matches the skipping form bit for
    // bit, and every load can be in flight together
    const __amdgpu_buffer_rsrc_t rin = mkbuf(a.in, a.in_bytes);
    const uint32_t cb = (uint32_t)((size_t)b * a.Hin * a.Win * a.C + g * 8);
    typename Tr<T>::Raw xr[NR][3], wr[9];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const int y = iy1 + k * rstep;
        // rows only output rows past the bottom edge would read are skipped
        const bool oky = k < rows_in && (unsigned)y < (unsigned)a.Hin;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int ix = ix0 + kx * a.dil;
            const bool ok = oky && (unsigned)ix < (unsigned)a.Win;
            bld8(xr[k][kx], rin, ok ? (cb + (uint32_t)((y * a.Win + ix) * a.C)) * (uint32_t)sizeof(T) : OOB);
        }
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) ld8(wr[t], wt + t * a.C);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t % 3;
        float4 w0, w1, x0, x1;
        raw4(wr[t], w0, w1);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            raw4(xr[ky + j * RB][kx], x0, x1);
            if constexpr (IRELU) { x0 = relu4(x0); x1 = relu4(x1); }   // padding taps are 0 either way
            fma8(acc[j], x0, x1, w0, w1);
        }
    }
    float4 b0, b1;
    ld8f(reinterpret_cast<const float *>(a.bias) + g * 8, b0, b1);
    auto r6 = [](float v) {
        if constexpr (ACT == 2) return fminf(fmaxf(v, 0.f), 6.f);
        else if constexpr (ACT == 1) return fmaxf(v, 0.f);
        else return v;
    };
    T *o = reinterpret_cast<T *>(a.out) + (size_t)b * a.Hout * a.Wout * a.C + g * 8;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int r = r1 + j * ph;
        if (r < a.Hout) {
            T *oj = o + ((size_t)r * a.Wout + ox) * a.C;
            st4(oj, make_float4(r6(acc[j][0].x + b0.x), r6(acc[j][0].y + b0.y), r6(acc[j][1].x + b0.z), r6(acc[j][1].y + b0.w)));
            st4(oj + 4, make_float4(r6(acc[j][2].x + b1.x), r6(acc[j][2].y + b1.y), r6(acc[j][3].x + b1.z), r6(acc[j][3].y + b1.w)));
        }
    }
}

// ------------------------------------------------------------------ image pooling
// Partial channel sums over a fixed pixel chunk per workgroup: part[b][chunk][c] (f32). Thread =
// 8 channels (one 16-B load per pixel) x one of `lanes` pixel lanes striding the chunk; the lanes'
// sums are added in lane order through LDS (deterministic, no atomics). Needs C % 8 == 0, C <= 2048.
template <typename T>
__global__ void __launch_bounds__(256) dl_gap_kernel(const DlPoolArgs a) {
    __shared__ float red[256 * 8];
    const int b = blockIdx.y, chunk = blockIdx.x;
    const int HW = a.H * a.W;
    const int p0 = chunk * a.chunk_px, p1 = min(HW, p0 + a.chunk_px);
    const int groups = a.C >> 3, lanes = 256 / groups;
    const int g = threadIdx.x % groups, l = threadIdx.x / groups;
    if (l < lanes) {
        const T *x = reinterpret_cast<const T *>(a.x) + (size_t)b * HW * a.CS + g * 8;
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
        for (int p = p0 + l; p < p1; p += lanes) {
            typename Tr<T>::Raw r;
            ld8(r, x + (size_t)p * a.CS);
            float4 u, v;
            raw4(r, u, v);
            s[0] += u.x; s[1] += u.y; s[2] += u.z; s[3] += u.w;
            s[4] += v.x; s[5] += v.y; s[6] += v.z; s[7] += v.w;
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) red[(l * groups + g) * 8 + c] = s[c];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.C; c += 256) {
        float acc = 0.f;
        for (int k = 0; k < lanes; ++k) acc += red[(k * groups + (c >> 3)) * 8 + (c & 7)];
        a.part[((size_t)b * a.nchunks + chunk) * a.C + c] = acc;
    }
}

// Mean per (image, channel): partials summed in a fixed order, rounded to T as a stored tensor would
// be; written over chunk 0 of the partials (each thread reads its own channel's column first).
template <typename T>
__global__ void __launch_bounds__(256) dl_pool_mean_kernel(const DlPoolArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.B * a.C) return;
    const int b = i / a.C, c = i - b * a.C;
    const float inv = 1.0f / (float)(a.H * a.W);
    // eight interleaved partial sums (chunk k into lane k % 8), then added in lane order: eight loads
    // in flight instead of a chain of nchunks dependent ones (18 -> 5.5 us at 67 chunks x 16 x 320)
    float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float *pp = a.part + (size_t)b * a.nchunks * a.C + c;
    int k = 0;
    for (; k + 8 <= a.nchunks; k += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] += pp[(size_t)(k + u) * a.C];
    }
    for (int u = 0; k < a.nchunks; ++k, ++u) q[u] += pp[(size_t)k * a.C];
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += q[u];
    a.part[(size_t)b * a.nchunks * a.C + c] = (float)(T)(s * inv);
}

// One wave per output (image b, row m): out[b][m] = W[m] . in[b] + bias[m] (lanes stride the input,
// butterfly reduction); stage 0: the image-pooling 1x1 (ReLU, rounded to T) into y; stage 1: its
// columns of the concat projection plus the projection bias -> the per-image bias z.
template <typename T, int STAGE>
__global__ void __launch_bounds__(256) dl_pool_gemv_kernel(const DlPoolArgs a) {
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int rows = STAGE == 0 ? a.cmid : a.cout, cols = STAGE == 0 ? a.C : a.cmid;
    if (wv >= a.B * rows) return;
    const int b = wv / rows, m = wv - b * rows;
    const float *w = (STAGE == 0 ? a.wp : a.wq) + (size_t)m * cols;
    const float *in = STAGE == 0 ? a.part + (size_t)b * a.nchunks * a.C : a.y + (size_t)b * a.cmid;
    float s = 0.f;
    for (int c = lane; c < cols; c += 64) s = fmaf(w[c], in[c], s);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) {
        if (STAGE == 0) a.y[(size_t)b * a.cmid + m] = (float)(T)fmaxf(s + a.bp[m], 0.f);
        else a.z[(size_t)b * a.z_stride + m] = s + a.bq[m];
    }
}

// ------------------------------------------------------------------ logits -> class map
// TF resize_bilinear (align_corners = True, legacy scaler): in = out * ((in_size - 1) / (out_size - 1))
// in f32; top = floor(in), bottom = min(top + 1, in_size - 1), lerp = in - top;
// value = top_row + (bottom_row - top_row) * y_lerp with row = left + (right - left) * x_lerp.
// Then argmax over classes (first maximum).
constexpr int AM_PX = 8, AM_PY = 1, AM_C = 24;   // classes held in registers (LCS <= AM_C uses this kernel)
// Round 6 (MobileNetV2 B = 64, per-op HIP events): the class loops fully unrolled (no s_set_gpr_idx),
// the corner differences once per cell and packed f32 lerps: 140 -> 102-108 us; the same without the
// class loop (AM_ABL = 1) 42 us. Tried and dropped: the logit rows staged in LDS per 8-row workgroup
// (252 us) and wave-staged whole-line stores (142 us, with the rolled loop).
#ifndef AM_OPT
#define AM_OPT 1   // corner differences once per cell + packed f32 lerps (0: the per-pixel scalar chain)
#endif
#ifndef AM_ABL
#define AM_ABL 0   // debug ablation (wrong classes): 1 = no class loop
#endif
// One thread = AM_PX consecutive output pixels in each of AM_PY consecutive rows; the 4 corner logit
// vectors are reloaded only when the corner cell (x0, y0) changes (at the 65 -> 513 scale of 1/8, once
// per 8 pixels of a row). Class ids of a run go out as 16-B stores (two int64) where the address
// allows (46 -> 44 us). Measured at B = 64: AM_PY = 2 167 us, AM_PY = 4 (B = 16) 66 vs 44 us, AM_PX = 4
// 149 vs 148 us — fewer threads cost more than the L2 corner reads they save.
__global__ void __launch_bounds__(256) dl_resize_argmax_kernel(const DlArgmaxArgs a) {
#pragma clang fp contract(off)
    const int qx = (a.Wo + AM_PX - 1) / AM_PX, qy = (a.Ho + AM_PY - 1) / AM_PY;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.B * qy * qx) return;
    const int xq = i % qx, t = i / qx, yq = t % qy, b = t / qy;
    const float *base = a.logits + (size_t)b * a.h * a.w * a.LCS;
    float tl[AM_C], tr[AM_C], bl[AM_C], br[AM_C];
    int curx = -1, cury = -1;
    const int xb = xq * AM_PX, nx = min(AM_PX, a.Wo - xb);
    for (int r = 0; r < AM_PY; ++r) {
        const int y = yq * AM_PY + r;
        if (y >= a.Ho) break;
        const float in_y = (float)y * a.sy;
        const int y0 = (int)floorf(in_y), y1 = min(y0 + 1, a.h - 1);
        const float ly = in_y - (float)y0;
        const float *row0 = base + (size_t)y0 * a.w * a.LCS, *row1 = base + (size_t)y1 * a.w * a.LCS;
        uint32_t packed[2] = {0u, 0u};      // the run's class ids, one byte each (ncls <= AM_C < 256)
        for (int j = 0; j < nx; ++j) {
            const int x = xb + j;
            const float in_x = (float)x * a.sx;
            const int x0 = (int)floorf(in_x), x1 = min(x0 + 1, a.w - 1);
            const float lx = in_x - (float)x0;
            if (x0 != curx || y0 != cury) {
                curx = x0;
                cury = y0;
                // every loop over classes is fully unrolled with predicates, not a runtime break: a
                // partly rolled loop indexes tl[] .. br[] with s_set_gpr_idx (serialising), the form
                // the kernel had until round 6
#pragma unroll
                for (int c0 = 0; c0 < AM_C; c0 += 4) {
                    const bool in = c0 < a.LCS;
                    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
                    const float4 q0 = in ? ld4f(row0 + x0 * a.LCS + c0) : z, q1 = in ? ld4f(row0 + x1 * a.LCS + c0) : z;
                    const float4 q2 = in ? ld4f(row1 + x0 * a.LCS + c0) : z, q3 = in ? ld4f(row1 + x1 * a.LCS + c0) : z;
                    tl[c0] = q0.x; tl[c0 + 1] = q0.y; tl[c0 + 2] = q0.z; tl[c0 + 3] = q0.w;
                    tr[c0] = q1.x; tr[c0 + 1] = q1.y; tr[c0 + 2] = q1.z; tr[c0 + 3] = q1.w;
                    bl[c0] = q2.x; bl[c0 + 1] = q2.y; bl[c0 + 2] = q2.z; bl[c0 + 3] = q2.w;
                    br[c0] = q3.x; br[c0 + 1] = q3.y; br[c0 + 2] = q3.z; br[c0 + 3] = q3.w;
                }
#if AM_OPT
                // the corner differences once per cell (the same f32 subtractions TF's lerp does per pixel)
#pragma unroll
                for (int c = 0; c < AM_C; ++c) {
                    tr[c] = tr[c] - tl[c];
                    br[c] = br[c] - bl[c];
                }
#endif
            }
            float best = 0.f;
            int bi = 0;
#if AM_ABL
            best = lx + ly;
#elif AM_OPT
            // two classes per packed f32 op (v_pk_mul_f32 / v_pk_add_f32: per-lane IEEE, as the scalar chain)
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 lx2 = {lx, lx}, ly2 = {ly, ly};
#pragma unroll
            for (int c = 0; c < AM_C; c += 2) {
                const f2 t2 = (f2){tl[c], tl[c + 1]} + (f2){tr[c], tr[c + 1]} * lx2;
                const f2 b2 = (f2){bl[c], bl[c + 1]} + (f2){br[c], br[c + 1]} * lx2;
                const f2 v2 = t2 + (b2 - t2) * ly2;
                if (c == 0 || (c < a.ncls && v2.x > best)) { best = v2.x; bi = c; }
                if (c + 1 < a.ncls && v2.y > best) { best = v2.y; bi = c + 1; }
            }
#else
#pragma unroll
            for (int c = 0; c < AM_C; ++c) {
                if (c >= a.ncls) break;
                const float top = tl[c] + (tr[c] - tl[c]) * lx;
                const float bot = bl[c] + (br[c] - bl[c]) * lx;
                const float v = top + (bot - top) * ly;
                if (c == 0 || v > best) { best = v; bi = c; }
            }
#endif
            if (j < 4) packed[0] |= (uint32_t)bi << (8 * j);
            else packed[1] |= (uint32_t)bi << (8 * (j - 4));
        }
        int res[AM_PX];
#pragma unroll
        for (int j = 0; j < AM_PX; ++j) res[j] = (int)((packed[j >> 2] >> (8 * (j & 3))) & 0xffu);
        // rows of odd width start 8-B aligned: a misaligned run writes its first and last pixel alone
        // and the six between in pairs
        int64_t *o = a.out + ((size_t)b * a.Hout + y) * a.Wout + xb;
        auto st2 = [](int64_t *p, int u, int v) {
            *reinterpret_cast<longlong2 *>(p) = make_longlong2((long long)u, (long long)v);
        };
        if (nx == AM_PX) {
            if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
#pragma unroll
                for (int j = 0; j < AM_PX; j += 2) st2(o + j, res[j], res[j + 1]);
            } else {
                o[0] = res[0];
#pragma unroll
                for (int j = 1; j < AM_PX - 1; j += 2) st2(o + j, res[j], res[j + 1]);
                o[AM_PX - 1] = res[AM_PX - 1];
            }
        } else {
#pragma unroll
            for (int j = 0; j < AM_PX; ++j)
                if (j < nx) o[j] = res[j];
        }
    }
}

// Any class count: one thread per output pixel, float4 corner loads.
__global__ void __launch_bounds__(256) dl_resize_argmax_generic(const DlArgmaxArgs a) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.B * a.Ho * a.Wo) return;
    const int x = i % a.Wo, t = i / a.Wo, y = t % a.Ho, b = t / a.Ho;
    const float in_y = (float)y * a.sy, in_x = (float)x * a.sx;
    const int y0 = (int)floorf(in_y), x0 = (int)floorf(in_x);
    const int y1 = min(y0 + 1, a.h - 1), x1 = min(x0 + 1, a.w - 1);
    const float ly = in_y - (float)y0, lx = in_x - (float)x0;
    const float *base = a.logits + (size_t)b * a.h * a.w * a.LCS;
    const float *tl = base + ((size_t)y0 * a.w + x0) * a.LCS, *tr = base + ((size_t)y0 * a.w + x1) * a.LCS;
    const float *bl = base + ((size_t)y1 * a.w + x0) * a.LCS, *br = base + ((size_t)y1 * a.w + x1) * a.LCS;
    float best = 0.f;
    int bi = 0;
    // LCS is a multiple of 4 and every row 16-B aligned: 4 classes per corner load
    for (int c0 = 0; c0 < a.ncls; c0 += 4) {
        const float4 q[4] = {ld4f(tl + c0), ld4f(tr + c0), ld4f(bl + c0), ld4f(br + c0)};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = c0 + j;
            if (c >= a.ncls) break;
            const float vtl = get(q[0], j), vtr = get(q[1], j), vbl = get(q[2], j), vbr = get(q[3], j);
            const float top = vtl + (vtr - vtl) * lx;
            const float bot = vbl + (vbr - vbl) * lx;
            const float v = top + (bot - top) * ly;
            if (c == 0 || v > best) { best = v; bi = c; }
        }
    }
    a.out[((size_t)b * a.Hout + y) * a.Wout + x] = (int64_t)bi;
}

// Feature resize for the decoder: one thread = 8 channels of one output pixel; the four corner
// vectors are 16-B (bf16) / 2 x 16-B (f32) loads; contraction off so the lerps round as TF's do.
template <typename T>
__global__ void __launch_bounds__(256) dl_resize_kernel(const DlResizeArgs a) {
#pragma clang fp contract(off)
    const int groups = a.C >> 3;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.B * a.Ho * a.Wo * groups) return;
    const int g = i % groups, q = i / groups;
    const int x = q % a.Wo, t = q / a.Wo, y = t % a.Ho, b = t / a.Ho;
    const float in_y = (float)y * a.sy, in_x = (float)x * a.sx;
    const int y0 = (int)floorf(in_y), x0 = (int)floorf(in_x);
    const int y1 = min(y0 + 1, a.h - 1), x1 = min(x0 + 1, a.w - 1);
    const float ly = in_y - (float)y0, lx = in_x - (float)x0;
    const T *base = reinterpret_cast<const T *>(a.in) + (size_t)b * a.h * a.w * a.in_cs + g * 8;
    using Raw = typename Tr<T>::Raw;
    Raw r[4];
    ld8(r[0], base + ((size_t)y0 * a.w + x0) * a.in_cs);
    ld8(r[1], base + ((size_t)y0 * a.w + x1) * a.in_cs);
    ld8(r[2], base + ((size_t)y1 * a.w + x0) * a.in_cs);
    ld8(r[3], base + ((size_t)y1 * a.w + x1) * a.in_cs);
    float4 v[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k) raw4(r[k], v[k][0], v[k][1]);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float tl = get(v[0][j >> 2], j & 3), tr = get(v[1][j >> 2], j & 3);
        const float bl = get(v[2][j >> 2], j & 3), br = get(v[3][j >> 2], j & 3);
        const float top = tl + (tr - tl) * lx;
        const float bot = bl + (br - bl) * lx;
        o[j] = top + (bot - top) * ly;
    }
    T *op = reinterpret_cast<T *>(a.out) + (((size_t)b * a.Ho + y) * a.Wo + x) * a.out_cs + a.out_off + g * 8;
    st4(op, make_float4(o[0], o[1], o[2], o[3]));
    st4(op + 4, make_float4(o[4], o[5], o[6], o[7]));
}

// Max pooling (DlMaxPoolArgs): one thread = 8 channels of one output pixel; the taps inside the input
// only (TF pads max pooling with -inf); the result is one of the inputs, so it is exact in T
template <typename T>
__global__ void __launch_bounds__(256) dl_maxpool_kernel(const DlMaxPoolArgs a) {
    const int groups = a.C >> 3;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.B * a.Hout * a.Wout * groups) return;
    const int g = i % groups, q = i / groups;
    const int x = q % a.Wout, t = q / a.Wout, y = t % a.Hout, b = t / a.Hout;
    const T *base = reinterpret_cast<const T *>(a.in) + (size_t)b * a.Hin * a.Win * a.C + g * 8;
    using Raw = typename Tr<T>::Raw;
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    for (int dy = 0; dy < a.k; ++dy) {
        const int iy = y * a.stride - a.pad_t + dy;
        if ((unsigned)iy >= (unsigned)a.Hin) continue;
        for (int dx = 0; dx < a.k; ++dx) {
            const int ix = x * a.stride - a.pad_l + dx;
            if ((unsigned)ix >= (unsigned)a.Win) continue;
            Raw r;
            ld8(r, base + ((size_t)iy * a.Win + ix) * a.C);
            float4 v[2];
            raw4(r, v[0], v[1]);
#pragma unroll
            for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], get(v[j >> 2], j & 3));
        }
    }
    T *op = reinterpret_cast<T *>(a.out) + (((size_t)b * a.Hout + y) * a.Wout + x) * a.C + g * 8;
    st4(op, make_float4(m[0], m[1], m[2], m[3]));
    st4(op + 4, make_float4(m[4], m[5], m[6], m[7]));
}

// ------------------------------------------------------------------ launchers
hipError_t dl_launch_prep(int prec, const DlPrepArgs &a, hipStream_t s) {
    const int n = a.B * a.Hc * a.Wc;
    const dim3 g((n + 255) / 256);
    if (prec == PREC_BF16) hipLaunchKernelGGL(dl_prep_kernel<__bf16>, g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(dl_prep_kernel<float>, g, dim3(256), 0, s, a);
    return hipGetLastError();
}

// k-step prefetch depth of the bf16 conv (template PD): BUGSEG_DL_PD=1|2|3 forces one for A/B runs
static int conv_pd(const DlConvArgs &a, int nb) {
    static const int env = [] { const char *e = std::getenv("BUGSEG_DL_PD"); return e ? std::atoi(e) : 0; }();
    if (env >= 1 && env <= 3) return env;
    (void)a; (void)nb;
    // measured (16 frames, 513x513, per-op HIP events): two steps ahead is 1.3% faster over the 38
    // conv launches than one (1609 vs 1631 us); three is between (1620 us); no op gains more than 3%
    return 2;
}

template <int NB, int PD>
static void conv_bf16(bool out_f32, const DlConvArgs &a, const dim3 g, hipStream_t s) {
    if (out_f32) hipLaunchKernelGGL((dl_conv_kernel<__bf16, true, false, NB, PD>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dl_conv_kernel<__bf16, false, false, NB, PD>), g, dim3(256), 0, s, a);
}

template <int NB>
static void conv_nb(int prec, bool out_f32, bool dwf, const DlConvArgs &a, hipStream_t s) {
    const dim3 g(((a.M + NB * 64 - 1) / (NB * 64)) * (a.NP / 64));
    if (prec == PREC_BF16 && !dwf) {   // NB = 8: bf16 only, no depthwise fusion (register budget)
        const int pd = a.tap_packed ? 1 : conv_pd(a, NB);
        if (pd == 3) conv_bf16<NB, 3>(out_f32, a, g, s);
        else if (pd == 2) conv_bf16<NB, 2>(out_f32, a, g, s);
        else conv_bf16<NB, 1>(out_f32, a, g, s);
    } else if constexpr (NB == 8) {
        return;
    } else if (prec == PREC_BF16) {
        hipLaunchKernelGGL((dl_conv_kernel<__bf16, false, true, NB>), g, dim3(256), 0, s, a);
    } else {
        if (dwf) hipLaunchKernelGGL((dl_conv_kernel<float, false, true, NB>), g, dim3(256), 0, s, a);
        else if (out_f32) hipLaunchKernelGGL((dl_conv_kernel<float, true, false, NB>), g, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((dl_conv_kernel<float, false, false, NB>), g, dim3(256), 0, s, a);
    }
}

// the LDS-staged GEMM form applies to plain 1x1 convolutions (bf16; BUGSEG_DL_GEMM=0 turns it off)
static bool gemm_ok(int prec, const DlConvArgs &a) {
    const char *e = std::getenv("BUGSEG_DL_GEMM");
    if (e && *e == '0') return false;
    return prec == PREC_BF16 && !a.dw_w && !a.tap_packed && a.kh == 1 && a.kw == 1 && a.stride == 1 && a.pad_t == 0 &&
           a.pad_l == 0 && a.Hin == a.Hout && a.Win == a.Wout && a.cinP % 32 == 0 && a.NP % 64 == 0 &&
           (size_t)a.NP * a.cinP * 2 < ((size_t)1 << 31);
}

// the 128 x 128 glds tile for deep, wide 1x1s (K >= 256 and 256+ output rows in whole 128-row tiles;
// BUGSEG_DL_G128=0 turns it off). Measured (per-op HIP events): Xception's pointwise layers 3.14 ->
// 2.60 ms per 16-frame forward (462 -> 558 TFLOP/s), the ASPP 1x1s 3% faster; MobileNetV2's
// 576 / 960 -> 96..320 projections (HBM-bound, NP % 128 = 64) 1-8% slower, so they stay on
// dl_gemm_kernel
static bool gemm128_ok(const DlConvArgs &a) {
    const char *e = std::getenv("BUGSEG_DL_G128");
    return !(e && *e == '0') && a.cinP >= 256 && a.NP >= 256 && a.NP % 128 == 0 && a.CS % 8 == 0;
}

// implicit-GEMM k x k conv on the glds tile: bf16, dense (not tap-packed, no fused depthwise), every
// 64-channel k-stage inside one tap (cinP = CS, a multiple of 64); 128 x 128 tiles when the outputs
// come in whole 128-channel tiles, else 256 pixels x 64 channels. BUGSEG_DL_IG=0 sends these to
// dl_conv_kernel for A/B runs, BUGSEG_DL_IG64=0 only the 64-channel ones. Measured (ResNet-101, B = 16,
// per-op HIP events): the implicit GEMM 1,723 -> 2,827 frames/s (3x3s 3,826 -> 1,715 us, ASPP atrous
// 1,859 -> 847, root 825 -> 518); the 256 x 64 tile for the 64-channel root / block-1 convs then
// 2,827 -> 2,939 (root 518 -> 390 us, 3x3s 1,715 -> 1,633)
static bool igemm_ok(int prec, const DlConvArgs &a) {
    const char *e = std::getenv("BUGSEG_DL_IG"), *e64 = std::getenv("BUGSEG_DL_IG64");
    const bool ig64 = !(e64 && *e64 == '0');
    return !(e && *e == '0') && (ig64 || a.NP % 128 == 0) && prec == PREC_BF16 && !a.dw_w && !a.tap_packed &&
           a.taps > 1 && a.zero && a.cinP == a.CS && a.cinP % 64 == 0 && a.NP % 64 == 0 &&
           (size_t)a.NP * a.taps * a.cinP * 2 < ((size_t)1 << 31);
}

template <bool CONV, int TPX>
static void launch_g2(bool out_f32, const DlConvArgs &a, hipStream_t s) {
    const dim3 g(((a.M + TPX - 1) / TPX) * ((a.NP + G2_T * G2_T / TPX - 1) / (G2_T * G2_T / TPX)));
    if (a.res) {
        if (out_f32) hipLaunchKernelGGL((dl_gemm128_kernel<true, CONV, true, TPX>), g, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((dl_gemm128_kernel<false, CONV, true, TPX>), g, dim3(256), 0, s, a);
    } else {
        if (out_f32) hipLaunchKernelGGL((dl_gemm128_kernel<true, CONV, false, TPX>), g, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((dl_gemm128_kernel<false, CONV, false, TPX>), g, dim3(256), 0, s, a);
    }
}

hipError_t dl_launch_conv_group(int prec, const DlConvGroup &g, hipStream_t s) {
    if (g.n < 2 || g.n > DL_GROUP_MAX) return hipErrorNotSupported;
    for (int i = 0; i < g.n; ++i) {
        const DlConvArgs &a = g.a[i];
        if (!igemm_ok(prec, a) || a.res || a.NP % 128 || a.M != g.a[0].M || a.NP != g.a[0].NP) return hipErrorNotSupported;
    }
    DlConvGroup h = g;
    h.tiles = ((g.a[0].M + G2_T - 1) / G2_T) * (g.a[0].NP / G2_T);
    hipLaunchKernelGGL((dl_gemm128_group_kernel<true, 128>), dim3(h.tiles * g.n), dim3(256), 0, s, h);
    return hipGetLastError();
}

hipError_t dl_launch_conv(int prec, bool out_f32, const DlConvArgs &a, hipStream_t s) {
    const bool dwf = a.dw_w != nullptr;
    if (igemm_ok(prec, a)) {
        if (a.NP % 128 == 0) launch_g2<true, 128>(out_f32, a, s);
        else launch_g2<true, 256>(out_f32, a, s);
        return hipGetLastError();
    }
    if (gemm_ok(prec, a) && gemm128_ok(a)) {
        launch_g2<false, 128>(out_f32, a, s);
        return hipGetLastError();
    }
    if (const char *e = std::getenv("BUGSEG_DL_G2ALL"); e && *e != '0' && gemm_ok(prec, a) && a.CS % 8 == 0) {
        // (A/B knob) every other 1x1 on the glds tile: 1 = 128 x 128 where the outputs come in 128s,
        // else 256 x 64; 2 = 256 x 64 always
        if ((*e == '1' && a.NP % 128 == 0) || *e == '3') launch_g2<false, 128>(out_f32, a, s);
        else launch_g2<false, 256>(out_f32, a, s);
        return hipGetLastError();
    }
    if (gemm_ok(prec, a)) {
        const dim3 g(((a.M + GM_TM - 1) / GM_TM) * (a.NP / GM_TN));
        const char *pe = std::getenv("BUGSEG_DL_GPD2"), *te = std::getenv("BUGSEG_DL_GTM");
        const bool pd2 = pe && *pe == '1' && a.cinP > GM_KT;
        // 128-pixel tiles below 2^19 output pixels (BUGSEG_DL_GTM=0 / 1 forces 256 / 128). Measured
        // (per-op HIP events): MobileNetV2 B = 64 9,240 -> 9,430 frames/s (the 65x65 projections
        // 110 -> 97 us, 212 -> 184 us; the 257^2 / 129^2 layers are slower with 128, hence the bound);
        // ResNet-101 B = 16 and Xception-65 B = 32 within +-0.3%. PD2 (BUGSEG_DL_GPD2=1: a second stage
        // in flight in registers) measured slower: 9,220 -> 8,935 (196-234 VGPRs: 2 workgroups per CU)
        const bool tm128 = te ? *te == '1' : a.M <= (1 << 19);
        if (tm128 && !pd2) {
            const dim3 g1(((a.M + 127) / 128) * (a.NP / GM_TN));
            if (a.res) {
                if (out_f32) hipLaunchKernelGGL((dl_gemm_kernel<true, true, false, 128>), g1, dim3(256), 0, s, a);
                else hipLaunchKernelGGL((dl_gemm_kernel<false, true, false, 128>), g1, dim3(256), 0, s, a);
            } else {
                if (out_f32) hipLaunchKernelGGL((dl_gemm_kernel<true, false, false, 128>), g1, dim3(256), 0, s, a);
                else hipLaunchKernelGGL((dl_gemm_kernel<false, false, false, 128>), g1, dim3(256), 0, s, a);
            }
        } else if (pd2) {
            if (a.res) {
                if (out_f32) hipLaunchKernelGGL((dl_gemm_kernel<true, true, true>), g, dim3(256), 0, s, a);
                else hipLaunchKernelGGL((dl_gemm_kernel<false, true, true>), g, dim3(256), 0, s, a);
            } else {
                if (out_f32) hipLaunchKernelGGL((dl_gemm_kernel<true, false, true>), g, dim3(256), 0, s, a);
                else hipLaunchKernelGGL((dl_gemm_kernel<false, false, true>), g, dim3(256), 0, s, a);
            }
        } else if (a.res) {
            if (out_f32) hipLaunchKernelGGL((dl_gemm_kernel<true, true>), g, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((dl_gemm_kernel<false, true>), g, dim3(256), 0, s, a);
        } else {
            if (out_f32) hipLaunchKernelGGL((dl_gemm_kernel<true, false>), g, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((dl_gemm_kernel<false, false>), g, dim3(256), 0, s, a);
        }
        return hipGetLastError();
    }
    if (a.nb == 8 && prec == PREC_BF16 && !dwf) conv_nb<8>(prec, out_f32, false, a, s);
    else if (a.nb >= 4) conv_nb<4>(prec, out_f32, dwf, a, s);
    else conv_nb<2>(prec, out_f32, dwf, a, s);
    return hipGetLastError();
}

template <typename T, int R, int ACT, bool IRELU>
static void launch_dw_t(const DlDwArgs &a, const dim3 g, hipStream_t s) {
    if (a.stride == 1) hipLaunchKernelGGL((dl_dw_kernel<T, true, R, ACT, IRELU>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dl_dw_kernel<T, false, R, ACT, IRELU>), g, dim3(256), 0, s, a);
}

// (act, in_relu) forms: MobileNetV2 (ReLU6, -), Xception pre-activation (none, ReLU in), Xception
// activated-inside / ASPP / decoder (ReLU, -)
template <typename T, int R>
static hipError_t launch_dw_a(const DlDwArgs &a, const dim3 g, hipStream_t s) {
    if (a.act == 2 && !a.in_relu) launch_dw_t<T, R, 2, false>(a, g, s);
    else if (a.act == 0 && a.in_relu) launch_dw_t<T, R, 0, true>(a, g, s);
    else if (a.act == 1 && !a.in_relu) launch_dw_t<T, R, 1, false>(a, g, s);
    else if (a.act == 0 && !a.in_relu) launch_dw_t<T, R, 0, false>(a, g, s);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

template <int R>
static hipError_t launch_dw_r(int prec, const DlDwArgs &a, hipStream_t s) {
    const int ph = a.stride == 1 ? a.dil : 1;
    const int n = a.B * ((a.Hout + R * ph - 1) / (R * ph) * ph) * a.Wout * (a.C >> 3);
    const dim3 g((n + 255) / 256);
    return prec == PREC_BF16 ? launch_dw_a<__bf16, R>(a, g, s) : launch_dw_a<float, R>(a, g, s);
}

// Output rows per thread (R). Measured (16 frames, 513x513, per-op HIP events, 17 launches): stride-1
// layers R = 2 / 4 / 8: 680 / 576 / 534 us in total, R = 8 fastest in every layer (246 VGPRs, two waves
// per SIMD); stride 2 keeps R = 2 (R = 4 / 8 within 1%). BUGSEG_DL_DWR=2|4|8 forces R for stride 1.
hipError_t dl_launch_dw(int prec, const DlDwArgs &a, hipStream_t s) {
    if (a.stride != 1 && (a.stride != 2 || a.dil != 1)) return hipErrorInvalidValue;   // TF: no strided atrous
    static const int env = [] { const char *e = std::getenv("BUGSEG_DL_DWR"); return e ? std::atoi(e) : 0; }();
    if (a.stride == 2) return launch_dw_r<2>(prec, a, s);
    if (env == 2) return launch_dw_r<2>(prec, a, s);
    if (env == 4) return launch_dw_r<4>(prec, a, s);
    return launch_dw_r<8>(prec, a, s);
}

hipError_t dl_launch_pool(int prec, const DlPoolArgs &a, hipStream_t s) {
    if ((a.C & 7) || a.C > 2048) return hipErrorInvalidValue;
    const dim3 g1(a.nchunks, a.B);
    if (prec == PREC_BF16) {
        hipLaunchKernelGGL(dl_gap_kernel<__bf16>, g1, dim3(256), 0, s, a);
        hipLaunchKernelGGL(dl_pool_mean_kernel<__bf16>, dim3((a.B * a.C + 255) / 256), dim3(256), 0, s, a);
        hipLaunchKernelGGL((dl_pool_gemv_kernel<__bf16, 0>), dim3((a.B * a.cmid + 3) / 4), dim3(256), 0, s, a);
        hipLaunchKernelGGL((dl_pool_gemv_kernel<__bf16, 1>), dim3((a.B * a.cout + 3) / 4), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(dl_gap_kernel<float>, g1, dim3(256), 0, s, a);
        hipLaunchKernelGGL(dl_pool_mean_kernel<float>, dim3((a.B * a.C + 255) / 256), dim3(256), 0, s, a);
        hipLaunchKernelGGL((dl_pool_gemv_kernel<float, 0>), dim3((a.B * a.cmid + 3) / 4), dim3(256), 0, s, a);
        hipLaunchKernelGGL((dl_pool_gemv_kernel<float, 1>), dim3((a.B * a.cout + 3) / 4), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t dl_launch_maxpool(int prec, const DlMaxPoolArgs &a, hipStream_t s) {
    if ((a.C & 7) || a.k < 1 || a.stride < 1) return hipErrorInvalidValue;
    const int n = a.B * a.Hout * a.Wout * (a.C >> 3);
    if (prec == PREC_BF16) hipLaunchKernelGGL(dl_maxpool_kernel<__bf16>, dim3((n + 255) / 256), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(dl_maxpool_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t dl_launch_resize(int prec, const DlResizeArgs &a, hipStream_t s) {
    if ((a.C & 7) || (a.in_cs & 7) || (a.out_cs & 7) || (a.out_off & 7)) return hipErrorInvalidValue;
    const int n = a.B * a.Ho * a.Wo * (a.C >> 3);
    if (prec == PREC_BF16) hipLaunchKernelGGL(dl_resize_kernel<__bf16>, dim3((n + 255) / 256), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(dl_resize_kernel<float>, dim3((n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t dl_launch_argmax(const DlArgmaxArgs &a, hipStream_t s) {
    if (a.LCS > AM_C) {
        const int n = a.B * a.Ho * a.Wo;
        hipLaunchKernelGGL(dl_resize_argmax_generic, dim3((n + 255) / 256), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    const int n = a.B * ((a.Ho + AM_PY - 1) / AM_PY) * ((a.Wo + AM_PX - 1) / AM_PX);
    hipLaunchKernelGGL(dl_resize_argmax_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace bugseg
