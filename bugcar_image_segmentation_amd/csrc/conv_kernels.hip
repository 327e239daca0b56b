// Implicit-GEMM convolution for gfx950 with the ENet epilogues fused in.
//
// Replaces the TF Conv2D / BN / PReLU / MaxPoolWithArgmax / MaxUnpool / Conv2DBackpropInput /
// ArgMax / SelectV2 kernels that run inside the reference's sess.run + tf.math.argmax
// (models.py:43-58). One launch = one convolution of ENet with everything that consumes its
// output element-wise (bias, activation, residual add, pooling / unpooling of the skip path,
// pixel shuffle of a stride-2 transposed conv, class argmax + remap) done in registers.
//
// Tiling (CDNA4, wave64): a 256-thread workgroup owns 4 * MR * 16 consecutive pixels of the
// GEMM grid; each wave owns MR 16-pixel column fragments and ALL output channels (NR 16-row
// fragments). MFMA v_mfma_f32_16x16x32_bf16 (or 8 x v_mfma_f32_16x16x4_f32 in the fp32 parity
// mode) takes A = weights (row = output channel) and B = pixels (column = pixel), so the
// accumulator puts 4 consecutive channels of one pixel in each lane. The B fragment (8
// consecutive k = 8 channels of one input pixel at one tap) is one 16-byte buffer load per lane
// straight into VGPRs. The layer's weights are staged in LDS once per workgroup; workgroups stride
// over tiles with an XCD-aware mapping.
//
// These layers move little data per pixel, so the VALU instruction count, not HBM, was what bound
// them (SQ counters: VALU-busy time ~ kernel time). The addressing is built to keep it low:
//   * pixel -> (frame, row, col) by magic-number division (2 VALU instead of a ~20-instruction
//     integer division), once per fragment per tile;
//   * the tap table holds each k group's byte delta ((dy*Win + dx)*CinS + c)*es precomputed, so a
//     B-fragment load is base + delta with a 2-compare bounds test, and padding taps / invalid
//     pixels are an out-of-range buffer offset that reads zeros (no branch, no zeroing moves);
//   * the wave index is made provably uniform, so per-fragment output offsets are scalar; the
//     coalesced LDS-staged stores use shifts (chunks per pixel is a power of two) and buffer
//     stores whose out-of-range offsets mask the tail.
#include "bugseg_internal.h"
#include "mfma_common.h"

#include <cstdlib>

namespace bugseg {

template <int NR> struct Cfg { static constexpr int MR = NR >= 4 ? 2 : 4; };

// LDS carve: [weights Npad x (Kpad+pad)] [tap table: Ksteps*4 x int4 {dy, dx, byte delta, 0}]
//            [bias, slope1, slope2: Npad floats each] [class LUT: 16 ints] [4 x output staging]
__host__ __device__ inline size_t conv_tap_offset(int es, const ConvArgs &a) {
    return ((size_t)a.Npad * (a.Kpad + 16 / es) * es + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t conv_const_offset(int es, const ConvArgs &a) {
    return conv_tap_offset(es, a) + (size_t)((a.Ksteps + 3) & ~3) * 4 * 16;   // padded to whole load chunks
}
__host__ __device__ inline size_t conv_stage_offset(int es, const ConvArgs &a) {
    return conv_const_offset(es, a) + (size_t)3 * a.Npad * sizeof(float) + 16 * sizeof(int);
}
constexpr int CLS_STR = 20;            // EPI_CLASSES staging: floats per output pixel (16 classes + pad)
constexpr int TAP_PAD = -(1 << 24);    // row offset of a padding k group / an invalid pixel: every test fails

// bf16: at least 3 (NR 8) / 4 waves per SIMD resident — the kernels are latency- and VALU-bound, so
// occupancy is worth a few registers; fp32 (parity mode) is left to the compiler.
template <typename T, int NR, int EPI>
__global__ void __launch_bounds__(256, sizeof(T) == 2 ? (NR == 8 ? 3 : 4) : 1) conv_kernel(const ConvArgs a) {
    span_enter(a.span);
    constexpr int MR = Cfg<NR>::MR;
    constexpr int TILE = 4 * MR * 16;
    constexpr int ES = (int)sizeof(T), EPC = 16 / ES;
    // k-steps per load chunk: 32 VGPRs of B fragments in flight (bf16; 16 beside NR 8's 64 accumulator
    // VGPRs); fp32 (parity mode) keeps half
    constexpr int KC = ES == 2 ? (MR >= 4 || NR >= 8 ? 2 : 4) : (MR >= 4 || NR >= 8 ? 1 : 2);
    using Raw = typename Tr<T>::Raw;
    using WRaw = typename WTr<T>::Raw;   // weight operand (fp32 mode: split-f16 parts)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63, col = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int KS = a.Kpad + EPC;                                      // LDS row stride (elements)
    T *wl = reinterpret_cast<T *>(smem);
    int4 *gt = reinterpret_cast<int4 *>(smem + conv_tap_offset(ES, a));
    float *cst = reinterpret_cast<float *>(smem + conv_const_offset(ES, a));
    {
        const int cpr = a.Kpad * ES / 16;
        const int total = a.Npad * cpr;
        const uint4 *src = reinterpret_cast<const uint4 *>(a.w);
        for (int i = tid; i < total; i += 256) {
            const int r = i / cpr, c = i - r * cpr;
            *reinterpret_cast<uint4 *>(smem + (size_t)r * KS * ES + c * 16) = src[i];
        }
        for (int i = tid; i < ((a.Ksteps + 3) & ~3) * 4; i += 256) {
            const int g = i < a.Ksteps * 4 ? a.gtab[i] : (int)0xffff0000u;
            const int dy = (int)(signed char)(g & 0xff), dx = (int)(signed char)((g >> 8) & 0xff);
            const int coff = (g >> 16) & 0xffff;
            gt[i] = coff == 0xffff ? make_int4(TAP_PAD, 0, 0, 0)
                                   : make_int4(dy, dx, ((dy * a.Win + dx) * a.CinS + coff) * ES, 0);
        }
        for (int i = tid; i < a.Npad; i += 256) {
            cst[i] = a.bias[i];
            cst[a.Npad + i] = a.slope1[i];
            cst[2 * a.Npad + i] = a.slope2[i];
        }
        if constexpr (EPI == EPI_CLASSES) {
            int *cl = reinterpret_cast<int *>(cst + 3 * a.Npad);
            if (tid < 16) cl[tid] = a.lut ? (int)a.lut[tid] : tid;
        }
    }
    __syncthreads();
    const float *cbias = cst, *cs1 = cst + a.Npad, *cs2 = cst + 2 * a.Npad;
    T *stage_base = reinterpret_cast<T *>(smem + conv_stage_offset(ES, a));
    const auto rin = mkbuf(a.in, a.in_bytes);
    const auto rout = mkbuf(a.out, a.out_bytes);
    const auto rres = mkbuf(a.res, a.res_bytes);
    const bool fast = a.slopes_le1;
    const bool bia = bias_in_acc(NR, a.Ksteps);            // bias placement (mfma_common.h), wave-uniform
    auto act1 = [&](float4 v, int c) { return fast ? prelu4m(v, ld4f(cs1 + c)) : prelu4(v, ld4f(cs1 + c)); };
    auto act2 = [&](float4 v, int c) { return fast ? prelu4m(v, ld4f(cs2 + c)) : prelu4(v, ld4f(cs2 + c)); };

    const int HWg = a.Hg * a.Wg;
    // fp32 mode range scaling (bugseg_internal.h RangeArgs): the input measured by its producer, the
    // weights' exponent sw[0]; the accumulators are multiplied back (scl false: nothing to do); the
    // output's max |v| is measured for its consumer
    constexpr bool F32 = ES == 4;
    bool scl = false;
    float xm = 1.f, bm = 1.f, om = 1.f, amo = 0.f;
    if constexpr (F32) {
        if (!a.rg.off) {
            const int sx = rng_exp_meas(rng_read(a.rg)), e = sx + a.rg.sw[0];
            scl = (sx | e) != 0;
            xm = rng_pow2(sx); bm = rng_pow2(e); om = rng_pow2(-e);
        }
    }
    // XCD-aware tile walk: gridDim.x is a multiple of 8; group x = blockIdx%8 owns the contiguous
    // chunk [x*C, (x+1)*C) of tiles (speed only; any placement is correct).
    const int G = gridDim.x, grp = blockIdx.x & 7, slot = blockIdx.x >> 3, nslots = G >> 3;
    const int C = (a.ntiles + 7) >> 3;

    for (int i = slot; i < C; i += nslots) {
        const int tile = grp * C + i;
        if (tile >= a.ntiles) break;
        // per-lane GEMM pixel of each fragment: (frame, row, col), input-window origin and byte base
        int pn[MR], py[MR], px[MR], y0[MR], x0[MR];
        uint32_t boff[MR];
        bool pv[MR];
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            const int p = tile * TILE + wave * MR * 16 + m * 16 + col;
            pv[m] = p < a.M;
            const uint32_t pp = pv[m] ? (uint32_t)p : 0u;
            pn[m] = (int)fdiv(pp, a.mHWg, a.sHWg);
            const uint32_t r = pp - (uint32_t)(pn[m] * HWg);
            py[m] = (int)fdiv(r, a.mWg, a.sWg);
            px[m] = (int)r - py[m] * a.Wg;
            y0[m] = pv[m] ? py[m] * a.stride : TAP_PAD;
            x0[m] = px[m] * a.stride;
            boff[m] = (uint32_t)(((pn[m] * a.Hin + py[m] * a.stride) * a.Win + x0[m]) * a.CinS) * ES;
        }
        // Epilogue operands that do not depend on the accumulators are requested before the k loop, so
        // their latency hides under it: the staged residual chunks (EPI_RESADD) and the unpooling
        // indices + low-res main values (EPI_RESUNPOOL). Kept raw; converted where used.
        constexpr int RQ = (NR * 4 / EPC) > 0 ? NR * 4 / EPC : 1;      // >= 16*CPR/64 chunks per lane
        uint4 rpre[EPI == EPI_RESADD ? MR : 1][RQ];
        uint32_t upid[EPI == EPI_RESUNPOOL ? MR : 1][NR];
        MvRaw<T> upmv[EPI == EPI_RESUNPOOL ? MR : 1][NR];
        const int CPR = 1 << a.cpr_sh;
        if constexpr (EPI == EPI_RESADD) {
            if (a.stage_ok && a.resCS == a.outC) {
#pragma unroll
                for (int m = 0; m < MR; ++m) {
                    const int p0 = tile * TILE + wave * MR * 16 + m * 16;
#pragma unroll
                    for (int k = 0; k < RQ; ++k) {
                        const int q = lane + 64 * k;
                        const bool ok = q < 16 * CPR && p0 + (q >> a.cpr_sh) < a.M;
                        rpre[m][k] = bld16(rres, ok ? (uint32_t)(p0 * a.outC + q * EPC) * ES : OOB);
                    }
                }
            }
        }
        if constexpr (EPI == EPI_RESUNPOOL) {
            const auto ridx = mkbuf(a.idx_in, a.idx_bytes);
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                const uint32_t lpix = (uint32_t)((pn[m] * a.resH + (py[m] >> 1)) * a.resW + (px[m] >> 1));
#pragma unroll
                for (int n = 0; n < NR; ++n) {
                    const int c = n * 16 + kq * 4;
                    const bool ok = pv[m] && c < a.resC;
                    upid[m][n] = __builtin_amdgcn_raw_buffer_load_b32(ridx, ok ? (int)(lpix * a.idxCS + c) : (int)OOB, 0, 0);
                    upmv[m][n] = mvload<T>(rres, ok ? (lpix * a.resCS + c) * ES : OOB);
                }
            }
        }

        f32x4 acc[MR][NR];
#pragma unroll
        for (int m = 0; m < MR; ++m)
#pragma unroll
            for (int n = 0; n < NR; ++n)
                acc[m][n] = bia ? bias4(cbias + n * 16 + kq * 4) : (f32x4){0.f, 0.f, 0.f, 0.f};
        if constexpr (F32) {
            if (scl && bia) {
#pragma unroll
                for (int m = 0; m < MR; ++m)
#pragma unroll
                    for (int n = 0; n < NR; ++n) acc[m][n] = mul4(acc[m][n], bm);
            }
        }

        // KC k-steps per chunk: all their B-fragment loads are issued before the first MFMA, so a
        // tile waits on memory ceil(Ksteps / KC) times instead of Ksteps times (the tap table is padded
        // with always-out-of-range entries to whole chunks; MFMAs past Ksteps are skipped)
        for (int s0 = 0; s0 < a.Ksteps; s0 += KC) {
            Raw xf[KC][MR];
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) {
                const int4 g = gt[(s0 + kc) * 4 + kq];
#pragma unroll
                for (int m = 0; m < MR; ++m) {
                    const bool ok = (unsigned)(y0[m] + g.x) < (unsigned)a.Hin && (unsigned)(x0[m] + g.y) < (unsigned)a.Win;
                    bld8(xf[kc][m], rin, ok ? boff[m] + (uint32_t)g.z : OOB);
                }
            }
            if constexpr (F32) {
                if (scl) {
#pragma unroll
                    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                        for (int m = 0; m < MR; ++m) mul8(xf[kc][m], xm);
                }
            }
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) {
                if (s0 + kc >= a.Ksteps) break;
#pragma unroll
                for (int n = 0; n < NR; ++n) {
                    WRaw wf;
                    ld8(wf, wl + (n * 16 + col) * KS + (s0 + kc) * 32 + kq * 8);
#pragma unroll
                    for (int m = 0; m < MR; ++m) mma(acc[m][n], wf, xf[kc][m]);
                }
            }
        }

        // ------------------------------- epilogues -------------------------------------------
        if constexpr (F32) {
            if (scl) {
#pragma unroll
                for (int m = 0; m < MR; ++m)
#pragma unroll
                    for (int n = 0; n < NR; ++n) acc[m][n] = mul4(acc[m][n], om);
            }
        }
        if constexpr (EPI == EPI_CLASSES) {
            // n fragment = output phase (a,b) (NR == 4); rows = 16 (padded) classes, 4 per lane. The
            // fragment's 64 output pixels x 16 logits go to the wave's LDS region (pixel q = n*16 +
            // col); then each lane owns ONE output pixel — lane = a*32 + 2*col + b, so a wave's
            // byte stores are two runs of 32 consecutive pixels — and scans its classes in order.
            static_assert(NR == 4, "EPI_CLASSES expects 4 phases x 16 classes");
            float *cstg = reinterpret_cast<float *>(stage_base) + wave * (64 * CLS_STR);
            const int *clut = reinterpret_cast<const int *>(cst + 3 * a.Npad);
            const int ra = lane >> 5, rb = lane & 1, rc = (lane >> 1) & 15;
            const float *lv = cstg + ((ra * 2 + rb) * 16 + rc) * CLS_STR;
            const size_t plane = (size_t)a.Hout * a.Wout;
#pragma unroll
            for (int m = 0; m < MR; ++m) {
#pragma unroll
                for (int n = 0; n < NR; ++n) {
                    const int c = n * 16 + kq * 4;
                    static_assert(bias_in_acc(NR), "EPI_CLASSES: bias in the accumulator");
                    *reinterpret_cast<float4 *>(cstg + (n * 16 + col) * CLS_STR + kq * 4) = f4(acc[m][n]);
                }
                wave_lds_sync();
                const int p = tile * TILE + wave * MR * 16 + m * 16 + rc;
                if (p < a.M) {
                    const int qn = (int)fdiv((uint32_t)p, a.mHWg, a.sHWg), qr = p - qn * HWg;
                    const int qy = (int)fdiv((uint32_t)qr, a.mWg, a.sWg), qx = qr - qy * a.Wg;
                    const uint32_t opix = (uint32_t)((qn * a.Hout + 2 * qy + ra) * a.Wout + 2 * qx + rb);
                    float lg[16];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float4 v = ld4f(lv + 4 * r);
                        lg[4 * r] = v.x; lg[4 * r + 1] = v.y; lg[4 * r + 2] = v.z; lg[4 * r + 3] = v.w;
                    }
                    // lowest class index wins ties (tf.math.argmax, models.py:55)
                    float best = -INFINITY;
                    int bi = 0;
#pragma unroll
                    for (int k = 0; k < 16; ++k)
                        if (k < a.ncls && lg[k] > best) { best = lg[k]; bi = k; }
                    if (a.cls_out) a.cls_out[opix] = (uint8_t)clut[bi];
                    if (a.logits_out) {
                        float *lo = a.logits_out + (size_t)qn * a.ncls * plane + (opix - (size_t)qn * plane);
#pragma unroll
                        for (int k = 0; k < 16; ++k)
                            if (k < a.ncls) lo[(size_t)k * plane] = lg[k];
                    }
                }
                wave_lds_sync();
            }
        } else {
            // Output staging: each wave owns an LDS region; a 16-pixel fragment's results are written
            // there and leave as contiguous 16-B-per-lane stores (a per-lane NHWC store writes 16
            // partial lines per instruction). EPI_SHUFFLE stages the fragment's two output rows of 32
            // pixels. The RESADD residual comes in the same coalesced way.
            const bool staged = a.stage_ok;
            T *stg = stage_base + wave * a.stg_elems;
            const int OSTR = a.outC + EPC;
            const int csh = a.cpr_sh;
            // EPI_SHUFFLE: output phase and channel of accumulator fragment n (coutP is a multiple of 16)
            int phn[NR], cln[NR];
#pragma unroll
            for (int n = 0; n < NR; ++n) { phn[n] = n * 16 / a.coutP; cln[n] = n * 16 - phn[n] * a.coutP; }
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                const int p0 = tile * TILE + wave * MR * 16 + m * 16;    // first GEMM pixel (uniform)
                const int p = p0 + col;
                bool res_staged = false;
                if constexpr (EPI == EPI_RESADD) {
                    if (staged && a.resCS == a.outC) {
#pragma unroll
                        for (int k = 0; k < RQ; ++k) {
                            const int q = lane + 64 * k;
                            if (q < 16 * CPR)
                                *reinterpret_cast<uint4 *>(stg + (q >> csh) * OSTR + (q & (CPR - 1)) * EPC) = rpre[m][k];
                        }
                        wave_lds_sync();
                        res_staged = true;
                    }
                }
#pragma unroll
                for (int n = 0; n < NR; ++n) {
                    const int c = n * 16 + kq * 4;
                    float4 v = bia ? f4(acc[m][n]) : add4(f4(acc[m][n]), ld4f(cbias + c));
                    if constexpr (EPI == EPI_SHUFFLE) {
                        const int ph = phn[n], cl = cln[n] + kq * 4;
                        if (cl >= a.outC) continue;
                        v = act1(v, c);
                        if constexpr (F32) {
                            if (pv[m]) rng_acc4(amo, v);
                        }
                        if (staged) {
                            st4(stg + ((ph >> 1) * 32 + 2 * col + (ph & 1)) * OSTR + cl, v);
                        } else if (pv[m]) {
                            const int oy = 2 * py[m] + (ph >> 1), ox = 2 * px[m] + (ph & 1);
                            st4(reinterpret_cast<T *>(a.out) + ((size_t)(pn[m] * a.Hout + oy) * a.Wout + ox) * a.outC + cl, v);
                        }
                        continue;
                    }
                    if (c >= a.outC || !pv[m]) continue;
                    v = act1(v, c);
                    if constexpr (EPI == EPI_RESADD) {
                        if (res_staged) v = add4(v, ld4(stg + col * OSTR + c));
                        else if (c < a.resC) v = add4(v, bld4(rres, (uint32_t)(p * a.resCS + c) * ES, (const T *)nullptr));
                        v = act2(v, c);
                    } else if constexpr (EPI == EPI_RESPOOL) {
                        // main branch: MaxPool2d(2, 2, return_indices) of the block input, zero-padded
                        // to cout channels; first maximum in window order wins (strict >).
                        if (c < a.resC) {
                            const uint32_t rb0 = (uint32_t)(((pn[m] * a.resH + 2 * py[m]) * a.resW + 2 * px[m]) * a.resCS + c) * ES;
                            const uint32_t rstep[4] = {0u, (uint32_t)a.resCS * ES, (uint32_t)(a.resW * a.resCS) * ES,
                                                       (uint32_t)((a.resW + 1) * a.resCS) * ES};
                            float4 best = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
                            int bi[4] = {0, 0, 0, 0};
#pragma unroll
                            for (int pos = 0; pos < 4; ++pos) {
                                const float4 x = bld4(rres, rb0 + rstep[pos], (const T *)nullptr);
                                if (x.x > best.x) { best.x = x.x; bi[0] = pos; }
                                if (x.y > best.y) { best.y = x.y; bi[1] = pos; }
                                if (x.z > best.z) { best.z = x.z; bi[2] = pos; }
                                if (x.w > best.w) { best.w = x.w; bi[3] = pos; }
                            }
                            v = add4(v, best);
                            *reinterpret_cast<uint32_t *>(a.idx_out + (uint32_t)(p * a.idxCS + c)) =
                                (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
                        }
                        v = act2(v, c);
                    } else if constexpr (EPI == EPI_RESUNPOOL) {
                        // MaxUnpool2d(2): the low-res main value lands on the window position its
                        // pooling index recorded; every other position of the window is 0.
                        if (c < a.resC) {
                            const uint32_t id = upid[m][n];
                            const uint32_t pos = (uint32_t)(((py[m] & 1) << 1) | (px[m] & 1));
                            const float4 mv = mvcvt<T>(upmv[m][n]);
                            v.x += ((id & 0xff) == pos) ? mv.x : 0.f;
                            v.y += (((id >> 8) & 0xff) == pos) ? mv.y : 0.f;
                            v.z += (((id >> 16) & 0xff) == pos) ? mv.z : 0.f;
                            v.w += (((id >> 24) & 0xff) == pos) ? mv.w : 0.f;
                        }
                        v = act2(v, c);
                    }
                    if constexpr (F32) rng_acc4(amo, v);
                    if (staged) st4(stg + col * OSTR + c, v);
                    else st4(reinterpret_cast<T *>(a.out) + (size_t)p * a.outC + c, v);
                }
                if (!staged) continue;
                wave_lds_sync();
                if constexpr (EPI == EPI_SHUFFLE) {
                    // two output rows 2y, 2y+1, each 32 pixels from x = 2*px of the fragment's first pixel
                    const int n0 = (int)fdiv((uint32_t)p0, a.mHWg, a.sHWg), r0 = p0 - n0 * HWg;
                    const int yy = (int)fdiv((uint32_t)r0, a.mWg, a.sWg), xx = r0 - yy * a.Wg;
                    const int nq = 32 * CPR;
                    for (int q = lane; q < 2 * nq; q += 64) {
                        const int row = q >= nq, qq = q - row * nq;
                        const uint32_t off = p0 < a.M
                            ? (uint32_t)(((n0 * a.Hout + 2 * yy + row) * a.Wout + 2 * xx) * a.outC + qq * EPC) * ES : OOB;
                        bst16(rout, off, *reinterpret_cast<const uint4 *>(stg + (row * 32 + (qq >> csh)) * OSTR + (qq & (CPR - 1)) * EPC));
                    }
                } else {
                    for (int q = lane; q < 16 * CPR; q += 64) {
                        const int pix = q >> csh;
                        const uint32_t off = p0 + pix < a.M ? (uint32_t)(p0 * a.outC + q * EPC) * ES : OOB;
                        bst16(rout, off, *reinterpret_cast<const uint4 *>(stg + pix * OSTR + (q & (CPR - 1)) * EPC));
                    }
                }
                wave_lds_sync();
            }
        }
    }
    if constexpr (F32) rng_commit(amo, a.rg.amax_out);
    span_exit(a.span);
}

int conv_tile_pixels(int nr) { return 4 * (nr >= 4 ? 2 : 4) * 16; }

size_t conv_lds_bytes(int prec, const ConvArgs &a) {
    const int es = prec_es(prec);
    return conv_stage_offset(es, a) + (size_t)4 * a.stg_elems * es;
}

template <typename T, int NR>
static hipError_t launch_nr(int epi, const ConvArgs &a, dim3 grid, size_t lds, hipStream_t s) {
    switch (epi) {
    case EPI_PLAIN: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_PLAIN>), grid, dim3(256), lds, s, a); break;
    case EPI_RESADD: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_RESADD>), grid, dim3(256), lds, s, a); break;
    case EPI_RESPOOL: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_RESPOOL>), grid, dim3(256), lds, s, a); break;
    case EPI_RESUNPOOL: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_RESUNPOOL>), grid, dim3(256), lds, s, a); break;
    case EPI_SHUFFLE: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_SHUFFLE>), grid, dim3(256), lds, s, a); break;
    case EPI_CLASSES:
        if constexpr (NR == 4) { hipLaunchKernelGGL((conv_kernel<T, NR, EPI_CLASSES>), grid, dim3(256), lds, s, a); break; }
        return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_t(int nr, int epi, const ConvArgs &a, dim3 grid, size_t lds, hipStream_t s) {
    switch (nr) {
    case 1: return launch_nr<T, 1>(epi, a, grid, lds, s);
    case 2: return launch_nr<T, 2>(epi, a, grid, lds, s);
    case 4: return launch_nr<T, 4>(epi, a, grid, lds, s);
    case 8: return launch_nr<T, 8>(epi, a, grid, lds, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_conv(int prec, int nr, int epi, const ConvArgs &a, hipStream_t s) {
    // the initial block has its own tiled kernel (init_kernels.hip)
    if (epi == EPI_INIT || epi == EPI_INIT_BGR) return launch_init(prec, epi == EPI_INIT_BGR, a, s);
    // so has the class layer (cls_kernels.hip), when it has ENet's 16 input channels
    if (epi == EPI_CLASSES && cls_supported(a) && !std::getenv("BUGSEG_CLS_CONV")) return launch_cls(prec, a, s);
    // one workgroup per tile up to 2048 workgroups (8 per CU), rounded to a multiple of 8 for the
    // XCD-aware walk; larger grids stride.
    int g = a.ntiles < 2048 ? a.ntiles : 2048;
    g = (g + 7) & ~7;
    const size_t lds = conv_lds_bytes(prec, a);
    if (prec == PREC_BF16) return launch_t<__bf16>(nr, epi, a, dim3(g), lds, s);
    if (prec == PREC_F16) return launch_t<_Float16>(nr, epi, a, dim3(g), lds, s);
    return launch_t<float>(nr, epi, a, dim3(g), lds, s);
}

void fastdiv(uint32_t d, uint32_t &m, int &s) {
    if (d <= 1) { m = 0; s = -1; return; }
    int l = 0;
    while ((1ull << l) < d) ++l;                     // ceil(log2 d)
    m = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);   // ceil(2^(31+l) / d) < 2^32
    s = l - 1;
}

}  // namespace bugseg
