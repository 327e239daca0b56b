// The class layer: ENet's final transposed convolution (16 -> ncls, stride 2) + argmax + class LUT,
// i.e. the tail of the reference's sess.run + tf.math.argmax (models.py:43-58), in one streaming
// kernel (EPI_CLASSES launches of launch_conv land here when the layer has 16 input channels).
//
// GEMM view as conv_kernels.hip: a column is one input pixel, K = (tap of the 2x2 input
// neighbourhood, channel), rows = (output phase, class). The MFMA is v_mfma_f32_32x32x16_bf16
// (fp32 parity mode: split-f16 products, 3 x v_mfma_f32_32x32x16_f16 per tap): its accumulator gives
// lane (col, h) the 16 rows {8j + 4h + i}. Rows are permuted (the weights are gathered with the
// permutation, nothing is repacked) so that those 16 rows are the 16 classes of ONE output phase:
//   block b (two per column), lane half h  ->  phase 2b + h = output pixel (2y + b, 2x + h),
//   accumulator register c                 ->  class c.
// The argmax is therefore a scan of one lane's own registers — no staging, no cross-lane traffic — and
// one v_permlane32_swap pairs each lane with the horizontally adjacent output pixel for 2-byte stores.
//
// The whole layer's weights (64 rows x 4 taps x 16 channels) live in 32 VGPRs per lane for the
// kernel's lifetime; the only per-pixel traffic is the B fragments (one 16-B load per lane and tap,
// the next group's loads in flight while the current group computes) and the class bytes.
#include "bugseg_internal.h"
#include "cls_common.h"

namespace bugseg {

// Taps: the 2x2 input neighbourhood (dy, dx) = (s >> 1, s & 1) of the k = 3 layer in pack_tconv's
// order (D = {0, 1}, tap = ty * 2 + tx). LOGITS: the fp32 logits are written too (parity runs).
// The next group's loads are in flight while one computes (two groups ahead measured no faster,
// round 3: 37.3 vs 36.9 us per launch, 127 vs 109 VGPRs).
// CLS_ABL (debug ablation builds, wrong classes; scripts/gpu_r4_abl.sh): 1 = no MFMAs, 2 = no argmax,
// 4 = no class stores, 8 = no input loads
#ifndef CLS_ABL
#define CLS_ABL 0
#endif
#ifndef CLS_AUX
#define CLS_AUX 0          // class-map store policy (A/B knob; the BEV rasteriser reads them next)
#endif
#ifndef CLS_SPLIT1
#define CLS_SPLIT1 0       // fp32: each tap's operand split once per group for both blocks (A/B knob; round 6, with
                           // VGPR-form MFMAs: 109 -> 113 us per 64-frame launch — the up-front splits delay the MFMAs)
#endif
#ifndef CLS_BIAS_REG
#define CLS_BIAS_REG 1
#endif
// (Round 4 measured a low-register form — weights from LDS, the two blocks one after the other, 7 waves
// per SIMD instead of 4 — at 37.5 vs 34.7 us per 32-frame launch (fp16) and 75.3 vs 74.7 (fp32): the
// class layer is not occupancy-bound. Removed.)
// LK: the class map's group-max argmax (cls_common.h cls_argmax)
template <typename T, bool LOGITS, int LK = 0>
#ifndef CLS_OCC_F32
#define CLS_OCC_F32 1      // fp32: waves per SIMD the build is held to (A/B knob; 3: 28 VGPRs spilled, 109 -> 257 us)
#endif
__global__ void __launch_bounds__(256, sizeof(T) == 2 ? 4 : CLS_OCC_F32) cls_kernel(const ConvArgs a) {
    span_enter(a.span);
    constexpr int CLS_TAPS = 4;
    using Raw = typename Tr<T>::Raw;
    using WRaw = typename WTr<T>::Raw;   // weight operand (fp32 mode: split-f16 parts)
    constexpr int ES = (int)sizeof(T);
    __shared__ float sbias[64];
    const int tid = threadIdx.x, lane = tid & 63, col = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // a padding class (row (phase, c) with c >= ncls: zero weights) starts at -inf and stays there, so
    // the argmax needs no class mask (the logits of those rows are never written)
    if (tid < 64) sbias[tid] = (tid & 15) < a.ncls ? a.bias[tid] : -INFINITY;
    // the class LUT as 16 nibbles in a 64-bit scalar: class c -> (lut64 >> 4c) & 15
    const uint64_t lut64 = cls_lut64(a.lut);

    // weights: block b, row r = lane's col -> packed row (phase 2b + ((r >> 2) & 1), class 4 (r >> 3) + (r & 3));
    // this lane's k half = channels 8h .. 8h + 7 of each tap
    WRaw wr[2][CLS_TAPS];
    {
        const T *w = reinterpret_cast<const T *>(a.w);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int prow = cls_prow(b, col);
#pragma unroll
            for (int s = 0; s < CLS_TAPS; ++s) {
                ld8(wr[b][s], w + (size_t)prow * a.Kpad + s * 16 + 8 * h);
            }
        }
    }
    // A block whose dy = 1 taps (s = 2, 3) have all-zero weights skips them: output row 2y of the 3x3
    // transposed kernel never sees input row y + 1 (a wave-uniform choice, made once)
    bool short_blk[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) short_blk[b] = __ballot(nonzero(wr[b][2]) || nonzero(wr[b][3])) == 0;
    __syncthreads();

    // The accumulators start at the bias. pack_tconv (bugseg_runtime.cpp) writes the same per-class bias
    // into all four phases' rows, so sbias[(2b + h) * 16 + k] is one 16-vector for every block and lane
    // half: CLS_BIAS_REG holds it in 16 loop-long registers instead of reading it from LDS per group.
    auto ldbias = [&](int b) {
        // (the opaque offset keeps the compiler from hoisting these reads out of the group loop)
        int boff = (2 * b + h) * 16;
        asm volatile("" : "+v"(boff));
        const float4 *bb = reinterpret_cast<const float4 *>(sbias + boff);
        f32x16 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 q = bb[j];
            v[4 * j] = q.x; v[4 * j + 1] = q.y; v[4 * j + 2] = q.z; v[4 * j + 3] = q.w;
        }
        return v;
    };
    // (2-byte class maps only: the logits form and fp32 have no registers to spare)
    constexpr bool BREG = CLS_BIAS_REG && !LOGITS && sizeof(T) == 2;
    f32x16 bvec;
    if constexpr (BREG) bvec = ldbias(0);
    // fp32 mode range scaling (bugseg_internal.h RangeArgs): the input measured by its producer, the
    // weights' exponent; the accumulators are multiplied back (scl false: nothing to do)
    constexpr bool F32 = ES == 4;
    bool scl = false;
    float xm = 1.f, bm = 1.f, om = 1.f;
    if constexpr (F32) {
        if (!a.rg.off) {
            const int sx = rng_exp_meas(rng_read(a.rg)), e = sx + a.rg.sw[0];
            scl = (sx | e) != 0;
            xm = rng_pow2(sx); bm = rng_pow2(e); om = rng_pow2(-e);
        }
    }
    const auto rin = mkbuf(a.in, a.in_bytes);
    const int HWg = a.Hg * a.Wg;
    const size_t plane = (size_t)a.Hout * a.Wout;
    const int groups = (a.M + 31) >> 5;
    // XCD-aware: XCD x = blockIdx % 8 walks the contiguous run [x*C, (x+1)*C) of 32-pixel groups, its
    // waves interleaved over it
    const int xcd = blockIdx.x & 7, nw = (gridDim.x >> 3) * 4, wi = (blockIdx.x >> 3) * 4 + wave;
    const int C = (groups + 7) >> 3, g0 = xcd * C, g1 = g0 + C < groups ? g0 + C : groups;
    // tap s is a wave-uniform byte delta (the buffer load's scalar offset) from the lane's pixel,
    // valid where x + dx < Win and y + dy < Hin
    const uint32_t pixB = (uint32_t)(a.CinS * ES), rowB = (uint32_t)a.Win * pixB;

    // lane pixel of group g: the group's first pixel is divided out on the scalar unit (g is
    // wave-uniform; Hg * Wg, Wg >= 32 > 1), each lane then steps at most one row on
    // (the input grid is the class layer's own grid, cls_supported: a pixel's flat index p addresses
    // its input, and its output pixels (2y + h, 2x) sit at byte 4p - 2x + 2hWg of the class map)
    struct Px { uint32_t p; int n, y, x; bool ok; };
    auto pixel = [&](int g) -> Px {
        const uint32_t p0 = (uint32_t)g * 32u;
        const int n0 = (int)(__umulhi(p0, a.mHWg) >> a.sHWg);
        const uint32_t r = p0 - (uint32_t)(n0 * HWg);
        const int y0 = (int)(__umulhi(r, a.mWg) >> a.sWg), x0 = (int)r - y0 * a.Wg;
        Px q;
        q.p = p0 + (uint32_t)col;
        q.ok = (int)q.p < a.M;
        q.x = x0 + col;
        const bool wrap = q.x >= a.Wg;
        q.x = wrap ? q.x - a.Wg : q.x;
        q.y = y0 + (wrap ? 1 : 0);
        const bool wrapn = q.y >= a.Hg;
        q.y = wrapn ? 0 : q.y;
        q.n = n0 + (wrapn ? 1 : 0);          // (the logits path only)
        return q;
    };
    // (the group's pixel is computed once, with its loads, and handed to the step that consumes them)
    auto load = [&](int g, Raw (&xf)[CLS_TAPS], Px &q) {
        q = pixel(g);
        if constexpr ((CLS_ABL & 8) != 0) {
#pragma unroll
            for (int s = 0; s < CLS_TAPS; ++s) zero(xf[s]);
            if constexpr (sizeof(T) == 2) xf[0].v.x = (uint32_t)g;   // (something that varies, so nothing is hoisted)
            return;
        }
        const uint32_t base = q.p * pixB + (uint32_t)(8 * h * ES);
        const bool okx = q.x + 1 < a.Win, oky = q.y + 1 < a.Hin;
        const int v00 = (int)(q.ok ? base : OOB), v01 = (int)(q.ok && okx ? base : OOB);
        const int v10 = (int)(q.ok && oky ? base : OOB), v11 = (int)(q.ok && okx && oky ? base : OOB);
        const int vo[CLS_TAPS] = {v00, v01, v10, v11};
#pragma unroll
        for (int s = 0; s < CLS_TAPS; ++s) {
            const int d = (int)((uint32_t)(s >> 1) * rowB + (uint32_t)(s & 1) * pixB);
            if constexpr (sizeof(T) == 2) {
                xf[s].v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rin, vo[s], d, 0));
            } else {
                reinterpret_cast<RawF &>(xf[s]).a =
                    __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rin, vo[s], d, 0));
                reinterpret_cast<RawF &>(xf[s]).b =
                    __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rin, vo[s], d + 16, 0));
            }
        }
    };

    // one group: MFMAs, argmax, stores; `nxt` first receives the next group's loads (they fly during
    // this one; the two buffers alternate by unrolling, never by a runtime index).
    const auto rcls = mkbuf(a.cls_out, (uint32_t)((size_t)a.B * plane));
    auto step = [&](int g, const Raw (&cur)[CLS_TAPS], Raw (&nxt)[CLS_TAPS], const Px &q, Px &qn) {
        // unconditional: past the last group the loads are harmless (an out-of-range group reads
        // zeros, a neighbour's group is read and dropped), and a static count of loads in flight
        // lets the waits before the MFMAs name only this group's loads (a conditional prefetch
        // made the compiler wait vmcnt(3), i.e. for the next group's first load as well).
        load(g + nw, nxt, qn);
        // CLS_SPLIT1 (fp32): the four taps' hi / lo parts, scaled first when the launch scales (the same
        // parts the per-block split would make: bit-identical)
        constexpr bool S1 = F32 && CLS_SPLIT1;
        f16x8 sxh[S1 ? CLS_TAPS : 1], sxl[S1 ? CLS_TAPS : 1];
        if constexpr (S1) {
#pragma unroll
            for (int s = 0; s < CLS_TAPS; ++s) {
                RawF xq = reinterpret_cast<const RawF &>(cur[s]);
                if (scl) mul8(xq, xm);
                split_f16(xq, sxh[s], sxl[s]);
            }
        }
        // per block: accumulators from the bias, the taps' MFMAs, (parity runs) the logits, and the
        // argmax over this lane's classes = the sequential strict > scan from -inf of tf.math.argmax
        // (models.py:55): the maximum (v_max ignores NaN), then its first index; no class equal to the
        // maximum (all NaN) -> 0; all -inf -> 0 (class 0 equals the maximum). Both blocks' MFMAs go
        // first, then the two argmax scans interleaved
        auto taps = [&](int b, f32x16 &acc, auto sc) {
            auto tap = [&](int s) {
                if constexpr (S1) {
                    if constexpr (F32) mma32s(acc, reinterpret_cast<const RawS &>(wr[b][s]), sxh[s], sxl[s]);
                    return;
                }
                Raw xq = cur[s];
                if constexpr (decltype(sc)::value) mul8(reinterpret_cast<RawF &>(xq), xm);
                mma32(acc, wr[b][s], xq);
            };
            tap(0);
            tap(1);
            if (!short_blk[b]) {
                tap(2);
                tap(3);
            }
        };
        auto block = [&](int b, f32x16 &acc) {
            acc = BREG ? bvec : ldbias(b);
            if constexpr ((CLS_ABL & 1) != 0 && sizeof(T) == 2) { acc[0] += __builtin_bit_cast(float, cur[0].v.x & 1u); return; }
            bool done = false;
            if constexpr (F32) {
                if (scl) {
#pragma unroll
                    for (int c = 0; c < 16; ++c) acc[c] *= bm;
                    taps(b, acc, std::true_type());
#pragma unroll
                    for (int c = 0; c < 16; ++c) acc[c] *= om;
                    done = true;
                }
            }
            if (!done) taps(b, acc, std::false_type());
            if (LOGITS && q.ok) {
                float *lo = a.logits_out + (size_t)q.n * a.ncls * plane + (size_t)(2 * q.y + b) * a.Wout + 2 * q.x + h;
#pragma unroll
                for (int c = 0; c < 16; ++c)
                    if (c < a.ncls) lo[(size_t)c * plane] = acc[c];
            }
        };
        int cls[2];
        f32x16 acc[2];
        block(0, acc[0]);
        block(1, acc[1]);
        cls_argmax<LK>(acc, lut64, cls);
        if constexpr ((CLS_ABL & 2) != 0)
            for (int b = 0; b < 2; ++b) cls[b] = acc[b][b] > acc[b][5] ? 1 : 0;
        if (a.cls_out) {
            // lanes < 32 take output row 2y (their phase-(0,0) byte + the (0,1) byte of lane + 32), lanes
            // >= 32 row 2y + 1: one 2-byte store of pixels (2x, 2x + 1) each
            uint32_t c0 = (uint32_t)cls[0], c1 = (uint32_t)cls[1];
            pl32swap(c0, c1);
            // (32-bit offsets through a buffer descriptor: a masked lane's store is dropped)
            const uint32_t o = 4u * q.p - 2u * (uint32_t)q.x + (uint32_t)(2 * h * a.Wg);
            if (!(CLS_ABL & 4) || c0 == 77)
                __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(c0 | (c1 << 8)), rcls, q.ok ? (int)o : (int)OOB, 0, CLS_AUX);
        }
    };
    Raw xa[CLS_TAPS], xb[CLS_TAPS];
    Px qa, qb;
    int g = g0 + wi;
    if (g < g1) load(g, xa, qa);
    while (g < g1) {
        step(g, xa, xb, qa, qb);
        g += nw;
        if (g >= g1) break;
        step(g, xb, xa, qb, qa);
        g += nw;
    }
    span_exit(a.span);
}

// 16 input channels in two 8-channel groups per tap, the 4 taps of the k = 3 layer (Kpad = 4 x 16: a
// 3x3 stride-2 transposed conv with output exactly 2x has pad 1, so pack_tconv's D = {0, 1}), grids
// at least 32 wide; other class layers (k = 2, narrow grids) keep the generic conv path
bool cls_supported(const ConvArgs &a) {
    return a.CinS == 16 && a.Npad == 64 && a.Kpad == 64 && a.ncls >= 1 && a.ncls <= 16 && a.Wg >= 32 &&
           a.Hout == 2 * a.Hg && a.Wout == 2 * a.Wg && a.Hg == a.Hin && a.Wg == a.Win;
}

template <typename T>
static const void *cls_fun(bool lg, int lk) {
    if (lg) return (const void *)cls_kernel<T, true, 0>;         // (parity runs: the full scan)
    return lk == 1 ? (const void *)cls_kernel<T, false, 1> : lk == 2 ? (const void *)cls_kernel<T, false, 2>
                   : (const void *)cls_kernel<T, false, 0>;
}

hipError_t launch_cls(int prec, const ConvArgs &a, hipStream_t s) {
    // waves stream over 32-pixel groups: enough workgroups to fill every CU at 4 waves per SIMD,
    // a multiple of 8 for the XCD split
    const int groups = (a.M + 31) / 32;
    const bool lg = a.logits_out != nullptr;
    // the group-max argmax applies when the class map is the remap (a.lut) the kind names
    const int lk = a.lut && (a.lut_kind == 1 || a.lut_kind == 2) ? a.lut_kind : 0;
    const void *f = prec == PREC_BF16 ? cls_fun<__bf16>(lg, lk) : prec == PREC_F16 ? cls_fun<_Float16>(lg, lk) : cls_fun<float>(lg, lk);
    // one round of resident workgroups (occupancy API per kernel instance, cached per device:
    // bugseg_runtime.cpp occupancy_per_cu)
    const int per = occupancy_per_cu(f, 256, 0);
    const int cap = device_cus() * (per > 0 ? per : 4);
    int g = (groups + 3) / 4;
    g = g < cap ? g : cap;
    g = (g + 7) & ~7;
    void *args[] = {const_cast<ConvArgs *>(&a)};
    return hipLaunchKernel(f, dim3(g), dim3(256), args, 0, s);
}

}  // namespace bugseg
