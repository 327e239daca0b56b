// The class layer's arithmetic (ENet's final transposed convolution + tf.math.argmax + the class LUT,
// models.py:43-58), shared by the class kernel (cls_kernels.hip) and the C = 16 bottleneck with the
// class layer fused in (bneck_kernels.hip, FC >= 0), so both produce the same logits bit for bit and
// the same class for every pixel.
//
// MFMA v_mfma_f32_32x32x16 (fp32 parity mode: split-f16 products, 3 MFMAs per tap): a column is one
// input pixel, K = (tap of the 2x2 input neighbourhood, channel); the weights' rows are permuted so
// that the accumulator of lane (col, h) of block b holds the 16 classes of output pixel (2y + b, 2x + h)
// — the argmax is a scan of one lane's own registers.
#pragma once
#include "mfma_common.h"

namespace bugseg {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void mma32(f32x16 &acc, const RawB &w, const RawB &x) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, w.v), __builtin_bit_cast(bf16x8, x.v),
                                                  acc, 0, 0, 0);
}
__device__ __forceinline__ void mma32(f32x16 &acc, const RawH &w, const RawH &x) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, w.v), __builtin_bit_cast(f16x8, x.v),
                                                 acc, 0, 0, 0);
}
// fp32 parity mode: split-f16 products (mfma_common.h mma(RawS, RawF)) on the 32 x 32 shape: the
// lane's 8 channels (8h .. 8h + 7 of the tap) as hi / lo f16 parts, three MFMAs
__device__ __forceinline__ void mma32s(f32x16 &acc, const RawS &w, const f16x8 &xh, const f16x8 &xl) {
    const f16x8 wh = __builtin_bit_cast(f16x8, w.h), wl = __builtin_bit_cast(f16x8, w.l);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma32(f32x16 &acc, const RawS &w, const RawF &x) {
    f16x8 xh, xl;
    split_f16(x, xh, xl);
    mma32s(acc, w, xh, xl);
}

__device__ __forceinline__ bool nonzero(const RawB &r) { return (r.v.x | r.v.y | r.v.z | r.v.w) != 0u; }
__device__ __forceinline__ bool nonzero(const RawH &r) { return (r.v.x | r.v.y | r.v.z | r.v.w) != 0u; }
__device__ __forceinline__ bool nonzero(const RawS &r) {
    return (r.h.x | r.h.y | r.h.z | r.h.w | r.l.x | r.l.y | r.l.z | r.l.w) != 0u;
}

// LK (round 4): the remapped class maps need only the GROUP of the first maximal class, not its index.
// LK = 1: the 3-class map (models.py:56-58: {0, 1} -> 1, {2, 9} -> 0, the rest -> 2), LK = 2: the binary
// map (models.py:79-80: {0, 1} -> 1, the rest -> 0). Per pixel the groups' maxima (v_max3 over the
// members) and the overall maximum; when exactly one group attains it, that group holds the first
// maximal class and its value is the answer. Otherwise (a tie across groups, or no class equal to the
// maximum: all NaN) the full first-index scan decides, on a wave-uniform branch that noisy real-valued
// logits essentially never take. LK = 0: the full scan always (raw class ids, parity runs).
template <int LK> struct ClsGroups;
template <> struct ClsGroups<1> { static constexpr int N = 3; static constexpr uint32_t mask[3] = {0x0204u, 0x0003u, 0xfdf8u};
                                  static constexpr int val[3] = {0, 1, 2}; };
template <> struct ClsGroups<2> { static constexpr int N = 2; static constexpr uint32_t mask[3] = {0x0003u, 0xfffcu, 0u};
                                  static constexpr int val[3] = {1, 0, 0}; };

// the class map values of a lane's two output pixels (blocks b = 0, 1) from their 16 logits: the
// argmax of tf.math.argmax (models.py:55) = the sequential strict > scan from -inf: the maximum (v_max
// ignores NaN), then its first index; no class equal to the maximum (all NaN) -> 0; all -inf -> 0
// (class 0 equals the maximum). lut64: class c -> (lut64 >> 4c) & 15. Every lane of the wave calls it.
template <int LK>
__device__ __forceinline__ void cls_argmax(const f32x16 (&acc)[2], uint64_t lut64, int (&cls)[2]) {
    bool full = LK == 0;
    if constexpr (LK != 0) {
        // the groups' maxima, the maximum, which groups attain it
        using G = ClsGroups<LK>;
        bool tie = false;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            float gm[G::N];
#pragma unroll
            for (int k = 0; k < G::N; ++k) {
                float m = -INFINITY;
#pragma unroll
                for (int c = 0; c < 16; ++c)
                    if ((G::mask[k] >> c) & 1u) m = __builtin_fmaxf(m, acc[b][c]);
                gm[k] = m;
            }
            float mx = gm[0];
#pragma unroll
            for (int k = 1; k < G::N; ++k) mx = __builtin_fmaxf(mx, gm[k]);
            int hits = 0, v = 0;
#pragma unroll
            for (int k = 0; k < G::N; ++k) {
                const bool e = gm[k] == mx;
                hits += e ? 1 : 0;
                v = e ? G::val[k] : v;
            }
            cls[b] = v;
            tie |= hits != 1;
        }
        full = __ballot(tie) != 0;                // wave-uniform: rare
    }
    if (full) {
        float best[2];
        int bi[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            best[b] = acc[b][0];
#pragma unroll
            for (int c = 1; c < 16; ++c) best[b] = __builtin_fmaxf(best[b], acc[b][c]);
            bi[b] = 0;
        }
#pragma unroll
        for (int c = 15; c >= 0; --c)
#pragma unroll
            for (int b = 0; b < 2; ++b) bi[b] = acc[b][c] == best[b] ? c : bi[b];
#pragma unroll
        for (int b = 0; b < 2; ++b) cls[b] = (int)(lut64 >> (4 * bi[b])) & 15;
    }
}

// one block's class value (the fused class phase, bneck_kernels.hip: one accumulator block live at a
// time). The group-max result is exact wherever one group attains the maximum, and the full scan is
// exact always, so deciding the fallback per block (instead of over both blocks, as cls_argmax does)
// gives every pixel the same value
template <int LK>
__device__ __forceinline__ int cls_argmax1(const f32x16 &acc, uint64_t lut64) {
    int v = 0;
    bool full = LK == 0;
    if constexpr (LK != 0) {
        using G = ClsGroups<LK>;
        float gm[G::N];
#pragma unroll
        for (int k = 0; k < G::N; ++k) {
            float m = -INFINITY;
#pragma unroll
            for (int c = 0; c < 16; ++c)
                if ((G::mask[k] >> c) & 1u) m = __builtin_fmaxf(m, acc[c]);
            gm[k] = m;
        }
        float mx = gm[0];
#pragma unroll
        for (int k = 1; k < G::N; ++k) mx = __builtin_fmaxf(mx, gm[k]);
        int hits = 0;
#pragma unroll
        for (int k = 0; k < G::N; ++k) {
            const bool e = gm[k] == mx;
            hits += e ? 1 : 0;
            v = e ? G::val[k] : v;
        }
        full = __ballot(hits != 1) != 0;
    }
    if (full) {
        float best = acc[0];
#pragma unroll
        for (int c = 1; c < 16; ++c) best = __builtin_fmaxf(best, acc[c]);
        int bi = 0;
#pragma unroll
        for (int c = 15; c >= 0; --c) bi = acc[c] == best ? c : bi;
        v = (int)(lut64 >> (4 * bi)) & 15;
    }
    return v;
}

// the class LUT as 16 nibbles in a 64-bit scalar (lut: 16 bytes, nullptr = raw class ids)
__device__ __forceinline__ uint64_t cls_lut64(const uint8_t *lut) {
    uint64_t l = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) l |= (uint64_t)((lut ? (int)lut[c] : c) & 15) << (4 * c);
    return l;
}

// packed row of the class weights [64][64] feeding accumulator row r (0..31, a lane's col) of block b:
// phase 2b + ((r >> 2) & 1), class 4 (r >> 3) + (r & 3)
__host__ __device__ inline int cls_prow(int b, int r) { return (2 * b + ((r >> 2) & 1)) * 16 + 4 * (r >> 3) + (r & 3); }

}  // namespace bugseg
