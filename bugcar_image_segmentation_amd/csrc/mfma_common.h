// Device helpers shared by the MFMA kernels (conv_kernels.hip, bneck_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "bugseg_internal.h"

namespace bugseg {

// LDS hand-off between lanes of ONE wave: wait for the wave's LDS operations, keep the compiler
// from moving memory operations across (no s_barrier needed inside a wave).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

struct RawB { uint4 v; };          // 8 bf16
struct RawH { uint4 v; };          // 8 f16 (the fp16-storage mode: 3 more mantissa bits than bf16)
struct RawF { float4 a, b; };      // 8 f32

template <typename T> struct Tr;
template <> struct Tr<__bf16> { using Raw = RawB; };
template <> struct Tr<_Float16> { using Raw = RawH; };
template <> struct Tr<float> { using Raw = RawF; };

__device__ __forceinline__ void zero(RawB &r) { r.v = make_uint4(0, 0, 0, 0); }
__device__ __forceinline__ void zero(RawH &r) { r.v = make_uint4(0, 0, 0, 0); }
__device__ __forceinline__ void ld8(RawH &r, const _Float16 *p) { r.v = *reinterpret_cast<const uint4 *>(p); }
__device__ __forceinline__ void set3(RawH &r, float a, float b, float c) {
    f16x8 v = {(_Float16)a, (_Float16)b, (_Float16)c, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
    r.v = __builtin_bit_cast(uint4, v);
}
__device__ __forceinline__ void set8(RawH &r, const _Float16 (&v)[8]) {
    f16x8 b = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
    r.v = __builtin_bit_cast(uint4, b);
}
__device__ __forceinline__ void mma(f32x4 &acc, const RawH &w, const RawH &x) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, w.v), __builtin_bit_cast(f16x8, x.v), acc, 0, 0, 0);
}
__device__ __forceinline__ void zero(RawF &r) { r.a = make_float4(0.f, 0.f, 0.f, 0.f); r.b = r.a; }
__device__ __forceinline__ void ld8(RawB &r, const __bf16 *p) { r.v = *reinterpret_cast<const uint4 *>(p); }
__device__ __forceinline__ void ld8(RawF &r, const float *p) {
    r.a = reinterpret_cast<const float4 *>(p)[0];
    r.b = reinterpret_cast<const float4 *>(p)[1];
}

__device__ __forceinline__ void set3(RawB &r, float a, float b, float c) {
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    bf16x8 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
    r.v = __builtin_bit_cast(uint4, v);
}
__device__ __forceinline__ void set3(RawF &r, float a, float b, float c) {
    r.a = make_float4(a, b, c, 0.f);
    r.b = make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ void set8(RawB &r, const __bf16 (&v)[8]) {
    bf16x8 b = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
    r.v = __builtin_bit_cast(uint4, b);
}
__device__ __forceinline__ void set8(RawF &r, const float (&v)[8]) {
    r.a = make_float4(v[0], v[1], v[2], v[3]);
    r.b = make_float4(v[4], v[5], v[6], v[7]);
}

__device__ __forceinline__ void mma(f32x4 &acc, const RawB &w, const RawB &x) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w.v), __builtin_bit_cast(bf16x8, x.v),
                                                  acc, 0, 0, 0);
}
// fp32 parity mode, round 4: split-f16 products. The weights are packed on the host as two f16
// parts per element (bugseg_runtime.cpp Packer::push_w: hi = f16(w), lo = f16(w - hi); every 8
// consecutive k of a row are 32 B, the 8 hi parts then the 8 lo parts — the bytes of 8 floats), the
// f32 activation operand is split the same way in registers, and one f32 product becomes three
// v_mfma_f32_16x16x32_f16 (lo*hi + hi*lo + hi*hi, products exact in f32, f32 accumulation; the
// dropped lo*lo term and the parts' rounding leave ~2^-21 relative per product). 48 MFMA cycles per
// 32-k step instead of 256 for the 8 exact v_mfma_f32_16x16x4_f32. Emulated end to end at 480 x 640
// (scripts/split_precision_probe.py): max |dlogit| vs the fp32 oracle 2.1e-5 (exact f32 products:
// 1.5e-5), near-tie share 4.9e-5 (4.2e-5); bf16 splits need 6 products for the same (3 give 3.6).
// Operands must lie within the f16 range (|v| < 65504; f16 subnormals are kept: MODE.denorm).
struct RawS { uint4 h, l; };       // 8 weights as f16 hi parts + 8 f16 lo parts (fp32 mode)
template <typename T> struct WTr { using Raw = typename Tr<T>::Raw; };
template <> struct WTr<float> { using Raw = RawS; };
__device__ __forceinline__ void ld8(RawS &r, const float *p) {
    r.h = reinterpret_cast<const uint4 *>(p)[0];
    r.l = reinterpret_cast<const uint4 *>(p)[1];
}
__device__ __forceinline__ void zero(RawS &r) { r.h = make_uint4(0, 0, 0, 0); r.l = r.h; }
// the hi / lo f16 parts of element k of a packed fp32-mode weight row
__device__ __forceinline__ void wsplit_elem(const float *row, int k, _Float16 &hi, _Float16 &lo) {
    const _Float16 *p = reinterpret_cast<const _Float16 *>(row) + (k >> 3) * 16 + (k & 7);
    hi = p[0];
    lo = p[8];
}
__device__ __forceinline__ void set8(RawS &r, const _Float16 (&hi)[8], const _Float16 (&lo)[8]) {
    const f16x8 h = {hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
    const f16x8 l = {lo[0], lo[1], lo[2], lo[3], lo[4], lo[5], lo[6], lo[7]};
    r.h = __builtin_bit_cast(uint4, h);
    r.l = __builtin_bit_cast(uint4, l);
}
// x = hi + lo: hi = f16(x) (round to nearest even), lo = f16(x - hi) (x - hi is exact in f32). (A form
// with lo from v_fma_mixlo/mixhi_f16 — one instruction per element instead of ~2.5 — gave 1.6e-3 at
// 480 x 640 instead of 1.7e-5 on the GPU: those instructions evidently flush f16 subnormals, which the
// lo parts of small values are. The plain conversions keep them.)
__device__ __forceinline__ void split_f16(const RawF &x, f16x8 &hi, f16x8 &lo) {
    const float v[8] = {x.a.x, x.a.y, x.a.z, x.a.w, x.b.x, x.b.y, x.b.z, x.b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const _Float16 h = (_Float16)v[i];
        hi[i] = h;
        lo[i] = (_Float16)(v[i] - (float)h);
    }
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
// 2 floats times a (wave-uniform) scale, one v_pk_mul_f32; opaque to the compiler, which would fuse a
// scalar multiply feeding an f16 conversion into v_fma_mix* (those flush f16 subnormals: split_f16)
__device__ __forceinline__ f32x2 pkmul(f32x2 v, f32x2 s) {
    f32x2 r;
    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(v), "s"(s));
    return r;
}
#ifndef BUGSEG_RANGE
#define BUGSEG_RANGE 31    // fp32 range scaling; A/B builds clear bits to compile parts out: 1 operand scale8,
#endif                     // 2 accumulator mul4, 4 output max tracking (rng_acc / rng_commit), 8 mulp2, 16 rng_read
__device__ __forceinline__ RawF scale8(const RawF &x, float m) {
    if constexpr (!(BUGSEG_RANGE & 1)) return x;
    const f32x2 s = {m, m};
    const f32x2 a0 = pkmul((f32x2){x.a.x, x.a.y}, s), a1 = pkmul((f32x2){x.a.z, x.a.w}, s);
    const f32x2 b0 = pkmul((f32x2){x.b.x, x.b.y}, s), b1 = pkmul((f32x2){x.b.z, x.b.w}, s);
    RawF r;
    r.a = make_float4(a0.x, a0.y, a1.x, a1.y);
    r.b = make_float4(b0.x, b0.y, b1.x, b1.y);
    return r;
}
__device__ __forceinline__ void mma(f32x4 &acc, const RawS &w, const RawF &x) {
    f16x8 xh, xl;
    split_f16(x, xh, xl);
    const f16x8 wh = __builtin_bit_cast(f16x8, w.h), wl = __builtin_bit_cast(f16x8, w.l);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xh, acc, 0, 0, 0);
}
// both operands already split (fp32-mode activations stored as split parts, bneck_kernels.hip): the
// same three products in the same order as above, so the same result bit for bit
__device__ __forceinline__ void mma(f32x4 &acc, const RawS &w, const RawS &x) {
    const f16x8 wh = __builtin_bit_cast(f16x8, w.h), wl = __builtin_bit_cast(f16x8, w.l);
    const f16x8 xh = __builtin_bit_cast(f16x8, x.h), xl = __builtin_bit_cast(f16x8, x.l);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xh, acc, 0, 0, 0);
}
// 4 consecutive channels (first channel % 8 = sub: 0 or 4) of an 8-channel group stored as split-f16
// parts in the weight layout (32 B: the 8 hi parts, then the 8 lo parts), split as split_f16 does
__device__ __forceinline__ void st4s(float *grp, int sub, float4 v) {
    const float e[4] = {v.x, v.y, v.z, v.w};
    _Float16 h[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h[i] = (_Float16)e[i];
        l[i] = (_Float16)(e[i] - (float)h[i]);
    }
    const f16x4 hv = {h[0], h[1], h[2], h[3]}, lv = {l[0], l[1], l[2], l[3]};
    unsigned char *g = reinterpret_cast<unsigned char *>(grp);
    *reinterpret_cast<f16x4 *>(g + 2 * sub) = hv;
    *reinterpret_cast<f16x4 *>(g + 16 + 2 * sub) = lv;
}
// the same split, in the grouped layout of a 32-channel run (bneck_kernels.hip HL: the four 8-channel
// groups' hi parts, 16 B each, then their lo parts): 4 consecutive channels from ch (ch % 4 == 0)
__device__ __forceinline__ void st4hl(float *run, int ch, float4 v) {
    const float e[4] = {v.x, v.y, v.z, v.w};
    _Float16 h[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h[i] = (_Float16)e[i];
        l[i] = (_Float16)(e[i] - (float)h[i]);
    }
    const f16x4 hv = {h[0], h[1], h[2], h[3]}, lv = {l[0], l[1], l[2], l[3]};
    unsigned char *g = reinterpret_cast<unsigned char *>(run) + (ch >> 3) * 16 + (ch & 7) * 2;
    *reinterpret_cast<f16x4 *>(g) = hv;
    *reinterpret_cast<f16x4 *>(g + 64) = lv;
}
// exact f32 products (DeepLab's fp32 mode): sub-MFMA j contracts element j of every lane's 8-group
// (lane>>4 = group), so the 8 sub-MFMAs together cover the same 32 k as one bf16 MFMA.
__device__ __forceinline__ void mma(f32x4 &acc, const RawF &w, const RawF &x) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.a.x, x.a.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.a.y, x.a.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.a.z, x.a.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.a.w, x.a.w, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.b.x, x.b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.b.y, x.b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.b.z, x.b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.b.w, x.b.w, acc, 0, 0, 0);
}

__device__ __forceinline__ float4 ld4f(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 ld4(const __bf16 *p) {
    uint2 u = *reinterpret_cast<const uint2 *>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }
__device__ __forceinline__ void st4(__bf16 *p, float4 v) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 b = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    *reinterpret_cast<bf16x4 *>(p) = b;
}
// 4 floats <-> 4 bf16 packed in two dwords (round to nearest even, as the (__bf16) casts of st4)
__device__ __forceinline__ u32x2_t pack_bf16x4(float4 v) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 b = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    return __builtin_bit_cast(u32x2_t, b);
}
__device__ __forceinline__ float4 unpack_bf16x4(u32x2_t u) {
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
// 4 floats <-> 4 f16 in two dwords (round to nearest even, as the (_Float16) casts)
__device__ __forceinline__ u32x2_t pack_f16x4(float4 v) {
    f16x4 b = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    return __builtin_bit_cast(u32x2_t, b);
}
__device__ __forceinline__ float4 unpack_f16x4(u32x2_t u) {
    const f16x4 h = __builtin_bit_cast(f16x4, u);
    return make_float4((float)h.x, (float)h.y, (float)h.z, (float)h.w);
}
// the storage format of a 2-byte element type T (bf16 or f16)
template <typename T> __device__ __forceinline__ u32x2_t pack4(float4 v);
template <> __device__ __forceinline__ u32x2_t pack4<__bf16>(float4 v) { return pack_bf16x4(v); }
template <> __device__ __forceinline__ u32x2_t pack4<_Float16>(float4 v) { return pack_f16x4(v); }
template <typename T> __device__ __forceinline__ float4 unpack4(u32x2_t u);
template <> __device__ __forceinline__ float4 unpack4<__bf16>(u32x2_t u) { return unpack_bf16x4(u); }
template <> __device__ __forceinline__ float4 unpack4<_Float16>(u32x2_t u) { return unpack_f16x4(u); }
__device__ __forceinline__ float4 ld4(const _Float16 *p) { return unpack_f16x4(*reinterpret_cast<const u32x2_t *>(p)); }
__device__ __forceinline__ void st4(_Float16 *p, float4 v) { *reinterpret_cast<u32x2_t *>(p) = pack_f16x4(v); }

// v_permlane16_swap_b32 (gfx950): lanes of the odd 16-lane rows of `a` trade places with the lanes
// of the even rows of `b` one row below (lane l of row 2i+1 of a <-> lane l-16 of row 2i of b).
// An involution; measured on MI355X with scripts/permlane_probe.hip.
__device__ __forceinline__ void pl16swap(uint32_t &a, uint32_t &b) {
    const u32x2_t r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r.x;
    b = r.y;
}
// v_permlane32_swap: lanes 32-63 of a <-> lanes 0-31 of b
__device__ __forceinline__ void pl32swap(uint32_t &a, uint32_t &b) {
    const u32x2_t r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r.x;
    b = r.y;
}


__device__ __forceinline__ float ld1(const float *p) { return *p; }
__device__ __forceinline__ float ld1(const __bf16 *p) { return (float)*p; }
__device__ __forceinline__ float ld1(const _Float16 *p) { return (float)*p; }

// ---- buffer (SRSRC) memory ops: 32-bit byte offsets against a wave-uniform descriptor built from
// kernel arguments; an offset past the descriptor's size reads 0 and drops a store, which is how
// padding taps and masked lanes are handled without branches (OOB = any offset >= 2^31 here).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mkbuf(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bst16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, 0);
}
// Stores of a launch's output, which the launch itself never reads back: cache policy AUX (0 =
// default; 16 = sc1 write-through, the line leaves the XCD's L2; 2 = nt), so a kernel's output
// stream does not evict the input lines its neighbouring tiles still re-read from L2 (the phase-3
// residual, the halo rows of the next tile band). OUT_AUX_SEL(sel) names the per-kernel choice
// (sc1 for the C >= 64 bottleneck / C128 up / initial kernels), built with -DBUGSEG_OUT_AUX=-1.
// Measured (round 2, same box, alternating A/B twice): it makes those kernels 3-6% faster one stream
// at a time (C128 26.8 -> 25.4 us, PMC reads 66 -> 62 MB per launch) but the 2-stream bench 2.4%
// slower (37.1k -> 36.2k frames/s; why is not pinned down: with two shards interleaved, write-back
// lines still in L2 evidently serve more reads than they evict). So the default is 0 (off), except
// in bneck_kernels.hip and init_kernels.hip, re-measured after the kept residual and the LDS-DMA staging:
// 4-9% faster per launch and equal in the 2-stream bench, so those files select per kernel (-1).
#ifndef BUGSEG_OUT_AUX
#define BUGSEG_OUT_AUX 0
#endif
#define OUT_AUX_SEL(sel) (BUGSEG_OUT_AUX >= 0 ? BUGSEG_OUT_AUX : (sel))
template <int AUX>
__device__ __forceinline__ void bst16o(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void bst8o(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x2 v) {
    __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, AUX);
}
__device__ __forceinline__ void bld8(RawB &x, __amdgpu_buffer_rsrc_t r, uint32_t off) { x.v = bld16(r, off); }
__device__ __forceinline__ void bld8(RawH &x, __amdgpu_buffer_rsrc_t r, uint32_t off) { x.v = bld16(r, off); }
__device__ __forceinline__ void bld8(RawF &x, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    x.a = __builtin_bit_cast(float4, bld16(r, off));
    x.b = __builtin_bit_cast(float4, bld16(r, off + 16));
}
// 4 consecutive elements -> float4
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off, const float *) {
    return __builtin_bit_cast(float4, bld16(r, off));
}
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off, const __bf16 *) {
    const u32x2 u = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off, const _Float16 *) {
    return unpack_f16x4(__builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}

// 4 consecutive elements kept raw (prefetched early, converted where used)
template <typename T> struct MvRawT;
template <> struct MvRawT<__bf16> { using type = u32x2; };
template <> struct MvRawT<_Float16> { using type = u32x2; };
template <> struct MvRawT<float> { using type = u32x4; };
template <typename T> using MvRaw = typename MvRawT<T>::type;
template <typename T> __device__ __forceinline__ MvRaw<T> mvload(__amdgpu_buffer_rsrc_t r, uint32_t off);
template <> __device__ __forceinline__ u32x2 mvload<__bf16>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
}
template <> __device__ __forceinline__ u32x2 mvload<_Float16>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
}
template <> __device__ __forceinline__ u32x4 mvload<float>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
}
template <typename T> __device__ __forceinline__ float4 mvcvt(MvRaw<T> u);
template <> __device__ __forceinline__ float4 mvcvt<__bf16>(u32x2 u) {
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
template <> __device__ __forceinline__ float4 mvcvt<_Float16>(u32x2 u) { return unpack_f16x4(u); }
template <> __device__ __forceinline__ float4 mvcvt<float>(u32x4 u) {
    return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}

// Division by a runtime-invariant divisor d via a host-computed magic number (bugseg_runtime.cpp
// fastdiv()): q = umulhi(n, m) >> s for d >= 2, s < 0 encodes d == 1. Exact for 0 <= n < 2^31.
__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint32_t m, int s) {
    return s < 0 ? n : (__umulhi(n, m) >> s);
}

__device__ __forceinline__ float prelu(float v, float s) { return v > 0.f ? v : v * s; }
// == prelu when s <= 1 (v > 0: v*s <= v; v < 0: v*s >= v): 2 VALU instead of 3
// (a bare v_max_f32: fmaxf would add a NaN-quieting v_max per operand in IEEE mode)
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// storage rounding of an activation (the unfused plan stores it as T and reads it back)
__device__ __forceinline__ float4 round_t(float4 v, const __bf16 *) { return unpack_bf16x4(pack_bf16x4(v)); }
__device__ __forceinline__ float4 round_t(float4 v, const _Float16 *) { return unpack_f16x4(pack_f16x4(v)); }
__device__ __forceinline__ float4 round_t(float4 v, const float *) { return v; }

// Two 16-channel row fragments (quads qa, qb: lane kq holds channels 4kq..4kq+3 of each) -> the B
// operand of one 32-channel k-step (lane kq holds channels 8kq..8kq+7):
//   permlane32_swap: lanes kq 2,3 of qa <- lanes kq 0,1 of qb, lanes kq 0,1 of qb <- kq 2,3 of qa;
//   permlane16_swap: odd rows of qa' <-> even rows of qb'.
// Afterwards lane kq holds (qa'', qb'') = channels 8kq..8kq+3 and 8kq+4..8kq+7 (measured semantics:
// scripts/permlane_probe.hip). qb == 0 for a single fragment (k groups 2, 3 zero).
__device__ __forceinline__ void to_bop(RawB &r, float4 qa, float4 qb) {
    const u32x2_t a = pack_bf16x4(qa), b = pack_bf16x4(qb);
    uint32_t a0 = a.x, a1 = a.y, b0 = b.x, b1 = b.y;
    pl32swap(a0, b0);
    pl32swap(a1, b1);
    pl16swap(a0, b0);
    pl16swap(a1, b1);
    r.v = make_uint4(a0, a1, b0, b1);
}
__device__ __forceinline__ void to_bop(RawH &r, float4 qa, float4 qb) {
    const u32x2_t a = pack_f16x4(qa), b = pack_f16x4(qb);
    uint32_t a0 = a.x, a1 = a.y, b0 = b.x, b1 = b.y;
    pl32swap(a0, b0);
    pl32swap(a1, b1);
    pl16swap(a0, b0);
    pl16swap(a1, b1);
    r.v = make_uint4(a0, a1, b0, b1);
}
__device__ __forceinline__ void to_bop(RawF &r, float4 qa, float4 qb) {
    uint32_t a[4] = {__float_as_uint(qa.x), __float_as_uint(qa.y), __float_as_uint(qa.z), __float_as_uint(qa.w)};
    uint32_t b[4] = {__float_as_uint(qb.x), __float_as_uint(qb.y), __float_as_uint(qb.z), __float_as_uint(qb.w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        pl32swap(a[i], b[i]);
        pl16swap(a[i], b[i]);
    }
    r.a = make_float4(__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[2]), __uint_as_float(a[3]));
    r.b = make_float4(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[2]), __uint_as_float(b[3]));
}

// Launch spans (bugseg_debug_set_spans; null in normal runs — one scalar test per workgroup): thread 0
// of every workgroup folds the constant 100 MHz clock (s_memrealtime, one time base across XCDs) into
// its slot's [0] at entry (min) and [1] at exit (max) — 64 slots, 64 B apart, by workgroup index, so
// the atomics do not queue on one address — and the host's min / max over the slots is the launch's
// duration as the profiler defines it (first workgroup start to last workgroup end).
constexpr int SPAN_SLOTS = 64, SPAN_STRIDE = 8;     // u64 per slot stride (64 B)
__device__ __forceinline__ void span_enter(unsigned long long *s) {
    if (s && threadIdx.x == 0)
        atomicMin(s + (blockIdx.x & (SPAN_SLOTS - 1)) * SPAN_STRIDE, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void span_exit(unsigned long long *s) {
    if (s && threadIdx.x == 0)
        atomicMax(s + (blockIdx.x & (SPAN_SLOTS - 1)) * SPAN_STRIDE + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// ---- fp32 mode range scaling (round 5; bugseg_internal.h RangeArgs). Exponents are clamped to
// [-RNG_EMAX, RNG_EMAX] (tensors of max |v| in [2^-26, 2^54] are scaled exactly into the window; beyond
// that the split degrades gracefully) so every multiplier, a difference of two exponents plus a weight
// exponent, stays a normal float. Everything here is wave-uniform: exponents are scalars
// (readfirstlane) and multipliers are built from their bits on the scalar unit.
constexpr int RNG_EMAX = 40;
__device__ __forceinline__ int rng_clamp(int e) { return e < -RNG_EMAX ? -RNG_EMAX : e > RNG_EMAX ? RNG_EMAX : e; }
// floor(log2 m) of a finite m > 0
__device__ __forceinline__ int rng_log2(float m) { return __builtin_amdgcn_readfirstlane(__builtin_amdgcn_frexp_expf(m)) - 1; }
// a measured max |v| = m: 0 while m lies in [2^-2, 2^15) (or is 0 / not finite), else the exponent
// that brings it to [2^14, 2^15)
__device__ __forceinline__ int rng_exp_meas(float m) {
    if (!(m > 0.f) || !(m < INFINITY)) return 0;
    const int l = rng_log2(m);
    return l >= -2 && l < 15 ? 0 : rng_clamp(14 - l);
}
// a rigorous bound B of |t|: the preferred exponent p (the accumulator's, so no multiply) while the
// scaled bound lies in [2^3, 2^15), else the exponent that brings B to [2^14, 2^15). A bound that is
// not finite (|t| may exceed f32 itself) takes the largest down-scale, never the unscaled p; p itself
// (an accumulator exponent: a tensor exponent plus a weight exponent) is clamped to +-2 RNG_EMAX, so a
// chained accumulator exponent (this plus the next weight's) stays within +-3 RNG_EMAX = +-120
__device__ __forceinline__ int rng_exp_bound(float B, int p) {
    p = p < -2 * RNG_EMAX ? -2 * RNG_EMAX : p > 2 * RNG_EMAX ? 2 * RNG_EMAX : p;
    if (!(B < INFINITY)) return -RNG_EMAX;
    if (!(B > 0.f)) return p;
    const int l = rng_log2(B);
    return l + p >= 3 && l + p < 15 ? p : rng_clamp(14 - l);
}
// 2^e as a scalar: v_ldexp_f32 saturates (0 / inf beyond f32) where building the exponent bits would
// wrap into the sign or exponent field for |e| > 126 (a difference of two chained exponents can reach
// that only for pathological ranges); readfirstlane keeps it an SGPR. (Clamping e on the scalar unit
// instead cost the fp32 down C64 form 14 VGPRs and its third wave per SIMD: 141 -> 157 us per launch)
__device__ __forceinline__ float rng_pow2(int e) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(__builtin_ldexpf(1.f, e))));
}
// max |v| of a launch's input: the RNG_SLOTS words (four per lane, then a wave reduction)
// rng_read in two halves: the lane's slot load (issue it early) and the wave reduction (consume it
// after the launch's first operand loads are in flight, so no wave waits a memory latency for it alone)
__device__ __forceinline__ float rng_lane(const RangeArgs &r) {
    if constexpr (!(BUGSEG_RANGE & 16)) return 0.f;
    if (!r.amax_in) return r.amax_static;
    static_assert(RNG_SLOTS == 256, "one float4 of slots per lane");
    const float4 q = reinterpret_cast<const float4 *>(r.amax_in)[threadIdx.x & 63];
    return __builtin_fmaxf(__builtin_fmaxf(q.x, q.y), __builtin_fmaxf(q.z, q.w));
}
__device__ __forceinline__ float rng_reduce(float m) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, o));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(m)));
}
__device__ __forceinline__ float rng_read(const RangeArgs &r) { return rng_reduce(rng_lane(r)); }
// m = max(m, |v|) (v_max3 with abs modifiers: NaN operands are ignored, as v_max does)
// (compiler-visible maxNum of |.|: v_max_f32 with abs modifiers then one v_max3 into m — a chain of one
// dependent op per quad, schedulable; NaN operands are ignored, as v_max does)
__device__ __forceinline__ void rng_acc(float &m, float a, float b) {
    if constexpr (!(BUGSEG_RANGE & 4)) return;
    m = __builtin_fmaxf(m, __builtin_fmaxf(__builtin_fabsf(a), __builtin_fabsf(b)));
}
__device__ __forceinline__ void rng_acc4(float &m, float4 v) {
    if constexpr (!(BUGSEG_RANGE & 4)) return;
    m = __builtin_fmaxf(m, __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(v.x), __builtin_fabsf(v.y)),
                                           __builtin_fmaxf(__builtin_fabsf(v.z), __builtin_fabsf(v.w))));
}
// the wave's max into the launch's output words (a global atomic max on the float bits: |v| >= 0
// orders as unsigned; one slot per wave modulo RNG_SLOTS, so the atomics do not pile on one word)
__device__ __forceinline__ void rng_commit(float m, float *slots) {
    if (!(BUGSEG_RANGE & 4) || !slots) return;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, o));
    // (slot: this wave's index in the grid: the waves' atomics spread over every slot — 64 slots by
    // workgroup measured 4 us per C128 launch of same-address atomics queueing at the memory side)
    const unsigned wg = blockIdx.x * ((blockDim.x + 63) >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && m > 0.f)
        atomicMax(reinterpret_cast<unsigned int *>(slots) + (wg & (RNG_SLOTS - 1)), __float_as_uint(m));
}
// the workgroup's max into the output words with ONE atomic (rng_commit's per-wave atomics measured
// ~2-4 us per fp32 C128 launch: 8 waves x 256 workgroups on 256 words). Every wave of the workgroup
// calls it at the kernel's end; wm: NW floats of LDS nothing else uses any more (two barriers)
__device__ __forceinline__ void rng_commit_wg(float m, float *slots, float *wm, int nw) {
    if (!(BUGSEG_RANGE & 4) || !slots) return;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, o));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) wm[wave] = m;
    __syncthreads();
    if (wave == 0) {
        float t = lane < nw ? wm[lane] : 0.f;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t = __builtin_fmaxf(t, __shfl_xor(t, o));
        if (lane == 0 && t > 0.f)
            atomicMax(reinterpret_cast<unsigned int *>(slots) + (blockIdx.x & (RNG_SLOTS - 1)), __float_as_uint(t));
    }
}
__device__ __forceinline__ f32x4 mul4(f32x4 v, float s) {
    if constexpr (!(BUGSEG_RANGE & 2)) return v;
    return (f32x4){v[0] * s, v[1] * s, v[2] * s, v[3] * s};
}
__device__ __forceinline__ float4 mul4(float4 v, float s) {
    if constexpr (!(BUGSEG_RANGE & 2)) return v;
    return make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
}
// x *= s before a split, as an opaque v_mul_f32: a plain multiply feeding an f16 conversion is fused by
// the compiler into v_fma_mix*, which flushes f16 subnormals (see split_f16)
__device__ __forceinline__ float mulp2(float v, float s) {
    if constexpr (!(BUGSEG_RANGE & 8)) return v;
    float r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(s));
    return r;
}
__device__ __forceinline__ float4 mulp2(float4 v, float s) { return make_float4(mulp2(v.x, s), mulp2(v.y, s), mulp2(v.z, s), mulp2(v.w, s)); }
__device__ __forceinline__ void mul8(RawF &x, float s) {
    x.a = mulp2(x.a, s);
    x.b = mulp2(x.b, s);
}

// the fused bottleneck's exponents (bneck_kernels.hip, bneck2_kernels.hip): the multipliers of x, of
// the accumulators and of the internal tensors, from the launch's input range and the weights' bounds
struct BneckRange {
    float xm = 1.f, b1m = 1.f, o1m = 1.f, b2m = 1.f, o2m = 1.f, b2bm = 1.f, o2bm = 1.f, b3m = 1.f, o3m = 1.f;
    int rs1 = 0, re2b = 0;                            // asymmetric: t1a's exponent, the 1x5's accumulator exponent
    bool scl = false, any = false;                    // scl: phase 3 multiplies (e3 != 0)
};
template <bool ASYM>
__device__ __forceinline__ BneckRange bneck_range(const RangeArgs &g, float amx) {
    BneckRange r;
    if (g.off) return r;
    const int sx = rng_exp_meas(amx), e1 = sx + g.sw[0];
    const float B0 = g.n[0] * amx + g.c[0];
    const int s0 = rng_exp_bound(B0, e1), e2 = s0 + g.sw[1];
    const float B1 = g.n[1] * B0 + g.c[1];
    const int s1 = rng_exp_bound(B1, e2);
    int e2b = 0, s1b = 0;
    if constexpr (ASYM) {
        e2b = s1 + g.sw[2];
        s1b = rng_exp_bound(g.n[2] * B1 + g.c[2], e2b);
    }
    const int e3 = (ASYM ? s1b : s1) + g.sw[3];
    r.rs1 = s1; r.re2b = e2b;
    r.scl = e3 != 0;
    r.xm = rng_pow2(sx); r.b1m = rng_pow2(e1); r.o1m = rng_pow2(s0 - e1); r.b2m = rng_pow2(e2); r.o2m = rng_pow2(s1 - e2);
    r.b2bm = rng_pow2(e2b); r.o2bm = rng_pow2(s1b - e2b); r.b3m = rng_pow2(e3); r.o3m = rng_pow2(-e3);
    r.any = (sx | e1 | s0 | e2 | s1) != 0 || (ASYM ? (e2b != 0 || g.sw[3] != 0) : e3 != 0);
    return r;
}

__device__ __forceinline__ float4 prelu4m(float4 v, float4 s) {
    return make_float4(vmax(v.x, v.x * s.x), vmax(v.y, v.y * s.y), vmax(v.z, v.z * s.z), vmax(v.w, v.w * s.w));
}
// Accumulators start at the bias (the MFMA adds it for free) for outputs of fewer than 8 16-row
// fragments; with 8 (128 channels) the bias comes after, since bias-initialised accumulators are live
// across the k loop's loads and would spill. Both kernels follow this rule, so a fused bottleneck and
// its unfused launches stay bit-identical.
// A single-k-step launch (K <= 32: the 1x1 expansions, the up-block transposed conv) has no k loop
// for the bias-initialised accumulators to live across, so it always starts from the bias.
__host__ __device__ constexpr bool bias_in_acc(int nr, int ksteps = 2) { return nr < 8 || ksteps == 1; }
__device__ __forceinline__ f32x4 bias4(const float *p) {
    const float4 b = *reinterpret_cast<const float4 *>(p);
    return (f32x4){b.x, b.y, b.z, b.w};
}
__device__ __forceinline__ float4 prelu4(float4 v, float4 s) {
    return make_float4(prelu(v.x, s.x), prelu(v.y, s.y), prelu(v.z, s.z), prelu(v.w, s.w));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 f4(const f32x4 &v) { return make_float4(v[0], v[1], v[2], v[3]); }
__device__ __forceinline__ float get(const float4 &v, int r) { return r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w; }

}  // namespace bugseg
