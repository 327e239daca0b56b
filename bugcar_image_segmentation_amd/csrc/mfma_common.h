// Device helpers shared by the MFMA kernels (conv_kernels.hip, bneck_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace bugseg {

// LDS hand-off between lanes of ONE wave: wait for the wave's LDS operations, keep the compiler
// from moving memory operations across (no s_barrier needed inside a wave).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct RawB { uint4 v; };          // 8 bf16
struct RawF { float4 a, b; };      // 8 f32

template <typename T> struct Tr;
template <> struct Tr<__bf16> { using Raw = RawB; };
template <> struct Tr<float> { using Raw = RawF; };

__device__ __forceinline__ void zero(RawB &r) { r.v = make_uint4(0, 0, 0, 0); }
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

__device__ __forceinline__ void mma(f32x4 &acc, const RawB &w, const RawB &x) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w.v), __builtin_bit_cast(bf16x8, x.v),
                                                  acc, 0, 0, 0);
}
// fp32 parity mode: sub-MFMA j contracts element j of every lane's 8-group (lane>>4 = group),
// so the 8 sub-MFMAs together cover the same 32 k as one bf16 MFMA (exact f32 products).
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
__device__ __forceinline__ float ld1(const float *p) { return *p; }
__device__ __forceinline__ float ld1(const __bf16 *p) { return (float)*p; }

__device__ __forceinline__ float prelu(float v, float s) { return v > 0.f ? v : v * s; }
__device__ __forceinline__ float4 prelu4(float4 v, float4 s) {
    return make_float4(prelu(v.x, s.x), prelu(v.y, s.y), prelu(v.z, s.z), prelu(v.w, s.w));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 f4(const f32x4 &v) { return make_float4(v[0], v[1], v[2], v[3]); }
__device__ __forceinline__ float get(const float4 &v, int r) { return r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w; }

}  // namespace bugseg
