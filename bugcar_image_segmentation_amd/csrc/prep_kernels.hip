// ENET.preprocess (models.py:84-95) on the GPU, batched, plus the NCHW -> engine-input layout
// change for ENET.predict's feed (models.py:43-44).
//
// One thread per output pixel. The resize reproduces cv2.resize INTER_LINEAR on u8 (classic
// resizeGeneric_ fixed point, coefficient tables built on the host exactly as OpenCV builds
// them, see bugseg_runtime.cpp::build_resize_tables); the normalisation (x/256 - mean)/std is
// a per-channel 256-entry float64 table computed on the host with the reference's expression,
// so the f64 output equals NumPy's bit for bit and the f32 / bf16 outputs are its roundings.
// HBM-bound: 3 B read (x up to 4 taps, L1/L2-served) + 16 B (bf16 engine layout) written per pixel.
#include <algorithm>

#include "bugseg_internal.h"
#include "mfma_common.h"
#include "../../include/bugseg.h"

namespace bugseg {

__device__ __forceinline__ int sat16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
__device__ __forceinline__ int satu8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

__global__ void __launch_bounds__(256) preprocess_kernel(const PreArgs a) {
    const long total = (long)a.B * a.H * a.W;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int x = (int)(i % a.W);
        const long t = i / a.W;
        const int y = (int)(t % a.H);
        const int b = (int)(t / a.H);
        const uint8_t *src = a.bgr + (size_t)b * a.H0 * a.W0 * 3;
        int bgr[3];
        if (a.mode == 0) {
            const uint8_t *p = src + ((size_t)y * a.W0 + x) * 3;
            bgr[0] = p[0]; bgr[1] = p[1]; bgr[2] = p[2];
        } else if (a.mode == 1) {
            const uint8_t *p = src + ((size_t)(2 * y) * a.W0 + 2 * x) * 3;
            const size_t rs = (size_t)a.W0 * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) bgr[c] = (p[c] + p[c + 3] + p[rs + c] + p[rs + c + 3] + 2) >> 2;
        } else {
            const int sy0 = a.yofs[y], sy1 = sy0 + 1 < a.H0 ? sy0 + 1 : a.H0 - 1;
            const int b0 = a.yb[2 * y], b1 = a.yb[2 * y + 1];
            const int sx = a.xofs[x], a0 = a.xa[2 * x], a1 = a.xa[2 * x + 1];
            const uint8_t *r0 = src + (size_t)sy0 * a.W0 * 3, *r1 = src + (size_t)sy1 * a.W0 * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                int h0 = r0[sx * 3 + c] * a0, h1 = r1[sx * 3 + c] * a0;
                if (a1) { h0 += r0[(sx + 1) * 3 + c] * a1; h1 += r1[(sx + 1) * 3 + c] * a1; }
                int v;
                if (x * 3 + c < a.vec_end)       // VResizeLinearVec_32s8u rounding
                    v = satu8((((sat16(h0 >> 4) * b0) >> 16) + ((sat16(h1 >> 4) * b1) >> 16) + 2) >> 2);
                else                             // scalar FixedPtCast<int, uchar, 22>
                    v = satu8((h0 * b0 + h1 * b1 + (1 << 21)) >> 22);
                bgr[c] = v;
            }
        }
        if (a.out_layout == BUGSEG_PRE_BGR_U8) {
            uint8_t *o = reinterpret_cast<uint8_t *>(a.out) + i * 3;
            o[0] = (uint8_t)bgr[0]; o[1] = (uint8_t)bgr[1]; o[2] = (uint8_t)bgr[2];
            continue;
        }
        // BGR -> RGB (models.py:89), then the normalisation table (models.py:91)
        const double r = a.lut[0 * 256 + bgr[2]], g = a.lut[1 * 256 + bgr[1]], bl = a.lut[2 * 256 + bgr[0]];
        if (a.out_layout == BUGSEG_PRE_ENGINE) {
            if (a.prec == PREC_BF16) {
                typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
                bf16x8 v = {(__bf16)(float)r, (__bf16)(float)g, (__bf16)(float)bl, (__bf16)0.f,
                            (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
                reinterpret_cast<bf16x8 *>(a.out)[i] = v;
            } else if (a.prec == PREC_F16) {
                f16x8 v = {(_Float16)(float)r, (_Float16)(float)g, (_Float16)(float)bl, (_Float16)0.f,
                           (_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
                reinterpret_cast<f16x8 *>(a.out)[i] = v;
            } else {
                float4 *o = reinterpret_cast<float4 *>(a.out) + 2 * i;
                o[0] = make_float4((float)r, (float)g, (float)bl, 0.f);
                o[1] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        } else {
            const size_t plane = (size_t)a.H * a.W, base = (size_t)b * 3 * plane + (size_t)y * a.W + x;
            if (a.out_layout == BUGSEG_PRE_NCHW_F64) {
                double *o = reinterpret_cast<double *>(a.out);
                o[base] = r; o[base + plane] = g; o[base + 2 * plane] = bl;
            } else {
                float *o = reinterpret_cast<float *>(a.out);
                o[base] = (float)r; o[base + plane] = (float)g; o[base + 2 * plane] = (float)bl;
            }
        }
    }
}

hipError_t launch_preprocess(const PreArgs &a, hipStream_t s) {
    const long total = (long)a.B * a.H * a.W;
    long g = (total + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) nchw_to_input_kernel(const NchwArgs a) {
    const long plane = (long)a.H * a.W, total = (long)a.B * plane;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long b = i / plane, p = i - b * plane;
        float v[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const long o = (b * 3 + c) * plane + p;
            v[c] = a.is_f64 ? (float)reinterpret_cast<const double *>(a.x)[o] : reinterpret_cast<const float *>(a.x)[o];
        }
        if (a.prec == PREC_BF16) {
            typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
            bf16x8 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)0.f,
                        (__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
            reinterpret_cast<bf16x8 *>(a.out)[i] = o;
        } else if (a.prec == PREC_F16) {
            f16x8 o = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)0.f,
                       (_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
            reinterpret_cast<f16x8 *>(a.out)[i] = o;
        } else {
            float4 *o = reinterpret_cast<float4 *>(a.out) + 2 * i;
            o[0] = make_float4(v[0], v[1], v[2], 0.f);
            o[1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}

hipError_t launch_nchw_to_input(const NchwArgs &a, hipStream_t s) {
    const long total = (long)a.B * a.H * a.W;
    long g = (total + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(nchw_to_input_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
    return hipGetLastError();
}

// max |x| over n floats into RNG_SLOTS words (the fp32 mode's range of an engine input the caller
// supplied, bugseg_enet_forward; the BGR path's range is the normalisation table's, known statically)
__global__ void __launch_bounds__(256) amax_kernel(const float *x, size_t n, float *slots) {
    float m = 0.f;
    const size_t n4 = n / 4;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        rng_acc4(m, reinterpret_cast<const float4 *>(x)[i]);
    if (blockIdx.x == 0 && threadIdx.x < n - n4 * 4) rng_acc(m, x[n4 * 4 + threadIdx.x], 0.f);
    rng_commit(m, slots);
}
hipError_t launch_amax(const float *x, size_t n, float *slots, hipStream_t s) {
    const size_t blocks = std::min<size_t>((n / 4 + 255) / 256 + 1, 2048);
    hipLaunchKernelGGL(amax_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, n, slots);
    return hipGetLastError();
}

}  // namespace bugseg
