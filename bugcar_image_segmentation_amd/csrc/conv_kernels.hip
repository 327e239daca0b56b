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
// accumulator puts 4 consecutive channels of one pixel in each lane: NHWC stores and residual
// loads are 8/16-byte vectors. The B fragment (8 consecutive k = 8 channels of one input pixel
// at one tap) is one 16-byte (bf16) global load per lane straight into VGPRs — no LDS round
// trip, since every loaded pixel fragment is reused by NR MFMAs in registers. The whole layer's
// weights (<= 37 KB) are staged in LDS once per workgroup; workgroups stride over tiles with an
// XCD-aware mapping (blocks sharing blockIdx%8 walk one contiguous range of tiles, so the 3x3 /
// dilated halo re-reads of neighbouring tiles hit the same XCD's L2).
#include "bugseg_internal.h"
#include "mfma_common.h"

namespace bugseg {

template <int NR> struct Cfg { static constexpr int MR = NR >= 4 ? 2 : 4; };

// LDS carve: [weights Npad x (Kpad+pad)] [tap table] [normalisation table (EPI_INIT_BGR)]
//            [bias, slope1, slope2, pscale: Npad floats each] [4 x output staging]
__host__ __device__ inline size_t conv_const_offset(int es, const ConvArgs &a) {
    const size_t o = (size_t)a.Npad * (a.Kpad + 16 / es) * es + (size_t)a.Ksteps * 4 * sizeof(int) +
                     (a.nlut ? 3 * 256 * sizeof(float) : 0);
    return (o + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t conv_stage_offset(int es, const ConvArgs &a) {
    return conv_const_offset(es, a) + (size_t)4 * a.Npad * sizeof(float);
}

template <typename T, int NR, int EPI>
__global__ void __launch_bounds__(256) conv_kernel(const ConvArgs a) {
    constexpr int MR = Cfg<NR>::MR;
    constexpr int TILE = 4 * MR * 16;
    using Raw = typename Tr<T>::Raw;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6, col = lane & 15, kq = lane >> 4;
    const int KS = a.Kpad + 16 / (int)sizeof(T);                     // LDS row stride (elements)
    T *wl = reinterpret_cast<T *>(smem);
    int *gt = reinterpret_cast<int *>(smem + (size_t)a.Npad * KS * sizeof(T));
    {
        const int cpr = a.Kpad * (int)sizeof(T) / 16;
        const int total = a.Npad * cpr;
        const uint4 *src = reinterpret_cast<const uint4 *>(a.w);
        for (int i = tid; i < total; i += 256) {
            const int r = i / cpr, c = i - r * cpr;
            *reinterpret_cast<uint4 *>(smem + (size_t)r * KS * sizeof(T) + c * 16) = src[i];
        }
        for (int i = tid; i < a.Ksteps * 4; i += 256) gt[i] = a.gtab[i];
        if constexpr (EPI == EPI_INIT_BGR) {
            // normalisation table rounded exactly as the engine-input path rounds it (f64 -> f32 -> T)
            float *lut = reinterpret_cast<float *>(gt + a.Ksteps * 4);
            for (int i = tid; i < 3 * 256; i += 256) lut[i] = (float)(T)(float)a.nlut[i];
        }
        // per-channel epilogue constants (a global load per use would be a long-latency VMEM op
        // in every epilogue)
        float *cst = reinterpret_cast<float *>(smem + conv_const_offset((int)sizeof(T), a));
        for (int i = tid; i < a.Npad; i += 256) {
            cst[i] = a.bias[i];
            cst[a.Npad + i] = a.slope1[i];
            cst[2 * a.Npad + i] = a.slope2[i];
            cst[3 * a.Npad + i] = a.pscale[i];
        }
    }
    __syncthreads();
    const float *cbias = reinterpret_cast<const float *>(smem + conv_const_offset((int)sizeof(T), a));
    const float *cs1 = cbias + a.Npad, *cs2 = cbias + 2 * a.Npad, *cps = cbias + 3 * a.Npad;
    const float *nl = reinterpret_cast<const float *>(gt + a.Ksteps * 4);
    const uint8_t *bgr = reinterpret_cast<const uint8_t *>(a.in);
    T *stage_base = reinterpret_cast<T *>(smem + conv_stage_offset((int)sizeof(T), a));

    const T *in = reinterpret_cast<const T *>(a.in);
    const int HWg = a.Hg * a.Wg;
    // XCD-aware tile walk: gridDim.x is a multiple of 8; group x = blockIdx%8 owns the contiguous
    // chunk [x*C, (x+1)*C) of tiles (speed only; any placement is correct).
    const int G = gridDim.x, grp = blockIdx.x & 7, slot = blockIdx.x >> 3, nslots = G >> 3;
    const int C = (a.ntiles + 7) >> 3;

    for (int i = slot; i < C; i += nslots) {
        const int tile = grp * C + i;
        if (tile >= a.ntiles) break;
        int pn[MR], py[MR], px[MR];
        bool pv[MR];
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            const int p = tile * TILE + wave * MR * 16 + m * 16 + col;
            pv[m] = p < a.M;
            const int pp = pv[m] ? p : 0;
            pn[m] = pp / HWg;
            const int r = pp - pn[m] * HWg;
            py[m] = r / a.Wg;
            px[m] = r - py[m] * a.Wg;
        }
        f32x4 acc[MR][NR];
#pragma unroll
        for (int m = 0; m < MR; ++m)
#pragma unroll
            for (int n = 0; n < NR; ++n) acc[m][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

        int pmax[MR][3];      // EPI_INIT_BGR: running max of the raw bytes over this lane's pool taps
#pragma unroll
        for (int m = 0; m < MR; ++m) pmax[m][0] = pmax[m][1] = pmax[m][2] = -1;
        for (int s = 0; s < a.Ksteps; ++s) {
            const int g = gt[s * 4 + kq];
            const int dy = (int)(signed char)(g & 0xff), dx = (int)(signed char)((g >> 8) & 0xff);
            const int coff = (g >> 16) & 0xffff;
            Raw xf[MR];
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                const int iy = py[m] * a.stride + dy, ix = px[m] * a.stride + dx;
                const bool ok = pv[m] && coff != 0xffff && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
                if constexpr (EPI == EPI_INIT_BGR) {
                    // one tap of the 3x3 s2 p1 window = 3 raw bytes; normalised RGB + 5 zero channels
                    zero(xf[m]);
                    if (ok) {
                        const uint8_t *q = bgr + ((size_t)(pn[m] * a.Hin + iy) * a.Win + ix) * 3;
                        const int b0 = q[0], b1 = q[1], b2 = q[2];
                        set3(xf[m], nl[b2], nl[256 + b1], nl[512 + b0]);
                        if (a.pool_k == 3 || (dy >= 0 && dx >= 0)) {
                            pmax[m][0] = max(pmax[m][0], b2);
                            pmax[m][1] = max(pmax[m][1], b1);
                            pmax[m][2] = max(pmax[m][2], b0);
                        }
                    }
                } else {
                    if (ok)
                        ld8(xf[m], in + ((size_t)(pn[m] * a.Hin + iy) * a.Win + ix) * a.CinS + coff);
                    else
                        zero(xf[m]);
                }
            }
#pragma unroll
            for (int n = 0; n < NR; ++n) {
                Raw wf;
                ld8(wf, wl + (n * 16 + col) * KS + s * 32 + kq * 8);
#pragma unroll
                for (int m = 0; m < MR; ++m) mma(acc[m][n], wf, xf[m]);
            }
        }

        // ------------------------------- epilogues -------------------------------------------
        T *out = reinterpret_cast<T *>(a.out);
        int pmx[MR][3];
#pragma unroll
        for (int m = 0; m < MR; ++m)
#pragma unroll
            for (int c3 = 0; c3 < 3; ++c3) {
                int v = pmax[m][c3];
                if constexpr (EPI == EPI_INIT_BGR) {
                    v = max(v, __shfl_xor(v, 16, 64));
                    v = max(v, __shfl_xor(v, 32, 64));
                }
                pmx[m][c3] = v;
            }
        if constexpr (EPI == EPI_CLASSES) {
            // n fragment = output phase (a,b); rows = 16 (padded) classes, 4 per lane.
#pragma unroll
            for (int m = 0; m < MR; ++m) {
#pragma unroll
                for (int n = 0; n < NR; ++n) {
                    const int c = n * 16 + kq * 4;
                    const float4 b4 = ld4f(cbias + c);
                    const float4 v = add4(f4(acc[m][n]), b4);
                    float best = -INFINITY;
                    int bi = 0x7fffffff;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int cls = kq * 4 + r;
                        const float x = get(v, r);
                        if (cls < a.ncls && x > best) { best = x; bi = cls; }
                    }
                    // lowest class index wins ties (tf.math.argmax, models.py:55)
#pragma unroll
                    for (int off = 16; off <= 32; off <<= 1) {
                        const float ob = __shfl_xor(best, off, 64);
                        const int oi = __shfl_xor(bi, off, 64);
                        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
                    }
                    if (pv[m]) {
                        const int oy = 2 * py[m] + (n >> 1), ox = 2 * px[m] + (n & 1);
                        const size_t opix = (size_t)(pn[m] * a.Hout + oy) * a.Wout + ox;
                        if (a.cls_out && kq == 0) {
                            const int k = bi < 16 ? bi : 0;
                            a.cls_out[opix] = a.lut ? a.lut[k] : (uint8_t)k;
                        }
                        if (a.logits_out) {
                            const size_t plane = (size_t)a.Hout * a.Wout;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int cls = kq * 4 + r;
                                if (cls < a.ncls)
                                    a.logits_out[((size_t)pn[m] * a.ncls + cls) * plane + (size_t)oy * a.Wout + ox] = get(v, r);
                            }
                        }
                    }
                }
            }
        } else {
            // Output staging: each wave owns an LDS region; a 16-pixel fragment's results are written
            // there and leave as contiguous 16-B-per-lane stores (a per-lane NHWC store writes 16
            // partial lines per instruction). EPI_SHUFFLE stages the fragment's two output rows of 32
            // pixels. The RESADD residual comes in the same coalesced way.
            constexpr int EPC = 16 / (int)sizeof(T);
            const bool staged = EPI != EPI_SHUFFLE || a.stage_ok;
            T *stg = stage_base + wave * a.stg_elems;
            const int OSTR = a.outC + EPC;
            const T *res = reinterpret_cast<const T *>(a.res);
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                const int p0 = tile * TILE + wave * MR * 16 + m * 16;     // first GEMM pixel of the fragment
                const size_t gpix = (size_t)(pn[m] * a.Hg + py[m]) * a.Wg + px[m];
                bool res_staged = false;
                if constexpr (EPI == EPI_RESADD) {
                    if (a.resCS == a.outC) {
                        for (int q = lane; q < 16 * a.outC / EPC; q += 64) {
                            const int pp = p0 + q * EPC / a.outC;
                            uint4 v4 = make_uint4(0, 0, 0, 0);
                            if (pp < a.M) v4 = *reinterpret_cast<const uint4 *>(res + (size_t)p0 * a.outC + q * EPC);
                            *reinterpret_cast<uint4 *>(stg + (q * EPC / a.outC) * OSTR + (q * EPC) % a.outC) = v4;
                        }
                        wave_lds_sync();
                        res_staged = true;
                    }
                }
#pragma unroll
                for (int n = 0; n < NR; ++n) {
                    const int c = n * 16 + kq * 4;
                    float4 v = add4(f4(acc[m][n]), ld4f(cbias + c));
                    if constexpr (EPI == EPI_SHUFFLE) {
                        const int ph = c / a.coutP, cl = c - ph * a.coutP;
                        if (cl >= a.outC) continue;
                        v = prelu4(v, ld4f(cs1 + c));
                        if (staged) {
                            st4(stg + ((ph >> 1) * 32 + 2 * col + (ph & 1)) * OSTR + cl, v);
                        } else if (pv[m]) {
                            const int oy = 2 * py[m] + (ph >> 1), ox = 2 * px[m] + (ph & 1);
                            st4(out + ((size_t)(pn[m] * a.Hout + oy) * a.Wout + ox) * a.outC + cl, v);
                        }
                        continue;
                    }
                    if (c >= a.outC || !pv[m]) continue;
                    if constexpr (EPI == EPI_INIT_BGR) {
                        // pool channels: max over the window of the raw bytes (the table is increasing, so
                        // max(table(v)) == table(max(v))), reduced across the 4 lane groups above
                        const float4 ps = ld4f(cps + c);
                        float pv4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int ch = c + r - a.cconv;
                            if (ch < 0 || ch >= a.cpool) continue;
                            const int mx = pmx[m][ch];
                            pv4[r] = (mx >= 0 ? nl[ch * 256 + mx] : -INFINITY) * get(ps, r);
                        }
                        v = add4(v, make_float4(pv4[0], pv4[1], pv4[2], pv4[3]));
                        v = prelu4(v, ld4f(cs1 + c));
                    } else if constexpr (EPI == EPI_INIT) {
                        // concat(conv, maxpool(in)) -> BN -> act (InitialBlock); pool channels carry
                        // their BN as pscale (x) + bias.
                        const float4 ps = ld4f(cps + c);
                        float pv4[4] = {0.f, 0.f, 0.f, 0.f};
                        const int k = a.pool_k, pad = (k - 1) >> 1;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int ch = c + r - a.cconv;
                            if (ch < 0 || ch >= a.cpool) continue;
                            float mx = -INFINITY;
                            for (int wy = 0; wy < k; ++wy) {
                                const int iy = 2 * py[m] - pad + wy;
                                if ((unsigned)iy >= (unsigned)a.Hin) continue;
                                for (int wx = 0; wx < k; ++wx) {
                                    const int ix = 2 * px[m] - pad + wx;
                                    if ((unsigned)ix >= (unsigned)a.Win) continue;
                                    const float x = ld1(in + ((size_t)(pn[m] * a.Hin + iy) * a.Win + ix) * a.CinS + ch);
                                    mx = x > mx ? x : mx;
                                }
                            }
                            pv4[r] = mx * get(ps, r);
                        }
                        v = add4(v, make_float4(pv4[0], pv4[1], pv4[2], pv4[3]));
                        v = prelu4(v, ld4f(cs1 + c));
                    } else {
                        v = prelu4(v, ld4f(cs1 + c));
                    }
                    if constexpr (EPI == EPI_RESADD) {
                        if (res_staged) v = add4(v, ld4(stg + col * OSTR + c));
                        else if (c < a.resC) v = add4(v, ld4(res + gpix * a.resCS + c));
                        v = prelu4(v, ld4f(cs2 + c));
                    } else if constexpr (EPI == EPI_RESPOOL) {
                        // main branch: MaxPool2d(2, 2, return_indices) of the block input, zero-padded
                        // to cout channels; first maximum in window order wins (strict >).
                        if (c < a.resC) {
                            const T *rs = reinterpret_cast<const T *>(a.res);
                            float4 best = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
                            int bi[4] = {0, 0, 0, 0};
#pragma unroll
                            for (int pos = 0; pos < 4; ++pos) {
                                const int ry = 2 * py[m] + (pos >> 1), rx = 2 * px[m] + (pos & 1);
                                const float4 x = ld4(rs + ((size_t)(pn[m] * a.resH + ry) * a.resW + rx) * a.resCS + c);
                                if (x.x > best.x) { best.x = x.x; bi[0] = pos; }
                                if (x.y > best.y) { best.y = x.y; bi[1] = pos; }
                                if (x.z > best.z) { best.z = x.z; bi[2] = pos; }
                                if (x.w > best.w) { best.w = x.w; bi[3] = pos; }
                            }
                            v = add4(v, best);
                            *reinterpret_cast<uint32_t *>(a.idx_out + gpix * a.idxCS + c) =
                                (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
                        }
                        v = prelu4(v, ld4f(cs2 + c));
                    } else if constexpr (EPI == EPI_RESUNPOOL) {
                        // MaxUnpool2d(2): the low-res main value lands on the window position its
                        // pooling index recorded; every other position of the window is 0.
                        if (c < a.resC) {
                            const int ly = py[m] >> 1, lx = px[m] >> 1;
                            const size_t lpix = (size_t)(pn[m] * a.resH + ly) * a.resW + lx;
                            const uint32_t id = *reinterpret_cast<const uint32_t *>(a.idx_in + lpix * a.idxCS + c);
                            const uint32_t pos = (uint32_t)(((py[m] & 1) << 1) | (px[m] & 1));
                            const float4 mv = ld4(reinterpret_cast<const T *>(a.res) + lpix * a.resCS + c);
                            v.x += ((id & 0xff) == pos) ? mv.x : 0.f;
                            v.y += (((id >> 8) & 0xff) == pos) ? mv.y : 0.f;
                            v.z += (((id >> 16) & 0xff) == pos) ? mv.z : 0.f;
                            v.w += (((id >> 24) & 0xff) == pos) ? mv.w : 0.f;
                        }
                        v = prelu4(v, ld4f(cs2 + c));
                    }
                    st4(stg + col * OSTR + c, v);
                }
                if (!staged) continue;
                wave_lds_sync();
                if constexpr (EPI == EPI_SHUFFLE) {
                    // two output rows 2y, 2y+1, each 32 pixels from x = 2*px of the fragment's first lane
                    const int nq = 32 * a.outC / EPC;
                    const int n0 = __shfl(pn[m], 0, 64), y0 = __shfl(py[m], 0, 64), x0 = __shfl(px[m], 0, 64);
                    for (int q = lane; q < 2 * nq; q += 64) {
                        const int row = q >= nq, qq = q - row * nq;
                        if (p0 < a.M)
                            *reinterpret_cast<uint4 *>(out + ((size_t)(n0 * a.Hout + 2 * y0 + row) * a.Wout + 2 * x0) * a.outC + qq * EPC) =
                                *reinterpret_cast<const uint4 *>(stg + (row * 32 + qq * EPC / a.outC) * OSTR + (qq * EPC) % a.outC);
                    }
                } else {
                    for (int q = lane; q < 16 * a.outC / EPC; q += 64) {
                        if (p0 + q * EPC / a.outC < a.M)
                            *reinterpret_cast<uint4 *>(out + (size_t)p0 * a.outC + q * EPC) =
                                *reinterpret_cast<const uint4 *>(stg + (q * EPC / a.outC) * OSTR + (q * EPC) % a.outC);
                    }
                }
                wave_lds_sync();
            }
        }
    }
}

int conv_tile_pixels(int nr) { return 4 * (nr >= 4 ? 2 : 4) * 16; }

size_t conv_lds_bytes(int prec, const ConvArgs &a) {
    const int es = prec == PREC_BF16 ? 2 : 4;
    return conv_stage_offset(es, a) + (size_t)4 * a.stg_elems * es;
}

template <typename T, int NR>
static hipError_t launch_nr(int epi, const ConvArgs &a, dim3 grid, size_t lds, hipStream_t s) {
    switch (epi) {
    case EPI_PLAIN: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_PLAIN>), grid, dim3(256), lds, s, a); break;
    case EPI_RESADD: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_RESADD>), grid, dim3(256), lds, s, a); break;
    case EPI_RESPOOL: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_RESPOOL>), grid, dim3(256), lds, s, a); break;
    case EPI_RESUNPOOL: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_RESUNPOOL>), grid, dim3(256), lds, s, a); break;
    case EPI_INIT: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_INIT>), grid, dim3(256), lds, s, a); break;
    case EPI_SHUFFLE: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_SHUFFLE>), grid, dim3(256), lds, s, a); break;
    case EPI_CLASSES: hipLaunchKernelGGL((conv_kernel<T, NR, EPI_CLASSES>), grid, dim3(256), lds, s, a); break;
    case EPI_INIT_BGR:
        if constexpr (NR == 1) { hipLaunchKernelGGL((conv_kernel<T, NR, EPI_INIT_BGR>), grid, dim3(256), lds, s, a); break; }
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
    // one workgroup per tile up to 2048 workgroups (8 per CU), rounded to a multiple of 8 for the
    // XCD-aware walk; larger grids stride.
    int g = a.ntiles < 2048 ? a.ntiles : 2048;
    g = (g + 7) & ~7;
    const size_t lds = conv_lds_bytes(prec, a);
    if (prec == PREC_BF16) return launch_t<__bf16>(nr, epi, a, dim3(g), lds, s);
    return launch_t<float>(nr, epi, a, dim3(g), lds, s);
}

}  // namespace bugseg
