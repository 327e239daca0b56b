// Fused ENet regular / dilated / asymmetric bottleneck in ONE launch.
//
//   t0  = act1(W1 . x + b1)            1x1 projection C -> I (= C/4)     over the tile + halo
//   t1  = act2(W2 * t0 + b2)           3x3 (dilation d) or 5x1 then 1x5 over the tile
//   out = act_out(act3(W3 . t1 + b3) + x)                                 1x1 expansion + residual
//
// Unfused, each 128-channel bottleneck moves ~1024 B/pixel through HBM (x read twice, three internal
// tensors written and read); here x is read once (halo re-reads are L2 hits) and out written once:
// 512 B/pixel in bf16. The internal tensors never leave LDS:
//   * a 256-thread workgroup owns a TH x TW output tile of one frame; phase 1 computes t0 for the
//     tile plus a halo of (ry, rx) pixels (zero outside the image: t0 is what the 3x3 zero-pads);
//   * phase 2 accumulates its whole tile in registers, then (after a barrier) overwrites the t0
//     region with t1, so one LDS region serves both (asymmetric: t0 -> t1a -> t1, same trick);
//   * phase 3 streams 16-pixel fragments: MFMA with W3, residual from global (just read, L2/L1),
//     activation, 8-byte NHWC stores.
// MFMA operand mapping as conv_kernels.hip: A = weights (row = output channel) from LDS, B = 8
// channels of one pixel (16-B LDS or global read per lane), accumulator = 4 consecutive channels of
// one pixel per lane. All three weight matrices stay in LDS for the workgroup's lifetime.
#include "bugseg_internal.h"
#include "mfma_common.h"

namespace bugseg {

// Tile and workgroup shape per channel count. 128 channels: the LDS footprint (weights + halo or
// output staging, ~64-73 KB) allows two workgroups per CU, so they are 8-wave (512-thread) to put
// 16 waves on a CU; 64 / 16 channels (~28 KB): four 4-wave workgroups per CU — more independent
// tile pipelines (memory phase of one beside compute phase of another) for the same waves.
template <int C> struct BTile;
// OCC: waves per SIMD the bf16 build is held to (registers), matching what LDS allows.
template <> struct BTile<128> { static constexpr int TH = 16, TW = 16, NW = 8, OCC = 4; };
template <> struct BTile<64> { static constexpr int TH = 16, TW = 16, NW = 4, OCC = 5; };
template <> struct BTile<16> { static constexpr int TH = 16, TW = 16, NW = 4, OCC = 6; };

int bneck_tile_h(int C) { return C == 128 ? BTile<128>::TH : C == 64 ? BTile<64>::TH : BTile<16>::TH; }
int bneck_tile_w(int C) { return C == 128 ? BTile<128>::TW : C == 64 ? BTile<64>::TW : BTile<16>::TW; }
static int bneck_waves(int C) { return C == 128 ? BTile<128>::NW : C == 64 ? BTile<64>::NW : BTile<16>::NW; }

template <typename T, int C, bool ASYM>
__global__ void __launch_bounds__(BTile<C>::NW * 64, sizeof(T) == 2 ? BTile<C>::OCC : 1) bneck_kernel(const BneckArgs a) {
    using Raw = typename Tr<T>::Raw;
    constexpr int NW = BTile<C>::NW, NT = NW * 64;
    constexpr int I = C / 4;
    constexpr int IS = I < 8 ? 8 : I;                 // stored internal channels (8-channel groups)
    constexpr int NR1 = (I + 15) / 16;                // 16-row fragments of t0 / t1
    constexpr int NR3 = C / 16;                       // 16-row fragments of out
    constexpr int G1 = C / 8, KS1 = (G1 + 3) / 4;     // proj k groups / steps
    constexpr int TAPS = ASYM ? 5 : 9;
    constexpr int G2 = TAPS * IS / 8, KS2 = (G2 + 3) / 4;
    constexpr int G3 = IS / 8;                        // expand k groups (<= 4: one step)
    constexpr int TH = BTile<C>::TH, TW = BTile<C>::TW;
    constexpr int PAD = 16 / (int)sizeof(T);
    constexpr int PSTR = IS + PAD;                    // LDS pixel stride (elements)
    constexpr int NFT = TH * TW / 16;                 // 16-pixel fragments of the tile
    constexpr int NF2 = (NFT + NW - 1) / NW;          // ... per wave
    constexpr int TWA = TW + 4;                       // asymmetric: width of t1a (the 1x5's halo)
    constexpr int NFA = TH * TWA / 16;
    constexpr int NF2A = (NFA + NW - 1) / NW;
    constexpr int CH1 = KS1 >= 4 ? 3 : KS1 == 2 ? 4 : 8;   // phase-1 fragments whose loads fly together
    constexpr int EPC = 16 / (int)sizeof(T);          // elements per 16-B chunk
    constexpr int CPF = 16 * C / EPC;                 // 16-B chunks of one 16-pixel output fragment
    constexpr int CPL = (CPF + 63) / 64;              // ... per lane
    constexpr int OSTR = C + EPC;                     // phase-3 staging row stride (16-B padded)
    static_assert(NFT % NW == 0, "tile fragments must split evenly over the waves");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63, col = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably uniform: scalar fragment math
    const int K1S = KS1 * 32 + PAD, K2S = KS2 * 32 + PAD, K3S = 32 + PAD;
    T *w1 = reinterpret_cast<T *>(smem);
    T *w2 = w1 + NR1 * 16 * K1S;
    T *w2b = w2 + NR1 * 16 * K2S;                     // asymmetric second conv (1x5)
    T *w3 = w2b + (ASYM ? NR1 * 16 * K2S : 0);
    // per-channel epilogue constants live in LDS too: a global load per use was most of this
    // kernel's vector-memory instructions and a latency the epilogues waited on
    constexpr int NP1 = NR1 * 16;
    float *cb1 = reinterpret_cast<float *>(w3 + C * K3S), *cs1 = cb1 + NP1, *cb2 = cs1 + NP1, *cs2 = cb2 + NP1;
    float *cb2b = cs2 + NP1, *cs2b = cb2b + NP1, *cb3 = cs2b + NP1, *cs3 = cb3 + C, *cso = cs3 + C;
    T *ts = reinterpret_cast<T *>(cso + C);           // t0 / t1a / t1 region
    {
        auto stage = [&](T *dst, const void *src, int rows, int kpad, int kstride) {
            const int cpr = kpad * (int)sizeof(T) / 16;
            const uint4 *s = reinterpret_cast<const uint4 *>(src);
            for (int i = tid; i < rows * cpr; i += NT) {
                const int r = i / cpr, c = i - r * cpr;
                *reinterpret_cast<uint4 *>(reinterpret_cast<unsigned char *>(dst + (size_t)r * kstride) + c * 16) = s[i];
            }
        };
        stage(w1, a.w1, NR1 * 16, KS1 * 32, K1S);
        stage(w2, a.w2, NR1 * 16, KS2 * 32, K2S);
        if constexpr (ASYM) stage(w2b, a.w2b, NR1 * 16, KS2 * 32, K2S);
        stage(w3, a.w3, C, 32, K3S);
        for (int i = tid; i < NP1; i += NT) {
            cb1[i] = a.b1[i]; cs1[i] = a.s1[i]; cb2[i] = a.b2[i]; cs2[i] = a.s2[i];
            cb2b[i] = ASYM ? a.b2b[i] : 0.f; cs2b[i] = ASYM ? a.s2b[i] : 0.f;
        }
        for (int i = tid; i < C; i += NT) { cb3[i] = a.b3[i]; cs3[i] = a.s3[i]; cso[i] = a.s_out[i]; }
    }
    // x / out through buffer descriptors: 32-bit offsets, and an out-of-range offset reads 0 / drops
    // the store (mfma_common.h), so image-border masking costs one select per access
    const auto rxb = mkbuf(a.x, a.x_bytes);
    const auto rob = mkbuf(a.out, a.x_bytes);
    // the fused path is planned only when every slope is <= 1 (bugseg_runtime.cpp fusable_regular),
    // so PReLU is max(v, s*v); accumulators start at the bias
    auto act = [&](float4 v, const float *s) { return prelu4m(v, ld4f(s)); };
    const int ry = a.ry, rx = a.rx, d = a.d;
    const int HWW = TW + 2 * rx, HR = (TH + 2 * ry) * HWW;
    const int nf1 = (HR + 15) >> 4;

    // XCD-aware tile walk (see conv_kernels.hip)
    const int G = gridDim.x, grp = blockIdx.x & 7, slot = blockIdx.x >> 3, nslots = G >> 3;
    const int CH = (a.ntiles + 7) >> 3;
    for (int it = slot; it < CH; it += nslots) {
        const int tile = grp * CH + it;
        if (tile >= a.ntiles) break;
        const int n = tile / (a.tiles_y * a.tiles_x);
        const int tr = tile - n * a.tiles_y * a.tiles_x;
        const int ty0 = (tr / a.tiles_x) * TH, tx0 = (tr % a.tiles_x) * TW;
        const uint32_t xn = (uint32_t)(n * a.H * a.W) * (uint32_t)(C * sizeof(T));   // frame byte offset
        __syncthreads();   // weights staged (first tile) / previous tile done with ts

        // ---- phase 1: t0 = act1(W1 x + b1) over tile + halo, 0 outside the image. The loads of CH1
        // fragments are issued together before any of them is consumed (memory-level parallelism).
        for (int f0 = wave; f0 < nf1; f0 += NW * CH1) {
            Raw xf[CH1][KS1];
            bool okc[CH1];
#pragma unroll
            for (int c = 0; c < CH1; ++c) {
                const int h = (f0 + c * NW) * 16 + col;
                const int hy = (int)fdiv((uint32_t)h, a.mHWW, a.sHWW), hx = h - hy * HWW;
                const int iy = ty0 - ry + hy, ix = tx0 - rx + hx;
                okc[c] = h < HR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
#pragma unroll
                for (int s = 0; s < KS1; ++s) {
                    const int g = s * 4 + kq;
                    const bool ld = okc[c] && g < G1 && !(a.ablate & 1);
                    bld8(xf[c][s], rxb, ld ? xn + (uint32_t)((iy * a.W + ix) * C + g * 8) * (uint32_t)sizeof(T) : OOB);
                }
            }
#pragma unroll
            for (int c = 0; c < CH1; ++c) {
                const int h = (f0 + c * NW) * 16 + col;
                f32x4 acc[NR1];
#pragma unroll
                for (int r = 0; r < NR1; ++r) acc[r] = bias4(cb1 + r * 16 + kq * 4);
#pragma unroll
                for (int s = 0; s < KS1; ++s)
#pragma unroll
                    for (int r = 0; r < NR1; ++r) {
                        Raw wf;
                        ld8(wf, w1 + (r * 16 + col) * K1S + s * 32 + kq * 8);
                        mma(acc[r], wf, xf[c][s]);
                    }
                if (h < HR) {
#pragma unroll
                    for (int r = 0; r < NR1; ++r) {
                        const int ch = r * 16 + kq * 4;
                        if (ch >= IS) continue;
                        float4 v = act(f4(acc[r]), cs1 + ch);
                        if (!okc[c]) v = make_float4(0.f, 0.f, 0.f, 0.f);
                        st4(ts + h * PSTR + ch, v);
                    }
                }
            }
        }
        __syncthreads();

        // residual of phase 3 (x at the tile pixels), prefetched early (asymmetric: after its 5x1 pass,
        // to keep the two passes' live ranges apart) with coalesced 16-B loads: a fragment is 16
        // consecutive pixels of one tile row, i.e. one contiguous run of 16*C elements of x.
        uint4 res[NF2][CPL];
        auto prefetch_res = [&]() {
#pragma unroll
            for (int j = 0; j < NF2; ++j) {
                const int p0 = (wave + NW * j) * 16;
                const int oy = p0 / TW, ox0 = p0 - oy * TW, iy = ty0 + oy;
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    const int q = lane + 64 * k;
                    const int ix = tx0 + ox0 + q * EPC / C;
                    const bool ok = q < CPF && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
                    res[j][k] = bld16(rxb, ok ? xn + (uint32_t)((iy * a.W + tx0 + ox0) * C + q * EPC) * (uint32_t)sizeof(T) : OOB);
                }
            }
        };
        if constexpr (!ASYM) prefetch_res();

        // ---- phase 2: t1 = act2(W2 * t0 + b2) (asymmetric: t1a = 5x1 (t0); t1 = 1x5 (t1a))
        if constexpr (!ASYM) {
            f32x4 acc[NF2][NR1];
#pragma unroll
            for (int j = 0; j < NF2; ++j)
#pragma unroll
                for (int r = 0; r < NR1; ++r) acc[j][r] = bias4(cb2 + r * 16 + kq * 4);
#pragma unroll 1
            for (int s = 0; s < KS2; ++s) {
                const int g = s * 4 + kq;
                const int tap = g / (IS / 8), coff = (g - tap * (IS / 8)) * 8;
                const int dy = (tap / 3 - 1) * d, dx = (tap % 3 - 1) * d;
                Raw wf[NR1];
#pragma unroll
                for (int r = 0; r < NR1; ++r) ld8(wf[r], w2 + (r * 16 + col) * K2S + s * 32 + kq * 8);
#pragma unroll
                for (int j = 0; j < NF2; ++j) {
                    const int p = (wave + NW * j) * 16 + col;
                    const int oy = p / TW, ox = p - oy * TW;
                    Raw xf;
                    if (g < G2) ld8(xf, ts + ((oy + ry + dy) * HWW + (ox + rx + dx)) * PSTR + coff);
                    else zero(xf);
                    if (a.ablate & 2) continue;
#pragma unroll
                    for (int r = 0; r < NR1; ++r) mma(acc[j][r], wf[r], xf);
                }
            }
            __syncthreads();   // every wave is done reading t0
#pragma unroll
            for (int j = 0; j < NF2; ++j) {
                const int p = (wave + NW * j) * 16 + col;
#pragma unroll
                for (int r = 0; r < NR1; ++r) {
                    const int ch = r * 16 + kq * 4;
                    if (ch >= IS) continue;
                    st4(ts + p * PSTR + ch, act(f4(acc[j][r]), cs2 + ch));
                }
            }
        } else {
            {   // 5x1 over rows (taps dy = -2..2), output width TW+4 (the 1x5's halo)
                f32x4 acc[NF2A][NR1];
#pragma unroll
                for (int j = 0; j < NF2A; ++j)
#pragma unroll
                    for (int r = 0; r < NR1; ++r) acc[j][r] = bias4(cb2 + r * 16 + kq * 4);
#pragma unroll 1
                for (int s = 0; s < KS2; ++s) {
                    const int g = s * 4 + kq;
                    const int tap = g / (IS / 8), coff = (g - tap * (IS / 8)) * 8;
                    Raw wf[NR1];
#pragma unroll
                    for (int r = 0; r < NR1; ++r) ld8(wf[r], w2 + (r * 16 + col) * K2S + s * 32 + kq * 8);
#pragma unroll
                    for (int j = 0; j < NF2A; ++j) {
                        const int f = wave + NW * j;
                        const int p = f * 16 + col;
                        const int oy = p / TWA, ox = p - oy * TWA;
                        Raw xf;
                        if (g < G2 && f < NFA) ld8(xf, ts + ((oy + ry + tap - 2) * HWW + ox) * PSTR + coff);
                        else zero(xf);
#pragma unroll
                        for (int r = 0; r < NR1; ++r) mma(acc[j][r], wf[r], xf);
                    }
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < NF2A; ++j) {
                    const int f = wave + NW * j;
                    if (f >= NFA) continue;
                    const int p = f * 16 + col;
                    const int ox = p - (p / TWA) * TWA;
                    const bool inside = (unsigned)(tx0 - 2 + ox) < (unsigned)a.W;   // the 1x5 zero-pads t1a
#pragma unroll
                    for (int r = 0; r < NR1; ++r) {
                        const int ch = r * 16 + kq * 4;
                        if (ch >= IS) continue;
                        float4 v = act(f4(acc[j][r]), cs2 + ch);
                        if (!inside) v = make_float4(0.f, 0.f, 0.f, 0.f);
                        st4(ts + p * PSTR + ch, v);
                    }
                }
                __syncthreads();
            }
            {   // 1x5 over columns (taps dx = -2..2)
                f32x4 acc[NF2][NR1];
#pragma unroll
                for (int j = 0; j < NF2; ++j)
#pragma unroll
                    for (int r = 0; r < NR1; ++r) acc[j][r] = bias4(cb2b + r * 16 + kq * 4);
#pragma unroll 1
                for (int s = 0; s < KS2; ++s) {
                    const int g = s * 4 + kq;
                    const int tap = g / (IS / 8), coff = (g - tap * (IS / 8)) * 8;
                    Raw wf[NR1];
#pragma unroll
                    for (int r = 0; r < NR1; ++r) ld8(wf[r], w2b + (r * 16 + col) * K2S + s * 32 + kq * 8);
#pragma unroll
                    for (int j = 0; j < NF2; ++j) {
                        const int p = (wave + NW * j) * 16 + col;
                        const int oy = p / TW, ox = p - oy * TW;
                        Raw xf;
                        if (g < G2) ld8(xf, ts + (oy * TWA + ox + tap) * PSTR + coff);
                        else zero(xf);
#pragma unroll
                        for (int r = 0; r < NR1; ++r) mma(acc[j][r], wf[r], xf);
                    }
                }
                prefetch_res();
                __syncthreads();
#pragma unroll
                for (int j = 0; j < NF2; ++j) {
                    const int p = (wave + NW * j) * 16 + col;
#pragma unroll
                    for (int r = 0; r < NR1; ++r) {
                        const int ch = r * 16 + kq * 4;
                        if (ch >= IS) continue;
                        st4(ts + p * PSTR + ch, act(f4(acc[j][r]), cs2b + ch));
                    }
                }
            }
        }
        __syncthreads();

        // ---- phase 3: out = act_out(act3(W3 t1 + b3) + x). The t1 fragments go to registers, then
        // the t1 region becomes per-wave staging: residual chunks in, results over them, and the
        // fragment leaves as contiguous 16-B-per-lane stores (a per-lane NHWC store would write
        // 16 partial lines per instruction: the ablation showed stores dominating this kernel).
        Raw tf[NF2];
#pragma unroll
        for (int j = 0; j < NF2; ++j) {
            const int p = (wave + NW * j) * 16 + col;
            if (kq < G3) ld8(tf[j], ts + p * PSTR + kq * 8);
            else zero(tf[j]);
        }
        __syncthreads();
        T *stg = ts + wave * 16 * OSTR;
#pragma unroll
        for (int j = 0; j < NF2; ++j) {
            const int p0 = (wave + NW * j) * 16;
            const int oy = p0 / TW, ox0 = p0 - oy * TW, iy = ty0 + oy;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const int q = lane + 64 * k;
                if (q < CPF) *reinterpret_cast<uint4 *>(stg + (q * EPC / C) * OSTR + (q * EPC) % C) = res[j][k];
            }
            wave_lds_sync();
#pragma unroll
            for (int r = 0; r < NR3; ++r) {
                const int ch = r * 16 + kq * 4;
                f32x4 acc = bias_in_acc(NR3) ? bias4(cb3 + ch) : (f32x4){0.f, 0.f, 0.f, 0.f};
                Raw wf;
                ld8(wf, w3 + (r * 16 + col) * K3S + kq * 8);
                mma(acc, wf, tf[j]);
                T *sp = stg + col * OSTR + ch;
                float4 v = act(bias_in_acc(NR3) ? f4(acc) : add4(f4(acc), ld4f(cb3 + ch)), cs3 + ch);
                v = act(add4(v, ld4(sp)), cso + ch);
                st4(sp, v);
            }
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const int q = lane + 64 * k;
                const int ix = tx0 + ox0 + q * EPC / C;
                const bool ok = q < CPF && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W && !(a.ablate & 4);
                if (q < CPF)
                    bst16(rob, ok ? xn + (uint32_t)((iy * a.W + tx0 + ox0) * C + q * EPC) * (uint32_t)sizeof(T) : OOB,
                          *reinterpret_cast<const uint4 *>(stg + (q * EPC / C) * OSTR + (q * EPC) % C));
            }
            wave_lds_sync();
        }
    }
}

size_t bneck_lds_bytes(int prec, int C, bool asym, int ry, int rx) {
    const int es = prec == PREC_BF16 ? 2 : 4, pad = 16 / es;
    const int I = C / 4, IS = I < 8 ? 8 : I, NR1 = (I + 15) / 16;
    const int KS1 = (C / 8 + 3) / 4, KS2 = ((asym ? 5 : 9) * IS / 8 + 3) / 4;
    const int TH = bneck_tile_h(C), TW = bneck_tile_w(C);
    const size_t wts = (size_t)NR1 * 16 * (KS1 * 32 + pad) + (size_t)NR1 * 16 * (KS2 * 32 + pad) * (asym ? 2 : 1) +
                       (size_t)C * (32 + pad);
    const size_t halo = (size_t)(TH + 2 * ry) * (TW + 2 * rx) * (IS + pad);
    const size_t stage = (size_t)bneck_waves(C) * 16 * (C + pad);      // phase-3 output staging
    const size_t consts = ((size_t)6 * NR1 * 16 + 3 * (size_t)C) * sizeof(float);
    return (wts + (halo > stage ? halo : stage)) * es + consts;
}

template <typename T>
static hipError_t launch_t(int C, bool asym, const BneckArgs &a, dim3 g, size_t lds, hipStream_t s) {
#define BN_CASE(CC)                                                                                     \
    if (C == CC) {                                                                                      \
        if (asym) hipLaunchKernelGGL((bneck_kernel<T, CC, true>), g, dim3(BTile<CC>::NW * 64), lds, s, a);            \
        else hipLaunchKernelGGL((bneck_kernel<T, CC, false>), g, dim3(BTile<CC>::NW * 64), lds, s, a);                \
        return hipGetLastError();                                                                       \
    }
    BN_CASE(128)
    BN_CASE(64)
    BN_CASE(16)
#undef BN_CASE
    return hipErrorInvalidValue;
}

hipError_t launch_bneck(int prec, int C, bool asym, const BneckArgs &a, hipStream_t s) {
    const size_t lds = bneck_lds_bytes(prec, C, asym, a.ry, a.rx);
    static int attr_set[2][2][3] = {};
    int g = a.ntiles < 2048 ? a.ntiles : 2048;
    g = (g + 7) & ~7;
    const int ci = C == 128 ? 0 : C == 64 ? 1 : 2;
    if (lds > 64 * 1024 && !attr_set[prec][asym][ci]) {
        // dynamic LDS above 64 KB must be allowed per kernel
        hipError_t e;
        if (prec == PREC_BF16)
            e = C == 128 ? hipFuncSetAttribute(asym ? (const void *)bneck_kernel<__bf16, 128, true> : (const void *)bneck_kernel<__bf16, 128, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)
              : C == 64 ? hipFuncSetAttribute(asym ? (const void *)bneck_kernel<__bf16, 64, true> : (const void *)bneck_kernel<__bf16, 64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)
                        : hipFuncSetAttribute(asym ? (const void *)bneck_kernel<__bf16, 16, true> : (const void *)bneck_kernel<__bf16, 16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        else
            e = C == 128 ? hipFuncSetAttribute(asym ? (const void *)bneck_kernel<float, 128, true> : (const void *)bneck_kernel<float, 128, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)
              : C == 64 ? hipFuncSetAttribute(asym ? (const void *)bneck_kernel<float, 64, true> : (const void *)bneck_kernel<float, 64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)
                        : hipFuncSetAttribute(asym ? (const void *)bneck_kernel<float, 16, true> : (const void *)bneck_kernel<float, 16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set[prec][asym][ci] = 1;
    }
    if (prec == PREC_BF16) return launch_t<__bf16>(C, asym, a, dim3(g), lds, s);
    return launch_t<float>(C, asym, a, dim3(g), lds, s);
}

}  // namespace bugseg
