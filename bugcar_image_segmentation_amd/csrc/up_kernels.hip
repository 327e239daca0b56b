// Fused ENet upsampling bottleneck in ONE launch, entirely in registers.
//
//   main = BN(W_m . x)                       1x1 Cin -> Cout         (no activation)
//   e1   = act(W_e1 . x + b)                  1x1 Cin -> I            (I = Cin / 4)
//   t    = act(tconv2x2_s2(e1))               I -> I, 4 output phases (a, b)
//   out  = act_out(act(W_e2 . t + b) + unpool(main, idx))
//
// A 2x2 stride-2 transposed convolution maps each input pixel to exactly one 2x2 output block, and
// every other op here is per pixel, so the block is pointwise in the INPUT grid: a wave takes 16
// input pixels and produces their 64 output pixels with no halo and no LDS traffic beyond the
// weights. Unfused it is 3-4 launches that write and re-read the main tensor, e1 and the 4x larger
// t (up5 at 640x480: 12.5 MB/frame); fused it reads x and the pooling indices once and writes out
// once (5.2 MB/frame).
//
// MFMA mapping as conv_kernels.hip (A = weights, rows = output channels; B = 8 channels of one pixel
// per lane; accumulator quad = 4 channels of one pixel). An intermediate goes from accumulator
// quads to the next GEMM's B operand with two lane permutations: v_permlane32_swap then
// v_permlane16_swap turn the quads of two 16-channel row fragments into each lane's 8 consecutive
// channels (see to_bop). Every intermediate is rounded to the storage type exactly where the unfused
// launches store it, and each GEMM adds its bias where the unfused launch with that row count does
// (bias_in_acc), so the fused block is bit-identical to the unfused plan.
#include "bugseg_internal.h"
#include "mfma_common.h"

namespace bugseg {


// threads per workgroup: the 2-byte CIN = 128 form (46 KB of weights in LDS: 3 workgroups per CU) runs
// 8 waves per workgroup (UP_NT128), so the weights staged once per CU serve twice the waves
#ifndef UP_NT128
#define UP_NT128 512
#endif
template <typename T, int CIN>
__host__ __device__ constexpr int up_threads() { return sizeof(T) == 2 && CIN >= 128 ? UP_NT128 : 256; }

template <typename T, int CIN, int I, int COUT>
__global__ void __launch_bounds__((up_threads<T, CIN>()), (sizeof(T) == 2 ? (CIN >= 128 ? (UP_NT128 == 512 ? 4 : 2) : 3) : 1)) up_kernel(const UpArgs a) {
    span_enter(a.span);
    using Raw = typename Tr<T>::Raw;
    using WRaw = typename WTr<T>::Raw;   // weight operand (fp32 mode: split-f16 parts)
    constexpr int ES = (int)sizeof(T);
// fp32, the 128 -> 64 block: non-temporal output stores (round 5, B = 64, one stream: the bottleneck that
// reads them 13 us faster, this launch 7 us slower; the 64 -> 16 block lost 26 us for 7, so it keeps
// the default) — A/B knob UP_NT_F32 (0 off, 1 that block, 2 both)
#ifndef UP_NT_F32
#define UP_NT_F32 1
#endif
#ifndef UP_AUX_F32_LOW
#define UP_AUX_F32_LOW 0       // fp32 64 -> 16 block's policy (A/B knob)
#endif
#ifndef UP_NT_2B
#define UP_NT_2B 0
#endif
    constexpr int OAUX = (sizeof(T) == 4 && (UP_NT_F32 == 2 || (UP_NT_F32 == 1 && CIN >= 128))) || (sizeof(T) == 2 && UP_NT_2B && CIN >= 128) ? 2
                       : sizeof(T) == 4 && CIN < 128 ? UP_AUX_F32_LOW
                       : OUT_AUX_SEL(CIN >= 128 ? 16 : 0);   // sc1 output stores (mfma_common.h)
    constexpr int NR1 = (COUT + I) / 16;              // GEMM 1 rows: main then e1
    constexpr int NM = COUT / 16, NE = I / 16;        // row fragments of main / e1 (per tconv phase)
    constexpr int KS1 = CIN / 32;                     // GEMM 1 k-steps
    constexpr int NR2 = 4 * I / 16;                   // tconv rows (4 phases)
    constexpr int NR3 = COUT / 16;                    // expansion rows
    static_assert(COUT % 16 == 0 && I % 16 == 0 && CIN % 32 == 0 && I <= 32, "up_kernel shape");
    constexpr bool SWAP = ES == 2 && NR3 % 2 == 0;    // 16-B output chunks by lane-pair swaps (bneck phase 3)
// fp32, COUT = 64 (a pixel = two 128-B lines): LINES stores whole lines. An accumulator quad is 16 B
// (channels 16 r + 4 kq .. + 3 of pixel col), so a store per row block r writes 16 pixels x 64 B —
// half lines, and under the non-temporal policy each half went to HBM on its own (PMC, round 5: 422 MB
// written per 64-frame launch against 315 MB of output). With LINES the quads of row blocks 2 t and
// 2 t + 1 of pixels col and col ^ 8 are traded across lanes 8 apart (one DPP row rotation per dword),
// so each of the two stores per t writes the whole line t of 8 pixels (lanes col and col ^ 8: the
// line's two 64-B halves). Same values, other lanes: bit-identical output
#ifndef UP_F32_LINES
#define UP_F32_LINES 1
#endif
#ifndef UP_F32_LINES16
#define UP_F32_LINES16 0    // the C16 block's phase-pair form: measured slower (round 6, A/B: up C16 122 -> 134 us per 64-frame launch)
#endif
    constexpr bool LINES = ES == 4 && NR3 % 2 == 0 && UP_F32_LINES;
    // COUT = 16 (a pixel = 64 B): the two column phases of an output row are adjacent pixels, one line —
    // the even phase's quad waits in registers and is traded and stored with the odd one's
    constexpr bool LINES16 = ES == 4 && NR3 == 1 && UP_F32_LINES16;
    // bias placement of the unfused launches (bias_in_acc of their row counts): the main and e1
    // 1x1s both accumulate from the bias (the host plans this kernel only then), the tconv and the
    // expansion as their own row counts say
    static_assert(NM <= 4 && NE <= 4, "main / e1 launches must carry their bias in the accumulator");
    constexpr bool B1ACC = true;
    constexpr bool B2ACC = bias_in_acc(NR2, 1), B3ACC = bias_in_acc(NR3, 1);   // one k step each (K = I <= 32)
    // LDS: weights of the three GEMMs (+16 B row pad) and their per-row constants
    // row pads: bf16 16 elements (row strides 8 / 24 / 40 dwords mod 64: conflict-free ds_read_b128
    // groups, bneck_kernels.hip bneck_padw), fp32 16 B
    // (unpadded rows with XOR-swizzled chunks for CIN = 128 measured no faster in the 2-stream bench,
    // round 3, and were removed)
    constexpr int UPAD = ES == 2 ? 16 : 16 / ES;
    constexpr int K1S = CIN + UPAD, K2S = 32 + UPAD, K3S = 32 + UPAD;
    // element offset of the 8-element chunk c of a weight row (a lane's fragment read)
    auto wch = [](int, int c, int) -> int { return c * 8; };
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *w1s = reinterpret_cast<T *>(smem);
    T *w2s = w1s + NR1 * 16 * K1S;
    T *w3s = w2s + NR2 * 16 * K2S;
    float *cb1 = reinterpret_cast<float *>(w3s + NR3 * 16 * K3S), *cs1 = cb1 + NR1 * 16;
    float *cb2 = cs1 + NR1 * 16, *cs2 = cb2 + NR2 * 16;
    float *cb3 = cs2 + NR2 * 16, *cs3 = cb3 + NR3 * 16, *cso = cs3 + NR3 * 16;
    constexpr int NT = up_threads<T, CIN>();
    const int tid = threadIdx.x;
    {
        auto stage = [&](T *dst, const void *src, int rows, int kpad, int kstride) {
            const int cpr = kpad * ES / 16;
            const uint4 *s = reinterpret_cast<const uint4 *>(src);
            for (int i = tid; i < rows * cpr; i += NT) {
                const int r = i / cpr, c = i - r * cpr;
                // (c counts 16-B chunks: 8 elements in 2-byte storage, 4 in fp32, where nothing is swizzled)
                *reinterpret_cast<uint4 *>(dst + (size_t)r * kstride + c * (16 / ES)) = s[i];
            }
        };
        stage(w1s, a.w1, NR1 * 16, CIN, K1S);          // pair pack: K = CIN exactly (1x1, CinS = CIN)
        stage(w2s, a.w2, NR2 * 16, 32, K2S);
        stage(w3s, a.w3, NR3 * 16, 32, K3S);
        for (int i = tid; i < NR1 * 16; i += NT) { cb1[i] = a.b1[i]; cs1[i] = a.s1[i]; }
        for (int i = tid; i < NR2 * 16; i += NT) { cb2[i] = a.b2[i]; cs2[i] = a.s2[i]; }
        for (int i = tid; i < NR3 * 16; i += NT) { cb3[i] = a.b3[i]; cs3[i] = a.s3[i]; cso[i] = a.s_out[i]; }
    }
    __syncthreads();
    const int lane = tid & 63, col = lane & 15, kq = lane >> 4;
    const bool fast = a.slopes_le1;
    auto act = [&](float4 v, const float *s) { return fast ? prelu4m(v, ld4f(s)) : prelu4(v, ld4f(s)); };
    const auto rx = mkbuf(a.x, a.x_bytes);
    const auto ri = mkbuf(a.idx, a.idx_bytes);
    const auto ro = mkbuf(a.out, a.out_bytes);
    const int hw = a.h * a.w;
    const int nfrag = (a.M + 15) >> 4;
    const int gw = blockIdx.x * (NT / 64) + __builtin_amdgcn_readfirstlane(tid >> 6), nw = gridDim.x * (NT / 64);
    // fp32 mode range scaling (bugseg_internal.h RangeArgs): x measured by its producer, e1's output and
    // the tconv's from rigorous bounds; scl false (no multiply anywhere) when every exponent is 0
    constexpr bool F32 = ES == 4;
    bool scl = false;
    float xm = 1.f, b1m = 1.f, m1m = 1.f, o1m = 1.f, b2m = 1.f, o2m = 1.f, b3m = 1.f, o3m = 1.f;
    float amo = 0.f;
    if constexpr (F32) {
      const RangeArgs &g = a.rg;
      if (!g.off) {
        const float amx = rng_read(g);
        const int sx = rng_exp_meas(amx), e1 = sx + g.sw[0];
        const float Br = g.n[0] * amx + g.c[0];
        const int sr = rng_exp_bound(Br, e1), e2 = sr + g.sw[1];
        const int st = rng_exp_bound(g.n[1] * Br + g.c[1], e2), e3 = st + g.sw[2];
        scl = e3 != 0;                                // (only the expansion branches; the rest always multiplies)
        xm = rng_pow2(sx); b1m = rng_pow2(e1); m1m = rng_pow2(-e1); o1m = rng_pow2(sr - e1);
        b2m = rng_pow2(e2); o2m = rng_pow2(st - e2); b3m = rng_pow2(e3); o3m = rng_pow2(-e3);
      }
    }
    // (fp32: the accumulators start at the bias times their scale; always multiplied — a branch to scaled
    // copies of the GEMMs cost 46 VGPRs here — the multipliers are 1 when nothing needs scaling)
    auto bias_m = [&](const float *p, float m) -> f32x4 {
        f32x4 b = bias4(p);
        if constexpr (F32) b = mul4(b, m);
        return b;
    };

    // The grid is sized to the resident waves (launch_up) and each wave streams over fragments: the
    // next fragment's block input and pooling indices are in flight while this one computes.
    Raw xn[KS1];
    uint32_t idn[NM];
    auto load = [&](int f) {
        const int p = f * 16 + col;
        const bool pv = p < a.M;
#pragma unroll
        for (int s = 0; s < KS1; ++s) bld8(xn[s], rx, pv ? (uint32_t)(p * CIN + s * 32 + kq * 8) * ES : OOB);
        // pooling indices of this pixel's main channels (one byte per channel: window position)
#pragma unroll
        for (int r = 0; r < NM; ++r)
            idn[r] = __builtin_amdgcn_raw_buffer_load_b32(ri, pv ? (int)(p * a.idxCS + r * 16 + kq * 4) : (int)OOB, 0, 0);
    };
    if (gw < nfrag) load(gw);
    for (int f = gw; f < nfrag; f += nw) {
        // an opaque per-fragment offset keeps the weight fragments' LDS reads inside the loop for the
        // CIN = 128 form (hoisted, all 24 of GEMM 1's A fragments sat in registers: 226 VGPRs, 2 waves
        // per SIMD; in the loop 96 VGPRs, 3 per SIMD by LDS): up C64 37.8 -> 36.5 us per 32-frame
        // launch (round 3, fp16); the CIN = 64 form measured 35.1 -> 36.1 with it, so it keeps them hoisted
        int wofs = 0;
        if constexpr (CIN >= 128) asm volatile("" : "+v"(wofs));
        const T *w1 = w1s + wofs, *w2 = w2s + wofs, *w3 = w3s + wofs;
        const int p = f * 16 + col;
        const bool pv = p < a.M;
        const uint32_t pp = pv ? (uint32_t)p : 0u;
        const int n = (int)fdiv(pp, a.mHW, a.sHW), rr = (int)pp - n * hw;
        const int y = (int)fdiv((uint32_t)rr, a.mW, a.sW), x = rr - y * a.w;

        // ---- GEMM 1: [main; e1] = W1 . x  (the block input read once, 16 B per lane per k-step)
        Raw xf[KS1];
        uint32_t id[NM];
#pragma unroll
        for (int s = 0; s < KS1; ++s) xf[s] = xn[s];
#pragma unroll
        for (int r = 0; r < NM; ++r) id[r] = idn[r];
        if (f + nw < nfrag) load(f + nw);
        f32x4 acc1[NR1];
        static_assert(B1ACC, "GEMM 1 starts from the bias");
#pragma unroll
        for (int r = 0; r < NR1; ++r) acc1[r] = bias_m(cb1 + r * 16 + kq * 4, b1m);
#pragma unroll
        for (int s = 0; s < KS1; ++s) {
            Raw xq = xf[s];
            if constexpr (F32) xq = scale8(xf[s], xm);
#pragma unroll
            for (int r = 0; r < NR1; ++r) {
                WRaw wf;
                ld8(wf, w1 + (r * 16 + col) * K1S + wch(col, s * 4 + kq, CIN));
                mma(acc1[r], wf, xq);
            }
        }
        if constexpr (F32) {
            // main rows back to true units, e1 rows to their tconv operand's scale
#pragma unroll
            for (int r = 0; r < NR1; ++r) acc1[r] = mul4(acc1[r], r < NM ? m1m : o1m);
        }
        auto ep1 = [&](int r) {
            const int c = r * 16 + kq * 4;
            return round_t(act(f4(acc1[r]), cs1 + c), (const T *)nullptr);
        };
        float4 mv[NM];
#pragma unroll
        for (int r = 0; r < NM; ++r) mv[r] = ep1(r);
        Raw bop2;
        to_bop(bop2, ep1(NM), NE > 1 ? ep1(NM + 1) : make_float4(0.f, 0.f, 0.f, 0.f));

        // ---- per output phase (a, b): t = act(tconv) -> expansion -> + unpooled main -> act -> store
        const uint32_t obase = pv ? (uint32_t)((n * 2 * a.h + 2 * y) * (2 * a.w) + 2 * x) : 0u;   // output pixel (2y, 2x)
        // LINES: lanes col < 8 store pixels col (first store) and col + 8 (second), lanes col >= 8 pixels
        // col - 8 and col: the output base of the fragment's other pixel f * 16 + (col ^ 8)
        uint32_t obase_o = 0u;
        bool pv_o = false;
        if constexpr (LINES || LINES16) {
            const int po = f * 16 + (col ^ 8);
            pv_o = po < a.M;
            const uint32_t ppo = pv_o ? (uint32_t)po : 0u;
            const int no = (int)fdiv(ppo, a.mHW, a.sHW), rro = (int)ppo - no * hw;
            const int yo = (int)fdiv((uint32_t)rro, a.mW, a.sW), xo = rro - yo * a.w;
            obase_o = pv_o ? (uint32_t)((no * 2 * a.h + 2 * yo) * (2 * a.w) + 2 * xo) : 0u;
        }
        float4 ev_prev = make_float4(0.f, 0.f, 0.f, 0.f);   // LINES16: the even phase's quad
        // (not unrolled: one phase's weight fragments live at a time)
#pragma unroll 1
        for (int ph = 0; ph < 4; ++ph) {
            f32x4 acc2[NE];
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int r2 = ph * NE + e;
                static_assert(B2ACC, "the tconv starts from the bias");
                acc2[e] = bias_m(cb2 + r2 * 16 + kq * 4, b2m);
                WRaw wf;
                ld8(wf, w2 + (r2 * 16 + col) * K2S + wch(col, kq, 32));
                mma(acc2[e], wf, bop2);
                if constexpr (F32) acc2[e] = mul4(acc2[e], o2m);
            }
            auto ep2 = [&](int e) {
                const int c = (ph * NE + e) * 16 + kq * 4;
                return round_t(act(f4(acc2[e]), cs2 + c), (const T *)nullptr);
            };
            Raw bop3;
            to_bop(bop3, ep2(0), NE > 1 ? ep2(1) : make_float4(0.f, 0.f, 0.f, 0.f));
            const uint32_t pho = (uint32_t)((ph >> 1) * 2 * a.w + (ph & 1));
            const uint32_t opix = obase + pho;
            auto ep3 = [&](int r) {
                const int c = r * 16 + kq * 4;
                static_assert(B3ACC, "the expansion starts from the bias");
                f32x4 acc = bias_m(cb3 + c, b3m);
                WRaw wf;
                ld8(wf, w3 + (r * 16 + col) * K3S + wch(col, kq, 32));
                mma(acc, wf, bop3);
                float4 v = f4(acc);
                if constexpr (F32) {
                    if (scl) v = mul4(v, o3m);
                }
                v = act(v, cs3 + c);
                // MaxUnpool2d(2): the main value lands where its pooling index points
                const uint32_t w = id[r];
                const uint32_t pos = (uint32_t)ph;
                v.x += ((w & 0xff) == pos) ? mv[r].x : 0.f;
                v.y += (((w >> 8) & 0xff) == pos) ? mv[r].y : 0.f;
                v.z += (((w >> 16) & 0xff) == pos) ? mv[r].z : 0.f;
                v.w += (((w >> 24) & 0xff) == pos) ? mv[r].w : 0.f;
                return act(v, cso + c);
            };
            if constexpr (SWAP) {
#pragma unroll
                for (int t = 0; t < NR3 / 2; ++t) {
                    const u32x2_t p0 = pack4<T>(ep3(2 * t)), p1 = pack4<T>(ep3(2 * t + 1));
                    uint32_t x0 = p0.x, x1 = p0.y, y0 = p1.x, y1 = p1.y;
                    pl16swap(x0, y0);
                    pl16swap(x1, y1);
                    const int ch = (2 * t + (kq & 1)) * 16 + 8 * (kq >> 1);
                    bst16o<OAUX>(ro, pv ? (opix * COUT + ch) * ES : OOB, make_uint4(x0, x1, y0, y1));
                }
            } else if constexpr (LINES16) {
                const float4 v = ep3(0);
                rng_acc4(amo, v);
                if ((ph & 1) == 0) {
                    ev_prev = v;
                } else {
                    // line of input pixel p: output pixels (2y + ph / 2, 2x) and (.., 2x + 1), 32 channels
                    const bool lo8 = col < 8;
                    const uint32_t phe = pho - 1u;             // the even pixel of this row
                    const uint32_t pa = (lo8 ? obase : obase_o) + phe, pb = (lo8 ? obase_o : obase) + phe;
                    const bool va = lo8 ? pv : pv_o, vb = lo8 ? pv_o : pv;
                    const uint4 u0 = __builtin_bit_cast(uint4, ev_prev), u1 = __builtin_bit_cast(uint4, v);
                    const uint4 xs = lo8 ? u1 : u0;
                    uint4 ys;
                    ys.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.x, 0x128, 0xf, 0xf, false);
                    ys.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.y, 0x128, 0xf, 0xf, false);
                    ys.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.z, 0x128, 0xf, 0xf, false);
                    ys.w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.w, 0x128, 0xf, 0xf, false);
                    const int ch = (lo8 ? 0 : 16) + kq * 4;   // channel 16 + c of the even pixel = c of the odd one
                    bst16o<OAUX>(ro, va ? (pa * COUT + ch) * ES : OOB, lo8 ? u0 : ys);
                    bst16o<OAUX>(ro, vb ? (pb * COUT + ch) * ES : OOB, lo8 ? ys : u1);
                }
            } else if constexpr (LINES) {
                const bool lo8 = col < 8;
                // first store: pixel col & 7 (lanes col < 8 their own, col >= 8 the other's); second: + 8
                const uint32_t pa = lo8 ? obase + pho : obase_o + pho, pb = lo8 ? obase_o + pho : obase + pho;
                const bool va = lo8 ? pv : pv_o, vb = lo8 ? pv_o : pv;
                const int hc = lo8 ? 0 : 16;                  // channel half of the line this lane writes
#pragma unroll
                for (int t = 0; t < NR3 / 2; ++t) {
                    const float4 v0 = ep3(2 * t), v1 = ep3(2 * t + 1);
                    rng_acc4(amo, v0);
                    rng_acc4(amo, v1);
                    const uint4 u0 = __builtin_bit_cast(uint4, v0), u1 = __builtin_bit_cast(uint4, v1);
                    // lanes col < 8 send their block 2t + 1 quad, lanes col >= 8 their block 2t quad, to the
                    // lane 8 apart in the 16-lane row (row_ror:8 is its own inverse)
                    const uint4 xs = lo8 ? u1 : u0;
                    uint4 ys;
                    ys.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.x, 0x128, 0xf, 0xf, false);
                    ys.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.y, 0x128, 0xf, 0xf, false);
                    ys.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.z, 0x128, 0xf, 0xf, false);
                    ys.w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.w, 0x128, 0xf, 0xf, false);
                    const uint4 qa = lo8 ? u0 : ys, qb = lo8 ? ys : u1;
                    const int ch = t * 32 + hc + kq * 4;
                    bst16o<OAUX>(ro, va ? (pa * COUT + ch) * ES : OOB, qa);
                    bst16o<OAUX>(ro, vb ? (pb * COUT + ch) * ES : OOB, qb);
                }
            } else {
#pragma unroll
                for (int r = 0; r < NR3; ++r) {
                    const float4 v = ep3(r);
                    if constexpr (F32) rng_acc4(amo, v);
                    const uint32_t off = pv ? (opix * COUT + r * 16 + kq * 4) * ES : OOB;
                    if constexpr (ES == 2) bst8o<OAUX>(ro, off, pack4<T>(v));
                    else bst16o<OAUX>(ro, off, __builtin_bit_cast(uint4, v));
                }
            }
        }
    }
    if constexpr (F32) rng_commit(amo, a.rg.amax_out);
    span_exit(a.span);
}

template <typename T, int CIN, int I, int COUT>
static size_t up_lds() {
    constexpr int ES = (int)sizeof(T);
    constexpr int NR1 = (COUT + I) / 16, NR2 = 4 * I / 16, NR3 = COUT / 16;
    constexpr int UPAD = ES == 2 ? 16 : 16 / ES;      // = up_kernel's
    return (size_t)(NR1 * 16 * (CIN + UPAD) + NR2 * 16 * (32 + UPAD) + NR3 * 16 * (32 + UPAD)) * ES +
           (size_t)(2 * NR1 * 16 + 2 * NR2 * 16 + 3 * NR3 * 16) * sizeof(float);
}

bool up_supported(int cin, int it, int cout) {
    return (cin == 128 && it == 32 && cout == 64) || (cin == 64 && it == 16 && cout == 16);
}

template <int CI, int II, int CO>
static hipError_t launch_shape(int prec, const UpArgs &a, dim3 g, hipStream_t s) {
    if (prec == PREC_BF16) {
        const size_t lds = up_lds<__bf16, CI, II, CO>();
        hipLaunchKernelGGL((up_kernel<__bf16, CI, II, CO>), g, dim3(up_threads<__bf16, CI>()), lds, s, a);
    } else if (prec == PREC_F16) {
        const size_t lds = up_lds<_Float16, CI, II, CO>();
        hipLaunchKernelGGL((up_kernel<_Float16, CI, II, CO>), g, dim3(up_threads<_Float16, CI>()), lds, s, a);
    } else {
        const size_t lds = up_lds<float, CI, II, CO>();
        if (lds > 64 * 1024) {
            hipError_t e = allow_dynamic_lds((const void *)up_kernel<float, CI, II, CO>);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((up_kernel<float, CI, II, CO>), g, dim3(up_threads<float, CI>()), lds, s, a);
    }
    return hipGetLastError();
}

// workgroups resident at once (occupancy API, per kernel instance), cached
template <typename T, int CI, int II, int CO>
static int up_resident() {
    // (cached per device: bugseg_runtime.cpp occupancy_per_cu; the >64 KB LDS opt-in first, or the
    // occupancy API sees a kernel that cannot launch)
    if (up_lds<T, CI, II, CO>() > 64 * 1024) (void)allow_dynamic_lds((const void *)up_kernel<T, CI, II, CO>);
    const int per = occupancy_per_cu((const void *)up_kernel<T, CI, II, CO>, up_threads<T, CI>(), up_lds<T, CI, II, CO>());
    return device_cus() * (per > 0 ? per : 2);
}

hipError_t launch_up(int prec, int cin, int it, int cout, const UpArgs &a, hipStream_t s) {
    const int nfrag = (a.M + 15) / 16;
    const int wpg = (cin == 128 && prec != PREC_F32 ? UP_NT128 : 256) / 64;   // waves per workgroup (up_threads)
    int g = (nfrag + wpg - 1) / wpg;
    // one resident round of workgroups, each streaming over its fragments (prefetch in the kernel)
    const int res = cin == 128 ? (prec == PREC_BF16  ? up_resident<__bf16, 128, 32, 64>()
                                  : prec == PREC_F16 ? up_resident<_Float16, 128, 32, 64>()
                                                     : up_resident<float, 128, 32, 64>())
                               : (prec == PREC_BF16  ? up_resident<__bf16, 64, 16, 16>()
                                  : prec == PREC_F16 ? up_resident<_Float16, 64, 16, 16>()
                                                     : up_resident<float, 64, 16, 16>());
    if (g > res) g = res;
    if (g < 1) g = 1;
    if (cin == 128 && it == 32 && cout == 64) return launch_shape<128, 32, 64>(prec, a, dim3(g), s);
    if (cin == 64 && it == 16 && cout == 16) return launch_shape<64, 16, 16>(prec, a, dim3(g), s);
    return hipErrorInvalidValue;
}

}  // namespace bugseg
