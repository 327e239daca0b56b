// fp32 (parity mode) C = 128 regular / dilated bottleneck, two tiles in flight per CU (round 6,
// VERDICT r5 item 4). SURVEY.md §8(a) a2.3: 1x1 projection 128 -> 32, 3x3 (dilated) 32 -> 32, 1x1
// expansion 32 -> 128, BN folded, PReLU after each, residual add, PReLU — the block bneck_kernel
// (bneck_kernels.hip) computes, with the same products in the same order (bit-identical to it and to
// the unfused chain; tests/test_gpu_parity.py).
//
// Why another kernel: the fp32 C128 forms of bneck_kernel hold one 8-wave workgroup per CU (72.7 KB of
// split weights + a 50-63 KB t0 halo in LDS), so a CU runs one tile at a time: the projection's x loads,
// the middle conv, the expansion and the stores follow each other with the memory system idle during
// the compute phases (phase clocks, profiles/r05_f_fp32_stamps.md: a 16x16 tile 34.5k cycles, 26% of
// them barrier waits; SQ wait_any 0.55-0.59).
//
// Here ONE 16-wave workgroup per CU holds one copy of the weights and TWO t0 halo buffers, and its two
// 8-wave halves work on their own tiles, phase-shifted: in every step one half runs phase 1 (x loads +
// projection -> its t0 buffer) while the other runs phases 2 + 3 (middle conv from its t0 buffer,
// expansion, residual, stores) of its previous tile; each step ends at the workgroup barrier, and the
// halves swap roles. One barrier per step protects both buffers: half h writes t0[h] in step k, reads
// it in step k + 1, and writes it again in step k + 2 — every read of step k + 1 is behind the barrier.
// Every wave passes the same number of steps (a half without a tile runs empty steps), so the barrier
// counts always match.
//
// Layout (LDS, floats): split-f16 weights in the grouped hi / lo order (HL, see bneck_kernels.hip) with
// rows of 8 / 40 dwords mod 64 (136 / 296 / 40: conflict-free for ds_read_b128's lane groups
// {0-3,12-15,20-27} ... of MI355X_MICROARCH.md §LDS); two t0 buffers of 18 x 18 pixels x 32 channels
// UNPADDED (128 B: two buffers plus the weights fit 160 KB only so) with the pixel's eight 16-B chunks
// XOR-swizzled by (h & 7) — conflict-free for those lane groups over any run of consecutive pixels. 16 waves per CU = 4 per SIMD: 128 VGPRs, so the
// residual is re-read in phase 3 (issued before the middle conv; L2 hits — phase 1 of the same tile read
// it one step earlier) instead of kept from phase 1 as bneck_kernel's KEEPF does.
//
// MEASURED SLOWER, so not planned by default (BUGSEG_BNECK2=1 plans it; tests/test_gpu_parity.py keeps it
// bit-identical to the unfused chain). Round 6, B = 64, 480 x 640, A/B on one box: 103 us per launch
// against 87 us for bneck_kernel's 16 x 16 fp32 form (fp32 bench 18.9k vs 19.35k frames/s). Ablations:
// phases 2 + 3 alone 70 us, phase 1 alone 49 us — the two halves do overlap (103 < 119), but each phase
// runs ~2x slower than in bneck_kernel: at 4 waves per SIMD the 128-VGPR budget leaves one phase-1
// fragment pair's loads in flight instead of all of a wave's, no kept residual (8 L2 re-reads per
// fragment), and the middle conv fragment by fragment (no weight-read sharing). Without the k-step
// fences (122 VGPRs) or with the middle conv unrolled by 3: 105-106 us. The budget, not the schedule,
// bounds it; a form with 8 waves (two 4-wave halves, 256 VGPRs) would keep the registers but halve
// the waves per tile.
#include "bugseg_internal.h"
#include "mfma_common.h"

namespace bugseg {

namespace {
constexpr int P2_TH = 16, P2_TW = 16, P2_NWH = 8;          // tile; waves per half
constexpr int P2_C = 128, P2_I = 32, P2_NR1 = 2, P2_NR3 = 8, P2_KS1 = 4, P2_KS2 = 9;
constexpr int P2_HWW = P2_TW + 2, P2_HR = (P2_TH + 2) * P2_HWW;   // 18 x 18 halo
constexpr int P2_NF1 = (P2_HR + 15) / 16;                   // 21 halo fragments
constexpr int P2_NFT = P2_TH * P2_TW / 16;                  // 16 tile fragments (= tile rows)
constexpr int P2_NF2 = P2_NFT / P2_NWH;                     // 2 per wave
constexpr int P2_K1S = P2_KS1 * 32 + 8, P2_K2S = P2_KS2 * 32 + 8, P2_K3S = 32 + 8;   // rows 8 / 40 dwords mod 64
constexpr int P2_PSTR = P2_I;                                // t0 pixel: 32 floats, unpadded (swizzled)
constexpr int P2_W1 = P2_NR1 * 16 * P2_K1S, P2_W2 = P2_NR1 * 16 * P2_K2S, P2_W3 = P2_C * P2_K3S;
constexpr int P2_CONSTS = 4 * P2_NR1 * 16 + 3 * P2_C;       // cb1 cs1 cb2 cs2 | cb3 cs3 cso
constexpr int P2_ZP = 32;
constexpr int P2_TSF = P2_HR * P2_PSTR;                      // floats per t0 buffer
constexpr size_t P2_LDS = (size_t)(P2_W1 + P2_W2 + P2_W3 + P2_CONSTS + P2_ZP + 2 * P2_TSF) * 4;
static_assert(P2_LDS <= 160 * 1024, "two t0 buffers and one weight copy in 160 KB");
}  // namespace

#ifndef BNECK2_CH1
#define BNECK2_CH1 2      // phase-1 fragments whose x loads fly together (VGPRs: 32 each)
#endif
#ifndef BNECK2_U2
#define BNECK2_U2 1       // middle-conv k-steps unrolled together
#endif
#ifndef BNECK2_FENCE1
#define BNECK2_FENCE1 1   // phase 1: no weight read hoisted across k-steps (hoisted, they need 64 VGPRs)
#endif

template <bool SCL>
__device__ __forceinline__ void bneck2_body(const BneckArgs &a, float rlane, float *smem) {
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // lane coordinates re-derived inside each phase from an opaque copy of the lane id: everything
    // per-lane is then computed per step instead of hoisted out of the step loop as invariants (which
    // the 128-VGPR budget could only hold by spilling them)
    auto lane_xy = [](int &col, int &kq) {
        int l = (int)(threadIdx.x & 63);
        asm volatile("" : "+v"(l));
        col = l & 15;
        kq = l >> 4;
    };
    const int half = wave >> 3, hw = wave & 7;                // wave-uniform
    float *w1s = smem, *w2s = w1s + P2_W1, *w3s = w2s + P2_W2;
    float *cb1 = w3s + P2_W3, *cs1 = cb1 + 32, *cb2 = cs1 + 32, *cs2 = cb2 + 32;
    float *cb3 = cs2 + 32, *cs3 = cb3 + P2_C, *cso = cs3 + P2_C;
    float *zpad = cso + P2_C;
    float *ts = zpad + P2_ZP + half * P2_TSF;                 // this half's t0 buffer
    const auto rxb = mkbuf(a.x, a.x_bytes);
    const auto rob = mkbuf(a.out, a.x_bytes);
    auto act = [&](float4 v, const float *s) { return prelu4m(v, ld4f(s)); };   // slopes <= 1 (planned so)
    auto ldw = [](RawS &r, const float *p, int kq) {          // HL: hi chunk kq, lo chunk 4 + kq
        r.h = *reinterpret_cast<const uint4 *>(p + kq * 4);
        r.l = *reinterpret_cast<const uint4 *>(p + 16 + kq * 4);
    };
    // t0 chunk c (0..3 hi parts of groups 0..3, 4..7 lo parts) of halo pixel h: float offset
    auto tso = [](int h, int c) -> int { return h * P2_PSTR + ((c ^ (h & 7)) << 2); };

    BneckRange rg0;
    if constexpr (SCL) rg0 = bneck_range<false>(a.rg, rng_reduce(rlane));
    const bool scl = rg0.scl;
    const float xm = rg0.xm, b1m = rg0.b1m, o1m = rg0.o1m, b2m = rg0.b2m, o2m = rg0.o2m, b3m = rg0.b3m, o3m = rg0.o3m;
    float amo = 0.f;

    // XCD-aware tile walk as bneck_kernel's, per HALF: half-slot hs of the workgroup's XCD group takes
    // tiles grp * CH + hs, + nhs, ...
    const int G = gridDim.x, grp = blockIdx.x & 7, nhs = (G >> 3) * 2;
    const int CH = (a.ntiles + 7) >> 3;
    auto ntiles_of = [&](int hs) -> int {
        const int lim = min(CH, a.ntiles - grp * CH);
        return hs < lim ? (lim - hs + nhs - 1) / nhs : 0;
    };
    const int hs = (int)(blockIdx.x >> 3) * 2 + half;
    const int n0 = ntiles_of((int)(blockIdx.x >> 3) * 2), n1 = ntiles_of((int)(blockIdx.x >> 3) * 2 + 1);
    const int nmy = half ? n1 : n0;
    const int K = max(2 * n0, 2 * n1 + 1);                   // steps (workgroup-uniform)
    auto tile_geom = [&](int tile, int &n, int &oy0, int &ox0) {
        int t = tile;
        const int txi = t % a.tiles_x; t /= a.tiles_x;
        const int tyi = t % a.tiles_y; t /= a.tiles_y;
        const int ph = t % a.phases;
        n = t / a.phases;
        const int py = ph / a.dt, px = ph - py * a.dt;
        oy0 = py + a.dt * tyi * P2_TH;
        ox0 = px + a.dt * txi * P2_TW;
    };
    const int dt = a.dt;
    auto pix_base = [&](int n, int y, int x) -> uint32_t {   // channel 0 of image pixel (y, x), or OOB
        uint32_t v = (uint32_t)(n * a.H * a.W) * (uint32_t)(P2_C * 4) + (__umul24((uint32_t)y, (uint32_t)a.W) + (uint32_t)x) * (uint32_t)(P2_C * 4);
        asm volatile("" : "+v"(v));
        return y < a.H && x < a.W ? v : OOB;
    };

    // ---- phase 1 of tile `tile`: t0 = act1(W1 x + b1) over tile + halo (0 outside the image)
    auto phase1 = [&](int tile) {
        int n, oy0, ox0;
        tile_geom(tile, n, oy0, ox0);
        // opaque per-step offset: the weight-row addresses are computed here, not hoisted out of the step
        // loop as invariants (held across both phases they cost the 128-VGPR budget dozens of registers)
        int col, kq;
        lane_xy(col, kq);
        const float *w1 = w1s;
        const uint32_t xn = (uint32_t)(n * a.H * a.W) * (uint32_t)(P2_C * 4);
        constexpr int NFW = (P2_NF1 + P2_NWH - 1) / P2_NWH;     // 3: halo fragments per wave (at most)
#pragma unroll
        for (int c0 = 0; c0 < NFW; c0 += BNECK2_CH1) {
            RawF xf[BNECK2_CH1][P2_KS1];
            bool okc[BNECK2_CH1];
            int hc[BNECK2_CH1];
#pragma unroll
            for (int c = 0; c < BNECK2_CH1; ++c) {
                const int fh = hw + P2_NWH * (c0 + c);
                if (c0 + c >= NFW || fh >= P2_NF1) break;            // wave-uniform
                const int h = fh * 16 + col;
                const int hy = h / P2_HWW, hx = h - hy * P2_HWW;
                const int iy = oy0 + dt * (hy - 1), ix = ox0 + dt * (hx - 1);
                hc[c] = h;
                okc[c] = h < P2_HR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
#pragma unroll
                for (int s = 0; s < P2_KS1; ++s)
                    bld8(xf[c][s], rxb, okc[c] ? xn + ((__umul24((uint32_t)iy, (uint32_t)a.W) + (uint32_t)ix) * P2_C + (s * 4 + kq) * 8) * 4u : OOB);
            }
#pragma unroll
            for (int c = 0; c < BNECK2_CH1; ++c) {
                if (c0 + c >= NFW || hw + P2_NWH * (c0 + c) >= P2_NF1) break;   // wave-uniform
                f32x4 acc[P2_NR1];
#pragma unroll
                for (int r = 0; r < P2_NR1; ++r) acc[r] = bias4(cb1 + r * 16 + kq * 4);
                if constexpr (SCL) {
#pragma unroll
                    for (int r = 0; r < P2_NR1; ++r) acc[r] = mul4(acc[r], b1m);
                }
#pragma unroll
                for (int s = 0; s < P2_KS1; ++s) {
                    RawF xq = xf[c][s];
                    if constexpr (SCL) xq = scale8(xf[c][s], xm);
#pragma unroll
                    for (int r = 0; r < P2_NR1; ++r) {
                        RawS wf;
                        ldw(wf, w1 + (r * 16 + col) * P2_K1S + s * 32, kq);
                        mma(acc[r], wf, xq);
                    }
                    if (BNECK2_FENCE1) asm volatile("" ::: "memory");   // keeps the next k-step's weight reads here
                }
                if constexpr (SCL) {
#pragma unroll
                    for (int r = 0; r < P2_NR1; ++r) acc[r] = mul4(acc[r], o1m);
                }
                const int h = hc[c];
                if (h < P2_HR) {
#pragma unroll
                    for (int r = 0; r < P2_NR1; ++r) {
                        const int ch = r * 16 + kq * 4;
                        float4 v = act(f4(acc[r]), cs1 + ch);
                        if (!okc[c]) v = make_float4(0.f, 0.f, 0.f, 0.f);
                        // split as st4hl: hi parts into chunk g, lo parts into chunk 4 + g (g = ch / 8)
                        const float e[4] = {v.x, v.y, v.z, v.w};
                        _Float16 hh[4], ll[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            hh[i] = (_Float16)e[i];
                            ll[i] = (_Float16)(e[i] - (float)hh[i]);
                        }
                        const int g = ch >> 3, sub = ch & 7;
                        unsigned char *base = reinterpret_cast<unsigned char *>(ts);
                        *reinterpret_cast<f16x4 *>(base + tso(h, g) * 4 + sub * 2) = (f16x4){hh[0], hh[1], hh[2], hh[3]};
                        *reinterpret_cast<f16x4 *>(base + tso(h, 4 + g) * 4 + sub * 2) = (f16x4){ll[0], ll[1], ll[2], ll[3]};
                    }
                }
            }
        }
    };

    // ---- phases 2 + 3 of tile `tile` (its t0 in this half's buffer)
    auto phase23 = [&](int tile) {
        int n, oy0, ox0;
        tile_geom(tile, n, oy0, ox0);
        int col, kq;
        lane_xy(col, kq);
        const float *w2 = w2s, *w3 = w3s;
        const bool lo8 = col < 8;
        // fragment by fragment (j: tile row f = hw + 8 j, pixel column col): its residual loads (x at the
        // tile pixels, phase 3's quads) are issued first and land during its middle conv; then the
        // expansion. (Both fragments' middle convs together, sharing each k-step's weight reads, need
        // their accumulators and phase-3 operands live at once: past the 128-VGPR budget with the
        // residual in flight.) The products and their order per output are the same either way.
#pragma unroll 1
        for (int j = 0; j < P2_NF2; ++j) {
            const int f = hw + P2_NWH * j;
            const uint32_t po = pix_base(n, oy0 + dt * f, ox0 + dt * col);
            uint4 res[P2_NR3];
#pragma unroll
            for (int t = 0; t < P2_NR3; ++t) res[t] = bld16(rxb, po == OOB ? OOB : po + (uint32_t)(t * 16 + kq * 4) * 4u);
            // phase 2: t1 = act2(W2 * t0 + b2): k-step s = tap s (4 groups of 8 channels), (ky, kx) = (s / 3, s % 3)
            f32x4 acc[P2_NR1];
#pragma unroll
            for (int r = 0; r < P2_NR1; ++r) {
                acc[r] = bias4(cb2 + r * 16 + kq * 4);
                if constexpr (SCL) acc[r] = mul4(acc[r], b2m);
            }
#pragma unroll BNECK2_U2
            for (int s = 0; s < P2_KS2; ++s) {
                const int ky = s / 3, kx = s - ky * 3;
                RawS wf[P2_NR1];
#pragma unroll
                for (int r = 0; r < P2_NR1; ++r) ldw(wf[r], w2 + (r * 16 + col) * P2_K2S + s * 32, kq);
                int h = (f + ky) * P2_HWW + (col + kx);
                asm volatile("" : "+v"(h));
                RawS xf;
                xf.h = *reinterpret_cast<const uint4 *>(ts + tso(h, kq));
                xf.l = *reinterpret_cast<const uint4 *>(ts + tso(h, 4 + kq));
#pragma unroll
                for (int r = 0; r < P2_NR1; ++r) mma(acc[r], wf[r], xf);
                if (BNECK2_FENCE1) asm volatile("" ::: "memory");
            }
            if constexpr (SCL) {
#pragma unroll
                for (int r = 0; r < P2_NR1; ++r) acc[r] = mul4(acc[r], o2m);
            }
            RawF tf;
            to_bop(tf, act(f4(acc[0]), cs2 + kq * 4), act(f4(acc[1]), cs2 + 16 + kq * 4));
            // phase 3: out = act_out(act3(W3 t1 + b3) + x), whole-line stores (bneck_kernels.hip LINES)
            const uint32_t po_o = pix_base(n, oy0 + dt * f, ox0 + dt * (col ^ 8));
            const uint32_t pa = lo8 ? po : po_o, pb = lo8 ? po_o : po;
#pragma unroll
            for (int u = 0; u < P2_NR3 / 2; ++u) {
                float4 v2[2];
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int t = 2 * u + hh, ch = t * 16 + kq * 4;
                    f32x4 ac = bias4(cb3 + ch);
                    if (SCL || scl) ac = mul4(ac, b3m);
                    RawS wf;
                    ldw(wf, w3 + (t * 16 + col) * P2_K3S, kq);
                    mma(ac, wf, tf);
                    float4 v = f4(ac);
                    if (scl) v = mul4(v, o3m);
                    v = act(v, cs3 + ch);
                    v2[hh] = act(add4(v, __builtin_bit_cast(float4, res[t])), cso + ch);
                    rng_acc4(amo, v2[hh]);
                }
                const uint4 u0 = __builtin_bit_cast(uint4, v2[0]), u1 = __builtin_bit_cast(uint4, v2[1]);
                const uint4 xs = lo8 ? u1 : u0;
                uint4 ys;
                ys.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.x, 0x128, 0xf, 0xf, false);
                ys.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.y, 0x128, 0xf, 0xf, false);
                ys.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.z, 0x128, 0xf, 0xf, false);
                ys.w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.w, 0x128, 0xf, 0xf, false);
                const uint32_t cb = (uint32_t)(u * 32 + (lo8 ? 0 : 16) + kq * 4) * 4u;
                bst16o<16>(rob, pa == OOB ? OOB : pa + cb, lo8 ? u0 : ys);
                bst16o<16>(rob, pb == OOB ? OOB : pb + cb, lo8 ? ys : u1);
                if (BNECK2_FENCE1) asm volatile("" ::: "memory");   // the next row pair's weight reads stay here
            }
        }
    };

    // step k: half 0 runs phase 1 of its tile k / 2 (k even) or phases 2 + 3 of tile (k - 1) / 2; half 1
    // one step later
    for (int k = 0; k < K; ++k) {
        const int kk = k - half;
        if (kk >= 0) {
            const int i = kk >> 1;
            if (i < nmy) {
                const int tile = grp * CH + hs + i * nhs;
#ifndef BNECK2_SKIP
#define BNECK2_SKIP 0
#endif
                if ((kk & 1) == 0) { if (BNECK2_SKIP != 1) phase1(tile); }
                else { if (BNECK2_SKIP != 2) phase23(tile); }
            }
        }
        __syncthreads();
    }
    rng_commit_wg(amo, a.rg.amax_out, smem + P2_W1 + P2_W2 + P2_W3 + P2_CONSTS + P2_ZP, 2 * P2_NWH);
}

__global__ void __launch_bounds__(1024, 1) bneck2_f32_kernel(const BneckArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem2[];
    span_enter(a.span);
    {
        // a workgroup without a tile leaves before staging anything
        const int CH = (a.ntiles + 7) >> 3, lim = min(CH, a.ntiles - (int)(blockIdx.x & 7) * CH);
        if ((int)(blockIdx.x >> 3) * 2 >= lim) {
            span_exit(a.span);
            return;
        }
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int NW = 16;
    float *w1 = smem2, *w2 = w1 + P2_W1, *w3 = w2 + P2_W2;
    float *cb1 = w3 + P2_W3;
    // weights by LDS-DMA in the HL chunk order (bneck_kernels.hip pick()); rows of SR 16-B slots, the
    // last of each a pad slot (re-reads the row's first chunk; never read)
    {
        constexpr int SR1 = P2_K1S / 4, SR2 = P2_K2S / 4, SR3 = P2_K3S / 4;
        constexpr int CPR1 = P2_KS1 * 8, CPR2 = P2_KS2 * 8, CPR3 = 8;
        constexpr int S1 = P2_NR1 * 16 * SR1, S2 = P2_NR1 * 16 * SR2, S3 = P2_C * SR3, NSL = S1 + S2 + S3;
        for (int base = wave * 64; base < NSL; base += NW * 64) {          // wave-uniform
            const int q = base + lane;
            const uint4 *src;
            auto pick = [&](const void *w, int k, int SR, int CPR) {
                const int r = k / SR, c = k - r * SR;
                const int cs = (c & ~7) | ((c & 7) < 4 ? 2 * (c & 7) : 2 * (c & 3) + 1);
                src = (const uint4 *)w + r * CPR + (c < CPR ? cs : 0);
            };
            if (q < S1) pick(a.w1, q, SR1, CPR1);
            else if (q < S1 + S2) pick(a.w2, q - S1, SR2, CPR2);
            else pick(a.w3, q - S1 - S2, SR3, CPR3);
            if (q < NSL)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                                 (__attribute__((address_space(3))) void *)(smem2 + (size_t)base * 4), 16, 0, 0);
        }
    }
    const float rl = rng_lane(a.rg);
    {
        float *cs1 = cb1 + 32, *cb2 = cs1 + 32, *cs2 = cb2 + 32, *cb3 = cs2 + 32, *cs3 = cb3 + P2_C, *cso = cs3 + P2_C;
        float *zpad = cso + P2_C;
        if (tid < 32) { cb1[tid] = a.b1[tid]; cs1[tid] = a.s1[tid]; cb2[tid] = a.b2[tid]; cs2[tid] = a.s2[tid]; zpad[tid] = 0.f; }
        if (tid < P2_C) { cb3[tid] = a.b3[tid]; cs3[tid] = a.s3[tid]; cso[tid] = a.s_out[tid]; }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!a.rg.off && bneck_range<false>(a.rg, rng_reduce(rl)).any) bneck2_body<true>(a, rl, smem2);
    else bneck2_body<false>(a, rl, smem2);
    span_exit(a.span);
}

size_t bneck2_lds_bytes() { return P2_LDS; }

int bneck2_slots_per_cu() {
    static int cached = -1;
    if (cached < 0) {
        if (allow_dynamic_lds((const void *)bneck2_f32_kernel) != hipSuccess) return cached = 0;
        cached = occupancy_per_cu((const void *)bneck2_f32_kernel, 1024, P2_LDS);
    }
    return cached;
}

hipError_t launch_bneck2(const BneckArgs &a, hipStream_t s) {
    hipError_t e = allow_dynamic_lds((const void *)bneck2_f32_kernel);
    if (e != hipSuccess) return e;
    // one resident round: one workgroup per CU, each walking its two halves' tiles
    const char *ge = std::getenv("BUGSEG_BNECK_GRID");
    const int cap = ge && std::atoi(ge) > 0 ? std::atoi(ge) : device_cus() * std::max(1, bneck2_slots_per_cu());
    const int want = (a.ntiles + 1) / 2;                     // two tiles per workgroup at a time
    int g = want < cap ? want : cap;
    g = (g + 7) & ~7;
    void *args[] = {const_cast<BneckArgs *>(&a)};
    return hipLaunchKernel((const void *)bneck2_f32_kernel, dim3(g), dim3(1024), args, P2_LDS, s);
}

}  // namespace bugseg
