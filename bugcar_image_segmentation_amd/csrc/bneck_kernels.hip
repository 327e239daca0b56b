// Fused ENet regular / dilated / asymmetric bottleneck in ONE launch.
//
//   t0  = act1(W1 . x + b1)            1x1 projection C -> I (= C/4)     over the tile + halo
//   t1  = act2(W2 * t0 + b2)           3x3 (dilation d) or 5x1 then 1x5 over the tile
//   out = act_out(act3(W3 . t1 + b3) + x)                                 1x1 expansion + residual
//
// Unfused, each 128-channel bottleneck moves ~1024 B/pixel through HBM (x read twice, three internal
// tensors written and read); here x is read once (halo re-reads are L2 hits) and out written once:
// 512 B/pixel in bf16. The internal tensors never leave LDS:
//   * a workgroup owns a TH x TW tile of one frame; phase 1 computes t0 for the tile plus a halo ring
//     of R pixels (zero outside the image: t0 is what the middle conv zero-pads);
//   * phase 2 accumulates its whole tile in registers, then (after a barrier) overwrites the t0
//     region with t1, so one LDS region serves both (asymmetric: t0 -> t1a -> t1, same trick);
//   * phase 3 streams 16-pixel fragments: MFMA with W3, residual, activation and 16-B-per-lane
//     stores, all in registers (lane-pair transposes with v_permlane16_swap).
//
// Dilated tiling. A 3x3 conv of dilation d only couples pixels whose coordinates agree mod d, so a
// tile is a TH x TW block of ONE such phase: tile pixel (i, j) is image pixel (oy0 + d*i, ox0 + d*j),
// and the dilated conv is a plain 3x3 over tile coordinates with a one-pixel halo ring whatever d is
// (the d-pixel halo of a contiguous tile recomputes (16+2d)^2 / 16^2 of the projection: 2.25x at
// d = 4). NHWC keeps every pixel a contiguous C-element run, so strided pixels cost no extra lines.
//
// Tile shapes are template variants (BShape) picked per layer by the runtime (bugseg_runtime.cpp
// pick_bneck_variant) so that the tile count fills the resident workgroup slots in whole rounds. A
// tile may be transposed (a.tr: tile rows run along image columns; the middle conv's taps swap
// axes with it), so one 20 x 16 shape covers 60 x 80 at d = 1 (20 rows x 16 columns), d = 2 and
// d = 4 (20 columns x 16 rows of a 30 x 40 / 15 x 20 phase) in 15-16 tiles per frame. Fragments
// are 16-pixel runs of one tile row (TW is a multiple of 16), so a fragment's row is wave-uniform.
//
// MFMA operand mapping as conv_kernels.hip: A = weights (row = output channel) from LDS, B = 8
// channels of one pixel (16-B LDS or global read per lane), accumulator = 4 consecutive channels of
// one pixel per lane. All three weight matrices stay in LDS for the workgroup's lifetime.
#include <algorithm>
#include <cstdlib>

#include <type_traits>

#include "bugseg_internal.h"
// output stores: the per-kernel cache-policy choice (OUT_AUX_SEL: sc1 write-through for C >= 64).
// Round 2, after the kept residual and the LDS-DMA staging: 4-9% faster per launch (C128 20x16
// 23.3 -> 21.3 us, C64 35.1 -> 34.0 us, forward 0.80 -> 0.77 ms one stream at a time) and equal in
// the 2-stream bench (round 1 had measured it 2.4% slower there)
#ifndef BUGSEG_OUT_AUX
#define BUGSEG_OUT_AUX -1
#endif
#include "cls_common.h"

namespace bugseg {

// Debug build only (-DBUGSEG_STAMPS, scripts/stamp_probe.py): thread 0 of each workgroup records the
// shader clock at phase boundaries of every tile, stamps[tile * 8 + k]; slot 7 = workgroup index.
#ifdef BUGSEG_STAMPS
__device__ unsigned long long *bugseg_stamps;
#define STAMP(k) do { if (tid == 0 && bugseg_stamps) bugseg_stamps[(size_t)tile * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#define STAMP_WG() do { if (tid == 0 && bugseg_stamps) bugseg_stamps[(size_t)tile * 8 + 7] = blockIdx.x; } while (0)
// per workgroup: kernel entry and exit on the constant 100 MHz clock (s_memrealtime: one time base
// for every XCD) at [2^19 + 2 blockIdx.x (+1)]
#define STAMP_ENTRY(k) do { if (threadIdx.x == 0 && bugseg_stamps) bugseg_stamps[(1u << 19) + 2u * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP_ENTRY(k) do {} while (0)
#define STAMP(k) do {} while (0)
#define STAMP_WG() do {} while (0)
#endif

// s_waitcnt vmcnt(n) for a wave-uniform n (the immediate has to be a constant): waits until at most n
// of this wave's vector-memory operations are outstanding. n is clamped to 0..24 in steps of 2.
__device__ __forceinline__ void vm_wait_upto(int n) {
#define VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    switch (n) {
        VMW(2) VMW(4) VMW(6) VMW(8) VMW(10) VMW(12) VMW(14) VMW(16) VMW(18) VMW(20) VMW(22) VMW(24)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef VMW
}

// Tile shape variants per channel count: TH x TW tile pixels, NW waves per workgroup, OCC = waves
// per SIMD the bf16 build is held to (registers), matching what LDS allows. 128 channels: the LDS
// footprint (weights + halo or output staging, ~75 KB) allows two workgroups per CU, so they are
// 8-wave; 64 / 16 channels (~28-33 KB): four 4-wave workgroups per CU.
template <int C, int V> struct BShape;
// RP = residual fragments each wave prefetches before the middle conv (a ring refilled in phase 3
// when a wave has more fragments than that: an L2 round trip then sits on the phase-3 path).
// RD = row-dilated full-width tiles (symmetric blocks, large dilation d on narrow maps): a tile is
// TH rows d apart (one row phase) spanning all columns (W <= TW), so the middle conv's vertical taps
// are the tile's one-row halo and its horizontal taps stay inside the tile — masked at the image
// edge, no horizontal halo stored. 4 x 80 tiles cover 60 x 80 at d = 8 and d = 16 in 16 tiles per
// frame (the phase sub-images, 8 x 10 and 4 x 5, are far too small for square tiles).
template <> struct BShape<128, 0> { static constexpr int TH = 16, TW = 16, NW = 8, OCC = 4, RP = 2, RD = 0, WIDE = 1; };
template <> struct BShape<128, 1> { static constexpr int TH = 20, TW = 16, NW = 8, OCC = 4, RP = 2, RD = 0, WIDE = 1; };
template <> struct BShape<128, 2> { static constexpr int TH = 4, TW = 80, NW = 8, OCC = 4, RP = 2, RD = 1, WIDE = 0; };
template <> struct BShape<128, 3> { static constexpr int TH = 4, TW = 64, NW = 8, OCC = 4, RP = 2, RD = 1, WIDE = 1; };
// 8 x 16: the small-batch forms (batch 1: 40 C128 tiles at 60 x 80 instead of 15; 150 C64 tiles at
// 120 x 160 instead of 80), picked by the runtime's round model only when whole rounds are few
template <> struct BShape<128, 4> { static constexpr int TH = 8, TW = 16, NW = 8, OCC = 4, RP = 1, RD = 0, WIDE = 1; };
template <> struct BShape<64, 0> { static constexpr int TH = 16, TW = 16, NW = 4, OCC = 5, RP = 4, RD = 0, WIDE = 1; };
template <> struct BShape<64, 2> { static constexpr int TH = 8, TW = 16, NW = 4, OCC = 5, RP = 2, RD = 0, WIDE = 1; };
template <> struct BShape<64, 1> { static constexpr int TH = 20, TW = 16, NW = 4, OCC = 5, RP = 3, RD = 0, WIDE = 1; };
template <> struct BShape<16, 0> { static constexpr int TH = 16, TW = 16, NW = 4, OCC = 6, RP = 4, RD = 0, WIDE = 1; };
// 20 x 16: 7,680 tiles at 32 frames, 5 whole rounds of the 1,536 resident slots (16 x 16: 9,600 tiles,
// 6.25 rounds -> 7); the cost model picks it (32 x 16 and 16 x 32 tiles measured slower in round 3:
// 56.9 / 56.6 vs 49.4-50.4 us per launch, and were removed). Measured (round 3, fp16, B = 32): 48.0-48.4 vs 48.6-48.8 us
// per launch — equal within noise: the stage-5 block is not round-quantisation bound
template <> struct BShape<16, 1> { static constexpr int TH = 20, TW = 16, NW = 4, OCC = 6, RP = 4, RD = 0, WIDE = 1; };

// LDS strides (elements). bf16: a 16-lane group of ds_read_b128 (one 16-B k group of 16 pixels or
// weight rows) is conflict-free when the row stride is 8, 24, 40 or 56 dwords mod 64 (the SQ counters
// had 35% of LDS cycles in bank conflicts with the 16-B pads): weight rows pad 16 elements; t0
// pixels unpadded for 8 / 16 internal channels and 48 elements for 32 where the workgroup still fits
// twice per CU (WIDE; asymmetric and 4x80 tiles keep 40); fp32 (parity mode) keeps 16-B pads.
// (fp32 keeps 16-B pads: 32-B pads by the bf16 rule measured neutral on C = 128 with the split t0 below
// — 45.8 vs 45.8 us per launch — and slower on C = 64 / 16, 77.0 -> 81.5 / 96.7 -> 108.4 us; round 4)
// fp32 C = 128 (not the down form): HL, the grouped split layout (see the body) — weight rows and t0 pixels
// padded to 8 / 40 dwords mod 64, the conflict-free strides for its 16-B-per-lane reads
#ifndef BNECK_F32_HL
#define BNECK_F32_HL 1
#endif
// fp32 C = 64 (round 6): the weights in the same HL layout (rows 8 / 40 dwords mod 64) and
// t0 as two PLANES — every pixel's 16 channels' hi parts (32 B) in one, their lo parts in the other, 8
// dwords per pixel each, unpadded: the middle conv's 16-lane read groups then hit distinct banks (lanes
// col and col + 8 of a group read the same bank row but the other 8-channel group) — where the interleaved
// split layout (hi + lo per group, 20-dword pixels) was 2-way conflicted on every read (SQ: 35% of the
// C64 forms' LDS cycles), in less LDS (two planes of 8 dwords vs 20 dwords per pixel; the weights' wider
// pads fit in the difference, so the 8 x 16 form keeps its 4 workgroups per CU)
#ifndef BNECK_F32_HL64
#define BNECK_F32_HL64 1
#endif
__host__ __device__ constexpr bool bneck_hl(int es, int C, bool dn) {
    return BNECK_F32_HL && es == 4 && (C == 128 || (C == 64 && BNECK_F32_HL64)) && !dn;
}
__host__ __device__ constexpr bool bneck_pl(int es, int C, bool dn) { return bneck_hl(es, C, dn) && C == 64; }
__host__ __device__ constexpr int bneck_padw(int es, int C, bool wide, bool dn) {
    return bneck_hl(es, C, dn) ? 8 : es == 2 && (C != 128 || wide) ? 16 : 16 / es;
}
__host__ __device__ constexpr int bneck_pstr(int es, int IS, bool wide) {
    return es != 2 ? (BNECK_F32_HL && es == 4 && IS == 32 ? 40 : IS + 16 / es) : IS == 32 ? (wide ? 48 : 40) : IS;
}
static bool bneck_wide(int C, int v, bool asym) {
#define BW_CASE(CC, VV) if (C == CC && v == VV) return BShape<CC, VV>::WIDE && !asym;
    BW_CASE(128, 0) BW_CASE(128, 1) BW_CASE(128, 2) BW_CASE(128, 3) BW_CASE(128, 4) BW_CASE(64, 0) BW_CASE(64, 1) BW_CASE(64, 2) BW_CASE(16, 0) BW_CASE(16, 1)
#undef BW_CASE
    return false;
}

int bneck_variants(int C) { return C == 128 ? 6 : C == 16 ? 2 : 3; }   // C128 variant 5: bneck2_kernels.hip (fp32)

void bneck_shape(int C, int v, int &th, int &tw, int &nw, int *rd) {
    if (C == 128 && v == BNECK2_V) { th = 16; tw = 16; nw = 16; if (rd) *rd = 0; return; }
#define BS_CASE(CC, VV) if (C == CC && v == VV) { th = BShape<CC, VV>::TH; tw = BShape<CC, VV>::TW; nw = BShape<CC, VV>::NW; if (rd) *rd = BShape<CC, VV>::RD; return; }
    BS_CASE(128, 0) BS_CASE(128, 1) BS_CASE(128, 2) BS_CASE(128, 3) BS_CASE(128, 4) BS_CASE(64, 0) BS_CASE(64, 1) BS_CASE(64, 2) BS_CASE(16, 0) BS_CASE(16, 1)
#undef BS_CASE
    th = tw = nw = 0;
    if (rd) *rd = 0;
}

// CI > 0: the DOWNSAMPLING bottleneck with a CI-channel input at twice the
// output resolution: the projection is the 2x2 stride-2 conv (K = 4 CI), the middle conv the block's
// 3x3, and the residual is the main branch — maxpool 2x2 of the input, zero-padded from CI to C
// channels, its argmax indices written for the paired upsampling block. The pooling uses the
// projection's own B fragments (lane kq holds taps of one 8-channel group: the 4 taps in-lane for
// CI >= 32, two taps in-lane + one v_permlane32_swap for CI = 16) and leaves the pooled values in a
// small global scratch (a.pool) that phase 3 reads back as its residual (L2 hits).
// fp32 (parity mode): registers unconstrained (LDS bounds the C = 64 / 128 forms first), except C = 16,
// held to 4 waves per SIMD (5 spilled with the split t0 storage below; unconstrained: 16 AGPRs on top of 91 VGPRs)
#ifndef BNECK_F32_SPLIT_T0
#define BNECK_F32_SPLIT_T0 1
#endif
#ifndef BNECK_F32_OCC16
#define BNECK_F32_OCC16 4   // (5 spilled 32 B with the split t0: 102.0 vs 90.8 us per launch at 4)
#endif
// fp32 C = 64 / 128: waves per SIMD the build is held to (1 = registers unconstrained; A/B knob, round 4:
// with split-f16 products the fp32 forms are issue / latency bound at 2-3 waves per SIMD)
#ifndef BNECK_F32_OCC64
#define BNECK_F32_OCC64 1
#endif
#ifndef BNECK_F32_OCC64_V2
#define BNECK_F32_OCC64_V2 4   // the 8 x 16 C = 64 form: 127 VGPRs, no spills at 4 (round 5: 139.8 -> 137.9 us per launch; 1 = unconstrained, 154 VGPRs, 3 waves per SIMD)
#endif
#ifndef BNECK_F32_OCC128
#define BNECK_F32_OCC128 1
#endif
// fp32 mode range scaling (bugseg_internal.h RangeArgs, mfma_common.h): the exponents of x (measured by
// the launch that wrote it), t0, t1 (asymmetric: t1a, t1; rigorous bounds from x's range), as the
// multipliers of the accumulators. `any`: some multiply is needed — the asymmetric 1x5's output aside,
// whose exponent each tile decides from its own t1a. The kernel runs the body instantiated with no
// multiply at all first (SCL = false: the unscaled instruction stream; the scaled one measured 8% slower
// on the forward with every multiplier 1, round 5); that body reads the range only once its first
// tile's loads are in flight (a wait for the range words alone at kernel start cost the C128 launches
// ~4 us) and, if some exponent is non-zero, drains its loads and returns before computing anything —
// the kernel then runs the scaled body from the start.
template <typename T, int C, bool ASYM, int V, bool TR, int CI, bool SCL, int FC = -1>
__device__ __forceinline__ bool bneck_body(const BneckArgs &a, float rlane) {
    using Raw = typename Tr<T>::Raw;
    using WRaw = typename WTr<T>::Raw;   // weight operand (fp32 mode: split-f16 parts)
    constexpr int TH = BShape<C, V>::TH, TW = BShape<C, V>::TW, NW = BShape<C, V>::NW, NT = NW * 64;
    constexpr int I = CI > 0 ? CI / 4 : C / 4;      // internal channels (ENet: input / 4)
    constexpr int IS = I < 8 ? 8 : I;                 // stored internal channels (8-channel groups)
    constexpr int NR1 = (I + 15) / 16;                // 16-row fragments of t0 / t1
    constexpr int NR3 = C / 16;                       // 16-row fragments of out
    constexpr bool DN = CI > 0;                       // (I above already depends on it)
    // output store policy (mfma_common.h): sc1 for C >= 64; the fp32 C = 64 (non-down) form streams its
    // output non-temporally (nt) — round 5, B = 64, one stream: the blocks reading it (down C128, up C16)
    // 14-18 us faster per launch. nt measured worse for the fp32 C16 form (itself +4 us), the down forms
    // (down C64 +32 us) and the C128 forms (+10%) — A/B knobs BNECK_NT_F32_C64 / _C16 / _DN
#ifndef BNECK_NT_F32_C64
#define BNECK_NT_F32_C64 1
#endif
#ifndef BNECK_NT_F32_C16
#define BNECK_NT_F32_C16 0
#endif
#ifndef BNECK_NT_F32_DN
#define BNECK_NT_F32_DN 0
#endif
#ifndef BNECK_NT_2B_C64
#define BNECK_NT_2B_C64 1
#endif
    constexpr bool NTO = (sizeof(T) == 4 && ((CI == 0 && ((C == 64 && BNECK_NT_F32_C64) || (C == 16 && BNECK_NT_F32_C16))) ||
                                             (CI != 0 && BNECK_NT_F32_DN))) ||
                         (sizeof(T) == 2 && CI == 0 && C == 64 && BNECK_NT_2B_C64);
#ifndef BNECK_AUX_F32_C128
#define BNECK_AUX_F32_C128 16
#endif
#ifndef BNECK_AUX_F32_LOW
#define BNECK_AUX_F32_LOW 0    // fp32 forms that take the default policy (C16, down C64): A/B knob
#endif
    constexpr int OAUX = OUT_AUX_SEL(NTO ? 2 : (sizeof(T) == 4 && C == 128) ? BNECK_AUX_F32_C128
                                     : (C >= 64 && CI != 16) ? 16 : sizeof(T) == 4 ? BNECK_AUX_F32_LOW : 0);
    static_assert(!DN || (!ASYM && !TR && !BShape<C, V>::RD && (CI == 16 || CI % 32 == 0)), "down mode: plain tiles");
    constexpr int G1 = DN ? CI / 2 : C / 8, KS1 = (G1 + 3) / 4;   // proj k groups / steps (down: 4 taps x CI)
    constexpr int CG1 = CI / 8;                       // down: 8-channel groups per tap
    constexpr int TAPS = ASYM ? 5 : 9;
    constexpr int G2 = TAPS * IS / 8, KS2 = (G2 + 3) / 4;
    constexpr int G3 = IS / 8;                        // expand k groups (<= 4: one step)
    constexpr bool RD = BShape<C, V>::RD;
    static_assert(!(RD && ASYM), "row-dilated tiles are for 3x3 blocks");
    constexpr int RY = ASYM ? 2 : 1;                  // halo rows / columns of the middle conv (tile coordinates)
    constexpr int RX = RD ? 0 : RY;                   // row-dilated tiles span the width: no column halo
    constexpr int HWW = TW + 2 * RX, HR = (TH + 2 * RY) * HWW;
    constexpr int NF1 = (HR + 15) / 16;               // 16-pixel fragments of tile + halo
    constexpr bool WIDE = BShape<C, V>::WIDE && !ASYM;
    constexpr int PADW = bneck_padw((int)sizeof(T), C, WIDE, CI > 0);   // weight-row pad (elements)
    constexpr bool PL = bneck_pl((int)sizeof(T), C, CI > 0) && !ASYM;  // fp32 C = 64: t0 as hi / lo planes
    constexpr int PSTR = PL ? 8 : bneck_pstr((int)sizeof(T), IS, WIDE);  // LDS pixel stride (elements; PL: per plane)
    constexpr int NPX = TH * TW;
    constexpr int NFT = (NPX + 15) / 16;              // 16-pixel fragments of the tile
    constexpr int NF2 = (NFT + NW - 1) / NW;          // ... per wave (the last may be partial / absent)
    constexpr int TWA = TW + 4;                       // asymmetric: width of t1a (the 1x5's halo)
    constexpr int NPA = TH * TWA;
    constexpr int NFA = (NPA + 15) / 16;
    constexpr int NF2A = (NFA + NW - 1) / NW;
#ifndef BNECK_CH1_K2
#define BNECK_CH1_K2 4   // down C64: 49.9 -> 49.4 us at 5 (one spill; round 2); round 4, with DKEEP: 4 spills none, 48.6-49.5 -> 47.4-47.9 us (its 6 fragments per wave take two round trips either way); 6 spills 22
#endif
// k-steps of the symmetric middle conv unrolled together: 3 for C = 128 (9 k-steps; no spills, its
// launches 1-4% faster), 1 elsewhere (down C64 6% slower at 3; 2 and 9 spill on C = 128).
// -DBNECK_PH2_UNROLL=N forces one factor everywhere (A/B builds).
#ifndef BNECK_PH2_UNROLL
#define BNECK_PH2_UNROLL 0
#endif
#ifndef BNECK_ASYM_UNROLL
#define BNECK_ASYM_UNROLL 1    // k-steps of the asymmetric 5x1 / 1x5 passes unrolled together (A/B knob)
#endif
#ifndef BNECK_REG3_C64
#define BNECK_REG3_C64 0
#endif
// fp32 (parity mode) C = 64 with the register epilogue: no staging region, so the LDS footprint is the
// halo's (8 x 16 tile: 42.7 -> 39.7 KB, 3 -> 4 workgroups per CU); its quads are 16-B chunks already.
// Measured slower (round 3: 94.1 -> 104.7 us per launch: a pixel's 256 B leave as four 64-B pieces)
// fp32 C = 64 (non-down) with the register epilogue AND whole-line stores (LINES below; round 6, A/B knob):
// the residual is loaded in the same line layout and traded back with the same DPP row rotation.
// Bit-identical (44 fp32 parity cases) but measured slower: 8 x 16 138.8 -> 147.5 us per 64-frame launch
// (124 VGPRs, no spills; the half-staged LDS epilogue, HSTG, stays)
#ifndef BNECK_F32_LINES64
#define BNECK_F32_LINES64 0
#endif
#ifndef BNECK_REG3_C64_F32
#define BNECK_REG3_C64_F32 0
#endif
// fp32 C = 64: the staged epilogue one 32-channel half at a time (HSTG below). Measured (round 3, fp32,
// B = 32): the 8 x 16 form 94.2 -> 89.4 us per launch (3 -> 4 workgroups per CU), fp32 bench
// 13,890 -> 14,065-14,095 frames/s; bit-identical (GPU-tested)
#ifndef BNECK_F32_HSTG
#define BNECK_F32_HSTG 1
#endif
#ifndef BNECK_CH1_C64
#define BNECK_CH1_C64 6   // the symmetric 16x16 C64 form: all of a wave's 5-6 phase-1 fragments in one round trip (37.3 -> 36.0 us)
#endif
#ifndef BNECK_CH1_K8
#define BNECK_CH1_K8 1
#endif
#ifndef BNECK_CH1_K8_F32
#define BNECK_CH1_K8_F32 1   // fp32 down C128 (the only KS1 >= 8 form): phase-1 fragments in flight (A/B knob; 2: 241 VGPRs, no spills, 115.5-117.0 -> 120.2-121.6 us, round 5)
#endif
    constexpr int CH1 = KS1 >= 8 ? (sizeof(T) == 4 ? BNECK_CH1_K8_F32 : BNECK_CH1_K8) : KS1 >= 4 ? (NF1 + NW - 1) / NW
                    : KS1 == 2 ? (C == 64 && V == 0 && !DN && !ASYM ? BNECK_CH1_C64 : BNECK_CH1_K2) : 8;   // phase-1 fragments whose loads fly together
    // phase-3 chunking (see phase 3): bf16 with an even number of 16-row blocks swaps row pairs
    // into 16-B chunks; bf16 C = 16 stores 8-B quads (HALF); fp32 quads are 16-B chunks
    // REG3: the register epilogue (C = 128 and 16). C = 64 keeps the LDS-staged epilogue: its 128-B
    // pixels would be written as half lines by the register layout, which measured slower there
    // (44.7 vs 43.0 us per launch with t1 in registers).
    // (the down form's C = 64 launch measured faster with the register epilogue: 53 vs 55 us)
    constexpr bool REG3 = C != 64 || DN || BNECK_REG3_C64 || (sizeof(T) == 4 && (BNECK_REG3_C64_F32 || BNECK_F32_LINES64));
    constexpr bool SWAP = REG3 && sizeof(T) == 2 && NR3 % 2 == 0;
    constexpr bool HALF = REG3 && sizeof(T) == 2 && NR3 % 2 != 0;
    constexpr int EPC = 16 / (int)sizeof(T);          // elements per 16-B chunk
    constexpr int CPP = C / EPC;                      // 16-B chunks per pixel
    constexpr int CPF = 16 * CPP;                     // (staged) 16-B chunks of one 16-pixel fragment
    constexpr int CPL = (CPF + 63) / 64;              // ... per lane
    // HSTG (fp32 C = 64, staged epilogue): the fragment is staged one 32-channel half at a time — a
    // pixel's half is 128 B, one whole line, so the stores stay full-line while the staging region
    // halves (the 8 x 16 tile: 42.7 -> 39.7 KB of LDS, 3 -> 4 workgroups per CU)
    constexpr bool HSTG = !REG3 && sizeof(T) == 4 && C == 64 && BNECK_F32_HSTG;
    constexpr int OSTR = (HSTG ? C / 2 : C) + EPC;    // staged epilogue: row stride (16-B padded)
    constexpr int RQ3 = !REG3 ? CPL : SWAP ? NR3 / 2 : NR3;   // residual chunks per lane per fragment
    static_assert(TW % 16 == 0, "a fragment is a run of one tile row");
#ifndef BNECK_NBE
#define BNECK_NBE -1     // border fragments loaded with the kept ones (-1: per form, see phase 1)
#endif
#ifndef BNECK_KEEP
#define BNECK_KEEP 1
#endif
    // KEEP: the residual is the block input phase 1 already loaded. Phase 1 then walks the tile's
    // interior as phase 3's fragments (a run of one tile row, on the wave that will expand it) and the
    // halo border separately, and each wave keeps its interior fragments' x in registers through
    // phase 2 instead of re-reading them (an L2 / Infinity-Cache round trip per fragment; PMC: the
    // C128 launches fetched 1.67x their compulsory bytes with the re-read). 2-byte storage, symmetric
    // plain blocks, with the staged (C = 64) or the row-pair-swapped (C = 128) epilogue.
#ifndef BNECK_GLDS
#define BNECK_GLDS 1
#endif
#ifndef BNECK_CONST_GLDS
#define BNECK_CONST_GLDS 1   // epilogue constants by LDS-DMA: 0 off, 1 for C != 128 (C64 38.0 -> 36.5 us; C128 23.1 -> 23.5), 2 all
#endif
#ifndef BNECK_GLDS_PARTIAL
#define BNECK_GLDS_PARTIAL 1   // KEEP: the first tile waits for the weights only, not for its x loads
#endif
    constexpr bool GLDS = BNECK_GLDS;                 // weights staged by global_load_lds (see the staging)
#ifndef BNECK_KEEP_ASYM
// the asymmetric form keeps its residual too (round 4: with the single-pass 5x1 it spills 3 VGPRs and
// runs 26.7 vs 26.5 us per launch re-reading, i.e. equal, for ~25 MB less HBM traffic per launch;
// round 3, before that rewrite, it had spilled more and run 26.2 -> 27.2 us)
#define BNECK_KEEP_ASYM 1
#endif
#ifndef BNECK_KEEP_C64
// C = 64, 2-byte: the residual kept (16 x 16 and 8 x 16 tiles; the 20 x 16 tile's five fragments per wave
// exceed the kept-register budget). Round 2 (B = 32, two streams) measured it slower: 41.0 vs 38.0 us per
// launch. Round 6 (B = 64, one stream): the 20 x 16 form re-reads its residual from HBM (PMC 228 MB read
// per launch, 1.45x the 157 MB compulsory) while 16 x 16 kept reads 160 MB (1.02x) in 70.9 vs 71.8 us —
// so it is on, and the tile picker charges the 20 x 16 form for its re-read (bugseg_runtime.cpp)
#define BNECK_KEEP_C64 1
#endif
#ifndef BNECK_KEEP_F32
#define BNECK_KEEP_F32 1
#endif
#ifndef BNECK_KEEP_F32_ASYM
#define BNECK_KEEP_F32_ASYM 1
#endif
    // KEEPF (round 4): the fp32 C = 128 forms keep their residual too. One workgroup per CU (LDS), so
    // 256 VGPRs per lane: the 96 of the kept x replace the 64 of the residual ring. A lane's k-step s
    // chunk holds channels 32 s + 8 kq .. + 7 as two quads; phase 3 wants quad 16 r + 4 kq .. + 3 of
    // row block r: a row swap then a half swap per dword gather rows 2 s and 2 s + 1 (as in bf16)
    constexpr bool KEEPF = BNECK_KEEP_F32 && !DN && sizeof(T) == 4 && (!ASYM || BNECK_KEEP_F32_ASYM) && C == 128 && REG3 && !SWAP;
    constexpr bool KEEP = (BNECK_KEEP && !DN && sizeof(T) == 2 && (!ASYM || BNECK_KEEP_ASYM) && (SWAP || !REG3) && (C != 64 || BNECK_KEEP_C64) &&
                           NF2 * KS1 * 4 <= (C == 128 ? 48 : 32)) || KEEPF;   // kept VGPRs within the occupancy budget
    static_assert(!KEEP || !REG3 || (KEEPF ? 2 * KS1 == RQ3 : KS1 == RQ3), "kept x: one 16-B chunk per k-step and row pair");
#ifndef BNECK_EARLY_FREE
#define BNECK_EARLY_FREE 0   // A/B knob, off: bit-identical (GPU parity green) but measured neutral to slower (round 5:
                             // fp32 C128 16x16 85.8-86.2 -> 86.7-87.0 us, fp16 frames/s -0.3%): a tile's critical
                             // path is its waves with the most fragments, whichever barrier the others wait at
#endif
    // EARLY_FREE (kept x, register epilogue): phase 3 touches no LDS but the read-only weights and
    // constants (t1 goes from the accumulators to B operands in registers), so the t0 region is free
    // once every wave has finished phase 2. The barrier that protects it moves from the top of the next
    // tile to the end of phase 2 (the first tile keeps its top barrier: the weight staging), and a wave
    // done with its stores starts the next tile's projection while the others are still storing
    constexpr bool EARLY_FREE = BNECK_EARLY_FREE && KEEP && REG3;
#ifndef BNECK_DKEEP
#define BNECK_DKEEP 1
#endif
    // DKEEP (down forms, 2-byte storage): phase 1 walks the tile as KEEP does and the main-branch pool
    // of each interior fragment stays in registers, already in the kept-x chunk layout (lane kq:
    // channels 32 t + 8 kq .. + 7), as phase 3's residual — instead of a global scratch round trip
    // (PMC: down C64 read + wrote 1.33x, down C128 1.36x their compulsory bytes with the scratch).
    // Measured (round 3, fp16, B = 32): down C64 52.9 -> 48.1 us, down C128 33.7 -> 28.7 us
    // fp32 (round 5): the same walk; a pooled chunk is 8 floats (two 16-B words) in the
    // kept-x layout of KEEPF, turned into phase 3's row quads by the same two lane swaps (PMC before: down
    // C64 1.27x, down C128 1.37x their compulsory bytes with the scratch round trip)
#ifndef BNECK_DKEEP_F32
#define BNECK_DKEEP_F32 1
#endif
    constexpr bool DKEEP = BNECK_DKEEP && DN && ((sizeof(T) == 2 && SWAP) || (sizeof(T) == 4 && BNECK_DKEEP_F32 && REG3));
    constexpr int NPK = DN ? (CI + 31) / 32 : 1;      // DKEEP: pooled chunks (32 channels of the row pair) per lane and fragment
    constexpr int PKW = sizeof(T) == 4 ? 2 : 1;       // 16-B words per pooled chunk
    // LINES (fp32 register epilogue, C = 128, round 6; on the fp32 down C64 form it cost 4 VGPRs and the third
    // wave per SIMD): an accumulator quad is 16 B (channels 16 r + 4 kq ..
    // + 3 of pixel col), so one store per row r writes 16 pixels x 64 B — half lines. With LINES the quads
    // of rows 2u and 2u + 1 of pixels col and col ^ 8 are traded across lanes 8 apart (one DPP row
    // rotation per dword) and each of the two stores per u writes the whole 128-B line u of 8 pixels.
    // Same values, other lanes: bit-identical (the fp32 up C64 block's form of this cut its HBM writes
    // 422 -> 315 MB and its time 129 -> 111 us per 64-frame launch)
#ifndef BNECK_F32_LINES
#define BNECK_F32_LINES 1
#endif
    constexpr bool LINES64 = BNECK_F32_LINES64 && sizeof(T) == 4 && REG3 && C == 64 && !DN && !KEEP;   // residual from the ring
    constexpr bool LINES = (BNECK_F32_LINES && sizeof(T) == 4 && REG3 && C == 128 && (KEEPF || (DKEEP && PKW == 2)) && RQ3 % 2 == 0) ||
                           LINES64;
    // FC >= 0 (round 6): ENet's class layer fused into its last bottleneck (C = 16, 16 x 16 tiles), FC =
    // the class map's LUT kind (cls_common.h cls_argmax). Tiles overlap by one row and one column (a
    // 15 x 15 stride): phase 3 leaves the block output of all 16 x 16 tile pixels in LDS (otile) instead
    // of HBM, and the class phase computes the transposed conv + argmax of the 15 x 15 pixels whose 2 x 2
    // input neighbourhood lies in the tile (the 16th row / column is the next tile's first). The block
    // output never reaches HBM: 2 x 315 MB (fp32, B = 64) less traffic, one launch less. Bit-identical class
    // maps (GPU-tested) but MEASURED SLOWER (round 6, B = 64, 480 x 640, one stream): fp32 424 us vs 162 + 116
    // us for the two launches, fp16 156 vs 97 + 45 — the class layer is not HBM-bound (0.37 of HBM alone), so
    // the bytes saved buy little, while the out tile and class weights in LDS (fp32 63.5 KB per workgroup:
    // 2 instead of 4 per CU) and the class phase's serial 32x32 MFMA chains behind a per-tile barrier cost
    // the bottleneck its latency hiding. Opt-in (BUGSEG_CLS_FUSE=1, bugseg_runtime.cpp Plan::cls_ok).
    constexpr bool CLS = FC >= 0;
    static_assert(!CLS || (C == 16 && !ASYM && !DN && !TR && REG3 && !KEEP && !SWAP && TH == 16 && TW == 16 && NW == 4),
                  "class fusion: the 16 x 16 C16 form");
    // otile pixel stride (elements): 80 B (fp32) / 48 B — 5 / 3 16-B units, so the 16-B reads of any 16
    // consecutive pixels fall in distinct bank groups
    constexpr int OPS = sizeof(T) == 4 ? 20 : 24;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // fp32 (parity mode): t0 / t1a live in LDS as split-f16 parts (mfma_common.h st4s: the weights'
    // layout, 32 B per 8 channels as the f32 values take), split once when written rather than at every
    // one of the middle conv's 9 (asymmetric: 5 + 5) operand reads. Bit-identical (the same parts).
    using SRaw = typename std::conditional<sizeof(T) == 4 && BNECK_F32_SPLIT_T0, RawS, Raw>::type;
    // HL (fp32 C = 128, round 5): in LDS a 32-element k-step of a split weight row, and a t0 / t1a pixel's
    // 32 channels, hold the four 8-channel groups' hi parts (16 B each) and then their lo parts, instead of
    // hi + lo per group — so each of a lane's two 16-B reads is 4 dwords at 4 kq dwords apart, as in bf16,
    // and rows of 8 / 40 dwords mod 64 make every ds_read_b128 lane group conflict-free (SQ: 41% of the
    // LDS cycles of these forms were bank conflicts with 32-B groups). The weight staging permutes the
    // 16-B chunks (the packed matrices in HBM keep the shared layout); the same parts feed the same products
    constexpr bool HL = bneck_hl((int)sizeof(T), C, CI > 0) && !(C == 64 && ASYM);   // (no C64 asymmetric block in ENet)
    static_assert(!HL || (BNECK_F32_SPLIT_T0 && (IS == 32 || (PL && IS == 16)) && BNECK_GLDS), "HL: split t0 of 32 channels (PL: 16), LDS-DMA staging");
    constexpr int PLO = PL ? HR * PSTR : 0;           // PL: the lo plane's offset from the hi plane (elements)
    constexpr int ZP = HL ? 32 : 16;                  // zero-pad elements below ts
    auto st4t = [](T *p, int ch, float4 v) {
        if constexpr (PL) {
            // p = plane pixel base + ch: hi parts of channels ch .. ch + 3 into the hi plane, lo into the lo plane
            const float e[4] = {v.x, v.y, v.z, v.w};
            _Float16 hh[4], ll[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                hh[i] = (_Float16)e[i];
                ll[i] = (_Float16)(e[i] - (float)hh[i]);
            }
            unsigned char *b = reinterpret_cast<unsigned char *>(reinterpret_cast<float *>(p) - ch) + (ch >> 3) * 16 + (ch & 7) * 2;
            *reinterpret_cast<f16x4 *>(b) = (f16x4){hh[0], hh[1], hh[2], hh[3]};
            *reinterpret_cast<f16x4 *>(b + PLO * 4) = (f16x4){ll[0], ll[1], ll[2], ll[3]};
        } else if constexpr (HL) st4hl(reinterpret_cast<float *>(p) - ch, ch, v);
        else if constexpr (sizeof(T) == 4 && BNECK_F32_SPLIT_T0) st4s(reinterpret_cast<float *>(p) - (ch & 7), ch & 7, v);
        else st4(p, v);
    };

    span_enter(a.span);
    STAMP_ENTRY(0);
    // a workgroup without a tile leaves before staging anything (an LDS-DMA still in flight when
    // its wave ends would land in LDS the next workgroup on the CU already owns)
    {
        const int ch = (a.ntiles + 7) >> 3, sl = (int)(blockIdx.x >> 3);
        if (sl >= ch || (int)(blockIdx.x & 7) * ch + sl >= a.ntiles) return true;   // (the tile walk's first tile)
    }
    const int tid = threadIdx.x;
    const int lane = tid & 63, col = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably uniform: scalar fragment math
    // first channel of this lane's phase-3 chunk t
    auto chunk_ch = [&](int t) -> int { return SWAP ? (2 * t + (kq & 1)) * 16 + 8 * (kq >> 1) : t * 16 + kq * 4; };
    const int K1S = KS1 * 32 + PADW, K2S = KS2 * 32 + PADW, K3S = 32 + PADW;
    // A operand: group kq of the k-step at p (a weight row + 32 s)
    auto ldw = [&](WRaw &r, const T *p) {
        if constexpr (HL) {
            r.h = *reinterpret_cast<const uint4 *>(p + kq * 4);
            r.l = *reinterpret_cast<const uint4 *>(p + 16 + kq * 4);
        } else {
            ld8(r, p + kq * 8);
        }
    };
    T *w1 = reinterpret_cast<T *>(smem);
    T *w2 = w1 + NR1 * 16 * K1S;
    T *w2b = w2 + NR1 * 16 * K2S;                     // asymmetric second conv (1x5)
    T *w3 = w2b + (ASYM ? NR1 * 16 * K2S : 0);
    // per-channel epilogue constants live in LDS too: a global load per use was most of this
    // kernel's vector-memory instructions and a latency the epilogues waited on
    constexpr int NP1 = NR1 * 16;
    float *cb1 = reinterpret_cast<float *>(w3 + C * K3S), *cs1 = cb1 + NP1, *cb2 = cs1 + NP1, *cs2 = cb2 + NP1;
    float *cb2b = cs2 + NP1, *cs2b = cb2b + NP1, *cb3 = cs2b + NP1, *cs3 = cb3 + C, *cso = cs3 + C;
    // 16 zero elements: masked-off B fragments read them (an address select, not a divergent branch)
    T *zpad = reinterpret_cast<T *>(cso + C);
    T *ts = zpad + ZP;                                // t0 / t1a / t1 region
    float *wmx = reinterpret_cast<float *>(ts + HR * PSTR);   // fp32 asymmetric: NW per-wave max |t1a| slots
    // CLS: the tile's block output, the class weights as [8 (block, tap)][64 lanes] 16-B slots (fp32: the
    // hi parts, then a plane of the lo parts), the class bias (64 rows), per-wave tile maxima (fp32)
    T *otile = ts + HR * PSTR;
    uint4 *cwl = reinterpret_cast<uint4 *>(otile + (CLS ? NPX * OPS : 0));
    float *cbl = reinterpret_cast<float *>(cwl + (CLS ? (sizeof(T) == 4 ? 1024 : 512) : 0));
    float *cmx = cbl + 64;
    {
        // C = 16 (small weights, many short tiles): every load of the staging is issued before the
        // first LDS store (one L2 round trip at kernel start instead of one per 16-B chunk a thread
        // copies). Measured slower for C = 64 / 128 (48.8 / 31.8 vs 42 / 26.4 us: all workgroups
        // requesting every weight line at once), so those keep the chunk loop below.
        constexpr int CPR1 = KS1 * 32 * (int)sizeof(T) / 16, CPR2 = KS2 * 32 * (int)sizeof(T) / 16, CPR3 = 32 * (int)sizeof(T) / 16;
        constexpr int N1 = NR1 * 16 * CPR1, N2 = NR1 * 16 * CPR2, N3 = C * CPR3;
        constexpr int TOT = N1 + N2 * (ASYM ? 2 : 1) + N3;
        constexpr int PER = (TOT + NT - 1) / NT;
        uint4 buf[C == 16 ? PER : 1];
        auto locate = [&](int i, const uint4 *&src, unsigned char *&dst) -> bool {
            int r, c;
            if (i < N1) { r = i / CPR1; c = i - r * CPR1; src = (const uint4 *)a.w1 + i; dst = (unsigned char *)(w1 + r * K1S) + c * 16; return true; }
            i -= N1;
            if (i < N2) { r = i / CPR2; c = i - r * CPR2; src = (const uint4 *)a.w2 + i; dst = (unsigned char *)(w2 + r * K2S) + c * 16; return true; }
            i -= N2;
            if (ASYM && i < N2) { r = i / CPR2; c = i - r * CPR2; src = (const uint4 *)a.w2b + i; dst = (unsigned char *)(w2b + r * K2S) + c * 16; return true; }
            if (ASYM) i -= N2;
            if (i < N3) { r = i / CPR3; c = i - r * CPR3; src = (const uint4 *)a.w3 + i; dst = (unsigned char *)(w3 + r * K3S) + c * 16; return true; }
            return false;
        };
        if constexpr (GLDS) {
            // global_load_lds: the weight region of LDS is a run of 16-B slots (rows of K?S elements:
            // CPR? data chunks + the pad); each wave instruction fills 64 consecutive slots, a lane
            // fetching its slot's chunk (pad slots re-read the row's first chunk: never read). No
            // VGPR round trip and nothing waited for here: the loads fly with the first tile's x
            // loads and the first tile waits for all of them before its first barrier.
            (void)buf;
            constexpr int ES = (int)sizeof(T);
            constexpr int SR1 = (KS1 * 32 + PADW) * ES / 16, SR2 = (KS2 * 32 + PADW) * ES / 16, SR3 = (32 + PADW) * ES / 16;
            constexpr int S1 = NR1 * 16 * SR1, S2 = NR1 * 16 * SR2, S3 = C * SR3;
            constexpr int NSL = S1 + S2 * (ASYM ? 2 : 1) + S3;
            static_assert((KS1 * 32 + PADW) * ES % 16 == 0 && (KS2 * 32 + PADW) * ES % 16 == 0 && (32 + PADW) * ES % 16 == 0,
                          "weight rows are whole 16-B slots");
            for (int base = wave * 64; base < NSL; base += NT) {      // wave-uniform
                const int q = base + lane;
                const uint4 *src;
                auto pick = [&](const void *w, int k, int SR, int CPR) {   // slot k of one matrix
                    const int r = k / SR, c = k - r * SR;
                    // HL: LDS chunk d of each 8-chunk k-step is hi (d < 4) / lo part of group d % 4, packed
                    // chunk 2 (d % 4) + (d >= 4)
                    const int cs = HL ? (c & ~7) | ((c & 7) < 4 ? 2 * (c & 7) : 2 * (c & 3) + 1) : c;
                    src = (const uint4 *)w + r * CPR + (c < CPR ? cs : 0);
                };
                constexpr int O3 = S1 + S2 * (ASYM ? 2 : 1);   // first slot of w3
                if (q < S1) pick(a.w1, q, SR1, CPR1);
                else if (q < S1 + S2) pick(a.w2, q - S1, SR2, CPR2);
                else if (q < O3) pick(a.w2b, q - S1 - S2, SR2, CPR2);
                else pick(a.w3, q - O3, SR3, CPR3);
                if (base + lane < NSL)
                    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                                     (__attribute__((address_space(3))) void *)(smem + (size_t)base * 16), 16, 0, 0);
            }
        } else if constexpr (C == 16) {
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const uint4 *src;
                unsigned char *dst;
                if (locate(tid + k * NT, src, dst)) buf[k] = *src;
            }
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const uint4 *src;
                unsigned char *dst;
                if (locate(tid + k * NT, src, dst)) *reinterpret_cast<uint4 *>(dst) = buf[k];
            }
        } else {
            (void)buf;
            for (int i = tid; i < TOT; i += NT) {
                const uint4 *src;
                unsigned char *dst;
                if (locate(i, src, dst)) *reinterpret_cast<uint4 *>(dst) = *src;
            }
        }
        if constexpr (GLDS && (BNECK_CONST_GLDS == 2 || (BNECK_CONST_GLDS == 1 && C != 128))) {
            // the epilogue constants by LDS-DMA as well (one dword per lane, 64 per instruction,
            // spread over the waves): a plain load -> LDS store here would wait (vmcnt, in order)
            // for the weight DMA issued above and serialise the staging ahead of the x loads
            const float *srcs[9] = {a.b1, a.s1, a.b2, a.s2, a.b2b, a.s2b, a.b3, a.s3, a.s_out};
            float *dsts[9] = {cb1, cs1, cb2, cs2, cb2b, cs2b, cb3, cs3, cso};
            int item = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                if (!ASYM && (k == 4 || k == 5)) continue;          // unused without the 1x5 pass
                const int n = k < 6 ? NP1 : C;
#pragma unroll
                for (int c0 = 0; c0 < n; c0 += 64, ++item) {
                    if (item % NW != wave) continue;                // wave-uniform
                    if (c0 + lane < n)
                        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(srcs[k] + c0 + lane),
                                                         (__attribute__((address_space(3))) void *)(dsts[k] + c0), 4, 0, 0);
                }
            }
        } else {
            for (int i = tid; i < NP1; i += NT) {
                cb1[i] = a.b1[i]; cs1[i] = a.s1[i]; cb2[i] = a.b2[i]; cs2[i] = a.s2[i];
                cb2b[i] = ASYM ? a.b2b[i] : 0.f; cs2b[i] = ASYM ? a.s2b[i] : 0.f;
            }
            for (int i = tid; i < C; i += NT) { cb3[i] = a.b3[i]; cs3[i] = a.s3[i]; cso[i] = a.s_out[i]; }
        }
        if (tid < ZP) zpad[tid] = (T)0.f;
    }
    // CLS: the class layer's weights (packed [64][64]: row = phase * 16 + class, k = tap * 16 + channel) into
    // the lane slots its MFMAs read, its bias (padding classes at -inf: never the maximum), the LUT, and
    // which blocks skip the dy = 1 taps (all-zero weights: output row 2y never sees input row y + 1) —
    // the class kernel's rules (cls_kernels.hip), decided the same way
    using CRaw = typename WTr<T>::Raw;
    uint64_t lut64 = 0;
    bool cshort[2] = {false, false};
    if constexpr (CLS) {
        const T *cw = reinterpret_cast<const T *>(a.cw);
        for (int q = tid; q < 512; q += NT) {
            const int bs = q >> 6, ln = q & 63;
            const T *src = cw + (size_t)cls_prow(bs >> 2, ln & 31) * 64 + (bs & 3) * 16 + 8 * (ln >> 5);
            if constexpr (sizeof(T) == 4) {
                cwl[q] = reinterpret_cast<const uint4 *>(src)[0];
                cwl[512 + q] = reinterpret_cast<const uint4 *>(src)[1];
            } else {
                cwl[q] = *reinterpret_cast<const uint4 *>(src);
            }
        }
        if (tid < 64) cbl[tid] = (tid & 15) < a.ncls ? a.cbias[tid] : -INFINITY;
        lut64 = cls_lut64(a.lut);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            CRaw w2_, w3_;
            const T *r = cw + (size_t)cls_prow(b, lane & 31) * 64 + 8 * (lane >> 5);
            ld8(w2_, r + 32);
            ld8(w3_, r + 48);
            cshort[b] = __ballot(nonzero(w2_) || nonzero(w3_)) == 0;
        }
    }
    // x / out through buffer descriptors: 32-bit offsets, and an out-of-range offset reads 0 / drops
    // the store (mfma_common.h), so image-border masking costs one select per access
    // down mode: x is the (2H, 2W, CI) block input; the residual comes from the pooled scratch
    const auto rxb = mkbuf(DN ? a.xin : a.x, DN ? a.xin_bytes : a.x_bytes);
    const auto rob = mkbuf(a.out, a.x_bytes);
    const auto rpb = mkbuf(a.pool, a.pool_bytes);
    const auto rib = mkbuf(a.idx_out, a.idx_bytes);
    // the fused path is planned only when every slope is <= 1 (bugseg_runtime.cpp fusable_regular),
    // so PReLU is max(v, s*v); accumulators start at the bias
    auto act = [&](float4 v, const float *s) { return prelu4m(v, ld4f(s)); };
    const int dt = a.dt;                              // tiling dilation (1 for asymmetric blocks)
    constexpr bool tr = TR && !ASYM;                  // transposed tile

    constexpr bool F32 = sizeof(T) == 4;
    BneckRange rg0;                                   // SCL = false: every exponent 0 (checked at the first tile)
    if constexpr (F32 && SCL) rg0 = bneck_range<ASYM>(a.rg, rng_reduce(rlane));
    bool scl = rg0.scl;
    float xm = rg0.xm, b1m = rg0.b1m, o1m = rg0.o1m, b2m = rg0.b2m, o2m = rg0.o2m, b2bm = rg0.b2bm, o2bm = rg0.o2bm;
    float b3m = rg0.b3m, o3m = rg0.o3m;
    const int rs1 = rg0.rs1, re2b = rg0.re2b;
    float amo = 0.f;                                  // max |out| of this lane's stores
    // the projection of one fragment (SCL: operands and accumulators scaled)
    auto proj_mfma = [&](f32x4 (&acc)[NR1], const Raw (&xs)[KS1]) {
#pragma unroll
        for (int r = 0; r < NR1; ++r) acc[r] = bias4(cb1 + r * 16 + kq * 4);
        if constexpr (F32 && SCL) {
#pragma unroll
            for (int r = 0; r < NR1; ++r) acc[r] = mul4(acc[r], b1m);
#pragma unroll
            for (int s = 0; s < KS1; ++s) {
                const RawF xq = scale8(reinterpret_cast<const RawF &>(xs[s]), xm);
#pragma unroll
                for (int r = 0; r < NR1; ++r) {
                    WRaw wf;
                    ldw(wf, w1 + (r * 16 + col) * K1S + s * 32);
                    mma(acc[r], wf, xq);
                }
            }
#pragma unroll
            for (int r = 0; r < NR1; ++r) acc[r] = mul4(acc[r], o1m);
        } else {
#pragma unroll
            for (int s = 0; s < KS1; ++s)
#pragma unroll
                for (int r = 0; r < NR1; ++r) {
                    WRaw wf;
                    ldw(wf, w1 + (r * 16 + col) * K1S + s * 32);
                    mma(acc[r], wf, xs[s]);
                }
        }
    };

    // XCD-aware tile walk (see conv_kernels.hip): each XCD takes a contiguous run of tiles, so the
    // halo re-reads of neighbouring tiles hit the same L2
    const int G = gridDim.x, grp = blockIdx.x & 7, slot = blockIdx.x >> 3, nslots = G >> 3;
    const int CH = (a.ntiles + 7) >> 3;
    // tile -> frame n and image pixel (oy0, ox0) of tile pixel (0, 0): phase (py, px), tile row /
    // column of that phase's sub-image (scalar math). Tile pixel (i, j) is image (oy0 + dt i, ox0 +
    // dt j), or (oy0 + dt j, ox0 + dt i) transposed
    auto tile_geom = [&](int tile, int &n, int &oy0, int &ox0) {
        int t = tile;
        const int txi = t % a.tiles_x; t /= a.tiles_x;
        const int tyi = t % a.tiles_y; t /= a.tiles_y;
        const int ph = t % a.phases;
        n = t / a.phases;
        const int py = RD ? ph : ph / dt, px = RD ? 0 : ph - py * dt;   // RD: phases = row phases
        oy0 = py + dt * tyi * (tr ? TW : TH) - (CLS ? tyi : 0);    // (CLS: tiles 15 apart)
        ox0 = RD ? 0 : px + dt * txi * (tr ? TH : TW) - (CLS ? txi : 0);
    };
    Raw kx[KEEP ? NF2 : 1][KS1];                      // KEEP: this wave's interior fragments of x
    bool kok[KEEP ? NF2 : 1];
    // PREF (KEEP, register epilogue; A/B knob, off): as phase 3 finishes with a fragment's kept x, the
    // same registers receive that fragment's x of the workgroup's NEXT tile, so its loads fly during the
    // rest of this tile's phase 3. Measured slower (round 5, B = 64: fp32 C128 20x16 90.9 -> 100.6 us,
    // fp16 33.4 -> 34.4 us; the loads contend with phase 3's stores and cost the fp16 form 5 spilled VGPRs)
#ifndef BNECK_PREF
#define BNECK_PREF 0
#endif
    constexpr bool PREF = BNECK_PREF && KEEP && REG3 && !DN;
    bool pref = false;                                // this tile's kx already loaded (prefetched)
    for (int it = slot; it < CH; it += nslots) {
        const int tile = grp * CH + it;
        if (tile >= a.ntiles) break;
        int n, oy0, ox0;
        tile_geom(tile, n, oy0, ox0);
        float tmo = 0.f;                              // CLS, fp32: this lane's max |out| over the tile
        // the next tile of this workgroup's walk (PREF)
        const int ntile = grp * CH + it + nslots;
        const bool has_next = PREF && it + nslots < CH && ntile < a.ntiles;
        int nn = 0, noy0 = 0, nox0 = 0;
        if (has_next) tile_geom(ntile, nn, noy0, nox0);
        const int dtx = RD ? 1 : dt;                  // column step of the tile
        const uint32_t xn = (uint32_t)(n * a.H * a.W) * (uint32_t)(C * sizeof(T));   // frame byte offset
        const uint32_t xin_n = (uint32_t)(n * 4 * a.H * a.W) * (uint32_t)(CI * sizeof(T));   // down: input frame
        // byte offset of channel chunk `choff` of pixel pi (per lane, 0..15) of tile fragment f (wave
        // uniform), or OOB outside the image. A fragment is a run of one tile row: its row i is a
        // scalar and only the column j is per lane.
        auto pix_off = [&](int f, int pi, int choff) -> uint32_t {
            const int i = (f * 16) / TW, j = (f * 16) % TW + pi;
            const int y = oy0 + dt * (tr ? j : i), x = ox0 + dtx * (tr ? i : j);
            const bool ok = y < a.H && x < a.W;
            // 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate): coordinates < 2^24. The
            // offset is computed for every lane and pinned, so the mask is a select, not a divergent
            // branch around the arithmetic
            uint32_t v = xn + ((__umul24((uint32_t)y, (uint32_t)a.W) + (uint32_t)x) * C + choff) * (uint32_t)sizeof(T);
            asm volatile("" : "+v"(v));
            return ok ? v : OOB;
        };
        // byte offset of pixel pi of fragment f (channel 0), or OOB outside the image
        auto pix_base = [&](int f, int pi) -> uint32_t { return pix_off(f, pi, 0); };
        // residual source: x itself, or (down) the pooled scratch (CI channels; channels >= CI read 0)
        const auto rrb = DN ? rpb : rxb;
        const uint32_t pn = (uint32_t)(n * a.H * a.W) * (uint32_t)(CI * sizeof(T));
        auto res_off = [&](int f, int pi, int ch) -> uint32_t {
            if constexpr (!DN) {
                return pix_off(f, pi, ch);
            } else {
                const int i = (f * 16) / TW, j = (f * 16) % TW + pi;
                const int y = oy0 + dt * i, x = ox0 + dtx * j;
                const bool ok = y < a.H && x < a.W && ch < CI;
                uint32_t v = pn + ((__umul24((uint32_t)y, (uint32_t)a.W) + (uint32_t)x) * CI + ch) * (uint32_t)sizeof(T);
                asm volatile("" : "+v"(v));
                return ok ? v : OOB;
            }
        };
        // down: main-branch maxpool of output pixel (y, x) from the projection's B fragments (see the
        // kernel comment); the first maximum in window order wins (strict >, NaN / -inf never chosen:
        // as a key, larger value first, then lower window position; position 4 = no candidate -> 0)
        auto pool_store = [&](const Raw (&xs)[KS1], bool interior, int y, int x, uint4 (&pk)[NPK * PKW]) {
            if constexpr (DN) {
                if (__ballot(interior) == 0) return;          // halo-only fragment (wave-uniform)
                auto elems = [&](const Raw &r, float (&e)[8]) {
                    if constexpr (sizeof(T) == 2) {
                        const float4 lo = unpack4<T>((u32x2_t){r.v.x, r.v.y}), hi = unpack4<T>((u32x2_t){r.v.z, r.v.w});
                        e[0] = lo.x; e[1] = lo.y; e[2] = lo.z; e[3] = lo.w; e[4] = hi.x; e[5] = hi.y; e[6] = hi.z; e[7] = hi.w;
                    } else {
                        const RawF &f = reinterpret_cast<const RawF &>(r);
                        e[0] = f.a.x; e[1] = f.a.y; e[2] = f.a.z; e[3] = f.a.w; e[4] = f.b.x; e[5] = f.b.y; e[6] = f.b.z; e[7] = f.b.w;
                    }
                };
                const uint32_t pix = (uint32_t)((n * a.H + y) * a.W + x);
                auto emit = [&](int cc, const float (&bv)[8], const int (&bp)[8], bool wr, int kslot, bool kval) {
                    // 8 pooled channels (exact input values) + their window positions (4 = none -> 0)
                    uint32_t pw[8 * sizeof(T) / 4];
                    if constexpr (sizeof(T) == 2) {
                        // exact input values (the pool selects, it does not round): re-packing is lossless
                        const u32x2_t lo = pack4<T>(make_float4(bv[0], bv[1], bv[2], bv[3]));
                        const u32x2_t hi = pack4<T>(make_float4(bv[4], bv[5], bv[6], bv[7]));
                        pw[0] = lo.x; pw[1] = lo.y; pw[2] = hi.x; pw[3] = hi.y;
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) pw[i] = __float_as_uint(bv[i]);
                    }
                    uint32_t lo = 0, hi = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        lo |= (uint32_t)(bp[i] & 3) << (8 * i);
                        hi |= (uint32_t)(bp[4 + i] & 3) << (8 * i);
                    }
                    if constexpr (DKEEP) {
                        pk[kslot * PKW] = kval ? make_uint4(pw[0], pw[1], pw[2], pw[3]) : make_uint4(0u, 0u, 0u, 0u);
                        if constexpr (PKW == 2)
                            pk[kslot * PKW + 1] = kval ? make_uint4(pw[4], pw[5], pw[6], pw[7]) : make_uint4(0u, 0u, 0u, 0u);
                    } else {
                        (void)kslot; (void)kval;
                        const uint32_t po = wr ? (pix * CI + cc * 8) * (uint32_t)sizeof(T) : OOB;
#pragma unroll
                        for (int i = 0; i < (int)(8 * sizeof(T) / 16); ++i)
                            bst16(rpb, po == OOB ? OOB : po + 16 * i, make_uint4(pw[4 * i], pw[4 * i + 1], pw[4 * i + 2], pw[4 * i + 3]));
                    }
                    __builtin_amdgcn_raw_buffer_store_b64((u32x2_t){lo, hi}, rib, wr ? (int)(pix * a.idxCS + cc * 8) : (int)OOB, 0, 0);
                };
                // in window order: strict > from -inf (NaN and -inf never taken), position 4 = none
                auto seq = [](float &bv, int &bp, float v, int p) {
                    const bool t = v > bv;
                    bv = t ? v : bv;
                    bp = t ? p : bp;
                };
                if constexpr (CG1 >= 4) {
                    // k step s holds tap s / (CG1 / 4) of channel group (s % (CG1 / 4)) * 4 + kq
#pragma unroll
                    for (int hgrp = 0; hgrp < CG1 / 4; ++hgrp) {
                        float bv[8], e[8];
                        int bp[8];
#pragma unroll
                        for (int i = 0; i < 8; ++i) { bv[i] = -INFINITY; bp[i] = 4; }
#pragma unroll
                        for (int tap = 0; tap < 4; ++tap) {
                            elems(xs[tap * (CG1 / 4) + hgrp], e);
#pragma unroll
                            for (int i = 0; i < 8; ++i) seq(bv[i], bp[i], e[i], tap);
                        }
                        emit(hgrp * 4 + kq, bv, bp, interior, hgrp, true);
                    }
                } else {
                    // CI = 16: step s holds dy = s, dx = kq >> 1, group kq & 1; the dx = 1 half of the
                    // wave (lanes 32-63) is traded in with v_permlane32_swap and merged as a key
                    // (larger value, then lower position)
                    float bv[8], e[8];
                    int bp[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) { bv[i] = -INFINITY; bp[i] = 4; }
                    const int dx = kq >> 1;
#pragma unroll
                    for (int dy = 0; dy < 2; ++dy) {
                        elems(xs[dy], e);
#pragma unroll
                        for (int i = 0; i < 8; ++i) seq(bv[i], bp[i], e[i], dy * 2 + dx);
                    }
                    const bool lo_half = kq < 2;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        uint32_t v0 = __float_as_uint(bv[i]), v1 = v0, p0 = (uint32_t)bp[i], p1 = p0;
                        pl32swap(v0, v1);
                        pl32swap(p0, p1);
                        const float pv = __uint_as_float(lo_half ? v1 : v0);
                        const int pp = (int)(lo_half ? p1 : p0);
                        const bool t = pv > bv[i] || (pv == bv[i] && pp < bp[i]);
                        bv[i] = t ? pv : bv[i];
                        bp[i] = t ? pp : bp[i];
                    }
                    // both halves now agree; lanes 0-31 (groups kq = 0, 1) write
                    emit(kq & 1, bv, bp, interior && lo_half, 0, lo_half);   // (DKEEP: channels 16-31 are 0)
                }
            }
        };
        STAMP(0); STAMP_WG();
        // the first tile waits for the glds weight staging (each wave its own loads, then the
        // barrier makes every wave's visible); KEEP issues its x loads ahead of that wait
        const bool first = it == slot;
        if constexpr (!KEEP) {
            if (GLDS && first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();   // weights staged (first tile) / previous tile done with ts (and the patch)
            if constexpr (F32 && !SCL) {
                // the range words arrived with the loads issued before them: bail out to the scaled body
                if (first && bneck_range<ASYM>(a.rg, rng_reduce(rlane)).any) {
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                    __syncthreads();
                    return false;
                }
            }
        }
        STAMP(1);

        // ---- phase 1: t0 = act1(W1 x + b1) over tile + halo, 0 outside the image. The loads of CH1
        // fragments are issued together before any of them is consumed (memory-level parallelism).
        // halo index of pixel pi of interior fragment f (tile pixel (i, j) = halo (i + RY, j + RX))
        auto int_h = [&](int f) -> int {
            const int p = f * 16 + col, i = p / TW, j = p - i * TW;
            return (i + RY) * HWW + j + RX;
        };
        // loads of halo pixel h of the tile at (ty0, tx0) in frame byte offset txn (KS1 16-B chunks)
        auto load_hg = [&](int ty0, int tx0, uint32_t txn, int h, bool valid, Raw (&xs)[KS1]) -> bool {
            const int hy = h / HWW, hx = h - hy * HWW;
            const int iy = ty0 + dt * ((tr ? hx : hy) - RY), ix = tx0 + dtx * ((tr ? hy : hx) - RX);
            const bool ok = valid && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
#pragma unroll
            for (int s = 0; s < KS1; ++s) {
                const int g = s * 4 + kq;
                bld8(xs[s], rxb, ok && g < G1 ? txn + ((__umul24((uint32_t)iy, (uint32_t)a.W) + (uint32_t)ix) * C + g * 8) * (uint32_t)sizeof(T) : OOB);
            }
            return ok;
        };
        // KEEP / DKEEP walk: the tile's interior as phase 3's fragments (a run of one tile row, on the
        // wave that will expand it), then the halo border
        constexpr int NBD = HR - NPX, NFB = (NBD + 15) / 16;   // border pixels / fragments
        constexpr int NBW = (NFB + NW - 1) / NW;      // border fragments per wave (at most)
        constexpr int B0 = NFT % NW;                  // border fragment k runs on wave (B0 + k) % NW
        const int wb = wave >= B0 ? wave - B0 : wave - B0 + NW;   // this wave's first border fragment
        // halo index of border pixel b: the RY top and bottom halo rows, then the RX columns either
        // side of the TH interior rows
        auto bord_h = [&](int b) -> int {
            if (b < 2 * RY * HWW) {
                const int r = b / HWW, c = b - r * HWW;
                return (r < RY ? r : TH + r) * HWW + c;
            }
            if constexpr (RX > 0) {
                const int bb = b - 2 * RY * HWW, r = bb / (2 * RX), c = bb - r * (2 * RX);
                return (RY + r) * HWW + (c < RX ? c : TW + c);
            }
            return 0;
        };
        auto proj = [&](int h, bool valid, bool ok, const Raw (&xs)[KS1]) {
            f32x4 acc[NR1];
            proj_mfma(acc, xs);
            if (valid) {
#pragma unroll
                for (int r = 0; r < NR1; ++r) {
                    const int ch = r * 16 + kq * 4;
                    if (ch >= IS) continue;
                    float4 v = act(f4(acc[r]), cs1 + ch);
                    if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
                    st4t(ts + h * PSTR + ch, ch, v);
                }
            }
        };
        uint4 pres[DKEEP ? NF2 : 1][NPK * PKW];       // DKEEP: pooled residual of the interior fragments
        if constexpr (KEEP) {
            // every load of the wave's phase-1 work (its interior fragments, kept, and its share of
            // the border) is issued before the first MFMA: one memory round trip per tile
            auto load_h = [&](int h, bool valid, Raw (&xs)[KS1]) -> bool { return load_hg(oy0, ox0, xn, h, valid, xs); };
            Raw bx[NBW][KS1];
            int bh[NBW];
            bool bok[NBW];
            if (!pref) {
#pragma unroll
                for (int j = 0; j < NF2; ++j)
                    if (wave + NW * j < NFT) kok[j] = load_h(int_h(wave + NW * j), true, kx[j]);   // wave-uniform
            }
            auto load_b = [&](int k) {
                const int b = (wb + NW * k) * 16 + col;
                bh[k] = b < NBD ? bord_h(b) : 0;
                bok[k] = load_h(bh[k], b < NBD, bx[k]);
            };
            // the first NBE border fragments fly with the interior ones; any further ones (a wave
            // with two) are loaded after, which keeps the x registers within the occupancy budget
            // (C = 64 / 4x80: spills at 1; fp32 C128: 0 measured 1-4 us per 64-frame launch faster, round 5)
            constexpr int NBE = BNECK_NBE >= 0 ? BNECK_NBE : C == 128 && !RD && !ASYM && sizeof(T) == 2 ? 1 : 0;
#pragma unroll
            for (int k = 0; k < NBE && k < NBW; ++k)
                if (wb + NW * k < NFB) load_b(k);     // wave-uniform
            // (x loads touch no LDS, so they go ahead of the barrier that frees ts). The first tile
            // waits for the weight LDS-DMA only: it was issued before this wave's x loads, and vmcnt
            // retires in order, so "at most nld outstanding" leaves the x loads in flight for the
            // projections to consume one fragment at a time
            if (GLDS && first) {
                int nld = 0;
                constexpr int LPS = sizeof(T) == 4 ? 2 : 1;   // 16-B loads per k-step chunk (fp32: two)
#pragma unroll
                for (int j = 0; j < NF2; ++j) nld += wave + NW * j < NFT ? KS1 * LPS : 0;
#pragma unroll
                for (int k = 0; k < NBE && k < NBW; ++k) nld += wb + NW * k < NFB ? KS1 * LPS : 0;
                vm_wait_upto(BNECK_GLDS_PARTIAL ? (nld < 24 ? nld & ~1 : 24) : 0);   // (fewer outstanding: still after the weights)
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (!EARLY_FREE || first) __builtin_amdgcn_s_barrier();   // weights staged (first tile) / previous tile done with ts
            asm volatile("" ::: "memory");
            if constexpr (F32 && !SCL) {
                // the range words arrived with the loads issued before them: bail out to the scaled body
                if (first && bneck_range<ASYM>(a.rg, rng_reduce(rlane)).any) {
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                    __syncthreads();
                    return false;
                }
            }
#pragma unroll
            for (int j = 0; j < NF2; ++j)
                if (wave + NW * j < NFT) proj(int_h(wave + NW * j), true, kok[j], kx[j]);
#pragma unroll
            for (int k = 0; k < NBW; ++k) {
                const int fb = wb + NW * k;
                if (fb >= NFB) break;
                if (k >= NBE) load_b(k);
                proj(bh[k], fb * 16 + col < NBD, bok[k], bx[k]);
            }
        } else if constexpr (DKEEP) {
            // down forms: the wave's interior fragments, then its border share, CH1 fragments' loads in
            // flight at a time (the 2x2 stride-2 taps of the block input)
            constexpr int NQ = NF2 + NBW;
            auto load_dn = [&](int h, bool valid, Raw (&xs)[KS1]) -> bool {
                const int hy = h / HWW, hx = h - hy * HWW;
                const int iy = oy0 + hy - 1, ix = ox0 + hx - 1;
                const bool ok = valid && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
#pragma unroll
                for (int s = 0; s < KS1; ++s) {
                    const int g = s * 4 + kq;
                    const int tap = g / CG1, cc = g - tap * CG1;   // pack_conv's K order: dy = tap >> 1, dx = tap & 1
                    const uint32_t sy = (uint32_t)(2 * iy + (tap >> 1)), sx = (uint32_t)(2 * ix + (tap & 1));
                    uint32_t v = xin_n + ((__umul24(sy, (uint32_t)(2 * a.W)) + sx) * CI + cc * 8) * (uint32_t)sizeof(T);
                    asm volatile("" : "+v"(v));
                    bld8(xs[s], rxb, ok && g < G1 ? v : OOB);
                }
                return ok;
            };
#pragma unroll
            for (int j = 0; j < NF2; ++j)
#pragma unroll
                for (int k = 0; k < NPK * PKW; ++k) pres[j][k] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int q0 = 0; q0 < NQ; q0 += CH1) {
                Raw xf[CH1][KS1];
                bool okc[CH1], vq[CH1];
                int hq[CH1];
#pragma unroll
                for (int c = 0; c < CH1; ++c) {
                    const int q = q0 + c;
                    if (q >= NQ) break;
                    if (q < NF2) {
                        const int f = wave + NW * q;
                        vq[c] = f < NFT;
                        hq[c] = vq[c] ? int_h(f) : 0;
                    } else {
                        const int b = (wb + NW * (q - NF2)) * 16 + col;
                        vq[c] = b < NBD;
                        hq[c] = vq[c] ? bord_h(b) : 0;
                    }
                    okc[c] = load_dn(hq[c], vq[c], xf[c]);
                }
#pragma unroll
                for (int c = 0; c < CH1; ++c) {
                    const int q = q0 + c;
                    if (q >= NQ) break;
                    if (q < NF2) {
                        const int f = wave + NW * q;
                        if (f >= NFT) continue;               // wave-uniform
                        proj(hq[c], true, okc[c], xf[c]);
                        const int p = f * 16 + col, ti = p / TW, tj = p - ti * TW;
                        pool_store(xf[c], okc[c], oy0 + ti, ox0 + tj, pres[q]);
                    } else {
                        if (wb + NW * (q - NF2) >= NFB) continue;   // wave-uniform
                        proj(hq[c], vq[c], okc[c], xf[c]);
                    }
                }
            }
        } else
        for (int f0 = wave; f0 < NF1; f0 += NW * CH1) {
            Raw xf[CH1][KS1];
            bool okc[CH1];
#pragma unroll
            for (int c = 0; c < CH1; ++c) {
                const int h = (f0 + c * NW) * 16 + col;
                const int hy = h / HWW, hx = h - hy * HWW;
                const int iy = oy0 + dt * ((tr ? hx : hy) - RY), ix = ox0 + dtx * ((tr ? hy : hx) - RX);
                okc[c] = h < HR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
#pragma unroll
                for (int s = 0; s < KS1; ++s) {
                    const int g = s * 4 + kq;
                    const bool ld = okc[c] && g < G1;
                    if constexpr (DN) {
                        // 2x2 stride-2 tap (tap = g / CG1: dy = tap >> 1, dx = tap & 1), pack_conv's K order
                        const int tap = g / CG1, cc = g - tap * CG1;
                        const uint32_t sy = (uint32_t)(2 * iy + (tap >> 1)), sx = (uint32_t)(2 * ix + (tap & 1));
                        uint32_t v = xin_n + ((__umul24(sy, (uint32_t)(2 * a.W)) + sx) * CI + cc * 8) * (uint32_t)sizeof(T);
                        asm volatile("" : "+v"(v));
                        bld8(xf[c][s], rxb, ld ? v : OOB);
                    } else {
                        bld8(xf[c][s], rxb, ld ? xn + ((__umul24((uint32_t)iy, (uint32_t)a.W) + (uint32_t)ix) * C + g * 8) * (uint32_t)sizeof(T) : OOB);
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < CH1; ++c) {
                const int h = (f0 + c * NW) * 16 + col;
                f32x4 acc[NR1];
                proj_mfma(acc, xf[c]);
                if (h < HR) {
#pragma unroll
                    for (int r = 0; r < NR1; ++r) {
                        const int ch = r * 16 + kq * 4;
                        if (ch >= IS) continue;
                        float4 v = act(f4(acc[r]), cs1 + ch);
                        if (!okc[c]) v = make_float4(0.f, 0.f, 0.f, 0.f);
                        st4t(ts + h * PSTR + ch, ch, v);
                    }
                }
                if constexpr (DN) {
                    const int hy = h / HWW, hx = h - hy * HWW;
                    const bool interior = okc[c] && hy >= 1 && hy <= TH && hx >= 1 && hx <= TW;
                    uint4 pkd[NPK * PKW];
                    pool_store(xf[c], interior, oy0 + (hy - 1), ox0 + (hx - 1), pkd);
                }
            }
        }
        STAMP(2);
        __syncthreads();
        STAMP(3);

        // residual of phase 3 (x at the tile pixels), loaded in the layout phase 3 stores in (see
        // there): per lane and row pair t of the expansion, one 16-B chunk of its pixel. RP fragments
        // are prefetched before the middle conv (asymmetric: after its 5x1 pass, to keep the two
        // passes' live ranges apart); phase 3 refills the ring as it consumes it.
        constexpr int RP = BShape<C, V>::RP < NF2 ? BShape<C, V>::RP : NF2;
        uint4 res[RP][RQ3];
        // staged epilogue: lane chunk k of a fragment is channel chunk sc_ch(k) of its pixel sc_px(k)
        // (coalesced 16-B loads and stores); HSTG: chunks 0 .. CPL/2 - 1 are the first 32-channel half
        auto sc_q = [&](int k) -> int { return HSTG ? lane + 64 * (k % (CPL / 2)) : lane + 64 * k; };
        auto sc_px = [&](int k) -> int { return HSTG ? sc_q(k) / (CPP / 2) : sc_q(k) / CPP; };
        auto sc_ch = [&](int k) -> int {
            return HSTG ? (k / (CPL / 2)) * (CPP / 2) + sc_q(k) % (CPP / 2) : sc_q(k) % CPP;
        };
        auto load_res = [&](int j, uint4 (&r)[RQ3]) {
            if constexpr (!REG3) {
                const int f = wave + NW * j;
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    const uint32_t off = res_off(f, sc_px(k), sc_ch(k) * EPC);
                    r[k] = bld16(rrb, HSTG || sc_q(k) < CPF ? off : OOB);
                }
                return;
            }
            if constexpr (LINES64) {
                // whole lines, as LINES stores them: per u, line u of pixels col and col ^ 8 (the lane's 16 B
                // of each); phase 3 trades them back into its row 2u / 2u + 1 quads (see there)
                const uint32_t pc = pix_base(wave + NW * j, col), po8 = pix_base(wave + NW * j, col ^ 8);
                const bool lo8 = col < 8;
                const uint32_t pa = lo8 ? pc : po8, pb = lo8 ? po8 : pc;
#pragma unroll
                for (int u = 0; u < RQ3 / 2; ++u) {
                    const uint32_t cb = (uint32_t)(u * 32 + (lo8 ? 0 : 16) + kq * 4) * (uint32_t)sizeof(T);
                    r[2 * u] = bld16(rrb, pa == OOB ? OOB : pa + cb);
                    r[2 * u + 1] = bld16(rrb, pb == OOB ? OOB : pb + cb);
                }
                return;
            }
            const uint32_t po = DN ? 0u : pix_base(wave + NW * j, col);
#pragma unroll
            for (int t = 0; t < RQ3; ++t) {
                const uint32_t off = DN ? res_off(wave + NW * j, col, chunk_ch(t))
                                        : po == OOB ? OOB : po + (uint32_t)chunk_ch(t) * (uint32_t)sizeof(T);
                if constexpr (HALF) {
                    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rrb, (int)off, 0, 0);
                    r[t] = make_uint4(v.x, v.y, 0u, 0u);
                } else {
                    r[t] = bld16(rrb, off);
                }
            }
        };
        auto prefetch_res = [&]() {
#pragma unroll
            for (int j = 0; j < RP; ++j) load_res(j, res[j]);
        };
        if constexpr (!ASYM && !KEEP && !DKEEP) prefetch_res();

        // t1 never goes through LDS: each wave's middle-conv accumulators (quads: lane kq holds channels
        // 4kq..4kq+3 of a pixel) are rounded as the unfused plan stores them and turned into the
        // expansion's B operand (lane kq: channels 8kq..8kq+7) with two lane swaps (to_bop) — the
        // expansion of a fragment runs on the wave that computed it, so no barrier is needed either
        Raw tf[NF2];
        auto to_tf = [&](f32x4 (&acc)[NF2][NR1], const float *cs, float om, bool mul) {
            if constexpr (F32) {
                if (mul) {
#pragma unroll
                    for (int j = 0; j < NF2; ++j)
#pragma unroll
                        for (int r = 0; r < NR1; ++r) acc[j][r] = mul4(acc[j][r], om);
                }
            }
#pragma unroll
            for (int j = 0; j < NF2; ++j) {
                const float4 q0 = act(f4(acc[j][0]), cs + kq * 4);
                const float4 q1 = NR1 > 1 ? act(f4(acc[j][NR1 > 1 ? 1 : 0]), cs + 16 + kq * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
                to_bop(tf[j], q0, q1);
            }
        };
        // accumulators starting at the bias (fp32, mul: times m, the accumulator's scale)
        auto bias_m = [&](const float *p, float m, bool mul) -> f32x4 {
            f32x4 b = bias4(p);
            if constexpr (F32)
                if (mul) b = mul4(b, m);
            return b;
        };
        static_assert(NR1 <= 2, "t1 in registers: at most 32 internal channels");

        // ---- phase 2: t1 = act2(W2 * t0 + b2) (asymmetric: t1a = 5x1 (t0); t1 = 1x5 (t1a))
        if constexpr (!ASYM) {
            f32x4 acc[NF2][NR1];
#pragma unroll
            for (int j = 0; j < NF2; ++j)
#pragma unroll
                for (int r = 0; r < NR1; ++r) acc[j][r] = bias_m(cb2 + r * 16 + kq * 4, b2m, SCL);
            // (fp32 C = 16 / 64 non-down forms: 3 as well — round 5, B = 64: C16 166.8 -> 163.4 us, C64 8x16
            // 145.0 -> 143.9 us; the fp32 down C64 form lost 12 us at 3, so it keeps 1)
            constexpr int PH2U = BNECK_PH2_UNROLL > 0 ? BNECK_PH2_UNROLL
                               : ((C == 128 && !DN && !(KEEP && V == 2)) || (sizeof(T) == 4 && C != 128 && !DN)) ? 3 : 1;
#pragma unroll PH2U
            for (int s = 0; s < KS2; ++s) {
                const int g = s * 4 + kq;
                const int tap = g / (IS / 8), coff = (g - tap * (IS / 8)) * 8;
                const int ky = tap / 3, kx = tap - ky * 3;
                // tap offset in tile axes (RD: the column offset is (kx - 1) d inside the tile)
                const int ti = tr ? kx : ky, tj = RD ? (kx - 1) * dt : tr ? ky : kx;
                WRaw wf[NR1];
#pragma unroll
                for (int r = 0; r < NR1; ++r) ldw(wf[r], w2 + (r * 16 + col) * K2S + s * 32);
#pragma unroll
                for (int j = 0; j < NF2; ++j) {
                    if (wave + NW * j >= NFT) continue;       // wave-uniform
                    int p = (wave + NW * j) * 16 + col;
                    if constexpr (NPX % 16 != 0) p = p < NPX ? p : 0;   // partial fragment: read anything, discarded
                    const int oy = p / TW, ox = p - oy * TW;
                    SRaw xf;
                    const bool in = g < G2 && (!RD || (unsigned)(ox + tj) < (unsigned)TW);
                    int off = ((oy + ti) * HWW + (ox + tj)) * PSTR + (HL ? coff >> 1 : coff);
                    asm volatile("" : "+v"(off));
                    if constexpr (PL) {
                        xf.h = *reinterpret_cast<const uint4 *>(in ? ts + off : zpad);
                        xf.l = *reinterpret_cast<const uint4 *>(in ? ts + PLO + off : zpad);
                    } else if constexpr (HL) {
                        const int o = in ? off : -ZP;         // masked: the zero pad just below ts
                        xf.h = *reinterpret_cast<const uint4 *>(ts + o);
                        xf.l = *reinterpret_cast<const uint4 *>(ts + o + 16);
                    } else {
                        ld8(xf, ts + (in ? off : -16));       // masked: the zero pad just below ts
                    }
#pragma unroll
                    for (int r = 0; r < NR1; ++r) mma(acc[j][r], wf[r], xf);
                }
            }
            STAMP(4);
            to_tf(acc, cs2, o2m, SCL);
        } else {
            // 5x1 over rows (taps dy = -2..2), output width TW+4 (the 1x5's halo). (Run in two fragment
            // halves with the residual kept in registers it measured slower, round 3: 28.2 vs 26.2 us)
            f32x4 acc5[NF2A][NR1];
#pragma unroll
            for (int j = 0; j < NF2A; ++j)
#pragma unroll
                for (int r = 0; r < NR1; ++r) acc5[j][r] = bias_m(cb2 + r * 16 + kq * 4, b2m, SCL);
#pragma unroll BNECK_ASYM_UNROLL
            for (int s = 0; s < KS2; ++s) {
                const int g = s * 4 + kq;
                const int tap = g / (IS / 8), coff = (g - tap * (IS / 8)) * 8;
                WRaw wf[NR1];
#pragma unroll
                for (int r = 0; r < NR1; ++r) ldw(wf[r], w2 + (r * 16 + col) * K2S + s * 32);
#pragma unroll
                for (int j = 0; j < NF2A; ++j) {
                    const int f = wave + NW * j;
                    if (f >= NFA) continue;
                    int p = f * 16 + col;
                    if constexpr (NPA % 16 != 0) p = p < NPA ? p : 0;
                    const int oy = p / TWA, ox = p - oy * TWA;
                    SRaw xf;
                    if constexpr (HL) {
                        const T *q = g < G2 ? ts + ((oy + tap) * HWW + ox) * PSTR + (coff >> 1) : zpad;
                        xf.h = *reinterpret_cast<const uint4 *>(q);
                        xf.l = *reinterpret_cast<const uint4 *>(q + 16);
                    } else {
                        ld8(xf, g < G2 ? ts + ((oy + tap) * HWW + ox) * PSTR + coff : zpad);
                    }
#pragma unroll
                    for (int r = 0; r < NR1; ++r) mma(acc5[j][r], wf[r], xf);
                }
            }
            __syncthreads();
            // t1a of fragment j, row block r: act2, zero outside the image columns (the 1x5 zero-pads t1a)
            float m1a = 0.f;                          // fp32: max |t1a| of the tile (the 1x5's output bound)
#pragma unroll
            for (int j = 0; j < NF2A; ++j)
#pragma unroll
                for (int r = 0; r < NR1; ++r) {
                    const int f = wave + NW * j, p = f * 16 + col, ch = r * 16 + kq * 4;
                    if (f < NFA && p < NPA && ch < IS) {
                        const int ox = p - (p / TWA) * TWA;
                        const bool inside = (unsigned)(ox0 - 2 + ox) < (unsigned)a.W;
                        float4 v = f4(acc5[j][r]);
                        if constexpr (F32 && SCL) v = mul4(v, o2m);
                        v = act(v, cs2 + ch);
                        v = inside ? v : make_float4(0.f, 0.f, 0.f, 0.f);
                        if constexpr (F32) rng_acc4(m1a, v);
                        st4t(ts + p * PSTR + ch, ch, v);
                    }
                }
            if constexpr (F32) {
                // the bound of t1 = act(1x5 (t1a)) from the tile's measured t1a (n2b max|t1a| + c2b)
                // rather than from x's (n2b (n2 B0 + c2) + c2b: 1e5-3e5 for the default weights, past
                // the window, where the tile's is ~3e3): one slot per wave, read after the barrier
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) m1a = __builtin_fmaxf(m1a, __shfl_xor(m1a, o));
                if (lane == 0) wmx[wave] = m1a;
            }
            __syncthreads();
            if constexpr (F32) {
                if (!a.rg.off) {
                    float mt = 0.f;
#pragma unroll
                    for (int w = 0; w < NW; ++w) mt = __builtin_fmaxf(mt, wmx[w]);
                    mt = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(mt))) * rng_pow2(-rs1);
                    const int s1b = rng_exp_bound(a.rg.n[2] * mt + a.rg.c[2], re2b), e3 = s1b + a.rg.sw[3];
                    o2bm = rng_pow2(s1b - re2b); b3m = rng_pow2(e3); o3m = rng_pow2(-e3);
                    scl = e3 != 0;
                }
            }
            {   // 1x5 over columns (taps dx = -2..2)
                f32x4 acc[NF2][NR1];
#pragma unroll
                for (int j = 0; j < NF2; ++j)
#pragma unroll
                    for (int r = 0; r < NR1; ++r) acc[j][r] = bias_m(cb2b + r * 16 + kq * 4, b2bm, SCL);
#pragma unroll BNECK_ASYM_UNROLL
                for (int s = 0; s < KS2; ++s) {
                    const int g = s * 4 + kq;
                    const int tap = g / (IS / 8), coff = (g - tap * (IS / 8)) * 8;
                    WRaw wf[NR1];
#pragma unroll
                    for (int r = 0; r < NR1; ++r) ldw(wf[r], w2b + (r * 16 + col) * K2S + s * 32);
#pragma unroll
                    for (int j = 0; j < NF2; ++j) {
                        if (wave + NW * j >= NFT) continue;
                        int p = (wave + NW * j) * 16 + col;
                        if constexpr (NPX % 16 != 0) p = p < NPX ? p : 0;
                        const int oy = p / TW, ox = p - oy * TW;
                        SRaw xf;
                        if constexpr (HL) {
                            const T *q = g < G2 ? ts + (oy * TWA + ox + tap) * PSTR + (coff >> 1) : zpad;
                            xf.h = *reinterpret_cast<const uint4 *>(q);
                            xf.l = *reinterpret_cast<const uint4 *>(q + 16);
                        } else {
                            ld8(xf, g < G2 ? ts + (oy * TWA + ox + tap) * PSTR + coff : zpad);
                        }
#pragma unroll
                        for (int r = 0; r < NR1; ++r) mma(acc[j][r], wf[r], xf);
                    }
                }
                if constexpr (!KEEP) prefetch_res();
                to_tf(acc, cs2b, o2bm, SCL || o2bm != 1.f);
            }
        }

        // ---- phase 3: out = act_out(act3(W3 t1 + b3) + x), entirely in registers. An accumulator
        // quad is 4 consecutive channels of one pixel (lane = (pixel col, quad kq)); in bf16 two
        // rows' quads of lanes kq and kq^1 are traded with v_permlane16_swap so that each lane holds
        // 8 consecutive channels (16 B) of its pixel: row 2t + (kq & 1), channels 8 (kq >> 1) ...
        // +7 — one wave store then writes 16 pixels x 64 contiguous bytes. The residual arrives in
        // that chunk layout and the same (involutive) swap returns it to accumulator quads. fp32
        // quads are already 16-B chunks; C = 16 (one row) stores its 8-B quads (a 16-pixel
        // fragment of 32-B pixels is one 512-B run). No LDS staging, no wave syncs.
        if constexpr (!REG3) {
            // staged epilogue: the t0 region becomes per-wave staging (once every wave is done
            // reading t0) — residual chunks in, results over them, and the fragment leaves as
            // contiguous 16-B-per-lane stores
            __syncthreads();
            STAMP(5);
            T *stg = ts + wave * 16 * OSTR;
            if constexpr (HSTG) {
                static_assert(!KEEP && CPL % 2 == 0 && NR3 % 2 == 0, "half staging: fp32 C = 64");
#pragma unroll
                for (int j = 0; j < NF2; ++j) {
                    if (wave + NW * j >= NFT) break;      // wave-uniform
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
#pragma unroll
                        for (int kk = 0; kk < CPL / 2; ++kk) {
                            const int k = h * (CPL / 2) + kk;
                            *reinterpret_cast<uint4 *>(stg + sc_px(k) * OSTR + (sc_ch(k) - h * (CPP / 2)) * EPC) = res[j % RP][k];
                        }
                        if (h == 1 && j + RP < NF2 && wave + NW * (j + RP) < NFT) load_res(j + RP, res[j % RP]);
                        wave_lds_sync();
#pragma unroll
                        for (int rr = 0; rr < NR3 / 2; ++rr) {
                            const int r = h * (NR3 / 2) + rr;
                            const int ch = r * 16 + kq * 4;
                            static_assert(bias_in_acc(NR3, 1), "expansion: one k step, bias in the accumulator");
                            f32x4 acc = bias_m(cb3 + ch, b3m, SCL || scl);
                            WRaw wf;
                            ldw(wf, w3 + (r * 16 + col) * K3S);
                            mma(acc, wf, tf[j]);
                            T *sp = stg + col * OSTR + (ch - h * (C / 2));
                            float4 v = f4(acc);
                            if constexpr (F32) {
                                if (scl) v = mul4(v, o3m);
                            }
                            v = act(v, cs3 + ch);
                            v = act(add4(v, ld4(sp)), cso + ch);
                            if constexpr (F32) rng_acc4(amo, v);
                            st4(sp, v);
                        }
                        wave_lds_sync();
#pragma unroll
                        for (int kk = 0; kk < CPL / 2; ++kk) {
                            const int k = h * (CPL / 2) + kk;
                            const uint32_t off = pix_off(wave + NW * j, sc_px(k), sc_ch(k) * EPC);
                            bst16o<OAUX>(rob, off, *reinterpret_cast<const uint4 *>(stg + sc_px(k) * OSTR + (sc_ch(k) - h * (CPP / 2)) * EPC));
                        }
                        wave_lds_sync();
                    }
                }
                STAMP(6);
                continue;
            }
#pragma unroll
            for (int j = 0; j < NF2; ++j) {
                if (wave + NW * j >= NFT) break;          // wave-uniform
                if constexpr (KEEP) {
                    // the kept x: lane (col, kq) holds channels 8 (4 s + kq) .. + 7 of pixel col
#pragma unroll
                    for (int s = 0; s < KS1; ++s)
                        if (s * 4 + kq < G1) *reinterpret_cast<uint4 *>(stg + col * OSTR + (s * 4 + kq) * EPC) = kx[j][s].v;
                } else {
#pragma unroll
                    for (int k = 0; k < CPL; ++k) {
                        const int q = lane + 64 * k;
                        if (q < CPF) *reinterpret_cast<uint4 *>(stg + (q / CPP) * OSTR + (q % CPP) * EPC) = res[j % RP][k];
                    }
                    if (j + RP < NF2 && wave + NW * (j + RP) < NFT) load_res(j + RP, res[j % RP]);
                }
                wave_lds_sync();
#pragma unroll
                for (int r = 0; r < NR3; ++r) {
                    const int ch = r * 16 + kq * 4;
                    f32x4 acc = bias_m(cb3 + ch, b3m, SCL || scl);
                    WRaw wf;
                    ldw(wf, w3 + (r * 16 + col) * K3S);
                    mma(acc, wf, tf[j]);
                    T *sp = stg + col * OSTR + ch;
                    float4 v = f4(acc);
                    if constexpr (F32) {
                        if (scl) v = mul4(v, o3m);
                    }
                    v = act(v, cs3 + ch);
                    v = act(add4(v, ld4(sp)), cso + ch);
                    if constexpr (F32) rng_acc4(amo, v);
                    st4(sp, v);
                }
                wave_lds_sync();
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    const int q = lane + 64 * k;
                    if (q < CPF) {
                        const uint32_t off = pix_off(wave + NW * j, q / CPP, (q % CPP) * EPC);
                        bst16o<OAUX>(rob, off, *reinterpret_cast<const uint4 *>(stg + (q / CPP) * OSTR + (q % CPP) * EPC));
                    }
                }
                wave_lds_sync();
            }
            STAMP(6);
            continue;
        }
        if constexpr (EARLY_FREE) __syncthreads();        // every wave done reading t0 / t1a: the next tile may write them
        STAMP(5);
#pragma unroll
        for (int j = 0; j < NF2; ++j) {
            if (wave + NW * j >= NFT) break;              // wave-uniform
            const uint32_t po = pix_base(wave + NW * j, col);
            // kept fp32 x (KEEPF) / pooled fp32 main branch (DKEEP) -> residual quads in place: chunk s
            // (lane kq: channels 32 s + 8 kq .. + 7) becomes .a = row 2 s, .b = row 2 s + 1
            auto to_quads = [&](RawF &k) {
                uint32_t a[4] = {__float_as_uint(k.a.x), __float_as_uint(k.a.y), __float_as_uint(k.a.z), __float_as_uint(k.a.w)};
                uint32_t b[4] = {__float_as_uint(k.b.x), __float_as_uint(k.b.y), __float_as_uint(k.b.z), __float_as_uint(k.b.w)};
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    pl16swap(a[d], b[d]);
                    pl32swap(a[d], b[d]);
                }
                k.a = make_float4(__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[2]), __uint_as_float(a[3]));
                k.b = make_float4(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[2]), __uint_as_float(b[3]));
            };
            if constexpr (DKEEP && PKW == 2) {
#pragma unroll
                for (int s = 0; s < NPK; ++s) to_quads(reinterpret_cast<RawF &>(pres[j][2 * s]));
            }
            if constexpr (KEEPF) {
#pragma unroll
                for (int s = 0; s < KS1; ++s) to_quads(reinterpret_cast<RawF &>(kx[j][s]));
            }
            auto out3 = [&](int r, const f32x4 &acc) {
                const int ch = r * 16 + kq * 4;
                float4 v = f4(acc);
                if constexpr (F32) {
                    if (scl) v = mul4(v, o3m);
                }
                return act(v, cs3 + ch);
            };
            if constexpr (LINES) {
                // whole-line stores (see LINES): rows 2u / 2u + 1 of pixels col and col ^ 8 traded across
                // lanes 8 apart, then line u of pixel col & 7 and of pixel (col & 7) + 8
                const uint32_t po_o = pix_base(wave + NW * j, col ^ 8);
                const bool lo8 = col < 8;
                const uint32_t pa = lo8 ? po : po_o, pb = lo8 ? po_o : po;
#pragma unroll
                for (int u = 0; u < RQ3 / 2; ++u) {
                    float4 v2[2];
                    // LINES64: the ring holds line u of pixels pa / pb (load_res); lane col's row 2u quad is its
                    // own first word (lo8) or lane col - 8's second, row 2u + 1 the mirror image
                    uint4 rl[2];
                    if constexpr (LINES64) {
                        const uint4 l1 = res[j % RP][2 * u], l2 = res[j % RP][2 * u + 1];
                        const uint4 xs = lo8 ? l2 : l1;
                        uint4 ys;
                        ys.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.x, 0x128, 0xf, 0xf, false);
                        ys.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.y, 0x128, 0xf, 0xf, false);
                        ys.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.z, 0x128, 0xf, 0xf, false);
                        ys.w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.w, 0x128, 0xf, 0xf, false);
                        rl[0] = lo8 ? l1 : ys;
                        rl[1] = lo8 ? ys : l2;
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int t = 2 * u + h;
                        uint4 rc;
                        if constexpr (LINES64) {
                            rc = rl[h];
                        } else if constexpr (KEEPF) {
                            const RawF &k = reinterpret_cast<const RawF &>(kx[j][t >> 1]);
                            rc = __builtin_bit_cast(uint4, (t & 1) ? k.b : k.a);
                        } else {
                            rc = t < 2 * NPK ? pres[j][t < 2 * NPK ? t : 0] : make_uint4(0u, 0u, 0u, 0u);
                        }
                        f32x4 acc = bias_m(cb3 + t * 16 + kq * 4, b3m, SCL || scl);
                        WRaw wf;
                        ldw(wf, w3 + (t * 16 + col) * K3S);
                        mma(acc, wf, tf[j]);
                        v2[h] = act(add4(out3(t, acc), __builtin_bit_cast(float4, rc)), cso + t * 16 + kq * 4);
                        rng_acc4(amo, v2[h]);
                    }
                    const uint4 u0 = __builtin_bit_cast(uint4, v2[0]), u1 = __builtin_bit_cast(uint4, v2[1]);
                    const uint4 xs = lo8 ? u1 : u0;
                    uint4 ys;
                    ys.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.x, 0x128, 0xf, 0xf, false);
                    ys.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.y, 0x128, 0xf, 0xf, false);
                    ys.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.z, 0x128, 0xf, 0xf, false);
                    ys.w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)xs.w, 0x128, 0xf, 0xf, false);
                    const uint32_t cb = (uint32_t)(u * 32 + (lo8 ? 0 : 16) + kq * 4) * (uint32_t)sizeof(T);
                    bst16o<OAUX>(rob, pa == OOB ? OOB : pa + cb, lo8 ? u0 : ys);
                    bst16o<OAUX>(rob, pb == OOB ? OOB : pb + cb, lo8 ? ys : u1);
                }
                if constexpr (LINES64)   // (the ring's refill, as below)
                    if (j + RP < NF2 && wave + NW * (j + RP) < NFT) load_res(j + RP, res[j % RP]);
                continue;
            }
#pragma unroll
            for (int t = 0; t < RQ3; ++t) {
                const uint32_t off = po == OOB ? OOB : po + (uint32_t)chunk_ch(t) * (uint32_t)sizeof(T);
                uint4 rc;
                if constexpr (KEEPF) {
                    const RawF &k = reinterpret_cast<const RawF &>(kx[j][t >> 1]);
                    rc = __builtin_bit_cast(uint4, (t & 1) ? k.b : k.a);
                } else if constexpr (KEEP) rc = reinterpret_cast<const RawH &>(kx[j][t]).v;
                else if constexpr (DKEEP && PKW == 2) rc = t < 2 * NPK ? pres[j][t < 2 * NPK ? t : 0] : make_uint4(0u, 0u, 0u, 0u);
                else if constexpr (DKEEP) rc = t < NPK ? pres[j][t < NPK ? t : 0] : make_uint4(0u, 0u, 0u, 0u);
                else rc = res[j % RP][t];
                if constexpr (SWAP) {
                    const int r0 = 2 * t, r1 = 2 * t + 1;
                    f32x4 acc0 = bias4(cb3 + r0 * 16 + kq * 4);   // (2-byte storage: no range scaling)
                    f32x4 acc1 = bias4(cb3 + r1 * 16 + kq * 4);
                    WRaw w0, w1;
                    ldw(w0, w3 + (r0 * 16 + col) * K3S);
                    ldw(w1, w3 + (r1 * 16 + col) * K3S);
                    mma(acc0, w0, tf[j]);
                    mma(acc1, w1, tf[j]);
                    // residual chunk -> quads of rows r0 / r1
                    uint32_t a0 = rc.x, a1 = rc.y, b0 = rc.z, b1 = rc.w;
                    if constexpr (KEEP || DKEEP) {
                        // kept x (lane kq: channels 32 t + 8 kq .. + 7, dwords d0..d3): row r0's quad
                        // of lane kq lives in lane kq / 2 (d0, d1 or d2, d3), row r1's in lane 2 + kq / 2;
                        // a row swap then a half swap of (d0, d2) and of (d1, d3) gathers both
                        a0 = rc.x; b0 = rc.z; a1 = rc.y; b1 = rc.w;
                        pl16swap(a0, b0);
                        pl32swap(a0, b0);
                        pl16swap(a1, b1);
                        pl32swap(a1, b1);
                    } else {
                        pl16swap(a0, b0);
                        pl16swap(a1, b1);
                    }
                    float4 v0 = act(add4(out3(r0, acc0), unpack4<T>((u32x2_t){a0, a1})), cso + r0 * 16 + kq * 4);
                    float4 v1 = act(add4(out3(r1, acc1), unpack4<T>((u32x2_t){b0, b1})), cso + r1 * 16 + kq * 4);
                    u32x2_t p0 = pack4<T>(v0), p1 = pack4<T>(v1);
                    uint32_t x0 = p0.x, x1 = p0.y, y0 = p1.x, y1 = p1.y;
                    pl16swap(x0, y0);
                    pl16swap(x1, y1);
                    bst16o<OAUX>(rob, off, make_uint4(x0, x1, y0, y1));
                } else {
                    const int r = t;
                    f32x4 acc = bias_m(cb3 + r * 16 + kq * 4, b3m, SCL || scl);
                    WRaw wf;
                    ldw(wf, w3 + (r * 16 + col) * K3S);
                    mma(acc, wf, tf[j]);
                    // (CLS: into the out tile, as the unfused plan would store it)
                    T *ot = otile + ((wave + NW * j) * 16 + col) * OPS + chunk_ch(t);
                    if constexpr (HALF) {
                        float4 v = act(add4(out3(r, acc), unpack4<T>((u32x2_t){rc.x, rc.y})), cso + r * 16 + kq * 4);
                        if constexpr (CLS) *reinterpret_cast<u32x2_t *>(ot) = pack4<T>(v);
                        else bst8o<OAUX>(rob, off, pack4<T>(v));
                    } else {
                        float4 v = act(add4(out3(r, acc), __builtin_bit_cast(float4, rc)), cso + r * 16 + kq * 4);
                        if constexpr (CLS) {
                            rng_acc4(tmo, v);
                            *reinterpret_cast<float4 *>(ot) = v;
                        } else {
                            if constexpr (F32) rng_acc4(amo, v);
                            bst16o<OAUX>(rob, off, __builtin_bit_cast(uint4, v));
                        }
                    }
                }
            }
            if constexpr (!KEEP && !DKEEP)
                if (j + RP < NF2 && wave + NW * (j + RP) < NFT) load_res(j + RP, res[j % RP]);
            if constexpr (PREF) {
                if (has_next) {
                    const uint32_t nxn = (uint32_t)(nn * a.H * a.W) * (uint32_t)(C * sizeof(T));
                    kok[j] = load_hg(noy0, nox0, nxn, int_h(wave + NW * j), true, kx[j]);
                }
            }
        }
        if constexpr (CLS) {
            // ---- class phase: ENet's final transposed conv (16 -> ncls, 3x3 stride 2) + argmax + LUT of the
            // tile's 15 x 15 inner pixels from the out tile, the class kernel's arithmetic (cls_common.h):
            // 8 groups of 32 pixels (tile rows 2g, 2g + 1; column 15 and row 15 are the next tiles'), two per
            // wave; lane (c, h) holds channels 8h .. 8h + 7 of its pixel's four taps (the 2 x 2 neighbourhood;
            // 0 outside the image, as the class kernel's masked loads) and gets output pixels (2y + b, 2x + h).
            // fp32 range scaling: the input exponent from the TILE's measured max |out| (the class kernel's
            // is the batch's: equal whenever both lie in the measured window), the weights' exponent csw
            float xm = 1.f, bm = 1.f, om = 1.f;
            bool csc = false;
            if constexpr (F32) {
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) tmo = __builtin_fmaxf(tmo, __shfl_xor(tmo, o));
                if (lane == 0) cmx[wave] = tmo;
            }
            __syncthreads();                          // every wave's rows of the out tile written
            if constexpr (F32) {
                if (!a.rg.off) {
                    float mt = 0.f;
#pragma unroll
                    for (int w = 0; w < NW; ++w) mt = __builtin_fmaxf(mt, cmx[w]);
                    mt = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(mt)));
                    const int sx = rng_exp_meas(mt), e = sx + a.csw;
                    csc = (sx | e) != 0;
                    xm = rng_pow2(sx); bm = rng_pow2(e); om = rng_pow2(-e);
                }
            }
            // (an opaque lane id: lane-derived addresses recomputed here rather than hoisted out of the
            // tile loop, where they would stay live through phases 1-3 and spill)
            int ln = lane;
            asm volatile("" : "+v"(ln));
            const int c32 = ln & 31, hh = ln >> 5;
            const auto rcls = mkbuf(a.cls_out, a.cls_bytes);
            const uint32_t W2 = (uint32_t)(2 * a.W), plane = (uint32_t)(2 * a.H) * W2;
#pragma unroll 1
            for (int gq = 0; gq < 2; ++gq) {
                const int i = 2 * (wave * 2 + gq) + (c32 >> 4), jj = c32 & 15;
                const int y = oy0 + i, x = ox0 + jj;
                // tap s of this lane's pixel, read when its MFMAs issue (LDS; nothing held across blocks)
                auto tap_x = [&](int s, Raw &xq) {
                    const int dy = s >> 1, dx = s & 1;
                    const bool ok = i + dy < TH && jj + dx < TW && y + dy < a.H && x + dx < a.W;
                    int off = ((i + dy) * TW + jj + dx) * OPS + 8 * hh;
                    asm volatile("" : "+v"(off));
                    ld8(xq, ok ? otile + off : zpad);
                };
                int cls[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    f32x16 acc;
                    const float4 *bb = reinterpret_cast<const float4 *>(cbl + (2 * b + hh) * 16);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 v = bb[q];
                        acc[4 * q] = v.x; acc[4 * q + 1] = v.y; acc[4 * q + 2] = v.z; acc[4 * q + 3] = v.w;
                    }
                    auto taps = [&](auto sc) {
#pragma unroll
                        for (int s = 0; s < 4; ++s) {
                            if (s >= 2 && cshort[b]) break;       // wave-uniform
                            CRaw w;
                            if constexpr (sizeof(T) == 4) {
                                w.h = cwl[(b * 4 + s) * 64 + ln];
                                w.l = cwl[512 + (b * 4 + s) * 64 + ln];
                            } else {
                                w.v = cwl[(b * 4 + s) * 64 + ln];
                            }
                            Raw xq;
                            tap_x(s, xq);
                            if constexpr (decltype(sc)::value) mul8(reinterpret_cast<RawF &>(xq), xm);
                            mma32(acc, w, xq);
                        }
                    };
                    bool done = false;
                    if constexpr (F32) {
                        if (csc) {
#pragma unroll
                            for (int c = 0; c < 16; ++c) acc[c] *= bm;
                            taps(std::true_type());
#pragma unroll
                            for (int c = 0; c < 16; ++c) acc[c] *= om;
                            done = true;
                        }
                    }
                    if (!done) taps(std::false_type());
                    cls[b] = cls_argmax1<(FC < 0 ? 0 : FC)>(acc, lut64);
                }
                // lanes < 32 store output row 2y (pixels 2x, 2x + 1: theirs and lane + 32's block 0), lanes
                // >= 32 row 2y + 1
                uint32_t c0 = (uint32_t)cls[0], c1 = (uint32_t)cls[1];
                pl32swap(c0, c1);
                const bool valid = i < TH - 1 && jj < TW - 1 && y < a.H && x < a.W;
                const uint32_t o = (uint32_t)n * plane + (uint32_t)(2 * y + hh) * W2 + 2u * (uint32_t)x;
                __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(c0 | (c1 << 8)), rcls, valid ? (int)o : (int)OOB, 0, 0);
            }
        }
        pref = has_next;
        STAMP(6);
    }
    if constexpr (F32) rng_commit_wg(amo, a.rg.amax_out, reinterpret_cast<float *>(ts), NW);
    span_exit(a.span);
    STAMP_ENTRY(1);
    return true;
}

template <typename T, int C, bool ASYM, int V, bool TR, int CI = 0>
__global__ void __launch_bounds__((BShape<C, V>::NW * 64), (sizeof(T) == 2 ? BShape<C, V>::OCC : C == 16 ? BNECK_F32_OCC16 : C == 64 ? (V == 2 ? BNECK_F32_OCC64_V2 : BNECK_F32_OCC64) : BNECK_F32_OCC128)) bneck_kernel(const BneckArgs a) {
    if constexpr (sizeof(T) == 4) {
        const float rl = rng_lane(a.rg);              // issued first, consumed after the first tile's loads
        if (!bneck_body<T, C, ASYM, V, TR, CI, false>(a, rl)) bneck_body<T, C, ASYM, V, TR, CI, true>(a, rl);
    } else {
        bneck_body<T, C, ASYM, V, TR, CI, false>(a, 0.f);
    }
}

// C = 16 with the class layer fused (FC = the class map's LUT kind); launch bounds as the C = 16 form
template <typename T, int FC>
__global__ void __launch_bounds__(256, (sizeof(T) == 2 ? BShape<16, 0>::OCC : BNECK_F32_OCC16)) bneck_cls_kernel(const BneckArgs a) {
    if constexpr (sizeof(T) == 4) {
        const float rl = rng_lane(a.rg);
        if (!bneck_body<T, 16, false, 0, false, 0, false, FC>(a, rl)) bneck_body<T, 16, false, 0, false, 0, true, FC>(a, rl);
    } else {
        bneck_body<T, 16, false, 0, false, 0, false, FC>(a, 0.f);
    }
}

#ifdef BUGSEG_STAMPS
extern "C" int bugseg_debug_set_stamps(void *p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(bugseg_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif

// the C = 64 2-byte forms that keep their residual in registers (BNECK_KEEP_C64): all but 20 x 16
bool bneck_keeps_c64(int prec, int v) { return BNECK_KEEP_C64 && prec != PREC_F32 && v != 1; }

size_t bneck_lds_bytes(int prec, int C, bool asym, int v, int cin, bool cls) {
    if (C == 128 && v == BNECK2_V) return prec == PREC_F32 && !asym && cin == 0 ? bneck2_lds_bytes() : (size_t)1 << 30;
    int TH, TW, NW, RD;
    bneck_shape(C, v, TH, TW, NW, &RD);
    const int es = prec_es(prec), pad = 16 / es;
    const int I = cin > 0 ? cin / 4 : C / 4, IS = I < 8 ? 8 : I, NR1 = (I + 15) / 16;
    const int KS1 = ((cin > 0 ? cin / 2 : C / 8) + 3) / 4, KS2 = ((asym ? 5 : 9) * IS / 8 + 3) / 4;
    const int R = asym ? 2 : 1, RX = RD ? 0 : R;
    const bool wide = bneck_wide(C, v, asym);
    const int padw = bneck_padw(es, C, wide, cin > 0);
    const int zp = bneck_hl(es, C, cin > 0) ? 32 : 16;
    const size_t wts = (size_t)NR1 * 16 * (KS1 * 32 + padw) + (size_t)NR1 * 16 * (KS2 * 32 + padw) * (asym ? 2 : 1) +
                       (size_t)C * (32 + padw);
    const size_t halo = (size_t)(TH + 2 * R) * (TW + 2 * RX) * (bneck_pl(es, C, cin > 0) && !asym ? 16 : bneck_pstr(es, IS, wide));
    const bool staged = C == 64 && !BNECK_REG3_C64 && !(es == 4 && (BNECK_REG3_C64_F32 || (BNECK_F32_LINES64 && cin == 0)));
    const bool hstg = staged && es == 4 && BNECK_F32_HSTG;            // fp32 C = 64: one 32-channel half at a time
    const size_t stage = staged ? (size_t)NW * 16 * ((hstg ? C / 2 : C) + pad) : 0;    // staged epilogue (REG3 off)
    const size_t consts = ((size_t)6 * NR1 * 16 + 3 * (size_t)C) * sizeof(float);
    // class fusion (C = 16): the out tile, the class weights, bias and the per-wave tile maxima
    const size_t clsb = cls ? (size_t)TH * TW * (es == 4 ? 20 : 24) * es + (es == 4 ? 16384 : 8192) + 64 * 4 + (size_t)NW * 4 : 0;
    return (wts + zp + (halo > stage ? halo : stage)) * es + consts +   // + the zero pad
           (asym && es == 4 ? (size_t)NW * sizeof(float) : 0) + clsb;      // + fp32 asymmetric max slots
}

// kernel symbol of (precision, C, asym, variant, transposed); nullptr if not built
template <typename T>
static const void *kfun(int C, bool asym, int v, bool tr) {
#define BK_CASE(CC, VV) \
    if (C == CC && v == VV && !tr) return asym ? (const void *)bneck_kernel<T, CC, true, VV, false> : (const void *)bneck_kernel<T, CC, false, VV, false>;
    BK_CASE(128, 0) BK_CASE(128, 1) BK_CASE(128, 4) BK_CASE(64, 0) BK_CASE(64, 1) BK_CASE(64, 2) BK_CASE(16, 0)
#undef BK_CASE
    // (2-byte storage only: the fp32 instance spills 9 VGPRs)
    if constexpr (sizeof(T) == 2)
        if (C == 16 && v == 1 && !tr) return asym ? nullptr : (const void *)bneck_kernel<T, 16, false, 1, false>;
    if (C == 128 && v == 1 && tr && !asym) return (const void *)bneck_kernel<T, 128, false, 1, true>;
    if (C == 128 && v == 2 && !tr && !asym) return (const void *)bneck_kernel<T, 128, false, 2, false>;
    if (C == 128 && v == 3 && !tr && !asym) return (const void *)bneck_kernel<T, 128, false, 3, false>;
    return nullptr;
}
// downsampling forms: ENet's down1 (16 -> 64 at 120x160) and down2 (64 -> 128 at 60x80)
template <typename T>
static const void *kfun_down(int C, int v, int cin) {
    if (C == 64 && v == 0 && cin == 16) return (const void *)bneck_kernel<T, 64, false, 0, false, 16>;
    if (C == 128 && v == 1 && cin == 64) return (const void *)bneck_kernel<T, 128, false, 1, false, 64>;
    return nullptr;
}

static const void *bneck_fun(int prec, int C, bool asym, int v, bool tr, int cin) {
    if (cin > 0)
        return asym || tr ? nullptr
               : prec == PREC_BF16 ? kfun_down<__bf16>(C, v, cin)
               : prec == PREC_F16  ? kfun_down<_Float16>(C, v, cin)
                                   : kfun_down<float>(C, v, cin);
    return prec == PREC_BF16 ? kfun<__bf16>(C, asym, v, tr) : prec == PREC_F16 ? kfun<_Float16>(C, asym, v, tr)
                                                            : kfun<float>(C, asym, v, tr);
}

int bneck_slots_per_cu(int prec, int C, bool asym, int v, bool tr, int cin) {
    if (C == 128 && v == BNECK2_V) {
        // planned only with BUGSEG_BNECK2=1: measured slower (round 6, B = 64, A/B on one box: 103 vs 87 us
        // per launch; bneck2_kernels.hip says why)
        const char *on = std::getenv("BUGSEG_BNECK2");
        return prec == PREC_F32 && !asym && !tr && cin == 0 && on && *on == '1' ? bneck2_slots_per_cu() : 0;
    }
    // (cached per device and form: launch_bneck asks on every launch; bugseg_runtime.cpp occupancy_per_cu)
    const void *f = bneck_fun(prec, C, asym, v, tr, cin);
    int th, tw, nw;
    bneck_shape(C, v, th, tw, nw, nullptr);
    if (!f || allow_dynamic_lds(f) != hipSuccess) return 0;
    return occupancy_per_cu(f, nw * 64, bneck_lds_bytes(prec, C, asym, v, cin));
}

hipError_t launch_bneck(int prec, int C, bool asym, int v, const BneckArgs &a, hipStream_t s, int cin) {
    if (C == 128 && v == BNECK2_V)
        return prec == PREC_F32 && !asym && !a.tr && cin == 0 ? launch_bneck2(a, s) : hipErrorInvalidValue;
    const void *f = bneck_fun(prec, C, asym, v, a.tr != 0, cin);
    if (!f) return hipErrorInvalidValue;
    int th, tw, nw;
    bneck_shape(C, v, th, tw, nw, nullptr);
    const size_t lds = bneck_lds_bytes(prec, C, asym, v, cin);
    if (lds > 64 * 1024) {
        hipError_t e = allow_dynamic_lds(f);
        if (e != hipSuccess) return e;
    }
    // grid: one round of resident workgroups (each walks ntiles / grid tiles, staging its weights
    // once), or the earlier fixed cap of 2048 (BUGSEG_BNECK_GRID=cap: A/B knob, 0 = resident slots)
    // (read per launch, so a test can force multi-tile walks at any shape)
    const int n_cu = device_cus();
    const char *ge = std::getenv("BUGSEG_BNECK_GRID");
    const int grid_cap = ge ? std::atoi(ge) : 0;
    int cap = grid_cap;
    if (cap <= 0) {
        // (BUGSEG_BNECK_GRID=-k: 1/k of the resident slots, at least one per CU — leaves room for a
        // concurrent shard's launch on another stream; A/B knob)
        const int spc = bneck_slots_per_cu(prec, C, asym, v, a.tr != 0, cin);
        const int per = grid_cap < 0 ? std::max(1, spc / -grid_cap) : spc;
        cap = spc > 0 && n_cu > 0 ? per * n_cu : 2048;
    }
    int g = a.ntiles < cap ? a.ntiles : cap;
    g = (g + 7) & ~7;
    void *args[] = {const_cast<BneckArgs *>(&a)};
    return hipLaunchKernel(f, dim3(g), dim3(nw * 64), args, lds, s);
}

template <typename T>
static const void *kfun_cls(int lk) {
    return lk == 1 ? (const void *)bneck_cls_kernel<T, 1> : lk == 2 ? (const void *)bneck_cls_kernel<T, 2>
                   : (const void *)bneck_cls_kernel<T, 0>;
}

hipError_t launch_bneck_cls(int prec, const BneckArgs &a, hipStream_t s) {
    const int lk = a.lut && (a.lut_kind == 1 || a.lut_kind == 2) ? a.lut_kind : 0;
    const void *f = prec == PREC_BF16 ? kfun_cls<__bf16>(lk) : prec == PREC_F16 ? kfun_cls<_Float16>(lk) : kfun_cls<float>(lk);
    const size_t lds = bneck_lds_bytes(prec, 16, false, 0, 0, true);
    if (lds > 64 * 1024) {
        hipError_t e = allow_dynamic_lds(f);
        if (e != hipSuccess) return e;
    }
    // one round of resident workgroups, as launch_bneck
    const int spc = occupancy_per_cu(f, 256, lds), n_cu = device_cus();
    const char *ge = std::getenv("BUGSEG_BNECK_GRID");
    const int grid_cap = ge ? std::atoi(ge) : 0;
    const int cap = grid_cap > 0 ? grid_cap : spc > 0 && n_cu > 0 ? spc * n_cu : 2048;
    int g = a.ntiles < cap ? a.ntiles : cap;
    g = (g + 7) & ~7;
    void *args[] = {const_cast<BneckArgs *>(&a)};
    return hipLaunchKernel(f, dim3(g), dim3(256), args, lds, s);
}

}  // namespace bugseg
