// Internal interface between the host runtime (bugseg_runtime.cpp) and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace bugseg {

// ---- implicit-GEMM convolution (conv_kernels.hip) -------------------------------------------
// GEMM view: rows = output channels (MFMA A operand = packed weights [Npad][Kpad]),
// columns = pixels of the GEMM grid (MFMA B operand gathered from the NHWC input), K = (tap, ci).
// The k dimension is walked in 8-channel groups; gtab[g] = dy | dx<<8 | coff<<16 (0xffff = pad).
enum Epi {
    EPI_PLAIN = 0,     // out = act1(acc + bias)
    EPI_RESADD = 1,    // out = act2(act1(acc + bias) + res)                       regular bottleneck
    EPI_RESPOOL = 2,   // out = act2(act1(acc + bias) + pad(maxpool2x2(res)))     downsampling bottleneck
    EPI_RESUNPOOL = 3, // out = act2(act1(acc + bias) + unpool(res, idx))         upsampling bottleneck
    EPI_INIT = 4,      // out = act1(acc + bias + pscale * maxpool_k(in))          initial block concat
    EPI_SHUFFLE = 5,   // 4 phases -> pixel (2y+a, 2x+b): transposed conv s2     upsampling ext tconv
    EPI_CLASSES = 6,   // 4 phases x 16 classes -> argmax + LUT / f32 logits      final transposed conv
    EPI_INIT_BGR = 7,  // EPI_INIT reading raw BGR u8 frames: normalise via LUT on load (preprocess fused)
    EPI_COUNT = 8
};

enum Prec { PREC_F32 = 0, PREC_BF16 = 1, PREC_F16 = 2 };
// bytes per stored element: fp32 parity mode 4; bf16 / f16 storage modes 2
inline constexpr int prec_es(int prec) { return prec == PREC_F32 ? 4 : 2; }

// ---- fp32 mode: range scaling of the split-f16 operands (round 5; mfma_common.h "range scaling").
// The fp32 mode's products take f16 hi / lo parts (|v| < 65504, full precision for |v| >= 2^-3), so
// every operand is brought into that window by an exact power of two: each stored tensor's max |v| is
// measured by the launch that writes it (atomic max into RNG_SLOTS words, spread over the slots by
// workgroup), the launch that reads it derives its exponent from it, the tensors that never leave a
// fused launch take theirs from a rigorous bound (|t_i| <= n_i |t_(i-1)| + c_i from the weights' row
// sums), and the weights carry a static exponent (packed w = w * 2^sw). The epilogues multiply the
// accumulators back. Exact in f32 (powers of two); when every exponent is 0 — activations and
// weights inside the window, the common case — no multiply runs at all (a wave-uniform branch).
constexpr int RNG_SLOTS = 256;   // (4 per lane of the reading wave; the writing waves spread over them)
struct RangeArgs {
    const float *amax_in;   // RNG_SLOTS words holding max |x| of the launch's input (nullptr: amax_static)
    float *amax_out;        // RNG_SLOTS words the launch max-accumulates max |out| into (nullptr: not measured)
    float amax_static;      // max |x| when amax_in is nullptr (the BGR input: the normalisation table's max)
    int sw[4];              // weight exponents of the launch's matrices, in launch order
    float n[3], c[3];       // internal tensors: |t_i| <= n[i] * |t_(i-1)| + c[i], t_(-1) = the input
    int off;                // BUGSEG_F32_RANGE=0 (A/B, negative control of tests/test_gpu_range.py): no scaling
};
// weight exponent of a matrix whose largest |w| is m (the measured-tensor window of the kernels)
int range_weight_exp(double m);
hipError_t launch_amax(const float *x, size_t n, float *slots, hipStream_t s);

struct ConvArgs {
    const void *in;      // NHWC input (B, Hin, Win, CinS)
    int B, Hin, Win, CinS;
    int Hg, Wg;          // GEMM pixel grid (output grid, or the input grid for phase convs)
    int stride;
    int M;               // B * Hg * Wg
    int Ksteps, Kpad, Npad;
    const void *w;       // packed weights [Npad][Kpad]
    const int *gtab;     // [Ksteps * 4]
    const float *bias, *slope1, *slope2, *pscale;   // [Npad]
    int cconv, cpool, pool_k;                        // EPI_INIT
    const void *res;     // residual source tensor
    int resH, resW, resC, resCS;                     // its grid, valid channels, channel stride
    const uint8_t *idx_in;                           // EPI_RESUNPOOL (low-res grid)
    uint8_t *idx_out;                                // EPI_RESPOOL (output grid)
    int idxCS;                                       // channel stride of the index tensors
    void *out;           // NHWC output (B, Hout, Wout, outC)
    int Hout, Wout, outC;
    int coutP;           // per-phase padded channel count (EPI_SHUFFLE / EPI_CLASSES)
    int ncls;            // EPI_CLASSES
    const uint8_t *lut;  // EPI_CLASSES: 16-entry class remap (nullptr: raw class id)
    int lut_kind;        // EPI_CLASSES: which remap `lut` is — 0 any / none, 1 the 3-class map (models.py:56-58),
                         // 2 the binary map (models.py:79-80): the class kernel's group-max argmax
    uint8_t *cls_out;    // EPI_CLASSES: (B, Hout, Wout) u8, may be nullptr
    float *logits_out;   // EPI_CLASSES: (B, ncls, Hout, Wout) f32 NCHW, may be nullptr
    const double *nlut;  // EPI_INIT_BGR: [3][256] normalisation table, RGB order (models.py:91)
    float naff[6];       // EPI_INIT_BGR, naff_on: the table as fmaf(v, naff[c], naff[3 + c]) (exact, see bugseg_runtime.cpp)
    int naff_on;
    int pool_scan;       // init (A/B and tests): 1 = the per-tap pool scan instead of the packed f16 form
    int ntiles;
    int stg_elems;       // per-wave output staging (elements)
    int stage_ok;        // EPI_SHUFFLE: fragments never straddle an input row (Wg % 16 == 0, M % 16 == 0)
    // derived on the host (finish_conv_args): magic divisors, buffer sizes, staging shifts
    uint32_t mHWg, mWg; int sHWg, sWg;               // fdiv by Hg*Wg and by Wg
    uint32_t in_bytes, out_bytes, res_bytes, idx_bytes;
    int cpr_sh;          // log2(outC / (16 B / elem)): 16-B chunks per output pixel (power of two)
    int slopes_le1;      // every slope1 / slope2 <= 1: PReLU as max(v, s*v)
    RangeArgs rg;        // fp32 mode: the input's measured range, sw[0] = the weights' exponent
    unsigned long long *span;   // launch span (bugseg_debug_set_spans): [min entry, max exit] clock, or null
};

// magic number for fdiv (mfma_common.h): divisor d >= 1
void fastdiv(uint32_t d, uint32_t &m, int &s);

// Launch-path caches (bugseg_runtime.cpp), keyed by the current device and guarded by a mutex (several
// host threads, several devices per process): CUs of the device; resident workgroups per CU of kernel f
// at (threads, dynamic LDS) from the occupancy API (0 on failure); the >64 KB dynamic-LDS opt-in, once
// per (device, kernel).
int device_cus();
int occupancy_per_cu(const void *f, int threads, size_t lds);
hipError_t allow_dynamic_lds(const void *f);

// Launch one convolution. nr = Npad / 16 in {1, 2, 4, 8}. Returns hipSuccess or the launch error.
hipError_t launch_conv(int prec, int nr, int epi, const ConvArgs &a, hipStream_t s);
// pixels per tile for a given nr (sizes the grid)
int conv_tile_pixels(int nr);
size_t conv_lds_bytes(int prec, const ConvArgs &a);

// ---- class layer (cls_kernels.hip): EPI_CLASSES launches with 16 input channels land here.
bool cls_supported(const ConvArgs &a);
hipError_t launch_cls(int prec, const ConvArgs &a, hipStream_t s);

// ---- initial block (init_kernels.hip): EPI_INIT / EPI_INIT_BGR launches of launch_conv land here.
// Requires the initial block's shape (3x3 s2 p1 conv of 3 channels packed as tap*8 + c, pool_k 2|3).
hipError_t launch_init(int prec, bool bgr, const ConvArgs &a, hipStream_t s);
// the normalisation table's exact affine form: candidates within NAFF_R ulps of base (init_kernels.hip)
constexpr int NAFF_R = 64;
hipError_t launch_naff_search(int prec, const double *nlut, const float *base, uint8_t *ok, hipStream_t s);

// ---- fused regular / dilated / asymmetric bottleneck (bneck_kernels.hip) ---------------------
struct BneckArgs {
    const void *x;       // block input (B, H, W, C) NHWC
    void *out;           // block output, same shape
    int B, H, W;
    int dt, phases;      // tiling dilation (the middle conv's dilation; 1 for asymmetric) and the phase
                         // count: dt^2, or dt for row-dilated full-width variants
    int tr;              // transposed tiles: tile rows run along image columns (symmetric blocks only)
    int tiles_x, tiles_y, ntiles;   // tiles per phase sub-image row / column; B * phases * tiles_y * tiles_x
    const void *w1, *w2, *w2b, *w3;                   // packed [Npad][Kpad] (w2b: asymmetric 1x5)
    const float *b1, *s1, *b2, *s2, *b2b, *s2b, *b3, *s3, *s_out;
    uint32_t x_bytes;                                 // bytes of x (== out)
    int slopes_le1;                                   // every PReLU slope <= 1: max(v, s*v)
    // downsampling blocks (cin > 0 in launch_bneck): x is unused; xin = block input (B, 2H, 2W, cin),
    // pool = scratch for the pooled main branch (B, H, W, cin), idx_out = its window positions
    const void *xin;
    void *pool;
    uint8_t *idx_out;
    int idxCS;
    uint32_t xin_bytes, pool_bytes, idx_bytes;
    RangeArgs rg;        // fp32 mode: sw = {w1, w2, w2b, w3}; n / c: t0, t1 (asym: t1a), t1 (asym)
    unsigned long long *span;   // launch span (bugseg_debug_set_spans), or null
    // the class layer fused into the C = 16 block (launch_bneck_cls; out is not written): its packed weights
    // [64][64] and bias [64] (the EPI_CLASSES op's), the class map (B, 2H, 2W) u8 and its size, the LUT
    // (16 bytes, nullptr = raw ids) and its kind (ConvArgs::lut_kind), the class count, the weights' exponent
    const void *cw;
    const float *cbias;
    uint8_t *cls_out;
    uint32_t cls_bytes;
    const uint8_t *lut;
    int lut_kind, ncls, csw;
};
// tile-shape variants of the fused kernel for C channels: 0 .. bneck_variants(C) - 1
int bneck_variants(int C);
bool bneck_keeps_c64(int prec, int v);
// rd (optional): 1 for a row-dilated full-width variant (tiles_x = 1, phases = d, needs W <= tw)
void bneck_shape(int C, int v, int &th, int &tw, int &nw, int *rd = nullptr);
// cin > 0: the downsampling form (bneck_kernels.hip) with a cin-channel input; built for (64, v0,
// cin 16) and (128, v1, cin 64)
size_t bneck_lds_bytes(int prec, int C, bool asym, int v, int cin = 0, bool cls = false);
// resident workgroups per CU (occupancy API); 0 if (C, asym, v, tr, cin) is not built
int bneck_slots_per_cu(int prec, int C, bool asym, int v, bool tr, int cin = 0);
hipError_t launch_bneck(int prec, int C, bool asym, int v, const BneckArgs &a, hipStream_t s, int cin = 0);
// the C = 16 block with the class layer fused (variant 0, untransposed; tiles 15 apart: tiles_x =
// ceil(W / 15), tiles_y = ceil(H / 15)); bneck_lds_bytes(..., cls = true) its LDS
hipError_t launch_bneck_cls(int prec, const BneckArgs &a, hipStream_t s);
// variant BNECK2_V of C = 128 (fp32, symmetric, untransposed 16 x 16 tiles): bneck2_kernels.hip, one
// 16-wave workgroup per CU running two phase-shifted tiles on one weight copy
constexpr int BNECK2_V = 5;
size_t bneck2_lds_bytes();
int bneck2_slots_per_cu();
hipError_t launch_bneck2(const BneckArgs &a, hipStream_t s);

// ---- fused upsampling bottleneck (up_kernels.hip) ----------------------------------------------
struct UpArgs {
    const void *x;            // block input (B, h, w, Cin) NHWC
    const uint8_t *idx;       // pooling indices of the paired down block (B, h, w, idxCS), byte = window position
    void *out;                // (B, 2h, 2w, Cout)
    int M, h, w, idxCS;       // M = B * h * w input pixels
    uint32_t mHW, mW; int sHW, sW;                    // fdiv by h * w and by w
    const void *w1, *w2, *w3;                         // [main; e1] pair, tconv (4 phases), expansion
    const float *b1, *s1, *b2, *s2, *b3, *s3, *s_out;
    uint32_t x_bytes, idx_bytes, out_bytes;
    int slopes_le1;
    RangeArgs rg;             // fp32 mode: sw = {pair, tconv, expansion}; n / c: e1 output, tconv output
    unsigned long long *span; // launch span (bugseg_debug_set_spans), or null
};
bool up_supported(int cin, int it, int cout);
hipError_t launch_up(int prec, int cin, int it, int cout, const UpArgs &a, hipStream_t s);

// ---- preprocess / layout (prep_kernels.hip) --------------------------------------------------
struct PreArgs {
    const uint8_t *bgr;  // (B, H0, W0, 3)
    int B, H0, W0, H, W;
    int mode;            // 0 copy, 1 area 2x, 2 linear fixed point
    const int *xofs;     // [W]
    const short *xa;     // [2W]
    const int *yofs;     // [H]
    const short *yb;     // [2H]
    int vec_end;         // row elements < vec_end use the vectorised vertical rounding
    const double *lut;   // [3][256] normalisation, RGB channel order
    int out_layout;      // BUGSEG_PRE_*
    int prec;            // engine precision (out_layout == ENGINE)
    void *out;
};
hipError_t launch_preprocess(const PreArgs &a, hipStream_t s);

struct NchwArgs {
    const void *x; int is_f64; int B, H, W; int prec; void *out;
};
hipError_t launch_nchw_to_input(const NchwArgs &a, hipStream_t s);

// ---- BEV rasteriser (bev_kernels.hip) --------------------------------------------------------
struct BevArgs {
    const uint8_t *seg;  // (B, in_rows, in_cols)
    int B, in_rows, in_cols;
    double Mi[9];        // inverse bev matrix (cv::invert closed form, computed on the host)
    int bw0;             // warpPerspective x-block width
    int warp_w, warp_h, occ_w_px, occ_h_px, occ_w, occ_h, left_x, top_y;
    double ifx, ify;     // resizeNN inverse scales
    int ros_layout;
    int variant;         // 0 create_occupancy_grid, 1 create_occupancy_grid_binary
    int8_t *out;
    // laserscan-like mode (bev.py:216-240 / :143-164): the rasteriser also writes the polar warp's
    // source grid (variant 0: the template cells; 1: the encoded grid as uint8) to `cells`, and for
    // variant 0 leaves `out` to the final laserscan kernel
    int laserscan;
    uint8_t *cells;      // (B, occ_h, occ_w)
    // polar tables (host-built, bugseg_runtime.cpp polar_tables) and per-row minima
    const int32_t *fmap; // (ph, pw): source cell x | y << 16, or -1
    const int32_t *imap; // (occ_h, occ_w): polar rho | row << 16, or -1
    int pw, ph;
    int32_t *rmin;       // (B, ph)
    int hit;             // polar value that is an obstacle: 3 (variant 0) or 100 (variant 1)
    // warp-tap table (bev_kernels.hip): per grid cell, the warpPerspective taps of the 25 template
    // pixels of the 5x5 window around the pixel the cell samples, two 8-B entries per 16-B slot, SoA
    // [BEV_SLOTS][occ_h*occ_w] (the 3x3 around the sample first); a property of the geometry only,
    // built once per calibration by launch_bev_table and shared by every frame
    uint4 *wtab;
    // band-staged form: the (band, row part) work items (bev_items_offset in the table), far bands first;
    // set by the host from the band records after the table build (bugseg_runtime.cpp bev_occgrid)
    int nitems;
};
hipError_t launch_bev(const BevArgs &a, hipStream_t s);
hipError_t launch_bev_table(const BevArgs &a, hipStream_t s);
size_t bev_table_bytes(int occ_w, int occ_h);   // tap table + per-band class-map boxes

// the band-staged forms cut the grid into bands of BEV_BAND rows (one class-map box each)
constexpr int BEV_BAND = 4;
__host__ __device__ inline int bev_bands(int occ_h) { return (occ_h + BEV_BAND - 1) / BEV_BAND; }
constexpr int BEV_WIN = 25, BEV_SLOTS = 13;
// table layout (bytes from its start): tap table [BEV_SLOTS][cells] uint4; the band records (per band
// BEV_BOXREC int4: (P, rows per part, 0, 0), then its BEV_BAND row-part boxes); the compact table
// [BEV_WIN][cells] u32 + the outside-template mask plane [cells] u32; the work items (int2 (band,
// part), at most BEV_BAND per band)
constexpr int BEV_BOXREC = 5;
__host__ __device__ inline size_t bev_records_offset(int occ_w, int occ_h) { return (size_t)occ_w * occ_h * BEV_SLOTS * 16; }
__host__ __device__ inline size_t bev_ctab_offset(int occ_w, int occ_h) {
    return (bev_records_offset(occ_w, occ_h) + (size_t)bev_bands(occ_h) * BEV_BOXREC * 16 + 255) & ~(size_t)255;
}
__host__ __device__ inline size_t bev_items_offset(int occ_w, int occ_h) {
    return (bev_ctab_offset(occ_w, occ_h) + (size_t)occ_w * occ_h * (BEV_WIN + 1) * 4 + 255) & ~(size_t)255;
}

}  // namespace bugseg
