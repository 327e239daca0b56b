// ENet initial block, both input forms, as one tiled kernel:
//
//   out = act(BN(concat(conv3x3_s2(x) [cconv ch], maxpool_k_s2(x) [3 ch])))
//
// x is either the raw BGR u8 frame (EPI_INIT_BGR: ENET.preprocess fused, models.py:84-95 — the
// (v/256 - mean)/std table is applied as the bytes enter LDS) or the engine input (EPI_INIT:
// NHWC, 8 storage channels, 3 used). A 256-thread workgroup owns an 8 x 32 output tile:
//   * the 17 x 65 x 3 input patch is read once — thread q < 195 owns byte column q of all 17 rows,
//     each row one contiguous run, 17 buffer loads in flight per thread, out-of-frame ones masked by
//     an out-of-range offset — and stored normalised in LDS (zero outside the frame = the conv's
//     zero padding);
//   * K = 27 dense, ordered so that lanes of k group kq < 3 read the 8 consecutive patch elements
//     (3 pixels x 3 channels, minus the last) of window row kq with four 4-byte LDS reads, and group 3
//     the three leftovers: one v_mfma_f32_16x16x32 per 16 output pixels;
//   * the pool channels: lane (col, kq) computes the 3 window maxima of pixel col of fragment kq
//     (the table is increasing, so this is the table of the max byte; taps outside the frame are
//     excluded as MaxPool2d's -inf padding is), then every lane fetches its fragment's maxima with
//     ds_bpermute — the max work is spread over all 64 lanes instead of the 16 that hold pool
//     channels;
//   * the accumulator layout (4 consecutive channels of one pixel per lane) makes the 16-channel
//     NHWC row of a 16-pixel fragment one contiguous 512-B (bf16) store across the wave.
// The generic implicit-GEMM path this replaces was VALU-bound (per-lane 3-byte gathers, integer
// divisions, a 16-lane pool loop the whole wave executed). Both input forms go through the same
// arithmetic, so forward_bgr == preprocess + forward bit for bit.
#include <cstdlib>
#include <type_traits>

#include "bugseg_internal.h"
// output stores: sc1 write-through (OUT_AUX_SEL, as bneck_kernels.hip): measured 44.9-46.9 -> 43.7-44.2
// us, the 2-stream bench unchanged
#ifndef BUGSEG_OUT_AUX
#define BUGSEG_OUT_AUX -1
#endif
#include "mfma_common.h"

namespace bugseg {

// INIT_ABL (debug ablation builds, wrong results; scripts/gpu_r4_abl.sh): 1 = no normalisation table
// (the byte itself), 2 = no output stores, 4 = no pool channels, 8 = no patch loads
#ifndef INIT_ABL
#define INIT_ABL 0
#endif

#ifndef INIT_POOL_PK
#define INIT_POOL_PK 1
#endif
constexpr int IT_H = 8, IT_W = 32;                        // output tile
constexpr int IP_H = 2 * IT_H + 1, IP_W = 2 * IT_W + 1;   // input patch (pixels)
constexpr int IP_RS = IP_W * 3 + 1;                       // LDS patch row stride (elements, even)
constexpr int IP_PATCH = (IP_H * IP_RS + 7) & ~7;           // one patch buffer (elements, 16-B multiple)
#ifndef INIT_NT_2B
#define INIT_NT_2B 0      // 2-byte output stores non-temporal (A/B knob)
#endif
#ifndef INIT_NT_F32
#define INIT_NT_F32 1     // fp32 output stores non-temporal: the down block that reads them 11 us faster, this 2 us slower (round 5)
#endif
#ifndef INIT_DB
#define INIT_DB 1
#endif
#ifndef INIT_OCC2
#define INIT_OCC2 6                                          // 2-byte storage: waves per SIMD the registers allow
#endif

// k -> (window row, element of the row's 9-run), the B/A fragment K order described above
__device__ __forceinline__ void init_k(int kq, int j, int &dy, int &e) {
    if (kq < 3) { dy = kq; e = j; }
    else { dy = j; e = j < 3 ? 8 : -1; }
}

template <typename T, bool BGR>
__global__ void __launch_bounds__(256, sizeof(T) == 2 ? INIT_OCC2 : 1) init_kernel(const ConvArgs a) {   // (fp16 with the packed pool took 82 registers: 5 waves per SIMD)
    span_enter(a.span);
    // INIT_DB: two patch buffers — the next tile's patch is stored while this one is computed, one
    // barrier per tile instead of two
    __shared__ __attribute__((aligned(16))) T patch_buf[(INIT_DB ? 2 : 1) * IP_PATCH];
    __shared__ float lut[BGR ? 3 * 256 : 1];
    using Raw = typename Tr<T>::Raw;
    using WRaw = typename WTr<T>::Raw;   // weight operand (fp32 mode: split-f16 parts)
    const int tid = threadIdx.x;
    const int lane = tid & 63, col = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if constexpr (BGR) {
        // rounded exactly as the engine-input path rounds it (f64 -> f32 -> T)
        if (!(sizeof(T) == 2 && a.naff_on))
            for (int i = tid; i < 3 * 256; i += 256) lut[i] = (float)(T)(float)a.nlut[i];
    }
    // A operand (weights), loop-invariant: row = output channel `col`, k = 8*kq + j in the order of
    // init_k, from the generic packing [Npad][Kpad] with k' = tap * 8 + c.
    WRaw wf;
    if constexpr (sizeof(T) == 4) {
        // fp32 mode: the split-f16 parts of each weight (mfma_common.h RawS)
        const float *wp = reinterpret_cast<const float *>(a.w) + (size_t)col * a.Kpad;
        _Float16 hi[8], lo[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int dy, e;
            init_k(kq, j, dy, e);
            hi[j] = lo[j] = (_Float16)0.f;
            if (e >= 0) wsplit_elem(wp, (dy * 3 + e / 3) * 8 + e % 3, hi[j], lo[j]);
        }
        set8(wf, hi, lo);
    } else {
        const T *wp = reinterpret_cast<const T *>(a.w);
        T wv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int dy, e;
            init_k(kq, j, dy, e);
            wv[j] = e >= 0 ? wp[col * a.Kpad + (dy * 3 + e / 3) * 8 + e % 3] : (T)0.f;
        }
        set8(wf, wv);
    }
    const int c0 = kq * 4;
    const float4 b4 = ld4f(a.bias + c0), s4 = ld4f(a.slope1 + c0), p4 = ld4f(a.pscale + c0);
    // fp32 mode range scaling (bugseg_internal.h RangeArgs): the input's range (the BGR path: the
    // normalisation table's max, static), the weights' exponent; scl false: nothing to do
    constexpr bool F32 = sizeof(T) == 4;
    bool scl = false;
    float xm = 1.f, bm = 1.f, om = 1.f, amo = 0.f;
    if constexpr (F32) {
        if (!a.rg.off) {
            const int sx = rng_exp_meas(rng_read(a.rg)), e = sx + a.rg.sw[0];
            scl = (sx | e) != 0;
            xm = rng_pow2(sx); bm = rng_pow2(e); om = rng_pow2(-e);
        }
    }
    const int po = a.pool_k == 3 ? 0 : 1;                  // pool window: patch offsets po .. 2
    const uint32_t in_bytes = BGR ? (uint32_t)((size_t)a.B * a.Hin * a.Win * 3)
                                  : (uint32_t)((size_t)a.B * a.Hin * a.Win * a.CinS * sizeof(T));
    const auto rin = mkbuf(a.in, in_bytes);
    const auto rout = mkbuf(a.out, (uint32_t)((size_t)a.B * a.Hg * a.Wg * a.outC * sizeof(T)));

    // patch column owned by this thread (constant over tiles)
    const int q = tid, px = q / 3, cb = q - px * 3;
    const bool qok = q < IP_W * 3;
    const int dpatch = BGR ? px * 3 + (2 - cb) : q;        // BGR byte cb is RGB channel 2 - cb (models.py:87)
    const int lbase = (2 - cb) * 256;
    // the table's exact affine form (bf16 / fp16, when the host found one: bugseg_runtime.cpp
    // find_affine): this thread's channel constants, no LDS lookups
    const float na = a.naff[2 - cb], nb = a.naff[5 - cb];

    const int tiles_x = (a.Wg + IT_W - 1) / IT_W, tiles_y = (a.Hg + IT_H - 1) / IT_H;
    const int per = tiles_x * tiles_y, ntiles = a.B * per;
    // LDS slot of this thread's patch column: threads past the patch width write the row pad element
    // (never read), so the stores need no branch
    const int dslot = qok ? dpatch : IP_RS - 1;
    // XCD-aware tile walk (see conv_kernels.hip)
    const int G = gridDim.x, grp = blockIdx.x & 7, slot = blockIdx.x >> 3, nslots = G >> 3;
    const int CH = (ntiles + 7) >> 3;
    // tile -> (frame, tile row, tile column): magic-number divisions (launch_init), no scalar loops
    struct Tile { int n, ty0, tx0, iy0, ix0; };
    auto geom = [&](int tile) {
        Tile t;
        t.n = (int)fdiv((uint32_t)tile, a.mHWg, a.sHWg);
        const int tr = tile - t.n * per;
        const int tyi = (int)fdiv((uint32_t)tr, a.mWg, a.sWg);
        t.ty0 = tyi * IT_H; t.tx0 = (tr - tyi * tiles_x) * IT_W;
        t.iy0 = 2 * t.ty0 - 1; t.ix0 = 2 * t.tx0 - 1;
        return t;
    };
    constexpr uint32_t PB = BGR ? 3u : 8u * (uint32_t)sizeof(T);       // bytes per input pixel (CinS = 8)
    const uint32_t qoff = BGR ? (uint32_t)q : (uint32_t)(px * PB + cb * sizeof(T));
    const uint32_t rowB = (uint32_t)a.Win * PB;
    // ---- patch loads of a tile: all 17 issued before any is consumed
    // (the whole offset goes in voffset: the descriptor's range check does not cover soffset).
    // One vector base per tile plus a scalar row step, no per-row masking: a row or column outside the
    // frame reads a harmless byte (another row of the batch, or nothing: a negative offset wraps past
    // the buffer's range and reads 0) and is zeroed when stored below
    uint32_t raw[IP_H];
    auto load_raw = [&](const Tile &t) {
        const uint32_t base = (uint32_t)((t.n * a.Hin + t.iy0) * a.Win + t.ix0) * PB + qoff;
#pragma unroll
        for (int r = 0; r < IP_H; ++r) {
            const int off = (int)(base + (uint32_t)r * rowB);
            if constexpr ((INIT_ABL & 8) != 0) raw[r] = (uint32_t)(off + r);
            else if constexpr (BGR) raw[r] = __builtin_amdgcn_raw_buffer_load_b8(rin, off, 0, 0);
            else if constexpr (sizeof(T) == 2) raw[r] = __builtin_amdgcn_raw_buffer_load_b16(rin, off, 0, 0);
            else raw[r] = __builtin_amdgcn_raw_buffer_load_b32(rin, off, 0, 0);
        }
    };
    // INIT_PF: the next tile's patch loads are issued as soon as this tile's patch is in LDS, so they
    // fly during this tile's MFMA / pool / stores (the raw registers are free by then). Measured
    // (round 3, fp16, B = 32): 44.5 -> 43.6 us per launch (68 VGPRs, 6 waves per SIMD; the grid is
    // the resident workgroup count)
#ifndef INIT_PF
#define INIT_PF 1
#endif
    // this thread's patch column of tile t, from the raw bytes, into patch buffer dst
    // (rows outside the frame exist only in the first and last tile rows: a uniform fast path)
    auto store_patch = [&](const Tile &t, T *dst) {
        const bool colok = qok && (unsigned)(t.ix0 + px) < (unsigned)a.Win;
        auto store_rows = [&](auto full_rows) {
#pragma unroll
            for (int r = 0; r < IP_H; ++r) {
                const bool ok = colok && (decltype(full_rows)::value || (unsigned)(t.iy0 + r) < (unsigned)a.Hin);
                T v;
                if constexpr (BGR) {
                    // f16: through f32, as the separate preprocess stores the engine input (prep_kernels.hip)
                    if constexpr ((INIT_ABL & 1) != 0) v = (T)(float)(raw[r] & 0xff);
                    else if (sizeof(T) == 2 && a.naff_on) v = (T)__builtin_fmaf((float)(raw[r] & 0xff), na, nb);
                    else if constexpr (__is_same(T, _Float16)) v = (T)(float)lut[lbase + (int)(raw[r] & 0xff)];
                    else v = (T)lut[lbase + (int)(raw[r] & 0xff)];
                }
                else if constexpr (sizeof(T) == 2) v = __builtin_bit_cast(T, (unsigned short)raw[r]);
                else v = __builtin_bit_cast(T, raw[r]);
                dst[r * IP_RS + dslot] = ok ? v : (T)0.f;
            }
        };
        if (t.iy0 >= 0 && t.iy0 + IP_H <= a.Hin) store_rows(std::true_type());
        else store_rows(std::false_type());
    };
    if (slot < CH && grp * CH + slot < ntiles) load_raw(geom(grp * CH + slot));
    if constexpr (INIT_DB) {
        // prologue: the first tile's patch into buffer 0, the second tile's loads in flight
        __syncthreads();   // lut staged
        if (slot < CH && grp * CH + slot < ntiles) {
            store_patch(geom(grp * CH + slot), patch_buf);
            if (slot + nslots < CH && grp * CH + slot + nslots < ntiles) load_raw(geom(grp * CH + slot + nslots));
        }
    }
    int pbuf = 0;
    for (int it = slot; it < CH; it += nslots) {
        const int tile = grp * CH + it;
        if (tile >= ntiles) break;
        const Tile tg = geom(tile);
        const int n = tg.n, ty0 = tg.ty0, tx0 = tg.tx0, iy0 = tg.iy0, ix0 = tg.ix0;
        const T *patch = patch_buf + pbuf * IP_PATCH;
        if constexpr (INIT_DB) {
            __syncthreads();   // this tile's patch complete; the other buffer's last reader (the previous tile) done
            const int tn = tile + nslots;   // (the walk's next tile: same XCD group, next slot round)
            if (it + nslots < CH && tn < ntiles) {
                store_patch(geom(tn), patch_buf + (pbuf ^ 1) * IP_PATCH);
                if (it + 2 * nslots < CH && tn + nslots < ntiles) load_raw(geom(tn + nslots));
            }
            pbuf ^= 1;
        } else {
            if (!INIT_PF && it != slot) load_raw(tg);
            __syncthreads();   // lut staged / previous tile done with the patch
            store_patch(tg, patch_buf);
            if (INIT_PF) {
                const int tn = tile + nslots;   // (the walk's next tile: same XCD group, next slot round)
                if (it + nslots < CH && tn < ntiles) load_raw(geom(tn));
            }
            __syncthreads();
        }

        // ---- pool maxima: lane (col, kq) -> pixel col of fragment f = kq (row 2*wave + (f>>1))
        float pm[3];
        if (__is_same(T, _Float16) && INIT_POOL_PK && !a.pool_scan) {
            // fp16 (round 4): a window row's 9 elements (3 pixels x 3 channels) as 5 aligned dwords
            // (ds_read_b32; the row starts 4-B aligned) and the maxima as packed f16 pairs — (ch0, ch1)
            // from dwords 0, 1:2 (shifted by one element) and 3, ch2 from halves of dwords 1, 2 and 4.
            // Excluded taps (outside the frame; pool_k 2's row / column 0) are -inf. The same maxima as
            // the per-tap scan: max is exact in f16 as in f32
            const int lr = 2 * wave + (kq >> 1), lc = (kq & 1) * 16 + col;
            const uint32_t *pw = reinterpret_cast<const uint32_t *>(patch + 2 * lr * IP_RS + 6 * lc);
            const bool row0 = po > 0 || iy0 + 2 * lr < 0, col0 = po > 0 || ix0 + 2 * lc < 0;
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            const uint32_t NINF2 = 0xFC00FC00u, NINF = 0xFC00u;
            auto pmax = [](uint32_t x, uint32_t y) {
                return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(h2, x), __builtin_bit_cast(h2, y)));
            };
            uint32_t m01 = NINF2, m2 = NINF2;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const uint32_t *r = pw + dy * (IP_RS / 2);
                const uint32_t d0 = r[0], d1 = r[1], d2 = r[2], d3 = r[3], d4 = r[4];
                const uint32_t p01 = col0 ? NINF2 : d0;                              // (ch0, ch1) of dx 0
                const uint32_t q01 = __builtin_amdgcn_alignbyte(d2, d1, 2);          // (ch0, ch1) of dx 1
                const uint32_t a01 = pmax(pmax(p01, q01), d3);                        // d3: dx 2
                const uint32_t c2a = (col0 ? NINF : (d1 & 0xffffu)) | (d2 & 0xffff0000u);   // (ch2 dx 0, ch2 dx 1)
                const uint32_t a2 = pmax(c2a, (d4 & 0xffffu) | (d4 << 16));          // ch2 dx 2 in both halves
                const bool skip = dy == 0 && row0;
                m01 = skip ? m01 : pmax(m01, a01);
                m2 = skip ? m2 : pmax(m2, a2);
            }
            const h2 v01 = __builtin_bit_cast(h2, m01), v2 = __builtin_bit_cast(h2, m2);
            pm[0] = (INIT_ABL & 4) ? 0.f : (float)v01.x;
            pm[1] = (INIT_ABL & 4) ? 0.f : (float)v01.y;
            pm[2] = (INIT_ABL & 4) ? 0.f : (float)__builtin_elementwise_max(v2.x, v2.y);
        } else {
            const int lr = 2 * wave + (kq >> 1), lc = (kq & 1) * 16 + col;
            const T *pp = patch + 2 * lr * IP_RS + 6 * lc;
            const bool top = iy0 + 2 * lr < 0, left = ix0 + 2 * lc < 0;   // window row/col 0 outside the frame
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                float mx = -INFINITY;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    if (dy < po || (dy == 0 && top)) continue;
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        if (dx < po || (dx == 0 && left)) continue;
                        mx = fmaxf(mx, (float)pp[dy * IP_RS + dx * 3 + ch]);
                    }
                }
                pm[ch] = (INIT_ABL & 4) ? 0.f : mx;
            }
        }

#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int lr = 2 * wave + (f >> 1), lc = (f & 1) * 16 + col;
            const T *pp = patch + 2 * lr * IP_RS + 6 * lc;   // window origin (tap dy = dx = 0)
            Raw xf;
            if (kq < 3) {
                const T *src = pp + kq * IP_RS;
                if constexpr (sizeof(T) == 2) {
                    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(src);
                    xf.v = make_uint4(s32[0], s32[1], s32[2], s32[3]);
                } else {
                    const float2 *s2 = reinterpret_cast<const float2 *>(src);
                    const float2 u0 = s2[0], u1 = s2[1], u2 = s2[2], u3 = s2[3];
                    xf.a = make_float4(u0.x, u0.y, u1.x, u1.y);
                    xf.b = make_float4(u2.x, u2.y, u3.x, u3.y);
                }
            } else {
                T xv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[j] = j < 3 ? pp[j * IP_RS + 8] : (T)0.f;
                set8(xf, xv);
            }
            f32x4 acc = (f32x4){b4.x, b4.y, b4.z, b4.w};   // the MFMA adds the bias
            bool done = false;
            if constexpr (F32) {
                if (scl) {
                    mul8(reinterpret_cast<RawF &>(xf), xm);
                    acc = mul4(acc, bm);
                    mma(acc, wf, xf);
                    acc = mul4(acc, om);
                    done = true;
                }
            }
            if (!done) mma(acc, wf, xf);
            float4 v = f4(acc);
            // this fragment's pool maxima for pixel col live in lane col + 16 f
            float pv[4] = {0.f, 0.f, 0.f, 0.f};
            const int src = (col + 16 * f) << 2;
            float pf[3];
#pragma unroll
            for (int ch = 0; ch < 3; ++ch)
                pf[ch] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(pm[ch])));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ch = c0 + r - a.cconv;
                if (ch >= 0 && ch < a.cpool) pv[r] = (ch == 0 ? pf[0] : ch == 1 ? pf[1] : pf[2]) * get(p4, r);
            }
            v = prelu4(add4(v, make_float4(pv[0], pv[1], pv[2], pv[3])), s4);
            const int oy = ty0 + lr, ox = tx0 + lc;
            const bool ok = oy < a.Hg && ox < a.Wg && c0 < a.outC && (!(INIT_ABL & 2) || v.x == 12345.f);
            if constexpr (F32) {
                if (ok) rng_acc4(amo, v);
            }
            const uint32_t off = ok ? (uint32_t)(((n * a.Hg + oy) * a.Wg + ox) * a.outC + c0) * (uint32_t)sizeof(T) : OOB;
            if constexpr (sizeof(T) == 2) {
                bst8o<INIT_NT_2B ? 2 : OUT_AUX_SEL(16)>(rout, off, pack4<T>(v));
            } else {
                bst16o<INIT_NT_F32 ? 2 : OUT_AUX_SEL(16)>(rout, off, __builtin_bit_cast(uint4, v));
            }
        }
    }
    if constexpr (F32) rng_commit(amo, a.rg.amax_out);
    span_exit(a.span);
}

// The exact affine form of the normalisation table (bf16 / fp16 storage): candidate k of channel c is the
// f32 pair (a, b) = (base[c], base[3 + c]) moved by (da, db) ulps, |da|, |db| <= NAFF_R; it is exact when
// T(fmaf(v, a, b)) == T((float)nlut[c][v]) — the stored table value, bits compared — for all 256
// bytes v. Evaluated here with the device's own conversions, so the init kernel's fmaf form is the
// table's value by construction. ok[c * NAFF_N^2 + (da + R) * NAFF_N + db + R] = 1 when exact.
struct NaffBase { float v[6]; };
template <typename T>
__global__ void __launch_bounds__(256) naff_search_kernel(const double *nlut, NaffBase base, uint8_t *ok) {
    constexpr int N = 2 * NAFF_R + 1, NC = N * N;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 3 * NC) return;
    const int c = i / NC, k = i - c * NC, da = k / N - NAFF_R, db = k % N - NAFF_R;
    const float a = __int_as_float(__float_as_int(base.v[c]) + da), b = __int_as_float(__float_as_int(base.v[3 + c]) + db);
    bool good = true;
    for (int v = 0; v < 256 && good; ++v) {
        const T want = (T)(float)nlut[c * 256 + v], got = (T)__builtin_fmaf((float)v, a, b);
        good = __builtin_bit_cast(unsigned short, want) == __builtin_bit_cast(unsigned short, got);
    }
    ok[i] = good ? 1 : 0;
}
hipError_t launch_naff_search(int prec, const double *nlut, const float *base, uint8_t *ok, hipStream_t s) {
    NaffBase b;
    for (int i = 0; i < 6; ++i) b.v[i] = base[i];
    const int n = 3 * (2 * NAFF_R + 1) * (2 * NAFF_R + 1), g = (n + 255) / 256;
    if (prec == PREC_BF16) hipLaunchKernelGGL(naff_search_kernel<__bf16>, dim3(g), dim3(256), 0, s, nlut, b, ok);
    else hipLaunchKernelGGL(naff_search_kernel<_Float16>, dim3(g), dim3(256), 0, s, nlut, b, ok);
    return hipGetLastError();
}

int init_tiles(const ConvArgs &a) {
    return a.B * ((a.Hg + IT_H - 1) / IT_H) * ((a.Wg + IT_W - 1) / IT_W);
}

hipError_t launch_init(int prec, bool bgr, const ConvArgs &args, hipStream_t s) {
    // the kernel's tile divisions: (mHWg, sHWg) by the tiles per frame, (mWg, sWg) by the tiles per row
    // (the initial block's launch uses neither field otherwise)
    ConvArgs a = args;
    const int tiles_x = (a.Wg + IT_W - 1) / IT_W, tiles_y = (a.Hg + IT_H - 1) / IT_H;
    fastdiv((uint32_t)(tiles_x * tiles_y), a.mHWg, a.sHWg);
    fastdiv((uint32_t)tiles_x, a.mWg, a.sWg);
    // one round of resident workgroups (occupancy API per kernel instance, cached), each walking its
    // tiles with the next patch in flight
    auto resident = [](const void *f) {
        const int per = occupancy_per_cu(f, 256, 0);   // (cached per device: bugseg_runtime.cpp)
        return device_cus() * (per > 0 ? per : 8);
    };
    const void *f = prec == PREC_BF16 ? (bgr ? (const void *)init_kernel<__bf16, true> : (const void *)init_kernel<__bf16, false>)
                  : prec == PREC_F16  ? (bgr ? (const void *)init_kernel<_Float16, true> : (const void *)init_kernel<_Float16, false>)
                                      : (bgr ? (const void *)init_kernel<float, true> : (const void *)init_kernel<float, false>);
    const int cap = resident(f);
    int g = init_tiles(a);
    g = g < cap ? g : cap;
    g = g & ~7 ? g & ~7 : 8;
    a.pool_scan = getenv("BUGSEG_INIT_POOL_SCAN") != nullptr;
    if (prec == PREC_BF16) {
        if (bgr) hipLaunchKernelGGL((init_kernel<__bf16, true>), dim3(g), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((init_kernel<__bf16, false>), dim3(g), dim3(256), 0, s, a);
    } else if (prec == PREC_F16) {
        if (bgr) hipLaunchKernelGGL((init_kernel<_Float16, true>), dim3(g), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((init_kernel<_Float16, false>), dim3(g), dim3(256), 0, s, a);
    } else {
        if (bgr) hipLaunchKernelGGL((init_kernel<float, true>), dim3(g), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((init_kernel<float, false>), dim3(g), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace bugseg
