// bugseg host runtime: the native engine behind include/bugseg.h.
//
// Replaces what the reference gets from the TensorFlow C++ runtime (GraphDef import + Session
// executor, models.py:21-44) and from OpenCV (resize / warpPerspective / morphology / resize-NN,
// models.py:87-89, bev.py:182-212):
//   * parses the BSG1 weight blob (enet_spec.py), folds batch-norm into the convolutions in double,
//     packs every convolution for the MFMA kernels ([Npad][Kpad] rows, 8-channel k groups, tap
//     table) and uploads all of it in ONE device allocation;
//   * expands the ENet block list into a launch plan per (B, H, W): one fused conv launch per
//     convolution (89 for canonical ENet), ping-pong activation buffers + per-downsample pooling
//     indices carved from ONE device arena, sized for the batch (HBM is 288 GB: the arena for
//     B=64 at 640x480 is a few GB and stays resident between calls);
//   * enqueues on the caller's stream; no host synchronisation, no allocation once a plan exists.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "bugseg_internal.h"
#include "../../include/bugseg.h"

using namespace bugseg;

// ---- launch-path caches (bugseg_internal.h)
namespace {
std::mutex g_occ_mu;
struct OccKey { int dev; const void *f; int threads; size_t lds; int val; };
std::vector<OccKey> g_occ;          // val: resident workgroups per CU; f == nullptr: the CU count
int current_device() {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess ? d : 0;
}
}  // namespace
int bugseg::device_cus() {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_occ_mu);
    for (const OccKey &k : g_occ)
        if (k.dev == dev && !k.f) return k.val;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    g_occ.push_back({dev, nullptr, 0, 0, n});
    return n;
}
int bugseg::occupancy_per_cu(const void *f, int threads, size_t lds) {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_occ_mu);
    for (const OccKey &k : g_occ)
        if (k.dev == dev && k.f == f && k.threads == threads && k.lds == lds) return k.val;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, threads, lds) != hipSuccess || n < 0) n = 0;
    g_occ.push_back({dev, f, threads, lds, n});
    return n;
}
hipError_t bugseg::allow_dynamic_lds(const void *f) {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_occ_mu);
    for (const OccKey &k : g_occ)
        if (k.dev == dev && k.f == f && k.threads == -1) return hipSuccess;
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess) g_occ.push_back({dev, f, -1, 0, 1});
    return e;
}

// the weights' exponent for the fp32 mode's split-f16 products: 0 while the largest |w| lies in the
// kernels' measured window [2^-2, 2^15) (mfma_common.h rng_exp_meas), else the exponent that brings it
// to [2^14, 2^15), clamped as the kernels clamp
int bugseg::range_weight_exp(double m) {
    if (!(m > 0) || !std::isfinite(m)) return 0;
    int e = 0;
    (void)std::frexp(m, &e);
    const int l = e - 1;
    if (l >= -2 && l < 15) return 0;
    return std::max(-40, std::min(40, 14 - l));   // (mfma_common.h RNG_EMAX)
}

namespace {

thread_local std::string g_thread_err;

struct UnitDesc {
    int kind = 0, cout = 0, cin = 0, kh = 0, kw = 0, stride = 1, pad_h = 0, pad_w = 0, dil_h = 1, dil_w = 1, out_pad = 0;
    float eps = 0.f;
    std::vector<float> w, b, gamma, beta, mean, var, slope;
};

struct BlockDesc {
    int type = 0;
    int attrs[8] = {0};
    std::vector<UnitDesc> units;
    std::vector<std::vector<float>> extra;
};

enum { BT_INITIAL = 1, BT_REGULAR = 2, BT_DOWN = 3, BT_UP = 4, BT_FULLCONV = 5 };

// One packed convolution launch (weights resident on the device).
struct Packed {
    int Npad = 0, Kpad = 0, Ksteps = 0, nr = 0;
    int CinS = 0;      // input storage channels
    int stride = 1;    // on the GEMM grid
    int cout = 0;      // valid output channels (per phase)
    int coutP = 0;     // per-phase padded channels
    int phases = 1;
    double macs_per_px = 0;   // MACs per GEMM pixel (flop accounting)
    size_t o_w = 0, o_gtab = 0, o_bias = 0, o_s1 = 0, o_s2 = 0, o_ps = 0;
    // fp32 mode range scaling (bugseg_internal.h RangeArgs): the weights' exponent (packed w = w * 2^sw)
    // and per packed row the bound terms of its activated output: sum |w|, |bias|, max(1, |slope|)
    int sw = 0;
    std::vector<float> rabs, rbias, rslope;
};

struct Op {
    int kind = 0;          // 0: conv_kernel launch, 1: fused bottleneck launch, 2: fused upsampling block
    ConvArgs a;
    int nr = 0, epi = 0;
    BneckArgs bn;
    UpArgs up;
    int up_cin = 0, up_it = 0, up_cout = 0;
    int bn_c = 0, bn_var = 0, bn_cin = 0;   // bn_cin > 0: a downsampling block (cin input channels)
    bool bn_asym = false;
    double bytes = 0, flops = 0;
    double layer_bytes = -1;   // per-layer (unfused) algorithmic bytes of the work; -1: same as bytes
    Op() {
        std::memset(&a, 0, sizeof(a));
        std::memset(&bn, 0, sizeof(bn));
        std::memset(&up, 0, sizeof(up));
    }
};

struct Plan {
    int B = 0, H = 0, W = 0;
    std::vector<Op> ops;
    float *words = nullptr;  // fp32 mode: RNG_SLOTS range words per measured tensor (block 0: the engine input)
    size_t words_bytes = 0;
    void *arena = nullptr;
    size_t arena_bytes = 0;
    bool pinned = false;     // a forward on this arena was captured into a graph: never freed before destroy
    std::vector<unsigned char *> idx;   // per block: its pooling-index tensor in the arena (down blocks), else null
    std::vector<size_t> idx_bytes;
    // ENet's last bottleneck (C = 16) and the class layer as ONE launch (bneck_kernels.hip, class fusion;
    // opt-in, BUGSEG_CLS_FUSE=1: measured slower, see there): possible for this plan (cls_ok: the plan ends
    // with that bottleneck feeding the class kernel), and taken by the last forward (cls_on: a class-map
    // output, both ops in its range). The last op then launches nothing; its plan_op tag is "fused".
    bool cls_ok = false, cls_on = false;
};

inline int round_up(int v, int m) { return (v + m - 1) / m * m; }
inline int pow2_nr(int npad) {   // 16-row fragments, rounded up to 1, 2, 4 or 8
    int nr = npad / 16;
    int p = 1;
    while (p < nr) p <<= 1;
    return p;
}

}  // namespace

struct bugseg_ctx {
    int device = 0;
    int prec = PREC_F32;
    float naff[6] = {};                            // exact affine form of the normalisation table (find_affine)
    bool naff_on = false;
    float norm_amax = 0.f;                         // max |table| (the BGR input's range, fp32 range scaling)
    bool range_off = false;                        // BUGSEG_F32_RANGE=0 at load_weights: no fp32 range scaling (A/B)
    unsigned long long *spans = nullptr;           // bugseg_debug_set_spans: 512 u64 of launch-span slots per op, or null
    int spans_ops = 0;                             // ... for ops [0, spans_ops) only (the caller's buffer size)
    std::string err;
    bool loaded = false;
    int ncls = 0;
    std::vector<BlockDesc> blocks;
    // packed weights: host staging + one device allocation
    std::vector<Packed> packed;
    std::vector<std::vector<int>> block_convs;     // per block: indices into packed
    std::vector<unsigned char> host_w;
    void *dev_w = nullptr;
    void *dev_luts = nullptr;                      // [0..15] lut3, [16..31] binary, then 3x256 f64 norm lut
    Plan plan;
    // preprocess resize tables (mode 2), one per recent (H0, W0, H, W): read-only once built, shared by
    // every stream; pinned: used by a call that was captured into a graph — never evicted while the
    // context lives (as the BEV and polar tables)
    struct PreTab { int key[4] = {0, 0, 0, 0}; void *tab = nullptr; bool pinned = false; };
    std::vector<PreTab> pre_tabs;
    // Private non-blocking stream for one-time table builds: a table is built and waited for there
    // before the caller's work is enqueued, so it never needs a sync of the caller's (or any other)
    // stream, and a first call made while the caller's stream is being captured into a graph works.
    hipStream_t setup = nullptr;
    // laserscan mode: polar tables per grid geometry (occ_w, occ_h, variant), read-only once built
    struct PolarTab { int key[3] = {0, 0, -1}; int pw = 0, ph = 0; void *tab = nullptr; bool pinned = false; };
    std::vector<PolarTab> polar_tabs;  // tab: fmap (ph*pw int32) then imap (occ_h*occ_w int32)
    // laserscan batch scratch of bugseg_bev_occgrid (the caller-workspace entry bugseg_bev_occgrid_ws
    // needs none): cells (B*occ_h*occ_w u8, 256-B aligned) then rmin (B*ph int32). Keyed by stream
    // so that calls enqueued on different streams of one context never share intermediate buffers.
    struct LsScratch { void *stream = nullptr; void *p = nullptr; size_t bytes = 0; uint64_t used = 0; bool pinned = false; };
    std::vector<LsScratch> ls_scratch;
    uint64_t use_clock = 0;
    // BEV warp-tap tables (bev_kernels.hip bev_table_kernel), one per recent geometry (read-only
    // once built, shared by every stream); key = the geometry fields of BevArgs. pinned: used by a
    // call that was captured into a graph — never evicted while the context lives.
    struct BevTab { std::vector<unsigned char> key; uint4 *tab = nullptr; bool pinned = false; int nitems = 0; };
    std::vector<BevTab> bev_tabs;
    // memory retired while a stream was capturing (a graph may reference it): freed at destroy
    std::vector<void *> graveyard;
};

namespace {

int fail(bugseg_ctx *c, int code, const std::string &m) {
    if (c) c->err = m;
    else g_thread_err = m;
    return code;
}

// True when `stream` is being captured into a graph (or its capture state cannot be read, which HIP
// reports for the legacy stream while another stream captures: treated as capturing, so nothing
// that synchronises is attempted).
bool stream_capturing(void *stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &st) != hipSuccess) return true;
    return st != hipStreamCaptureStatusNone;
}

// Lets this thread allocate and wait on the private setup stream while one of its streams is
// capturing in the global mode (torch.cuda.graph's default): those calls do not touch the capture.
struct RelaxCapture {
    hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
    RelaxCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
    ~RelaxCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
};

hipStream_t setup_stream(bugseg_ctx *c) {
    if (!c->setup && hipStreamCreateWithFlags(&c->setup, hipStreamNonBlocking) != hipSuccess) c->setup = nullptr;
    return c->setup;
}

// Free device memory that work already enqueued on some stream may still read. Outside a capture
// that takes a device sync (only the rare evictions come here: a 5th table geometry, a 9th stream
// on the scratch-owning entry); during a capture the memory is kept until the context is destroyed.
void retire(bugseg_ctx *c, void *p, bool capturing) {
    if (!p) return;
    if (capturing) { c->graveyard.push_back(p); return; }
    (void)hipDeviceSynchronize();
    (void)hipFree(p);
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// ---------------------------------------------------------------- blob parsing
struct Reader {
    const unsigned char *p, *end;
    bool ok = true;
    template <typename T> T get() {
        T v{};
        if (p + sizeof(T) > end) { ok = false; return v; }
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    std::vector<float> tensor() {
        uint32_t n = get<uint32_t>();
        std::vector<float> v;
        if (!ok || (size_t)(end - p) / 4 < (size_t)n) { ok = false; return v; }   // (no pointer past the end)
        v.resize(n);
        if (n) std::memcpy(v.data(), p, (size_t)n * 4);   // (memcpy from / to NULL is UB even for 0 bytes)
        p += (size_t)n * 4;
        return v;
    }
};

bool parse_blob(const void *blob, size_t bytes, std::vector<BlockDesc> &out, int &ncls, std::string &why) {
    Reader r{(const unsigned char *)blob, (const unsigned char *)blob + bytes};
    char magic[4];
    for (int i = 0; i < 4; ++i) magic[i] = r.get<char>();
    if (!r.ok || std::memcmp(magic, "BSG1", 4) != 0) { why = "bad magic (expected BSG1)"; return false; }
    uint32_t ver = r.get<uint32_t>(), nb = r.get<uint32_t>(), nc = r.get<uint32_t>();
    if (!r.ok || ver != 1) { why = "unsupported blob version"; return false; }
    if (nb == 0 || nb > 4096 || nc == 0 || nc > 16) { why = "bad block/class count"; return false; }
    ncls = (int)nc;
    for (uint32_t b = 0; b < nb; ++b) {
        BlockDesc bd;
        bd.type = (int)r.get<uint32_t>();
        for (int i = 0; i < 8; ++i) bd.attrs[i] = r.get<int32_t>();
        uint32_t nu = r.get<uint32_t>();
        if (!r.ok || nu > 16) { why = "bad unit count"; return false; }
        for (uint32_t u = 0; u < nu; ++u) {
            UnitDesc ud;
            int32_t iv[11];
            for (int i = 0; i < 11; ++i) iv[i] = r.get<int32_t>();
            ud.kind = iv[0]; ud.cout = iv[1]; ud.cin = iv[2]; ud.kh = iv[3]; ud.kw = iv[4]; ud.stride = iv[5];
            ud.pad_h = iv[6]; ud.pad_w = iv[7]; ud.dil_h = iv[8]; ud.dil_w = iv[9]; ud.out_pad = iv[10];
            ud.eps = r.get<float>();
            ud.w = r.tensor(); ud.b = r.tensor(); ud.gamma = r.tensor(); ud.beta = r.tensor();
            ud.mean = r.tensor(); ud.var = r.tensor(); ud.slope = r.tensor();
            if (!r.ok) { why = "truncated unit"; return false; }
            if (ud.cout <= 0 || ud.cin <= 0 || ud.kh <= 0 || ud.kw <= 0 || ud.cout > 128 || ud.cin > 128 || ud.kh > 7 || ud.kw > 7) {
                why = "unit dims out of range"; return false;
            }
            const size_t nw = (size_t)ud.cout * ud.cin * ud.kh * ud.kw;
            const size_t c = (size_t)ud.cout;
            if (ud.w.size() != nw || ud.b.size() != c || ud.gamma.size() != c || ud.beta.size() != c ||
                ud.mean.size() != c || ud.var.size() != c || ud.slope.size() != c) {
                why = "unit tensor size mismatch"; return false;
            }
            bd.units.push_back(std::move(ud));
        }
        uint32_t ne = r.get<uint32_t>();
        if (!r.ok || ne > 16) { why = "bad extra count"; return false; }
        for (uint32_t e = 0; e < ne; ++e) bd.extra.push_back(r.tensor());
        if (!r.ok) { why = "truncated extras"; return false; }
        out.push_back(std::move(bd));
    }
    return true;
}

// ---------------------------------------------------------------- packing
// IEEE binary16 bits of a finite float, round to nearest even (the fp16-storage mode's weights);
// overflow to +-inf, underflow through the subnormals to +-0 — as a (_Float16) cast does
uint16_t f32_to_f16(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const int32_t exp = (int32_t)((u >> 23) & 0xff) - 127 + 15;
    uint32_t man = u & 0x7fffffu;
    if (((u >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00u | (man ? 0x200u : 0u));   // inf / nan
    if (exp >= 31) return (uint16_t)(sign | 0x7c00u);
    if (exp <= 0) {                                  // subnormal half (or zero)
        if (exp < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - exp;                  // 24-bit significand -> 10 + exp bits
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) ++h;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)exp << 10) | (man >> 13);
    const uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;   // may carry into the exponent (-> inf): correct
    return (uint16_t)(sign | h);
}
// the float value of IEEE binary16 bits (exact)
float f16_to_f32(uint16_t h) {
    const float s = (h & 0x8000u) ? -1.f : 1.f;
    const int e = (h >> 10) & 31, m = h & 1023;
    if (e == 31) return m ? std::nanf("") : s * INFINITY;
    if (e == 0) return s * std::ldexp((float)m, -24);
    return s * std::ldexp((float)(m | 1024), e - 25);
}

struct Packer {
    int prec;
    std::vector<unsigned char> &buf;
    size_t push(const void *d, size_t n) {
        size_t off = round_up((int)buf.size(), 256);
        buf.resize(off + n);
        std::memcpy(buf.data() + off, d, n);
        return off;
    }
    size_t push_w(const std::vector<double> &w, int sw = 0) {
        if (prec == PREC_F16) {
            std::vector<uint16_t> h(w.size());
            for (size_t i = 0; i < w.size(); ++i) h[i] = f32_to_f16((float)w[i]);
            return push(h.data(), h.size() * 2);
        }
        if (prec == PREC_BF16) {
            std::vector<uint16_t> h(w.size());
            for (size_t i = 0; i < w.size(); ++i) {
                float f = (float)w[i];
                uint32_t u;
                std::memcpy(&u, &f, 4);
                u = u + 0x7fffu + ((u >> 16) & 1u);     // round to nearest even (weights are finite)
                h[i] = (uint16_t)(u >> 16);
            }
            return push(h.data(), h.size() * 2);
        }
        // fp32 parity mode: the split-f16 operand of mfma_common.h (RawS): per 8 consecutive k of a
        // row (rows are whole 32-k steps), the 8 hi parts f16(w) then the 8 lo parts f16(w - hi),
        // w * 2^sw rounded to f32 first (the f32 weight the exact-product path used, times the power of
        // two that brings the matrix into the split's window: range_weight_exp)
        // (rows are whole 32-k steps, so w.size() is a multiple of 8; a partial last group would be
        // zero-padded to 8, never written past the buffer)
        const double scale = std::ldexp(1.0, sw);
        std::vector<uint16_t> h((w.size() + 7) / 8 * 16, 0);
        for (size_t g = 0; g < w.size(); g += 8)
            for (size_t i = 0; i < 8 && g + i < w.size(); ++i) {
                const float f = (float)(w[g + i] * scale);
                const uint16_t hi = f32_to_f16(f);
                h[2 * g + i] = hi;
                h[2 * g + 8 + i] = f32_to_f16(f - f16_to_f32(hi));   // exact difference in f32
            }
        return push(h.data(), h.size() * 2);
    }
    size_t push_f(const std::vector<float> &v) { return push(v.data(), v.size() * 4); }
};

void bn_fold(const UnitDesc &u, std::vector<double> &scale, std::vector<double> &shift) {
    scale.resize(u.cout);
    shift.resize(u.cout);
    for (int c = 0; c < u.cout; ++c) {
        const double s = (double)u.gamma[c] / std::sqrt((double)u.var[c] + (double)u.eps);
        scale[c] = s;
        shift[c] = ((double)u.b[c] - (double)u.mean[c]) * s + (double)u.beta[c];
    }
}

int gentry(int dy, int dx, int coff) { return (dy & 0xff) | ((dx & 0xff) << 8) | (coff << 16); }

// fp32 mode range scaling: the weight exponent of the packed matrix and its rows' bound terms
// (bugseg_internal.h RangeArgs). w: the folded [Npad][Kpad] matrix; bias / slope per row.
void range_stats(Packed &p, int prec, const std::vector<double> &w, const std::vector<float> &bias,
                 const std::vector<float> &slope) {
    const char *off = std::getenv("BUGSEG_F32_RANGE");          // (read at pack time: load_weights)
    p.sw = 0;
    p.rabs.assign(p.Npad, 0.f);
    p.rbias.assign(p.Npad, 0.f);
    p.rslope.assign(p.Npad, 1.f);
    double mx = 0;
    for (int r = 0; r < p.Npad; ++r) {
        double sa = 0;
        for (int k = 0; k < p.Kpad; ++k) {
            const double v = std::fabs(w[(size_t)r * p.Kpad + k]);
            sa += v;
            mx = std::max(mx, v);
        }
        p.rabs[r] = (float)sa;
        p.rbias[r] = std::fabs(bias[r]);
        p.rslope[r] = std::max(1.f, std::fabs(slope[r]));
    }
    if (prec == PREC_F32 && !(off && *off == '0')) p.sw = range_weight_exp(mx);
}
// |act(W x + b)| <= n |x| + c over the rows [r0, r1) of a packed matrix (a 1e-4 margin for the f32
// arithmetic the kernels evaluate the bound in)
void row_bound(const Packed &p, int r0, int r1, float &n, float &c) {
    n = c = 0.f;
    for (int r = r0; r < r1 && r < (int)p.rabs.size(); ++r) {
        n = std::max(n, p.rabs[r] * p.rslope[r]);
        c = std::max(c, p.rbias[r] * p.rslope[r]);
    }
    n *= 1.0001f;
    c *= 1.0001f;
}

// Ordinary convolution (OIHW weights) on an NHWC input with CinS storage channels.
Packed pack_conv(Packer &pk, const UnitDesc &u, int CinS, const std::vector<float> *slope2) {
    Packed p;
    const int taps = u.kh * u.kw, CG = CinS / 8;
    const int Kgroups = taps * CG;
    p.Ksteps = (Kgroups + 3) / 4;
    p.Kpad = p.Ksteps * 32;
    p.cout = u.cout;
    p.coutP = round_up(u.cout, 16);
    p.nr = pow2_nr(p.coutP);
    p.Npad = p.nr * 16;
    p.CinS = CinS;
    p.stride = u.stride;
    p.macs_per_px = (double)u.cout * u.cin * taps;
    std::vector<double> scale, shift;
    bn_fold(u, scale, shift);
    std::vector<double> w((size_t)p.Npad * p.Kpad, 0.0);
    for (int co = 0; co < u.cout; ++co)
        for (int ci = 0; ci < u.cin; ++ci)
            for (int ky = 0; ky < u.kh; ++ky)
                for (int kx = 0; kx < u.kw; ++kx) {
                    const int tap = ky * u.kw + kx;
                    w[(size_t)co * p.Kpad + tap * CinS + ci] =
                        (double)u.w[(((size_t)co * u.cin + ci) * u.kh + ky) * u.kw + kx] * scale[co];
                }
    std::vector<int> gt(p.Ksteps * 4, gentry(0, 0, 0xffff));
    for (int g = 0; g < Kgroups; ++g) {
        const int tap = g / CG, ky = tap / u.kw, kx = tap % u.kw;
        gt[g] = gentry(ky * u.dil_h - u.pad_h, kx * u.dil_w - u.pad_w, (g % CG) * 8);
    }
    std::vector<float> bias(p.Npad, 0.f), s1(p.Npad, 0.f), s2(p.Npad, 0.f), ps(p.Npad, 0.f);
    for (int c = 0; c < u.cout; ++c) {
        bias[c] = (float)shift[c];
        s1[c] = u.slope[c];
        if (slope2) s2[c] = (*slope2)[c];
    }
    range_stats(p, pk.prec, w, bias, s1);
    p.o_w = pk.push_w(w, p.sw);
    p.o_gtab = pk.push(gt.data(), gt.size() * 4);
    p.o_bias = pk.push_f(bias);
    p.o_s1 = pk.push_f(s1);
    p.o_s2 = pk.push_f(s2);
    p.o_ps = pk.push_f(ps);
    return p;
}

// Two 1x1 convolutions over the same input as ONE launch (the upsampling block's main 1x1 and its
// extension branch's first 1x1, which both read the block input): rows [0, m.cout) are m's,
// rows [m.cout, m.cout + e.cout) e's, each with its own folded BN and slope. Bit-identical per output
// channel to the two separate launches when both pack to the same bias placement.
Packed pack_conv_pair(Packer &pk, const UnitDesc &m, const UnitDesc &e, int CinS) {
    UnitDesc u = m;
    u.cout = m.cout + e.cout;
    u.w.insert(u.w.end(), e.w.begin(), e.w.end());
    u.b.insert(u.b.end(), e.b.begin(), e.b.end());
    auto cat = [](std::vector<float> a, const std::vector<float> &b) { a.insert(a.end(), b.begin(), b.end()); return a; };
    // BN folds per channel (the caller requires m.eps == e.eps)
    u.gamma = cat(m.gamma, e.gamma);
    u.beta = cat(m.beta, e.beta);
    u.mean = cat(m.mean, e.mean);
    u.var = cat(m.var, e.var);
    u.slope = cat(m.slope, e.slope);
    return pack_conv(pk, u, CinS, nullptr);
}

// Stride-2 transposed convolution (IOHW weights) as a 4-phase convolution over the INPUT grid:
// output pixel (2i+a, 2j+b) = sum over taps (dy,dx) of in[i+dy][j+dx] . W[ky = a+pad-2dy][kx = b+pad-2dx]
// (PyTorch/ONNX semantics y = 2i - pad + ky). GEMM row n = phase * coutP + co.
Packed pack_tconv(Packer &pk, const UnitDesc &u, int CinS, std::string &why, int choff = 0) {
    Packed p;
    if (u.stride != 2 || u.kh != u.kw || u.pad_h != u.pad_w) { why = "tconv: only square stride-2 kernels"; return p; }
    const int k = u.kh, pad = u.pad_h;
    if (-2 - 2 * pad + k + u.out_pad != 0) { why = "tconv: output must be exactly 2x the input"; return p; }
    std::vector<int> D;
    for (int d = -3; d <= 3; ++d) {
        bool any = false;
        for (int a = 0; a < 2; ++a) { const int kk = a + pad - 2 * d; any |= kk >= 0 && kk < k; }
        if (any) D.push_back(d);
    }
    // input groups: cstore(u.cin) channels starting at channel `choff` of a CinS-channel tensor
    const int nd = (int)D.size(), taps = nd * nd, CG = round_up(u.cin, 8) / 8;
    const int Kgroups = taps * CG;
    p.Ksteps = (Kgroups + 3) / 4;
    p.Kpad = p.Ksteps * 32;
    p.cout = u.cout;
    p.coutP = round_up(u.cout, 16);
    p.phases = 4;
    p.nr = pow2_nr(4 * p.coutP);
    p.Npad = p.nr * 16;
    if (p.Npad != 4 * p.coutP || p.nr > 8) { why = "tconv: unsupported channel count"; return p; }
    p.CinS = CinS;
    p.stride = 1;
    p.macs_per_px = (double)u.cout * u.cin * k * k;       // per INPUT pixel
    std::vector<double> scale, shift;
    bn_fold(u, scale, shift);
    std::vector<double> w((size_t)p.Npad * p.Kpad, 0.0);
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int ty = 0; ty < nd; ++ty)
                for (int tx = 0; tx < nd; ++tx) {
                    const int ky = a + pad - 2 * D[ty], kx = b + pad - 2 * D[tx];
                    if (ky < 0 || ky >= k || kx < 0 || kx >= k) continue;
                    const int tap = ty * nd + tx;
                    for (int co = 0; co < u.cout; ++co)
                        for (int ci = 0; ci < u.cin; ++ci)
                            w[(size_t)((a * 2 + b) * p.coutP + co) * p.Kpad + tap * CG * 8 + ci] =
                                (double)u.w[(((size_t)ci * u.cout + co) * k + ky) * k + kx] * scale[co];
                }
    std::vector<int> gt(p.Ksteps * 4, gentry(0, 0, 0xffff));
    for (int g = 0; g < Kgroups; ++g) {
        const int tap = g / CG;
        gt[g] = gentry(D[tap / nd], D[tap % nd], choff + (g % CG) * 8);
    }
    std::vector<float> bias(p.Npad, 0.f), s1(p.Npad, 0.f), s2(p.Npad, 0.f), ps(p.Npad, 0.f);
    for (int ph = 0; ph < 4; ++ph)
        for (int c = 0; c < u.cout; ++c) {
            bias[ph * p.coutP + c] = (float)shift[c];
            s1[ph * p.coutP + c] = u.slope[c];
        }
    range_stats(p, pk.prec, w, bias, s1);
    p.o_w = pk.push_w(w, p.sw);
    p.o_gtab = pk.push(gt.data(), gt.size() * 4);
    p.o_bias = pk.push_f(bias);
    p.o_s1 = pk.push_f(s1);
    p.o_s2 = pk.push_f(s2);
    p.o_ps = pk.push_f(ps);
    return p;
}

int cstore(int c) { return round_up(c, 8); }

bool pack_all(bugseg_ctx *ctx, std::string &why) {
    ctx->packed.clear();
    ctx->block_convs.clear();
    ctx->host_w.clear();
    Packer pk{ctx->prec, ctx->host_w};
    int cur_c = 3;
    std::vector<int> down_cin(ctx->blocks.size(), -1);
    for (size_t bi = 0; bi < ctx->blocks.size(); ++bi) {
        const BlockDesc &b = ctx->blocks[bi];
        std::vector<int> ids;
        auto add = [&](const Packed &p) { ctx->packed.push_back(p); ids.push_back((int)ctx->packed.size() - 1); };
        auto expect_units = [&](size_t n) { return b.units.size() == n; };
        switch (b.type) {
        case BT_INITIAL: {
            const int cin = b.attrs[0], cconv = b.attrs[1], pk_k = b.attrs[2];
            if (bi != 0 || !expect_units(1) || cin != 3 || cconv + cin > 16 || (pk_k != 2 && pk_k != 3) ||
                b.extra.size() != 6) { why = "initial block malformed"; return false; }
            const UnitDesc &u = b.units[0];
            if (u.cout != cconv || u.cin != cin || u.kh != 3 || u.kw != 3 || u.stride != 2 || u.pad_h != 1 || u.pad_w != 1) {
                why = "initial conv must be 3x3 s2 p1"; return false;
            }
            Packed p = pack_conv(pk, u, 8, nullptr);
            // pool channels [cconv, cconv+cin): BN of the concat as scale + shift, their own slope
            std::vector<float> bias(p.Npad), s1(p.Npad), ps(p.Npad, 0.f);
            std::memcpy(bias.data(), ctx->host_w.data() + p.o_bias, p.Npad * 4);
            std::memcpy(s1.data(), ctx->host_w.data() + p.o_s1, p.Npad * 4);
            const std::vector<float> &g = b.extra[0], &be = b.extra[1], &mu = b.extra[2], &va = b.extra[3],
                                     &ep = b.extra[4], &sl = b.extra[5];
            if ((int)g.size() != cin || ep.size() != 1 || (int)sl.size() != cin) { why = "initial extras malformed"; return false; }
            for (int c = 0; c < cin; ++c) {
                const double s = (double)g[c] / std::sqrt((double)va[c] + (double)ep[0]);
                ps[cconv + c] = (float)s;
                bias[cconv + c] = (float)((double)be[c] - (double)mu[c] * s);
                s1[cconv + c] = sl[c];
            }
            std::memcpy(ctx->host_w.data() + p.o_bias, bias.data(), p.Npad * 4);
            std::memcpy(ctx->host_w.data() + p.o_s1, s1.data(), p.Npad * 4);
            std::memcpy(ctx->host_w.data() + p.o_ps, ps.data(), p.Npad * 4);
            p.cout = cconv + cin;
            add(p);
            cur_c = cconv + cin;
            break;
        }
        case BT_DOWN: {
            const int cin = b.attrs[0], cout = b.attrs[1];
            if (!expect_units(3) || b.extra.size() != 1 || cin != cur_c || cout < cin) { why = "down block malformed"; return false; }
            const UnitDesc &u1 = b.units[0], &u2 = b.units[1], &u3 = b.units[2];
            if (u1.kh != 2 || u1.kw != 2 || u1.stride != 2 || u1.cin != cin || u2.stride != 1 || u3.kh != 1 ||
                u3.kw != 1 || u3.cout != cout || (int)b.extra[0].size() != cout) { why = "down block units malformed"; return false; }
            add(pack_conv(pk, u1, cstore(cin), nullptr));
            add(pack_conv(pk, u2, cstore(u1.cout), nullptr));
            add(pack_conv(pk, u3, cstore(u2.cout), &b.extra[0]));
            down_cin[bi] = cin;
            cur_c = cout;
            break;
        }
        case BT_REGULAR: {
            const int ch = b.attrs[0];
            if ((b.units.size() != 3 && b.units.size() != 4) || b.extra.size() != 1 || ch != cur_c) {
                why = "regular block malformed"; return false;
            }
            int c = ch;
            for (size_t i = 0; i < b.units.size(); ++i) {
                const UnitDesc &u = b.units[i];
                if (u.kind != 0 || u.cin != c || u.stride != 1) { why = "regular block unit chain malformed"; return false; }
                const bool last = i + 1 == b.units.size();
                add(pack_conv(pk, u, cstore(c), last ? &b.extra[0] : nullptr));
                c = u.cout;
            }
            if (c != ch || (int)b.extra[0].size() != ch) { why = "regular block must preserve channels"; return false; }
            break;
        }
        case BT_UP: {
            const int cin = b.attrs[0], cout = b.attrs[1], ref = b.attrs[2];
            if (!expect_units(4) || b.extra.size() != 1 || cin != cur_c || ref < 0 || ref >= (int)bi ||
                ctx->blocks[ref].type != BT_DOWN || down_cin[ref] != cout) { why = "up block malformed"; return false; }
            const UnitDesc &um = b.units[0], &u1 = b.units[1], &ut = b.units[2], &u2 = b.units[3];
            if (um.kh != 1 || um.cout != cout || u1.kh != 1 || ut.kind != 1 || ut.kh != 2 || u2.kh != 1 || u2.cout != cout) {
                why = "up block units malformed"; return false;
            }
            add(pack_conv(pk, um, cstore(cin), nullptr));
            add(pack_conv(pk, u1, cstore(cin), nullptr));
            Packed t = pack_tconv(pk, ut, cstore(u1.cout), why);
            if (!why.empty()) return false;
            add(t);
            add(pack_conv(pk, u2, cstore(ut.cout), &b.extra[0]));
            // ids 4 (and 5): the main 1x1 and the extension 1x1 packed as ONE matrix over the block
            // input (rows: main then extension, each with its own folded BN and slope). Used by the
            // fused upsampling kernel (up_kernels.hip), or, where that kernel is not built for the
            // shape, as one conv launch whose output the tconv reads from channel cout on (id 5) —
            // that needs a power-of-two count of 16-B chunks per pixel (the conv epilogue's staged
            // stores). Both require the two halves to fold their bias the same way (bias_in_acc).
            const int es = prec_es(ctx->prec), mc = cstore(um.cout) + cstore(u1.cout);
            const int chunks = mc * es / 16;
            const int nr_pair = pow2_nr(round_up(um.cout, 16) + round_up(u1.cout, 16));
            auto bias_acc = [](int nr) { return nr < 8; };     // mfma_common.h bias_in_acc
            const bool same_bias = bias_acc(pow2_nr(round_up(um.cout, 16))) && bias_acc(pow2_nr(round_up(u1.cout, 16)));
            if (um.cout % 16 == 0 && u1.cout % 16 == 0 && um.eps == u1.eps && same_bias) {
                add(pack_conv_pair(pk, um, u1, cstore(cin)));
                if ((chunks & (chunks - 1)) == 0 && nr_pair <= 8 && bias_acc(nr_pair) && !std::getenv("BUGSEG_NO_PAIR")) {
                    Packed t2 = pack_tconv(pk, ut, mc, why, cstore(um.cout));
                    if (!why.empty()) return false;
                    add(t2);
                }
            }
            cur_c = cout;
            break;
        }
        case BT_FULLCONV: {
            if (!expect_units(1) || bi + 1 != ctx->blocks.size()) { why = "fullconv must be the last block"; return false; }
            const UnitDesc &u = b.units[0];
            if (u.kind != 1 || u.cin != cur_c || u.cout != ctx->ncls || u.cout > 16) { why = "fullconv malformed"; return false; }
            Packed t = pack_tconv(pk, u, cstore(cur_c), why);
            if (!why.empty()) return false;
            if (t.coutP != 16) { why = "fullconv: classes must fit 16"; return false; }
            add(t);
            cur_c = u.cout;
            break;
        }
        default:
            why = "unknown block type";
            return false;
        }
        ctx->block_convs.push_back(ids);
    }
    if (ctx->blocks.empty() || ctx->blocks.back().type != BT_FULLCONV) { why = "model must end in fullconv"; return false; }
    return true;
}

// ---------------------------------------------------------------- plan
struct Shape { int H, W, C; };   // C = storage channels

ConvArgs base_args(const bugseg_ctx *ctx, const Packed &p) {
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    const unsigned char *d = (const unsigned char *)ctx->dev_w;
    a.Ksteps = p.Ksteps;
    a.Kpad = p.Kpad;
    a.Npad = p.Npad;
    a.w = d + p.o_w;
    a.gtab = (const int *)(d + p.o_gtab);
    a.bias = (const float *)(d + p.o_bias);
    a.slope1 = (const float *)(d + p.o_s1);
    a.slope2 = (const float *)(d + p.o_s2);
    a.pscale = (const float *)(d + p.o_ps);
    a.stride = p.stride;
    a.CinS = p.CinS;
    a.coutP = p.coutP;
    return a;
}

// A regular block runs as ONE fused launch (bneck_kernels.hip) when its shape is one the fused
// kernel is built for and a tile variant covers the layer efficiently (pick_bneck_variant);
// otherwise as its 3-4 conv launches. BUGSEG_NO_FUSE=1 forces the unfused plan (A/B testing;
// results are bit-identical).
bool fusable_regular(const bugseg_ctx *ctx, const BlockDesc &b, const std::vector<int> &ids, int &r, int &d) {
    const char *env = std::getenv("BUGSEG_NO_FUSE");     // read per plan build (plans are cached)
    if (env && *env && *env != '0') return false;
    // the fused kernel computes PReLU as max(v, s*v), exact only for slopes <= 1
    for (const int id : ids) {
        const Packed &p = ctx->packed[id];
        const float *s1 = (const float *)(ctx->host_w.data() + p.o_s1), *s2 = (const float *)(ctx->host_w.data() + p.o_s2);
        for (int c = 0; c < p.Npad; ++c)
            if (!(s1[c] <= 1.f) || !(s2[c] <= 1.f)) return false;
    }
    const int C = b.attrs[0];
    if (C != 128 && C != 64 && C != 16) return false;
    const int nu = (int)b.units.size();
    const UnitDesc &u1 = b.units[0], &u3 = b.units[nu - 1];
    if (u1.kh != 1 || u1.kw != 1 || u1.cout != C / 4 || u3.kh != 1 || u3.kw != 1 || u3.cin != C / 4) return false;
    if (nu == 4) {
        const UnitDesc &a = b.units[1], &c = b.units[2];
        if (a.kh != 5 || a.kw != 1 || a.pad_h != 2 || a.pad_w != 0 || a.dil_h != 1 ||
            c.kh != 1 || c.kw != 5 || c.pad_h != 0 || c.pad_w != 2 || c.dil_w != 1 || a.cout != C / 4 || c.cout != C / 4)
            return false;
        r = 2; d = 1;
    } else {
        const UnitDesc &m = b.units[1];
        if (m.kh != 3 || m.kw != 3 || m.dil_h != m.dil_w || m.pad_h != m.dil_h || m.pad_w != m.dil_w || m.cout != C / 4)
            return false;
        d = m.dil_h;
        r = 1;
    }
    return true;
}

// The downsampling block in one fused launch (bneck_kernels.hip, cin > 0): ENet's two shapes
// (16 -> 64, 64 -> 128, internal cin / 4), 2x2 stride-2 projection, 3x3 middle conv, PReLU slopes
// <= 1. -> the tile variant (C64: 16x16, C128: 20x16, untransposed) or -1.
int fusable_down(const bugseg_ctx *ctx, const BlockDesc &b, const std::vector<int> &ids) {
    const char *env = std::getenv("BUGSEG_NO_FUSE");
    if (env && *env && *env != '0') return -1;
    const int cin = b.attrs[0], C = b.attrs[1];
    const int v = C == 64 && cin == 16 ? 0 : C == 128 && cin == 64 ? 1 : -1;
    if (v < 0 || b.units.size() != 3) return -1;
    for (const int id : ids) {
        const Packed &p = ctx->packed[id];
        const float *s1 = (const float *)(ctx->host_w.data() + p.o_s1), *s2 = (const float *)(ctx->host_w.data() + p.o_s2);
        for (int c = 0; c < p.Npad; ++c)
            if (!(s1[c] <= 1.f) || !(s2[c] <= 1.f)) return -1;
    }
    const UnitDesc &u1 = b.units[0], &u2 = b.units[1], &u3 = b.units[2];
    const int I = cin / 4;                              // ENet: internal = input channels / 4
    if (u1.kh != 2 || u1.kw != 2 || u1.stride != 2 || u1.pad_h != 0 || u1.pad_w != 0 || u1.cin != cin || u1.cout != I)
        return -1;
    if (u2.kh != 3 || u2.kw != 3 || u2.stride != 1 || u2.pad_h != 1 || u2.pad_w != 1 || u2.dil_h != 1 || u2.dil_w != 1 ||
        u2.cin != I || u2.cout != I)
        return -1;
    if (u3.kh != 1 || u3.kw != 1 || u3.cin != I || u3.cout != C) return -1;
    if (bneck_slots_per_cu(ctx->prec, C, false, v, false, cin) <= 0) return -1;
    return v;
}

// Tile variant of a fused bottleneck layer: the variant whose estimated time is least, where a
// launch costs (rounds of resident workgroups) x (per-tile cost) and the per-tile cost is the
// per-wave fragment count of the two tile phases (weights from in-kernel phase clocks of the 16x16
// C128 tile, scripts/stamp_probe.py: ~3.8k cycles per halo fragment per wave in the projection,
// ~7.5k per tile fragment per wave in the middle conv + expansion, ~4.5k fixed). Returns -1 when no
// variant keeps at least 60 % of the computed tile pixels inside the image (large dilations on small
// feature maps: the unfused launches are cheaper). BUGSEG_BNECK_VARIANT forces a variant.
int pick_bneck_variant(const bugseg_ctx *ctx, int C, bool asym, int d, int B, int H, int W, int &tiles_y, int &tiles_x,
                       int &tr, int &rdv) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0) cus = 256;
    const char *force = std::getenv("BUGSEG_BNECK_VARIANT");
    if (const char *fc = std::getenv(("BUGSEG_BNECK_VARIANT_C" + std::to_string(C)).c_str())) force = fc;   // debug
    if (asym)
        if (const char *fa = std::getenv("BUGSEG_BNECK_VARIANT_ASYM")) force = fa;   // debug
    const int R = asym ? 2 : 1;
    const int hs = (H + d - 1) / d, ws = (W + d - 1) / d;    // phase sub-image (largest phase)
    int best = -1;
    double best_cost = 0;
    for (int v = 0; v < bneck_variants(C); ++v) {
        int th, tw, nw, rd;
        bneck_shape(C, v, th, tw, nw, &rd);
        if (bneck_lds_bytes(ctx->prec, C, asym, v) > 160 * 1024) continue;
        if (rd && (asym || W > tw || d < 2)) continue;        // row-dilated tiles span the width
        const bool forced = force && *force && std::atoi(force) == v;
        for (int t = 0; t < (asym || rd ? 1 : 2); ++t) {
            const int spc = bneck_slots_per_cu(ctx->prec, C, asym, v, t != 0);
            if (spc <= 0) continue;                           // this orientation is not built
            const int slots = spc * cus;
            const int ty = rd ? (hs + th - 1) / th : t ? (hs + tw - 1) / tw : (hs + th - 1) / th;
            const int tx = rd ? 1 : t ? (ws + th - 1) / th : (ws + tw - 1) / tw;
            const double ntiles = (double)B * (rd ? d : d * d) * ty * tx;
            const double eff = (double)H * W / (ntiles / B * th * tw);
            const double nf1 = std::ceil((th + 2.0 * R) * (tw + (rd ? 0.0 : 2.0 * R)) / 16.0), nft = std::ceil(th * tw / 16.0);
            double tile = 3.8 * std::ceil(nf1 / nw) + 7.5 * std::ceil(nft / nw) + 4.5;
            // 2-byte C = 64: a form that re-reads its residual pays for it (PMC, round 6, B = 64: 20 x 16 reads
            // 1.45x its compulsory bytes and runs 71.8 us against 70.9 for the kept 16 x 16 form)
            if (C == 64 && !asym && ctx->prec != PREC_F32 && bneck_keeps_c64(ctx->prec, 0) && !bneck_keeps_c64(ctx->prec, v))
                tile *= 1.15;
            const double cost = std::ceil(ntiles / slots) * tile;
            if (!forced && eff < 0.6) continue;
            if (best < 0 || (forced && best != v) || cost < best_cost) {
                best = v; best_cost = cost; tiles_y = ty; tiles_x = tx; tr = t; rdv = rd;
            }
        }
        if (forced && best == v) break;
    }
    return best;
}

// Walk the network for (B, H, W). With fill == false only the buffer sizes are computed.
struct Walker {
    bugseg_ctx *ctx;
    int B, H, W;
    size_t es;
    // buffer sizes (bytes) and pointers
    size_t szX = 0, szT = 0, szM = 0;
    std::vector<size_t> szIdx;
    unsigned char *X[2] = {nullptr, nullptr}, *T[3] = {nullptr, nullptr, nullptr}, *Mb = nullptr;
    std::vector<unsigned char *> idx;
    std::vector<Op> ops;
    // fp32 mode range scaling (bugseg_internal.h RangeArgs): RNG_SLOTS words per measured tensor, block 0
    // for the engine input; which block holds the range of each buffer's current contents
    float *words = nullptr;
    int nwords = 1;
    std::vector<std::pair<const void *, float *>> wmap;
    static int max_words(size_t nblocks) { return (int)(4 * nblocks + 4); }
    float *take_words() {
        float *w = words && es == 4 ? words + (size_t)nwords * RNG_SLOTS : nullptr;
        ++nwords;
        return w;
    }
    void wrote(const void *buf, float *w) {
        for (auto &e : wmap)
            if (e.first == buf) { e.second = w; return; }
        wmap.push_back({buf, w});
    }
    float *words_of(const void *buf) const {
        if (es != 4) return nullptr;
        if (!buf) return words;                          // the engine input
        for (const auto &e : wmap)
            if (e.first == buf) return e.second;
        return nullptr;
    }

    size_t tbytes(const Shape &s) const { return (size_t)B * s.H * s.W * s.C * es; }

    void conv(const Packed &p, int epi, const void *in, Shape si, Shape sg, void *out, Shape so, Op &op) {
        ConvArgs a = base_args(ctx, p);
        a.in = in; a.B = B; a.Hin = si.H; a.Win = si.W;
        a.Hg = sg.H; a.Wg = sg.W; a.M = B * sg.H * sg.W;
        a.out = out; a.Hout = so.H; a.Wout = so.W; a.outC = so.C;
        a.ntiles = (a.M + conv_tile_pixels(p.nr) - 1) / conv_tile_pixels(p.nr);
        const int epc = 16 / (int)es;
        a.stg_elems = epi == EPI_CLASSES ? 64 * 20 * 4 / (int)es      // 64 pixels x 20 floats (conv_kernels.hip CLS_STR)
                    : epi == EPI_SHUFFLE ? 64 * (so.C + epc) : 16 * (so.C + epc);
        // PReLU as max(v, s*v) is exact when every slope of the launch is <= 1
        const float *s1 = (const float *)(ctx->host_w.data() + p.o_s1), *s2 = (const float *)(ctx->host_w.data() + p.o_s2);
        a.slopes_le1 = 1;
        for (int c = 0; c < p.Npad; ++c)
            if (!(s1[c] <= 1.f) || !(s2[c] <= 1.f)) a.slopes_le1 = 0;
        // fp32 range scaling: the input's measured range, the weights' exponent, this output measured
        a.rg.amax_in = words_of(in);
        a.rg.sw[0] = p.sw;
        a.rg.off = ctx->range_off;
        if (out && epi != EPI_CLASSES) {
            a.rg.amax_out = take_words();
            wrote(out, a.rg.amax_out);
        }
        op.a = a; op.nr = p.nr; op.epi = epi;
        op.flops = 2.0 * p.macs_per_px * a.M;
        op.bytes = (double)B * si.H * si.W * si.C * es + (double)p.Npad * p.Kpad * es +
                   (epi == EPI_CLASSES ? 0.0 : (double)B * so.H * so.W * so.C * es);
    }

    bool run(bool fill, std::string &why) {
        es = prec_es(ctx->prec);
        if (H % 8 || W % 8 || H <= 0 || W <= 0 || B <= 0) { why = "H and W must be positive multiples of 8"; return false; }
        const size_t nb = ctx->blocks.size();
        if (!fill) szIdx.assign(nb, 0);
        Shape cur{H, W, 8};
        const unsigned char *curp = nullptr;    // engine input, patched per call
        int xi = 0;
        ops.clear();
        nwords = 1;
        wmap.clear();
        for (size_t bi = 0; bi < nb; ++bi) {
            const BlockDesc &b = ctx->blocks[bi];
            const std::vector<int> &ids = ctx->block_convs[bi];
            auto P = [&](int i) -> const Packed & { return ctx->packed[ids[i]]; };
            unsigned char *dst = X[xi];
            switch (b.type) {
            case BT_INITIAL: {
                Shape so{H / 2, W / 2, cstore(P(0).cout)};
                szX = std::max(szX, tbytes(so));
                if (fill) {
                    Op op;
                    conv(P(0), EPI_INIT, curp, cur, so, dst, so, op);
                    op.a.cconv = b.attrs[1]; op.a.cpool = b.attrs[0]; op.a.pool_k = b.attrs[2];
                    op.a.CinS = 8;
                    ops.push_back(op);
                }
                cur = so;
                break;
            }
            case BT_DOWN: {
                Shape s1{cur.H / 2, cur.W / 2, cstore(P(0).cout)}, s2{s1.H, s1.W, cstore(P(1).cout)};
                Shape so{s1.H, s1.W, cstore(P(2).cout)};
                const int idxCS = cstore(b.attrs[0]);
                szT = std::max({szT, tbytes(s1), tbytes(s2)});
                szX = std::max(szX, tbytes(so));
                if (!fill) szIdx[bi] = (size_t)B * so.H * so.W * idxCS;
                const int dv = cur.C == b.attrs[0] ? fusable_down(ctx, b, ids) : -1;
                if (dv >= 0) {
                    // one launch: 2x2 projection + 3x3 + expansion + pooled main branch (pooled values
                    // through the T[0] scratch, read back as the residual)
                    const Shape sp{so.H, so.W, idxCS};
                    szT = std::max(szT, tbytes(sp));
                    if (fill) {
                        Op op;
                        op.kind = 1;
                        op.bn_c = b.attrs[1];
                        op.bn_var = dv;
                        op.bn_cin = b.attrs[0];
                        BneckArgs &q = op.bn;
                        std::memset(&q, 0, sizeof(q));
                        const unsigned char *dw = (const unsigned char *)ctx->dev_w;
                        const Packed &p1 = P(0), &p2 = P(1), &p3 = P(2);
                        int th, tw, nw;
                        bneck_shape(op.bn_c, dv, th, tw, nw, nullptr);
                        q.x = nullptr; q.out = dst; q.B = B; q.H = so.H; q.W = so.W;
                        q.dt = 1; q.phases = 1; q.tr = 0;
                        q.tiles_y = (so.H + th - 1) / th; q.tiles_x = (so.W + tw - 1) / tw;
                        q.ntiles = B * q.tiles_y * q.tiles_x;
                        q.w1 = dw + p1.o_w; q.b1 = (const float *)(dw + p1.o_bias); q.s1 = (const float *)(dw + p1.o_s1);
                        q.w2 = dw + p2.o_w; q.b2 = (const float *)(dw + p2.o_bias); q.s2 = (const float *)(dw + p2.o_s1);
                        q.w2b = q.w2; q.b2b = q.b2; q.s2b = q.s2;
                        q.w3 = dw + p3.o_w; q.b3 = (const float *)(dw + p3.o_bias); q.s3 = (const float *)(dw + p3.o_s1);
                        q.s_out = (const float *)(dw + p3.o_s2);
                        q.slopes_le1 = 1;
                        q.x_bytes = (uint32_t)std::min<size_t>(tbytes(so), 0x7fffffff);
                        q.xin = curp;
                        q.xin_bytes = (uint32_t)std::min<size_t>(tbytes(cur), 0x7fffffff);
                        q.pool = T[0];
                        q.pool_bytes = (uint32_t)std::min<size_t>(tbytes(sp), 0x7fffffff);
                        q.idx_out = idx[bi]; q.idxCS = idxCS;
                        q.idx_bytes = (uint32_t)std::min<size_t>((size_t)B * so.H * so.W * idxCS, 0x7fffffff);
                        q.rg.amax_in = words_of(curp);
                        q.rg.off = ctx->range_off;
                        q.rg.sw[0] = p1.sw; q.rg.sw[1] = p2.sw; q.rg.sw[2] = p2.sw; q.rg.sw[3] = p3.sw;
                        row_bound(p1, 0, p1.cout, q.rg.n[0], q.rg.c[0]);
                        row_bound(p2, 0, p2.cout, q.rg.n[1], q.rg.c[1]);
                        q.rg.amax_out = take_words();
                        wrote(dst, q.rg.amax_out);
                        const double px = (double)B * so.H * so.W;
                        double wb = 0, fl = 0;
                        for (int i = 0; i < 3; ++i) { wb += (double)P(i).Npad * P(i).Kpad * es; fl += 2.0 * P(i).macs_per_px * px; }
                        op.flops = fl;
                        // x read once, out + indices written once (the pooled scratch round trip is L2)
                        op.bytes = (double)tbytes(cur) + (double)tbytes(so) + px * idxCS + wb;
                        op.layer_bytes = (double)tbytes(cur) * 2 + 2.0 * (tbytes(s1) + tbytes(s2)) + (double)tbytes(so) +
                                         px * idxCS + wb;
                        ops.push_back(op);
                    }
                    cur = so;
                    break;
                }
                if (fill) {
                    Op o1, o2, o3;
                    conv(P(0), EPI_PLAIN, curp, cur, s1, T[0], s1, o1);
                    conv(P(1), EPI_PLAIN, T[0], s1, s2, T[1], s2, o2);
                    conv(P(2), EPI_RESPOOL, T[1], s2, so, dst, so, o3);
                    o3.a.res = curp; o3.a.resH = cur.H; o3.a.resW = cur.W; o3.a.resC = b.attrs[0]; o3.a.resCS = cur.C;
                    o3.a.idx_out = idx[bi]; o3.a.idxCS = idxCS;
                    o3.bytes += (double)B * cur.H * cur.W * cur.C * es + (double)B * so.H * so.W * idxCS;
                    ops.push_back(o1); ops.push_back(o2); ops.push_back(o3);
                }
                cur = so;
                break;
            }
            case BT_REGULAR: {
                const int nu = (int)b.units.size();
                Shape s = cur;
                const unsigned char *src = curp;
                int rr = 0, dd = 1, ty = 0, tx = 0, ttr = 0, trd = 0, var = -1;
                if (fusable_regular(ctx, b, ids, rr, dd))
                    var = pick_bneck_variant(ctx, b.attrs[0], nu == 4, dd, B, cur.H, cur.W, ty, tx, ttr, trd);
                if (var >= 0) {
                    // one launch: projection + middle conv + expansion + residual, internals in LDS
                    szX = std::max(szX, tbytes(cur));
                    if (fill) {
                        Op op;
                        op.kind = 1;
                        op.bn_c = b.attrs[0];
                        op.bn_asym = nu == 4;
                        op.bn_var = var;
                        BneckArgs &q = op.bn;
                        std::memset(&q, 0, sizeof(q));
                        const unsigned char *dw = (const unsigned char *)ctx->dev_w;
                        const Packed &p1 = P(0), &p2 = P(1), &p3 = P(nu - 1), &p2b = P(nu == 4 ? 2 : 1);
                        q.x = curp; q.out = dst; q.B = B; q.H = cur.H; q.W = cur.W;
                        q.dt = dd; q.phases = trd ? dd : dd * dd; q.tr = ttr;
                        q.tiles_y = ty; q.tiles_x = tx;
                        q.ntiles = B * q.phases * ty * tx;
                        q.w1 = dw + p1.o_w; q.b1 = (const float *)(dw + p1.o_bias); q.s1 = (const float *)(dw + p1.o_s1);
                        q.w2 = dw + p2.o_w; q.b2 = (const float *)(dw + p2.o_bias); q.s2 = (const float *)(dw + p2.o_s1);
                        q.w2b = dw + p2b.o_w; q.b2b = (const float *)(dw + p2b.o_bias); q.s2b = (const float *)(dw + p2b.o_s1);
                        q.w3 = dw + p3.o_w; q.b3 = (const float *)(dw + p3.o_bias); q.s3 = (const float *)(dw + p3.o_s1);
                        q.s_out = (const float *)(dw + p3.o_s2);
                        q.rg.amax_in = words_of(curp);
                        q.rg.off = ctx->range_off;
                        q.rg.sw[0] = p1.sw; q.rg.sw[1] = p2.sw; q.rg.sw[2] = p2b.sw; q.rg.sw[3] = p3.sw;
                        row_bound(p1, 0, p1.cout, q.rg.n[0], q.rg.c[0]);
                        row_bound(p2, 0, p2.cout, q.rg.n[1], q.rg.c[1]);
                        row_bound(p2b, 0, p2b.cout, q.rg.n[2], q.rg.c[2]);
                        q.rg.amax_out = take_words();
                        wrote(dst, q.rg.amax_out);
                        q.slopes_le1 = 1;
                        const std::pair<size_t, int> slopes[] = {{p1.o_s1, p1.Npad}, {p2.o_s1, p2.Npad}, {p2b.o_s1, p2b.Npad},
                                                                 {p3.o_s1, p3.Npad}, {p3.o_s2, p3.Npad}};
                        for (const auto &sv : slopes) {
                            const float *sl = (const float *)(ctx->host_w.data() + sv.first);
                            for (int c = 0; c < sv.second; ++c)
                                if (!(sl[c] <= 1.f)) q.slopes_le1 = 0;
                        }
                        double fl = 0, wb = 0, lb = 0;
                        const double px = (double)B * cur.H * cur.W;
                        for (int i = 0; i < nu; ++i) {
                            fl += 2.0 * P(i).macs_per_px * px;
                            wb += (double)P(i).Npad * P(i).Kpad * es;
                            lb += px * (cstore(b.units[i].cin) + cstore(b.units[i].cout)) * es;   // layer by layer
                        }
                        op.flops = fl;
                        op.bytes = 2.0 * px * cur.C * es + wb;             // what this launch must move
                        op.layer_bytes = lb + px * cur.C * es + wb;        // + the residual re-read
                        ops.push_back(op);
                    }
                    break;
                }
                for (int i = 0; i < nu; ++i) {
                    const UnitDesc &u = b.units[i];
                    const bool last = i + 1 == nu;
                    Shape so{s.H, s.W, cstore(u.cout)};
                    unsigned char *o = last ? dst : T[i % 3];
                    if (!last) szT = std::max(szT, tbytes(so));
                    else szX = std::max(szX, tbytes(so));
                    if (fill) {
                        Op op;
                        conv(P(i), last ? EPI_RESADD : EPI_PLAIN, src, s, so, o, so, op);
                        if (last) {
                            op.a.res = curp; op.a.resH = cur.H; op.a.resW = cur.W; op.a.resC = b.attrs[0]; op.a.resCS = cur.C;
                            op.bytes += (double)B * cur.H * cur.W * cur.C * es;
                        }
                        ops.push_back(op);
                    }
                    s = so;
                    src = o;
                }
                cur = s;
                break;
            }
            case BT_UP: {
                const int ref = b.attrs[2];
                Shape sm{cur.H, cur.W, cstore(P(0).cout)}, s1{cur.H, cur.W, cstore(P(1).cout)};
                Shape st{cur.H * 2, cur.W * 2, cstore(P(2).cout)}, so{cur.H * 2, cur.W * 2, cstore(P(3).cout)};
                szM = std::max(szM, tbytes(sm));
                szT = std::max({szT, tbytes(s1), tbytes(st)});
                szX = std::max(szX, tbytes(so));
                const int cin_b = b.attrs[0], cout_b = b.attrs[1], it_b = P(1).cout;
                const char *nf = std::getenv("BUGSEG_NO_FUSE");
                const bool fuse_up = ids.size() >= 5 && up_supported(cin_b, it_b, cout_b) && cur.C == cin_b &&
                                     so.C == cout_b && !(nf && *nf && *nf != '0');
                if (fuse_up) {
                    // one launch: x read once, out written once, everything else in registers
                    if (fill) {
                        Op op;
                        op.kind = 2;
                        op.up_cin = cin_b; op.up_it = it_b; op.up_cout = cout_b;
                        UpArgs &q = op.up;
                        const unsigned char *dw = (const unsigned char *)ctx->dev_w;
                        const Packed &p1 = P(4), &p2 = P(2), &p3 = P(3);
                        q.x = curp; q.idx = idx[ref]; q.out = dst;
                        q.M = B * cur.H * cur.W; q.h = cur.H; q.w = cur.W;
                        q.idxCS = cstore(ctx->blocks[ref].attrs[0]);
                        fastdiv((uint32_t)(cur.H * cur.W), q.mHW, q.sHW);
                        fastdiv((uint32_t)cur.W, q.mW, q.sW);
                        q.w1 = dw + p1.o_w; q.b1 = (const float *)(dw + p1.o_bias); q.s1 = (const float *)(dw + p1.o_s1);
                        q.w2 = dw + p2.o_w; q.b2 = (const float *)(dw + p2.o_bias); q.s2 = (const float *)(dw + p2.o_s1);
                        q.w3 = dw + p3.o_w; q.b3 = (const float *)(dw + p3.o_bias); q.s3 = (const float *)(dw + p3.o_s1);
                        q.s_out = (const float *)(dw + p3.o_s2);
                        q.rg.amax_in = words_of(curp);
                        q.rg.off = ctx->range_off;
                        q.rg.sw[0] = p1.sw; q.rg.sw[1] = p2.sw; q.rg.sw[2] = p3.sw;
                        row_bound(p1, cout_b, cout_b + it_b, q.rg.n[0], q.rg.c[0]);   // the pair's e1 rows
                        row_bound(p2, 0, p2.Npad, q.rg.n[1], q.rg.c[1]);
                        q.rg.amax_out = take_words();
                        wrote(dst, q.rg.amax_out);
                        q.x_bytes = (uint32_t)std::min<size_t>((size_t)B * cur.H * cur.W * cur.C * es, 0x7fffffff);
                        q.idx_bytes = (uint32_t)std::min<size_t>((size_t)B * cur.H * cur.W * q.idxCS, 0x7fffffff);
                        q.out_bytes = (uint32_t)std::min<size_t>((size_t)B * so.H * so.W * so.C * es, 0x7fffffff);
                        q.slopes_le1 = 1;
                        const std::pair<size_t, int> sl[] = {{p1.o_s1, p1.Npad}, {p2.o_s1, p2.Npad}, {p3.o_s1, p3.Npad},
                                                             {p3.o_s2, p3.Npad}};
                        for (const auto &v : sl) {
                            const float *f = (const float *)(ctx->host_w.data() + v.first);
                            for (int c = 0; c < v.second; ++c)
                                if (!(f[c] <= 1.f)) q.slopes_le1 = 0;
                        }
                        const double px = (double)B * cur.H * cur.W;
                        double wb = 0, fl = 0;
                        for (int i = 0; i < 4; ++i) { wb += (double)P(i).Npad * P(i).Kpad * es; fl += 2.0 * P(i).macs_per_px * px; }
                        op.flops = fl;
                        op.bytes = px * cur.C * es + px * q.idxCS + 4.0 * px * so.C * es + wb;   // x + idx in, out
                        op.layer_bytes = px * cur.C * es * 2 + px * (sm.C + s1.C) * es + px * s1.C * es + 4.0 * px * st.C * es * 2 +
                                         px * sm.C * es + px * q.idxCS + 4.0 * px * so.C * es + wb;
                        ops.push_back(op);
                    }
                    cur = so;
                    break;
                }
                const bool pair = ids.size() == 6;
                // paired: the main and extension 1x1 outputs share one tensor (main channels first)
                Shape sp{cur.H, cur.W, pair ? sm.C + s1.C : sm.C};
                szM = std::max(szM, tbytes(sp));
                if (fill && pair) {
                    Op om1, ot, o2;
                    conv(P(4), EPI_PLAIN, curp, cur, sp, Mb, sp, om1);
                    conv(P(5), EPI_SHUFFLE, Mb, sp, sp, T[1], st, ot);
                    ot.bytes -= (double)B * sp.H * sp.W * sm.C * es;    // reads only the extension half
                    conv(P(3), EPI_RESUNPOOL, T[1], st, so, dst, so, o2);
                    o2.a.res = Mb; o2.a.resH = sp.H; o2.a.resW = sp.W; o2.a.resC = b.attrs[1]; o2.a.resCS = sp.C;
                    o2.a.idx_in = idx[ref]; o2.a.idxCS = cstore(ctx->blocks[ref].attrs[0]);
                    o2.bytes += (double)B * sm.H * sm.W * sm.C * es + (double)B * sm.H * sm.W * o2.a.idxCS;
                    ops.push_back(om1); ops.push_back(ot); ops.push_back(o2);
                } else if (fill) {
                    Op om, o1, ot, o2;
                    conv(P(0), EPI_PLAIN, curp, cur, sm, Mb, sm, om);
                    conv(P(1), EPI_PLAIN, curp, cur, s1, T[0], s1, o1);
                    conv(P(2), EPI_SHUFFLE, T[0], s1, s1, T[1], st, ot);
                    conv(P(3), EPI_RESUNPOOL, T[1], st, so, dst, so, o2);
                    o2.a.res = Mb; o2.a.resH = sm.H; o2.a.resW = sm.W; o2.a.resC = b.attrs[1]; o2.a.resCS = sm.C;
                    o2.a.idx_in = idx[ref]; o2.a.idxCS = cstore(ctx->blocks[ref].attrs[0]);
                    o2.bytes += (double)B * sm.H * sm.W * sm.C * es + (double)B * sm.H * sm.W * o2.a.idxCS;
                    ops.push_back(om); ops.push_back(o1); ops.push_back(ot); ops.push_back(o2);
                }
                cur = so;
                break;
            }
            case BT_FULLCONV: {
                Shape so{cur.H * 2, cur.W * 2, P(0).cout};
                if (so.H != H || so.W != W) { why = "network does not return to the input resolution"; return false; }
                if (fill) {
                    Op op;
                    conv(P(0), EPI_CLASSES, curp, cur, cur, nullptr, so, op);
                    op.a.ncls = ctx->ncls;
                    ops.push_back(op);
                }
                cur = so;
                break;
            }
            }
            if (b.type != BT_FULLCONV) {
                curp = dst;
                xi ^= 1;
            }
        }
        return true;
    }
};

// Derived launch fields (conv_kernels.hip): magic divisors, buffer-descriptor sizes (every tensor
// must be addressable with 31-bit byte offsets), the staging shift. false: a tensor is too large.
bool finish_conv_args(ConvArgs &a, int epi, size_t es) {
    fastdiv((uint32_t)(a.Hg * a.Wg), a.mHWg, a.sHWg);
    fastdiv((uint32_t)a.Wg, a.mWg, a.sWg);
    const double in_b = (double)a.B * a.Hin * a.Win * a.CinS * es;
    const double out_b = epi == EPI_CLASSES ? 0.0 : (double)a.B * a.Hout * a.Wout * a.outC * es;
    const double res_b = a.res ? (double)a.B * a.resH * a.resW * a.resCS * es : 0.0;
    const double idx_b = a.idx_out ? (double)a.M * a.idxCS : a.idx_in ? (double)a.B * a.resH * a.resW * a.idxCS : 0.0;
    const double lim = 2147483648.0;
    if (in_b >= lim || out_b >= lim || res_b >= lim || idx_b >= lim ||
        (epi == EPI_CLASSES && (double)a.B * a.Hout * a.Wout * a.ncls * 4.0 >= 4.0 * lim))
        return false;
    a.in_bytes = (uint32_t)in_b; a.out_bytes = (uint32_t)out_b;
    a.res_bytes = (uint32_t)res_b; a.idx_bytes = (uint32_t)idx_b;
    const int epc = 16 / (int)es, cpr = a.outC / epc;
    a.cpr_sh = -1;
    if (a.outC % epc == 0 && cpr > 0 && (cpr & (cpr - 1)) == 0)
        for (a.cpr_sh = 0; (1 << a.cpr_sh) < cpr; ++a.cpr_sh) {}
    a.stage_ok = a.cpr_sh >= 0 && (epi != EPI_SHUFFLE || (a.Wg % 16 == 0 && a.M % 16 == 0));
    return true;
}

bool build_plan(bugseg_ctx *ctx, int B, int H, int W, std::string &why, void *stream = nullptr) {
    Plan &pl = ctx->plan;
    if (pl.arena && pl.B == B && pl.H == H && pl.W == W) return true;
    Walker w{ctx, B, H, W};
    if (!w.run(false, why)) return false;
    auto al = [](size_t v) { return (v + 4095) / 4096 * 4096; };
    size_t total = 2 * al(w.szX) + 3 * al(w.szT) + al(w.szM);
    for (size_t s : w.szIdx) total += al(s);
    const size_t words_bytes = ctx->prec == PREC_F32 ? (size_t)Walker::max_words(ctx->blocks.size()) * RNG_SLOTS * 4 : 0;
    total += al(words_bytes);
    const bool cap = stream_capturing(stream);
    RelaxCapture relax;                 // the first forward at a shape may itself be captured
    if (pl.arena) {
        // a forward of the old shape may still be running (or be part of a captured graph)
        retire(ctx, pl.arena, cap || pl.pinned);
        pl.arena = nullptr;
        pl.pinned = false;
    }
    if (hipMalloc(&pl.arena, total) != hipSuccess) { why = "hipMalloc of the activation arena failed"; pl.arena = nullptr; return false; }
    unsigned char *p = (unsigned char *)pl.arena;
    w.X[0] = p; p += al(w.szX);
    w.X[1] = p; p += al(w.szX);
    for (int i = 0; i < 3; ++i) { w.T[i] = p; p += al(w.szT); }
    w.Mb = p; p += al(w.szM);
    w.idx.assign(w.szIdx.size(), nullptr);
    for (size_t i = 0; i < w.szIdx.size(); ++i) if (w.szIdx[i]) { w.idx[i] = p; p += al(w.szIdx[i]); }
    w.words = words_bytes ? (float *)p : nullptr;
    p += al(words_bytes);
    if (!w.run(true, why)) return false;
    if (words_bytes && w.nwords > Walker::max_words(ctx->blocks.size())) { why = "range words: plan too long"; return false; }
    for (Op &op : w.ops) {
        if (op.kind == 1) {
            const double bytes = (double)op.bn.B * op.bn.H * op.bn.W * op.bn_c * w.es;
            const double in_bytes = op.bn_cin ? 4.0 * op.bn.B * op.bn.H * op.bn.W * op.bn_cin * w.es : 0.0;
            if (bytes >= 2147483648.0 || in_bytes >= 2147483648.0) { why = "batch too large for 32-bit tensor offsets"; return false; }
            op.bn.x_bytes = (uint32_t)bytes;
            continue;
        }
        if (!finish_conv_args(op.a, op.epi, w.es)) { why = "batch too large for 32-bit tensor offsets"; return false; }
    }
    pl.ops = std::move(w.ops);
    pl.cls_ok = false;
    pl.cls_on = false;
    if (pl.ops.size() >= 2) {
        const Op &l = pl.ops.back(), &q = pl.ops[pl.ops.size() - 2];
        const char *fe = std::getenv("BUGSEG_CLS_FUSE");
        pl.cls_ok = fe && *fe == '1' && l.kind == 0 && l.epi == EPI_CLASSES && cls_supported(l.a) &&
                    !std::getenv("BUGSEG_CLS_CONV") && q.kind == 1 && q.bn_c == 16 && !q.bn_asym && q.bn_cin == 0 &&
                    q.bn.dt == 1 && q.bn.phases == 1 && q.bn.out == l.a.in && l.a.B == q.bn.B && l.a.Hin == q.bn.H &&
                    l.a.Win == q.bn.W && (double)B * l.a.Hout * l.a.Wout < 2147483648.0;
    }
    pl.idx = w.idx;
    pl.idx_bytes = w.szIdx;
    pl.words = w.words;
    pl.words_bytes = words_bytes;
    pl.B = B; pl.H = H; pl.W = W;
    pl.arena_bytes = total;
    return true;
}

// ---------------------------------------------------------------- preprocess tables
void linear_coeffs(int dsize, int ssize, double scale, int *ofs, short *a01) {
#pragma clang fp contract(off)
    for (int d = 0; d < dsize; ++d) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)std::floor(f);
        f -= (float)s;
        if (s < 0) { f = 0.f; s = 0; }
        if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
        ofs[d] = s;
        long v0 = std::lrintf((1.f - f) * 2048.f), v1 = std::lrintf(f * 2048.f);
        a01[2 * d] = (short)std::min(32767L, std::max(-32768L, v0));
        a01[2 * d + 1] = (short)std::min(32767L, std::max(-32768L, v1));
    }
}

}  // namespace

// =============================================================== C ABI
extern "C" {

int bugseg_version(void) { return 100; }

const char *bugseg_last_error(const bugseg_ctx *ctx) { return ctx ? ctx->err.c_str() : g_thread_err.c_str(); }

int bugseg_create(int device, int precision, bugseg_ctx **out) {
    if (!out) return fail(nullptr, BUGSEG_EINVAL, "out is NULL");
    *out = nullptr;
    if (precision != BUGSEG_FP32 && precision != BUGSEG_BF16 && precision != BUGSEG_F16)
        return fail(nullptr, BUGSEG_EINVAL, "precision must be BUGSEG_FP32, BUGSEG_BF16 or BUGSEG_F16");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(nullptr, BUGSEG_EINVAL, "no such HIP device: " + std::to_string(device));
    bugseg_ctx *c = new (std::nothrow) bugseg_ctx();
    if (!c) return fail(nullptr, BUGSEG_ENOMEM, "out of host memory");
    c->device = device;
    c->prec = precision == BUGSEG_BF16 ? PREC_BF16 : precision == BUGSEG_F16 ? PREC_F16 : PREC_F32;
    DeviceGuard g(device);
    // class remap tables (models.py:56-58 and :79-80) + the normalisation table (models.py:17-18, 91)
    unsigned char tab[32 + 3 * 256 * 8];
    const uint8_t lut3[16] = {1, 1, 0, 2, 2, 2, 2, 2, 2, 0, 2, 2, 2, 2, 2, 2};
    const uint8_t lutb[16] = {1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    std::memcpy(tab, lut3, 16);
    std::memcpy(tab + 16, lutb, 16);
    const double mean[3] = {0.485, 0.456, 0.406}, stdv[3] = {0.229, 0.224, 0.225};
    for (int ch = 0; ch < 3; ++ch)
        for (int v = 0; v < 256; ++v) {
            const double x = ((double)v / 256.0 - mean[ch]) / stdv[ch];
            std::memcpy(tab + 32 + (ch * 256 + v) * 8, &x, 8);
            c->norm_amax = std::max(c->norm_amax, (float)std::fabs(x) * 1.0001f);
        }

    {
        // uploaded on the context's private stream (never the legacy stream, which would join a capture
        // in progress on another stream), so a context may be created while a stream is capturing
        RelaxCapture relax;
        hipStream_t s = setup_stream(c);
        hipError_t e = s ? hipMalloc(&c->dev_luts, sizeof(tab)) : hipErrorInvalidValue;
        if (e == hipSuccess) e = hipMemcpyAsync(c->dev_luts, tab, sizeof(tab), hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        // bf16 / fp16: the fused initial block evaluates the table as one fmaf per byte when an f32
        // pair (a, b) near (1 / (256 std), -mean / std) reproduces all 256 stored values of a channel
        // bit for bit (searched on the device, with its own conversions: init_kernels.hip
        // naff_search_kernel) — no LDS lookups, whose data-dependent addresses conflict; fp32 keeps
        // the table. BUGSEG_INIT_TABLE=1 forces the table (A/B)
        if (e == hipSuccess && c->prec != PREC_F32) {
            float base[6];
            for (int ch = 0; ch < 3; ++ch) {
                base[ch] = (float)(1.0 / (256.0 * stdv[ch]));
                base[3 + ch] = (float)(-mean[ch] / stdv[ch]);
            }
            constexpr int N = 2 * NAFF_R + 1;
            std::vector<uint8_t> okh((size_t)3 * N * N);
            uint8_t *okd = nullptr;
            hipError_t e2 = hipMalloc(&okd, okh.size());
            if (e2 == hipSuccess) e2 = launch_naff_search(c->prec, (const double *)((const unsigned char *)c->dev_luts + 32), base, okd, s);
            if (e2 == hipSuccess) e2 = hipMemcpyAsync(okh.data(), okd, okh.size(), hipMemcpyDeviceToHost, s);
            if (e2 == hipSuccess) e2 = hipStreamSynchronize(s);
            if (okd) (void)hipFree(okd);
            bool all = e2 == hipSuccess;
            for (int ch = 0; ch < 3 && all; ++ch) {
                int best = -1, bestd = 1 << 30;
                for (int k = 0; k < N * N; ++k) {
                    const int da = k / N - NAFF_R, db = k % N - NAFF_R, d = std::max(std::abs(da), std::abs(db));
                    if (okh[(size_t)ch * N * N + k] && d < bestd) { best = k; bestd = d; }
                }
                if (best < 0) { all = false; break; }
                int32_t ia, ib;
                std::memcpy(&ia, &base[ch], 4);
                std::memcpy(&ib, &base[3 + ch], 4);
                ia += best / N - NAFF_R;
                ib += best % N - NAFF_R;
                std::memcpy(&c->naff[ch], &ia, 4);
                std::memcpy(&c->naff[3 + ch], &ib, 4);
            }
            c->naff_on = all;
        }
        if (e != hipSuccess) {
            if (c->dev_luts) (void)hipFree(c->dev_luts);
            if (c->setup) (void)hipStreamDestroy(c->setup);
            delete c;
            return fail(nullptr, BUGSEG_EHIP, std::string("device allocation failed: ") + hipGetErrorString(e));
        }
    }
    *out = c;
    return BUGSEG_OK;
}

int bugseg_destroy(bugseg_ctx *ctx) {
    if (!ctx) return BUGSEG_OK;
    DeviceGuard g(ctx->device);
    (void)hipDeviceSynchronize();
    if (ctx->dev_w) (void)hipFree(ctx->dev_w);
    if (ctx->dev_luts) (void)hipFree(ctx->dev_luts);
    if (ctx->plan.arena) (void)hipFree(ctx->plan.arena);
    for (auto &t : ctx->pre_tabs) if (t.tab) (void)hipFree(t.tab);
    for (auto &t : ctx->polar_tabs) if (t.tab) (void)hipFree(t.tab);
    for (auto &s : ctx->ls_scratch) if (s.p) (void)hipFree(s.p);
    for (auto &t : ctx->bev_tabs) if (t.tab) (void)hipFree(t.tab);
    for (void *p : ctx->graveyard) (void)hipFree(p);
    if (ctx->setup) (void)hipStreamDestroy(ctx->setup);
    delete ctx;
    return BUGSEG_OK;
}

int bugseg_load_weights(bugseg_ctx *ctx, const void *blob, size_t bytes) {
    if (!ctx || !blob) return fail(ctx, BUGSEG_EINVAL, "NULL argument");
    DeviceGuard g(ctx->device);
    std::vector<BlockDesc> blocks;
    int ncls = 0;
    std::string why;
    if (!parse_blob(blob, bytes, blocks, ncls, why)) return fail(ctx, BUGSEG_EFORMAT, "weight blob: " + why);
    ctx->blocks = std::move(blocks);
    ctx->ncls = ncls;
    ctx->loaded = false;
    {
        const char *off = std::getenv("BUGSEG_F32_RANGE");
        ctx->range_off = off && *off == '0';
    }
    if (!pack_all(ctx, why)) return fail(ctx, BUGSEG_EFORMAT, "weight blob: " + why);
    (void)hipDeviceSynchronize();
    if (ctx->dev_w) {
        // a captured graph's kernels hold pointers into the old weights (and arena): kept until destroy
        if (ctx->plan.pinned) ctx->graveyard.push_back(ctx->dev_w);
        else (void)hipFree(ctx->dev_w);
        ctx->dev_w = nullptr;
    }
    if (ctx->plan.arena) {
        if (ctx->plan.pinned) ctx->graveyard.push_back(ctx->plan.arena);   // a captured graph may use it
        else (void)hipFree(ctx->plan.arena);
        ctx->plan = Plan();
    }
    if (hipMalloc(&ctx->dev_w, ctx->host_w.size()) != hipSuccess ||
        hipMemcpy(ctx->dev_w, ctx->host_w.data(), ctx->host_w.size(), hipMemcpyHostToDevice) != hipSuccess)
        return fail(ctx, BUGSEG_EHIP, "uploading weights failed");
    ctx->loaded = true;
    return BUGSEG_OK;
}

int bugseg_num_classes(const bugseg_ctx *ctx) { return ctx && ctx->loaded ? ctx->ncls : 0; }

size_t bugseg_input_bytes(const bugseg_ctx *ctx, int B, int H, int W) {
    if (!ctx || B <= 0 || H <= 0 || W <= 0) return 0;
    return (size_t)B * H * W * 8 * prec_es(ctx->prec);
}

int bugseg_preprocess(bugseg_ctx *ctx, const uint8_t *bgr, int B, int H0, int W0, int H, int W, int out_layout,
                      void *out, void *stream) {
    if (!ctx || !bgr || !out) return fail(ctx, BUGSEG_EINVAL, "NULL argument");
    if (B <= 0 || H0 <= 0 || W0 <= 0 || H <= 0 || W <= 0) return fail(ctx, BUGSEG_EINVAL, "bad shape");
    if (out_layout < BUGSEG_PRE_ENGINE || out_layout > BUGSEG_PRE_BGR_U8) return fail(ctx, BUGSEG_EINVAL, "bad out_layout");
    DeviceGuard g(ctx->device);
    PreArgs a;
    std::memset(&a, 0, sizeof(a));
    a.bgr = bgr; a.B = B; a.H0 = H0; a.W0 = W0; a.H = H; a.W = W;
    a.lut = (const double *)((const unsigned char *)ctx->dev_luts + 32);
    a.out_layout = out_layout; a.prec = ctx->prec; a.out = out;
    a.vec_end = W * 3 - (W * 3) % 8;
    if (H0 == H && W0 == W) {
        a.mode = 0;
    } else {
        const double sx = 1.0 / ((double)W / W0), sy = 1.0 / ((double)H / H0);
        const int isx = (int)std::lrint(sx), isy = (int)std::lrint(sy);
        const double eps = 2.220446049250313e-16;
        if (std::fabs(sx - isx) < eps && std::fabs(sy - isy) < eps && isx == 2 && isy == 2) {
            a.mode = 1;
        } else {
            a.mode = 2;
            const int key[4] = {H0, W0, H, W};
            const size_t need = (size_t)W * 4 + (size_t)W * 4 + (size_t)H * 4 + (size_t)H * 4;
            const bool cap = stream_capturing(stream);
            bugseg_ctx::PreTab *hit = nullptr;
            for (auto &t : ctx->pre_tabs)
                if (std::memcmp(t.key, key, sizeof(key)) == 0) hit = &t;
            if (!hit) {
                std::vector<unsigned char> h(need);
                int *xo = (int *)h.data();
                short *xa = (short *)(h.data() + (size_t)W * 4);
                int *yo = (int *)(h.data() + (size_t)W * 8);
                short *yb = (short *)(h.data() + (size_t)W * 8 + (size_t)H * 4);
                linear_coeffs(W, W0, sx, xo, xa);
                linear_coeffs(H, H0, sy, yo, yb);
                if (ctx->pre_tabs.size() >= 4) {            // keep 4 geometries: evict the oldest unpinned one
                    for (size_t i = 0; i < ctx->pre_tabs.size(); ++i)
                        if (!ctx->pre_tabs[i].pinned) {
                            // work enqueued on any stream may still read it: retire syncs (or defers)
                            retire(ctx, ctx->pre_tabs[i].tab, cap);
                            ctx->pre_tabs.erase(ctx->pre_tabs.begin() + (long)i);
                            break;
                        }
                }
                // built on the private stream and waited for there, so the caller's stream is never
                // synchronised and a capture in progress on it stays valid
                bugseg_ctx::PreTab t;
                std::memcpy(t.key, key, sizeof(key));
                RelaxCapture relax;
                hipStream_t st = setup_stream(ctx);
                hipError_t e = st ? hipMalloc(&t.tab, need) : hipErrorInvalidValue;
                if (e == hipSuccess) e = hipMemcpyAsync(t.tab, h.data(), need, hipMemcpyHostToDevice, st);
                if (e == hipSuccess) e = hipStreamSynchronize(st);
                if (e != hipSuccess) {
                    if (t.tab) (void)hipFree(t.tab);
                    return fail(ctx, BUGSEG_EHIP, std::string("resize table upload failed: ") + hipGetErrorString(e));
                }
                ctx->pre_tabs.push_back(t);
                hit = &ctx->pre_tabs.back();
            }
            if (cap) hit->pinned = true;
            unsigned char *t = (unsigned char *)hit->tab;
            a.xofs = (const int *)t;
            a.xa = (const short *)(t + (size_t)W * 4);
            a.yofs = (const int *)(t + (size_t)W * 8);
            a.yb = (const short *)(t + (size_t)W * 8 + (size_t)H * 4);
        }
    }
    hipError_t e = launch_preprocess(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ctx, BUGSEG_EHIP, std::string("preprocess launch: ") + hipGetErrorString(e));
    return BUGSEG_OK;
}

int bugseg_nchw_to_input(bugseg_ctx *ctx, const void *x, int is_f64, int B, int H, int W, void *out, void *stream) {
    if (!ctx || !x || !out) return fail(ctx, BUGSEG_EINVAL, "NULL argument");
    if (B <= 0 || H <= 0 || W <= 0) return fail(ctx, BUGSEG_EINVAL, "bad shape");
    DeviceGuard g(ctx->device);
    NchwArgs a{x, is_f64 ? 1 : 0, B, H, W, ctx->prec, out};
    hipError_t e = launch_nchw_to_input(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ctx, BUGSEG_EHIP, std::string("layout launch: ") + hipGetErrorString(e));
    return BUGSEG_OK;
}

// the class-fused launch's arguments (Plan::cls_ok): the last bottleneck's, 15 x 15-strided 16 x 16
// tiles, no block output or range words written, the class op's weights / bias / output / LUT
static BneckArgs cls_fused_args(const Plan &pl) {
    const Op &q = pl.ops[pl.ops.size() - 2], &l = pl.ops.back();
    BneckArgs a = q.bn;
    a.rg.amax_out = nullptr;
    a.tr = 0;
    a.tiles_y = (a.H + 14) / 15;
    a.tiles_x = (a.W + 14) / 15;
    a.ntiles = a.B * a.tiles_y * a.tiles_x;
    a.cw = l.a.w;
    a.cbias = l.a.bias;
    a.cls_out = l.a.cls_out;
    a.cls_bytes = (uint32_t)((size_t)l.a.B * l.a.Hout * l.a.Wout);
    a.lut = l.a.lut;
    a.lut_kind = l.a.lut_kind;
    a.ncls = l.a.ncls;
    a.csw = l.a.rg.sw[0];
    return a;
}

// one plan op, with its launch-span slots when bugseg_debug_set_spans armed them
static hipError_t launch_op(const bugseg_ctx *ctx, int i, hipStream_t s) {
    const Plan &pl = ctx->plan;
    const Op &o = pl.ops[(size_t)i];
    unsigned long long *sp = ctx->spans && i < ctx->spans_ops ? ctx->spans + 512 * (size_t)i : nullptr;   // (mfma_common.h: 64 slots x 64 B)
    if (pl.cls_on && i + 2 == (int)pl.ops.size()) { BneckArgs q = cls_fused_args(pl); q.span = sp; return launch_bneck_cls(ctx->prec, q, s); }
    if (pl.cls_on && i + 1 == (int)pl.ops.size()) return hipSuccess;   // (ran within op i - 1)
    if (o.kind == 1) { BneckArgs q = o.bn; q.span = sp; return launch_bneck(ctx->prec, o.bn_c, o.bn_asym, o.bn_var, q, s, o.bn_cin); }
    if (o.kind == 2) { UpArgs q = o.up; q.span = sp; return launch_up(ctx->prec, o.up_cin, o.up_it, o.up_cout, q, s); }
    ConvArgs q = o.a;
    q.span = sp;
    return launch_conv(ctx->prec, o.nr, o.epi, q, s);
}

static int enet_forward(bugseg_ctx *ctx, const void *in, bool bgr, int B, int H, int W, int out_kind, void *out,
                        void *stream, int first_op = 0, int last_op = -1) {
    if (!ctx || !in || !out) return fail(ctx, BUGSEG_EINVAL, "NULL argument");
    if (!ctx->loaded) return fail(ctx, BUGSEG_ESTATE, "no weights loaded");
    if (out_kind < BUGSEG_OUT_LOGITS_F32 || out_kind > BUGSEG_OUT_BINARY_U8) return fail(ctx, BUGSEG_EINVAL, "bad out_kind");
    DeviceGuard g(ctx->device);
    std::string why;
    if (!build_plan(ctx, B, H, W, why, stream)) return fail(ctx, BUGSEG_EINVAL, why);
    Plan &pl = ctx->plan;
    if (stream_capturing(stream)) pl.pinned = true;
    Op &first = pl.ops.front();
    first.a.in = in;
    first.epi = bgr ? EPI_INIT_BGR : EPI_INIT;
    first.a.nlut = bgr ? (const double *)((const unsigned char *)ctx->dev_luts + 32) : nullptr;
    first.a.naff_on = bgr && ctx->naff_on && !std::getenv("BUGSEG_INIT_TABLE");
    std::memcpy(first.a.naff, ctx->naff, sizeof(ctx->naff));
    // fp32 range scaling: the BGR input's range is the normalisation table's (static); an engine input
    // the caller supplied is measured (block 0 of the range words)
    first.a.rg.amax_in = bgr ? nullptr : pl.words;
    first.a.rg.amax_static = bgr ? ctx->norm_amax : 0.f;
    ConvArgs &last = pl.ops.back().a;
    last.cls_out = nullptr; last.logits_out = nullptr; last.lut = nullptr; last.lut_kind = 0;
    const uint8_t *luts = (const uint8_t *)ctx->dev_luts;
    switch (out_kind) {
    case BUGSEG_OUT_LOGITS_F32: last.logits_out = (float *)out; break;
    case BUGSEG_OUT_CLASS15_U8: last.cls_out = (uint8_t *)out; break;
    case BUGSEG_OUT_CLASS3_U8: last.cls_out = (uint8_t *)out; last.lut = luts; last.lut_kind = 1; break;
    case BUGSEG_OUT_BINARY_U8: last.cls_out = (uint8_t *)out; last.lut = luts + 16; last.lut_kind = 2; break;
    }
    const int nops = (int)pl.ops.size();
    if (last_op < 0 || last_op > nops) last_op = nops;
    if (first_op < 0 || first_op > last_op) return fail(ctx, BUGSEG_EINVAL, "bad op range");
    if (pl.words && first_op == 0) {
        // every launch max-accumulates its output's range: cleared once per forward (a memset node when captured)
        hipError_t e = hipMemsetAsync(pl.words, 0, pl.words_bytes, (hipStream_t)stream);
        if (e == hipSuccess && !bgr) e = launch_amax((const float *)in, (size_t)B * H * W * 8, pl.words, (hipStream_t)stream);
        if (e != hipSuccess) return fail(ctx, BUGSEG_EHIP, std::string("range words: ") + hipGetErrorString(e));
    }
    pl.cls_on = pl.cls_ok && out_kind != BUGSEG_OUT_LOGITS_F32 && first_op <= nops - 2 && last_op == nops;
    for (int i = first_op; i < last_op; ++i) {
        hipError_t e = launch_op(ctx, i, (hipStream_t)stream);
        if (e != hipSuccess) return fail(ctx, BUGSEG_EHIP, "conv launch " + std::to_string(i) + ": " + hipGetErrorString(e));
    }
    return BUGSEG_OK;
}

int bugseg_enet_forward(bugseg_ctx *ctx, const void *in, int B, int H, int W, int out_kind, void *out, void *stream) {
    return enet_forward(ctx, in, false, B, H, W, out_kind, out, stream);
}

int bugseg_enet_forward_bgr(bugseg_ctx *ctx, const uint8_t *bgr, int B, int H, int W, int out_kind, void *out,
                            void *stream) {
    return enet_forward(ctx, bgr, true, B, H, W, out_kind, out, stream);
}

int bugseg_enet_forward_bgr_ops(bugseg_ctx *ctx, const uint8_t *bgr, int B, int H, int W, int out_kind, void *out,
                                int first_op, int last_op, void *stream) {
    return enet_forward(ctx, bgr, true, B, H, W, out_kind, out, stream, first_op, last_op);
}

}  // extern "C"

namespace {

// ---- laserscan-like mode: cv::warpPolar's remap tables (imgwarp.cpp 4.x), built on the host once
// per geometry. Forward: polar (rho, phi) -> grid cell, phi the row of a ph x pw polar image,
// x = (float)(rho*Kmag) * cos(Kangle*phi) + cx in double, rounded to float, then half-to-even to a
// short (remap INTER_NEAREST). Inverse: grid cell -> (rho, polar row) through hal::magnitude32f /
// fastAtan32f (the AVX2 dispatch: fused polynomial) on float offsets, the BORDER_WRAP row of
// copyMakeBorder folded into the row index. -1 = outside (BORDER_TRANSPARENT).
#pragma clang fp contract(off)
const float kAtanP1 = 0.9997878412794807f * (float)(180 / 3.1415926535897932384626433832795);
const float kAtanP3 = -0.3258083974640975f * (float)(180 / 3.1415926535897932384626433832795);
const float kAtanP5 = 0.1555786518463281f * (float)(180 / 3.1415926535897932384626433832795);
const float kAtanP7 = -0.04432655554792128f * (float)(180 / 3.1415926535897932384626433832795);

float fast_atan_rad(float y, float x) {
    const float ax = std::fabs(x), ay = std::fabs(y);
    const float c = std::min(ax, ay) / (std::max(ax, ay) + (float)2.220446049250313e-16);
    const float cc = c * c;
    float a = std::fma(std::fma(std::fma(cc, kAtanP7, kAtanP5), cc, kAtanP3), cc, kAtanP1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a * (float)(3.1415926535897932384626433832795 / 180);
}

int round_short(float v) {
    const long r = std::lrint(v);
    return (int)(r < -32768 ? -32768 : r > 32767 ? 32767 : r);
}

void polar_tables(int pw, int ph, double max_radius, float cx, float cy, int w, int h, std::vector<int32_t> &fmap,
                  std::vector<int32_t> &imap) {
    const double CV_2PI = 6.283185307179586476925286766559;
    const double Kangle = CV_2PI / ph, Kmag = max_radius / pw;
    fmap.resize((size_t)pw * ph);
    for (int phi = 0; phi < ph; ++phi) {
        const double KKy = Kangle * phi, cp = std::cos(KKy), sp = std::sin(KKy);
        for (int rho = 0; rho < pw; ++rho) {
            const float r = (float)(rho * Kmag);
            const float mx = (float)(r * cp + (double)cx), my = (float)(r * sp + (double)cy);
            const int sx = round_short(mx), sy = round_short(my);
            fmap[(size_t)phi * pw + rho] = ((unsigned)sx < (unsigned)w && (unsigned)sy < (unsigned)h) ? (sx | (sy << 16)) : -1;
        }
    }
    imap.resize((size_t)w * h);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const float bx = (float)x - cx, by = (float)y - cy;
            const float mag = std::sqrt(std::fma(bx, bx, by * by));
            const float ang = fast_atan_rad(by, bx);
            const double rho = mag / Kmag, phi = ang / Kangle;
            const float mx = (float)rho, my = (float)phi + 1;
            const int X = round_short(mx), Y = round_short(my);
            int32_t v = -1;
            if ((unsigned)X < (unsigned)pw && (unsigned)Y < (unsigned)(ph + 2)) {
                const int row = Y == 0 ? ph - 1 : (Y == ph + 1 ? 0 : Y - 1);
                v = X | (row << 16);
            }
            imap[(size_t)y * w + x] = v;
        }
}
#pragma clang fp contract(on)

// warpPolar dsize: (-1, -1) -> (round(L), round(L*pi)) for create_occupancy_grid (bev.py:219); the
// explicit (w, h) of create_occupancy_grid_binary (bev.py:146). False if the tables cannot hold it.
bool polar_dims(const bugseg_bev_params *p, int &pw, int &ph) {
    const int w = p->occ_w, h = p->occ_h, L = std::max(w, h);
    pw = p->variant ? w : (int)std::lrint((double)L);
    ph = p->variant ? h : (int)std::lrint((double)L * 3.1415926535897932384626433832795);
    return pw > 0 && ph > 0 && pw <= 32767 && ph <= 32767 && w <= 32767 && h <= 32767;
}

// Laserscan batch scratch: cells (B*occ_h*occ_w u8, 256-B aligned) then rmin (B*ph int32).
size_t ls_cells_bytes(int B, const bugseg_bev_params *p) { return ((size_t)B * p->occ_w * p->occ_h + 255) & ~(size_t)255; }
size_t ls_workspace_bytes(int B, const bugseg_bev_params *p, int ph) {
    return ls_cells_bytes(B, p) + (size_t)B * ph * sizeof(int32_t);
}

// The polar tables of a laserscan call (built once per grid geometry on the setup stream, waited
// for there); fills a.fmap / imap / pw / ph / hit.
int prepare_polar(bugseg_ctx *ctx, const bugseg_bev_params *p, BevArgs &a, bool cap) {
    const int w = p->occ_w, h = p->occ_h, L = std::max(w, h);
    int pw, ph;
    if (!polar_dims(p, pw, ph)) return fail(ctx, BUGSEG_EINVAL, "laserscan grid too large for the polar tables");
    bugseg_ctx::PolarTab *hit = nullptr;
    for (auto &t : ctx->polar_tabs)
        if (t.key[0] == w && t.key[1] == h && t.key[2] == p->variant) hit = &t;
    if (!hit) {
        std::vector<int32_t> fmap, imap;
        polar_tables(pw, ph, (double)L, (float)(w / 2.0 - 1), (float)h, w, h, fmap, imap);
        if (ctx->polar_tabs.size() >= 4) {            // keep 4 geometries: evict the oldest unpinned one
            for (size_t i = 0; i < ctx->polar_tabs.size(); ++i)
                if (!ctx->polar_tabs[i].pinned) {
                    retire(ctx, ctx->polar_tabs[i].tab, cap);
                    ctx->polar_tabs.erase(ctx->polar_tabs.begin() + (long)i);
                    break;
                }
        }
        RelaxCapture relax;
        hipStream_t s = setup_stream(ctx);
        if (!s) return fail(ctx, BUGSEG_EHIP, "could not create the table-build stream");
        bugseg_ctx::PolarTab t;
        t.key[0] = w; t.key[1] = h; t.key[2] = p->variant;
        t.pw = pw; t.ph = ph;
        const size_t bytes = (fmap.size() + imap.size()) * sizeof(int32_t);
        if (hipMalloc(&t.tab, bytes) != hipSuccess) return fail(ctx, BUGSEG_ENOMEM, "polar table allocation failed");
        hipError_t e = hipMemcpyAsync(t.tab, fmap.data(), fmap.size() * 4, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync((int32_t *)t.tab + fmap.size(), imap.data(), imap.size() * 4, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            (void)hipFree(t.tab);
            return fail(ctx, BUGSEG_EHIP, std::string("polar table upload: ") + hipGetErrorString(e));
        }
        ctx->polar_tabs.push_back(t);
        hit = &ctx->polar_tabs.back();
    }
    if (cap) hit->pinned = true;
    a.laserscan = 1;
    a.fmap = (const int32_t *)hit->tab;
    a.imap = (const int32_t *)hit->tab + (size_t)pw * ph;
    a.pw = pw; a.ph = ph;
    a.hit = p->variant ? 100 : 3;
    return BUGSEG_OK;
}

// The scratch-owning entry's per-stream laserscan scratch (bugseg_bev_occgrid without a workspace).
int internal_scratch(bugseg_ctx *ctx, void *stream, size_t need, bool cap, void *&out) {
    bugseg_ctx::LsScratch *sc = nullptr;
    for (auto &x : ctx->ls_scratch) if (x.stream == stream) sc = &x;
    if (!sc) {
        if (ctx->ls_scratch.size() >= 8) {            // 8 streams: evict the least recently used unpinned one
            long victim = -1;
            for (size_t i = 0; i < ctx->ls_scratch.size(); ++i)
                if (!ctx->ls_scratch[i].pinned && (victim < 0 || ctx->ls_scratch[i].used < ctx->ls_scratch[(size_t)victim].used))
                    victim = (long)i;
            if (victim >= 0) {
                retire(ctx, ctx->ls_scratch[(size_t)victim].p, cap);
                ctx->ls_scratch.erase(ctx->ls_scratch.begin() + victim);
            }
        }
        ctx->ls_scratch.push_back(bugseg_ctx::LsScratch());
        sc = &ctx->ls_scratch.back();
        sc->stream = stream;
    }
    sc->used = ++ctx->use_clock;
    if (need > sc->bytes) {
        // work already enqueued on this stream (or captured from it) may still use the old buffer
        retire(ctx, sc->p, cap || sc->pinned);
        sc->p = nullptr;
        sc->bytes = 0;
        RelaxCapture relax;
        if (hipMalloc(&sc->p, need) != hipSuccess) return fail(ctx, BUGSEG_ENOMEM, "laserscan scratch allocation failed");
        sc->bytes = need;
    }
    if (cap) sc->pinned = true;
    out = sc->p;
    return BUGSEG_OK;
}

int bev_occgrid(bugseg_ctx *ctx, const uint8_t *seg, int B, const bugseg_bev_params *p, int8_t *out, bool own_ws,
                void *ws, size_t ws_bytes, void *stream) {
    if (!ctx || !seg || !p || !out) return fail(ctx, BUGSEG_EINVAL, "NULL argument");
    if (B <= 0 || p->in_rows <= 0 || p->in_cols <= 0 || p->warp_w <= 0 || p->warp_h <= 0 || p->occ_w <= 0 ||
        p->occ_h <= 0 || p->occ_w_px <= 0 || p->occ_h_px <= 0)
        return fail(ctx, BUGSEG_EINVAL, "bad BEV geometry");
    if (p->variant != 0 && p->variant != 1) return fail(ctx, BUGSEG_EINVAL, "variant must be 0 or 1");
    if (p->laserscan != 0 && p->laserscan != 1) return fail(ctx, BUGSEG_EINVAL, "laserscan must be 0 or 1");
    DeviceGuard g(ctx->device);
    BevArgs a;
    std::memset(&a, 0, sizeof(a));
    a.seg = seg; a.B = B; a.in_rows = p->in_rows; a.in_cols = p->in_cols;
    {
        // cv::invert(M) closed-form 3x3 branch (DECOMP_LU), as warpPerspective does without WARP_INVERSE_MAP
#pragma clang fp contract(off)
        const double *S = p->M;
        double d = S[0] * (S[4] * S[8] - S[5] * S[7]) - S[1] * (S[3] * S[8] - S[5] * S[6]) + S[2] * (S[3] * S[7] - S[4] * S[6]);
        if (d != 0.0) {
            d = 1.0 / d;
            a.Mi[0] = (S[4] * S[8] - S[5] * S[7]) * d;
            a.Mi[1] = (S[2] * S[7] - S[1] * S[8]) * d;
            a.Mi[2] = (S[1] * S[5] - S[2] * S[4]) * d;
            a.Mi[3] = (S[5] * S[6] - S[3] * S[8]) * d;
            a.Mi[4] = (S[0] * S[8] - S[2] * S[6]) * d;
            a.Mi[5] = (S[2] * S[3] - S[0] * S[5]) * d;
            a.Mi[6] = (S[3] * S[7] - S[4] * S[6]) * d;
            a.Mi[7] = (S[1] * S[6] - S[0] * S[7]) * d;
            a.Mi[8] = (S[0] * S[4] - S[1] * S[3]) * d;
        }
    }
    const int bh0 = std::min(16, p->warp_h);
    a.bw0 = std::min(1024 / bh0, p->warp_w);
    a.warp_w = p->warp_w; a.warp_h = p->warp_h;
    a.occ_w_px = p->occ_w_px; a.occ_h_px = p->occ_h_px; a.occ_w = p->occ_w; a.occ_h = p->occ_h;
    a.left_x = p->left_x; a.top_y = p->top_y;
    a.ifx = 1.0 / ((double)p->occ_w / p->occ_w_px);
    a.ify = 1.0 / ((double)p->occ_h / p->occ_h_px);
    a.ros_layout = p->ros_layout;
    a.variant = p->variant;
    a.out = out;
    if (p->laserscan) {
        // check the workspace before anything is built or enqueued
        int pw, ph;
        if (!polar_dims(p, pw, ph)) return fail(ctx, BUGSEG_EINVAL, "laserscan grid too large for the polar tables");
        if (!own_ws && (!ws || ws_bytes < ls_workspace_bytes(B, p, ph)))
            return fail(ctx, BUGSEG_EINVAL, "laserscan workspace missing or smaller than bugseg_bev_workspace_bytes()");
    }
    const bool cap = stream_capturing(stream);
    {
        // the geometry's warp-tap table: built once on the setup stream and waited for there, then
        // shared read-only by every call on any stream
        std::vector<unsigned char> key(sizeof(double) * 11 + sizeof(int) * 12);
        unsigned char *kp = key.data();
        auto put = [&](const void *v, size_t n) { std::memcpy(kp, v, n); kp += n; };
        put(a.Mi, sizeof(a.Mi)); put(&a.ifx, sizeof(double)); put(&a.ify, sizeof(double));
        const int ik[12] = {a.in_rows, a.in_cols, a.bw0, a.warp_w, a.warp_h, a.occ_w_px, a.occ_h_px, a.occ_w, a.occ_h,
                            a.left_x, a.top_y, 0};
        put(ik, sizeof(ik));
        bugseg_ctx::BevTab *hit = nullptr;
        for (auto &t : ctx->bev_tabs) if (t.key == key) hit = &t;
        if (!hit) {
            const size_t cells = (size_t)a.occ_h * a.occ_w;
            if (cells * BEV_SLOTS > (size_t)1 << 31) return fail(ctx, BUGSEG_EINVAL, "occupancy grid too large");
            if (ctx->bev_tabs.size() >= 4) {            // keep 4 geometries: evict the oldest unpinned one
                for (size_t i = 0; i < ctx->bev_tabs.size(); ++i)
                    if (!ctx->bev_tabs[i].pinned) {
                        retire(ctx, ctx->bev_tabs[i].tab, cap);
                        ctx->bev_tabs.erase(ctx->bev_tabs.begin() + (long)i);
                        break;
                    }
            }
            RelaxCapture relax;
            hipStream_t s = setup_stream(ctx);
            if (!s) return fail(ctx, BUGSEG_EHIP, "could not create the table-build stream");
            bugseg_ctx::BevTab t;
            t.key = key;
            if (hipMalloc(&t.tab, bev_table_bytes(a.occ_w, a.occ_h)) != hipSuccess)
                return fail(ctx, BUGSEG_ENOMEM, "BEV table allocation failed");
            a.wtab = t.tab;
            hipError_t e = launch_bev_table(a, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);   // only the build itself is waited for
            // the band-staged form's work items from the band records: one per (band, row part), the
            // far bands first: with the item-major workgroup order their workgroups (the longest-lived,
            // in-kernel clocks: 20 us at the median against 15 for the near bands) are dispatched first.
            // 26.2 -> 23.7 us per 32 frames against nearest-first (scripts/gpu_r4_far.sh)
            const int nb = bev_bands(a.occ_h);
            std::vector<int4> rec((size_t)nb * BEV_BOXREC);
            std::vector<int2> items;
            if (e == hipSuccess)
                e = hipMemcpyAsync(rec.data(), (unsigned char *)t.tab + bev_records_offset(a.occ_w, a.occ_h),
                                   rec.size() * sizeof(int4), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess) {
                // (BUGSEG_BEV_NEAR_FIRST=1: the earlier order, nearest bands first; A/B)
                const char *nf = std::getenv("BUGSEG_BEV_NEAR_FIRST");
                const bool near_first = nf && std::atoi(nf) != 0;
                for (int i = 0; i < nb; ++i) {
                    const int b = near_first ? nb - 1 - i : i;
                    for (int k = 0; k < std::max(1, std::min(BEV_BAND, rec[(size_t)b * BEV_BOXREC].x)); ++k) items.push_back(make_int2(b, k));
                }
                e = hipMemcpyAsync((unsigned char *)t.tab + bev_items_offset(a.occ_w, a.occ_h), items.data(),
                                   items.size() * sizeof(int2), hipMemcpyHostToDevice, s);
            }
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            t.nitems = (int)items.size();
            if (e != hipSuccess) {
                (void)hipFree(t.tab);
                return fail(ctx, BUGSEG_EHIP, std::string("BEV table: ") + hipGetErrorString(e));
            }

            ctx->bev_tabs.push_back(std::move(t));
            hit = &ctx->bev_tabs.back();
        }
        if (cap) hit->pinned = true;
        a.wtab = hit->tab;
        a.nitems = hit->nitems;
    }
    if (p->laserscan) {
        int rc = prepare_polar(ctx, p, a, cap);
        if (rc != BUGSEG_OK) return rc;
        if (own_ws) {
            rc = internal_scratch(ctx, stream, ls_workspace_bytes(B, p, a.ph), cap, ws);
            if (rc != BUGSEG_OK) return rc;
        }
        a.cells = (uint8_t *)ws;
        a.rmin = (int32_t *)((unsigned char *)ws + ls_cells_bytes(B, p));
    }
    hipError_t e = launch_bev(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ctx, BUGSEG_EHIP, std::string("bev launch: ") + hipGetErrorString(e));
    return BUGSEG_OK;
}

}  // namespace

extern "C" {

int bugseg_bev_occgrid(bugseg_ctx *ctx, const uint8_t *seg, int B, const bugseg_bev_params *p, int8_t *out, void *stream) {
    return bev_occgrid(ctx, seg, B, p, out, true, nullptr, 0, stream);
}

size_t bugseg_bev_workspace_bytes(const bugseg_bev_params *p, int B) {
    int pw, ph;
    if (!p || B <= 0 || p->occ_w <= 0 || p->occ_h <= 0 || !p->laserscan || !polar_dims(p, pw, ph)) return 0;
    return ls_workspace_bytes(B, p, ph);
}

int bugseg_bev_occgrid_ws(bugseg_ctx *ctx, const uint8_t *seg, int B, const bugseg_bev_params *p, int8_t *out,
                          void *workspace, size_t workspace_bytes, void *stream) {
    return bev_occgrid(ctx, seg, B, p, out, false, workspace, workspace_bytes, stream);
}

// ---- test hooks (host only: no device, no HIP call) — tests/asan drives them under ASan + UBSan
int bugseg_debug_parse_pack(const void *blob, size_t bytes, int precision, int *ncls) {
    if (!blob) return fail(nullptr, BUGSEG_EINVAL, "NULL blob");
    bugseg_ctx c;                                     // host state only; nothing to free on the device
    c.prec = precision == BUGSEG_BF16 ? PREC_BF16 : precision == BUGSEG_F16 ? PREC_F16 : PREC_F32;
    std::string why;
    if (!parse_blob(blob, bytes, c.blocks, c.ncls, why)) return fail(nullptr, BUGSEG_EFORMAT, "weight blob: " + why);
    if (!pack_all(&c, why)) return fail(nullptr, BUGSEG_EFORMAT, "weight blob: " + why);
    if (ncls) *ncls = c.ncls;
    return BUGSEG_OK;
}

int bugseg_debug_set_spans(bugseg_ctx *ctx, void *spans, int n_ops) {
    if (!ctx) return fail(ctx, BUGSEG_EINVAL, "NULL ctx");
    if (spans && n_ops <= 0) return fail(ctx, BUGSEG_EINVAL, "spans: n_ops must be positive");
    ctx->spans = (unsigned long long *)spans;
    ctx->spans_ops = spans ? n_ops : 0;
    return BUGSEG_OK;
}

int bugseg_debug_pool_indices(bugseg_ctx *ctx, int B, int H, int W, int block, void *dst, size_t bytes, int *idx_cs,
                              void *stream) {
    if (!ctx || !dst) return fail(ctx, BUGSEG_EINVAL, "NULL argument");
    if (!ctx->loaded) return fail(ctx, BUGSEG_ESTATE, "no weights loaded");
    Plan &pl = ctx->plan;
    if (!pl.arena || pl.B != B || pl.H != H || pl.W != W) return fail(ctx, BUGSEG_ESTATE, "no forward has run at these dimensions");
    if (block < 0 || block >= (int)pl.idx.size() || !pl.idx[(size_t)block])
        return fail(ctx, BUGSEG_EINVAL, "block " + std::to_string(block) + " is not a downsampling block");
    if (bytes != pl.idx_bytes[(size_t)block])
        return fail(ctx, BUGSEG_EINVAL, "index tensor is " + std::to_string(pl.idx_bytes[(size_t)block]) + " bytes");
    if (idx_cs) *idx_cs = cstore(ctx->blocks[(size_t)block].attrs[0]);
    DeviceGuard g(ctx->device);
    hipError_t e = hipMemcpyAsync(dst, pl.idx[(size_t)block], bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ctx, BUGSEG_EHIP, std::string("pool indices copy: ") + hipGetErrorString(e));
    return BUGSEG_OK;
}

int bugseg_debug_ctx_info(const bugseg_ctx *ctx, int what, int arg) {
    if (!ctx) return -1;
    switch (what) {
    case 0: return ctx->naff_on ? 1 : 0;
    case 1: return ctx->range_off ? 1 : 0;
    case 2: return arg >= 0 && arg < (int)ctx->packed.size() ? ctx->packed[(size_t)arg].sw : -1000;
    default: return -1;
    }
}

int bugseg_debug_polar_tables(int w, int h, int variant, int32_t *fmap, size_t fmap_n, int32_t *imap, size_t imap_n,
                              int *pw_out, int *ph_out) {
    if (w <= 0 || h <= 0 || w > 32767 || h > 32767) return fail(nullptr, BUGSEG_EINVAL, "bad grid");
    const int L = std::max(w, h);
    const int pw = variant ? w : (int)std::lrint((double)L);
    const int ph = variant ? h : (int)std::lrint((double)L * 3.1415926535897932384626433832795);
    if (ph > 32767) return fail(nullptr, BUGSEG_EINVAL, "grid too large for the polar tables");
    std::vector<int32_t> f, im;
    polar_tables(pw, ph, (double)L, (float)(w / 2.0 - 1), (float)h, w, h, f, im);
    if (pw_out) *pw_out = pw;
    if (ph_out) *ph_out = ph;
    if (fmap) std::memcpy(fmap, f.data(), std::min(fmap_n, f.size()) * sizeof(int32_t));
    if (imap) std::memcpy(imap, im.data(), std::min(imap_n, im.size()) * sizeof(int32_t));
    return BUGSEG_OK;
}

int bugseg_plan_info(bugseg_ctx *ctx, int B, int H, int W, int out_kind, int bgr_input, int *n_launches, double *alg_bytes,
                     double *plan_bytes, double *flops) {
    if (!ctx) return fail(ctx, BUGSEG_EINVAL, "NULL ctx");
    if (!ctx->loaded) return fail(ctx, BUGSEG_ESTATE, "no weights loaded");
    DeviceGuard g(ctx->device);
    std::string why;
    if (!build_plan(ctx, B, H, W, why)) return fail(ctx, BUGSEG_EINVAL, why);
    double lb = 0, pb = 0, fl = 0;
    for (const Op &op : ctx->plan.ops) {
        pb += op.bytes;
        lb += op.layer_bytes >= 0 ? op.layer_bytes : op.bytes;
        fl += op.flops;
    }
    // final epilogue output
    const double fin = out_kind == BUGSEG_OUT_LOGITS_F32 ? (double)B * H * W * ctx->ncls * 4 : (double)B * H * W;
    // class fusion: the last bottleneck's output is neither written nor read back
    if (ctx->plan.cls_ok && out_kind != BUGSEG_OUT_LOGITS_F32) {
        const Op &q = ctx->plan.ops[ctx->plan.ops.size() - 2];
        pb -= 2.0 * q.bn.B * q.bn.H * q.bn.W * q.bn_c * prec_es(ctx->prec);
    }
    // raw BGR input (bugseg_enet_forward_bgr): 3 bytes per pixel instead of the 8-channel engine input
    double adj = bgr_input ? (double)B * H * W * (8.0 * prec_es(ctx->prec) - 3.0) : 0.0;
    if (n_launches) *n_launches = (int)ctx->plan.ops.size();
    if (alg_bytes) *alg_bytes = lb + fin - adj;
    if (plan_bytes) *plan_bytes = pb + fin - adj;
    if (flops) *flops = fl;
    return BUGSEG_OK;
}

int bugseg_plan_op(bugseg_ctx *ctx, int B, int H, int W, int op, char *kernel, int kernel_len, double *alg_bytes,
                   double *plan_bytes, double *flops) {
    if (!ctx) return fail(ctx, BUGSEG_EINVAL, "NULL ctx");
    if (!ctx->loaded) return fail(ctx, BUGSEG_ESTATE, "no weights loaded");
    Plan &pl = ctx->plan;
    if (!pl.arena || pl.B != B || pl.H != H || pl.W != W) return fail(ctx, BUGSEG_ESTATE, "no forward has run at these dimensions");
    if (op < 0 || op >= (int)pl.ops.size()) return fail(ctx, BUGSEG_EINVAL, "op index out of range");
    const Op &o = pl.ops[op];
    const int nops = (int)pl.ops.size();
    std::string tag;
    if (pl.cls_on && op + 1 == nops) {
        // ran within the previous op (class fusion)
        if (kernel && kernel_len > 0) std::snprintf(kernel, (size_t)kernel_len, "fused");
        if (alg_bytes) *alg_bytes = 0;
        if (plan_bytes) *plan_bytes = 0;
        if (flops) *flops = 0;
        return BUGSEG_OK;
    }
    if (pl.cls_on && op + 2 == nops) {
        // the last bottleneck and the class layer in one launch: block input in, class map out
        const Op &l = pl.ops.back();
        const double outb = (double)o.bn.B * o.bn.H * o.bn.W * o.bn_c * prec_es(ctx->prec);
        const double fin = (double)B * H * W;
        if (kernel && kernel_len > 0) std::snprintf(kernel, (size_t)kernel_len, "bneck C16+classes 16x16");
        const double lb_b = o.layer_bytes >= 0 ? o.layer_bytes : o.bytes, lb_l = l.layer_bytes >= 0 ? l.layer_bytes : l.bytes;
        if (alg_bytes) *alg_bytes = lb_b + lb_l + fin;
        if (plan_bytes) *plan_bytes = o.bytes - outb + (l.bytes - outb) + fin;
        if (flops) *flops = o.flops + l.flops;
        return BUGSEG_OK;
    }
    if (o.kind == 2) {
        tag = "up C" + std::to_string(o.up_cout);
    } else if (o.kind == 1) {
        int th, tw, nw;
        bneck_shape(o.bn_c, o.bn_var, th, tw, nw, nullptr);
        tag = std::string(o.bn_cin ? "down C" : o.bn_var == BNECK2_V && o.bn_c == 128 ? "bneck2 C" : "bneck C") +
              std::to_string(o.bn_c) + (o.bn_asym ? " asym" : "") + " " + std::to_string(th) + "x" + std::to_string(tw);
        (void)nw;
    }
    else if (o.epi == EPI_INIT || o.epi == EPI_INIT_BGR) tag = "init";
    else if (o.epi == EPI_CLASSES && cls_supported(o.a) && !std::getenv("BUGSEG_CLS_CONV")) tag = "classes";
    else tag = "conv NR" + std::to_string(o.nr) + " E" + std::to_string(o.epi);
    if (kernel && kernel_len > 0) {
        std::strncpy(kernel, tag.c_str(), (size_t)kernel_len - 1);
        kernel[kernel_len - 1] = 0;
    }
    double lb = o.layer_bytes >= 0 ? o.layer_bytes : o.bytes, pb = o.bytes;
    const int es = prec_es(ctx->prec);
    if (o.kind == 0 && o.epi == EPI_INIT_BGR) {           // raw BGR input: 3 B/px, not the 8-channel engine input
        const double adj = (double)B * H * W * (8.0 * es - 3.0);
        lb -= adj; pb -= adj;
    }
    if (o.kind == 0 && o.epi == EPI_CLASSES) {            // the output the last forward asked for
        const double fin = o.a.logits_out ? (double)B * H * W * ctx->ncls * 4 : (double)B * H * W;
        lb += fin; pb += fin;
    }
    if (alg_bytes) *alg_bytes = lb;
    if (plan_bytes) *plan_bytes = pb;
    if (flops) *flops = o.flops;
    return BUGSEG_OK;
}

int bugseg_plan_launch_op(bugseg_ctx *ctx, int B, int H, int W, int op, void *stream) {
    if (!ctx) return fail(ctx, BUGSEG_EINVAL, "NULL ctx");
    if (!ctx->loaded) return fail(ctx, BUGSEG_ESTATE, "no weights loaded");
    Plan &pl = ctx->plan;
    if (!pl.arena || pl.B != B || pl.H != H || pl.W != W || !pl.ops.front().a.in)
        return fail(ctx, BUGSEG_ESTATE, "no forward has run at these dimensions");
    if (op < 0 || op >= (int)pl.ops.size()) return fail(ctx, BUGSEG_EINVAL, "op index out of range");
    DeviceGuard g(ctx->device);
    hipError_t e = launch_op(ctx, op, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ctx, BUGSEG_EHIP, "launch of op " + std::to_string(op) + ": " + hipGetErrorString(e));
    return BUGSEG_OK;
}

}  // extern "C"
