// DeepLabV3 executor behind the C ABI (include/bugseg.h, bugseg_dl_*): SURVEY.md §8(f) row 3.
//
// The graph builder is host-side Python (deeplab_spec.py): it folds batch-norm, packs weights for
// the kernels into one blob, and lowers the network to a flat op list with buffer ids for a batch
// size. This executor owns the device copies (weights, one activation arena per plan), validates
// every op's shapes against its buffers before anything is launched, and enqueues the launches on
// the caller's stream. It knows nothing about MobileNetV2, Xception or ASPP beyond the op kinds.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "bugseg_internal.h"
#include "deeplab_internal.h"
#include "../../include/bugseg.h"

using namespace bugseg;

namespace {

thread_local std::string g_dl_err;

enum { OP_PREP = 1, OP_CONV = 2, OP_DW = 3, OP_POOL = 4, OP_ARGMAX = 5, OP_RESIZE = 6, OP_MAXPOOL = 7 };

struct DlOp {
    int f[BUGSEG_DL_OP_FIELDS];
};

}  // namespace

struct bugseg_dl {
    int device = 0, prec = 0;
    std::string err;
    void *dev_w = nullptr;
    size_t w_bytes = 0, zero_off = 0;
    std::vector<DlOp> ops;
    std::vector<int> group_len;   // per op: > 1 at the first of that many same-shape convs run as one launch
    std::vector<size_t> buf_bytes, buf_off;
    void *arena = nullptr;
    int B = 0, Hc = 0, Wc = 0;
    // the last forward's I/O (profiling hook)
    const uint8_t *last_rgb = nullptr;
    int64_t *last_out = nullptr;
    int last_H = 0, last_W = 0;
};

namespace {

int dl_fail(bugseg_dl *c, int code, const std::string &m) {
    if (c) c->err = m;
    else g_dl_err = m;
    return code;
}

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DevGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

void *bufp(bugseg_dl *c, int id) { return static_cast<char *>(c->arena) + c->buf_off[id]; }

bool in_w(const bugseg_dl *c, long off, long bytes) { return off >= 0 && bytes >= 0 && off + bytes <= (long)c->w_bytes; }
bool buf_ok(const bugseg_dl *c, int id, double bytes) {
    return id >= 0 && id < (int)c->buf_bytes.size() && bytes <= (double)c->buf_bytes[id];
}

// Shape / bounds validation of one op against the plan's buffers and the weight blob.
bool in_range(int v, int lo, int hi) { return v >= lo && v <= hi; }

bool check_op(const bugseg_dl *c, const DlOp &o, std::string &why) {
    const int *f = o.f;
    const double es = c->prec == PREC_BF16 ? 2.0 : 4.0;
    const int B = c->B;
    // every field that enters integer arithmetic here or in run_op is bounded first (no overflow):
    // spatial sizes <= 16384, channels <= 8192, kernel extents <= 15, strides / dilations <= 255
    constexpr int SP = 16384, CH = 8192;
    switch (f[0]) {
    case OP_PREP:
        if (!buf_ok(c, f[1], (double)B * c->Hc * c->Wc * 8 * es)) { why = "prep: destination buffer too small"; return false; }
        return true;
    case OP_CONV: {
        const int src = f[1], dst = f[2], res = f[3], Hin = f[4], Win = f[5], CS = f[6], Hout = f[7], Wout = f[8];
        const int kh = f[9], kw = f[10], stride = f[11], dil = f[12], cinP = f[15], NP = f[16];
        const long w_off = f[17], b_off = f[18];
        const int act = f[19], res_cs = f[20], out_cs = f[21], out_off = f[22], cout = f[23], out_f32 = f[24];
        const int bimg = f[25], bimg_stride = f[26];
        if (!in_range(Hin, 1, SP) || !in_range(Win, 1, SP) || !in_range(Hout, 1, SP) || !in_range(Wout, 1, SP) ||
            !in_range(kh, 1, 15) || !in_range(kw, 1, 15) || !in_range(stride, 1, 255) || !in_range(dil, 1, 255) ||
            !in_range(f[13], 0, 255) || !in_range(f[14], 0, 255) || !in_range(CS, 8, CH) || !in_range(cinP, 32, CH) ||
            !in_range(NP, 64, CH) || !in_range(res_cs, 0, CH) || !in_range(out_cs, 8, CH) || !in_range(out_off, 0, CH) ||
            !in_range(cout, 8, CH) || !in_range(bimg_stride, 0, 1 << 20) || (f[31] != 0 && f[31] != 1 && f[31] != 2) ||
            (double)B * Hout * Wout >= 2147483648.0) { why = "conv: field out of range"; return false; }
        if (Hin < 1 || Win < 1 || Hout < 1 || Wout < 1 || kh < 1 || kw < 1 || stride < 1 || dil < 1 || CS < 8 ||
            CS % 8 || cinP % 32 || cinP < 32 || NP % 64 || NP < 64 || act < 0 || act > 3 || cout < 8 || cout % 8 ||
            cout > NP || out_off % 8 || out_off + cout > out_cs) { why = "conv: bad shape"; return false; }
        if (!buf_ok(c, src, (double)B * Hin * Win * CS * es)) { why = "conv: source buffer too small"; return false; }
        if (!buf_ok(c, dst, (double)B * Hout * Wout * out_cs * (out_f32 ? 4.0 : es))) { why = "conv: destination too small"; return false; }
        if (res >= 0 && (res_cs < cout || !buf_ok(c, res, (double)B * Hout * Wout * res_cs * es))) { why = "conv: residual too small"; return false; }
        if (bimg >= 0 && (bimg_stride < NP || !buf_ok(c, bimg, (double)B * bimg_stride * 4.0))) { why = "conv: per-image bias too small"; return false; }
        const long wk = f[31] ? (long)((kh * kw + 3) / 4) * 32 : (long)kh * kw * cinP;
        if (f[31] && (CS != 8 || f[27] >= 0)) { why = "conv: tap packing needs an 8-channel input"; return false; }
        if (!in_w(c, w_off, (long)NP * wk * (long)es) || !in_w(c, b_off, (long)NP * 4) || w_off % 16 || b_off % 16) {
            why = "conv: weights out of the blob"; return false;
        }
        if ((double)B * Hin * Win * CS * es >= 2147483648.0) { why = "conv: input exceeds 31-bit offsets"; return false; }
        if (f[30] != 0 && f[30] != 2 && f[30] != 4 && f[30] != 8) { why = "conv: pixel fragments per wave must be 2, 4 or 8"; return false; }
        if (f[27] >= 0) {   // depthwise-fused projection: 1x1 over the dw output grid (Hout, Wout)
            const int dws = f[29] & 0xff, dwd = (f[29] >> 8) & 0xff, pt = (f[29] >> 16) & 0xff, pl = (f[29] >> 24) & 0xff;
            if (kh != 1 || kw != 1 || stride != 1 || f[13] || f[14] || dws < 1 || dwd < 1 ||
                (Hout - 1) * dws - pt > Hin - 1 + 2 * dwd || (Wout - 1) * dws - pl > Win - 1 + 2 * dwd) {
                why = "conv: bad depthwise-fused geometry"; return false;
            }
            if (!in_w(c, f[27], 9L * CS * (long)es) || !in_w(c, f[28], (long)CS * 4) || f[27] % 16 || f[28] % 16) {
                why = "conv: depthwise weights out of the blob"; return false;
            }
        }
        return true;
    }
    case OP_DW: {
        const int src = f[1], dst = f[2], Hin = f[3], Win = f[4], C = f[5], Hout = f[6], Wout = f[7];
        const long w_off = f[12], b_off = f[13];
        if (!in_range(Hin, 1, SP) || !in_range(Win, 1, SP) || !in_range(Hout, 1, SP) || !in_range(Wout, 1, SP) ||
            !in_range(C, 8, CH) || !in_range(f[8], 1, 255) || !in_range(f[9], 1, 255) || !in_range(f[10], 0, 255) ||
            !in_range(f[11], 0, 255) || (double)B * Hout * Wout >= 2147483648.0) { why = "dw: field out of range"; return false; }
        if (C < 8 || C % 8 || Hin < 1 || Win < 1 || Hout < 1 || Wout < 1 || f[8] < 1 || f[9] < 1) { why = "dw: bad shape"; return false; }
        if (!in_range(f[14], 0, 2) || !in_range(f[15], 0, 1) || (f[15] && f[14])) { why = "dw: bad activation flags"; return false; }
        if (f[8] != 1 && (f[8] != 2 || f[9] != 1)) { why = "dw: stride 2 with dilation (TF has no strided atrous)"; return false; }
        if (!buf_ok(c, src, (double)B * Hin * Win * C * es) || !buf_ok(c, dst, (double)B * Hout * Wout * C * es)) { why = "dw: buffer too small"; return false; }
        if ((double)B * Hin * Win * C * es >= 2147483648.0) { why = "dw: input exceeds 31-bit offsets"; return false; }
        if (!in_w(c, w_off, 9L * C * (long)es) || !in_w(c, b_off, (long)C * 4) || w_off % 16 || b_off % 16) { why = "dw: weights out of the blob"; return false; }
        return true;
    }
    case OP_POOL: {
        const int src = f[1], part = f[2], z = f[3], H = f[4], W = f[5], C = f[6], CS = f[7], chunk = f[8], nch = f[9];
        const int cmid = f[10], cout = f[11], zs = f[16];
        if (!in_range(H, 1, SP) || !in_range(W, 1, SP) || !in_range(CS, 1, CH)) { why = "pool: field out of range"; return false; }
        if (C < 1 || C > 2048 || C % 8 || CS < C || cmid < 1 || cmid > 1024 || cout < 1 || zs < cout || chunk < 1 || nch < 1 ||
            (long)chunk * nch < (long)H * W) { why = "pool: bad shape"; return false; }
        if (!buf_ok(c, src, (double)B * H * W * CS * es) || !buf_ok(c, part, (double)B * nch * C * 4.0) ||
            !buf_ok(c, z, (double)B * zs * 4.0) || !buf_ok(c, f[17], (double)B * cmid * 4.0)) { why = "pool: buffer too small"; return false; }
        if (!in_w(c, f[12], (long)cmid * C * 4) || !in_w(c, f[13], (long)cmid * 4) || !in_w(c, f[14], (long)cout * cmid * 4) ||
            !in_w(c, f[15], (long)cout * 4)) { why = "pool: weights out of the blob"; return false; }
        return true;
    }
    case OP_ARGMAX: {
        const int lg = f[1], h = f[2], w = f[3], LCS = f[4], ncls = f[5];
        if (!in_range(h, 1, SP) || !in_range(w, 1, SP) || !in_range(LCS, 1, CH)) { why = "argmax: field out of range"; return false; }
        if (h < 1 || w < 1 || ncls < 1 || LCS < ncls || LCS % 4) { why = "argmax: bad shape"; return false; }
        if (!buf_ok(c, lg, (double)B * h * w * LCS * 4.0)) { why = "argmax: logits buffer too small"; return false; }
        return true;
    }
    case OP_RESIZE: {
        const int src = f[1], dst = f[2], h = f[3], w = f[4], in_cs = f[5], C = f[6], Ho = f[7], Wo = f[8];
        const int out_cs = f[9], out_off = f[10];
        if (!in_range(h, 1, SP) || !in_range(w, 1, SP) || !in_range(Ho, 1, SP) || !in_range(Wo, 1, SP) ||
            !in_range(in_cs, 8, CH) || !in_range(C, 8, CH) || !in_range(out_cs, 8, CH) || !in_range(out_off, 0, CH) ||
            (double)B * Ho * Wo * out_cs >= 2147483648.0) { why = "resize: field out of range"; return false; }
        if (C % 8 || in_cs % 8 || out_cs % 8 || out_off % 8 || C > in_cs || out_off + C > out_cs) { why = "resize: bad shape"; return false; }
        if (!buf_ok(c, src, (double)B * h * w * in_cs * es) || !buf_ok(c, dst, (double)B * Ho * Wo * out_cs * es)) {
            why = "resize: buffer too small"; return false;
        }
        return true;
    }
    case OP_MAXPOOL: {
        const int src = f[1], dst = f[2], Hin = f[3], Win = f[4], C = f[5], Hout = f[6], Wout = f[7];
        if (!in_range(Hin, 1, SP) || !in_range(Win, 1, SP) || !in_range(Hout, 1, SP) || !in_range(Wout, 1, SP) ||
            !in_range(C, 8, CH) || !in_range(f[8], 1, 15) || !in_range(f[9], 1, 255) || !in_range(f[10], 0, 15) ||
            !in_range(f[11], 0, 15) || (double)B * Hout * Wout * C >= 2147483648.0) { why = "maxpool: field out of range"; return false; }
        if (C % 8 || (Hout - 1) * f[9] - f[10] > Hin - 1 || (Wout - 1) * f[9] - f[11] > Win - 1) { why = "maxpool: bad shape"; return false; }
        if (!buf_ok(c, src, (double)B * Hin * Win * C * es) || !buf_ok(c, dst, (double)B * Hout * Wout * C * es)) {
            why = "maxpool: buffer too small"; return false;
        }
        return true;
    }
    default:
        why = "unknown op kind " + std::to_string(f[0]);
        return false;
    }
}

// Runs of consecutive k x k CONV ops of one shape that read the same buffer and write the same one
// (the ASPP's atrous branches, each at its channel offset of the concat): same input / output
// geometry, packing, no residual, depthwise or per-image bias, 2-byte output. -> per op, the length
// of the run starting there (1 = launched alone); the launcher still checks each member's form.
std::vector<int> conv_groups(const std::vector<DlOp> &ops) {
    std::vector<int> len(ops.size(), 1);
    auto alone_ok = [](const int *f) {
        return f[0] == OP_CONV && f[3] < 0 && f[9] > 1 && f[10] > 1 && f[24] == 0 && f[25] < 0 && f[27] < 0 && f[31] == 0;
    };
    auto same = [](const int *x, const int *y) {
        for (int k : {1, 2, 4, 5, 6, 7, 8, 9, 10, 15, 16, 21})
            if (x[k] != y[k]) return false;
        return true;
    };
    for (size_t i = 0; i < ops.size();) {
        size_t n = 1;
        if (alone_ok(ops[i].f))
            while (i + n < ops.size() && (int)n < DL_GROUP_MAX && alone_ok(ops[i + n].f) && same(ops[i].f, ops[i + n].f)) ++n;
        if (n > 1) len[i] = (int)n;
        i += n;
    }
    return len;
}

// The DlConvArgs of CONV op o (run_op and the grouped launch in bugseg_dl_forward).
DlConvArgs conv_args(bugseg_dl *c, const DlOp &o, const uint8_t *rgb, int H, int W) {
    const int *f = o.f;
    const char *wb = static_cast<const char *>(c->dev_w);
    const int B = c->B;
    DlConvArgs a{};
    a.in = bufp(c, f[1]);
    a.B = B; a.Hin = f[4]; a.Win = f[5]; a.CS = f[6];
    a.Hout = f[7]; a.Wout = f[8]; a.M = B * a.Hout * a.Wout;
    a.kh = f[9]; a.kw = f[10]; a.taps = a.kh * a.kw; a.stride = f[11]; a.dil = f[12]; a.pad_t = f[13]; a.pad_l = f[14];
    a.cinP = f[15]; a.NP = f[16];
    a.w = wb + f[17];
    a.bias = reinterpret_cast<const float *>(wb + f[18]);
    a.act = f[19];
    a.res = f[3] >= 0 ? bufp(c, f[3]) : nullptr;
    a.res_cs = f[20];
    a.out = bufp(c, f[2]); a.out_cs = f[21]; a.out_off = f[22]; a.cout = f[23];
    a.bias_img = f[25] >= 0 ? static_cast<const float *>(bufp(c, f[25])) : nullptr;
    a.bias_img_stride = f[26];
    a.in_bytes = (uint32_t)((size_t)B * a.Hin * a.Win * a.CS * (c->prec == PREC_BF16 ? 2 : 4));
    a.nb = f[30] == 8 ? 8 : f[30] == 4 ? 4 : 2;
    a.zero = wb + c->zero_off;
    a.tap_packed = f[31] != 0;
    if (f[31] == 2) { a.rgb = rgb; a.img_h = H; a.img_w = W; }   // stem with the preprocessing fused
    if (f[27] >= 0) {
        a.dw_w = wb + f[27];
        a.dw_b = reinterpret_cast<const float *>(wb + f[28]);
        a.dw_stride = f[29] & 0xff; a.dw_dil = (f[29] >> 8) & 0xff;
        a.dw_pt = (f[29] >> 16) & 0xff; a.dw_pl = (f[29] >> 24) & 0xff;
    }
    fastdiv((uint32_t)(a.Hout * a.Wout), a.mHW, a.sHW);
    fastdiv((uint32_t)a.Wout, a.mW, a.sW);
    return a;
}

hipError_t run_op(bugseg_dl *c, const DlOp &o, const uint8_t *rgb, int H, int W, int64_t *out, hipStream_t s) {
    const int *f = o.f;
    const char *wb = static_cast<const char *>(c->dev_w);
    const int B = c->B;
    switch (f[0]) {
    case OP_PREP: {
        DlPrepArgs a{rgb, B, H, W, c->Hc, c->Wc, bufp(c, f[1])};
        return dl_launch_prep(c->prec, a, s);
    }
    case OP_CONV: {
        const DlConvArgs a = conv_args(c, o, rgb, H, W);
        return dl_launch_conv(c->prec, f[24] != 0, a, s);
    }
    case OP_DW: {
        DlDwArgs a{};
        a.in = bufp(c, f[1]); a.out = bufp(c, f[2]);
        a.B = B; a.Hin = f[3]; a.Win = f[4]; a.C = f[5]; a.Hout = f[6]; a.Wout = f[7];
        a.M = B * a.Hout * a.Wout; a.stride = f[8]; a.dil = f[9]; a.pad_t = f[10]; a.pad_l = f[11];
        a.w = wb + f[12];
        a.in_bytes = (uint32_t)((size_t)B * a.Hin * a.Win * a.C * (c->prec == PREC_BF16 ? 2 : 4));
        a.bias = reinterpret_cast<const float *>(wb + f[13]);
        a.act = f[14]; a.in_relu = f[15];
        fastdiv((uint32_t)(a.Hout * a.Wout), a.mHW, a.sHW);
        fastdiv((uint32_t)a.Wout, a.mW, a.sW);
        return dl_launch_dw(c->prec, a, s);
    }
    case OP_RESIZE: {
        DlResizeArgs a{};
        a.in = bufp(c, f[1]); a.out = bufp(c, f[2]);
        a.B = B; a.h = f[3]; a.w = f[4]; a.in_cs = f[5]; a.C = f[6]; a.Ho = f[7]; a.Wo = f[8];
        a.out_cs = f[9]; a.out_off = f[10];
        a.sy = a.Ho > 1 ? (float)(a.h - 1) / (float)(a.Ho - 1) : 0.f;
        a.sx = a.Wo > 1 ? (float)(a.w - 1) / (float)(a.Wo - 1) : 0.f;
        return dl_launch_resize(c->prec, a, s);
    }
    case OP_POOL: {
        DlPoolArgs a{};
        a.x = bufp(c, f[1]); a.part = static_cast<float *>(bufp(c, f[2])); a.z = static_cast<float *>(bufp(c, f[3]));
        a.B = B; a.H = f[4]; a.W = f[5]; a.C = f[6]; a.CS = f[7]; a.chunk_px = f[8]; a.nchunks = f[9];
        a.cmid = f[10]; a.cout = f[11];
        a.wp = reinterpret_cast<const float *>(wb + f[12]); a.bp = reinterpret_cast<const float *>(wb + f[13]);
        a.wq = reinterpret_cast<const float *>(wb + f[14]); a.bq = reinterpret_cast<const float *>(wb + f[15]);
        a.z_stride = f[16];
        a.y = static_cast<float *>(bufp(c, f[17]));
        return dl_launch_pool(c->prec, a, s);
    }
    case OP_MAXPOOL: {
        DlMaxPoolArgs a{};
        a.in = bufp(c, f[1]); a.out = bufp(c, f[2]);
        a.B = B; a.Hin = f[3]; a.Win = f[4]; a.C = f[5]; a.Hout = f[6]; a.Wout = f[7];
        a.k = f[8]; a.stride = f[9]; a.pad_t = f[10]; a.pad_l = f[11];
        return dl_launch_maxpool(c->prec, a, s);
    }
    case OP_ARGMAX: {
        DlArgmaxArgs a{};
        a.logits = static_cast<const float *>(bufp(c, f[1]));
        a.B = B; a.h = f[2]; a.w = f[3]; a.LCS = f[4]; a.ncls = f[5];
        a.sy = c->Hc > 1 ? (float)(a.h - 1) / (float)(c->Hc - 1) : 0.f;
        a.sx = c->Wc > 1 ? (float)(a.w - 1) / (float)(c->Wc - 1) : 0.f;
        a.Ho = H; a.Wo = W; a.Hout = H; a.Wout = W;
        a.out = out;
        return dl_launch_argmax(a, s);
    }
    }
    return hipErrorInvalidValue;
}

}  // namespace

extern "C" {

int bugseg_dl_create(int device, int precision, bugseg_dl **out) {
    if (!out || (precision != BUGSEG_FP32 && precision != BUGSEG_BF16)) return dl_fail(nullptr, BUGSEG_EINVAL, "bad argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return dl_fail(nullptr, BUGSEG_EINVAL, "no such HIP device");
    auto *c = new bugseg_dl();
    c->device = device;
    c->prec = precision == BUGSEG_BF16 ? PREC_BF16 : PREC_F32;
    *out = c;
    return BUGSEG_OK;
}

int bugseg_dl_destroy(bugseg_dl *c) {
    if (!c) return BUGSEG_OK;
    DevGuard g(c->device);
    if (c->dev_w) (void)hipFree(c->dev_w);
    if (c->arena) (void)hipFree(c->arena);
    delete c;
    return BUGSEG_OK;
}

int bugseg_dl_load_weights(bugseg_dl *c, const void *blob, size_t bytes) {
    if (!c || !blob || bytes == 0 || bytes >= (size_t)1 << 31) return dl_fail(c, BUGSEG_EINVAL, "bad weight blob");
    DevGuard g(c->device);
    if (c->dev_w) { (void)hipDeviceSynchronize(); (void)hipFree(c->dev_w); c->dev_w = nullptr; }
    // the blob, then 256 zero bytes at a 256-B boundary (the implicit-GEMM conv's padding taps read them)
    const size_t zoff = (bytes + 255) / 256 * 256;
    if (hipMalloc(&c->dev_w, zoff + 256) != hipSuccess) return dl_fail(c, BUGSEG_ENOMEM, "weight allocation failed");
    if (hipMemcpy(c->dev_w, blob, bytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(static_cast<char *>(c->dev_w) + zoff, 0, 256) != hipSuccess) return dl_fail(c, BUGSEG_EHIP, "weight upload failed");
    c->zero_off = zoff;
    c->w_bytes = bytes;
    c->ops.clear();
    c->group_len.clear();
    return BUGSEG_OK;
}

}  // extern "C"

namespace {
// Host-only validation of a whole plan (bugseg_dl_set_plan, and the ASan test hook below): every op
// against the new buffers and a weight blob of w_bytes. -> arena layout in off / total.
int validate_plan(bugseg_dl *c, int prec, size_t w_bytes, const int32_t *ops, int nops, const uint64_t *buf_bytes, int nbufs,
                  int B, int Hc, int Wc, std::vector<DlOp> &v, std::vector<size_t> &bb, std::vector<size_t> &off,
                  size_t &total) {
    if (!ops || nops < 1 || nops > 4096 || nbufs < 1 || nbufs > 64 || !buf_bytes || B < 1 || Hc < 2 || Wc < 2 ||
        Hc > 8192 || Wc > 8192)
        return dl_fail(c, BUGSEG_EINVAL, "bad plan");
    v.resize(nops);
    std::memcpy(v.data(), ops, sizeof(DlOp) * (size_t)nops);
    bb.assign(buf_bytes, buf_bytes + nbufs);
    off.resize(nbufs);
    total = 0;
    for (int i = 0; i < nbufs; ++i) {
        if (bb[i] > ((uint64_t)1 << 40)) return dl_fail(c, BUGSEG_EINVAL, "buffer " + std::to_string(i) + " too large");
        off[i] = total;
        total += (bb[i] + 255) & ~(size_t)255;
    }
    bugseg_dl probe;
    probe.prec = prec; probe.w_bytes = w_bytes; probe.buf_bytes = bb; probe.B = B; probe.Hc = Hc; probe.Wc = Wc;
    for (int i = 0; i < nops; ++i) {
        std::string why;
        if (!check_op(&probe, v[i], why)) return dl_fail(c, BUGSEG_EINVAL, "op " + std::to_string(i) + ": " + why);
    }
    return BUGSEG_OK;
}
}  // namespace

extern "C" {

// Test hook (host only, no device): the validation bugseg_dl_set_plan runs, for a blob of w_bytes.
int bugseg_dl_debug_check_plan(const int32_t *ops, int nops, const uint64_t *buf_bytes, int nbufs, int B, int Hc, int Wc,
                               int precision, size_t w_bytes) {
    std::vector<DlOp> v;
    std::vector<size_t> bb, off;
    size_t total = 0;
    return validate_plan(nullptr, precision == BUGSEG_BF16 ? PREC_BF16 : PREC_F32, w_bytes, ops, nops, buf_bytes, nbufs, B,
                         Hc, Wc, v, bb, off, total);
}

int bugseg_dl_set_plan(bugseg_dl *c, const int32_t *ops, int nops, const uint64_t *buf_bytes, int nbufs, int B, int Hc, int Wc) {
    if (!c) return dl_fail(c, BUGSEG_EINVAL, "bad plan");
    if (!c->dev_w) return dl_fail(c, BUGSEG_ESTATE, "plan before weights");
    std::vector<DlOp> v;
    std::vector<size_t> bb, off;
    size_t total = 0;
    // validate against the new plan before touching the old one
    const int rc = validate_plan(c, c->prec, c->w_bytes, ops, nops, buf_bytes, nbufs, B, Hc, Wc, v, bb, off, total);
    if (rc != BUGSEG_OK) return rc;
    DevGuard g(c->device);
    if (c->arena) {
        (void)hipDeviceSynchronize();   // a forward of the old plan may still be running on any stream
        (void)hipFree(c->arena);
        c->arena = nullptr;
    }
    if (hipMalloc(&c->arena, total) != hipSuccess) return dl_fail(c, BUGSEG_ENOMEM, "activation arena allocation failed");
    c->ops = std::move(v);
    c->group_len = conv_groups(c->ops);
    c->buf_bytes = std::move(bb);
    c->buf_off = std::move(off);
    c->B = B; c->Hc = Hc; c->Wc = Wc;
    return BUGSEG_OK;
}

int bugseg_dl_forward(bugseg_dl *c, const uint8_t *rgb_dev, int B, int H, int W, int64_t *out_dev, void *stream) {
    if (!c || !rgb_dev || !out_dev) return dl_fail(c, BUGSEG_EINVAL, "null argument");
    if (c->ops.empty()) return dl_fail(c, BUGSEG_ESTATE, "forward before set_plan");
    if (B != c->B || H < 1 || W < 1 || H > c->Hc || W > c->Wc)
        return dl_fail(c, BUGSEG_EINVAL, "input (" + std::to_string(B) + ", " + std::to_string(H) + ", " + std::to_string(W) +
                                             ") does not fit the plan (B = " + std::to_string(c->B) + ", crop " +
                                             std::to_string(c->Hc) + "x" + std::to_string(c->Wc) + ")");
    DevGuard g(c->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const char *ge = std::getenv("BUGSEG_DL_GROUP");
    const bool group = !(ge && *ge == '0');
    for (size_t i = 0; i < c->ops.size(); ++i) {
        const int n = group ? c->group_len[i] : 1;
        if (n > 1) {   // same-shape convs as one launch (the ASPP's atrous branches)
            DlConvGroup grp{};
            grp.n = n;
            for (int k = 0; k < n; ++k) grp.a[k] = conv_args(c, c->ops[i + k], rgb_dev, H, W);
            const hipError_t e = dl_launch_conv_group(c->prec, grp, s);
            if (e == hipSuccess) { i += n - 1; continue; }
            if (e != hipErrorNotSupported) return dl_fail(c, BUGSEG_EHIP, "grouped launch at op " + std::to_string(i) + ": " + hipGetErrorString(e));
            (void)hipGetLastError();
        }
        const hipError_t e = run_op(c, c->ops[i], rgb_dev, H, W, out_dev, s);
        if (e != hipSuccess) return dl_fail(c, BUGSEG_EHIP, "launch of op " + std::to_string(i) + ": " + hipGetErrorString(e));
    }
    c->last_rgb = rgb_dev; c->last_out = out_dev; c->last_H = H; c->last_W = W;
    return BUGSEG_OK;
}

int bugseg_dl_launch_op(bugseg_dl *c, int op, void *stream) {
    if (!c || op < 0 || op >= (int)c->ops.size() || !c->last_rgb) return dl_fail(c, BUGSEG_EINVAL, "no such op / no forward yet");
    DevGuard g(c->device);
    const hipError_t e = run_op(c, c->ops[op], c->last_rgb, c->last_H, c->last_W, c->last_out, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? BUGSEG_OK : dl_fail(c, BUGSEG_EHIP, hipGetErrorString(e));
}

int bugseg_dl_read_buffer(bugseg_dl *c, int buf, void *dst_dev, size_t bytes, void *stream) {
    if (!c || !dst_dev || !c->arena || buf < 0 || buf >= (int)c->buf_bytes.size() || bytes > c->buf_bytes[buf])
        return dl_fail(c, BUGSEG_EINVAL, "no such buffer / too many bytes");
    DevGuard g(c->device);
    const hipError_t e = hipMemcpyAsync(dst_dev, bufp(c, buf), bytes, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? BUGSEG_OK : dl_fail(c, BUGSEG_EHIP, hipGetErrorString(e));
}

const char *bugseg_dl_last_error(const bugseg_dl *c) { return c ? c->err.c_str() : g_dl_err.c_str(); }

}  // extern "C"
