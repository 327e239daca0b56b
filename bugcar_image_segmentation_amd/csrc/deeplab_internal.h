// Internal interface between the DeepLab executor (deeplab_runtime.cpp) and its gfx950 kernels
// (deeplab_kernels.hip). SURVEY.md §8(f) row 3 / BASELINE config 4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bugseg {

struct DlPrepArgs {
    const uint8_t *rgb;  // (B, H, W, 3) u8, the ImageTensor feed (models.py:123-124)
    int B, H, W;         // H <= Hc, W <= Wc
    int Hc, Wc;          // crop size (513): the padded engine input
    void *out;           // (B, Hc, Wc, 8) T
};

struct DlConvArgs {
    const void *in;      // NHWC (B, Hin, Win, CS) T
    int B, Hin, Win, CS;
    int Hout, Wout, M;   // M = B * Hout * Wout
    int kh, kw, taps, stride, dil, pad_t, pad_l;
    int cinP;            // input channels padded to 32 (packing of w)
    int NP;              // output channels padded to 64 (rows of w)
    const void *w;       // [NP][taps][cinP] T
    const float *bias;   // [NP]
    const float *bias_img;  // optional per-image bias (B, bias_img_stride) f32
    int bias_img_stride;
    int act;             // 0 none, 1 ReLU, 2 ReLU6 (before the residual add), 3 ReLU after the residual add
                         // (ResNet: relu(shortcut + residual))
    const void *res;     // optional residual NHWC T, (B, Hout, Wout, res_cs)
    int res_cs;
    void *out;           // NHWC (B, Hout, Wout, out_cs), channels [out_off, out_off + cout)
    int out_cs, out_off, cout;
    uint32_t in_bytes;
    uint32_t mHW, mW; int sHW, sW;   // fdiv by Hout * Wout and by Wout
    // depthwise-fused projection (dw_w != nullptr): `in` is the depthwise conv's INPUT (B, Hin, Win, CS)
    // and the 1x1 conv's B operand is computed on load: relu6(sum_taps in * dw_w + dw_b), rounded to T
    const void *dw_w;    // [9][CS] T
    const float *dw_b;   // [CS]
    int dw_stride, dw_dil, dw_pt, dw_pl;
    int nb;              // pixel fragments per wave: 2 (128-px workgroup tile), 4 (256 px) or 8 (bf16, 512 px)
    int tap_packed;      // CS == 8: w is [NP][ceil(taps / 4) * 32], k = tap * 8 + c
    // tap-packed only: when rgb != nullptr the input is the raw (B, img_h, img_w, 3) u8 RGB batch and
    // the (B, Hin, Win, 8) operand is formed on load (dl_prep_kernel's padding and normalisation)
    const uint8_t *rgb;
    int img_h, img_w;
    const void *zero;    // >= 16 zero bytes (after the weight blob): the implicit-GEMM conv's padding taps
};

// n same-shape implicit-GEMM convs (bf16 out, no residual) as one launch (dl_launch_conv_group)
constexpr int DL_GROUP_MAX = 4;
struct DlConvGroup {
    DlConvArgs a[DL_GROUP_MAX];
    int n, tiles;   // tiles: set by the launcher
};

struct DlDwArgs {
    const void *in;      // (B, Hin, Win, C) T
    int B, Hin, Win, C;
    int Hout, Wout, M, stride, dil, pad_t, pad_l;
    const void *w;       // [9][C] T
    const float *bias;   // [C]
    void *out;           // (B, Hout, Wout, C) T
    uint32_t mHW, mW; int sHW, sW;
    uint32_t in_bytes;
    int act;             // 0 none, 1 ReLU, 2 ReLU6 (MobileNetV2: 2; Xception's pre-activation modules: 0)
    int in_relu;         // ReLU applied to the input as it is loaded (Xception: activation before the
                         // separable conv, the un-rectified tensor still feeding the module's skip)
};

// Bilinear resize, align_corners (TF1 ResizeBilinear, the formula of the argmax stage) of a T tensor
// into channels [out_off, out_off + C) of another: the DeepLabV3+ decoder's upsampling of the ASPP
// output to the low-level feature size before the concat.
struct DlResizeArgs {
    const void *in;      // (B, h, w, in_cs) T, channels [0, C) used
    int B, h, w, in_cs, C;
    float sy, sx;        // (h - 1) / (Ho - 1), (w - 1) / (Wo - 1) in f32
    int Ho, Wo;
    void *out;           // (B, Ho, Wo, out_cs) T
    int out_cs, out_off;
};

struct DlPoolArgs {
    const void *x;       // (B, H, W, CS) T: the ASPP input
    int B, H, W, C, CS;
    int chunk_px, nchunks;
    float *part;         // (B, nchunks, C) scratch
    int cmid, cout;
    float *y;            // (B, cmid) scratch: the image-pooling branch output
    const float *wp, *bp;    // image-pooling 1x1: [cmid][C], [cmid]
    const float *wq, *bq;    // its columns of the concat projection: [cout][cmid], projection bias [cout]
    float *z;            // (B, z_stride) per-image projection bias
    int z_stride;
};

struct DlArgmaxArgs {
    const float *logits; // (B, h, w, LCS) f32
    int B, h, w, LCS, ncls;
    float sy, sx;        // (h - 1) / (Hc - 1), (w - 1) / (Wc - 1) in f32
    int Ho, Wo;          // output rows / cols (the un-padded image)
    int Hout, Wout;      // output tensor dims (== Ho, Wo)
    int64_t *out;        // (B, Hout, Wout)
};

// Max pooling, TF 'SAME' / 'VALID' geometry given as pads (taps outside the input are skipped, i.e. -inf
// padding): ResNet's 3x3 s2 root pool, and with k = 1 its strided-identity shortcut (resnet_utils.subsample)
struct DlMaxPoolArgs {
    const void *in;      // (B, Hin, Win, C) T
    int B, Hin, Win, C;
    int Hout, Wout, k, stride, pad_t, pad_l;
    void *out;           // (B, Hout, Wout, C) T
};

hipError_t dl_launch_prep(int prec, const DlPrepArgs &a, hipStream_t s);
hipError_t dl_launch_maxpool(int prec, const DlMaxPoolArgs &a, hipStream_t s);
hipError_t dl_launch_conv_group(int prec, const DlConvGroup &g, hipStream_t s);   // hipErrorNotSupported: launch singly
hipError_t dl_launch_conv(int prec, bool out_f32, const DlConvArgs &a, hipStream_t s);
hipError_t dl_launch_dw(int prec, const DlDwArgs &a, hipStream_t s);
hipError_t dl_launch_pool(int prec, const DlPoolArgs &a, hipStream_t s);
hipError_t dl_launch_argmax(const DlArgmaxArgs &a, hipStream_t s);
hipError_t dl_launch_resize(int prec, const DlResizeArgs &a, hipStream_t s);

}  // namespace bugseg
