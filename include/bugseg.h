/*
 * bugseg — MI355X-native (gfx950) ENet segmentation -> BEV occupancy-grid path, C ABI.
 *
 * The reference exposes no FFI: its boundary is the Python plugin API of models.py / bev.py /
 * occgrid_to_ros.py. These entry points are what that API's Python shims
 * (bugcar_image_segmentation_amd/{models,bev,occgrid_to_ros}.py, bound with ctypes) call; each
 * cites the reference interface it replaces. A ctypes binding a maintainer would add to the
 * reference itself is shown in INTEGRATION.md.
 *
 * Conventions
 *  - Every pointer argument named *_dev is a DEVICE pointer owned by the caller (e.g. a
 *    torch tensor's data_ptr()). The library owns only its weights, tables and scratch.
 *  - `stream` is a hipStream_t (NULL = the legacy default stream). All work of one call is
 *    enqueued on it; calls return without synchronising.
 *  - Return 0 on success or a negative BUGSEG_E* code; bugseg_last_error() explains it.
 *  - Calls on one context must not overlap in time from several host threads.
 *  - A context's forward activation arena is ONE set of buffers: ENet forwards of one context must
 *    all be enqueued on one stream (run concurrent frame shards on one context each, as
 *    pipeline.py does). BEV calls of one context may be enqueued on several streams at once: the
 *    warp-tap and polar tables are read-only once built, and the laserscan batch scratch is either
 *    the caller's workspace (bugseg_bev_occgrid_ws) or kept per stream (bugseg_bev_occgrid).
 *  - Stream order, graphs: the BEV entry points never synchronise the caller's stream or the
 *    device. A table for a new geometry is built on the context's private stream and waited for
 *    there before the call enqueues its work, so the first call at a new geometry or batch may be
 *    captured into a HIP graph (so may the first forward at a shape). Memory a captured call used
 *    (arena, tables, scratch) is kept until bugseg_destroy. The rare eviction of an uncaptured
 *    table (a 5th geometry) and arena reallocation at a new shape outside a capture synchronise
 *    the device first, so nothing in flight reads freed memory.
 *  - Tensor shapes: activations are NHWC. The "engine input" tensor is (B, H, W, 8): RGB plus 5
 *    zero channels, in the context precision (f32, bf16 or f16).
 */
#ifndef BUGSEG_H
#define BUGSEG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bugseg_ctx bugseg_ctx;

enum {
    BUGSEG_OK = 0,
    BUGSEG_EINVAL = -1,   /* bad argument / shape (reference: AssertionError, bev.py:169)     */
    BUGSEG_ENOMEM = -2,
    BUGSEG_EHIP = -3,     /* HIP runtime error                                                 */
    BUGSEG_EFORMAT = -4,  /* malformed weight blob (reference: GraphDef ParseFromString error)  */
    BUGSEG_ESTATE = -5    /* e.g. forward before load_weights                                  */
};

/* Precisions: activations and weights stored as f32 (the parity mode), bf16 (the throughput mode) or
 * f16 (the same bytes and MFMA rate as bf16 with 3 more mantissa bits: closer class agreement with
 * fp32; range +-65504). Products accumulate in f32 in every mode. */
enum { BUGSEG_FP32 = 0, BUGSEG_BF16 = 1, BUGSEG_F16 = 2 };

/* out_kind of bugseg_enet_forward */
enum {
    BUGSEG_OUT_LOGITS_F32 = 0,  /* (B, C, H, W) f32 NCHW — the TF output tensor "CATkrIDy/concat:0" (models.py:16,52) */
    BUGSEG_OUT_CLASS15_U8 = 1,  /* (B, H, W) u8 raw argmax class id (models.py:55)                    */
    BUGSEG_OUT_CLASS3_U8 = 2,   /* (B, H, W) u8 in {0,1,2}: ENET.predict (models.py:55-58,67)         */
    BUGSEG_OUT_BINARY_U8 = 3    /* (B, H, W) u8 in {0,1}:   ENET.predict_binary (models.py:78-81)     */
};

/* out_layout of bugseg_preprocess */
enum {
    BUGSEG_PRE_ENGINE = 0,      /* (B, H, W, 8) engine input, context precision                      */
    BUGSEG_PRE_NCHW_F64 = 1,    /* (B, 3, H, W) f64: exactly ENET.preprocess's array (models.py:84-95) */
    BUGSEG_PRE_NCHW_F32 = 2,    /* (B, 3, H, W) f32: what TF casts the feed to                         */
    BUGSEG_PRE_BGR_U8 = 3       /* (B, H, W, 3) u8: the resized BGR frame only (models.py:87), for
                                   bugseg_enet_forward_bgr, which fuses the rest of preprocess    */
};

/* Geometry of bev_transform_tools.create_occupancy_grid (bev.py:166-195), computed on the host
 * by the Python shim exactly as the reference computes it. */
typedef struct {
    double M[9];        /* forward bev matrix, row-major (bev.py:182 _bev_matrix)                */
    int in_rows;        /* segmap rows  (== "input image size"[0], assert at bev.py:169)        */
    int in_cols;        /* segmap cols  (== "input image size"[1])                               */
    int warp_w;         /* after_warp_width  (bev.py:178; dsize of warpPerspective, bev.py:182)  */
    int warp_h;         /* after_warp_height (bev.py:179)                                        */
    int occ_w_px;       /* bev.py:174 */
    int occ_h_px;       /* bev.py:176 */
    int occ_w;          /* bev.py:173 grid cells across */
    int occ_h;          /* bev.py:175 grid cells down   */
    int left_x;         /* bev.py:183 */
    int top_y;          /* bev.py:184 */
    int ros_layout;     /* 0: reference (occ_h, occ_w) grid; 1: ROS data order = flip(0)+rot90ccw
                           of it, (occ_w, occ_h) row-major (occgrid_to_ros.py:18-25)            */
    int variant;        /* 0: create_occupancy_grid (bev.py:166-246): occupied = template {1,3},
                              encoding {0:-1, 1:100, 2:0, 3:100};
                           1: create_occupancy_grid_binary (bev.py:97-165): occupied = {1}, the
                              reference's uint8 encoding {0:-1, 1:100, 2:0, 3:-100}               */
    int laserscan;      /* 1: laserscan-like mode ("is_laserscan", bev.py:37): variant 0 keeps only the
                              obstacle cells nearest the vehicle along each polar ray, the rest of
                              the obstacles become unknown (bev.py:216-240); variant 1 returns TWO
                              grids per frame, out_dev = (2, B, ...): the encoded grid, then the
                              polar re-projection of its nearest obstacles (bev.py:143-164)        */
} bugseg_bev_params;

/* Library version (major*10000 + minor*100 + patch). */
int bugseg_version(void);

/* Create / destroy a context on HIP device `device`, computing in `precision` (BUGSEG_FP32 is the
 * parity mode: logits within 1e-3 of the fp32 oracle; BUGSEG_BF16 / BUGSEG_F16 the throughput modes).
 * Replaces ENET.__init__'s tf.compat.v1.Session() (models.py:21-22). */
int bugseg_create(int device, int precision, bugseg_ctx **out);
int bugseg_destroy(bugseg_ctx *ctx);

/* Load a BSG1 weight blob (format: bugcar_image_segmentation_amd/enet_spec.py) from HOST memory;
 * folds batch-norm, packs weights for the MFMA kernels and uploads them.
 * Replaces GFile(...).read() + GraphDef.ParseFromString + import_graph_def (models.py:25-30). */
int bugseg_load_weights(bugseg_ctx *ctx, const void *blob, size_t bytes);

/* Number of classes of the loaded model (0 before load). */
int bugseg_num_classes(const bugseg_ctx *ctx);

/* Bytes of the engine-input tensor for (B, H, W) in the context precision. */
size_t bugseg_input_bytes(const bugseg_ctx *ctx, int B, int H, int W);

/* ENET.preprocess (models.py:84-95) on a batch: BGR u8 (B, H0, W0, 3) -> resize to (H, W)
 * (cv2.resize INTER_LINEAR fixed point; identity when equal) -> BGR->RGB -> (x/256-mean)/std.
 * out_layout: BUGSEG_PRE_*. */
int bugseg_preprocess(bugseg_ctx *ctx, const uint8_t *bgr_dev, int B, int H0, int W0, int H, int W,
                      int out_layout, void *out_dev, void *stream);

/* (B, 3, H, W) NCHW float (is_f64 ? f64 : f32) -> engine input (B, H, W, 8). This is the feed of
 * ENET.predict's sess.run (models.py:43-44), which receives ENET.preprocess's NCHW array. */
int bugseg_nchw_to_input(bugseg_ctx *ctx, const void *x_dev, int is_f64, int B, int H, int W,
                         void *out_dev, void *stream);

/* ENet forward + fused argmax/remap epilogue. in_dev: engine input (B, H, W, 8); H and W must be
 * multiples of 8. out_kind: BUGSEG_OUT_*. Replaces sess.run + tf.math.argmax + tf.where
 * (models.py:43-58, 71-80). */
int bugseg_enet_forward(bugseg_ctx *ctx, const void *in_dev, int B, int H, int W, int out_kind,
                        void *out_dev, void *stream);

/* Same as bugseg_enet_forward, but reading raw BGR u8 frames (B, H, W, 3) already at the model
 * resolution: BGR->RGB and (x/256-mean)/std (models.py:89-91) are applied while the initial block
 * loads its input, so the normalised tensor never exists in HBM. Results are identical to
 * bugseg_preprocess(ENGINE) followed by bugseg_enet_forward. */
int bugseg_enet_forward_bgr(bugseg_ctx *ctx, const uint8_t *bgr_dev, int B, int H, int W, int out_kind,
                            void *out_dev, void *stream);

/* bugseg_enet_forward_bgr enqueuing only launches [first_op, last_op) of the forward's plan
 * (last_op = -1: to the end; bugseg_plan_info gives the count). Calling it for [0, k) and then for
 * [k, -1) enqueues exactly the full forward; in between the caller may record an event, so another
 * stream's work can start at a chosen point of this forward (pipeline.py: the shard offset).
 * fp32 range precondition: the range words (the measured max |.| of every stored activation, which
 * pick the launches' power-of-two exponents) are cleared, and the input measured, only by a range that
 * starts at op 0; launches of a range starting at first_op > 0 read the words the earlier launches of
 * the SAME forward wrote — so call [0, k) before [k, -1) on the same input, as pipeline.py does.
 * Started at k > 0 without it, a range uses whatever the last forward left (stale exponents: still
 * overflow-safe, as the words only grow, but not necessarily those of a full forward on this input). */
int bugseg_enet_forward_bgr_ops(bugseg_ctx *ctx, const uint8_t *bgr_dev, int B, int H, int W, int out_kind,
                                void *out_dev, int first_op, int last_op, void *stream);

/* Fused BEV rasteriser over a batch of class maps: seg_dev (B, in_rows, in_cols) u8
 * -> out_dev (B, occ_h, occ_w) int8 (or the ROS layout, see ros_layout).
 * Replaces bev_transform_tools.create_occupancy_grid (bev.py:166-246) or, with variant = 1,
 * create_occupancy_grid_binary (bev.py:97-165), either branch (p->laserscan). The laserscan mode
 * keeps polar tables per geometry in the context and its batch scratch per (context, stream). */
int bugseg_bev_occgrid(bugseg_ctx *ctx, const uint8_t *seg_dev, int B, const bugseg_bev_params *p,
                       int8_t *out_dev, void *stream);

/* The stream-ordered form of bugseg_bev_occgrid: the laserscan batch scratch is a caller-owned
 * device workspace of at least bugseg_bev_workspace_bytes(p, B) bytes (0 when p->laserscan is 0:
 * workspace may then be NULL), used only by the work this call enqueues on `stream` — so the caller's
 * allocator orders its reuse (e.g. torch's caching allocator, graph pools included). */
size_t bugseg_bev_workspace_bytes(const bugseg_bev_params *p, int B);
int bugseg_bev_occgrid_ws(bugseg_ctx *ctx, const uint8_t *seg_dev, int B, const bugseg_bev_params *p,
                          int8_t *out_dev, void *workspace_dev, size_t workspace_bytes, void *stream);

/* Plan introspection for the bench / roofline, for the engine-input entry (bgr_input = 0) or
 * bugseg_enet_forward_bgr (bgr_input = 1), context precision:
 *   n_launches  kernel launches of one forward;
 *   alg_bytes   the network's per-layer algorithmic traffic (every convolution reads its input and
 *               writes its output once, residual branches re-read the block input, weights once per
 *               layer) — a property of the model and shape, the SURVEY.md §8(d) definition;
 *   plan_bytes  the compulsory traffic of this plan (fused launches keep internals on chip);
 *   flops       2 x MACs. */
int bugseg_plan_info(bugseg_ctx *ctx, int B, int H, int W, int out_kind, int bgr_input, int *n_launches,
                     double *alg_bytes, double *plan_bytes, double *flops);

/* Profiling hooks (no reference counterpart): one launch of the cached plan for (B, H, W), as the
 * last forward call at those dimensions left it (its input / output buffers must still be alive).
 * bugseg_plan_op: kernel tag ("init", "conv NR<n> E<epilogue>", "bneck C<c>[ asym]") and the
 * launch's per-layer algorithmic bytes, the bytes it must move, and its flops.
 * bugseg_plan_launch_op: enqueue that one launch on `stream` (bench.py times kernels with it). In
 * the fp32 mode it reads the range words as the last forward left them (see
 * bugseg_enet_forward_bgr_ops) and max-accumulates its own output's into them. */
int bugseg_plan_op(bugseg_ctx *ctx, int B, int H, int W, int op, char *kernel, int kernel_len, double *alg_bytes,
                   double *plan_bytes, double *flops);
int bugseg_plan_launch_op(bugseg_ctx *ctx, int B, int H, int W, int op, void *stream);

/* Last error message of ctx (or of the calling thread when ctx is NULL). Never NULL. */
const char *bugseg_last_error(const bugseg_ctx *ctx);

/* Test hooks (no reference counterpart; host only: no device is touched). The weight-blob parser
 * and packer of bugseg_load_weights, and the polar-table builder of the laserscan mode, for the
 * host-sanitizer tests (tests/asan: truncated / corrupted blobs under ASan + UBSan). Errors go to
 * bugseg_last_error(NULL). */
int bugseg_debug_parse_pack(const void *blob, size_t bytes, int precision, int *ncls);
int bugseg_debug_polar_tables(int w, int h, int variant, int32_t *fmap, size_t fmap_n, int32_t *imap, size_t imap_n,
                              int *pw, int *ph);
/* Test hook: a context fact. what = 0: the fused initial block normalises bytes with the exact affine
 * form (bf16 / fp16; 0 = the table), 1: fp32 range scaling switched off (BUGSEG_F32_RANGE=0 at load),
 * 2: the weights' exponent of packed convolution `arg` (fp32 range scaling; -1000 if no such conv).
 * Returns -1 for an unknown `what` or a NULL ctx. */
int bugseg_debug_ctx_info(const bugseg_ctx *ctx, int what, int arg);
/* Measurement hook (bench.py's in-step kernel table): arm launch spans. spans = device memory of
 * 512 x uint64 per plan op for n_ops ops (NULL disarms): 64 slots 64 B apart, slot k = [k*8] entry,
 * [k*8+1] exit; every later launch of op i < n_ops folds the constant 100 MHz GPU clock into the slots
 * of op i (workgroup w into slot w % 64: min at entry, max at exit) — the caller sets entries to
 * UINT64_MAX and exits to 0 before the run it reads and takes the min / max over the slots. Ops at or
 * beyond n_ops (a plan of another shape) are never armed. Launches already captured keep their slots. */
int bugseg_debug_set_spans(bugseg_ctx *ctx, void *spans, int n_ops);
/* Test hook (tests/test_gpu_range.py): copy the pooling indices the last forward at (B, H, W) wrote for
 * downsampling block `block` (index into the block list) to device memory dst, on `stream`: u8 NHWC
 * (B, h, w, idx_cs), one byte per channel = the window position 2*dy + dx of the first maximum
 * (MaxPoolWithArgmax, models.py:43-44 inside enet.pb). bytes must equal the tensor's size. */
int bugseg_debug_pool_indices(bugseg_ctx *ctx, int B, int H, int W, int block, void *dst, size_t bytes, int *idx_cs,
                              void *stream);

/* ---- DeepLabV3 (BASELINE config 4) -------------------------------------
 * Replaces DeepLabV3 (models.py:98-136): tf.compat.v1.Session + GraphDef import (models.py:105-113)
 * and sess.run("ImageTensor:0" u8 -> "SemanticPredictions:0" int64) (models.py:115-125).
 * The graph builder is host code (deeplab_spec.py): it folds batch-norm, packs the weights into
 * one blob (bugseg_dl_load_weights) and lowers the network to a flat op list over numbered
 * activation buffers for one batch size and crop (bugseg_dl_set_plan). Op records are
 * BUGSEG_DL_OP_FIELDS int32 each; kinds and field meanings are documented in deeplab_spec.py
 * (lower()) and validated here against the buffers and the blob before the plan is accepted. */
#define BUGSEG_DL_OP_FIELDS 32
typedef struct bugseg_dl bugseg_dl;

int bugseg_dl_create(int device, int precision, bugseg_dl **out);
int bugseg_dl_destroy(bugseg_dl *dl);
/* weight blob in HOST memory (bf16 / f32 per the precision, as packed by deeplab_spec.pack) */
int bugseg_dl_load_weights(bugseg_dl *dl, const void *blob, size_t bytes);
/* ops: nops * BUGSEG_DL_OP_FIELDS int32; buf_bytes[nbufs]: arena layout; B frames of at most
 * Hc x Wc (the crop size: 513 for the standard export) */
int bugseg_dl_set_plan(bugseg_dl *dl, const int32_t *ops, int nops, const uint64_t *buf_bytes, int nbufs,
                       int B, int Hc, int Wc);
/* rgb_dev: (B, H, W, 3) u8 RGB, H <= Hc, W <= Wc (padded with the mean pixel to the crop, as the
 * export's preprocessing does); out_dev: (B, H, W) int64 class ids. */
int bugseg_dl_forward(bugseg_dl *dl, const uint8_t *rgb_dev, int B, int H, int W, int64_t *out_dev, void *stream);
/* Profiling hook: enqueue op `op` of the plan alone, on the last forward's I/O buffers. */
int bugseg_dl_launch_op(bugseg_dl *dl, int op, void *stream);
/* Test hook: copy `bytes` of activation buffer `buf` (deeplab_spec.lower's numbering; 7 = the f32
 * logits at the backbone resolution) to a device pointer, on `stream`. */
int bugseg_dl_read_buffer(bugseg_dl *dl, int buf, void *dst_dev, size_t bytes, void *stream);
const char *bugseg_dl_last_error(const bugseg_dl *dl);
/* Test hook (host only): the plan validation of bugseg_dl_set_plan against a weight blob of w_bytes;
 * errors go to bugseg_dl_last_error(NULL). */
int bugseg_dl_debug_check_plan(const int32_t *ops, int nops, const uint64_t *buf_bytes, int nbufs, int B, int Hc, int Wc,
                               int precision, size_t w_bytes);

#ifdef __cplusplus
}
#endif
#endif /* BUGSEG_H */
