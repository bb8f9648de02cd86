/*
 * ydbl.h — C ABI of libydbl.so, the MI355X (gfx950) kernels behind the
 * YOLO-DBL inference hot path (backbone/neck conv stack, Detect decode,
 * class-wise NMS).
 *
 * Boundary rules:
 *   - every entry point is stateless and reentrant, takes caller-owned DEVICE
 *     pointers plus an explicit hipStream_t (passed as void*), and only
 *     enqueues work on that stream (graph-capturable: no malloc, no sync);
 *   - the return value is 0 on success, otherwise a YDBL_E* code, and
 *     ydbl_last_error() returns a thread-local message (the Python layer
 *     raises RuntimeError with it, mirroring the reference's exceptions /
 *     asserts, e.g. U/utils/ops.py:217-218, U/data/loaders.py:554-560);
 *   - activations are NHWC.  A "view" is (pointer, N, H, W, C, channel
 *     stride cs): element (n,y,x,c) lives at ptr[((n*H+y)*W+x)*cs + c].
 *     Writing into a channel slice of a wider buffer (cs > C) is how Concat,
 *     chunk() and C2f/C3 concatenations are done without copies.
 *
 * Reference interfaces replaced (paths relative to
 * /root/reference/models/YOLO/ultralytics):
 *   ydbl_conv2d_nhwc       <- nn/modules/conv.py:39-63 Conv.forward_fuse (conv+bias+SiLU after
 *                             nn/tasks.py:207-235 fuse), conv.py:91-108 DSConv pointwise+BN+SiLU,
 *                             nn.Conv2d 1x1 in Detect/LSKblock/DySample, nn.Linear in AdaHG
 *   ydbl_dsconv_nhwc       <- DSConv.forward conv.py:91-108 (dw + pw + BN + SiLU, one kernel)
 *   ydbl_dwconv2d_nhwc     <- depthwise nn.Conv2d (DSConv.dw conv.py:98, DWConv conv.py:128-133,
 *                             GhostConv.cv2 conv.py:194, LSKblock.conv0/conv_spatial LSKA.py:31-32)
 *   ydbl_dwconv2d_pair_nhwc<- LSKblock.forward LSKA.py:40-41 (conv0 -> conv_spatial, one launch)
 *   ydbl_letterbox         <- BasePredictor.preprocess engine/predictor.py:116-134 for ndarray frames:
 *                             LetterBox.__call__ data/augment.py:1535-1597 (cv2.resize INTER_LINEAR,
 *                             copyMakeBorder 114) + BGR->RGB + HWC->CHW + float /255
 *   ydbl_input_nchw_to_nhwc<- BasePredictor.preprocess engine/predictor.py:116-134 (+ LoadTensor /255)
 *   ydbl_conv_stem         <- preprocess (predictor.py:116-134) fused with the first backbone Conv
 *                             (conv.py:39-63 after fuse), reading the NCHW fp32 batch directly
 *   ydbl_bottleneck_nhwc   <- Bottleneck.forward nn/modules/block.py:355-357 (cv1 -> cv2 [+ x], both
 *                             Conv = conv.py:39-63 after fuse) as one kernel
 *   ydbl_conv_stem2        <- preprocess + the backbone's first two Convs (layers 0-1 of the DBL yamls:
 *                             Conv(3,C0,3,1) -> Conv(C0,2*C0,3,2), conv.py:39-63 after fuse), fp16
 *   ydbl_gate_add          <- FullPAD_Tunnel.forward nn/modules/block.py:1954-1956
 *   ydbl_pool_up_concat    <- FuseModule.forward block.py:1831-1840, DownsampleConv block.py:1927
 *   ydbl_dysample(_ex)     <- DySample.sample modules_upsample/DySample.py:48-61 (grid_sample border)
 *   ydbl_dysample2         <- DySample.forward DySample.py:63-81 (offset conv + sample, one launch)
 *   ydbl_lsk_gate          <- LSKblock.forward LSKA.py:40-52 (mean/max, 7x7 squeeze, sigmoid gating)
 *   ydbl_lsk_attn/_out     <- LSKblock.forward LSKA.py:43-52 (conv1 | conv2 + stats; gate + conv + x *)
 *   ydbl_hg_*              <- AdaHyperedgeGen/AdaHGConv block.py:1627-1708 (ydbl_hg_fused: the whole
 *                             AdaHGConv incl. pre_head_proj block.py:1645, one call)
 *   ydbl_detect_decode     <- Detect._inference head.py:143-181 + DFL block.py:79-83 +
 *                             make_anchors/dist2bbox utils/tal.py:333-357 + NMS candidate
 *                             filter utils/ops.py:234-276
 *   ydbl_pred_candidates   <- utils/ops.py:234-276 on a [B,4+nc,A] prediction tensor
 *   ydbl_nms               <- utils/ops.py:278-310 (+ torchvision.ops.nms, torchvision 0.23.0),
 *                             with clip_boxes utils/ops.py:319-338 as reached through
 *                             scale_boxes :92-127 for tensor sources (gain 1, pad 0)
 *   ydbl_match_predictions <- DetectionValidator._process_batch models/yolo/detect/val.py:209-227
 *                             (box_iou utils/metrics.py:52-71 + BaseValidator.match_predictions
 *                             engine/validator.py:222-262, non-scipy branch)
 */
#ifndef YDBL_H
#define YDBL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { YDBL_OK = 0, YDBL_EINVAL = 1, YDBL_ELAUNCH = 2, YDBL_ECAPACITY = 3 };
enum { YDBL_F32 = 0, YDBL_F16 = 1 };
enum { YDBL_ACT_NONE = 0, YDBL_ACT_SILU = 1, YDBL_ACT_GELU = 2, YDBL_ACT_SIGMOID = 3 };
enum { YDBL_RES_NONE = 0, YDBL_RES_ADD = 1, YDBL_RES_MUL = 2 };

typedef struct {
  void* ptr;  /* device pointer to element (0,0,0,0) of the view */
  int32_t n, h, w, c;
  int32_t cs; /* channel stride in elements (>= c) */
  int32_t dtype;
} ydbl_view;

/* Dense (groups = 1) convolution, implicit GEMM on MFMA (f16: 16x16x32, f32: exact 16x16x4).
 * y = act(conv(x, w) + bias); then res_mode ADD: y = r + y, MUL: y = r * y.
 * w: [cout][kh][kw][cin] in the view dtype, with cin == x.c (x.c must be a multiple of 8),
 *    rows padded to kpad = round_up(kh*kw*cin, 32) elements with zeros.
 * bias: fp32 [cout] or NULL.  r: view or NULL.
 * x.c, y.c multiples of 8 except y.c may be < 8 only when y.cs is a multiple of 4. */
typedef struct {
  ydbl_view x, y, r;
  const void* w;
  const float* bias;
  int32_t kh, kw, stride, pad, dil;
  int32_t kpad;
  int32_t act, res_mode;
  /* Optional second output, FullPAD_Tunnel (nn/modules/block.py:1954-1956) fused into the layer
   * that produces one of its inputs: y2 = a2 * v + b2 * r2, v = the value stored to y (rounded to
   * the view dtype first).  y2.ptr == NULL disables it; y2/r2 have y's shape and dtype. */
  ydbl_view y2, r2;
  float a2, b2;
  /* fp8 operands (f16 activations only): when dq != NULL, w holds OCP e4m3 bytes [cout][kpad]
   * quantized with per-output-channel scales sw, activations are quantized to e4m3 with
   * x * qscale (saturated to +-448) as they are staged, and dq[co] = 1 / (sw[co] * qscale)
   * dequantizes the fp32 accumulator before bias and activation. */
  const float* dq;
  float qscale;
  /* optional split-K scratch (fp32 partial tiles; f16 convs only): workspace_bytes >= ydbl_conv_workspace(d) lets the deep-K
   * wave-split-K path split its k-loop over up to 4 workgroups per tile when the map gives too few tiles to fill the
   * chip (the 20^2 / 40^2 maps of small sub-batches), the partials summed in fixed order by a second kernel that
   * runs the fused epilogue; NULL / too small: no split (same result up to the fp32 summation order) */
  void* workspace;
  int64_t workspace_bytes;
} ydbl_conv_desc;
int ydbl_conv2d_nhwc(const ydbl_conv_desc* d, void* stream);
int64_t ydbl_conv_workspace(const ydbl_conv_desc* d);

/* DSConv in one kernel (conv.py:91-108): y = act(pw(dw(x)) + bias) [+ r], BN folded into pw.
 * dw_w fp32 [k*k][cin], pw_w [cout][kpad] in the view dtype (kpad = round_up(cin, 32), zero
 * padded), bias fp32 [cout].  cin multiple of 32 (f16) / 16 (f32).  The depthwise output is
 * rounded to the view dtype (the reference's intermediate tensor) and never leaves LDS.
 * dw_bias (fp32 [cin] or NULL) and dw_act extend it to the Detect head's DWConv -> Conv1x1 pair
 * (head.py:93-101: dw = SiLU(BN(dwconv)), folded): dw output = dw_act(dw(x) + dw_bias). */
typedef struct {
  ydbl_view x, y, r;
  const float* dw_w;
  const void* pw_w;
  const float* bias;
  int32_t k, stride, pad, dil;
  int32_t kpad, act, res_mode;
  const float* dw_bias;
  int32_t dw_act;
  /* optional trailing 1x1 conv (Detect cls conv cv3[i][2], head.py:93-101) over y's 64 channels:
   * tail_y[p][k] = sum_c tail_w[k][c] * y[p][c] + tail_b[k], k < tail_n <= 4 (y is still written) */
  const float* tail_w;
  const float* tail_b;
  ydbl_view tail_y;
  int32_t tail_n;
  /* optional trailing GEMM (C3's cv3 after its last bottleneck, nn/modules/block.py:259-273, for DSC3k
   * block.py:1447-1503): g2_y[p] = g2_act(g2_w [y[p] ; g2_x[p]] + g2_b), y = this DSConv's output (after
   * the residual), rounded to the view dtype, kept on chip and NOT stored.  g2_w [g2_y.c][y.c + g2_x.c] in
   * the view dtype (k contiguous), g2_b fp32.  Built for fp16, k 7 stride 1, x.c == y.c == g2_x.c ==
   * g2_y.c in {64, 128} (DSC3k2's DSC3k with e = 1); g2_w == NULL disables it. */
  const void* g2_w;
  const float* g2_b;
  ydbl_view g2_x, g2_y;
  int32_t g2_act;
  /* optional leading 1x1 conv (C3's merged cv2 | cv1 ahead of its first DSBottleneck, block.py:259-273 for
   * DSC3k block.py:1447-1503): g0_y[p] = g0_act(g0_w g0_x[p] + g0_b), all g0_y.c channels written, and this
   * DSConv's x is the last x.c channels of g0_y, recomputed on the tile's halo from g0_x instead of read back
   * (x must be exactly that channel slice of g0_y).  g0_w [g0_y.c][g0_x.c] in the view dtype (k contiguous),
   * g0_b fp32.  Built for fp16, k 3 stride 1, g0_x.c == x.c == y.c == 64, g0_y.c == 128; g0_w == NULL
   * disables it. */
  const void* g0_w;
  const float* g0_b;
  ydbl_view g0_x, g0_y;
  int32_t g0_act;
} ydbl_dsconv_desc;
int ydbl_dsconv_nhwc(const ydbl_dsconv_desc* d, void* stream);

/* Depthwise convolution (groups = C), fp32 arithmetic.
 * y = act(dwconv(x, w) + bias), then res_mode ADD: y = r + y (GhostBottleneck identity shortcut).
 * w: fp32 [kh][kw][c]; bias: fp32 [c] or NULL; r: view or ignored. */
typedef struct {
  ydbl_view x, y, r;
  const float* w;
  const float* bias;
  int32_t kh, kw, stride, pad, dil;
  int32_t act, res_mode;
} ydbl_dwconv_desc;
int ydbl_dwconv2d_nhwc(const ydbl_dwconv_desc* d, void* stream);

/* Two chained depthwise convs, d1.x == d0.y: LSKblock's conv0 (5x5) -> conv_spatial (7x7, dil 3)
 * (modules_attention/LSKA.py:40-41).  One launch with the whole map in LDS when H*W <= 512 (the P5
 * maps at 640), bit-identical to the two ydbl_dwconv2d_nhwc launches it falls back to otherwise. */
int ydbl_dwconv2d_pair_nhwc(const ydbl_dwconv_desc* d0, const ydbl_dwconv_desc* d1, void* stream);

/* Input binding: the batch a graph-captured plan reads, chosen when the plan RUNS (YOLO.predict on a device tensor
 * without a staging copy).  When a kernel below gets a non-NULL `bind`, it takes the NCHW fp32 batch pointer from the
 * device word *bind->x (16-byte aligned, the same shape as x) and the scale from the device scalar *bind->amax, the
 * batch maximum, by LoadTensor's rule (U/data/loaders.py:561-566: x / 255 when max > 1 + FLT_EPSILON, else x; the
 * division is the multiply by fp32(1/255) that the GPU division computes) -- instead of x and scale.  A record
 * with both pointers NULL is no binding (x and scale are used); exactly one NULL is an error. */
typedef struct {
  const float* const* x; /* device word holding the batch pointer */
  const float* amax;     /* device fp32 scalar: the batch maximum */
} ydbl_input_bind;

/* The batch maximum of an input binding, on the device (LoadTensor's /255 decision, U/data/loaders.py:561-566), in
 * one launch: amax[0] = max of the n floats at x (16-byte aligned; NaN propagates as in torch.max) and, when scale
 * is not NULL, scale[0] = fp32(1/255) if amax > 1 + FLT_EPSILON else 1.  work: ydbl_batch_max_work_ints() int32
 * prepared by ydbl_batch_max_work_init (every call leaves them so); one work buffer per stream in flight. */
int32_t ydbl_batch_max_work_ints(void);
void ydbl_batch_max_work_init(int32_t* host_work);
int ydbl_batch_max(const float* x, int64_t n, int32_t* work, float* amax, float* scale, void* stream);
/* The same with the batch pointer read from the device word *xword when the launch runs (the first launch of a
 * captured predict graph, include/ydbl.h ydbl_input_bind); the batch must be 16-byte aligned. */
int ydbl_batch_max_bound(const float* const* xword, int64_t n, int32_t* work, float* amax, float* scale,
                         void* stream);

/* NCHW fp32 image batch -> NHWC view (channels >= 3 zero-filled up to y.cs), optional scale (1/255); bind: NULL or
 * the input binding above. */
int ydbl_input_nchw_to_nhwc(const float* x, int32_t n, int32_t c, int32_t h, int32_t w, float scale,
                            const ydbl_view* y, const ydbl_input_bind* bind, void* stream);

/* Stem: y = act(conv_kxk(x * scale) + bias) straight from an NCHW fp32 batch x [n][cin][h][w]
 * (cin = 3), w fp32 [cout][cin][k][k] (torch layout, BN folded), bias fp32 [cout]; y NHWC view with
 * y.c = cout (multiple of 4, <= 64); k = 3, pad = 1, stride 1 or 2.  In f16 mode the scaled input is rounded
 * to f16 before the conv (the reference's .half() input); arithmetic is fp32. */
int ydbl_conv_stem(const float* x, int32_t n, int32_t cin, int32_t h, int32_t w, float scale, const float* wt,
                   const float* bias, int32_t k, int32_t stride, int32_t act, const ydbl_view* y,
                   const ydbl_input_bind* bind, void* stream);

/* y = a + gate * b (FullPAD_Tunnel). */
int ydbl_gate_add(const ydbl_view* a, const ydbl_view* b, float gate, const ydbl_view* y, void* stream);

/* y[..., off0:] = avgpool2(p_lo); y[..., off1:] = p_mid; y[..., off2:] = nearest_up2(p_hi).
 * Any of p_lo / p_mid / p_hi may be NULL (DownsampleConv uses p_lo only). */
int ydbl_pool_up_concat(const ydbl_view* p_lo, const ydbl_view* p_mid, const ydbl_view* p_hi,
                        const ydbl_view* y, void* stream);

/* DySample 'lp' x2 sampling: off view [n,h,w,8*groups] in x's dtype (fp16 in half mode, as the reference's
 * .half() offset conv produces it) holding 0.25*offset+init_pos
 * (channel k = coord*4g + group*4 + i*2 + j), bilinear border grid_sample of x into y [n,2h,2w,c]. */
int ydbl_dysample(const ydbl_view* x, const ydbl_view* off, int32_t groups, const ydbl_view* y, void* stream);
/* Same, descriptor form with an optional second output (y2.ptr != NULL): y2 = a2 * y + b2 * r2 -- a
 * FullPAD_Tunnel (nn/modules/block.py:1954-1956) fed by this DySample, fused into its epilogue. */
typedef struct {
  ydbl_view x, off;
  int32_t groups;
  ydbl_view y, y2, r2;
  float a2, b2;
} ydbl_dysample_desc;
int ydbl_dysample_ex(const ydbl_dysample_desc* d, void* stream);
/* The whole DySample forward (DySample.py:48-81: offset conv + grid_sample) in one launch: off_w [8*groups][c]
 * in x's dtype holds the offset conv weights * 0.25 (K contiguous), off_b fp32 [8*groups] = 0.25 * bias +
 * init_pos (both folds exact); the offsets are rounded to x's dtype as the two-launch path stores them, and the
 * result is bit-identical to ydbl_conv2d_nhwc + ydbl_dysample_ex.  groups = 4, c / groups in {16, 32, 64}. */
typedef struct {
  ydbl_view x;
  const void* off_w;
  const float* off_b;
  int32_t groups;
  ydbl_view y, y2, r2;
  float a2, b2;
} ydbl_dysample2_desc;
int ydbl_dysample2(const ydbl_dysample2_desc* d, void* stream);

/* LSKblock gate: attn view = [a1 | a2] (2*half channels, each half = dim/2);
 * agg = [mean_c, max_c](attn); sig = sigmoid(conv7x7(agg) + sb); out = a1*sig0 + a2*sig1.
 * sw: fp32 [2][2][7][7] (torch layout), sb: fp32 [2]. */
int ydbl_lsk_gate(const ydbl_view* attn, const float* sw, const float* sb, const ydbl_view* out,
                  void* workspace, void* stream);
int64_t ydbl_lsk_gate_workspace(int32_t n, int32_t h, int32_t w);
/* LSKblock after its depthwise pair (LSKA.py:43-52) in two launches, fp16, dim in {256, 512}:
 *   ydbl_lsk_attn: attn = [conv1(a1) + b1 | conv2(a2) + b2] (w12 rows 0..dim/2-1 = conv1, the rest conv2,
 *                  each [dim/2][dim] K-contiguous fp16, b12 fp32 [dim]) and, per pixel, agg = [mean_c, max_c](attn)
 *                  (fp32 [n*h*w][2] in `agg`, the rounded attn reduced in ydbl_lsk_gate's order);
 *   ydbl_lsk_out:  y = x * (conv(a1' * sig0 + a2' * sig1) + b), sig = sigmoid(squeeze7x7(agg) + sb), w [dim][dim/2]
 *                  fp16 K-contiguous, b fp32 [dim] -- the gate never leaves the CU.
 * Bit-identical to ydbl_conv2d_nhwc (conv1, conv2) + ydbl_lsk_gate + ydbl_conv2d_nhwc (conv, RES_MUL) where
 * those run the block GEMM (dim 256).  a1, a2, attn, x, y: [n,h,w,dim] views (channel stride multiple of 8). */
typedef struct {
  ydbl_view x, a1, a2, attn, y;
  const void* w12;
  const float* b12;
  const float* sw;  /* conv_squeeze fp32 [2][2][7][7] */
  const float* sb;  /* [2] */
  const void* w;
  const float* b;
  float* agg;       /* ydbl_lsk_gate_workspace(n, h, w) bytes */
} ydbl_lsk_desc;
int ydbl_lsk_attn(const ydbl_lsk_desc* d, void* stream);
int ydbl_lsk_out(const ydbl_lsk_desc* d, void* stream);

/* Adaptive hypergraph (AdaHGConv), tokens = NHWC pixels of view x (D = x.c, N = h*w). */
typedef struct {
  ydbl_view x;      /* tokens X (input, also the residual) */
  ydbl_view xp;     /* pre_head_proj(X), produced by ydbl_conv2d_nhwc */
  ydbl_view y;      /* output: GELU(node_proj(A @ He)) + X */
  int32_t num_edges, num_heads;
  const float* proto_base;  /* [E][D] */
  const float* ctx_w;       /* [E*D][2D] (context 'both') */
  const float* ctx_b;       /* [E*D] */
  const float* edge_w;      /* [D][D] */
  const float* edge_b;      /* [D] */
  const float* node_w;      /* [D][D] */
  const float* node_b;      /* [D] */
  void* workspace;          /* ydbl_hg_workspace() bytes */
  const void* pre_w;        /* [D][D] pre_head_proj weight in x's dtype (ydbl_hg_fused only; else NULL) */
  const float* pre_b;       /* [D] pre_head_proj bias (ydbl_hg_fused only) */
} ydbl_hg_desc;
int64_t ydbl_hg_workspace(int32_t n, int32_t tokens, int32_t dim, int32_t edges);
/* stage 1: context stats + prototypes (run before the xp GEMM or after; independent of xp) */
int ydbl_hg_context(const ydbl_hg_desc* d, void* stream);
/* stage 2: logits, softmax over tokens, vertex->edge->vertex, residual (needs xp) */
int ydbl_hg_propagate(const ydbl_hg_desc* d, void* stream);
/* The whole AdaHGConv (block.py:1582-1708, pre_head_proj included: xp unused, pre_w/pre_b set) as five plain
 * kernels: three over (64-token slice, image) workgroups writing per-slice partials, two merging them (stream
 * order is the only synchronisation); head_dim 16, (dim, edges) in {64, 128} x {4, 8}.  workspace:
 * ydbl_hg_fused_workspace() bytes, uninitialised memory is fine; -1 = unsupported shape. */
int64_t ydbl_hg_fused_workspace(int32_t n, int32_t tokens, int32_t dim, int32_t edges, int32_t dtype);
int ydbl_hg_fused(const ydbl_hg_desc* d, void* stream);

/* Detect decode + NMS candidate extraction.
 * box[l]: fp32 view [n,h_l,w_l,64] (DFL logits), cls[l]: fp32 view [n,h_l,w_l,nc].
 * Writes, when y_ref != NULL, the reference output layout y[n][4+nc][A] (xywh pixels, sigmoid).
 * Candidates per image (cap each): xyxy boxes, score, class, original flat index
 * (anchor for single-label, anchor*nc+cls for multi-label); cand_count[n] (int32) is
 * zeroed by this call.  classes/ncls: optional class filter. */
typedef struct {
  ydbl_view box[3], cls[3];
  int32_t nl, nc;
  float stride[3];
  float conf_thres;
  int32_t multi_label;
  const int32_t* classes; int32_t nclasses;
  float* y_ref;
  float* cand_box;     /* [n][cap][4] */
  float* cand_score;   /* [n][cap] */
  int32_t* cand_cls;   /* [n][cap] */
  int32_t* cand_idx;   /* [n][cap] */
  int32_t* cand_count; /* [n] */
  int32_t cap;
} ydbl_decode_desc;
int ydbl_detect_decode(const ydbl_decode_desc* d, void* stream);

/* NMS candidates straight from a prediction tensor in the reference layout
 * pred fp32 [n][4+nc][A] (xywh pixels, class scores), as U/utils/ops.py:234-276 reads it.
 * Same candidate outputs / semantics as ydbl_detect_decode. */
typedef struct {
  const float* pred;
  int32_t n, nc, A;
  float conf_thres;
  int32_t multi_label;
  const int32_t* classes; int32_t nclasses;
  float* cand_box; float* cand_score; int32_t* cand_cls; int32_t* cand_idx; int32_t* cand_count;
  int32_t cap;
} ydbl_pred_cand_desc;
int ydbl_pred_candidates(const ydbl_pred_cand_desc* d, void* stream);

/* Batched class-offset NMS over the candidates of ydbl_detect_decode.
 * out: fp32 [n][max_det][6] = x1,y1,x2,y2,conf,cls (kept, score order; rows past the count zeroed),
 * out_count int32 [n].  out_stride / count_stride (0 = dense): floats between images of out (>= max_det * 6)
 * and int32s between images of out_count -- e.g. one record per image [max_det*6 floats | count | pad], so
 * the boxes and counts of a batch-sharded predict travel in ONE all-gather (ydbl.parallel).
 * Semantics of U/utils/ops.py:278-310 + torchvision nms: candidates above max_nms are cut to the
 * max_nms highest scores; boxes offset by cls*max_wh (0 if agnostic); stable descending sort;
 * suppress j if IoU(i,j) > iou_thres (double compare); keep <= max_det.
 * clip_w/clip_h > 0: clamp kept boxes to [0,w]x[0,h] (scale_boxes with gain 1, pad 0).
 * per_image (schedule only, same output): 0 = the class-split sweep for non-agnostic NMS (one workgroup per image
 * and class group + a merge: the faster form when images carry thousands of candidates, e.g. validation's
 * conf 0.001); nonzero = one workgroup per image (the faster form when every image has at most 1024 candidates,
 * the pair-matrix path: predict's conf 0.25 -- DBL-n bs32 +0.8 %, profiles/r05/r05_nms_per_image_ab.txt). */
typedef struct {
  const float* cand_box; const float* cand_score; const int32_t* cand_cls; const int32_t* cand_idx;
  const int32_t* cand_count;
  int32_t n, cap;
  double iou_thres;
  int32_t max_det, max_nms, agnostic;
  float max_wh;
  float clip_w, clip_h;
  float* out; int32_t* out_count;
  void* workspace;
  int64_t out_stride, count_stride;
  int32_t per_image;
} ydbl_nms_desc;
int64_t ydbl_nms_workspace(int32_t n, int32_t cap, int32_t max_nms);
int ydbl_nms(const ydbl_nms_desc* d, void* stream);

/* Stem pair (fp16): y = SiLU(conv3x3_s2(SiLU(conv3x3_s1(x * scale) + b0)) + b1), NHWC [n][ceil(h/2)][ceil(w/2)][2*c0],
 * from the NCHW fp32 batch x [n][3][h][w]; the full-resolution intermediate never leaves LDS.
 * params: device blob of ydbl_conv_stem2_params_size(c0) bytes filled on the HOST by
 * ydbl_conv_stem2_pack from fp32 weights w0 [c0][3][3][3], b0 [c0], w1 [2*c0][c0][3][3], b1 [2*c0]
 * (BN already folded); c0 = 8 or 16.  The first conv's bias enters the MFMA as an fp16 weight on a constant-1 input
 * slot (the reference's .half() bias), the second conv's is added in fp32. */
typedef struct {
  const float* x;
  int32_t n, cin, h, w;
  float scale;
  int32_t c0;
  const void* params;
  ydbl_view y;
  ydbl_input_bind bind; /* {NULL, NULL}: read x / scale */
} ydbl_stem2_desc;
int64_t ydbl_conv_stem2_params_size(int32_t c0);
int ydbl_conv_stem2_pack(const float* w0, const float* b0, const float* w1, const float* b1, int32_t c0, void* out);
int ydbl_conv_stem2(const ydbl_stem2_desc* d, void* stream);

/* Fused Bottleneck (fp16): y = [x +] SiLU(conv3x3(SiLU(conv3x3(x) + b1)) + b2), c -> c/2 -> c channels,
 * stride 1, pad 1 (Bottleneck(c, c, shortcut, e=0.5) with Conv = conv + folded BN + SiLU); the c/2
 * intermediate never leaves LDS.  x, y: NHWC fp16 views of the same shape with x.c == y.c == c
 * (c = 16, 32 or 64), y must not alias x.  params: device blob of ydbl_bottleneck_params_size(c)
 * bytes filled on the HOST by ydbl_bottleneck_pack from fp32 w1 [c/2][c][3][3], b1 [c/2],
 * w2 [c][c/2][3][3], b2 [c] (BN folded).  tile_h: 0 = auto, else 8 or 16 output rows per workgroup (or 9 for
 * c 64 / c_mid 32). */
typedef struct {
  ydbl_view x, y;
  int32_t c;
  int32_t add;
  int32_t tile_h;
  const void* params;
  int32_t c_mid;     /* intermediate channels: 0 = c/2 (Bottleneck e=0.5); 64 with c = 64 (Detect box branch) */
  int32_t pw;        /* 1: params from ydbl_detect_box_pack, y = conv1x1(cv2 output) + b3 (c = c_mid = 64) */
} ydbl_bottleneck_desc;
int64_t ydbl_bottleneck_params_size(int32_t c);
int ydbl_bottleneck_pack(const float* w1, const float* b1, const float* w2, const float* b2, int32_t c, void* out);
/* Same kernel for any (c, c_mid) pair it is built for -- (16,8) (32,16) (64,32) (64,64): two chained
 * 3x3 stride-1 Conv+SiLU, c -> c_mid -> c.  (64,64) replaces the Detect head's box-branch
 * cv2[i][0] -> cv2[i][1] (nn/modules/head.py:86-90) at 64 channels. */
int64_t ydbl_conv3x3_pair_params_size(int32_t c, int32_t c_mid);
int ydbl_conv3x3_pair_pack(const float* w1, const float* b1, const float* w2, const float* b2, int32_t c,
                           int32_t c_mid, void* out);
/* Detect box branch of one level, cv2[i] = Conv3x3(c_in,64) -> Conv3x3(64,64) -> Conv2d 1x1(64,64)+bias
 * (nn/modules/head.py:86-90), as one launch: desc.c = desc.c_mid = 64, desc.pw = 1, x.c = c_in in {64, 128}. */
int64_t ydbl_detect_box_params_size(int32_t c_in, int32_t c);
int ydbl_detect_box_pack(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                         const float* b3, int32_t c_in, int32_t c, void* out);
int ydbl_bottleneck_nhwc(const ydbl_bottleneck_desc* d, void* stream);

/* LetterBox a batch of HWC uint8 BGR frames into one fp32 NCHW RGB canvas batch (values /255).
 * src: frames back to back, frame i at src + src_off[i] (int64 device array);
 * meta int32 device array [n][6] = (h, w, unpad_h, unpad_w, top, left) as LetterBox computes them
 * on the host; out fp32 [n][3][out_h][out_w]; pad_value is the border colour (114).
 * Resize = OpenCV 4.x uint8 INTER_LINEAR (see letterbox.hip for the exact fixed-point rules). */
typedef struct {
  const uint8_t* src; const int64_t* src_off; const int32_t* meta;
  int32_t n, out_h, out_w;
  float pad_value;
  float* out;
} ydbl_letterbox_desc;
int ydbl_letterbox(const ydbl_letterbox_desc* d, void* stream);

/* mAP true-positive matrix of a batch of NMS outputs against ground-truth labels.
 * det fp32 [n][max_det][6] (x1,y1,x2,y2,conf,cls) + det_count int32 [n] (ydbl_nms outputs);
 * labels grouped by image: gt_box fp32 [n_gt][4] xyxy, gt_cls fp32 [n_gt], gt_ofs int32 [n+1]
 * (image b owns labels gt_ofs[b] .. gt_ofs[b+1]-1, gt_ofs[n] == n_gt, original order kept);
 * iouv fp32 [n_iou] thresholds; single_cls: detections count as class 0.
 * correct uint8 [n][max_det][n_iou]: 1 where the detection is a TP at that IoU threshold
 * (rows >= det_count are zeroed).  Bit-exact with the reference for distinct IoUs; an exact IoU
 * tie between two same-class labels of one detection resolves to the larger label index. */
typedef struct {
  const float* det; const int32_t* det_count;
  int32_t n, max_det;
  const float* gt_box; const float* gt_cls; const int32_t* gt_ofs;
  int32_t n_gt;
  const float* iouv; int32_t n_iou;
  int32_t single_cls;
  uint8_t* correct;
  void* workspace; /* ydbl_match_workspace(n, max_det, n_gt, n_iou) bytes */
} ydbl_match_desc;
int64_t ydbl_match_workspace(int32_t n, int32_t max_det, int32_t n_gt, int32_t n_iou);
int ydbl_match_predictions(const ydbl_match_desc* d, void* stream);

const char* ydbl_last_error(void);
const char* ydbl_version(void);

#ifdef __cplusplus
}
#endif
#endif /* YDBL_H */
