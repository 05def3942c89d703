/*
 * isg.h — C-ABI of libisg.so, the MI355X (gfx950) kernels behind the
 * instance-segmentation hot path.
 *
 * The reference (YanMiaoW/instanceSegmentation) is pure Python with no FFI; every
 * entry point below replaces the torch eager kernels that one reference call site
 * runs (file:line into /root/reference). The Python host
 * (instancesegmentation_amd/_lib.py, ctypes) binds exactly these symbols; see
 * INTEGRATION.md for the binding a maintainer adds on the reference side.
 *
 * Conventions:
 *   - all tensors are fp32 NCHW device pointers owned by the caller (torch's caching
 *     allocator); the library never allocates, frees or synchronises;
 *   - "virtual" inputs (isg_vtensor) are raw conv outputs plus a per-channel
 *     transform applied on load (BatchNorm fwd + activation, or BatchNorm bwd);
 *     channel segments let a consumer read a concat without materialising it;
 *   - every call enqueues on the caller's hipStream_t and returns 0, or a negative
 *     status with a thread-local message in isg_last_error();
 *   - functions are stateless and re-entrant (backward runs on torch's autograd
 *     worker thread).
 */
#ifndef ISG_H
#define ISG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* isg_stream_t; /* == hipStream_t */

#define ISG_OK 0
#define ISG_ERR_INVALID -1
#define ISG_ERR_UNSUPPORTED -2
#define ISG_ERR_HIP -3

#define ISG_MAX_SEGS 3
#define ISG_MAX_CH 512
#define ISG_LIST_CHUNK 32
/* Every cross-workgroup accumulator (BN statistics, PReLU slope and bias sums) is kept
 * in ISG_STAT_REP replicas, each workgroup adding into one chosen by its block index,
 * so at most (workgroups / ISG_STAT_REP) atomics contend on an address; readers sum the
 * replicas. An accumulator "of n values" therefore occupies ISG_STAT_REP*n doubles,
 * replica r at offset r*n. (Overridable at build time for experiments; the Python side
 * reads the count back through isg_stat_replicas.) */
#ifndef ISG_STAT_REP
#define ISG_STAT_REP 4
#endif

enum { ISG_ACT_NONE = 0, ISG_ACT_RELU = 1, ISG_ACT_PRELU = 2 };
enum { ISG_XF_PLAIN = 0, ISG_XF_BN_FWD = 1, ISG_XF_BN_BWD = 2 };
enum { ISG_SINK_STORE = 0, ISG_SINK_ACCUM = 1, ISG_SINK_ACTBWD = 2, ISG_SINK_NONE = 3 };

/* One BatchNorm2d layer (segment.py:41 `nn.BatchNorm2d(c2)`; eps 1e-5, momentum 0.1).
 * stats layout: [sum(C) | sumsq(C) | gsum(C) | gxsum(C)] in double; sum/sumsq are of
 * the raw (pre-BN, bias included) conv output over N*H*W, gsum of the gradient g
 * w.r.t. the BN output and gxsum of g*(y - mean), accumulated centred so the BN
 * backward never cancels against mean*gsum. train=0 uses the running statistics.
 * The 4*C block is replicated ISG_STAT_REP times (4*C*ISG_STAT_REP doubles). */
typedef struct {
    const float* gamma;
    const float* beta;
    const float* running_mean;
    const float* running_var;
    double* stats;
    int32_t C;
    int32_t train;
    float count; /* N*H*W */
    float eps;
    /* Finalised per-channel coefficients (8*C floats), or NULL: forward [C][4] =
     * (mean, gamma*rstd, beta, 0) then backward [C][4] = (A, B, mean, C) of
     * dy = A*g + B*(y - mean) + C. Written by isg_bn_finalize once per layer and step
     * so consumers read 16 bytes per channel instead of reducing the fp64 replicas;
     * NULL makes every consumer derive them from `stats` (or the running stats). */
    float* coef;
} isg_bn;

/* A channel segment of a virtual tensor.
 *   PLAIN : v = p
 *   BN_FWD: v = act((p - mean) * gamma*rstd + beta)            (Conv.forward, segment.py:44-45)
 *           with y non-NULL (a residual block's tail read by its consumer):
 *           v = act((p - mean) * gamma*rstd + beta + y)        (segment.py:75-77: out += residual;
 *           prelu) — accepted only by the 1x1 stride-1 conv forward, one segment (any
 *           sinks: a stacked sibling pair's two)
 *   BN_BWD: v = dL/d(conv output) rebuilt from g (= dL/d BN-output) and the forward
 *           raw y: A*g + B*(y - mean) + C                       (BatchNorm2d backward) */
typedef struct {
    const float* p;
    const float* y;        /* BN_BWD: saved raw output (NULL: y = p, with p's n_stride);
                              BN_FWD: residual term or NULL */
    int64_t n_stride;      /* elements between images of p */
    int64_t y_n_stride;
    int32_t C;
    int32_t xform;
    int32_t act;           /* BN_FWD only */
    int32_t pad_;
    const float* slope;    /* PReLU weight [C] (segment.py:24 nn.PReLU(planes)) */
    isg_bn bn;
} isg_vseg;

typedef struct {
    isg_vseg s[ISG_MAX_SEGS];
    int32_t nseg;
    int32_t N, H, W;       /* C = sum of segment channels */
    /* non-NULL: the consumer also writes the transformed values v here ([N][C][H][W] at
     * mat_n_stride per image) — the materialised block output a residual tail would have
     * written; 1x1 stride-1 conv forward with one segment only */
    float* mat;
    int64_t mat_n_stride;
    /* the residual term's own BatchNorm (a tail of two BatchNorm'd conv outputs,
     * segment.py:147-148, 202-207): when rbn.stats or rbn.coef is set the residual form
     * reads act(BN(p) + BN2(y)) */
    isg_bn rbn;
} isg_vtensor;

/* Where a kernel writes channels [c0, c0+C) of its result.
 *   STORE : p = v + bias; optional BN sum/sumsq into stats   (forward conv outputs)
 *   ACCUM : p += v                                            (gradient of a consumed tensor)
 *   ACTBWD: v is dL/dz for z = act(BN(y)); writes g = v*act'(BN(y)) into p and
 *           accumulates bn.stats gsum/gxsum and the PReLU slope gradient.
 *           Residual form (r non-NULL; a block tail's backward folded into the input
 *           gradient of the next block's first 1x1, segment.py:75-77): v' = v + old,
 *           z = BN(y) + r, g = v'*act'(z) into p and, when p2 is non-NULL, also into p2
 *           (the residual term's gradient; STORE, or ACCUM with p2_accum); statistics as
 *           ACTBWD with v'. Accepted only by the 1x1 stride-1 input gradient with one
 *           sink (any gradient segments: a stacked sibling pair's two). */
typedef struct {
    float* p;
    int64_t n_stride;
    int32_t c0, C;
    int32_t mode;
    int32_t act;
    const float* bias;
    double* stats;         /* STORE/ACCUM: a BN-layout block (4*C per replica) whose
                              sum/sumsq halves receive the output sums, or NULL */
    const float* y;        /* ACTBWD */
    int64_t y_n_stride;
    const float* slope;    /* ACTBWD + PRELU */
    double* slope_grad;    /* ACTBWD + PRELU, C doubles per replica */
    isg_bn bn;             /* ACTBWD; bn.stats==NULL means "no BN" (identity) */
    const float* r;        /* ACTBWD residual form: the tail's residual term, or NULL */
    int64_t r_n_stride;
    const float* old;      /* ACTBWD residual form: gradient already accumulated for v, or NULL */
    int64_t old_n_stride;
    float* p2;             /* ACTBWD residual form: second output of g, or NULL */
    int64_t p2_n_stride;
    int32_t p2_accum;      /* p2 += g instead of p2 = g */
    int32_t pad2_;
    isg_bn rbn;            /* ACTBWD residual form: the residual's own BatchNorm (stats or coef
                              set): z = BN(y) + BN2(r); rbn.stats receives Σg and Σg(r - mean2) */
} isg_sink;

typedef struct {
    isg_sink s[ISG_MAX_SEGS];
    int32_t nsink;
    int32_t pad_;
} isg_sinks;

typedef struct {
    int32_t N, Ci, H, W;         /* conv input  */
    int32_t Co, OH, OW;          /* conv output */
    int32_t KH, KW, SH, SW, PH, PW, DH, DW;
    int32_t groups;              /* 1 (dense) or Ci == Co (depthwise) */
    /* input channels of the weight tensor when the conv reads only its first Ci (0 = Ci):
     * the keypoint stem runs the dense conv over the RGB channels of a weight
     * [Co][w_ci][KH][KW] (isg_kp_stem below); tap_conv forward / tap_wgrad only */
    int32_t w_ci;
    int32_t pad_;
} isg_conv_geom;

/* Residual-block tail: out = act(sum_i term_i), term_i = vtensor channel-aligned
 * with the output, optionally nearest-upsampled x2 (segment.py:76-77, 107-109,
 * 147-148, 202-207, 255-259, 331-333). */
typedef struct {
    isg_vseg term[3];
    int32_t up[3];
    int32_t nterm;
    int32_t act;
    const float* slope;
    float* out;
    int64_t out_n_stride;
    int32_t N, C, H, W;
} isg_tail;

typedef struct {
    isg_tail f;
    const float* dout;        /* dL/d out */
    int64_t dout_n_stride;
    float* g;                 /* dL/d(sum) written here when non-NULL */
    int64_t g_n_stride;
    float* dterm[3];          /* PLAIN terms: gradient destination (ACCUM or store) */
    int64_t dterm_n_stride[3];
    int32_t dterm_accum[3];
    double* slope_grad;
} isg_tail_grad;

/* ---- forward / backward building blocks -------------------------------- */

/* Dense or depthwise conv forward: y = conv(x) (+bias, BN stats) into `out` sinks.
 * Replaces nn.Conv2d.forward inside Conv (segment.py:39-45) and the bare convs at
 * segment.py:91-92, 323, 343, 437. Dense convs run as implicit GEMM on
 * v_mfma_f32_16x16x4_f32; depthwise on VALU. */
int32_t isg_conv_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                     const isg_sinks* out, isg_stream_t stream);

/* Input gradient of a conv: dx = conv^T(dy, w) into per-segment sinks. */
int32_t isg_conv_dgrad(const isg_conv_geom* g, const isg_vtensor* dy, const float* w,
                       const isg_sinks* dx, isg_stream_t stream);

/* Weight/bias gradient: dw += sum dy (x) im2col(x); dbias += sum dy (either may be
 * NULL), into fp64 accumulators that the caller zeroes before the first contribution and
 * folds to fp32 with isg_sum_replicas (nrep 1). */
int32_t isg_conv_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                       double* dw, double* dbias, isg_stream_t stream);

/* Weight-gradient replicas. A dW element receives one atomic add from every workgroup
 * along the pixel dimension (hundreds); same-address atomics serialise at the memory
 * side (~40 ns each), so the wgrad kernels add into one of `nrep` replicas of dw/dbias
 * (replica r at dw + r*rep_stride elements), chosen per workgroup, and one
 * isg_sum_replicas pass folds them at the end of the backward.
 *
 * The replicas are fp64 and every addend is a workgroup's fp32 partial (reduced in a fixed
 * order inside the workgroup): an fp64 sum of fp32 values is EXACT — so the same whatever
 * order the atomics land in — as long as the running sum stays within 2^29 of the smallest
 * addend's magnitude (53 - 24 significand bits), and otherwise off by at most 2^-53 of
 * the running sum, 2^-29 of the fp32 result's rounding step. The fold sums the replicas in
 * fixed order and rounds once to fp32. With the BatchNorm statistics (fp64 sums of fp32
 * workgroup partials, the same argument) the backward is reproducible bit for bit across
 * runs WHILE every element's partials span less than 2^29 in magnitude; outside that range
 * an fp64 sum can differ in its last bit with the atomic order, which can flip the fp32
 * rounding: then within 1 fp32 ulp, not bitwise. The fixtures and the bench batch stay
 * inside the range (tests/test_gpu_trainer.py::test_backward_is_bitwise_reproducible
 * asserts exact equality of logits and gradients there). The summed
 * LOSS is not covered: isg_bce_sigmoid adds fp64 workgroup partials (not fp32 ones), so its
 * last bits depend on the atomic order. With fp32 replicas nothing was reproducible
 * (VERDICT r04). */
#define ISG_WREP 16
int32_t isg_conv_wgrad_rep(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                           double* dw, double* dbias, int64_t rep_stride, int32_t nrep,
                           isg_stream_t stream);
/* Both backward halves of one depthwise layer (segment.py:63-64 groups=planes, the
 * Bottleneck blocks' 3x3 / 5x1 / 1x5): dx through the one sink `dx` (as isg_conv_dgrad;
 * NULL or nsink 0 skips it) and dw / dbias accumulated into replicas (as
 * isg_conv_wgrad_rep; dw NULL skips it), in ONE launch when both tile kernels apply
 * (same-size layer, W % 4 == 0, 16-B aligned sink rows): the dy tile is staged once. Same
 * partials and reduction order as the two calls, so the results are bitwise theirs. */
int32_t isg_depthwise_bwd(const isg_conv_geom* g, const isg_vtensor* dy, const float* w,
                          const isg_sinks* dx, const isg_vtensor* x, double* dw, double* dbias,
                          int64_t rep_stride, int32_t nrep, isg_stream_t stream);
/* dst[i] = (float) sum_{r<nrep} src[r*stride + i] for i < n (fp64, fixed order). */
int32_t isg_sum_replicas(float* dst, const double* src, int64_t n, int32_t nrep, int64_t stride,
                         isg_stream_t stream);

/* ConvTranspose2d forward (segment.py:305-306, 435-436) with kernel = 2*stride,
 * weight [Ci][Co][K][K], as a sub-pixel direct kernel. geom describes the transposed
 * conv: input (N,Ci,H,W) -> output (N,Co,OH,OW), KH=KW=K, SH=SW=s, PH=PW=p. */
int32_t isg_convT_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                      const isg_sinks* out, isg_stream_t stream);

/* Max-pool k x k stride k (segment.py:29, 145) of a virtual tensor into a slice. */
int32_t isg_maxpool_fwd(const isg_vtensor* x, int32_t k, float* out, int64_t out_n_stride,
                        isg_stream_t stream);
/* Route dL/d out to the arg-max of each window (first max wins, torch CPU semantics). */
int32_t isg_maxpool_bwd(const isg_vtensor* x, int32_t k, const float* dout,
                        int64_t dout_n_stride, const isg_sinks* dx, isg_stream_t stream);

int32_t isg_tail_fwd(const isg_tail* t, isg_stream_t stream);
int32_t isg_tail_bwd(const isg_tail_grad* t, isg_stream_t stream);

/* BatchNorm running-stat update for `nitems` layers; `items` is a HOST array (copied
 * into kernel arguments in chunks of ISG_LIST_CHUNK) (torch BatchNorm2d train semantics):
 * rm = (1-m) rm + m mean; rv = (1-m) rv + m var*M/(M-1); nbt += 1. */
typedef struct {
    const double* stats;
    float* running_mean;
    float* running_var;
    int64_t* num_batches_tracked;
    int32_t C;
    float count;
    float momentum;
    int32_t pad_;
} isg_bn_update;
int32_t isg_bn_update_running(const isg_bn_update* items, int32_t nitems, isg_stream_t stream);

/* Coefficient finalisation for `nitems` BatchNorm layers (HOST array, chunked like
 * isg_bn_update_running): from the replicated fp64 statistics write items[i].coef's
 * forward half (bwd == 0, after the forward statistics are complete) or backward half
 * (bwd == 1, after the gsum/gxsum statistics are complete). Same fp64 formulas the
 * consumers would evaluate (BatchNorm2d train: biased variance, eps). */
int32_t isg_bn_finalize(const isg_bn* items, int32_t nitems, int32_t bwd, isg_stream_t stream);

/* Parameter-gradient finalisation (HOST item array, like isg_bn_update_running):
 *   dgamma = rstd*gxsum, dbeta = gsum,
 *   dbias(conv before BN) = sum of rebuilt dy, dslope = double accumulator -> float. */
typedef struct {
    const double* stats;       /* BN stats (4*C per replica) or NULL */
    const float* gamma;
    const float* running_mean; /* eval-mode backward */
    const float* running_var;
    float* dgamma;
    float* dbeta;
    float* dconv_bias;         /* may be NULL */
    const double* slope_acc;   /* may be NULL (then stats describe a BN) */
    float* dslope;
    int32_t C;
    int32_t train;
    float count;
    float eps;
    int32_t slope_stride;      /* replica stride of slope_acc in doubles: C for a PReLU
                                  slope, 4*C for the sum half of a sink's stats block */
    int32_t pad_;
} isg_grad_final;
int32_t isg_grad_finalize(const isg_grad_final* items, int32_t nitems, isg_stream_t stream);

/* The end of a world-size-1 training step as ONE launch (train_instance.py:379-380:
 * the gradient complete, then optimizer.step()): fold the weight-gradient replicas
 * (isg_sum_replicas) into `grad` and apply Adam (isg_adam_dev's arithmetic, step already
 * advanced by isg_step_inc) to every folded element; finalise the statistics-derived
 * gradients of the `ngf` items (isg_grad_finalize) into `grad` and apply Adam to those; update
 * the running statistics of the `nbnu` BatchNorm layers (isg_bn_update_running). `gf` and
 * `bnu` are DEVICE arrays. owner[i]: bit 0 = Adam updates element i (a used parameter),
 * bit 1 = a grad_final item writes grad[i] (the fold skips it). Bitwise the result of those
 * separate calls. hyper = (lr, beta1, beta2, eps, weight_decay), device doubles. */
typedef struct {
    float* grad;
    const double* rep;         /* nrep replicas, replica stride n */
    int64_t n;
    int32_t nrep;
    int32_t ngf;
    float* param;
    float* exp_avg;
    float* exp_avg_sq;
    const uint8_t* owner;
    const int32_t* step;
    const double* hyper;
    const isg_grad_final* gf;
    const isg_bn_update* bnu;
    int32_t nbnu;
    int32_t pad_;
} isg_step_tail_args;
int32_t isg_step_tail(const isg_step_tail_args* args, isg_stream_t stream);
/* step += 1 on the device (the 1-based Adam step of isg_step_tail / isg_adam_dev). */
int32_t isg_step_inc(int32_t* step, isg_stream_t stream);

/* sigmoid + nn.BCELoss(mean) forward and backward in one pass (segment.py:534,
 * train_instance.py:299,378-379), torch clamp semantics: log clamped at -100,
 * dL/dp = (p-y)/max(p(1-p),1e-12)/n, dL/dlogit = dL/dp * p(1-p).
 * loss_acc: one double (sum); dlogits may be NULL. */
int32_t isg_bce_sigmoid(const float* logits, const float* target, int64_t n, double* loss_acc,
                        float* dlogits, float grad_scale, isg_stream_t stream);
int32_t isg_sigmoid_fwd(const float* x, float* y, int64_t n, isg_stream_t stream);
int32_t isg_sigmoid_bwd(const float* y, const float* dy, float* dx, int64_t n,
                        isg_stream_t stream);

/* torch.optim.Adam (defaults lr 1e-3, betas (0.9,0.999), eps 1e-8; train_instance.py:297)
 * over a flat fp32 buffer. `live` (uint8 per element, may be NULL) masks parameters
 * whose grad is None (they are skipped, as torch does). step is 1-based. The
 * hyperparameters are doubles, as torch's python floats: 1-beta and the bias corrections
 * are rounded from them the way torch does, so a torch optimizer state continues here
 * bit-for-bit in the update formula. */
int32_t isg_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                 const uint8_t* live, int64_t n, int32_t step, double lr, double beta1,
                 double beta2, double eps, double weight_decay, isg_stream_t stream);

/* Same update with the step counter in device memory: *step is incremented on the
 * stream first, then used — the launch sequence can be captured in a HIP graph and
 * replayed (the host-side form bakes `step` into the kernel arguments). */
int32_t isg_adam_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                     const uint8_t* live, int64_t n, int32_t* step, double lr, double beta1,
                     double beta2, double eps, double weight_decay, isg_stream_t stream);

int32_t isg_fill_f64(double* p, int64_t n, double v, isg_stream_t stream);

/* Timestamp t of the chip-global 100 MHz counter (s_memrealtime) when this launch runs on
 * the stream, accumulated into buf (uint64, two's complement): buf[slot] += sign < 0 ? -t : t
 * (slot 0 or 1), buf[2] = max(buf[2], t), buf[3] = min(buf[3], t). A (-, +) pair around one
 * op of the executor's list (the OP_STAMP record) sums that op's time where it runs in the
 * step, over every replay of one HIP graph (bench.py's roofline; ROCm rejects timing events
 * recorded under graph capture). */
int32_t isg_stamp(uint64_t* buf, int32_t slot, int32_t sign, isg_stream_t stream);

/* ---- infer post-process (build-defined; infer.py:32-36 is a stub) -------- */

/* A13: paste K crop probability maps [K,S,S] back onto an HxW canvas through their
 * crop windows boxes[K][4] = (x0,y0,x1,y1), bilinear, uint8 by truncation of p*255
 * (train_instance.py:398-399). Contract: oracle/maskops_oracle.py (bit-exact). */
int32_t isg_mask_paste(const float* prob, int32_t K, int32_t S, const int32_t* boxes,
                       int32_t H, int32_t W, uint8_t* out, isg_stream_t stream);

/* A14: per-mask count/sum/score and greedy mask-NMS (K <= 256). keep[K] receives the
 * kept indices in keep order, *nkeep their number (both device memory).
 * work: isg_mask_nms_workspace(K,H,W) bytes, caller-owned. */
int64_t isg_mask_nms_workspace(int32_t K, int32_t H, int32_t W);
int32_t isg_mask_nms(const uint8_t* masks, int32_t K, int32_t H, int32_t W, float iou_thr,
                     void* work, float* scores_out, int32_t* keep, int32_t* nkeep,
                     isg_stream_t stream);

/* A13 + A14 in one pass (the infer product path): isg_mask_paste's canvases written and
 * bit-packed for the NMS in the same kernel (no memset, no re-read of the canvases),
 * then isg_mask_nms's intersections and greedy suppression. Same outputs, bit-exact to
 * isg_mask_paste followed by isg_mask_nms; work: isg_mask_nms_workspace(K,H,W) bytes. */
int32_t isg_mask_paste_nms(const float* prob, int32_t K, int32_t S, const int32_t* boxes,
                           int32_t H, int32_t W, float iou_thr, uint8_t* masks, void* work,
                           float* scores_out, int32_t* keep, int32_t* nkeep, isg_stream_t stream);

/* ---- infer pre-process ----------------------------- */

/* Per-instance crop: window k = (x0,y0,x1,y1) of an HxWx3 uint8 RGB image (instance box
 * +/- 16 px, may reach outside the image) resampled to SxS, rounded to uint8 and
 * normalised to [-1,1] into out[K][3][S][S]; pixels outside valid[k] = (x0,y0,x1,y1)
 * (the image minus what the centring translation moved out of the frame) read as the
 * fill value 0. Replaces the reference's translate + CropAndPad + Resize +
 * ToTensor/Normalize test branch (train_instance.py:139-196, :80-85; imgaug/cv2 absent:
 * contract frozen in oracle/infer_oracle.py, bit-exact). */
int32_t isg_instance_crop(const uint8_t* image, int32_t H, int32_t W, const int32_t* windows,
                          const int32_t* valid, int32_t K, int32_t S, float* out,
                          isg_stream_t stream);

/* keypoint2heatmaps (train_instance.py:33-68) for K instances: keypoints[K][nparts][3] =
 * (x, y, visible) in double, out[K][nparts][H][W] float32 (zeroed, then each visible
 * keypoint's window written with the float32 of the double-precision Gaussian). */
int32_t isg_keypoint_heatmaps(const double* keypoints, int32_t K, int32_t nparts, int32_t H,
                              int32_t W, double sigma, double threshold, float* out,
                              isg_stream_t stream);

/* ---- keypoint stem ------------------------------------ */

/* The stem of Segment(20) (init_head_s4, segment.py:19-31, on cat(image, heatmaps),
 * segment.py:531-532) with the 17 heatmaps (train_instance.py:33-68) never written to
 * HBM: map j of image n is exp(-((x-kx)^2+(y-ky)^2)/sigma^2) (double, stored float) inside
 * keypoint j's window [max(0,int(kx-r)), min(W-1,int(kx+r+1))) x (same in y), where it
 * exceeds the threshold, and 0 elsewhere; keypoints[n][j] = (kx, ky, visible > 0).
 *   fwd  : y[n][co] += sum_{j,tap} w[co][c_kp0+j][tap] * map_j   over the output pixels a
 *          window reaches (y holds the dense conv of the first c_kp0 channels + bias);
 *          stats (BN sum / sum^2 replicas, 4*Co doubles each) get the change of sum and
 *          sum^2 of every changed pixel
 *   wgrad: dw[co][c_kp0+j][tap] += sum_p dy[co][p] * map_j(tap(p)), dy a vtensor
 *   pool : out[n][c0+j] = max_pool(map_j, k) (k x k windows, stride k)
 * geom: the conv (Ci = the weight's input channels, Co <= 16, groups 1). */
typedef struct {
    const double* kp;            /* [N][nparts][3] */
    int32_t nparts, c_kp0;
    double sigma, threshold;
    isg_conv_geom g;
    const float* w;              /* fwd */
    float* y;                    /* fwd: raw conv output [N][Co][OH][OW] */
    int64_t y_n_stride;
    double* stats;               /* fwd: NULL or the output's BN statistics block */
    isg_vtensor dy;              /* wgrad */
    double* dw;                  /* wgrad: [Co][Ci][KH][KW] fp64 (+ replicas) */
    int64_t rep_stride;
    int32_t nrep;
    int32_t k;                   /* pool: window */
    float* out;                  /* pool */
    int64_t out_n_stride;
} isg_kp_stem;

int32_t isg_kp_stem_fwd(const isg_kp_stem* a, isg_stream_t stream);
int32_t isg_kp_stem_wgrad(const isg_kp_stem* a, isg_stream_t stream);
int32_t isg_kp_pool(const isg_kp_stem* a, isg_stream_t stream);

/* ---- fused mask head (segment.py:435-438, 504-505) ------------------------ */

/* bottle6_1 = ConvTranspose2d(16 -> 4, k8, s4, p2) followed by bottle6_2 = Conv2d(4 -> 1,
 * 3x3, p1) (no nonlinearity between them), with the 4-channel full-resolution
 * intermediate kept on chip (never recomputed in the backward).
 *   fwd: out = logits [N,1,4Hi,4Wi]; when `ring` is non-NULL also the UN-cropped
 *        intermediate (bias included) on the one-pixel ring just outside the 4Hi x 4Wi
 *        image, per image [4 channels][ISG_HEAD_RING(Hi, Wi)]: row -1 (columns -1 .. 4Wi),
 *        row 4Hi (same), column -1 (rows 0 .. 4Hi-1), column 4Wi (same). The backward
 *        needs it (the 3x3's weight gradient border term).
 *   bwd: dx (sinks: STORE / ACCUM without statistics) = dL/dx; dw1/db1/dw2/db2 += the
 *        parameter gradients, added into replica (workgroup % nrep) of each (replica r at
 *        + r*rep_stride elements; NULL skips one); `ring` as written by the forward
 *        (required). Replaces the unfused isg_convT_fwd + isg_conv_fwd (+ their dgrad /
 *        wgrad) pair, which round-trips the intermediate through HBM. */
#define ISG_HEAD_RING(Hi, Wi) (2 * (4 * (int64_t)(Wi) + 2) + 2 * 4 * (int64_t)(Hi))
typedef struct {
    isg_vtensor x;               /* [N,16,Hi,Wi] */
    const float* w1;             /* ConvTranspose2d weight [16][4][8][8] */
    const float* b1;             /* [4] or NULL */
    const float* w2;             /* Conv2d weight [1][4][3][3] */
    const float* b2;             /* [1] or NULL */
    float* out;                  /* fwd */
    int64_t out_n_stride;
    const float* dout;           /* bwd: dL/dlogits */
    int64_t dout_n_stride;
    isg_sinks dx;                /* bwd */
    double* dw1;                 /* bwd: fp64 accumulators (+ replicas, isg_conv_wgrad_rep) */
    double* db1;
    double* dw2;
    double* db2;
    int64_t rep_stride;
    int32_t nrep;
    int32_t N, Hi, Wi;
    int32_t pad_;
    float* ring;                 /* [N][4][ISG_HEAD_RING(Hi, Wi)] (fwd: written if non-NULL; bwd: read) */
    /* bwd: non-NULL = each workgroup STORES its fp32 dW1 partial here ([blocks][4096],
     * isg_mask_head_part_floats) instead of adding it into dw1, and isg_mask_head_fold
     * adds the partials into dw1's replicas later (off the critical path: the end-of-
     * workgroup fp64 atomics of the 4096 dW1 values were the kernel's tail) */
    float* dw1_part;
} isg_mask_head;

int32_t isg_mask_head_fwd(const isg_mask_head* a, isg_stream_t stream);
int32_t isg_mask_head_bwd(const isg_mask_head* a, isg_stream_t stream);
/* floats of the backward's dW1 partial slab for an N x 16 x Hi x Wi input */
int64_t isg_mask_head_part_floats(int32_t N, int32_t Hi, int32_t Wi);
/* dw1 replicas += the partial slab (fp64 sums of the fp32 partials: exact, so the result
 * is the one of the in-kernel atomics, bit for bit) */
int32_t isg_mask_head_fold(const isg_mask_head* a, isg_stream_t stream);

/* ---- plan executor ------------------------------------------------------ */

/* A recorded op list (built once per input shape by the Python planner) replayed
 * with a table of base pointers: pointer = table[slot] + byte offset. */
typedef struct {
    int32_t slot;
    int32_t pad_;
    int64_t offset;
} isg_ref;

int32_t isg_exec(const void* ops, int32_t nops, void* const* table, isg_stream_t stream);

/* Same, with a side stream: ops flagged "side" in their record header (the weight
 * gradients, which nothing later in the list reads) are forked onto `side` after every
 * op issued before them on `stream`; ops flagged "join" (and the end of the list) wait
 * for all forked work. side == NULL runs everything on `stream`. Under HIP-graph
 * capture the fork/join become graph edges, so the weight gradients overlap the
 * input-gradient chain. Header flags (api.cpp OpHdr.flags): bit 0 side, bit 1 join,
 * bit 2 fork-now (the side op depends on everything issued on `stream` so far; consecutive
 * fork-now ops share one fork), bits 8+ of a join: how many of the most recent side ops it
 * does NOT wait for (0: all). Side ops are otherwise issued in batches of 16 behind one
 * fork each. */
int32_t isg_exec_ms(const void* ops, int32_t nops, void* const* table, isg_stream_t stream,
                    isg_stream_t side);

/* Same with a second side stream: a forked batch made only of weight gradients (independent
 * atomic accumulations) is dealt alternately over `side` and `side2`, so two of their small
 * grids run at once; every other side op stays in order on `side`. side2 == NULL is
 * isg_exec_ms. */
int32_t isg_exec_ms2(const void* ops, int32_t nops, void* const* table, isg_stream_t stream,
                     isg_stream_t side, isg_stream_t side2);

/* sizeof() of the ABI structs and executor records (0 vtensor, 1 sinks, 2 conv record,
 * 3 wgrad record, 4 pool record, 5 tail, 6 tail_grad, 7 bn_update, 8 grad_final,
 * 9 bce record, 10 conv_geom, 11 bn, 12 vseg, 13 sink, 14 sum_rep record, 15 kp_stem,
 * 16 mask_head, 17 stamp record, 18 depthwise-backward record, 19 step tail) so
 * bindings can verify layouts. */
int32_t isg_record_size(int32_t which);

const char* isg_last_error(void);
int32_t isg_abi_version(void);
/* ISG_STAT_REP the library was built with (accumulator replica count). */
int32_t isg_stat_replicas(void);

#ifdef __cplusplus
}
#endif
#endif
