// C-ABI front of libisg.so: error plumbing, conv dispatch (dense MFMA vs depthwise
// VALU) and the plan executor (include/isg.h).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/isg.h"
#include "residual.h"

static thread_local std::string g_last_error;

int32_t isg_set_error(int32_t code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int32_t isg_check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return isg_set_error(ISG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return ISG_OK;
}

// implemented in conv_mfma.hip / dw_convt.hip
int32_t isg_dense_conv_fwd(const isg_conv_geom*, const isg_vtensor*, const float*, const isg_sinks*,
                           hipStream_t);
int32_t isg_dense_conv_dgrad(const isg_conv_geom*, const isg_vtensor*, const float*, const isg_sinks*,
                             hipStream_t);
int32_t isg_dense_conv_wgrad(const isg_conv_geom*, const isg_vtensor*, const isg_vtensor*, double*,
                             double*, int64_t, int32_t, hipStream_t);
int32_t isg_depthwise_fwd(const isg_conv_geom*, const isg_vtensor*, const float*, const isg_sinks*,
                          hipStream_t);
int32_t isg_depthwise_dgrad(const isg_conv_geom*, const isg_vtensor*, const float*, const isg_sinks*,
                            hipStream_t);
int32_t isg_depthwise_wgrad(const isg_conv_geom*, const isg_vtensor*, const isg_vtensor*, double*,
                            double*, int64_t, int32_t, hipStream_t);

static int32_t check_geom(const isg_conv_geom* g) {
    if (!g) return isg_set_error(ISG_ERR_INVALID, "conv: NULL geometry");
    if (g->N < 1 || g->Ci < 1 || g->Co < 1 || g->H < 1 || g->W < 1 || g->KH < 1 || g->KW < 1 ||
        g->SH < 1 || g->SW < 1 || g->DH < 1 || g->DW < 1 || g->PH < 0 || g->PW < 0)
        return isg_set_error(ISG_ERR_INVALID, "conv: invalid geometry");
    const int oh = (g->H + 2 * g->PH - g->DH * (g->KH - 1) - 1) / g->SH + 1;
    const int ow = (g->W + 2 * g->PW - g->DW * (g->KW - 1) - 1) / g->SW + 1;
    if (oh != g->OH || ow != g->OW)
        return isg_set_error(ISG_ERR_INVALID, "conv: output %dx%d but geometry gives %dx%d", g->OH,
                             g->OW, oh, ow);
    if (g->groups != 1 && !(g->groups == g->Ci && g->Ci == g->Co))
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv: groups=%d (dense or depthwise only)",
                             g->groups);
    if (g->w_ci < 0 || (g->w_ci > 0 && (g->w_ci < g->Ci || g->groups != 1)))
        return isg_set_error(ISG_ERR_INVALID, "conv: weight input channels %d < Ci %d", g->w_ci,
                             g->Ci);
    return ISG_OK;
}

static bool geom_ok(const isg_conv_geom* g) { return check_geom(g) == ISG_OK; }

int32_t isg_tap_conv(const isg_conv_geom*, const isg_vtensor*, const float*, const isg_sinks*,
                     bool, hipStream_t);
int32_t isg_pw_gemm(const isg_conv_geom*, const isg_vtensor*, const float*, const isg_sinks*, bool,
                    hipStream_t);

// the residual forms (isg.h) exist for the 1x1 stride-1 dense conv only
static bool pointwise(const isg_conv_geom* g) {
    return g->KH == 1 && g->KW == 1 && g->SH == 1 && g->SW == 1 && g->PH == 0 && g->PW == 0 &&
           g->DH == 1 && g->DW == 1 && g->groups == 1 && g->w_ci == 0;
}
// segments covering `cin` channels in (forward: one), consecutive sinks covering all `cout`
// rows out (input gradient: one)
static bool res_shape_ok(const isg_vtensor* v, int cin, const isg_sinks* k, int cout, bool dgrad) {
    if (v->nseg < 1 || v->nseg > ISG_MAX_SEGS || k->nsink < 1 || k->nsink > ISG_MAX_SEGS) return false;
    if (dgrad ? k->nsink != 1 : v->nseg != 1) return false;
    int c = 0;
    for (int i = 0; i < v->nseg; ++i) c += v->s[i].C;
    if (c != cin) return false;
    c = 0;
    for (int i = 0; i < k->nsink; ++i) {
        if (k->s[i].c0 != c) return false;
        c += k->s[i].C;
    }
    return c == cout;
}
int32_t isg_s2k5_fwd(const isg_conv_geom*, const isg_vtensor*, const float*, const isg_sinks*,
                     hipStream_t);
int32_t isg_s2k5_wgrad(const isg_conv_geom*, const isg_vtensor*, const isg_vtensor*, double*, double*,
                       int64_t, int32_t, hipStream_t);
int32_t isg_tap_wgrad(const isg_conv_geom*, const isg_vtensor*, const isg_vtensor*, double*, double*,
                      int64_t, int32_t, hipStream_t);

// a conv over the first Ci of the weight's w_ci input channels (the keypoint stem's RGB
// part): only tap_conv / tap_wgrad index the weight with a separate channel count
static bool partial_w(const isg_conv_geom* g) { return g->w_ci > 0 && g->w_ci != g->Ci; }

static isg_vtensor resolve_y(const isg_vtensor* v) { return isg_resolve_y(v); }  // residual.h

extern "C" {

const char* isg_last_error(void) { return g_last_error.c_str(); }
int32_t isg_abi_version(void) { return 11; }
int32_t isg_stat_replicas(void) { return ISG_STAT_REP; }

int32_t isg_conv_fwd(const isg_conv_geom* g, const isg_vtensor* x_, const float* w,
                     const isg_sinks* out, isg_stream_t st) {
    if (int32_t e = check_geom(g)) return e;
    if (!x_ || !out) return isg_set_error(ISG_ERR_INVALID, "conv fwd: NULL tensor");
    if (isg_sinks_res(out)) return isg_set_error(ISG_ERR_UNSUPPORTED, "conv fwd: residual sink form");
    if (isg_vt_res(x_)) {  // a folded residual tail: the slab 1x1 GEMM or nothing
        if (!pointwise(g) || !res_shape_ok(x_, g->Ci, out, g->Co, false))
            return isg_set_error(ISG_ERR_UNSUPPORTED, "conv fwd: residual input needs a 1x1 conv and one segment");
        return isg_pw_gemm(g, x_, w, out, false, st);
    }
    const isg_vtensor xr = resolve_y(x_);
    const isg_vtensor* x = &xr;
    if (partial_w(g)) {
        // the stem's RGB layer 1 (5x5 s2, weight over w_ci = 20 channels): s2k5_fwd_kernel
        const int32_t s = isg_s2k5_fwd(g, x, w, out, st);
        if (s != 0) return s < 0 ? s : ISG_OK;
        const int32_t t = isg_tap_conv(g, x, w, out, false, st);
        if (t < 0) return t;
        return t ? ISG_OK : isg_set_error(ISG_ERR_UNSUPPORTED, "conv fwd: w_ci %d != Ci %d off tap_conv", g->w_ci, g->Ci);
    }
    if (g->groups == 1) return isg_dense_conv_fwd(g, x, w, out, st);
    return isg_depthwise_fwd(g, x, w, out, st);
}

int32_t isg_conv_dgrad(const isg_conv_geom* g, const isg_vtensor* dy_, const float* w,
                       const isg_sinks* dx, isg_stream_t st) {
    if (int32_t e = check_geom(g)) return e;
    if (!dy_ || !dx) return isg_set_error(ISG_ERR_INVALID, "conv dgrad: NULL tensor");
    if (isg_vt_res(dy_)) return isg_set_error(ISG_ERR_UNSUPPORTED, "conv dgrad: residual input form");
    const isg_vtensor dyr = resolve_y(dy_);
    const isg_vtensor* dy = &dyr;
    if (isg_sinks_res(dx)) {  // a folded residual tail's backward: the slab 1x1 GEMM or nothing
        if (!pointwise(g) || !res_shape_ok(dy, g->Co, dx, g->Ci, true))
            return isg_set_error(ISG_ERR_UNSUPPORTED, "conv dgrad: residual sink needs a 1x1 conv and one sink");
        return isg_pw_gemm(g, dy, w, dx, true, st);
    }
    if (partial_w(g)) return isg_set_error(ISG_ERR_UNSUPPORTED, "conv dgrad with w_ci != Ci");
    if (g->groups == 1) return isg_dense_conv_dgrad(g, dy, w, dx, st);
    return isg_depthwise_dgrad(g, dy, w, dx, st);
}

int32_t isg_conv_wgrad_rep(const isg_conv_geom* g, const isg_vtensor* dy_, const isg_vtensor* x_,
                           double* dw, double* dbias, int64_t rep_stride, int32_t nrep,
                           isg_stream_t st) {
    if (int32_t e = check_geom(g)) return e;
    if (isg_vt_res(dy_) || isg_vt_res(x_))
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: residual input form");
    const isg_vtensor dyr = resolve_y(dy_), xr = resolve_y(x_);
    const isg_vtensor *dy = &dyr, *x = &xr;
    if (nrep < 1 || (nrep > 1 && rep_stride <= 0))
        return isg_set_error(ISG_ERR_INVALID, "conv wgrad: bad replicas %d / stride %lld", nrep,
                             (long long)rep_stride);
    if (!dy_ || !x_) return isg_set_error(ISG_ERR_INVALID, "conv wgrad: NULL tensor");
    if (partial_w(g)) {
        // the stem's RGB layer 1 (weight over w_ci = 20 channels): s2k5_wgrad_kernel
        const int32_t s = isg_s2k5_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);
        if (s != 0) return s < 0 ? s : ISG_OK;
        const int32_t t = isg_tap_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);
        if (t < 0) return t;
        return t ? ISG_OK : isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: w_ci %d != Ci %d off tap_wgrad", g->w_ci, g->Ci);
    }
    if (g->groups == 1) return isg_dense_conv_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);
    return isg_depthwise_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);
}

int32_t isg_conv_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                       double* dw, double* dbias, isg_stream_t st) {
    return isg_conv_wgrad_rep(g, dy, x, dw, dbias, 0, 1, st);
}

// ---- plan executor ----------------------------------------------------------------
// Blob layout, per op (all 8-byte aligned):
//   int32 kind, int32 desc_bytes, int32 nfix, int32 pad
//   desc_bytes of the op's argument record (one of the structs below)
//   nfix x { int32 loc, int32 slot, int64 offset }: *(void**)(desc+loc) = table[slot]+offset
enum {
    OP_CONV_FWD = 1,
    OP_CONV_DGRAD = 2,
    OP_CONV_WGRAD = 3,
    OP_CONVT_FWD = 4,
    OP_MAXPOOL_FWD = 5,
    OP_MAXPOOL_BWD = 6,
    OP_TAIL_FWD = 7,
    OP_TAIL_BWD = 8,
    OP_BN_UPDATE = 9,
    OP_GRAD_FINAL = 10,
    OP_BCE = 11,
    OP_MEMSET = 12,
    OP_SUM_REP = 13,
    OP_BN_FINAL = 14,
    OP_KP_STEM_FWD = 15,
    OP_KP_STEM_WGRAD = 16,
    OP_KP_POOL = 17,
    OP_HEAD_FWD = 18,
    OP_HEAD_BWD = 19,
    OP_STAMP = 20,
    OP_DW_BWD = 21,
    OP_STEP_TAIL = 24,
    OP_STEP_INC = 25,
    OP_HEAD_FOLD = 22,
};

struct ConvRec {
    isg_conv_geom g;
    isg_vtensor a;
    const float* w;
    isg_sinks out;
};
struct WgradRec {
    isg_conv_geom g;
    isg_vtensor dy;
    isg_vtensor x;
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int32_t nrep;
    int32_t pad_;
};
struct SumRepRec {
    float* dst;
    const double* src;
    int64_t n;
    int64_t stride;
    int32_t nrep;
    int32_t pad_;
};
struct PoolRec {
    isg_vtensor x;
    int32_t k;
    int32_t pad_;
    float* out;
    int64_t out_ns;
    const float* dout;
    int64_t dout_ns;
    isg_sinks dx;
};
struct ListRec {  // followed in the record by n items (host memory)
    int32_t n;
    int32_t pad_;  // OP_BN_FINAL: 0 forward / 1 backward coefficients
};
struct BceRec {
    const float* logits;
    const float* target;
    int64_t n;
    double* loss;
    float* dlogits;
    float grad_scale;
    int32_t pad_;
};
struct MemsetRec {
    void* p;
    int64_t bytes;
};
struct StepIncRec {  // OP_STEP_INC: isg_step_inc
    int32_t* step;
};
struct DwBwdRec {  // OP_DW_BWD: isg_depthwise_bwd
    isg_conv_geom g;
    isg_vtensor dy;
    const float* w;
    isg_sinks dx;
    isg_vtensor x;
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int32_t nrep, pad_;
};
struct StampRec {  // OP_STAMP: isg_stamp(buf, slot, sign)
    uint64_t* buf;
    int32_t slot;
    int32_t sign;
};

struct OpHdr {
    int32_t kind, desc_bytes, nfix, flags;  // flags: ISG_OPF_SIDE | ISG_OPF_JOIN
};
enum { ISG_OPF_SIDE = 1, ISG_OPF_JOIN = 2, ISG_OPF_FORK_NOW = 4 };  // FORK_NOW: forked at the next main-stream op
// flags >> 8 of a JOIN: how many of the most recent side records (in list order) the op does
// NOT depend on — it waits only for the side work up to the one before them (engine.py
// _join_exclusions); 0 = wait for all side work
constexpr int kJoinExclShift = 8;

// fork / join events of the executor's side streams, per device (created on first use,
// never destroyed; timing disabled): ev[0] fork, ev[1] join of side stream 0, ev[2] join
// of side stream 1
constexpr int kForkPool = 16;  // fork events of side-stream batches, used round robin
constexpr int kDonePool = 64;  // batch-completion events (partial joins), round robin
static int32_t side_events(hipEvent_t* join, hipEvent_t* join2, hipEvent_t** forks, hipEvent_t** done) {
    static hipEvent_t ev[64][2 + kForkPool + 2 * kDonePool];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return isg_set_error(ISG_ERR_HIP, "exec: no device for the side stream");
    if (!ev[dev][0]) {
        for (int i = 0; i < 2 + kForkPool + 2 * kDonePool; ++i)
            if (hipEventCreateWithFlags(&ev[dev][i], hipEventDisableTiming) != hipSuccess)
                return isg_check_launch("exec: side-stream events");
    }
    *join = ev[dev][0];
    *join2 = ev[dev][1];
    *forks = &ev[dev][2];
    *done = &ev[dev][2 + kForkPool];
    return ISG_OK;
}
struct Fix {
    int32_t loc, slot;
    int64_t offset;
};

// wgrad.hip: grouped 1x1 weight gradients (the executor's side-stream batches)
int32_t isg_pwg_plan_bytes();
int32_t isg_pwg_group_max();
int32_t isg_pwg_plan(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                     double* dbias, int64_t rep_stride, int32_t nrep, void* plan);
int32_t isg_pwg_run(const void* const* plans, int32_t n, hipStream_t st);

static int32_t run_op(int32_t kind, char* buf, isg_stream_t st) {
    int32_t rc = 0;
    switch (kind) {
        case OP_CONV_FWD: {
            auto* r = (ConvRec*)buf;
            rc = isg_conv_fwd(&r->g, &r->a, r->w, &r->out, st);
            break;
        }
        case OP_CONV_DGRAD: {
            auto* r = (ConvRec*)buf;
            rc = isg_conv_dgrad(&r->g, &r->a, r->w, &r->out, st);
            break;
        }
        case OP_CONV_WGRAD: {
            auto* r = (WgradRec*)buf;
            rc = isg_conv_wgrad_rep(&r->g, &r->dy, &r->x, r->dw, r->dbias, r->rep_stride,
                                    r->nrep < 1 ? 1 : r->nrep, st);
            break;
        }
        case OP_CONVT_FWD: {
            auto* r = (ConvRec*)buf;
            rc = isg_convT_fwd(&r->g, &r->a, r->w, &r->out, st);
            break;
        }
        case OP_MAXPOOL_FWD: {
            auto* r = (PoolRec*)buf;
            rc = isg_maxpool_fwd(&r->x, r->k, r->out, r->out_ns, st);
            break;
        }
        case OP_MAXPOOL_BWD: {
            auto* r = (PoolRec*)buf;
            rc = isg_maxpool_bwd(&r->x, r->k, r->dout, r->dout_ns, &r->dx, st);
            break;
        }
        case OP_TAIL_FWD:
            rc = isg_tail_fwd((const isg_tail*)buf, st);
            break;
        case OP_TAIL_BWD:
            rc = isg_tail_bwd((const isg_tail_grad*)buf, st);
            break;
        case OP_BN_UPDATE: {
            auto* r = (ListRec*)buf;
            rc = isg_bn_update_running((const isg_bn_update*)(buf + sizeof(ListRec)), r->n, st);
            break;
        }
        case OP_BN_FINAL: {
            auto* r = (ListRec*)buf;
            rc = isg_bn_finalize((const isg_bn*)(buf + sizeof(ListRec)), r->n, r->pad_, st);
            break;
        }
        case OP_GRAD_FINAL: {
            auto* r = (ListRec*)buf;
            rc = isg_grad_finalize((const isg_grad_final*)(buf + sizeof(ListRec)), r->n, st);
            break;
        }
        case OP_BCE: {
            auto* r = (BceRec*)buf;
            rc = isg_bce_sigmoid(r->logits, r->target, r->n, r->loss, r->dlogits, r->grad_scale, st);
            break;
        }
        case OP_SUM_REP: {
            auto* r = (SumRepRec*)buf;
            rc = isg_sum_replicas(r->dst, r->src, r->n, r->nrep, r->stride, st);
            break;
        }
        case OP_KP_STEM_FWD:
            rc = isg_kp_stem_fwd((const isg_kp_stem*)buf, st);
            break;
        case OP_KP_STEM_WGRAD:
            rc = isg_kp_stem_wgrad((const isg_kp_stem*)buf, st);
            break;
        case OP_KP_POOL:
            rc = isg_kp_pool((const isg_kp_stem*)buf, st);
            break;
        case OP_HEAD_FWD:
            rc = isg_mask_head_fwd((const isg_mask_head*)buf, st);
            break;
        case OP_HEAD_BWD:
            rc = isg_mask_head_bwd((const isg_mask_head*)buf, st);
            break;
        case OP_HEAD_FOLD:
            rc = isg_mask_head_fold((const isg_mask_head*)buf, st);
            break;
        case OP_DW_BWD: {
            auto* r = (DwBwdRec*)buf;
            rc = isg_depthwise_bwd(&r->g, &r->dy, r->w, &r->dx, &r->x, r->dw, r->dbias, r->rep_stride,
                                   r->nrep, st);
            break;
        }
        case OP_STAMP: {
            auto* r = (StampRec*)buf;
            rc = isg_stamp(r->buf, r->slot, r->sign, st);
            break;
        }
        case OP_STEP_TAIL:
            rc = isg_step_tail((const isg_step_tail_args*)buf, st);
            break;
        case OP_STEP_INC: {
            auto* r = (StepIncRec*)buf;
            rc = isg_step_inc(r->step, st);
            break;
        }
        case OP_MEMSET: {
            auto* r = (MemsetRec*)buf;
            if (hipMemsetAsync(r->p, 0, (size_t)r->bytes, st) != hipSuccess)
                rc = isg_check_launch("memset");
            break;
        }
        default:
            return isg_set_error(ISG_ERR_INVALID, "exec: unknown op kind %d", kind);
    }
    return rc;
}

int32_t isg_exec_ms2(const void* ops, int32_t nops, void* const* table, isg_stream_t main_st,
                     isg_stream_t side, isg_stream_t side2) {
    const char* p = (const char*)ops;
    alignas(16) char buf[8192];
    hipEvent_t ev_join = nullptr, ev_join2 = nullptr, *ev_forks = nullptr, *ev_done = nullptr;
    bool forked = false, forked2 = false;  // side-stream work outstanding since the last join
    // weight gradients deferred per fork. Round 6 (eager issue, fused step tail,
    // profiles/r08e_ab_side_batch.txt): 16 -> 3.385 ms/step, 8: 3.377, 24: 3.407, 48: 3.67 —
    // a batch of 48 held the first weight gradients until deep into the backward and then
    // flooded the chain's kernels (round 3 had measured 48 best: 4.365 vs 4.415 at 24)
    constexpr int batch = 16;
    // grouped 1x1 weight gradients in weight-gradient batches (4.04 -> 3.96
    // ms/step, 2 interleaved 200-step pairs)
    constexpr bool pwg_group_on = true;
    struct Batch {
        std::vector<std::pair<int32_t, std::string>> ops;
        hipEvent_t ev;
    };
    std::vector<std::pair<int32_t, std::string>> pending;
    int pool_next = 0;
    // partial joins: for every issued batch, the side-record count after it and the events
    // recorded behind it on the side stream(s) it used
    struct Done {
        int upto;
        hipEvent_t e1, e2;
    };
    std::vector<Done> done_list;
    int done_next = 0;
    int nside = 0;  // side records seen so far (list order)
    int issued = 0;  // side records issued so far
    int deal = 0;  // weight gradients alternate between the side streams across batches too
    bool side_serial = false;  // a side-only batch ran on `side` since side 2 last waited for it
    auto launch = [&](Batch& bt) -> int32_t {
        // a batch of weight gradients only (independent accumulations into the replica
        // buffers) is dealt over both side streams: their grids (128-512 workgroups) leave
        // most of the chip idle one at a time; anything else keeps its order on stream 0
        // (the step counter too: it touches nothing else — as a non-spread batch at the head
        // of the backward it had kept every later batch off side 2, round 6)
        bool spread = side2 != nullptr;
        for (auto& op : bt.ops)
            spread = spread && (op.first == OP_CONV_WGRAD || op.first == OP_KP_STEM_WGRAD ||
                                op.first == OP_HEAD_FOLD || op.first == OP_GRAD_FINAL ||
                                op.first == OP_BN_UPDATE || op.first == OP_STEP_INC);
        // a batch behind a side-only one (the gradient finalisation lists behind the replica
        // fold at ISG_SIDE_CLOSE=1) may read what that one writes: it stays on `side`, in order
        if (spread && side_serial) spread = false;
        if (hipStreamWaitEvent(side, bt.ev, 0) != hipSuccess ||
            (spread && hipStreamWaitEvent(side2, bt.ev, 0) != hipSuccess))
            return isg_check_launch("exec: fork side stream");
        if (!spread && forked2) {
            // a non-weight-gradient batch (e.g. the replica fold / gradient finalisation at
            // ISG_SIDE_CLOSE=1) runs on `side` only: order it after side2's outstanding
            // weight-gradient accumulations, which it may read
            forked2 = false;
            if (hipEventRecord(ev_join2, side2) != hipSuccess || hipStreamWaitEvent(side, ev_join2, 0) != hipSuccess)
                return isg_check_launch("exec: order side stream after side stream 2");
        }
        side_serial = side_serial || (!spread && side2 != nullptr);
        forked = true;
        forked2 = forked2 || spread;
        alignas(16) char pb[8192];
        // consecutive one-op batches (the stem's weight gradients, forked one by one behind
        // its input-gradient chain) land on different side streams and overlap
        auto next_st = [&]() { return spread && (deal++ & 1) ? side2 : side; };
        bool all_wgrad = true;
        for (auto& op : bt.ops)
            all_wgrad = all_wgrad && (op.first == OP_CONV_WGRAD || op.first == OP_KP_STEM_WGRAD ||
                                      op.first == OP_HEAD_FOLD);
        if (!pwg_group_on || !all_wgrad) {
            for (auto& op : bt.ops) {
                std::memcpy(pb, op.second.data(), op.second.size());
                if (int32_t e = run_op(op.first, pb, next_st())) return e;
            }
            return ISG_OK;
        }
        // a batch of weight gradients only (independent accumulations): the 1x1 ones that
        // would run on pwg_kernel go out grouped, up to isg_pwg_group_max() per launch of
        // one instantiation (wgrad.hip pwg_group_kernel); each group at its first member
        const size_t n = bt.ops.size();
        const int gmax = isg_pwg_group_max();
        std::vector<std::vector<char>> plans(n);
        std::vector<int> key(n, 0);
        for (size_t i = 0; i < n; ++i) {
            if (bt.ops[i].first != OP_CONV_WGRAD) continue;
            std::memcpy(pb, bt.ops[i].second.data(), bt.ops[i].second.size());
            auto* r = (WgradRec*)pb;
            if (!geom_ok(&r->g)) continue;
            plans[i].resize((size_t)isg_pwg_plan_bytes());
            key[i] = isg_pwg_plan(&r->g, &r->dy, &r->x, r->dw, r->dbias, r->rep_stride,
                                  r->nrep < 1 ? 1 : r->nrep, plans[i].data());
        }
        std::vector<char> done(n, 0);
        for (size_t i = 0; i < n; ++i) {
            if (done[i]) continue;
            if (key[i] > 0) {
                const void* grp[8];
                int m = 0;
                for (size_t j = i; j < n && m < gmax && m < 8; ++j)
                    if (!done[j] && key[j] == key[i]) {
                        grp[m++] = plans[j].data();
                        done[j] = 1;
                    }
                if (int32_t e = isg_pwg_run(grp, m, next_st())) return e;
                continue;
            }
            std::memcpy(pb, bt.ops[i].second.data(), bt.ops[i].second.size());
            if (int32_t e = run_op(bt.ops[i].first, pb, next_st())) return e;
        }
        return ISG_OK;
    };
    auto close_batch = [&]() -> int32_t {  // the pending batch forks here and is issued
        if (pending.empty()) return ISG_OK;
        Batch bt;
        bt.ops.swap(pending);
        bt.ev = ev_forks[pool_next++ % kForkPool];
        if (hipEventRecord(bt.ev, main_st) != hipSuccess) return isg_check_launch("exec: fork point");
        if (int32_t e = launch(bt)) return e;
        issued += (int)bt.ops.size();
        // its completion on the side stream(s) holding outstanding work, for a later partial
        // join (side 2 behind this batch covers it too when the batch did not use side 2)
        Done d{issued, ev_done[2 * (done_next % kDonePool)], nullptr};
        if (hipEventRecord(d.e1, side) != hipSuccess) return isg_check_launch("exec: batch done");
        if (forked2) {
            d.e2 = ev_done[2 * (done_next % kDonePool) + 1];
            if (hipEventRecord(d.e2, side2) != hipSuccess) return isg_check_launch("exec: batch done 2");
        }
        ++done_next;
        done_list.push_back(d);
        return ISG_OK;
    };
    // wait for the side work up to side record `upto` (exclusive count) only
    auto join_upto = [&](int upto) -> int32_t {
        if (upto > issued)
            if (int32_t e = close_batch()) return e;
        for (const Done& d : done_list) {
            if (d.upto < upto) continue;
            if (hipStreamWaitEvent(main_st, d.e1, 0) != hipSuccess ||
                (d.e2 && hipStreamWaitEvent(main_st, d.e2, 0) != hipSuccess))
                return isg_check_launch("exec: partial join");
            return ISG_OK;
        }
        return ISG_OK;  // (nothing issued up to there: no side work to wait for)
    };
    auto join = [&]() -> int32_t {
        if (int32_t e = close_batch()) return e;
        side_serial = false;  // later forks start from the main stream, which waits for both
        if (forked) {
            forked = false;
            if (hipEventRecord(ev_join, side) != hipSuccess || hipStreamWaitEvent(main_st, ev_join, 0) != hipSuccess)
                return isg_check_launch("exec: join side stream");
        }
        if (forked2) {
            forked2 = false;
            if (hipEventRecord(ev_join2, side2) != hipSuccess || hipStreamWaitEvent(main_st, ev_join2, 0) != hipSuccess)
                return isg_check_launch("exec: join side stream 2");
        }
        return ISG_OK;
    };
    // a FORK_NOW record's batch is issued when the next main-stream record (or a join, or
    // the end) comes: consecutive forked records share one fork event on the main stream
    // (each event record there cost the main queue ~6 us of idle, round-6 kernel trace;
    // interleaved A/B 3.212-3.221 vs 3.231-3.245 ms/step)
    bool fork_due = false;
    for (int i = 0; i < nops; ++i) {
        OpHdr h;
        std::memcpy(&h, p, sizeof(h));
        isg_stream_t st = main_st;
        if (fork_due && !((h.flags & ISG_OPF_SIDE) && side)) {
            fork_due = false;
            if (int32_t e = close_batch()) return e;
        }
        if ((h.flags & ISG_OPF_JOIN) && side) {
            const int excl = h.flags >> kJoinExclShift;
            if (excl > 0 && excl <= nside) {
                if (int32_t e = join_upto(nside - excl)) return e;
            } else if (int32_t e = join()) {
                return e;
            }
        }
        if ((h.flags & ISG_OPF_SIDE) && side) {
            // the op depends on everything issued so far on the main stream
            if (!ev_join) {
                if (int32_t e = side_events(&ev_join, &ev_join2, &ev_forks, &ev_done)) return e;
            }
            st = side;
            ++nside;
        }
        p += sizeof(h);
        if (h.desc_bytes < 0 || h.desc_bytes > (int)sizeof(buf))
            return isg_set_error(ISG_ERR_INVALID, "exec: op %d bad desc size %d", i, h.desc_bytes);
        std::memcpy(buf, p, h.desc_bytes);
        p += (h.desc_bytes + 7) & ~7;
        for (int f = 0; f < h.nfix; ++f) {
            Fix fx;
            std::memcpy(&fx, p, sizeof(fx));
            p += sizeof(fx);
            char* base = fx.slot >= 0 ? (char*)table[fx.slot] : nullptr;
            void* v = base ? base + fx.offset : nullptr;
            std::memcpy(buf + fx.loc, &v, sizeof(v));
        }
        int32_t rc = 0;
        if (side && st == side) {
            // deferred: launched in batches behind one fork (a later fork only adds
            // dependencies, so batching is always safe)
            pending.emplace_back(h.kind, std::string(buf, buf + h.desc_bytes));
            if ((int)pending.size() >= batch) {
                fork_due = false;
                rc = close_batch();
            } else if (h.flags & ISG_OPF_FORK_NOW) {
                fork_due = true;
            }
        } else {
            rc = run_op(h.kind, buf, st);
        }
        if (rc) {
            std::string m = g_last_error;
            return isg_set_error(rc, "exec op %d (kind %d): %s", i, h.kind, m.c_str());
        }
    }
    return join();
}

int32_t isg_exec_ms(const void* ops, int32_t nops, void* const* table, isg_stream_t main_st,
                    isg_stream_t side) {
    return isg_exec_ms2(ops, nops, table, main_st, side, nullptr);
}

int32_t isg_exec(const void* ops, int32_t nops, void* const* table, isg_stream_t st) {
    return isg_exec_ms2(ops, nops, table, st, nullptr, nullptr);
}

// sizes of the executor records, so the Python planner can verify its ctypes mirrors
int32_t isg_record_size(int32_t which) {
    switch (which) {
        case 0: return (int32_t)sizeof(isg_vtensor);
        case 1: return (int32_t)sizeof(isg_sinks);
        case 2: return (int32_t)sizeof(ConvRec);
        case 3: return (int32_t)sizeof(WgradRec);
        case 4: return (int32_t)sizeof(PoolRec);
        case 5: return (int32_t)sizeof(isg_tail);
        case 6: return (int32_t)sizeof(isg_tail_grad);
        case 7: return (int32_t)sizeof(isg_bn_update);
        case 8: return (int32_t)sizeof(isg_grad_final);
        case 9: return (int32_t)sizeof(BceRec);
        case 10: return (int32_t)sizeof(isg_conv_geom);
        case 11: return (int32_t)sizeof(isg_bn);
        case 12: return (int32_t)sizeof(isg_vseg);
        case 13: return (int32_t)sizeof(isg_sink);
        case 14: return (int32_t)sizeof(SumRepRec);
        case 15: return (int32_t)sizeof(isg_kp_stem);
        case 16: return (int32_t)sizeof(isg_mask_head);
        case 17: return (int32_t)sizeof(StampRec);
        case 18: return (int32_t)sizeof(DwBwdRec);
        case 19: return (int32_t)sizeof(isg_step_tail_args);
        default: return -1;
    }
}

}  // extern "C"
