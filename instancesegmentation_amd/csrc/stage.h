// Staging helpers: virtual-tensor channels addressed with WAVE-UNIFORM channel indices.
//
// A kernel that maps lanes to pixels and waves to (channel, row) slots keeps every
// per-channel quantity — segment, base pointer, image stride, BatchNorm coefficients,
// activation — in scalar registers: the per-element work is one address add, one global
// load and one fused transform. (Mapping lanes to channels instead costs an LDS table
// read, 64-bit address arithmetic and selects per element, which made the first staging
// loops instruction-bound at ~10 us per 64-pixel tile.)
#pragma once
#include "common.h"

// One channel of a vtensor (c must be wave-uniform so this stays in SGPRs).
struct ChSrc {
    const float* p;  // channel base, image 0
    const float* y;  // BN_BWD: saved forward output; BN_FWD: residual term (else == p)
    int ns, yns;     // elements between images
    int xf, act;
};

// The addressing fields of a vtensor's segments, read once with constant indices into
// plain registers. Selecting between fields of the kernel-argument struct directly lets
// the compiler turn "select of loads" into "load of a selected address", which forces a
// copy of the whole argument struct to scratch.
struct VtLite {
    const float *p0, *p1, *p2, *y0, *y1, *y2;
    int ns0, ns1, ns2, yns0, yns1, yns2, xf0, xf1, xf2, act0, act1, act2;
    int c1, c2;
};

ISG_DEV VtLite vt_lite(const isg_vtensor& vt) {
    VtLite l;
    l.p0 = vt.s[0].p; l.p1 = vt.s[1].p; l.p2 = vt.s[2].p;
    l.y0 = vt.s[0].y; l.y1 = vt.s[1].y; l.y2 = vt.s[2].y;
    l.ns0 = (int)vt.s[0].n_stride; l.ns1 = (int)vt.s[1].n_stride; l.ns2 = (int)vt.s[2].n_stride;
    l.yns0 = (int)vt.s[0].y_n_stride; l.yns1 = (int)vt.s[1].y_n_stride;
    l.yns2 = (int)vt.s[2].y_n_stride;
    l.xf0 = vt.s[0].xform; l.xf1 = vt.s[1].xform; l.xf2 = vt.s[2].xform;
    l.act0 = vt.s[0].act; l.act1 = vt.s[1].act; l.act2 = vt.s[2].act;
    l.c1 = vt.nseg > 1 ? vt.s[0].C : 1 << 30;
    l.c2 = vt.nseg > 2 ? vt.s[0].C + vt.s[1].C : 1 << 30;
    return l;
}

ISG_DEV ChSrc ch_src(const VtLite& l, int c, int hw) {
    ChSrc r;
    const float* y;
    int cl;
    if (c >= l.c2) {
        r.p = l.p2; y = l.y2; r.ns = l.ns2; r.yns = l.yns2; r.xf = l.xf2; r.act = l.act2;
        cl = c - l.c2;
    } else if (c >= l.c1) {
        r.p = l.p1; y = l.y1; r.ns = l.ns1; r.yns = l.yns1; r.xf = l.xf1; r.act = l.act1;
        cl = c - l.c1;
    } else {
        r.p = l.p0; y = l.y0; r.ns = l.ns0; r.yns = l.yns0; r.xf = l.xf0; r.act = l.act0;
        cl = c;
    }
    r.p += (int64_t)cl * hw;
    // no separate y: y is the input itself, with the input's image stride
    const bool hy = (r.xf == ISG_XF_BN_BWD || r.xf == ISG_XF_BN_FWD) && y;
    r.y = hy ? y + (int64_t)cl * hw : r.p;
    r.yns = hy ? r.yns : r.ns;
    return r;
}

// fp64 evaluation from the statistics (eval mode, or direct ABI calls without
// isg_bn.coef): out of line so its code exists once; bn passed by value (registers),
// a reference to the kernel argument would copy the whole argument struct to scratch.
__device__ __noinline__ ChanCoef coef_slow(isg_bn bn, const float* slope, int cl, int bwd) {
    return bwd ? bwd_coef(bn, cl) : fwd_coef(bn, slope, cl);
}

// Coefficients of channel cl of one segment.
ISG_DEV ChanCoef seg_coefs(const isg_vseg& sg, int cl) {
    ChanCoef k = {0.f, 1.f, 0.f, 0.f};
    if (sg.xform == ISG_XF_BN_FWD) {
        if (sg.bn.coef) {
            const f32x4 f = reinterpret_cast<const f32x4*>(sg.bn.coef)[cl];
            k = ChanCoef{f[0], f[1], f[2], sg.slope ? sg.slope[cl] : 0.f};
        } else if (sg.bn.stats || !sg.bn.train) {
            k = coef_slow(sg.bn, sg.slope, cl, 0);
        } else {
            k.c3 = sg.slope ? sg.slope[cl] : 0.f;  // activation only
        }
    } else if (sg.xform == ISG_XF_BN_BWD) {
        if (sg.bn.coef) {
            const f32x4 f = reinterpret_cast<const f32x4*>(sg.bn.coef)[sg.bn.C + cl];
            k = ChanCoef{f[0], f[1], f[2], f[3]};
        } else {
            k = coef_slow(sg.bn, nullptr, cl, 1);
        }
    }
    return k;
}

// Coefficients of channel c of a vtensor (common.h ChanCoef conventions). Segments are
// addressed with constant indices only: a runtime index into the kernel-argument struct
// makes hipcc copy the whole struct to scratch.
ISG_DEV ChanCoef vt_coef(const isg_vtensor& vt, int c) {
    const int c1 = vt.s[0].C, c2 = c1 + vt.s[1].C;
    if (vt.nseg > 2 && c >= c2) return seg_coefs(vt.s[2], c - c2);
    if (vt.nseg > 1 && c >= c1) return seg_coefs(vt.s[1], c - c1);
    return seg_coefs(vt.s[0], c);
}

// Per-channel staging record kept in LDS (built once per block by one thread per
// channel): a wave-uniform channel index reads it with one broadcast LDS access.
struct ChT {
    const float* p;  // channel base, image 0
    const float* y;  // BN_BWD saved forward output (else == p)
    int ns, yns;
    int xf, act;
    ChanCoef k;
};

ISG_DEV ChT ch_table_entry(const isg_vtensor& vt, int c, int hw) {
    const ChSrc s = ch_src(vt_lite(vt), c, hw);
    ChT t;
    t.p = s.p; t.y = s.y; t.ns = s.ns; t.yns = s.yns; t.xf = s.xf; t.act = s.act;
    t.k = vt_coef(vt, c);
    return t;
}

// v = transform of raw x (and saved y for BN_BWD); xf/act uniform -> scalar branches
ISG_DEV float ch_xform(int xf, int act, const ChanCoef& k, float x, float y) {
    if (xf == ISG_XF_PLAIN) return x;
    if (xf == ISG_XF_BN_FWD) return apply_act((x - k.c0) * k.c1 + k.c2, act, k.c3);
    return k.c0 * x + k.c1 * (y - k.c2) + k.c3;
}

// ch_xform for a PER-LANE channel, branch-free: staging loops whose items span channels
// within a wave otherwise turn every transform into a divergent branch tree (measured on
// the stem layer-2 weight gradient: 786 branches, 14 us of staging per tile). The record
// folds the three forms into one straight-line evaluation with identical arithmetic:
// PLAIN (k = 0, 1, 0, neg 1), BN_FWD + activation (z > 0 ? z : z * neg; ReLU neg 0,
// PReLU neg = slope, none 1), BN_BWD (isb).
struct XfLin {
    ChanCoef k;
    float neg, isb;
};

ISG_DEV XfLin xf_lin(int xf, int act, const ChanCoef& k) {
    XfLin r;
    r.k = xf == ISG_XF_PLAIN ? ChanCoef{0.f, 1.f, 0.f, 0.f} : k;
    r.neg = (xf != ISG_XF_BN_FWD || act == ISG_ACT_NONE) ? 1.f : act == ISG_ACT_RELU ? 0.f : k.c3;
    r.isb = xf == ISG_XF_BN_BWD ? 1.f : 0.f;
    return r;
}

ISG_DEV float xf_lin_apply(const XfLin& l, float x, float y) {
    float zf = (x - l.k.c0) * l.k.c1 + l.k.c2;
    zf = zf > 0.f ? zf : zf * l.neg;
    const float zb = l.k.c0 * x + l.k.c1 * (y - l.k.c2) + l.k.c3;
    return l.isb != 0.f ? zb : zf;
}

// the same with a BN_FWD channel's residual term y added before the activation when
// isr = 1 (isg_vseg residual form; a block tail's BN(y3) + x, then PReLU): the tail's own
// order of operations, (BN value) + residual
ISG_DEV float xf_lin_apply_r(const XfLin& l, float x, float y, float isr) {
    float zf = (x - l.k.c0) * l.k.c1 + l.k.c2;
    zf = zf + isr * y;
    zf = zf > 0.f ? zf : zf * l.neg;
    const float zb = l.k.c0 * x + l.k.c1 * (y - l.k.c2) + l.k.c3;
    return l.isb != 0.f ? zb : zf;
}

// ch_xform for a WAVE-UNIFORM channel: the transform kind moves to SGPRs, so the
// per-element selection is a scalar branch (a VGPR kind branches per element with exec
// masking). Only for callers whose channel is the same in every lane of the wave.
ISG_DEV float ch_xform_u(int xf, int act, const ChanCoef& k, float x, float y) {
    return ch_xform(__builtin_amdgcn_readfirstlane(xf), __builtin_amdgcn_readfirstlane(act), k, x, y);
}

ISG_DEV int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// A wave-uniform pointer moved into SGPRs (each 32-bit half through readfirstlane), so
// loads off it use the scalar-base + 32-bit vector-offset addressing form.
template <class T>
ISG_DEV T* uniform_ptr(T* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// An opaque copy of v: the compiler must recompute whatever depends on it (stops it from
// hoisting per-item address arithmetic out of a loop into dozens of live registers).
ISG_DEV int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// sum over the 16 lanes of a DPP row (lanes sharing l>>4), result in every lane
ISG_DEV float dpp_row16_sum(float v) {
    int x = __builtin_bit_cast(int, v);
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
    x = __builtin_bit_cast(int, v);
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
    x = __builtin_bit_cast(int, v);
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));
    x = __builtin_bit_cast(int, v);
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false));
    return v;
}

// Per-output-row sink record kept in LDS (one per GEMM row = output channel), resolved
// once per workgroup: the epilogue reads it with a broadcast LDS access.
struct SinkRow {
    float* p;        // channel base, image 0
    const float* y;  // ACTBWD: saved forward output
    int64_t ns, yns;
    int mode, act;   // mode -1: row past M
    float bias;
    int pad_;
    SinkCoef f;
};

// one sink's row record
ISG_DEV SinkRow sink_row1(const isg_sink& k, int m, int64_t hw) {
    SinkRow q = {};
    const int cl = m - k.c0;
    q.p = k.p ? k.p + (int64_t)cl * hw : nullptr;
    q.y = k.y ? k.y + (int64_t)cl * hw : nullptr;
    q.ns = k.n_stride;
    q.yns = k.y_n_stride;
    q.mode = k.mode;
    q.act = k.act;
    q.bias = k.bias ? k.bias[cl] : 0.f;
    q.f = SinkCoef{0.f, 1.f, 0.f, 0.f};
    if (k.mode == ISG_SINK_ACTBWD) {
        if (k.bn.stats || !k.bn.train) {
            const ChanCoef f = k.bn.coef ? fwd_coef(k.bn, nullptr, cl) : coef_slow(k.bn, nullptr, cl, 0);
            q.f.mean = f.c0; q.f.scale = f.c1; q.f.beta = f.c2;
        }
        q.f.slope = k.slope ? k.slope[cl] : 0.f;
    }
    return q;
}
// Row m's record. (Round 6, measured: choosing the sink first and reading it at a constant
// index in per-sink branches made the stem's layer-2 forward 37.6 -> 64.1 us — the branches
// around loads in the prologue drained every load in flight; the per-lane struct select
// below keeps the prologue one round trip.)
ISG_DEV SinkRow sink_row(const isg_sinks& sk, int m, int64_t hw) {
    const int s = sink_of(sk, m);
    return sink_row1(s == 2 ? sk.s[2] : (s == 1 ? sk.s[1] : sk.s[0]), m, hw);
}

// Apply row q's sink to value v at flat offset (n, pix); returns the values to reduce
// (STORE/ACCUM: v, v^2; ACTBWD: g, g*(y-mean), PReLU slope contribution).
ISG_DEV void sink_row_apply(const SinkRow& q, int n, int64_t pix, float v, float& s0, float& s1,
                            float& s2) {
    const int64_t off = (int64_t)n * q.ns + pix;
    if (q.mode == ISG_SINK_STORE) {
        v += q.bias;
        gst(q.p, off, v);
        s0 = v;
        s1 = v * v;
    } else if (q.mode == ISG_SINK_ACCUM) {
        gst(q.p, off, gld(q.p, off) + v);
        s0 = v;
        s1 = v * v;
    } else if (q.mode == ISG_SINK_ACTBWD) {
        const float y = gld(q.y, (int64_t)n * q.yns + pix);
        const float z = (y - q.f.mean) * q.f.scale + q.f.beta;
        float gv = v;
        if (q.act == ISG_ACT_RELU) {
            gv = z > 0.f ? v : 0.f;
        } else if (q.act == ISG_ACT_PRELU) {
            gv = z > 0.f ? v : v * q.f.slope;
            s2 = z > 0.f ? 0.f : z * v;
        }
        gst(q.p, off, gv);
        s0 = gv;
        s1 = gv * (y - q.f.mean);
    }
}

// ---- branch-free table construction ----------------------------------------------------
// With finalised BatchNorm coefficients (isg_bn.coef, written by the per-layer
// finalisation) every per-channel record is a few plain loads. The *_issue helpers issue
// them with no control flow (a NULL pointer is replaced by an always-valid one and the
// value discarded in *_finish), so a kernel can put them in flight together with its
// weight and activation loads: any branch around a load makes the compiler drain the
// whole memory queue (s_waitcnt vmcnt(0)) at the join, which serialised the first slab
// kernels into one HBM round trip per load.
// "fast" = every record comes from plain branch-free loads: finalised coefficients, or
// (training mode) the statistics replicas evaluated in coef_finish / sink_finish
// (consumer-side finalisation). Eval mode (running statistics) takes the slow path.
ISG_DEV bool seg_fast(const isg_vseg& s) {
    if (s.xform == ISG_XF_BN_FWD || s.xform == ISG_XF_BN_BWD) return s.bn.coef || s.bn.train;
    return true;
}
ISG_DEV bool vt_fast(const isg_vtensor& v) {
    bool ok = seg_fast(v.s[0]);
    if (v.nseg > 1) ok = ok && seg_fast(v.s[1]);
    if (v.nseg > 2) ok = ok && seg_fast(v.s[2]);
    return ok;
}
ISG_DEV bool sink_fast(const isg_sink& k) {
    return k.mode != ISG_SINK_ACTBWD || k.bn.coef || k.bn.train;
}
ISG_DEV bool sinks_fast(const isg_sinks& sk) {
    bool ok = sink_fast(sk.s[0]);
    if (sk.nsink > 1) ok = ok && sink_fast(sk.s[1]);
    if (sk.nsink > 2) ok = ok && sink_fast(sk.s[2]);
    return ok;
}

// Per-lane segment selection must not select between kernel-argument fields directly:
// hipcc turns "select of two kernarg loads" into "load of a selected kernarg address",
// i.e. a per-lane global load (and a wait) for every field. The fields are first made
// opaque scalars (readfirstlane), then selected with v_cndmask.
ISG_DEV int sgpr_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <class T>
ISG_DEV T* sgpr_p(T* p) { return uniform_ptr(p); }

ISG_DEV float sgpr_f(float v) { return __builtin_bit_cast(float, sgpr_i(__builtin_bit_cast(int, v))); }

struct SegLite {
    const float *p, *y, *coef, *slope, *gamma, *beta;
    const double* stats;
    int ns, yns, xf, act, bnC, C;
    float count, eps;
};
ISG_DEV SegLite seg_lite(const isg_vseg& g) {
    SegLite l;
    l.p = sgpr_p(g.p); l.y = sgpr_p(g.y); l.coef = sgpr_p((const float*)g.bn.coef);
    l.slope = sgpr_p(g.slope);
    l.gamma = sgpr_p(g.bn.gamma); l.beta = sgpr_p(g.bn.beta);
    l.stats = sgpr_p((const double*)g.bn.stats);
    l.ns = sgpr_i((int)g.n_stride); l.yns = sgpr_i((int)g.y_n_stride);
    l.xf = sgpr_i(g.xform); l.act = sgpr_i(g.act); l.bnC = sgpr_i(g.bn.C); l.C = sgpr_i(g.C);
    l.count = sgpr_f(g.bn.count); l.eps = sgpr_f(g.bn.eps);
    return l;
}

// Consumer-side BatchNorm finalisation in the caller's load round trip: the ISG_STAT_REP
// replicas of NG statistics groups of one channel (NG = 2: sum, sum^2; NG = 4: + gsum,
// gxsum for BatchNorm backward) plus gamma / beta, issued branch-free — a NULL `stats`
// (finalised coefficients present, or no BatchNorm) reads a valid dummy address instead
// and stat_finish never looks at the values.
template <int NG>
struct StatLoad {
    double v[NG][ISG_STAT_REP];
    float gamma, beta;
};
template <int NG>
ISG_DEV StatLoad<NG> stat_issue(const double* stats, const float* gamma, const float* beta,
                                int bnC, int cl, const float* any, bool issue = true) {
    StatLoad<NG> r;
    if (!issue) {  // lane-invariant: no channel of the launch needs its statistics
        r.gamma = r.beta = 0.f;
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int q = 0; q < ISG_STAT_REP; ++q) r.v[g][q] = 0.0;
        return r;
    }
    const bool on = stats != nullptr;
    const double* sp = on ? stats : reinterpret_cast<const double*>(any);
    // address = base + q * sq + g * sg: with `on` folded into the strides (not a select per
    // load) the compiler keeps one load per slot instead of branching into a single shared
    // load and copying it, whose join waited out every load in flight (vmcnt(0))
    int sq = on ? 4 * bnC : 0, sg = on ? bnC : 0, s0 = on ? cl : 0;
    asm volatile("" : "+v"(sq), "+v"(sg), "+v"(s0));
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int q = 0; q < ISG_STAT_REP; ++q)
            r.v[g][q] = gld_d(sp, (int64_t)q * sq + (int64_t)g * sg + s0);
    r.gamma = gld(gamma && on ? gamma + cl : any, 0);
    r.beta = gld(beta && on ? beta + cl : any, 0);
    return r;
}
template <int NG>
ISG_DEV double stat_sum(const StatLoad<NG>& r, int g) {  // rep_sum's order
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < ISG_STAT_REP; ++q) s += r.v[g][q];
    return s;
}
struct VtSel {
    SegLite s0, s1, s2;
    int nseg;
};
ISG_DEV VtSel vt_sel(const isg_vtensor& vt) {
    VtSel v;
    v.nseg = sgpr_i(vt.nseg);
    v.s0 = seg_lite(vt.s[0]);
    v.s1 = seg_lite(vt.s[1]);
    v.s2 = seg_lite(vt.s[2]);
    return v;
}
#define ISG_SEL3(s, f, v) ((s) == 2 ? (v).s2.f : ((s) == 1 ? (v).s1.f : (v).s0.f))

template <int NG = 4>
struct CoefLoad {
    f32x4 f;
    float sl;
    StatLoad<NG> st;
};

ISG_DEV int vt_seg(const VtSel vt, int c, int& cl) {
    const int c1 = vt.nseg > 1 ? vt.s0.C : 1 << 30;
    const int c2 = vt.nseg > 2 ? vt.s0.C + vt.s1.C : 1 << 30;
    const int s = c >= c2 ? 2 : (c >= c1 ? 1 : 0);
    cl = c - (s == 2 ? c2 : (s == 1 ? c1 : 0));
    return s;
}

// NG: statistics groups to load for consumer-side finalisation — 2 when no segment is
// BN_BWD, 4 otherwise (a BN_FWD channel then loads its 2 groups twice)
template <int NG = 4>
ISG_DEV CoefLoad<NG> coef_issue(const VtSel vt, int c, bool stat_on = true) {
    int cl;
    const int s = vt_seg(vt, c, cl);
    const float* coef = ISG_SEL3(s, coef, vt);
    const float* slope = ISG_SEL3(s, slope, vt);
    const float* p = ISG_SEL3(s, p, vt);
    const int xf = ISG_SEL3(s, xf, vt);
    const int bnC = ISG_SEL3(s, bnC, vt);
    const int idx = xf == ISG_XF_BN_BWD ? bnC + cl : cl;
    const float* cp = coef ? coef + 4 * (int64_t)idx : p;
    const float* sp = slope ? slope + cl : p;
    const bool bn = xf == ISG_XF_BN_FWD || xf == ISG_XF_BN_BWD;
    const double* st = bn && !coef ? ISG_SEL3(s, stats, vt) : nullptr;
    CoefLoad<NG> r;
    r.f = f32x4{gld(cp, 0), gld(cp, 1), gld(cp, 2), gld(cp, 3)};
    r.sl = gld(sp, 0);
    r.st = stat_issue<NG>(st, ISG_SEL3(s, gamma, vt), ISG_SEL3(s, beta, vt), bnC, cl, p, stat_on);
    return r;
}

template <int NG = 4>
ISG_DEV ChanCoef coef_finish(const VtSel vt, int c, const CoefLoad<NG>& r) {
    int cl;
    const int s = vt_seg(vt, c, cl);
    const bool has_coef = ISG_SEL3(s, coef, vt) != nullptr;
    const bool has_stats = ISG_SEL3(s, stats, vt) != nullptr;
    const bool has_slope = ISG_SEL3(s, slope, vt) != nullptr;
    const int xf = ISG_SEL3(s, xf, vt);
    ChanCoef k = {0.f, 1.f, 0.f, 0.f};
    if (xf == ISG_XF_BN_FWD) {
        if (has_coef) {
            k.c0 = r.f[0]; k.c1 = r.f[1]; k.c2 = r.f[2];
        } else if (has_stats) {  // training mode, consumer-side finalisation
            double mean, rstd;
            mean_rstd_of(stat_sum(r.st, 0), stat_sum(r.st, 1), ISG_SEL3(s, count, vt),
                         ISG_SEL3(s, eps, vt), mean, rstd);
            k = fwd_coef_of(mean, rstd, r.st.gamma, r.st.beta, 0.f);
        }
        k.c3 = has_slope ? r.sl : 0.f;
    } else if (xf == ISG_XF_BN_BWD) {
        if (has_coef) {
            k = ChanCoef{r.f[0], r.f[1], r.f[2], r.f[3]};
        } else if constexpr (NG == 4) {
            double mean, rstd;
            mean_rstd_of(stat_sum(r.st, 0), stat_sum(r.st, 1), ISG_SEL3(s, count, vt),
                         ISG_SEL3(s, eps, vt), mean, rstd);
            k = bwd_coef_of(mean, rstd, r.st.gamma, stat_sum(r.st, 2), stat_sum(r.st, 3),
                            ISG_SEL3(s, count, vt));
        }
    }
    return k;
}

// addressing part of channel c (kernel arguments only, no memory access)
ISG_DEV ChSrc ch_addr(const VtSel vt, int c, int64_t hw) {
    int cl;
    const int s = vt_seg(vt, c, cl);
    ChSrc r;
    r.p = ISG_SEL3(s, p, vt) + (int64_t)cl * hw;
    r.ns = ISG_SEL3(s, ns, vt);
    r.yns = ISG_SEL3(s, yns, vt);
    r.xf = ISG_SEL3(s, xf, vt);
    r.act = ISG_SEL3(s, act, vt);
    const float* y = ISG_SEL3(s, y, vt);
    const bool hy = (r.xf == ISG_XF_BN_BWD || r.xf == ISG_XF_BN_FWD) && y;
    r.y = hy ? y + (int64_t)cl * hw : r.p;
    r.yns = hy ? r.yns : r.ns;
    return r;
}

struct SinkLite {
    float *p, *p2;
    const float *y, *coef, *bias, *slope, *gamma, *beta, *r, *old;
    const double* stats;
    int ns, yns, mode, act, c0, bnC, rns, ons, p2ns, p2acc;
    float count, eps;
};
ISG_DEV SinkLite sink_lite(const isg_sink& k) {
    SinkLite l;
    l.p = sgpr_p(k.p); l.y = sgpr_p(k.y); l.coef = sgpr_p((const float*)k.bn.coef);
    l.bias = sgpr_p(k.bias); l.slope = sgpr_p(k.slope);
    l.gamma = sgpr_p(k.bn.gamma); l.beta = sgpr_p(k.bn.beta);
    l.stats = sgpr_p((const double*)k.bn.stats);
    l.ns = sgpr_i((int)k.n_stride); l.yns = sgpr_i((int)k.y_n_stride);
    l.mode = sgpr_i(k.mode); l.act = sgpr_i(k.act); l.c0 = sgpr_i(k.c0); l.bnC = sgpr_i(k.bn.C);
    l.count = sgpr_f(k.bn.count); l.eps = sgpr_f(k.bn.eps);
    l.r = sgpr_p(k.r); l.old = sgpr_p(k.old); l.p2 = sgpr_p(k.p2);
    l.rns = sgpr_i((int)k.r_n_stride); l.ons = sgpr_i((int)k.old_n_stride);
    l.p2ns = sgpr_i((int)k.p2_n_stride);
    l.p2acc = sgpr_i(k.p2_accum);
    return l;
}
struct SkSel {
    SinkLite s0, s1, s2;
    int nsink;
};
ISG_DEV SkSel sk_sel(const isg_sinks& sk) {
    SkSel v;
    v.nsink = sgpr_i(sk.nsink);
    v.s0 = sink_lite(sk.s[0]);
    v.s1 = sink_lite(sk.s[1]);
    v.s2 = sink_lite(sk.s[2]);
    return v;
}

struct SinkLoad {
    f32x4 f;
    float bias, sl;
    StatLoad<2> st;  // ACTBWD without finalised coefficients: the output BN's statistics
};

ISG_DEV int sk_seg(const SkSel sk, int m, int& cl) {
    int s = 0;
    if (sk.nsink > 1 && m >= sk.s1.c0) s = 1;
    if (sk.nsink > 2 && m >= sk.s2.c0) s = 2;
    cl = m - ISG_SEL3(s, c0, sk);
    return s;
}

// `any` is a valid global address (stands in for NULL pointers)
ISG_DEV SinkLoad sink_issue(const SkSel sk, int m, const float* any, bool stat_on = true) {
    int cl;
    const int s = sk_seg(sk, m, cl);
    const float* coef = ISG_SEL3(s, coef, sk);
    const float* bias = ISG_SEL3(s, bias, sk);
    const float* slope = ISG_SEL3(s, slope, sk);
    const float* cp = coef ? coef + 4 * (int64_t)cl : any;
    const float* bp = bias ? bias + cl : any;
    const float* sp = slope ? slope + cl : any;
    const int mode = ISG_SEL3(s, mode, sk);
    const double* st = mode == ISG_SINK_ACTBWD && !coef ? ISG_SEL3(s, stats, sk) : nullptr;
    SinkLoad r;
    r.f = f32x4{gld(cp, 0), gld(cp, 1), gld(cp, 2), gld(cp, 3)};
    r.bias = gld(bp, 0);
    r.sl = gld(sp, 0);
    r.st = stat_issue<2>(st, ISG_SEL3(s, gamma, sk), ISG_SEL3(s, beta, sk), ISG_SEL3(s, bnC, sk), cl,
                         any, stat_on);
    return r;
}

ISG_DEV SinkRow sink_finish(const SkSel sk, int m, int64_t hw, const SinkLoad& l) {
    int cl;
    const int s = sk_seg(sk, m, cl);
    SinkRow q = {};
    float* p = ISG_SEL3(s, p, sk);
    const float* y = ISG_SEL3(s, y, sk);
    q.p = p ? p + (int64_t)cl * hw : nullptr;
    q.y = y ? y + (int64_t)cl * hw : nullptr;
    q.ns = ISG_SEL3(s, ns, sk);
    q.yns = ISG_SEL3(s, yns, sk);
    q.mode = ISG_SEL3(s, mode, sk);
    q.act = ISG_SEL3(s, act, sk);
    q.bias = ISG_SEL3(s, bias, sk) ? l.bias : 0.f;
    q.f = SinkCoef{0.f, 1.f, 0.f, 0.f};
    if (q.mode == ISG_SINK_ACTBWD) {
        if (ISG_SEL3(s, coef, sk)) {
            q.f.mean = l.f[0]; q.f.scale = l.f[1]; q.f.beta = l.f[2];
        } else if (ISG_SEL3(s, stats, sk)) {  // consumer-side finalisation (fwd_coef's math)
            double mean, rstd;
            mean_rstd_of(stat_sum(l.st, 0), stat_sum(l.st, 1), ISG_SEL3(s, count, sk),
                         ISG_SEL3(s, eps, sk), mean, rstd);
            const ChanCoef f = fwd_coef_of(mean, rstd, l.st.gamma, l.st.beta, 0.f);
            q.f.mean = f.c0; q.f.scale = f.c1; q.f.beta = f.c2;
        }
        q.f.slope = ISG_SEL3(s, slope, sk) ? l.sl : 0.f;
    }
    return q;
}

// sink_row_flush for a launch with ONE sink (k = sinks.s[0]): its fields are scalar
// kernel-argument loads. (sink_row_flush selects the sink per lane, which hipcc turns into
// per-lane global loads of kernel-argument fields, each waited for before the next: a
// serial chain of round trips at the very end of every 1x1 launch.)
ISG_DEV void sink_row_flush1(const isg_sink& k, int m, float r0, float r1, float r2) {
    const int cl = m - sgpr_i(k.c0);
    const int C = sgpr_i(k.C), mode = sgpr_i(k.mode);
    if (mode == ISG_SINK_STORE || mode == ISG_SINK_ACCUM) {
        double* const st = sgpr_p(k.stats);
        if (st) {
            double* sp = rep_ptr(st, 4 * C);
            atomicAdd(&sp[cl], (double)r0);
            atomicAdd(&sp[C + cl], (double)r1);
        }
    } else if (mode == ISG_SINK_ACTBWD) {
        double* const st = sgpr_p(k.bn.stats);
        if (st) {
            double* sp = rep_ptr(st, 4 * C);
            atomicAdd(&sp[2 * C + cl], (double)r0);
            atomicAdd(&sp[3 * C + cl], (double)r1);
        }
        double* const sg = sgpr_p(k.slope_grad);
        if (sg && sgpr_i(k.act) == ISG_ACT_PRELU) atomicAdd(&rep_ptr(sg, C)[cl], (double)r2);
    }
}

// Fold row m's block-reduced sums into the sink's replicated fp64 accumulators. The three
// sinks' fields are made scalars first and the lane's sink selected among them (v_cndmask):
// selecting the kernel-argument struct per lane made hipcc load every field per lane from
// kernel-argument memory, one waited global load after another (see sgpr_i).
struct FlushLite {
    double *st, *bst, *sg;
    int C, mode, act, c0;
};
ISG_DEV FlushLite flush_lite(const isg_sink& k) {
    FlushLite f;
    f.st = sgpr_p(k.stats); f.bst = sgpr_p(k.bn.stats); f.sg = sgpr_p(k.slope_grad);
    f.C = sgpr_i(k.C); f.mode = sgpr_i(k.mode); f.act = sgpr_i(k.act); f.c0 = sgpr_i(k.c0);
    return f;
}
ISG_DEV void sink_row_flush(const isg_sinks& sk, int m, float r0, float r1, float r2) {
    const int ns = sgpr_i(sk.nsink);
    const FlushLite f0 = flush_lite(sk.s[0]), f1 = flush_lite(sk.s[1]), f2 = flush_lite(sk.s[2]);
    int s = 0;  // sink_of's rule
    if (ns > 1 && m >= f1.c0) s = 1;
    if (ns > 2 && m >= f2.c0) s = 2;
#define ISG_FSEL(f) (s == 2 ? f2.f : (s == 1 ? f1.f : f0.f))
    double* const st = ISG_FSEL(st);
    double* const bst = ISG_FSEL(bst);
    double* const sg = ISG_FSEL(sg);
    const int C = ISG_FSEL(C), mode = ISG_FSEL(mode), act = ISG_FSEL(act);
    const int cl = m - ISG_FSEL(c0);
#undef ISG_FSEL
    if (mode == ISG_SINK_STORE || mode == ISG_SINK_ACCUM) {
        if (st) {
            double* sp = rep_ptr(st, 4 * C);
            atomicAdd(&sp[cl], (double)r0);
            atomicAdd(&sp[C + cl], (double)r1);
        }
    } else if (mode == ISG_SINK_ACTBWD) {
        if (bst) {
            double* sp = rep_ptr(bst, 4 * C);
            atomicAdd(&sp[2 * C + cl], (double)r0);
            atomicAdd(&sp[3 * C + cl], (double)r1);
        }
        if (sg && act == ISG_ACT_PRELU) atomicAdd(&rep_ptr(sg, C)[cl], (double)r2);
    }
}
