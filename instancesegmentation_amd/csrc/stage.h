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
    const float* y;  // BN_BWD: saved forward output of the channel (else == p)
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
    r.y = (r.xf == ISG_XF_BN_BWD && y) ? y + (int64_t)cl * hw : r.p;
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

ISG_DEV SinkRow sink_row(const isg_sinks& sk, int m, int64_t hw) {
    SinkRow q = {};
    const int s = sink_of(sk, m);
    const isg_sink& k = s == 2 ? sk.s[2] : (s == 1 ? sk.s[1] : sk.s[0]);
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

// Fold row m's block-reduced sums into the sink's replicated fp64 accumulators.
ISG_DEV void sink_row_flush(const isg_sinks& sk, int m, float r0, float r1, float r2) {
    const int s = sink_of(sk, m);
    const isg_sink& k = s == 2 ? sk.s[2] : (s == 1 ? sk.s[1] : sk.s[0]);
    const int cl = m - k.c0;
    if (k.mode == ISG_SINK_STORE || k.mode == ISG_SINK_ACCUM) {
        if (k.stats) {
            double* sp = rep_ptr(k.stats, 4 * k.C);
            atomicAdd(&sp[cl], (double)r0);
            atomicAdd(&sp[k.C + cl], (double)r1);
        }
    } else if (k.mode == ISG_SINK_ACTBWD) {
        if (k.bn.stats) {
            double* sp = rep_ptr(k.bn.stats, 4 * k.C);
            atomicAdd(&sp[2 * k.C + cl], (double)r0);
            atomicAdd(&sp[3 * k.C + cl], (double)r1);
        }
        if (k.slope_grad && k.act == ISG_ACT_PRELU) atomicAdd(&rep_ptr(k.slope_grad, k.C)[cl], (double)r2);
    }
}
