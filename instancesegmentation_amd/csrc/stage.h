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

ISG_DEV ChSrc ch_src(const isg_vtensor& vt, int c, int hw) {
    const int c1 = vt.s[0].C, c2 = c1 + vt.s[1].C;
    const bool s1 = vt.nseg > 1 && c >= c1, s2 = vt.nseg > 2 && c >= c2;
    // explicit selects: a runtime index into the kernel-argument struct would copy it
    const float* p = s2 ? vt.s[2].p : (s1 ? vt.s[1].p : vt.s[0].p);
    const float* y = s2 ? vt.s[2].y : (s1 ? vt.s[1].y : vt.s[0].y);
    const int64_t ns = s2 ? vt.s[2].n_stride : (s1 ? vt.s[1].n_stride : vt.s[0].n_stride);
    const int64_t yns = s2 ? vt.s[2].y_n_stride : (s1 ? vt.s[1].y_n_stride : vt.s[0].y_n_stride);
    const int xf = s2 ? vt.s[2].xform : (s1 ? vt.s[1].xform : vt.s[0].xform);
    const int act = s2 ? vt.s[2].act : (s1 ? vt.s[1].act : vt.s[0].act);
    const int cl = c - (s2 ? c2 : (s1 ? c1 : 0));
    ChSrc r;
    r.p = p + (int64_t)cl * hw;
    r.y = (xf == ISG_XF_BN_BWD && y) ? y + (int64_t)cl * hw : r.p;
    r.ns = (int)ns;
    r.yns = (int)yns;
    r.xf = xf;
    r.act = act;
    return r;
}

// Coefficients of channel c of a vtensor (common.h ChanCoef conventions).
ISG_DEV ChanCoef vt_coef(const isg_vtensor& vt, int c) {
    const int c1 = vt.s[0].C, c2 = c1 + vt.s[1].C;
    const int s = (vt.nseg > 2 && c >= c2) ? 2 : ((vt.nseg > 1 && c >= c1) ? 1 : 0);
    const isg_vseg& sg = s == 2 ? vt.s[2] : (s == 1 ? vt.s[1] : vt.s[0]);
    const int cl = c - (s == 2 ? c2 : (s == 1 ? c1 : 0));
    ChanCoef k = {0.f, 1.f, 0.f, 0.f};
    if (sg.xform == ISG_XF_BN_FWD) {
        if (sg.bn.stats || !sg.bn.train) k = fwd_coef(sg.bn, sg.slope, cl);
        else k.c3 = sg.slope ? sg.slope[cl] : 0.f;  // activation only
    } else if (sg.xform == ISG_XF_BN_BWD) {
        k = bwd_coef(sg.bn, cl);
    }
    return k;
}

// v = transform of raw x (and saved y for BN_BWD); xf/act uniform -> scalar branches
ISG_DEV float ch_xform(int xf, int act, const ChanCoef& k, float x, float y) {
    if (xf == ISG_XF_PLAIN) return x;
    if (xf == ISG_XF_BN_FWD) return apply_act((x - k.c0) * k.c1 + k.c2, act, k.c3);
    return k.c0 * x + k.c1 * (y - k.c2) + k.c3;
}

ISG_DEV int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }
