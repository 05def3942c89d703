#pragma once
#include "../../include/isg.h"

// Host checks of the residual forms (isg.h: a BN_FWD segment with y, vtensor.mat, the
// ACTBWD sink's r / old / p2): only the 1x1 stride-1 GEMM (pw_gemm.hip) implements them,
// every other entry point refuses them instead of silently dropping the residual.
inline bool isg_seg_res(const isg_vseg& s) { return s.xform == ISG_XF_BN_FWD && s.y; }
inline bool isg_vt_res(const isg_vtensor* v) {
    if (!v) return false;
    bool r = v->mat != nullptr || v->rbn.stats != nullptr || v->rbn.coef != nullptr;
    for (int i = 0; i < v->nseg && i < ISG_MAX_SEGS; ++i) r |= isg_seg_res(v->s[i]);
    return r;
}
// a BN_BWD segment without y (isg.h isg_vseg: y = p, at p's image stride), resolved at
// every public entry point that takes a vtensor, so no kernel has to know the convention
inline isg_vtensor isg_resolve_y(const isg_vtensor* v) {
    isg_vtensor r{};
    if (!v) return r;  // nseg 0: refused by the kernels' channel checks
    r = *v;
    for (int i = 0; i < r.nseg && i < ISG_MAX_SEGS; ++i)
        if (r.s[i].xform == ISG_XF_BN_BWD && !r.s[i].y) {
            r.s[i].y = r.s[i].p;
            r.s[i].y_n_stride = r.s[i].n_stride;
        }
    return r;
}
inline bool isg_sinks_res(const isg_sinks* k) {
    if (!k) return false;
    bool r = false;
    for (int i = 0; i < k->nsink && i < ISG_MAX_SEGS; ++i)
        r |= k->s[i].r || k->s[i].old || k->s[i].p2 || k->s[i].rbn.stats || k->s[i].rbn.coef;
    return r;
}
