// Element-wise / reduction kernels of the hot path (gfx950, HBM-streaming).
//
//  * residual-block tails  out = act(sum of BN'd / plain / upsampled terms)
//    (segment.py:76-77, 107-109, 147-148, 202-207, 255-259, 331-333) and their
//    backward, which also produces the BatchNorm-backward statistics of every BN term
//    and the PReLU slope gradient in the same pass;
//  * max-pool k x k / stride k (segment.py:29, 145) forward and backward;
//  * BatchNorm running-stat update and parameter-gradient finalisation;
//  * fused sigmoid + BCELoss (segment.py:534, train_instance.py:299,378);
//  * Adam (train_instance.py:297,380).
#include <cstring>

#include "common.h"

namespace {

constexpr int kThreads = 256;

ISG_DEV ChanCoef seg_coef(const isg_vseg& sg, int c) {
    ChanCoef k = {0.f, 1.f, 0.f, 0.f};
    if (sg.xform == ISG_XF_BN_FWD) {
        if (sg.bn.stats || !sg.bn.train) k = fwd_coef(sg.bn, sg.slope, c);
        else k.c3 = sg.slope ? sg.slope[c] : 0.f;
    } else if (sg.xform == ISG_XF_BN_BWD) {
        k = bwd_coef(sg.bn, c);
    }
    return k;
}

ISG_DEV float seg_val(const isg_vseg& sg, const ChanCoef& k, float x, float y) {
    if (sg.xform == ISG_XF_PLAIN) return x;
    if (sg.xform == ISG_XF_BN_FWD) return apply_act((x - k.c0) * k.c1 + k.c2, sg.act, k.c3);
    return k.c0 * x + k.c1 * (y - k.c2) + k.c3;
}

template <int NV>
ISG_DEV void block_reduce(float (&v)[NV], float* sh) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) sh[i * 4 + wave] = v[i];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = sh[i * 4] + sh[i * 4 + 1] + sh[i * 4 + 2] + sh[i * 4 + 3];
}

// ---- residual tail ----------------------------------------------------------------
// Thread unit: a 2x2 pixel quad of one (n, c) plane (H, W are even in this network:
// input sides are multiples of 16), so an x2-upsampled term is one
// low-resolution value per thread and its gradient is the quad's sum.
ISG_DEV float term_raw(const isg_vseg& t, int up, int n, int c, int H, int W, int y, int x,
                       float* yraw) {
    int64_t hw, pix;
    if (up) {
        const int h2 = H >> 1, w2 = W >> 1;
        hw = (int64_t)h2 * w2;
        pix = (int64_t)(y >> 1) * w2 + (x >> 1);
    } else {
        hw = (int64_t)H * W;
        pix = (int64_t)y * W + x;
    }
    *yraw = 0.f;
    return t.p[(int64_t)n * t.n_stride + (int64_t)c * hw + pix];
}

__global__ __launch_bounds__(kThreads) void tail_fwd_kernel(isg_tail t) {
    const int c = blockIdx.y, n = blockIdx.z;
    const int H = t.H, W = t.W;
    const int qw = W >> 1;
    const int64_t nq = (int64_t)(H >> 1) * qw;
    const int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (q >= nq) return;
    const int qy = (int)(q / qw), qx = (int)(q - (int64_t)qy * qw);
    const int64_t hw = (int64_t)H * W;
    // the quad's raw term values first: their loads do not depend on the coefficients
    // (consumer-side BatchNorm finalisation reads the statistics below), so both round
    // trips overlap instead of running back to back
    float2 raw[2][3];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            raw[dy][i] = make_float2(0.f, 0.f);
            if (i >= t.nterm) continue;
            const isg_vseg& tm = t.term[i];
            const int y = 2 * qy + dy;
            if (t.up[i]) {
                float dummy;
                const float x0 = term_raw(tm, 1, n, c, H, W, y, 2 * qx, &dummy);
                raw[dy][i] = make_float2(x0, x0);
            } else {
                const int64_t off = (int64_t)n * tm.n_stride + (int64_t)c * hw + (int64_t)y * W + 2 * qx;
                raw[dy][i] = *reinterpret_cast<const float2*>(tm.p + off);
            }
        }
    ChanCoef k[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        if (i < t.nterm) k[i] = seg_coef(t.term[i], c);
    const float slope = (t.act == ISG_ACT_PRELU) ? t.slope[c] : 0.f;
    float* out = t.out + (int64_t)n * t.out_n_stride + (int64_t)c * hw;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        float v[2] = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (i >= t.nterm) continue;
            const isg_vseg& tm = t.term[i];
            v[0] += seg_val(tm, k[i], raw[dy][i].x, 0.f);
            v[1] += seg_val(tm, k[i], raw[dy][i].y, 0.f);
        }
        float2 o;
        o.x = apply_act(v[0], t.act, slope);
        o.y = apply_act(v[1], t.act, slope);
        *reinterpret_cast<float2*>(out + (int64_t)(2 * qy + dy) * W + 2 * qx) = o;
    }
}

__global__ __launch_bounds__(kThreads) void tail_bwd_kernel(isg_tail_grad tg) {
    __shared__ float sh[8 * 4];
    const isg_tail& t = tg.f;
    const int c = blockIdx.y, n = blockIdx.z;
    const int H = t.H, W = t.W;
    const int qw = W >> 1;
    const int64_t nq = (int64_t)(H >> 1) * qw;
    const int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const bool valid = q < nq;
    const int qy = valid ? (int)(q / qw) : 0, qx = valid ? (int)(q - (int64_t)qy * qw) : 0;
    const int64_t hw = (int64_t)H * W;
    // every load of the quad first (dout and the raw terms), then the coefficients: the
    // loads do not depend on them, so the two round trips overlap (tail_fwd_kernel)
    float2 dld[2], rld[2][3];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const int y = 2 * qy + dy;
        const int64_t prow = (int64_t)y * W + 2 * qx;
        // unconditional (an invalid lane reads quad (0, 0) of its plane): a load behind a
        // per-lane branch makes the compiler drain the memory queue at the join
        dld[dy] = *reinterpret_cast<const float2*>(tg.dout + (int64_t)n * tg.dout_n_stride +
                                                   (int64_t)c * hw + prow);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            rld[dy][i] = make_float2(0.f, 0.f);
            if (i >= t.nterm) continue;
            const isg_vseg& tm = t.term[i];
            if (t.up[i]) {
                float dummy;
                const float x0 = term_raw(tm, 1, n, c, H, W, y, 2 * qx, &dummy);
                rld[dy][i] = make_float2(x0, x0);
            } else {
                rld[dy][i] = *reinterpret_cast<const float2*>(tm.p + (int64_t)n * tm.n_stride +
                                                              (int64_t)c * hw + prow);
            }
        }
    }
    // the old values of accumulated term gradients, in the same round trip
    float2 old[2][3];
    float oldup[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        oldup[i] = 0.f;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) old[dy][i] = make_float2(0.f, 0.f);
        if (i >= t.nterm || t.term[i].xform != ISG_XF_PLAIN || !tg.dterm[i] || !tg.dterm_accum[i]) continue;
        if (t.up[i]) {
            const int64_t lhw = (int64_t)(H >> 1) * (W >> 1);
            oldup[i] = tg.dterm[i][(int64_t)n * tg.dterm_n_stride[i] + (int64_t)c * lhw + (valid ? q : 0)];
        } else {
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
                old[dy][i] = *reinterpret_cast<const float2*>(
                    tg.dterm[i] + (int64_t)n * tg.dterm_n_stride[i] + (int64_t)c * hw +
                    (int64_t)(2 * qy + dy) * W + 2 * qx);
        }
    }
    ChanCoef k[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        if (i < t.nterm) k[i] = seg_coef(t.term[i], c);
    const float slope = (t.act == ISG_ACT_PRELU) ? t.slope[c] : 0.f;
    // red: [0..2] gsum per term (same g), [3..5] g*(y-mean) per term, [6] slope grad
    float red[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float gq[2][2];
    float upsum = 0.f;
    if (valid) {
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int y = 2 * qy + dy;
            const int64_t prow = (int64_t)y * W + 2 * qx;
            const float2 d = dld[dy];
            float pre[2] = {0.f, 0.f};
            float raw[3][2];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                raw[i][0] = raw[i][1] = 0.f;
                if (i >= t.nterm) continue;
                const isg_vseg& tm = t.term[i];
                raw[i][0] = rld[dy][i].x;
                raw[i][1] = rld[dy][i].y;
                pre[0] += seg_val(tm, k[i], raw[i][0], 0.f);
                pre[1] += seg_val(tm, k[i], raw[i][1], 0.f);
            }
            const float dv[2] = {d.x, d.y};
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                float g = dv[e];
                if (t.act == ISG_ACT_RELU) {
                    g = pre[e] > 0.f ? dv[e] : 0.f;
                } else if (t.act == ISG_ACT_PRELU) {
                    g = pre[e] > 0.f ? dv[e] : dv[e] * slope;
                    red[6] += pre[e] > 0.f ? 0.f : pre[e] * dv[e];
                }
                gq[dy][e] = g;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if (i >= t.nterm) continue;
                    if (t.term[i].xform == ISG_XF_BN_FWD) {
                        red[i] += g;
                        red[3 + i] += g * (raw[i][e] - k[i].c0);  // centred (c0 = mean)
                    }
                }
            }
            if (tg.g) {
                *reinterpret_cast<float2*>(tg.g + (int64_t)n * tg.g_n_stride + (int64_t)c * hw + prow) =
                    make_float2(gq[dy][0], gq[dy][1]);
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                if (i >= t.nterm || t.term[i].xform != ISG_XF_PLAIN || !tg.dterm[i] || t.up[i]) continue;
                float* dst = tg.dterm[i] + (int64_t)n * tg.dterm_n_stride[i] + (int64_t)c * hw + prow;
                float2 o = make_float2(gq[dy][0], gq[dy][1]);
                if (tg.dterm_accum[i]) {
                    o.x += old[dy][i].x;
                    o.y += old[dy][i].y;
                }
                *reinterpret_cast<float2*>(dst) = o;
            }
        }
        upsum = (gq[0][0] + gq[0][1]) + (gq[1][0] + gq[1][1]);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (i >= t.nterm || t.term[i].xform != ISG_XF_PLAIN || !tg.dterm[i] || !t.up[i]) continue;
            const int64_t lhw = (int64_t)(H >> 1) * (W >> 1);
            float* dst = tg.dterm[i] + (int64_t)n * tg.dterm_n_stride[i] + (int64_t)c * lhw + q;
            *dst = tg.dterm_accum[i] ? oldup[i] + upsum : upsum;
        }
    }
    bool need = (t.act == ISG_ACT_PRELU && tg.slope_grad);
    for (int i = 0; i < t.nterm; ++i) need |= (t.term[i].xform == ISG_XF_BN_FWD);
    if (!need) return;
    float rv[8] = {red[0], red[1], red[2], red[3], red[4], red[5], red[6], 0.f};
    block_reduce<8>(rv, sh);
    if (threadIdx.x == 0) {
        for (int i = 0; i < t.nterm; ++i) {
            const isg_vseg& tm = t.term[i];
            if (tm.xform == ISG_XF_BN_FWD && tm.bn.stats) {
                double* sp = rep_ptr(tm.bn.stats, 4 * tm.bn.C);
                atomicAdd(&sp[2 * tm.bn.C + c], (double)rv[i]);
                atomicAdd(&sp[3 * tm.bn.C + c], (double)rv[3 + i]);
            }
        }
        if (t.act == ISG_ACT_PRELU && tg.slope_grad)
            atomicAdd(&rep_ptr(tg.slope_grad, t.C)[c], (double)rv[6]);
    }
}

// ---- residual tail, 2 x 4 pixel units (W % 4 == 0, 16-B aligned planes) --------------
// The same tails as above with a thread owning two rows of 4 pixels: every full-resolution
// operand moves as 16-B accesses (an x2-upsampled term as one 8-B pair of low-resolution
// values per row pair), half the threads, workgroups and reductions of the quad form.
typedef f32x4 __attribute__((address_space(1)))* t4p;
typedef const f32x4 __attribute__((address_space(1)))* tc4p;
typedef float tf32x2 __attribute__((ext_vector_type(2)));
typedef const tf32x2 __attribute__((address_space(1)))* tc2p;
typedef tf32x2 __attribute__((address_space(1)))* t2p;

ISG_DEV f32x4 tail_term4(const isg_vseg& tm, int up, int n, int c, int H, int W, int y, int x4) {
    if (up) {
        const int w2 = W >> 1;
        const int64_t off = (int64_t)n * tm.n_stride + (int64_t)c * (H >> 1) * w2 + (int64_t)(y >> 1) * w2 + (x4 >> 1);
        const tf32x2 v = *(tc2p)((gcfloat_p)tm.p + off);
        return f32x4{v.x, v.x, v.y, v.y};
    }
    const int64_t off = (int64_t)n * tm.n_stride + (int64_t)c * H * W + (int64_t)y * W + x4;
    return *(tc4p)((gcfloat_p)tm.p + off);
}

__global__ __launch_bounds__(kThreads) void tail_fwd4_kernel(isg_tail t) {
    const int c = blockIdx.y, n = blockIdx.z;
    const int H = t.H, W = t.W;
    const int qw = W >> 2;
    const int nq = (H >> 1) * qw;
    const int q = blockIdx.x * kThreads + threadIdx.x;
    if (q >= nq) return;
    const int qy = q / qw, x4 = (q - qy * qw) * 4;
    f32x4 raw[2][3];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            raw[dy][i] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (i < t.nterm) raw[dy][i] = tail_term4(t.term[i], t.up[i], n, c, H, W, 2 * qy + dy, x4);
        }
    ChanCoef k[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        if (i < t.nterm) k[i] = seg_coef(t.term[i], c);
    const float slope = (t.act == ISG_ACT_PRELU) ? t.slope[c] : 0.f;
    float* out = t.out + (int64_t)n * t.out_n_stride + (int64_t)c * H * W;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (i >= t.nterm) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] += seg_val(t.term[i], k[i], raw[dy][i][e], 0.f);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = apply_act(o[e], t.act, slope);
        *(t4p)((gfloat_p)out + (int64_t)(2 * qy + dy) * W + x4) = o;
    }
}

__global__ __launch_bounds__(kThreads) void tail_bwd4_kernel(isg_tail_grad tg) {
    __shared__ float sh[8 * 4];
    const isg_tail& t = tg.f;
    const int c = blockIdx.y, n = blockIdx.z;
    const int H = t.H, W = t.W;
    const int qw = W >> 2;
    const int nq = (H >> 1) * qw;
    const int q0 = blockIdx.x * kThreads + threadIdx.x;
    const bool valid = q0 < nq;
    const int q = valid ? q0 : 0;  // invalid lanes load unit 0 (no per-lane branch on loads)
    const int qy = q / qw, x4 = (q - qy * qw) * 4;
    const int64_t hw = (int64_t)H * W;
    const int w2 = W >> 1;
    const int64_t lhw = (int64_t)(H >> 1) * w2;
    f32x4 dld[2], rld[2][3], old[2][3];
    tf32x2 oldup[3];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const int64_t prow = (int64_t)(2 * qy + dy) * W + x4;
        dld[dy] = *(tc4p)((gcfloat_p)tg.dout + (int64_t)n * tg.dout_n_stride + (int64_t)c * hw + prow);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            rld[dy][i] = old[dy][i] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (i >= t.nterm) continue;
            rld[dy][i] = tail_term4(t.term[i], t.up[i], n, c, H, W, 2 * qy + dy, x4);
            if (t.term[i].xform == ISG_XF_PLAIN && tg.dterm[i] && tg.dterm_accum[i] && !t.up[i])
                old[dy][i] = *(tc4p)((gcfloat_p)tg.dterm[i] + (int64_t)n * tg.dterm_n_stride[i] +
                                     (int64_t)c * hw + prow);
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        oldup[i] = tf32x2{0.f, 0.f};
        if (i < t.nterm && t.term[i].xform == ISG_XF_PLAIN && tg.dterm[i] && tg.dterm_accum[i] && t.up[i])
            oldup[i] = *(tc2p)((gcfloat_p)tg.dterm[i] + (int64_t)n * tg.dterm_n_stride[i] + (int64_t)c * lhw +
                               (int64_t)qy * w2 + (x4 >> 1));
    }
    ChanCoef k[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        if (i < t.nterm) k[i] = seg_coef(t.term[i], c);
    const float slope = (t.act == ISG_ACT_PRELU) ? t.slope[c] : 0.f;
    float red[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    f32x4 gq[2];
    if (valid) {
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
            const int64_t prow = (int64_t)(2 * qy + dy) * W + x4;
            f32x4 pre = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                if (i >= t.nterm) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) pre[e] += seg_val(t.term[i], k[i], rld[dy][i][e], 0.f);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float dv = dld[dy][e];
                float g = dv;
                if (t.act == ISG_ACT_RELU) {
                    g = pre[e] > 0.f ? dv : 0.f;
                } else if (t.act == ISG_ACT_PRELU) {
                    g = pre[e] > 0.f ? dv : dv * slope;
                    red[6] += pre[e] > 0.f ? 0.f : pre[e] * dv;
                }
                gq[dy][e] = g;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if (i >= t.nterm || t.term[i].xform != ISG_XF_BN_FWD) continue;
                    red[i] += g;
                    red[3 + i] += g * (rld[dy][i][e] - k[i].c0);  // centred (c0 = mean)
                }
            }
            if (tg.g) *(t4p)((gfloat_p)tg.g + (int64_t)n * tg.g_n_stride + (int64_t)c * hw + prow) = gq[dy];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                if (i >= t.nterm || t.term[i].xform != ISG_XF_PLAIN || !tg.dterm[i] || t.up[i]) continue;
                f32x4 o = gq[dy];
                if (tg.dterm_accum[i]) o += old[dy][i];
                *(t4p)((gfloat_p)tg.dterm[i] + (int64_t)n * tg.dterm_n_stride[i] + (int64_t)c * hw + prow) = o;
            }
        }
        // x2-upsampled terms: each low-resolution pixel's gradient is its 2x2 block's sum
        const tf32x2 us = {(gq[0][0] + gq[0][1]) + (gq[1][0] + gq[1][1]),
                           (gq[0][2] + gq[0][3]) + (gq[1][2] + gq[1][3])};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (i >= t.nterm || t.term[i].xform != ISG_XF_PLAIN || !tg.dterm[i] || !t.up[i]) continue;
            tf32x2 o = us;
            if (tg.dterm_accum[i]) o += oldup[i];
            *(t2p)((gfloat_p)tg.dterm[i] + (int64_t)n * tg.dterm_n_stride[i] + (int64_t)c * lhw +
                   (int64_t)qy * w2 + (x4 >> 1)) = o;
        }
    }
    bool need = (t.act == ISG_ACT_PRELU && tg.slope_grad);
    for (int i = 0; i < t.nterm; ++i) need |= (t.term[i].xform == ISG_XF_BN_FWD);
    if (!need) return;
    float rv[8] = {red[0], red[1], red[2], red[3], red[4], red[5], red[6], 0.f};
    block_reduce<8>(rv, sh);
    if (threadIdx.x == 0) {
        for (int i = 0; i < t.nterm; ++i) {
            const isg_vseg& tm = t.term[i];
            if (tm.xform == ISG_XF_BN_FWD && tm.bn.stats) {
                double* sp = rep_ptr(tm.bn.stats, 4 * tm.bn.C);
                atomicAdd(&sp[2 * tm.bn.C + c], (double)rv[i]);
                atomicAdd(&sp[3 * tm.bn.C + c], (double)rv[3 + i]);
            }
        }
        if (t.act == ISG_ACT_PRELU && tg.slope_grad)
            atomicAdd(&rep_ptr(tg.slope_grad, t.C)[c], (double)rv[6]);
    }
}

// the 2 x 4 form applies: W % 4 == 0 and every full-resolution plane 16-B aligned (the
// upsampled terms 8-B), image strides multiples of 4 floats
bool al(const void* p, int b) { return ((uintptr_t)p % b) == 0; }
bool tail4_ok(const isg_tail& t, const isg_tail_grad* tg) {
    // planes of >= 128^2 pixels only: at 64^2 the halved grid (512 workgroups at 128
    // channels) measured 0.3-0.4 us slower per op, at 128^2 and up 1.3-2.5 us faster (r03v)
    if (t.W % 4 || (int64_t)t.H * t.W < 16384) return false;
    for (int i = 0; i < t.nterm; ++i) {
        const isg_vseg& s = t.term[i];
        if (!al(s.p, t.up[i] ? 8 : 16) || s.n_stride % (t.up[i] ? 2 : 4)) return false;
        if (tg && tg->dterm[i] && (!al(tg->dterm[i], t.up[i] ? 8 : 16) || tg->dterm_n_stride[i] % (t.up[i] ? 2 : 4)))
            return false;
    }
    if (!tg) return al(t.out, 16) && t.out_n_stride % 4 == 0;
    if (!al(tg->dout, 16) || tg->dout_n_stride % 4) return false;
    if (tg->g && (!al(tg->g, 16) || tg->g_n_stride % 4)) return false;
    return true;
}

// ---- max-pool ---------------------------------------------------------------------
struct PoolArgs {
    isg_vtensor x;
    int k;
    float* out;
    int64_t out_n_stride;
    const float* dout;
    int64_t dout_n_stride;
    isg_sinks dx;
};

template <bool BWD>
__global__ __launch_bounds__(kThreads) void maxpool_kernel(PoolArgs a) {
    __shared__ ChanCoef coef[ISG_MAX_CH];
    load_vt_coefs(a.x, coef, threadIdx.x, kThreads);
    __syncthreads();
    const int c = blockIdx.y, n = blockIdx.z;
    const int H = a.x.H, W = a.x.W, k = a.k;
    const int OH = H / k, OW = W / k;
    const int64_t ohw = (int64_t)OH * OW, hw = (int64_t)H * W;
    const int64_t op = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (op >= ohw) return;
    const int oy = (int)(op / OW), ox = (int)(op - (int64_t)oy * OW);
    // torch CPU max_pool2d: maxval=-inf, maxindex=window start; take val if
    // (val > maxval) || isnan(val)  -> first maximum wins, NaN propagates
    float best = -INFINITY;
    int bi = 0;
    if constexpr (!BWD) {
        // forward, k = 2 / 4: one vector load per window row (the 4x4 pool of the
        // 20-channel network input, segment.py:23, streams 168 MB), same visiting order
        const int s = (a.x.nseg > 1 && c >= a.x.s[0].C)
                          ? ((a.x.nseg > 2 && c >= a.x.s[0].C + a.x.s[1].C) ? 2 : 1) : 0;
        const int cb = s == 0 ? 0 : (s == 1 ? a.x.s[0].C : a.x.s[0].C + a.x.s[1].C);
        const isg_vseg& sg = s == 0 ? a.x.s[0] : (s == 1 ? a.x.s[1] : a.x.s[2]);
        const int xf = sg.xform, act = sg.act;
        if ((k == 4 || k == 2) && xf != ISG_XF_BN_BWD) {
            const float* base = sg.p + (int64_t)n * sg.n_stride + (int64_t)(c - cb) * hw;
            const ChanCoef kc = coef[c];
            auto tf = [&](float x) {
                return xf == ISG_XF_PLAIN ? x : apply_act((x - kc.c0) * kc.c1 + kc.c2, act, kc.c3);
            };
            for (int dy = 0; dy < k; ++dy) {
                const float* row = base + (int64_t)(oy * k + dy) * W + ox * k;
                float v[4];
                if (k == 4) {
                    const f32x4 q = *reinterpret_cast<const f32x4*>(row);
                    v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
                } else {
                    const float2 q = *reinterpret_cast<const float2*>(row);
                    v[0] = q.x; v[1] = q.y;
                }
                for (int dx = 0; dx < k; ++dx) {
                    const float x = tf(v[dx]);
                    if (x > best || isnan(x)) {
                        best = x;
                        bi = dy * k + dx;
                    }
                }
            }
            a.out[(int64_t)n * a.out_n_stride + (int64_t)c * ohw + op] = best;
            return;
        }
    }
    for (int dy = 0; dy < k; ++dy)
        for (int dx = 0; dx < k; ++dx) {
            const int64_t pix = (int64_t)(oy * k + dy) * W + ox * k + dx;
            const float v = vt_load(a.x, coef, n, c, hw, pix);
            if (v > best || isnan(v)) {
                best = v;
                bi = dy * k + dx;
            }
        }
    if (!BWD) {
        a.out[(int64_t)n * a.out_n_stride + (int64_t)c * ohw + op] = best;
    } else {
        const float d = a.dout[(int64_t)n * a.dout_n_stride + (int64_t)c * ohw + op];
        const int s = sink_of(a.dx, c);
        const isg_sink& sk = a.dx.s[s];
        const int cl = c - sk.c0;
        if (sk.mode == ISG_SINK_NONE) return;
        float* base = sk.p + (int64_t)n * sk.n_stride + (int64_t)cl * hw;
        for (int dy = 0; dy < k; ++dy)
            for (int dx = 0; dx < k; ++dx) {
                const int64_t pix = (int64_t)(oy * k + dy) * W + ox * k + dx;
                const float v = (dy * k + dx == bi) ? d : 0.f;
                if (sk.mode == ISG_SINK_ACCUM) {
                    if (v != 0.f) base[pix] += v;
                } else {
                    base[pix] = v;
                }
            }
    }
}

// ---- BatchNorm running stats & gradient finalisation -------------------------------
struct BnUpdateList {
    isg_bn_update it[ISG_LIST_CHUNK];
};
struct GradFinalList {
    isg_grad_final it[ISG_LIST_CHUNK];
};

ISG_DEV void bn_update_item(const isg_bn_update& u) {
    for (int c = threadIdx.x; c < u.C; c += blockDim.x) {
        const double M = (double)u.count;
        const double mean = rep_sum(u.stats, 4 * u.C, c) / M;
        double var = rep_sum(u.stats, 4 * u.C, u.C + c) / M - mean * mean;
        if (var < 0.0) var = 0.0;
        const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
        const float m = u.momentum;
        u.running_mean[c] = (1.f - m) * u.running_mean[c] + m * (float)mean;
        u.running_var[c] = (1.f - m) * u.running_var[c] + m * (float)unb;
    }
    if (threadIdx.x == 0 && u.num_batches_tracked) u.num_batches_tracked[0] += 1;
}

__global__ void bn_update_kernel(BnUpdateList items, int nitems) {
    const int it = blockIdx.x;
    if (it >= nitems) return;
    bn_update_item(items.it[it]);
}

struct BnFinalList {
    isg_bn it[ISG_LIST_CHUNK];
};

// fwd: coef[c] = (mean, gamma*rstd, beta, 0); bwd: coef[C + c] = (A, B, mean, Cc) — the
// exact values fwd_coef / bwd_coef (common.h) compute from the statistics.
__global__ void bn_finalize_kernel(BnFinalList items, int nitems, int bwd) {
    const int it = blockIdx.x;
    if (it >= nitems) return;
    isg_bn bn = items.it[it];
    float* out = bn.coef;
    bn.coef = nullptr;  // evaluate from the statistics
    for (int c = threadIdx.x; c < bn.C; c += blockDim.x) {
        if (!bwd) {
            const ChanCoef k = fwd_coef(bn, nullptr, c);
            reinterpret_cast<f32x4*>(out)[c] = f32x4{k.c0, k.c1, k.c2, 0.f};
        } else {
            const ChanCoef k = bwd_coef(bn, c);
            reinterpret_cast<f32x4*>(out)[bn.C + c] = f32x4{k.c0, k.c1, k.c2, k.c3};
        }
    }
}

// one layer (the executor's per-BN-point launches): a 64-B kernel argument instead of the
// ISG_LIST_CHUNK-item list
__global__ void bn_finalize1_kernel(isg_bn bn, int bwd) {
    float* out = bn.coef;
    bn.coef = nullptr;
    for (int c = threadIdx.x; c < bn.C; c += blockDim.x) {
        if (!bwd) {
            const ChanCoef k = fwd_coef(bn, nullptr, c);
            reinterpret_cast<f32x4*>(out)[c] = f32x4{k.c0, k.c1, k.c2, 0.f};
        } else {
            const ChanCoef k = bwd_coef(bn, c);
            reinterpret_cast<f32x4*>(out)[bn.C + c] = f32x4{k.c0, k.c1, k.c2, k.c3};
        }
    }
}

// one item's values; put(dst, value) stores each (grad_final_kernel: a plain store; the
// fused step tail: the store plus that element's Adam update)
template <class Put>
ISG_DEV void grad_final_item(const isg_grad_final& f, Put put) {
    for (int c = threadIdx.x; c < f.C; c += blockDim.x) {
        if (f.slope_acc) {
            put(f.dslope + c, (float)rep_sum(f.slope_acc, f.slope_stride, c));
            continue;
        }
        const double M = (double)f.count;
        double mean, rstd;
        if (f.train) {
            mean = rep_sum(f.stats, 4 * f.C, c) / M;
            double var = rep_sum(f.stats, 4 * f.C, f.C + c) / M - mean * mean;
            if (var < 0.0) var = 0.0;
            rstd = 1.0 / sqrt(var + (double)f.eps);
        } else {
            mean = (double)f.running_mean[c];
            rstd = 1.0 / sqrt((double)f.running_var[c] + (double)f.eps);
        }
        const double gs = rep_sum(f.stats, 4 * f.C, 2 * f.C + c);
        const double gxs = rep_sum(f.stats, 4 * f.C, 3 * f.C + c);  // sum g*(y - mean), centred
        const double dgamma = rstd * gxs;
        if (f.dgamma) put(f.dgamma + c, (float)dgamma);
        if (f.dbeta) put(f.dbeta + c, (float)gs);
        if (f.dconv_bias) {
            // sum over pixels of dy = A*g + B*(y-mean) + C  (BatchNorm backward)
            const double gam = (double)f.gamma[c];
            double db;
            if (f.train) {
                const double sy = rep_sum(f.stats, 4 * f.C, c);
                const double mg = gs / M, mgx = rstd * gxs / M;
                db = gam * rstd * (gs - M * mg) - gam * rstd * rstd * mgx * (sy - M * mean);
            } else {
                db = gam * rstd * gs;
            }
            put(f.dconv_bias + c, (float)db);
        }
    }
}

__global__ void grad_final_kernel(GradFinalList items, int nitems) {
    const int it = blockIdx.x;
    if (it >= nitems) return;
    grad_final_item(items.it[it], [](float* d, float v) { *d = v; });
}

// ---- sigmoid + BCE ----------------------------------------------------------------
// the per-element arithmetic of bce_kernel below, one 16-B quad per thread: both loads in
// flight at once and one pass (the strided loop waited out one load round trip per
// element group: 21 us for the 2 x 1024^2 logits of the bench step)
ISG_DEV float bce_elem(float x, float t, float grad_scale, float& g) {
#pragma clang fp contract(off)
    const float p = 1.f / (1.f + expf(-x));
    float lp = logf(p);
    float l1p = logf(1.f - p);
    lp = lp < -100.f ? -100.f : lp;
    l1p = l1p < -100.f ? -100.f : l1p;
    float den = (1.f - p) * p;
    den = den < 1e-12f ? 1e-12f : den;
    const float gp = grad_scale * (p - t) / den;
    g = gp * (1.f - p) * p;
    return -(t * lp + (1.f - t) * l1p);
}

// kBceQ quads per thread (all loads in flight): the loss sum is one fp64 atomic per
// workgroup on ONE address, which serialises — with a quad per thread (2048 workgroups at
// the bench size) those atomics alone took ~30 us
constexpr int kBceQ = 8;
__global__ __launch_bounds__(kThreads) void bce4_kernel(const float* logits, const float* target,
                                                         int64_t nq, double* loss_acc, float* dlogits,
                                                         float grad_scale) {
    __shared__ double sh[4];
    const int64_t i0 = (int64_t)blockIdx.x * kThreads * kBceQ + threadIdx.x;
    f32x4 x[kBceQ], t[kBceQ];
#pragma unroll
    for (int u = 0; u < kBceQ; ++u) {
        const int64_t i = i0 + (int64_t)u * kThreads;
        x[u] = gld4(logits, 4 * (i < nq ? i : 0));
        t[u] = gld4(target, 4 * (i < nq ? i : 0));
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < kBceQ; ++u) {
        const int64_t i = i0 + (int64_t)u * kThreads;
        const bool ok = i < nq;
        f32x4 g;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float ge;
            const float l = bce_elem(x[u][e], t[u][e], grad_scale, ge);
            g[e] = ge;
            acc += ok ? (double)l : 0.0;
        }
        if (ok && dlogits) gst4(dlogits, 4 * i, g);
    }
    acc = wave_sum_d(acc);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) sh[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(loss_acc, sh[0] + sh[1] + sh[2] + sh[3]);
}

__global__ __launch_bounds__(kThreads) void bce_kernel(const float* logits, const float* target,
                                                        int64_t n, double* loss_acc, float* dlogits,
                                                        float grad_scale) {
#pragma clang fp contract(off)
    __shared__ double sh[4];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kThreads) {
        const float x = logits[i];
        const float t = target[i];
        const float p = 1.f / (1.f + expf(-x));
        float lp = logf(p);
        float l1p = logf(1.f - p);
        lp = lp < -100.f ? -100.f : lp;
        l1p = l1p < -100.f ? -100.f : l1p;
        const float l = -(t * lp + (1.f - t) * l1p);
        acc += (double)l;
        if (dlogits) {
            // torch binary_cross_entropy_backward: grad*(p-t)/max((1-p)*p, 1e-12),
            // then sigmoid_backward: g*(1-p)*p
            float den = (1.f - p) * p;
            den = den < 1e-12f ? 1e-12f : den;
            const float gp = grad_scale * (p - t) / den;
            dlogits[i] = gp * (1.f - p) * p;
        }
    }
    acc = wave_sum_d(acc);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) sh[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(loss_acc, sh[0] + sh[1] + sh[2] + sh[3]);
}

__global__ void sigmoid_fwd_kernel(const float* x, float* y, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = 1.f / (1.f + expf(-x[i]));
}

__global__ void sigmoid_bwd_kernel(const float* y, const float* dy, float* dx, int64_t n) {
#pragma clang fp contract(off)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        dx[i] = dy[i] * (1.f - y[i]) * y[i];
}

// ---- Adam ---------------------------------------------------------------------------
// torch.optim.Adam single-tensor math (torch 2.10 _single_tensor_adam):
//   m.lerp_(g, 1-b1); v = v*b2 + (1-b2)*g*g; denom = sqrt(v)/sqrt(bc2) + eps;
//   p += (-lr/bc1) * m / denom
__global__ void adam_kernel(float* p, const float* g, float* m, float* v, const uint8_t* live,
                            int64_t n, float w1, float b2, float one_m_b2, float bc2_sqrt,
                            float neg_step, float eps, float wd) {
#pragma clang fp contract(off)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (live && !live[i]) continue;
        float gi = g[i];
        const float pi = p[i];
        if (wd != 0.f) gi = gi + wd * pi;
        float mi = m[i];
        mi = mi + w1 * (gi - mi);  // lerp with weight < 0.5
        float vi = v[i] * b2;
        vi = vi + one_m_b2 * gi * gi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        m[i] = mi;
        v[i] = vi;
        p[i] = pi + neg_step * mi / denom;
    }
}

// Graph-replayable form: the 1-based step lives in device memory (incremented by
// step_inc_kernel earlier in the same stream), bias corrections are formed in double
// exactly like torch's host-side python floats, then rounded to f32. The hyperparameters
// arrive as doubles (torch's python floats): torch rounds 1-beta1 and 1-beta2 from the
// DOUBLE betas (e.g. 1-0.999 -> 0.001f, where 1-(double)0.999f is 0.00099998713f) and forms
// the bias corrections from them, so a float beta would leave this kernel self-consistent
// but 1.3e-5 (relative) off torch's second moment whenever the optimizer state comes from
// torch (a reference checkpoint, train_instance.py:320-328).
struct AdamCoef {
    float neg_step, bc2_sqrt, w1, b2f, one_m_b2, epsf, wdf;
};
ISG_DEV AdamCoef adam_coef(int32_t step, double lr, double b1, double b2, double eps, double wd) {
#pragma clang fp contract(off)
    const double st = (double)step;
    const double bc1 = 1.0 - pow(b1, st);
    const double bc2 = 1.0 - pow(b2, st);
    AdamCoef k;
    k.neg_step = (float)(-(lr / bc1));
    k.bc2_sqrt = (float)sqrt(bc2);
    k.w1 = (float)(1.0 - b1);
    k.b2f = (float)b2;
    k.one_m_b2 = (float)(1.0 - b2);
    k.epsf = (float)eps;
    k.wdf = (float)wd;
    return k;
}
ISG_DEV void adam_elem(float* p, float* m, float* v, int64_t i, float gi, const AdamCoef& k) {
#pragma clang fp contract(off)
    const float pi = p[i];
    if (k.wdf != 0.f) gi = gi + k.wdf * pi;
    float mi = m[i];
    mi = mi + k.w1 * (gi - mi);
    float vi = v[i] * k.b2f;
    vi = vi + k.one_m_b2 * gi * gi;
    const float denom = sqrtf(vi) / k.bc2_sqrt + k.epsf;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi + k.neg_step * mi / denom;
}

__global__ void adam_dev_kernel(float* p, const float* g, float* m, float* v, const uint8_t* live,
                                int64_t n, const int32_t* step, double lr, double b1, double b2,
                                double eps, double wd) {
    const AdamCoef k = adam_coef(*step, lr, b1, b2, eps, wd);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (live && !live[i]) continue;
        adam_elem(p, m, v, i, g[i], k);
    }
}

// The end of a world-1 training step in ONE launch (isg.h isg_step_tail): workgroups
// [0, nfold) fold the weight-gradient replicas into the flat gradient and apply Adam to each
// folded element; the next ngf fold the statistics-derived gradients (grad_final_item) and
// apply Adam to those; the last nbnu update the BatchNorm running statistics. Element
// arithmetic is sum_rep_n_kernel's, grad_final_kernel's and adam_dev_kernel's (the same
// device functions), so the result is bitwise that of the separate launches, which ran as
// 1 + 5 + 1 (+1 step counter) launches hopping between streams, plus 3 BN-update launches
// on the forward's critical path.
template <int NREP>
__global__ __launch_bounds__(kThreads) void step_tail_kernel(isg_step_tail_args a, int nfold) {
    const int b = blockIdx.x;
    const double* hp = a.hyper;
    const AdamCoef k = adam_coef(*a.step, hp[0], hp[1], hp[2], hp[3], hp[4]);
    if (b < nfold) {
        const int64_t i = (int64_t)b * kThreads + threadIdx.x;
        if (i >= a.n) return;
        const uint8_t o = a.owner[i];
        if (o & 2) return;  // written by a grad_final item below
        double v[NREP];
#pragma unroll
        for (int r = 0; r < NREP; ++r) v[r] = gld_d(a.rep, r * a.n + i);
        double s = v[0];
#pragma unroll
        for (int r = 1; r < NREP; ++r) s += v[r];
        const float g = (float)s;
        a.grad[i] = g;
        if (o & 1) adam_elem(a.param, a.exp_avg, a.exp_avg_sq, i, g, k);
        return;
    }
    if (b < nfold + a.ngf) {
        const isg_grad_final f = a.gf[b - nfold];
        grad_final_item(f, [&](float* d, float g) {
            *d = g;
            const int64_t i = d - a.grad;
            if (a.owner[i] & 1) adam_elem(a.param, a.exp_avg, a.exp_avg_sq, i, g, k);
        });
        return;
    }
    if (b < nfold + a.ngf + a.nbnu) bn_update_item(a.bnu[b - nfold - a.ngf]);
}

__global__ void step_inc_kernel(int32_t* c) { *c += 1; }

// One timestamp of the chip-global 100 MHz counter, accumulated (isg_stamp): sign * t added
// to buf[slot] and t folded into the max (buf[2]) / min (buf[3]) — vector atomics whose
// results are not waited for, so the launch is as short as a launch gets.
__global__ void stamp_kernel(unsigned long long* buf, int slot, int sign) {
    if (threadIdx.x != 0) return;
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    atomicAdd(buf + slot, sign < 0 ? 0ull - t : t);
    atomicMax(buf + 2, t);
    atomicMin(buf + 3, t);
}

__global__ void fill_f64_kernel(double* p, int64_t n, double v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// Fold the ISG_WREP weight-gradient replicas: dst[i] = sum_r src[r*stride + i] (fixed
// order), 4 elements per lane with 16-B loads where the layout allows.
// NREP replicas known at compile time: every replica's load of the thread's 2 elements is
// issued before the first add (the runtime-count loop waited one round trip per replica:
// 23 us for the 16 x 266k fp64 replicas of the bench step); summed in replica order
template <int NREP>
__global__ __launch_bounds__(kThreads) void sum_rep_n_kernel(float* __restrict__ dst,
                                                             const double* __restrict__ src, int64_t n,
                                                             int64_t stride) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    double v[NREP];
#pragma unroll
    for (int r = 0; r < NREP; ++r) v[r] = gld_d(src, r * stride + i);
    double a = v[0];
#pragma unroll
    for (int r = 1; r < NREP; ++r) a += v[r];
    gst(dst, i, (float)a);
}

__global__ __launch_bounds__(kThreads) void sum_rep_kernel(float* __restrict__ dst,
                                                            const double* __restrict__ src,
                                                            int64_t n, int nrep, int64_t stride) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    const int64_t i4 = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 4;
    if (i4 >= n) return;
    if (i4 + 4 <= n && (stride & 3) == 0 && ((uintptr_t)src & 31) == 0 && ((uintptr_t)dst & 15) == 0) {
        const f64x2* s0 = reinterpret_cast<const f64x2*>(src + i4);
        f64x2 a0 = s0[0], a1 = s0[1];
        for (int r = 1; r < nrep; ++r) {
            const f64x2* sr = reinterpret_cast<const f64x2*>(src + r * stride + i4);
            a0 += sr[0];
            a1 += sr[1];
        }
        *reinterpret_cast<f32x4*>(dst + i4) = f32x4{(float)a0[0], (float)a0[1], (float)a1[0], (float)a1[1]};
        return;
    }
    for (int64_t i = i4; i < n && i < i4 + 4; ++i) {
        double acc = src[i];
        for (int r = 1; r < nrep; ++r) acc += src[r * stride + i];
        dst[i] = (float)acc;
    }
}

unsigned grid_for(int64_t n, int cap = 2048) {
    int64_t b = (n + kThreads - 1) / kThreads;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (unsigned)b;
}

}  // namespace

extern "C" {

int32_t isg_tail_fwd(const isg_tail* t, isg_stream_t st) {
    if ((t->H & 1) || (t->W & 1) || t->nterm < 1 || t->nterm > 3)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "tail fwd: H, W must be even, 1..3 terms");
    for (int i = 0; i < t->nterm; ++i)
        if (isg_seg_res(t->term[i])) return isg_set_error(ISG_ERR_UNSUPPORTED, "tail fwd: residual term form");
    if (tail4_ok(*t, nullptr)) {
        dim3 grid4((unsigned)((((int64_t)t->H / 2) * (t->W / 4) + kThreads - 1) / kThreads), t->C, t->N);
        hipLaunchKernelGGL(tail_fwd4_kernel, grid4, dim3(kThreads), 0, st, *t);
        return isg_check_launch("tail_fwd4_kernel");
    }
    dim3 grid((unsigned)((((int64_t)t->H / 2) * (t->W / 2) + kThreads - 1) / kThreads), t->C, t->N);
    hipLaunchKernelGGL(tail_fwd_kernel, grid, dim3(kThreads), 0, st, *t);
    return isg_check_launch("tail_fwd_kernel");
}

int32_t isg_tail_bwd(const isg_tail_grad* t, isg_stream_t st) {
    const isg_tail& f = t->f;
    if ((f.H & 1) || (f.W & 1) || f.nterm < 1 || f.nterm > 3)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "tail bwd: H, W must be even, 1..3 terms");
    for (int i = 0; i < f.nterm; ++i)
        if (isg_seg_res(f.term[i])) return isg_set_error(ISG_ERR_UNSUPPORTED, "tail bwd: residual term form");
    // the kernels load every accumulating term's old value before any write:
    // two terms accumulating into one destination would lose one contribution
    for (int i = 0; i < f.nterm; ++i)
        for (int j = i + 1; j < f.nterm; ++j)
            if (t->dterm[i] && t->dterm[i] == t->dterm[j] && (t->dterm_accum[i] || t->dterm_accum[j]))
                return isg_set_error(ISG_ERR_INVALID, "tail bwd: terms %d and %d share a gradient destination", i, j);
    if (tail4_ok(f, t)) {
        dim3 grid4((unsigned)((((int64_t)f.H / 2) * (f.W / 4) + kThreads - 1) / kThreads), f.C, f.N);
        hipLaunchKernelGGL(tail_bwd4_kernel, grid4, dim3(kThreads), 0, st, *t);
        return isg_check_launch("tail_bwd4_kernel");
    }
    dim3 grid((unsigned)((((int64_t)f.H / 2) * (f.W / 2) + kThreads - 1) / kThreads), f.C, f.N);
    hipLaunchKernelGGL(tail_bwd_kernel, grid, dim3(kThreads), 0, st, *t);
    return isg_check_launch("tail_bwd_kernel");
}

int32_t isg_maxpool_fwd(const isg_vtensor* x, int32_t k, float* out, int64_t out_n_stride,
                        isg_stream_t st) {
    if (k < 1 || x->H % k || x->W % k) return isg_set_error(ISG_ERR_UNSUPPORTED, "maxpool: H,W %% k");
    if (isg_vt_res(x)) return isg_set_error(ISG_ERR_UNSUPPORTED, "maxpool: residual input form");
    int C = 0;
    for (int i = 0; i < x->nseg; ++i) C += x->s[i].C;
    PoolArgs a{};
    a.x = *x; a.k = k; a.out = out; a.out_n_stride = out_n_stride;
    dim3 grid((unsigned)(((int64_t)(x->H / k) * (x->W / k) + kThreads - 1) / kThreads), C, x->N);
    hipLaunchKernelGGL(maxpool_kernel<false>, grid, dim3(kThreads), 0, st, a);
    return isg_check_launch("maxpool_kernel<fwd>");
}

int32_t isg_maxpool_bwd(const isg_vtensor* x, int32_t k, const float* dout, int64_t dout_n_stride,
                        const isg_sinks* dx, isg_stream_t st) {
    if (k < 1 || x->H % k || x->W % k) return isg_set_error(ISG_ERR_UNSUPPORTED, "maxpool: H,W %% k");
    if (isg_vt_res(x) || isg_sinks_res(dx)) return isg_set_error(ISG_ERR_UNSUPPORTED, "maxpool: residual form");
    int C = 0;
    for (int i = 0; i < x->nseg; ++i) C += x->s[i].C;
    for (int i = 0; i < dx->nsink; ++i)
        if (dx->s[i].mode == ISG_SINK_ACTBWD)
            return isg_set_error(ISG_ERR_UNSUPPORTED, "maxpool bwd: ACTBWD sink");
    PoolArgs a{};
    a.x = *x; a.k = k; a.dout = dout; a.dout_n_stride = dout_n_stride; a.dx = *dx;
    dim3 grid((unsigned)(((int64_t)(x->H / k) * (x->W / k) + kThreads - 1) / kThreads), C, x->N);
    hipLaunchKernelGGL(maxpool_kernel<true>, grid, dim3(kThreads), 0, st, a);
    return isg_check_launch("maxpool_kernel<bwd>");
}

int32_t isg_bn_update_running(const isg_bn_update* items, int32_t nitems, isg_stream_t st) {
    for (int b = 0; b < nitems; b += ISG_LIST_CHUNK) {
        const int n = nitems - b < ISG_LIST_CHUNK ? nitems - b : ISG_LIST_CHUNK;
        BnUpdateList l;
        memcpy(l.it, items + b, sizeof(isg_bn_update) * n);
        hipLaunchKernelGGL(bn_update_kernel, dim3(n), dim3(128), 0, st, l, n);
        if (int32_t e = isg_check_launch("bn_update_kernel")) return e;
    }
    return 0;
}

int32_t isg_bn_finalize(const isg_bn* items, int32_t nitems, int32_t bwd, isg_stream_t st) {
    for (int i = 0; i < nitems; ++i)
        if (!items[i].coef || !items[i].stats || (((uintptr_t)items[i].coef) & 15))
            return isg_set_error(ISG_ERR_INVALID, "bn_finalize: item %d needs stats and a 16-B aligned coef", i);
    if (nitems == 1) {
        hipLaunchKernelGGL(bn_finalize1_kernel, dim3(1), dim3(items[0].C > 64 ? 128 : 64), 0, st,
                           items[0], bwd ? 1 : 0);
        return isg_check_launch("bn_finalize1_kernel");
    }
    for (int b = 0; b < nitems; b += ISG_LIST_CHUNK) {
        const int n = nitems - b < ISG_LIST_CHUNK ? nitems - b : ISG_LIST_CHUNK;
        BnFinalList l;
        memcpy(l.it, items + b, sizeof(isg_bn) * n);
        hipLaunchKernelGGL(bn_finalize_kernel, dim3(n), dim3(128), 0, st, l, n, bwd ? 1 : 0);
        if (int32_t e = isg_check_launch("bn_finalize_kernel")) return e;
    }
    return 0;
}

int32_t isg_grad_finalize(const isg_grad_final* items, int32_t nitems, isg_stream_t st) {
    for (int b = 0; b < nitems; b += ISG_LIST_CHUNK) {
        const int n = nitems - b < ISG_LIST_CHUNK ? nitems - b : ISG_LIST_CHUNK;
        GradFinalList l;
        memcpy(l.it, items + b, sizeof(isg_grad_final) * n);
        hipLaunchKernelGGL(grad_final_kernel, dim3(n), dim3(128), 0, st, l, n);
        if (int32_t e = isg_check_launch("grad_final_kernel")) return e;
    }
    return 0;
}

int32_t isg_bce_sigmoid(const float* logits, const float* target, int64_t n, double* loss_acc,
                        float* dlogits, float grad_scale, isg_stream_t st) {
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (n % 4 == 0 && n / 4 < ((int64_t)1 << 31) && al16(logits) && al16(target) && (!dlogits || al16(dlogits))) {
        const int64_t q = n / 4;
        hipLaunchKernelGGL(bce4_kernel, dim3((unsigned)((q + kThreads * kBceQ - 1) / (kThreads * kBceQ))),
                           dim3(kThreads), 0, st,
                           logits, target, q, loss_acc, dlogits, grad_scale);
        return isg_check_launch("bce4_kernel");
    }
    hipLaunchKernelGGL(bce_kernel, dim3(grid_for(n, 1024)), dim3(kThreads), 0, st, logits, target, n,
                       loss_acc, dlogits, grad_scale);
    return isg_check_launch("bce_kernel");
}

int32_t isg_sigmoid_fwd(const float* x, float* y, int64_t n, isg_stream_t st) {
    hipLaunchKernelGGL(sigmoid_fwd_kernel, dim3(grid_for(n)), dim3(kThreads), 0, st, x, y, n);
    return isg_check_launch("sigmoid_fwd_kernel");
}

int32_t isg_sigmoid_bwd(const float* y, const float* dy, float* dx, int64_t n, isg_stream_t st) {
    hipLaunchKernelGGL(sigmoid_bwd_kernel, dim3(grid_for(n)), dim3(kThreads), 0, st, y, dy, dx, n);
    return isg_check_launch("sigmoid_bwd_kernel");
}

int32_t isg_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                 const uint8_t* live, int64_t n, int32_t step, double lr, double beta1, double beta2,
                 double eps, double weight_decay, isg_stream_t st) {
    if (step < 1) return isg_set_error(ISG_ERR_INVALID, "adam: step must be >= 1");
    // scalar math in double exactly like torch's python-side bias corrections
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    const float neg_step = (float)(-(lr / bc1));
    const float bc2_sqrt = (float)std::sqrt(bc2);
    hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(kThreads), 0, st, param, grad, exp_avg,
                       exp_avg_sq, live, n, (float)(1.0 - beta1), (float)beta2,
                       (float)(1.0 - beta2), bc2_sqrt, neg_step, (float)eps, (float)weight_decay);
    return isg_check_launch("adam_kernel");
}

int32_t isg_adam_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                     const uint8_t* live, int64_t n, int32_t* step, double lr, double beta1,
                     double beta2, double eps, double weight_decay, isg_stream_t st) {
    hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
    hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_for(n)), dim3(kThreads), 0, st, param, grad,
                       exp_avg, exp_avg_sq, live, n, step, lr, beta1, beta2, eps, weight_decay);
    return isg_check_launch("adam_dev_kernel");
}

int32_t isg_step_tail(const isg_step_tail_args* a, isg_stream_t st) {
    if (!a || !a->grad || !a->rep || !a->param || !a->exp_avg || !a->exp_avg_sq || !a->owner ||
        !a->step || !a->hyper || a->n < 0 || (a->ngf > 0 && !a->gf) || (a->nbnu > 0 && !a->bnu) ||
        a->ngf < 0 || a->nbnu < 0)
        return isg_set_error(ISG_ERR_INVALID, "step tail: NULL or negative argument");
    if (a->nrep != 16 && a->nrep != 8 && a->nrep != 4)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "step tail: %d replicas (4, 8 or 16)", a->nrep);
    const int64_t nfold = (a->n + kThreads - 1) / kThreads;
    const int64_t grid = nfold + a->ngf + a->nbnu;
    if (grid < 1) return ISG_OK;
    if (grid >= ((int64_t)1 << 31)) return isg_set_error(ISG_ERR_UNSUPPORTED, "step tail: %lld elements", (long long)a->n);
    if (a->nrep == 16) hipLaunchKernelGGL(step_tail_kernel<16>, dim3((unsigned)grid), dim3(kThreads), 0, st, *a, (int)nfold);
    else if (a->nrep == 8) hipLaunchKernelGGL(step_tail_kernel<8>, dim3((unsigned)grid), dim3(kThreads), 0, st, *a, (int)nfold);
    else hipLaunchKernelGGL(step_tail_kernel<4>, dim3((unsigned)grid), dim3(kThreads), 0, st, *a, (int)nfold);
    return isg_check_launch("step_tail_kernel");
}

int32_t isg_step_inc(int32_t* step, isg_stream_t st) {
    if (!step) return isg_set_error(ISG_ERR_INVALID, "step inc: NULL counter");
    hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
    return isg_check_launch("step_inc_kernel");
}

int32_t isg_sum_replicas(float* dst, const double* src, int64_t n, int32_t nrep, int64_t stride,
                         isg_stream_t st) {
    if (n <= 0) return 0;
    if (!dst || !src || nrep < 1 || (nrep > 1 && stride < n))
        return isg_set_error(ISG_ERR_INVALID, "sum_replicas: bad arguments");
    if (nrep == 16 || nrep == 8 || nrep == 4) {
        const int64_t b1 = (n + kThreads - 1) / kThreads;
        if (nrep == 16) hipLaunchKernelGGL(sum_rep_n_kernel<16>, dim3((unsigned)b1), dim3(kThreads), 0, st, dst, src, n, stride);
        else if (nrep == 8) hipLaunchKernelGGL(sum_rep_n_kernel<8>, dim3((unsigned)b1), dim3(kThreads), 0, st, dst, src, n, stride);
        else hipLaunchKernelGGL(sum_rep_n_kernel<4>, dim3((unsigned)b1), dim3(kThreads), 0, st, dst, src, n, stride);
        return isg_check_launch("sum_rep_n_kernel");
    }
    const int64_t blocks = ((n + 3) / 4 + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(sum_rep_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, st, dst, src, n,
                       nrep, stride);
    return isg_check_launch("sum_rep_kernel");
}

int32_t isg_stamp(uint64_t* buf, int32_t slot, int32_t sign, isg_stream_t st) {
    if (!buf || slot < 0 || slot > 1) return isg_set_error(ISG_ERR_INVALID, "stamp: bad arguments");
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, st, (unsigned long long*)buf, slot, sign);
    return isg_check_launch("stamp_kernel");
}

int32_t isg_fill_f64(double* p, int64_t n, double v, isg_stream_t st) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(fill_f64_kernel, dim3(grid_for(n)), dim3(kThreads), 0, st, p, n, v);
    return isg_check_launch("fill_f64_kernel");
}

}  // extern "C"
