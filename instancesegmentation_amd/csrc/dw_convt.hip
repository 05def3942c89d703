// Depthwise convolutions and sub-pixel transposed convolutions (VALU, gfx950).
//
// Depthwise: the dilated 3x3 (segment.py:64-65, 127-128, 167, 183, 226) and the
// 5x1 / 1x5 pair (segment.py:91-92, 96-97). AI is 2.5-4.5 flop/B (SURVEY.md
// appendix), so these are plain HBM-streaming kernels: one output pixel per lane,
// the channel's BN/activation coefficients held in registers, taps served by L1.
//
// Transposed conv (kernel = 2*stride, pad = stride/2; segment.py:305-306 k4s2p1 and
// :435-436 k8s4p2): every output pixel receives exactly 2x2 taps, so a lane owns one
// input-resolution cell and produces its full s x s output block for every output
// channel from the cell's 3x3 input neighbourhood. Weight indices are compile-time
// per (phase, tap) and wave-uniform, so they come from the scalar cache; the s x s
// block is written as s vectors of s floats (coalesced across lanes).
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

// single-segment virtual load with coefficients in registers
ISG_DEV float seg_load(const isg_vseg& sg, const ChanCoef& k, int n, int c, int64_t hw,
                       int64_t pix) {
    const float x = sg.p[(int64_t)n * sg.n_stride + (int64_t)c * hw + pix];
    if (sg.xform == ISG_XF_PLAIN) return x;
    if (sg.xform == ISG_XF_BN_FWD) return apply_act((x - k.c0) * k.c1 + k.c2, sg.act, k.c3);
    const float y = sg.y[(int64_t)n * sg.y_n_stride + (int64_t)c * hw + pix];
    return k.c0 * x + k.c1 * (y - k.c2) + k.c3;
}

// raw value of one source tap (x, and the saved y of a BN_BWD segment) -> transformed value
ISG_DEV float seg_xform(const isg_vseg& sg, const ChanCoef& k, float x, float y) {
    if (sg.xform == ISG_XF_PLAIN) return x;
    if (sg.xform == ISG_XF_BN_FWD) return apply_act((x - k.c0) * k.c1 + k.c2, sg.act, k.c3);
    return k.c0 * x + k.c1 * (y - k.c2) + k.c3;
}

// Block reduction of up to 3 floats; thread 0 returns the block totals.
template <int NV>
ISG_DEV void block_reduce(float (&v)[NV], float* sh /* [NV][4] */) {
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

// Single-channel sink application with the BN/act coefficients of that channel.
struct Sink1 {
    float mean, scale, beta, slope;
};

ISG_DEV Sink1 sink1_coef(const isg_sink& k, int cl) {
    Sink1 s = {0.f, 1.f, 0.f, 0.f};
    if (k.mode == ISG_SINK_ACTBWD) {
        if (k.bn.stats || !k.bn.train) {
            ChanCoef f = fwd_coef(k.bn, k.slope, cl);
            s.mean = f.c0; s.scale = f.c1; s.beta = f.c2;
        }
        s.slope = k.slope ? k.slope[cl] : 0.f;
    }
    return s;
}

ISG_DEV void sink1_apply(const isg_sink& k, const Sink1& f, int cl, int n, int64_t hw,
                         int64_t pix, float v, float (&red)[3]) {
    if (k.mode == ISG_SINK_NONE) return;
    const int64_t off = (int64_t)n * k.n_stride + (int64_t)cl * hw + pix;
    if (k.mode == ISG_SINK_STORE) {
        if (k.bias) v += k.bias[cl];
        k.p[off] = v;
        red[0] += v;
        red[1] += v * v;
    } else if (k.mode == ISG_SINK_ACCUM) {
        k.p[off] += v;
        red[0] += v;
        red[1] += v * v;
    } else {
        const float y = k.y[(int64_t)n * k.y_n_stride + (int64_t)cl * hw + pix];
        const float z = (y - f.mean) * f.scale + f.beta;
        float g = v;
        if (k.act == ISG_ACT_RELU) {
            g = z > 0.f ? v : 0.f;
        } else if (k.act == ISG_ACT_PRELU) {
            g = z > 0.f ? v : v * f.slope;
            red[2] += z > 0.f ? 0.f : z * v;
        }
        k.p[off] = g;
        red[0] += g;
        red[1] += g * (y - f.mean);
    }
}

ISG_DEV void sink1_flush(const isg_sink& k, int cl, const float (&red)[3]) {
    if (k.mode == ISG_SINK_STORE || k.mode == ISG_SINK_ACCUM) {
        if (k.stats) {
            double* sp = rep_ptr(k.stats, 4 * k.C);
            atomicAdd(&sp[cl], (double)red[0]);
            atomicAdd(&sp[k.C + cl], (double)red[1]);
        }
    } else if (k.mode == ISG_SINK_ACTBWD) {
        if (k.bn.stats) {
            double* sp = rep_ptr(k.bn.stats, 4 * k.C);
            atomicAdd(&sp[2 * k.C + cl], (double)red[0]);
            atomicAdd(&sp[3 * k.C + cl], (double)red[1]);
        }
        if (k.slope_grad && k.act == ISG_ACT_PRELU)
            atomicAdd(&rep_ptr(k.slope_grad, k.C)[cl], (double)red[2]);
    }
}

ISG_DEV bool sink1_needs_red(const isg_sink& k) {
    return ((k.mode == ISG_SINK_STORE || k.mode == ISG_SINK_ACCUM) && k.stats) ||
           k.mode == ISG_SINK_ACTBWD;
}

struct DwArgs {
    isg_vseg x;      // fwd: input; dgrad: dy
    isg_sink out;
    const float* w;  // [C][KH][KW]
    int N, C, H, W, OH, OW, KH, KW, PH, PW, DH, DW;
};

// forward (dgrad=false): out[c,oy,ox] = sum_t w[c,t] * x[c, oy-PH+kh*DH, ox-PW+kw*DW]
// dgrad (dgrad=true)   : dx[c,iy,ix] = sum_t w[c,t] * dy[c, iy+PH-kh*DH, ix+PW-kw*DW]
// KH_ x KW_: the tap grid at compile time (3x3, 5x1, 1x5 in this network), 0 = runtime.
// The taps' raw values are loaded before the channel's coefficients are evaluated (from
// the BatchNorm statistics when no finalisation launch wrote them), so the two round
// trips overlap; out-of-range taps stay unloaded (a branch-free form with clamped loads
// measured slower, round 2).
template <bool DGRAD, int KH_, int KW_>
__global__ __launch_bounds__(kThreads) void dw_kernel(DwArgs a) {
    __shared__ float sh[12];
    const int c = blockIdx.y, n = blockIdx.z;
    // source plane = x (fwd) or dy (dgrad); destination plane = out (fwd) or dx
    const int SH_ = DGRAD ? a.OH : a.H, SW_ = DGRAD ? a.OW : a.W;
    const int DH_ = DGRAD ? a.H : a.OH, DW_ = DGRAD ? a.W : a.OW;
    const int64_t dhw = (int64_t)DH_ * DW_, shw = (int64_t)SH_ * SW_;
    const int64_t pix = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    float red[3] = {0.f, 0.f, 0.f};
    if constexpr (KH_ > 0) {
        constexpr int KK = KH_ * KW_;
        const bool live = pix < dhw;
        const int oy = live ? (int)(pix / DW_) : 0, ox = live ? (int)(pix - (int64_t)oy * DW_) : 0;
        const float* xp = a.x.p + (int64_t)n * a.x.n_stride + (int64_t)c * shw;
        const bool bwd = a.x.xform == ISG_XF_BN_BWD;
        const float* yp = bwd ? a.x.y + (int64_t)n * a.x.y_n_stride + (int64_t)c * shw : xp;
        float xr[KK], yr[KK];
        bool ok[KK];
#pragma unroll
        for (int kh = 0; kh < KH_; ++kh)
#pragma unroll
            for (int kw = 0; kw < KW_; ++kw) {
                const int t = kh * KW_ + kw;
                const int iy = DGRAD ? oy + a.PH - kh * a.DH : oy - a.PH + kh * a.DH;
                const int ix = DGRAD ? ox + a.PW - kw * a.DW : ox - a.PW + kw * a.DW;
                ok[t] = live && iy >= 0 && iy < SH_ && ix >= 0 && ix < SW_;
                xr[t] = yr[t] = 0.f;
                if (ok[t]) {
                    xr[t] = xp[(int64_t)iy * SW_ + ix];
                    if (bwd) yr[t] = yp[(int64_t)iy * SW_ + ix];
                }
            }
        const ChanCoef k = seg_coef(a.x, c);
        const Sink1 f = sink1_coef(a.out, c);
        if (live) {
            const float* wc = a.w + c * KK;
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < KK; ++t)
                if (ok[t]) acc += wc[t] * seg_xform(a.x, k, xr[t], yr[t]);
            sink1_apply(a.out, f, c, n, dhw, pix, acc, red);
        }
    } else {
        const ChanCoef k = seg_coef(a.x, c);
        const Sink1 f = sink1_coef(a.out, c);
        if (pix < dhw) {
            const int oy = (int)(pix / DW_), ox = (int)(pix - (int64_t)oy * DW_);
            const float* wc = a.w + c * a.KH * a.KW;
            float acc = 0.f;
            for (int kh = 0; kh < a.KH; ++kh) {
                const int iy = DGRAD ? oy + a.PH - kh * a.DH : oy - a.PH + kh * a.DH;
                if (iy < 0 || iy >= SH_) continue;
                for (int kw = 0; kw < a.KW; ++kw) {
                    const int ix = DGRAD ? ox + a.PW - kw * a.DW : ox - a.PW + kw * a.DW;
                    if (ix < 0 || ix >= SW_) continue;
                    acc += wc[kh * a.KW + kw] * seg_load(a.x, k, n, c, shw, (int64_t)iy * SW_ + ix);
                }
            }
            sink1_apply(a.out, f, c, n, dhw, pix, acc, red);
        }
    }
    if (sink1_needs_red(a.out)) {
        block_reduce<3>(red, sh);
        if (threadIdx.x == 0) sink1_flush(a.out, c, red);
    }
}

// ---- LDS-tiled depthwise (round 3) -----------------------------------------------------
// One workgroup = one (image, channel) tile of 16 x 64 outputs; a thread owns 4 adjacent
// outputs of one row. The input region (tile + the taps' halo) is staged ONCE into LDS
// with the producer's BatchNorm / activation (or BatchNorm backward) applied once per
// element — the per-pixel kernel above transformed every input 9 times and issued 9
// (18 for BatchNorm backward) 4-B loads per output. Outputs leave as 16-B stores through
// the sink. Same-size convolutions only (stride 1, OH == H, OW == W, W % 4 == 0).
constexpr int kDtY = 16, kDtX = 64;
constexpr int kDtMaxR = kDtY + 2 * 4 * 2, kDtMaxC = kDtX + 2 * 4 * 2;  // halo <= 8 per side

template <bool DGRAD, int KH_, int KW_>
__global__ __launch_bounds__(kThreads) void dw_tile_kernel(DwArgs a) {
    __shared__ float Ts[kDtMaxR * kDtMaxC];
    __shared__ float sh[12];
    const int c = blockIdx.z % a.C, n = blockIdx.z / a.C;
    const int H = a.H, W = a.W;  // source == destination size
    const int oy0 = blockIdx.y * kDtY, ox0 = blockIdx.x * kDtX;
    // tap offsets relative to the output pixel: fwd +(k*D - P), dgrad +(P - k*D); the region
    // starts at the smallest
    const int ay0 = DGRAD ? a.PH - (KH_ - 1) * a.DH : -a.PH;
    const int ax0 = DGRAD ? a.PW - (KW_ - 1) * a.DW : -a.PW;
    const int RH = kDtY + (KH_ - 1) * a.DH, RW = kDtX + (KW_ - 1) * a.DW;
    const int64_t hw = (int64_t)H * W;
    const isg_vseg& sg = a.x;
    const float* xp = sg.p + (int64_t)n * sg.n_stride + (int64_t)c * hw;
    const bool bwd = sg.xform == ISG_XF_BN_BWD;
    const float* yp = bwd ? sg.y + (int64_t)n * sg.y_n_stride + (int64_t)c * hw : xp;
    // ---- stage: every element's raw load in flight, then the coefficients, then LDS
    constexpr int kU = (kDtMaxR * kDtMaxC + kThreads - 1) / kThreads;
    float xr[kU], yr[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        xr[u] = yr[u] = 0.f;
        if (u * kThreads >= RH * RW) continue;  // workgroup-uniform
        const int e = threadIdx.x + u * kThreads;
        const int rr = e / RW, cc = e - rr * RW;
        const int iy = oy0 + ay0 + rr, ix = ox0 + ax0 + cc;
        const bool ok = rr < RH && iy >= 0 && iy < H && ix >= 0 && ix < W;
        const int64_t o = ok ? (int64_t)iy * W + ix : 0;
        xr[u] = xp[o];
        yr[u] = bwd ? yp[o] : 0.f;
    }
    const ChanCoef k = seg_coef(sg, c);
    const Sink1 f = sink1_coef(a.out, c);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        if (u * kThreads >= RH * RW) continue;
        const int e = threadIdx.x + u * kThreads;
        const int rr = e / RW, cc = e - rr * RW;
        const int iy = oy0 + ay0 + rr, ix = ox0 + ax0 + cc;
        const bool ok = rr < RH && iy >= 0 && iy < H && ix >= 0 && ix < W;
        if (rr < RH) Ts[rr * kDtMaxC + cc] = ok ? seg_xform(sg, k, xr[u], yr[u]) : 0.f;  // zero padding after the transform
    }
    __syncthreads();
    // ---- compute: thread -> row ty, 4 outputs from column 4 * tq
    const int ty = threadIdx.x >> 4, tq = threadIdx.x & 15;
    const float* wc = a.w + c * KH_ * KW_;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < KH_; ++kh) {
        const int rrow = ty + (DGRAD ? (KH_ - 1 - kh) : kh) * a.DH;
#pragma unroll
        for (int kw = 0; kw < KW_; ++kw) {
            const float wv = wc[kh * KW_ + kw];
            const float* rp = Ts + rrow * kDtMaxC + 4 * tq + (DGRAD ? (KW_ - 1 - kw) : kw) * a.DW;
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] += wv * rp[j];
        }
    }
    // ---- sink: 16-B accesses, 4 outputs
    float red[3] = {0.f, 0.f, 0.f};
    const int oy = oy0 + ty, ox = ox0 + 4 * tq;
    if (oy < H && ox < W) {
        const isg_sink& o = a.out;
        const int64_t off = (int64_t)n * o.n_stride + (int64_t)c * hw + (int64_t)oy * W + ox;
        typedef f32x4 __attribute__((address_space(1)))* g4p;
        if (o.mode == ISG_SINK_STORE || o.mode == ISG_SINK_ACCUM) {
            f32x4 v = {acc[0], acc[1], acc[2], acc[3]};
            if (o.mode == ISG_SINK_STORE && o.bias) v += o.bias[c];
            if (o.mode == ISG_SINK_ACCUM) v += *(g4p)((gfloat_p)o.p + off);
            else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    red[0] += v[j];
                    red[1] += v[j] * v[j];
                }
            }
            if (o.mode == ISG_SINK_ACCUM) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    red[0] += acc[j];
                    red[1] += acc[j] * acc[j];
                }
            }
            *(g4p)((gfloat_p)o.p + off) = v;
        } else if (o.mode == ISG_SINK_ACTBWD) {
            const f32x4 y4 = *(const f32x4 __attribute__((address_space(1)))*)((gcfloat_p)o.y +
                              (int64_t)n * o.y_n_stride + (int64_t)c * hw + (int64_t)oy * W + ox);
            f32x4 g4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float z = (y4[j] - f.mean) * f.scale + f.beta;
                float gv = acc[j];
                if (o.act == ISG_ACT_RELU) {
                    gv = z > 0.f ? acc[j] : 0.f;
                } else if (o.act == ISG_ACT_PRELU) {
                    gv = z > 0.f ? acc[j] : acc[j] * f.slope;
                    red[2] += z > 0.f ? 0.f : z * acc[j];
                }
                g4[j] = gv;
                red[0] += gv;
                red[1] += gv * (y4[j] - f.mean);
            }
            *(g4p)((gfloat_p)o.p + off) = g4;
        }
    }
    if (sink1_needs_red(a.out)) {
        block_reduce<3>(red, sh);
        if (threadIdx.x == 0) sink1_flush(a.out, c, red);
    }
}

// 1: launched, 0: shape not for the tiled kernel
template <bool DGRAD>
int dw_tile_try(const isg_conv_geom* g, const DwArgs& a, hipStream_t st) {
    if (g->SH != 1 || g->SW != 1 || g->OH != g->H || g->OW != g->W || g->W % 4)
        return 0;
    const isg_sink& o = a.out;
    if (o.mode == ISG_SINK_NONE || ((uintptr_t)o.p & 15) || o.n_stride % 4 ||
        (o.mode == ISG_SINK_ACTBWD && (((uintptr_t)o.y & 15) || o.y_n_stride % 4)))
        return 0;
    if ((g->KH - 1) * g->DH > 16 || (g->KW - 1) * g->DW > 16) return 0;
    const dim3 grid((unsigned)((g->W + kDtX - 1) / kDtX), (unsigned)((g->H + kDtY - 1) / kDtY),
                    (unsigned)(g->Ci * g->N));
    if (g->KH == 3 && g->KW == 3) hipLaunchKernelGGL((dw_tile_kernel<DGRAD, 3, 3>), grid, dim3(kThreads), 0, st, a);
    else if (g->KH == 5 && g->KW == 1) hipLaunchKernelGGL((dw_tile_kernel<DGRAD, 5, 1>), grid, dim3(kThreads), 0, st, a);
    else if (g->KH == 1 && g->KW == 5) hipLaunchKernelGGL((dw_tile_kernel<DGRAD, 1, 5>), grid, dim3(kThreads), 0, st, a);
    else return 0;
    return 1;
}

template <bool DGRAD>
void dw_launch(const isg_conv_geom* g, const DwArgs& a, dim3 grid, hipStream_t st) {
    if (g->KH == 3 && g->KW == 3) hipLaunchKernelGGL((dw_kernel<DGRAD, 3, 3>), grid, dim3(kThreads), 0, st, a);
    else if (g->KH == 5 && g->KW == 1) hipLaunchKernelGGL((dw_kernel<DGRAD, 5, 1>), grid, dim3(kThreads), 0, st, a);
    else if (g->KH == 1 && g->KW == 5) hipLaunchKernelGGL((dw_kernel<DGRAD, 1, 5>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((dw_kernel<DGRAD, 0, 0>), grid, dim3(kThreads), 0, st, a);
}

// weight gradient: dw[c,t] += sum_p dy[c,p] * x[c, p + tap_t]; dbias[c] += sum_p dy.
// grid (splits, C): a block reduces ~kDwPix pixels of one channel, each lane kDwU pixels
// per pass with all their loads issued together, then adds its partials into one of
// nrep replicas of dw (include/isg.h ISG_WREP) so few atomics meet on one address.
constexpr int kMaxTaps = 9;
constexpr int kDwU = 4;
constexpr int kDwPix = kThreads * kDwU;
struct DwWgArgs {
    isg_vseg dy, x;
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int nrep;
    int N, C, H, W, OH, OW, KH, KW, PH, PW, DH, DW;
    int64_t pix_per_block;
};

__global__ __launch_bounds__(kThreads) void dw_wgrad_kernel(DwWgArgs a) {
    __shared__ float sh[(kMaxTaps + 1) * 4];
    const int c = blockIdx.y;
    const ChanCoef kd = seg_coef(a.dy, c);
    const ChanCoef kx = seg_coef(a.x, c);
    const int64_t ohw = (int64_t)a.OH * a.OW, xhw = (int64_t)a.H * a.W;
    const int64_t P = (int64_t)a.N * ohw;
    const int64_t pb = (int64_t)blockIdx.x * a.pix_per_block;
    int64_t pe = pb + a.pix_per_block;
    if (pe > P) pe = P;
    const int KK = a.KH * a.KW;
    int tdy[kMaxTaps], tdx[kMaxTaps];
#pragma unroll
    for (int t = 0; t < kMaxTaps; ++t) {
        const int kh = t < KK ? t / a.KW : 0, kw = t < KK ? t - kh * a.KW : 0;
        tdy[t] = kh * a.DH - a.PH;
        tdx[t] = kw * a.DW - a.PW;
    }
    float acc[kMaxTaps + 1];
#pragma unroll
    for (int t = 0; t <= kMaxTaps; ++t) acc[t] = 0.f;
    for (int64_t p0 = pb + threadIdx.x; p0 < pe; p0 += kDwPix) {
        float d[kDwU], xv[kDwU][kMaxTaps];
#pragma unroll
        for (int u = 0; u < kDwU; ++u) {
            const int64_t p = p0 + (int64_t)u * kThreads;
            const bool pv = p < pe;
            const int n = pv ? (int)(p / ohw) : 0;
            const int64_t pix = pv ? p - (int64_t)n * ohw : 0;
            const int oy = (int)(pix / a.OW), ox = (int)(pix - (int64_t)oy * a.OW);
            d[u] = pv ? seg_load(a.dy, kd, n, c, ohw, pix) : 0.f;
#pragma unroll
            for (int t = 0; t < kMaxTaps; ++t) {
                const int iy = oy + tdy[t], ix = ox + tdx[t];
                xv[u][t] = (pv && t < KK && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
                               ? seg_load(a.x, kx, n, c, xhw, (int64_t)iy * a.W + ix)
                               : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < kDwU; ++u) {
            acc[kMaxTaps] += d[u];
#pragma unroll
            for (int t = 0; t < kMaxTaps; ++t) acc[t] = fmaf(d[u], xv[u][t], acc[t]);
        }
    }
    block_reduce<kMaxTaps + 1>(acc, sh);
    if (threadIdx.x == 0) {
        const int64_t ro = (int64_t)((blockIdx.x + 7u * blockIdx.y) % (unsigned)a.nrep) * a.rep_stride;
        for (int t = 0; t < KK; ++t) atomicAdd(&a.dw[ro + c * KK + t], acc[t]);
        if (a.dbias) atomicAdd(&a.dbias[ro + c], acc[kMaxTaps]);
    }
}

// LDS-tiled depthwise weight gradient (round 3): one workgroup per (image, channel) 16 x 64
// tile of dy; the x region under the taps (tile + halo) staged ONCE into LDS with its
// BatchNorm / activation applied once per element, dy read as 16-B quads (BatchNorm backward
// rebuilt in registers); each lane accumulates its 4 pixels' products per tap, reduced over
// the workgroup and added into this workgroup's weight-gradient replica. Same-size layers,
// W % 4 == 0 (dw_wgrad_kernel otherwise).
template <int KH_, int KW_>
ISG_DEV void dw_wgrad_tile_body(const DwWgArgs& a, const unsigned bx, const unsigned by,
                                const unsigned bz) {
    constexpr int KK = KH_ * KW_;
    __shared__ float Ts[kDtMaxR * kDtMaxC];
    __shared__ float sh[(KK + 1) * 4];
    const int c = bz % a.C, n = bz / a.C;
    const int H = a.H, W = a.W;
    const int oy0 = by * kDtY, ox0 = bx * kDtX;
    const int RH = kDtY + (KH_ - 1) * a.DH, RW = kDtX + (KW_ - 1) * a.DW;
    const int64_t hw = (int64_t)H * W;
    const isg_vseg& sx = a.x;
    const isg_vseg& sd = a.dy;
    const float* xp = sx.p + (int64_t)n * sx.n_stride + (int64_t)c * hw;
    // this lane's 4 dy pixels (row ty, columns 4 tq ..)
    const int ty = threadIdx.x >> 4, tq = threadIdx.x & 15;
    const int oy = oy0 + ty, ox = ox0 + 4 * tq;
    const bool dv = oy < H && ox < W;
    const int64_t dpix = dv ? (int64_t)oy * W + ox : 0;
    typedef const f32x4 __attribute__((address_space(1)))* gc4p;
    const f32x4 d4 = *(gc4p)((gcfloat_p)sd.p + (int64_t)n * sd.n_stride + (int64_t)c * hw + dpix);
    const bool dbwd = sd.xform == ISG_XF_BN_BWD;
    const f32x4 y4 = dbwd ? *(gc4p)((gcfloat_p)sd.y + (int64_t)n * sd.y_n_stride + (int64_t)c * hw + dpix)
                          : f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int kU = (kDtMaxR * kDtMaxC + kThreads - 1) / kThreads;
    float xr[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        xr[u] = 0.f;
        if (u * kThreads >= RH * RW) continue;  // workgroup-uniform
        const int e = threadIdx.x + u * kThreads;
        const int rr = e / RW, cc = e - rr * RW;
        const int iy = oy0 - a.PH + rr, ix = ox0 - a.PW + cc;
        const bool ok = rr < RH && iy >= 0 && iy < H && ix >= 0 && ix < W;
        xr[u] = xp[ok ? (int64_t)iy * W + ix : 0];
    }
    const ChanCoef kx = seg_coef(sx, c);
    const ChanCoef kd = seg_coef(sd, c);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        if (u * kThreads >= RH * RW) continue;
        const int e = threadIdx.x + u * kThreads;
        const int rr = e / RW, cc = e - rr * RW;
        const int iy = oy0 - a.PH + rr, ix = ox0 - a.PW + cc;
        const bool ok = rr < RH && iy >= 0 && iy < H && ix >= 0 && ix < W;
        if (rr < RH) Ts[rr * kDtMaxC + cc] = ok ? seg_xform(sx, kx, xr[u], 0.f) : 0.f;
    }
    float dyv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) dyv[j] = dv ? seg_xform(sd, kd, d4[j], y4[j]) : 0.f;
    __syncthreads();
    float acc[KK + 1];
    acc[KK] = (dyv[0] + dyv[1]) + (dyv[2] + dyv[3]);
#pragma unroll
    for (int kh = 0; kh < KH_; ++kh)
#pragma unroll
        for (int kw = 0; kw < KW_; ++kw) {
            const float* rp = Ts + (ty + kh * a.DH) * kDtMaxC + 4 * tq + kw * a.DW;
            float v = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) v = fmaf(dyv[j], rp[j], v);
            acc[kh * KW_ + kw] = v;
        }
    block_reduce<KK + 1>(acc, sh);
    if (threadIdx.x == 0) {
        const int64_t ro = (int64_t)((bx + 3u * by + 7u * bz) % (unsigned)a.nrep) * a.rep_stride;
        for (int t = 0; t < KK; ++t) atomicAdd(&a.dw[ro + c * KK + t], acc[t]);
        if (a.dbias) atomicAdd(&a.dbias[ro + c], acc[KK]);
    }
}

template <int KH_, int KW_>
__global__ __launch_bounds__(kThreads) void dw_wgrad_tile_kernel(DwWgArgs a) {
    dw_wgrad_tile_body<KH_, KW_>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// ---- fused depthwise backward (round 5) ------------------------------------------------
// The input gradient and the weight gradient of one same-size depthwise layer in ONE
// launch: both tile kernels above stage the same dy tile (the BatchNorm-backward of the
// layer's output, rebuilt once per element), the input gradient with the taps' halo, the
// weight gradient without; here one workgroup stages the dy region once and the forward
// input x region (tile + halo, BatchNorm / activation applied) next to it, writes dx
// through the sink and adds the tap sums into its weight-gradient replica. The weight
// gradient stops being a side-stream graph node of its own (they ran at 15.5 us in the
// step against 9.5 us alone, sharing CUs with the input-gradient chain). Same partials and
// reduction order as the two tile kernels, so the results are bitwise those of the pair.
struct DwBwdArgs {
    DwArgs d;     // d.x = dy (one segment), d.out = the dx sink, d.w = the weights
    isg_vseg x;   // the layer's forward input
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int nrep;
};

template <int KH_, int KW_>
__global__ __launch_bounds__(kThreads) void dw_bwd_tile_kernel(DwBwdArgs b) {
    constexpr int KK = KH_ * KW_;
    __shared__ float Ds[kDtMaxR * kDtMaxC];
    __shared__ float Xs[kDtMaxR * kDtMaxC];
    __shared__ float sh[(3 + KK + 1) * 4];
    const DwArgs& a = b.d;
    const int c = blockIdx.z % a.C, n = blockIdx.z / a.C;
    const int H = a.H, W = a.W;
    const int oy0 = blockIdx.y * kDtY, ox0 = blockIdx.x * kDtX;
    // dy region: the input-gradient taps' offsets (dw_tile_kernel<true>); x region: the
    // forward taps' (dw_wgrad_tile_body); both RH x RW
    const int ay0 = a.PH - (KH_ - 1) * a.DH, ax0 = a.PW - (KW_ - 1) * a.DW;
    const int RH = kDtY + (KH_ - 1) * a.DH, RW = kDtX + (KW_ - 1) * a.DW;
    const int64_t hw = (int64_t)H * W;
    const isg_vseg& sd = a.x;
    const isg_vseg& sx = b.x;
    const float* dp = sd.p + (int64_t)n * sd.n_stride + (int64_t)c * hw;
    const bool bwd = sd.xform == ISG_XF_BN_BWD;
    const float* yp = bwd ? sd.y + (int64_t)n * sd.y_n_stride + (int64_t)c * hw : dp;
    const float* xp = sx.p + (int64_t)n * sx.n_stride + (int64_t)c * hw;
    constexpr int kU = (kDtMaxR * kDtMaxC + kThreads - 1) / kThreads;
    float dr[kU], yr[kU], xr[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        dr[u] = yr[u] = xr[u] = 0.f;
        if (u * kThreads >= RH * RW) continue;  // workgroup-uniform
        const int e = threadIdx.x + u * kThreads;
        const int rr = e / RW, cc = e - rr * RW;
        const int iy = oy0 + ay0 + rr, ix = ox0 + ax0 + cc;
        const bool ok = rr < RH && iy >= 0 && iy < H && ix >= 0 && ix < W;
        const int64_t o = ok ? (int64_t)iy * W + ix : 0;
        dr[u] = dp[o];
        yr[u] = bwd ? yp[o] : 0.f;
        const int jy = oy0 - a.PH + rr, jx = ox0 - a.PW + cc;
        const bool okx = rr < RH && jy >= 0 && jy < H && jx >= 0 && jx < W;
        xr[u] = xp[okx ? (int64_t)jy * W + jx : 0];
    }
    // the sink's operand of this lane's 4 outputs (ACTBWD: the saved forward output; ACCUM:
    // the old value) in the same round trip as the tiles, not behind the compute
    typedef f32x4 __attribute__((address_space(1)))* g4p;
    typedef const f32x4 __attribute__((address_space(1)))* gc4p;
    const int ty = threadIdx.x >> 4, tq = threadIdx.x & 15;
    const int oy = oy0 + ty, ox = ox0 + 4 * tq;
    const bool oin = oy < H && ox < W;
    const isg_sink& o = a.out;
    const int omode = o.mode;
    // (branch-free: a load behind a branch drains every load in flight at the join; a mode
    // without an operand reads the weights' first quad instead and never uses it)
    const bool has_op = omode == ISG_SINK_ACTBWD || omode == ISG_SINK_ACCUM;
    const int64_t opix = has_op ? (int64_t)c * hw + (int64_t)(oin ? oy : 0) * W + (oin ? ox : 0) : 0;
    const float* const osrc = omode == ISG_SINK_ACTBWD ? o.y + (int64_t)n * o.y_n_stride
                              : (omode == ISG_SINK_ACCUM ? o.p + (int64_t)n * o.n_stride : a.w);
    const f32x4 opre = *(gc4p)((gcfloat_p)osrc + opix);
    const ChanCoef kd = seg_coef(sd, c);
    const ChanCoef kx = seg_coef(sx, c);
    const Sink1 f = sink1_coef(a.out, c);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        if (u * kThreads >= RH * RW) continue;
        const int e = threadIdx.x + u * kThreads;
        const int rr = e / RW, cc = e - rr * RW;
        if (rr >= RH) continue;
        const int iy = oy0 + ay0 + rr, ix = ox0 + ax0 + cc;
        const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
        Ds[rr * kDtMaxC + cc] = ok ? seg_xform(sd, kd, dr[u], yr[u]) : 0.f;
        const int jy = oy0 - a.PH + rr, jx = ox0 - a.PW + cc;
        const bool okx = jy >= 0 && jy < H && jx >= 0 && jx < W;
        Xs[rr * kDtMaxC + cc] = okx ? seg_xform(sx, kx, xr[u], 0.f) : 0.f;
    }
    __syncthreads();
    // ---- input gradient (dw_tile_kernel<true>'s arithmetic)
    const float* wc = a.w + c * KK;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < KH_; ++kh) {
        const int rrow = ty + (KH_ - 1 - kh) * a.DH;
#pragma unroll
        for (int kw = 0; kw < KW_; ++kw) {
            const float wv = wc[kh * KW_ + kw];
            const float* rp = Ds + rrow * kDtMaxC + 4 * tq + (KW_ - 1 - kw) * a.DW;
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] += wv * rp[j];
        }
    }
    // ---- weight gradient of this lane's 4 dy pixels (dw_wgrad_tile_body's arithmetic);
    //      out-of-image dy pixels are the region's zero padding
    float dyv[4];
    {
        const float* dc = Ds + (ty - ay0) * kDtMaxC + 4 * tq - ax0;
#pragma unroll
        for (int j = 0; j < 4; ++j) dyv[j] = dc[j];
    }
    float red[3 + KK + 1];
#pragma unroll
    for (int i = 0; i < 3 + KK + 1; ++i) red[i] = 0.f;
    red[3 + KK] = (dyv[0] + dyv[1]) + (dyv[2] + dyv[3]);
#pragma unroll
    for (int kh = 0; kh < KH_; ++kh)
#pragma unroll
        for (int kw = 0; kw < KW_; ++kw) {
            const float* rp = Xs + (ty + kh * a.DH) * kDtMaxC + 4 * tq + kw * a.DW;
            float v = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) v = fmaf(dyv[j], rp[j], v);
            red[3 + kh * KW_ + kw] = v;
        }
    // ---- dx through the sink: 16-B accesses, 4 outputs
    if (oin) {
        const int64_t off = (int64_t)n * o.n_stride + (int64_t)c * hw + (int64_t)oy * W + ox;
        if (o.mode == ISG_SINK_STORE || o.mode == ISG_SINK_ACCUM) {
            f32x4 v = {acc[0], acc[1], acc[2], acc[3]};
            if (o.mode == ISG_SINK_STORE && o.bias) v += o.bias[c];
            if (o.mode == ISG_SINK_ACCUM) v += opre;
            else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    red[0] += v[j];
                    red[1] += v[j] * v[j];
                }
            }
            if (o.mode == ISG_SINK_ACCUM) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    red[0] += acc[j];
                    red[1] += acc[j] * acc[j];
                }
            }
            *(g4p)((gfloat_p)o.p + off) = v;
        } else if (o.mode == ISG_SINK_ACTBWD) {
            const f32x4 y4 = opre;
            f32x4 g4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float z = (y4[j] - f.mean) * f.scale + f.beta;
                float gv = acc[j];
                if (o.act == ISG_ACT_RELU) {
                    gv = z > 0.f ? acc[j] : 0.f;
                } else if (o.act == ISG_ACT_PRELU) {
                    gv = z > 0.f ? acc[j] : acc[j] * f.slope;
                    red[2] += z > 0.f ? 0.f : z * acc[j];
                }
                g4[j] = gv;
                red[0] += gv;
                red[1] += gv * (y4[j] - f.mean);
            }
            *(g4p)((gfloat_p)o.p + off) = g4;
        }
    }
    block_reduce<3 + KK + 1>(red, sh);
    if (threadIdx.x == 0) {
        if (sink1_needs_red(a.out)) {
            const float r3[3] = {red[0], red[1], red[2]};
            sink1_flush(a.out, c, r3);
        }
        const int64_t ro = (int64_t)((blockIdx.x + 3u * blockIdx.y + 7u * blockIdx.z) % (unsigned)b.nrep) *
                           b.rep_stride;
        for (int t = 0; t < KK; ++t) atomicAdd(&b.dw[ro + c * KK + t], (double)red[3 + t]);
        if (b.dbias) atomicAdd(&b.dbias[ro + c], (double)red[3 + KK]);
    }
}

// ---- transposed convolution, kernel 2S, stride S, pad S/2 --------------------------
struct CtArgs {
    isg_vseg x;      // [N][Ci][H][W]
    isg_sink out;    // [N][Co][H*S][W*S]
    const float* w;  // [Ci][Co][2S][2S]
    int N, Ci, H, W;
    int Co;          // all output channels; blockIdx.y selects CO of them
};

constexpr int kCtMaxCi = 128;

// CO output channels per thread, channel group blockIdx.y: the small up-sampling convs
// (bottle4_1up / bottle5_1up, 64^2 and 128^2 inputs) have only 32-128 blocks of input
// cells, so the output channels are spread over the grid's y dimension instead.
template <int S, int CO>
__global__ __launch_bounds__(kThreads) void convT_kernel(CtArgs a) {
    constexpr int K = 2 * S, P = S / 2;
    const int co0 = blockIdx.y * CO;
    __shared__ float sh[CO][2][4];
    // the input channels' coefficients once per workgroup (each thread evaluating every
    // channel's fp64 BatchNorm finalisation itself cost +6 us per launch, round 3)
    __shared__ ChanCoef cf[kCtMaxCi];
    for (int c = threadIdx.x; c < a.Ci; c += kThreads) cf[c] = seg_coef(a.x, c);
    __syncthreads();
    const int64_t hw = (int64_t)a.H * a.W;
    const int64_t cell = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t ncell = (int64_t)a.N * hw;
    const bool valid = cell < ncell;
    int n = 0, i = 0, j = 0;
    if (valid) {
        n = (int)(cell / hw);
        const int64_t r = cell - (int64_t)n * hw;
        i = (int)(r / a.W);
        j = (int)(r - (int64_t)i * a.W);
    }
    float acc[S][S][CO];
#pragma unroll
    for (int u = 0; u < S; ++u)
#pragma unroll
        for (int v = 0; v < S; ++v)
#pragma unroll
            for (int co = 0; co < CO; ++co) acc[u][v][co] = 0.f;

    const bool xbwd = a.x.xform == ISG_XF_BN_BWD;
    for (int ci = 0; ci < a.Ci; ++ci) {
        // the 3x3 neighbourhood: unconditional loads (clamped offsets), masked after the
        // transform, so the 9 loads and the channel's coefficients are in flight together
        // (measured: bottle6_1 44 -> 36 us; the same change made the depthwise kernels
        // slower, 11.7 -> 15.8 us, and was not kept there)
        const float* xp = a.x.p + (int64_t)n * a.x.n_stride + (int64_t)ci * hw;
        const float* yp = xbwd ? a.x.y + (int64_t)n * a.x.y_n_stride + (int64_t)ci * hw : xp;
        float rx[3][3], ry[3][3];
        bool ok[3][3];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                const int yy = i + dy - 1, xx = j + dx - 1;
                ok[dy][dx] = valid && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
                const int64_t o = ok[dy][dx] ? (int64_t)yy * a.W + xx : 0;
                rx[dy][dx] = gld(xp, o);
                ry[dy][dx] = xbwd ? gld(yp, o) : 0.f;
            }
        const ChanCoef kc = cf[ci];
        float nb[3][3];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
                nb[dy][dx] = ok[dy][dx] ? seg_xform(a.x, kc, rx[dy][dx], ry[dy][dx]) : 0.f;
        const float* wci = a.w + ((int64_t)ci * a.Co + co0) * K * K;
#pragma unroll
        for (int u = 0; u < S; ++u)
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const int kh = u + P - (dy - 1) * S;  // oh = i*S+u = (i+dy-1)*S - P + kh
                if (kh < 0 || kh >= K) continue;
#pragma unroll
                for (int v = 0; v < S; ++v)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const int kw = v + P - (dx - 1) * S;
                        if (kw < 0 || kw >= K) continue;
                        const float xv = nb[dy][dx];
#pragma unroll
                        for (int co = 0; co < CO; ++co)
                            acc[u][v][co] += xv * wci[(co * K + kh) * K + kw];
                    }
            }
    }
    // epilogue
    const isg_sink& o = a.out;
    const int OW = a.W * S;
    const int64_t ohw = hw * S * S;
    float s0[CO], s1[CO];
#pragma unroll
    for (int co = 0; co < CO; ++co) {
        s0[co] = 0.f;
        s1[co] = 0.f;
        const float b = o.bias ? o.bias[co0 + co] : 0.f;
        if (valid) {
            float* dst = o.p + (int64_t)n * o.n_stride + (int64_t)(co0 + co) * ohw;
#pragma unroll
            for (int u = 0; u < S; ++u) {
                float vals[S];
#pragma unroll
                for (int v = 0; v < S; ++v) {
                    vals[v] = acc[u][v][co] + b;
                    s0[co] += vals[v];
                    s1[co] += vals[v] * vals[v];
                }
                float* row = dst + (int64_t)(i * S + u) * OW + j * S;
                if constexpr (S == 4) {
                    *reinterpret_cast<f32x4*>(row) = f32x4{vals[0], vals[1], vals[2], vals[3]};
                } else {
#pragma unroll
                    for (int v = 0; v < S; ++v) row[v] = vals[v];
                }
            }
        }
    }
    if (o.stats) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
        for (int co = 0; co < CO; ++co) {
            const float a0 = wave_sum(s0[co]), a1 = wave_sum(s1[co]);
            if (lane == 0) {
                sh[co][0][wave] = a0;
                sh[co][1][wave] = a1;
            }
        }
        __syncthreads();
        if (threadIdx.x < CO) {
            const int co = threadIdx.x;
            const float t0 = sh[co][0][0] + sh[co][0][1] + sh[co][0][2] + sh[co][0][3];
            const float t1 = sh[co][1][0] + sh[co][1][1] + sh[co][1][2] + sh[co][1][3];
            double* sp = rep_ptr(o.stats, 4 * o.C);
            atomicAdd(&sp[co0 + co], (double)t0);
            atomicAdd(&sp[o.C + co0 + co], (double)t1);
        }
    }
}

}  // namespace

int32_t isg_depthwise_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                          const isg_sinks* out, hipStream_t st) {
    if (x->nseg != 1 || out->nsink != 1 || g->SH != 1 || g->SW != 1 || g->Ci != g->Co)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "depthwise fwd: need 1 seg/sink, stride 1");
    DwArgs a{x->s[0], out->s[0], w, g->N, g->Ci, g->H, g->W, g->OH, g->OW,
             g->KH, g->KW, g->PH, g->PW, g->DH, g->DW};
    if (dw_tile_try<false>(g, a, st)) return isg_check_launch("dw_tile_kernel<fwd>");
    dim3 grid((unsigned)(((int64_t)g->OH * g->OW + kThreads - 1) / kThreads), g->Ci, g->N);
    dw_launch<false>(g, a, grid, st);
    return isg_check_launch("dw_kernel<fwd>");
}

int32_t isg_depthwise_dgrad(const isg_conv_geom* g, const isg_vtensor* dy, const float* w,
                            const isg_sinks* dx, hipStream_t st) {
    if (dy->nseg != 1 || dx->nsink != 1 || g->SH != 1 || g->SW != 1 || g->Ci != g->Co)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "depthwise dgrad: need 1 seg/sink, stride 1");
    DwArgs a{dy->s[0], dx->s[0], w, g->N, g->Ci, g->H, g->W, g->OH, g->OW,
             g->KH, g->KW, g->PH, g->PW, g->DH, g->DW};
    if (dw_tile_try<true>(g, a, st)) return isg_check_launch("dw_tile_kernel<dgrad>");
    dim3 grid((unsigned)(((int64_t)g->H * g->W + kThreads - 1) / kThreads), g->Ci, g->N);
    dw_launch<true>(g, a, grid, st);
    return isg_check_launch("dw_kernel<dgrad>");
}

int32_t isg_depthwise_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                            double* dw, double* dbias, int64_t rep_stride, int32_t nrep,
                            hipStream_t st) {
    if (dy->nseg != 1 || x->nseg != 1 || g->KH * g->KW > kMaxTaps || x->s[0].xform == ISG_XF_BN_BWD)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "depthwise wgrad: need 1 seg, <= 9 taps, x not BN-backward");
    DwWgArgs a{};
    a.dy = dy->s[0]; a.x = x->s[0]; a.dw = dw; a.dbias = dbias;
    a.rep_stride = rep_stride; a.nrep = nrep;
    a.N = g->N; a.C = g->Ci; a.H = g->H; a.W = g->W; a.OH = g->OH; a.OW = g->OW;
    a.KH = g->KH; a.KW = g->KW; a.PH = g->PH; a.PW = g->PW; a.DH = g->DH; a.DW = g->DW;
    {
        const isg_vseg& d = a.dy;
        const bool ok = g->SH == 1 && g->SW == 1 && g->OH == g->H && g->OW == g->W && g->W % 4 == 0 &&
                        !((uintptr_t)d.p & 15) && d.n_stride % 4 == 0 &&
                        (d.xform != ISG_XF_BN_BWD || (!((uintptr_t)d.y & 15) && d.y_n_stride % 4 == 0)) &&
                        (g->KH - 1) * g->DH <= 16 && (g->KW - 1) * g->DW <= 16;
        const dim3 grid((unsigned)((g->W + kDtX - 1) / kDtX), (unsigned)((g->H + kDtY - 1) / kDtY),
                        (unsigned)(g->Ci * g->N));
        if (ok && g->KH == 3 && g->KW == 3) {
            hipLaunchKernelGGL((dw_wgrad_tile_kernel<3, 3>), grid, dim3(kThreads), 0, st, a);
            return isg_check_launch("dw_wgrad_tile_kernel");
        }
        if (ok && g->KH == 5 && g->KW == 1) {
            hipLaunchKernelGGL((dw_wgrad_tile_kernel<5, 1>), grid, dim3(kThreads), 0, st, a);
            return isg_check_launch("dw_wgrad_tile_kernel");
        }
        if (ok && g->KH == 1 && g->KW == 5) {
            hipLaunchKernelGGL((dw_wgrad_tile_kernel<1, 5>), grid, dim3(kThreads), 0, st, a);
            return isg_check_launch("dw_wgrad_tile_kernel");
        }
    }
    const int64_t P = (int64_t)g->N * g->OH * g->OW;
    // one pass of kDwPix pixels per block while that still leaves >= ~1024 blocks
    int64_t splits = (P + kDwPix - 1) / kDwPix;
    const int64_t maxsplit = std::max<int64_t>(1, 2048 / g->Ci);
    if (splits > maxsplit) splits = maxsplit;
    if (splits < 1) splits = 1;
    a.pix_per_block = (P + splits - 1) / splits;
    hipLaunchKernelGGL(dw_wgrad_kernel, dim3((unsigned)splits, g->Ci), dim3(kThreads), 0, st, a);
    return isg_check_launch("dw_wgrad_kernel");
}

// dx and dw of one depthwise layer (isg.h isg_depthwise_bwd): the fused tile kernel when
// both tile kernels would run, else the two separate entry points in order
int32_t isg_depthwise_bwd(const isg_conv_geom* g, const isg_vtensor* dy_, const float* w,
                          const isg_sinks* dx, const isg_vtensor* x_, double* dw, double* dbias,
                          int64_t rep_stride, int32_t nrep, hipStream_t st) {
    if (!g || !dy_ || !x_) return isg_set_error(ISG_ERR_INVALID, "depthwise bwd: NULL argument");
    // a BN_BWD segment with y NULL means y = p (isg.h): resolved here like the conv entry
    // points do, so neither the fused kernel nor the two fallbacks read through NULL
    const isg_vtensor dyr = isg_resolve_y(dy_), xr = isg_resolve_y(x_);
    const isg_vtensor *dy = &dyr, *x = &xr;
    if (g->groups <= 1 || g->groups != g->Ci || g->Ci != g->Co)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "depthwise bwd: not a depthwise layer");
    if (isg_vt_res(dy) || isg_vt_res(x) || isg_sinks_res(dx))
        return isg_set_error(ISG_ERR_UNSUPPORTED, "depthwise bwd: residual form");
    if (nrep < 1 || (nrep > 1 && rep_stride <= 0))
        return isg_set_error(ISG_ERR_INVALID, "depthwise bwd: bad replicas");
    const bool has_dx = dx && dx->nsink > 0;
    bool fuse = has_dx && dw && dy->nseg == 1 && x->nseg == 1 && dx->nsink == 1 &&
                x->s[0].xform != ISG_XF_BN_BWD && g->SH == 1 && g->SW == 1 && g->OH == g->H &&
                g->OW == g->W && g->W % 4 == 0 && (g->KH - 1) * g->DH <= 16 && (g->KW - 1) * g->DW <= 16;
    const int KH = g->KH, KW = g->KW;
    fuse = fuse && ((KH == 3 && KW == 3) || (KH == 5 && KW == 1) || (KH == 1 && KW == 5));
    if (fuse) {
        const isg_sink& o = dx->s[0];
        fuse = o.mode != ISG_SINK_NONE && !((uintptr_t)o.p & 15) && o.n_stride % 4 == 0 &&
               (o.mode != ISG_SINK_ACTBWD || (!((uintptr_t)o.y & 15) && o.y_n_stride % 4 == 0));
    }
    if (!fuse) {
        if (has_dx)
            if (int32_t e = isg_depthwise_dgrad(g, dy, w, dx, st)) return e;
        return dw ? isg_depthwise_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st) : ISG_OK;
    }
    DwBwdArgs b{};
    b.d = DwArgs{dy->s[0], dx->s[0], w, g->N, g->Ci, g->H, g->W, g->OH, g->OW,
                 g->KH, g->KW, g->PH, g->PW, g->DH, g->DW};
    b.x = x->s[0];
    b.dw = dw; b.dbias = dbias; b.rep_stride = nrep > 1 ? rep_stride : 0; b.nrep = nrep;
    const dim3 grid((unsigned)((g->W + kDtX - 1) / kDtX), (unsigned)((g->H + kDtY - 1) / kDtY),
                    (unsigned)(g->Ci * g->N));
    if (KH == 3) hipLaunchKernelGGL((dw_bwd_tile_kernel<3, 3>), grid, dim3(kThreads), 0, st, b);
    else if (KH == 5) hipLaunchKernelGGL((dw_bwd_tile_kernel<5, 1>), grid, dim3(kThreads), 0, st, b);
    else hipLaunchKernelGGL((dw_bwd_tile_kernel<1, 5>), grid, dim3(kThreads), 0, st, b);
    return isg_check_launch("dw_bwd_tile_kernel");
}

int32_t isg_convT_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                      const isg_sinks* out, isg_stream_t st) {
    if (isg_vt_res(x) || isg_sinks_res(out)) return isg_set_error(ISG_ERR_UNSUPPORTED, "convT fwd: residual form");
    if (x->nseg != 1 || out->nsink != 1 || out->s[0].mode != ISG_SINK_STORE || g->Ci > kCtMaxCi)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "convT fwd: need 1 seg / 1 STORE sink, Ci <= %d", kCtMaxCi);
    const int S = g->SH;
    if (g->SW != S || g->KH != 2 * S || g->KW != 2 * S || g->PH != S / 2 || g->PW != S / 2 ||
        g->OH != g->H * S || g->OW != g->W * S)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "convT fwd: need k=2s, p=s/2");
    CtArgs a{x->s[0], out->s[0], w, g->N, g->Ci, g->H, g->W, g->Co};
    const unsigned gx = (unsigned)(((int64_t)g->N * g->H * g->W + kThreads - 1) / kThreads);
    if (S != 2 && S != 4) return isg_set_error(ISG_ERR_UNSUPPORTED, "convT fwd: s=%d", S);
    // channels per thread: split the output channels until the grid has ~1024 blocks
    int cob = g->Co;
    while (cob > 1 && (int64_t)gx * (g->Co / cob) < 1024 && cob % 2 == 0) cob /= 2;
    if (cob > 4 || g->Co % cob) cob = g->Co % 4 == 0 ? 4 : (g->Co % 2 == 0 ? 2 : 1);
    const dim3 grid(gx, (unsigned)(g->Co / cob));
    if (S == 2 && cob == 4) hipLaunchKernelGGL((convT_kernel<2, 4>), grid, dim3(kThreads), 0, st, a);
    else if (S == 2 && cob == 2) hipLaunchKernelGGL((convT_kernel<2, 2>), grid, dim3(kThreads), 0, st, a);
    else if (S == 2) hipLaunchKernelGGL((convT_kernel<2, 1>), grid, dim3(kThreads), 0, st, a);
    else if (cob == 4) hipLaunchKernelGGL((convT_kernel<4, 4>), grid, dim3(kThreads), 0, st, a);
    else if (cob == 2) hipLaunchKernelGGL((convT_kernel<4, 2>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((convT_kernel<4, 1>), grid, dim3(kThreads), 0, st, a);
    return isg_check_launch("convT_kernel");
}
