// Direct VALU convolution for THIN stride-1 convs (few input and output channels, large
// planes): the mask-head 3x3 conv 4->1 at full resolution (segment.py:437) and its input
// gradient (1->4), and the 4->4 dense 3x3 of bottle5_2 (:242). On the MFMA tap kernel
// these shapes multiply 15/16 padding; here a lane owns one output pixel for all M
// output channels, reads its C x K x K window (neighbouring lanes share it through the
// vector cache) with the producer's transform applied, and routes each channel through
// its sink (store + bias + BN statistics, accumulate, or activation backward).
//
//   forward: out[m][p] = sum_{c,kh,kw} W[m][c][kh][kw] * x[c][p + (kh*D - P, kw*D - P)]
//   dgrad  : dx[m][q]  = sum_{c,kh,kw} W[c][m][kh][kw] * dy[c][q + (P - kh*D, P - kw*D)]
#include <algorithm>

#include "stage.h"

namespace {

constexpr int kThreads = 256;

struct ThinArgs {
    isg_vtensor src;
    isg_sinks out;
    const float* w;
    int N, SrcH, SrcW, DstH, DstW, P, D, dgrad;
};

template <int C, int M, int K>
__global__ __launch_bounds__(kThreads) void thin_conv_kernel(ThinArgs a) {
    constexpr int KK = K * K;
    __shared__ ChT tab[C];
    __shared__ SinkRow ri[M];
    __shared__ float ws[M * C * KK];
    __shared__ float red[4][3][M];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    if (tid < C) tab[tid] = ch_table_entry(a.src, tid, (int64_t)a.SrcH * a.SrcW);
    if (tid < M) ri[tid] = sink_row(a.out, tid, (int64_t)a.DstH * a.DstW);
    for (int i = tid; i < M * C * KK; i += kThreads) {
        const int m = i / (C * KK), r = i - m * C * KK, c = r / KK, t = r - c * KK;
        ws[i] = a.dgrad ? a.w[(c * M + m) * KK + t] : a.w[(m * C + c) * KK + t];
    }
    __syncthreads();

    const int64_t hw = (int64_t)a.DstH * a.DstW;
    const int64_t p = (int64_t)blockIdx.x * kThreads + tid;
    const bool pv = p < (int64_t)a.N * hw;
    const int n = pv ? (int)(p / hw) : 0;
    const int pix = pv ? (int)(p - (int64_t)n * hw) : 0;
    const int oy = pix / a.DstW, ox = pix - oy * a.DstW;
    float acc[M];
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const ChT t = tab[c];
        const float* xp = t.p + (int64_t)n * t.ns;
        const float* yp = t.y + (int64_t)n * t.yns;
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
            const int iy = a.dgrad ? oy + a.P - kh * a.D : oy - a.P + kh * a.D;
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
                const int ix = a.dgrad ? ox + a.P - kw * a.D : ox - a.P + kw * a.D;
                float v = 0.f;
                if (pv && (unsigned)iy < (unsigned)a.SrcH && (unsigned)ix < (unsigned)a.SrcW) {
                    const int64_t o = (int64_t)iy * a.SrcW + ix;
                    const float x = gld(xp, o);
                    v = ch_xform(t.xf, t.act, t.k, x, t.xf == ISG_XF_BN_BWD ? gld(yp, o) : x);
                }
#pragma unroll
                for (int m = 0; m < M; ++m) acc[m] += ws[(m * C + c) * KK + kh * K + kw] * v;
            }
        }
    }
    float s0[M], s1[M], s2[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        s0[m] = s1[m] = s2[m] = 0.f;
        if (pv) sink_row_apply(ri[m], n, pix, acc[m], s0[m], s1[m], s2[m]);
    }
    if (sinks_need_red(a.out)) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const float t0 = wave_sum(s0[m]), t1 = wave_sum(s1[m]), t2 = wave_sum(s2[m]);
            if (lane == 0) {
                red[wave][0][m] = t0;
                red[wave][1][m] = t1;
                red[wave][2][m] = t2;
            }
        }
        __syncthreads();
        if (tid < M) {
            float r3[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) r3[j] = ((red[0][j][tid] + red[1][j][tid]) + red[2][j][tid]) + red[3][j][tid];
            sink_row_flush(a.out, tid, r3[0], r3[1], r3[2]);
        }
    }
}

// One window row of the 4-pixel lane: source row iy, columns ox-1 .. ox+4, the producer's
// transform applied and zero padding outside the plane (after the transform). All loads
// are unconditional (clamped offsets), so a lane's rows are in flight together.
ISG_DEV void x4_window(const float* xp, const float* yp, bool bwd, const ChT& t, bool pv, int iy,
                       int ox, int H, int W, float (&v)[6]) {
    const bool rok = pv && (unsigned)iy < (unsigned)H;
    const int64_t o = (int64_t)(rok ? iy : 0) * W + ox;
    const bool lok = rok && ox > 0, rrok = rok && ox + 4 < W;
    const f32x4 c4 = gld4(xp, o);
    const float l = gld(xp, lok ? o - 1 : o), rr = gld(xp, rrok ? o + 4 : o);
    float y6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (bwd) {
        const f32x4 yc = gld4(yp, o);
        y6[0] = gld(yp, lok ? o - 1 : o);
        y6[1] = yc[0]; y6[2] = yc[1]; y6[3] = yc[2]; y6[4] = yc[3];
        y6[5] = gld(yp, rrok ? o + 4 : o);
    }
    const float raw[6] = {l, c4[0], c4[1], c4[2], c4[3], rr};
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = ch_xform_u(t.xf, t.act, t.k, raw[i], y6[i]);
    if (!lok) v[0] = 0.f;
    if (!rrok) v[5] = 0.f;
    if (!rok) {
#pragma unroll
        for (int i = 1; i < 5; ++i) v[i] = 0.f;
    }
}

// 3x3, pad 1, dilation 1, 4 consecutive output pixels per lane (DstW % 4 == 0): per
// (channel, window row) one 16-B load of the 4 centre columns plus the two edge columns.
template <int C, int M>
__global__ __launch_bounds__(kThreads) void thin_conv3_x4_kernel(ThinArgs a) {
    constexpr int KK = 9;
    __shared__ ChT tab[C];
    __shared__ SinkRow ri[M];
    __shared__ float ws[M * C * KK];
    __shared__ float red[4][3][M];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    if (tid < C) tab[tid] = ch_table_entry(a.src, tid, (int64_t)a.SrcH * a.SrcW);
    if (tid < M) ri[tid] = sink_row(a.out, tid, (int64_t)a.DstH * a.DstW);
    for (int i = tid; i < M * C * KK; i += kThreads) {
        const int m = i / (C * KK), r = i - m * C * KK, c = r / KK, t = r - c * KK;
        // dgrad: tap (kh, kw) reads dy at (+1-kh, +1-kw): store the weight at the
        // flipped tap so both directions index the window the same way
        ws[i] = a.dgrad ? a.w[(c * M + m) * KK + (KK - 1 - t)] : a.w[(m * C + c) * KK + t];
    }
    __syncthreads();

    const int wq = a.DstW >> 2;
    const int64_t hwq = (int64_t)a.DstH * wq;
    const int64_t q = (int64_t)blockIdx.x * kThreads + tid;
    const bool pv = q < (int64_t)a.N * hwq;
    const int n = pv ? (int)(q / hwq) : 0;
    const int r = pv ? (int)(q - (int64_t)n * hwq) : 0;
    const int oy = r / wq, ox = (r - oy * wq) * 4;
    float acc[M][4];
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[m][j] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const ChT t = tab[c];
        const float* xp = t.p + (int64_t)n * t.ns;
        const float* yp = t.y + (int64_t)n * t.yns;
        const bool bwd = t.xf == ISG_XF_BN_BWD;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            float v[6];
            x4_window(xp, yp, bwd, t, pv, oy - 1 + kh, ox, a.SrcH, a.SrcW, v);
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const float wv = ws[(m * C + c) * KK + kh * 3 + kw];
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[m][j] += wv * v[j + kw];
                }
        }
    }
    float s0[M], s1[M], s2[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        s0[m] = s1[m] = s2[m] = 0.f;
        if (pv) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float t0 = 0.f, t1 = 0.f, t2 = 0.f;
                sink_row_apply(ri[m], n, (int64_t)oy * a.DstW + ox + j, acc[m][j], t0, t1, t2);
                s0[m] += t0;
                s1[m] += t1;
                s2[m] += t2;
            }
        }
    }
    if (sinks_need_red(a.out)) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const float t0 = wave_sum(s0[m]), t1 = wave_sum(s1[m]), t2 = wave_sum(s2[m]);
            if (lane == 0) {
                red[wave][0][m] = t0;
                red[wave][1][m] = t1;
                red[wave][2][m] = t2;
            }
        }
        __syncthreads();
        if (tid < M) {
            float r3[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) r3[j] = ((red[0][j][tid] + red[1][j][tid]) + red[2][j][tid]) + red[3][j][tid];
            sink_row_flush(a.out, tid, r3[0], r3[1], r3[2]);
        }
    }
}

// Weight gradient of the thin 3x3 convs (pad 1, dilation 1, stride 1; M*C*9 <= 36):
//   dW[m][c][kh][kw] += sum_p dy[m][p] * x[c][p + (kh-1, kw-1)],  dbias[m] += sum_p dy[m][p]
// 4 consecutive pixels per lane (the forward's window rows), grid-stride over the quads;
// each workgroup reduces its partials (waves in fixed order) and adds them with one atomic
// per element into one of nrep replicas (include/isg.h ISG_WREP).
struct ThinWgArgs {
    isg_vtensor dy, x;
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int nrep;
    int N, H, W;
};

template <int C, int M>
__global__ __launch_bounds__(kThreads) void thin_wgrad3_x4_kernel(ThinWgArgs a) {
    constexpr int NA = M * C * 9 + M;  // weight partials + bias partials
    __shared__ ChT tx[C], ty[M];
    __shared__ float red[4][NA];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int64_t hw = (int64_t)a.H * a.W;
    if (tid < C) tx[tid] = ch_table_entry(a.x, tid, hw);
    if (tid < M) ty[tid] = ch_table_entry(a.dy, tid, hw);
    __syncthreads();
    float acc[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) acc[i] = 0.f;
    const int wq = a.W >> 2;
    const int64_t hwq = (int64_t)a.H * wq, nq = (int64_t)a.N * hwq;
    for (int64_t q = (int64_t)blockIdx.x * kThreads + tid; q < nq + kThreads - 1; q += (int64_t)gridDim.x * kThreads) {
        if (q - tid >= nq) break;  // wave-uniform exit once the whole block is past the end
        const bool pv = q < nq;
        const int64_t qq = pv ? q : 0;
        const int n = (int)(qq / hwq);
        const int r = (int)(qq - (int64_t)n * hwq);
        const int oy = r / wq, ox = (r - oy * wq) * 4;
        float d[M][4];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const ChT t = ty[m];
            const int64_t o = (int64_t)oy * a.W + ox;
            const f32x4 g4 = gld4(t.p + (int64_t)n * t.ns, o);
            f32x4 y4 = g4;
            if (t.xf == ISG_XF_BN_BWD) y4 = gld4(t.y + (int64_t)n * t.yns, o);
#pragma unroll
            for (int j = 0; j < 4; ++j) d[m][j] = pv ? ch_xform_u(t.xf, t.act, t.k, g4[j], y4[j]) : 0.f;
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const ChT t = tx[c];
            const float* xp = t.p + (int64_t)n * t.ns;
            const float* yp = t.y + (int64_t)n * t.yns;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                float v[6];
                x4_window(xp, yp, t.xf == ISG_XF_BN_BWD, t, pv, oy - 1 + kh, ox, a.H, a.W, v);
#pragma unroll
                for (int m = 0; m < M; ++m)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw) {
                        float s = acc[(m * C + c) * 9 + kh * 3 + kw];
#pragma unroll
                        for (int j = 0; j < 4; ++j) s = fmaf(d[m][j], v[j + kw], s);
                        acc[(m * C + c) * 9 + kh * 3 + kw] = s;
                    }
            }
        }
#pragma unroll
        for (int m = 0; m < M; ++m) acc[M * C * 9 + m] += (d[m][0] + d[m][1]) + (d[m][2] + d[m][3]);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const float t = wave_sum(acc[i]);
        if (lane == 0) red[wave][i] = t;
    }
    __syncthreads();
    if (tid < NA) {
        const float t = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
        const int64_t ro = (int64_t)(blockIdx.x % (unsigned)a.nrep) * a.rep_stride;
        if (tid < M * C * 9) atomicAdd(&a.dw[ro + tid], t);
        else if (a.dbias) atomicAdd(&a.dbias[ro + tid - M * C * 9], t);
    }
}

}  // namespace


// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
int32_t isg_thin_conv(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                      const isg_sinks* out, bool dgrad, hipStream_t st) {
    if (g->groups != 1 || g->SH != 1 || g->SW != 1 || g->KH != g->KW || g->PH != g->PW ||
        g->DH != g->DW)
        return 0;
    const int C = dgrad ? g->Co : g->Ci, M = dgrad ? g->Ci : g->Co, K = g->KH;
    ThinArgs a{};
    a.src = *src; a.out = *out; a.w = w; a.N = g->N;
    a.SrcH = dgrad ? g->OH : g->H; a.SrcW = dgrad ? g->OW : g->W;
    a.DstH = dgrad ? g->H : g->OH; a.DstW = dgrad ? g->W : g->OW;
    a.P = g->PH; a.D = g->DH; a.dgrad = dgrad ? 1 : 0;
    const int64_t P = (int64_t)g->N * a.DstH * a.DstW;
    dim3 grid((unsigned)((P + kThreads - 1) / kThreads));
    // 4 pixels per lane: 3x3 / pad 1 / dilation 1, same plane size, 16-B aligned rows
    const bool x4 = K == 3 && a.P == 1 && a.D == 1 && a.DstW % 4 == 0 && a.SrcW == a.DstW &&
                    a.SrcH == a.DstH;
    bool aligned = true;
    for (int i = 0; i < src->nseg; ++i)
        aligned &= ((uintptr_t)src->s[i].p % 16 == 0) && src->s[i].n_stride % 4 == 0 &&
                   (src->s[i].xform != ISG_XF_BN_BWD ||
                    ((uintptr_t)src->s[i].y % 16 == 0 && src->s[i].y_n_stride % 4 == 0));
    if (x4 && aligned) {
        dim3 g4((unsigned)((P / 4 + kThreads - 1) / kThreads));
        if (C == 4 && M == 1) hipLaunchKernelGGL((thin_conv3_x4_kernel<4, 1>), g4, dim3(kThreads), 0, st, a);
        else if (C == 1 && M == 4) hipLaunchKernelGGL((thin_conv3_x4_kernel<1, 4>), g4, dim3(kThreads), 0, st, a);
        else if (C == 4 && M == 4) hipLaunchKernelGGL((thin_conv3_x4_kernel<4, 4>), g4, dim3(kThreads), 0, st, a);
        else return 0;
        const int32_t e = isg_check_launch("thin_conv3_x4_kernel");
        return e ? e : 1;
    }
    if (C == 4 && M == 1 && K == 3) hipLaunchKernelGGL((thin_conv_kernel<4, 1, 3>), grid, dim3(kThreads), 0, st, a);
    else if (C == 1 && M == 4 && K == 3) hipLaunchKernelGGL((thin_conv_kernel<1, 4, 3>), grid, dim3(kThreads), 0, st, a);
    else if (C == 4 && M == 4 && K == 3) hipLaunchKernelGGL((thin_conv_kernel<4, 4, 3>), grid, dim3(kThreads), 0, st, a);
    else return 0;
    const int32_t e = isg_check_launch("thin_conv_kernel");
    return e ? e : 1;
}

// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
int32_t isg_thin_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                       double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st) {
    if (g->groups != 1 || g->SH != 1 || g->SW != 1 || g->KH != 3 || g->KW != 3 ||
        g->PH != 1 || g->PW != 1 || g->DH != 1 || g->DW != 1 || g->OH != g->H || g->OW != g->W ||
        g->W % 4 || dy->nseg != 1 || x->nseg != 1 || (g->w_ci > 0 && g->w_ci != g->Ci))
        return 0;
    auto al = [](const isg_vseg& sg) {
        return (uintptr_t)sg.p % 16 == 0 && sg.n_stride % 4 == 0 &&
               (sg.xform != ISG_XF_BN_BWD || ((uintptr_t)sg.y % 16 == 0 && sg.y_n_stride % 4 == 0));
    };
    if (!al(dy->s[0]) || !al(x->s[0])) return 0;
    ThinWgArgs a{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias;
    a.rep_stride = nrep > 1 ? rep_stride : 0;
    a.nrep = nrep < 1 ? 1 : nrep;
    a.N = g->N; a.H = g->H; a.W = g->W;
    const int64_t nq = (int64_t)g->N * g->H * (g->W / 4);
    // ~4 quads per lane: enough work per workgroup to amortise its reduction
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(2048, (nq + 4 * kThreads - 1) / (4 * kThreads)));
    if (g->Ci == 4 && g->Co == 1)
        hipLaunchKernelGGL((thin_wgrad3_x4_kernel<4, 1>), dim3((unsigned)blocks), dim3(kThreads), 0, st, a);
    else if (g->Ci == 1 && g->Co == 4)
        hipLaunchKernelGGL((thin_wgrad3_x4_kernel<1, 4>), dim3((unsigned)blocks), dim3(kThreads), 0, st, a);
    else
        return 0;
    const int32_t e = isg_check_launch("thin_wgrad3_x4_kernel");
    return e ? e : 1;
}
