// Dense convolution as implicit GEMM on v_mfma_f32_16x16x4_f32 (gfx950).
//
// Replaces the aten conv kernels behind every dense `nn.Conv2d` of the reference
// (segment.py:39-40 via Conv, :323/:343 uppool 1x1, :437 head 3x3), and — with the
// operand roles swapped — the ConvTranspose2d backward (segment.py:305, :435).
//
// One kernel serves two GEMM shapes, both "gather B from a virtual tensor":
//   FWD   : out[co][p]  = sum_k W[co][k]       * x_im2col[k][p]     (k = ci,kh,kw)
//   DGRAD : dx[ci][q]   = sum_k W'[ci][k]      * dy_gather[k][q]    (k = co,kh,kw)
// DGRAD is phase-grouped: blockIdx.y is the stride phase (ph,pw) of the input
// pixels a block produces, so only the taps that hit that phase enter K — the
// stride-2 5x5 stem dgrad does 25/4 instead of 25 taps per channel, and no lane
// ever multiplies a structural zero.
//
// MFMA lane maps (cdna_hip_programming.md §3, 16x16x4 f32):
//   A[i][k]: lane l holds i = l&15, k = l>>4   -> weights, row = output channel
//   B[k][j]: lane l holds k = l>>4, j = l&15   -> gathered activations, j = pixel
//   D[i][j]: lane l holds i = (l>>4)*4 + r, j = l&15
// so each lane gathers ONE activation per k-step and 16 lanes cover 16 consecutive
// output pixels (64-B coalesced segments for stride-1 sources).
#include "common.h"

namespace {

constexpr int kWaves = 4;
static_assert(kWaves == 4, "the epilogue sums the per-wave partials of 4 waves");
constexpr int kThreads = kWaves * 64;
constexpr int kKtabMax = 1024;
constexpr int kMaxRows = 256;

struct KEnt {
    int c;   // gathered channel
    int by;  // source row offset
    int bx;  // source col offset
    int wk;  // weight offset
};

struct GemmArgs {
    isg_vtensor src;   // gathered operand
    isg_sinks out;     // where rows go
    const float* w;
    int mode;          // 0 FWD, 1 DGRAD
    int N;
    int TH, TW;        // tile pixel space per image (per phase for DGRAD)
    int SrcH, SrcW;
    int my, mx;
    int DstH, DstW;
    int dmy, dmx;
    int M;             // rows (output channels)
    int wrs;           // weight row stride
    // conv geometry (for table construction)
    int Ci, Co, KH, KW, SH, SW, PH, PW, DH, DW, H, W, OH, OW;
};

__device__ int pos_mod(int a, int m) {
    int r = a % m;
    return r < 0 ? r + m : r;
}

template <int MT>
__global__ __launch_bounds__(kThreads) void gemm_conv_kernel(GemmArgs a) {
    __shared__ KEnt ktab[kKtabMax];
    __shared__ ChanCoef coef[ISG_MAX_CH];
    __shared__ SinkCoef scoef[kMaxRows];
    // per-wave partials (summed in wave order before the flush: deterministic, no LDS atomics)
    __shared__ float red[kWaves][3][kMaxRows];
    __shared__ int s_K, s_oy0, s_ox0, s_TH, s_TW;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int kk = lane >> 4;
    const int pl = lane & 15;
    const int KK = a.KH * a.KW;

    // ---- per-block K table --------------------------------------------------
    if (a.mode == 0) {
        const int K = a.Ci * KK;
        for (int k = tid; k < K; k += kThreads) {
            int ci = k / KK, t = k - ci * KK;
            int kh = t / a.KW, kw = t - kh * a.KW;
            ktab[k] = KEnt{ci, kh * a.DH - a.PH, kw * a.DW - a.PW, k};
        }
        if (tid == 0) { s_K = K; s_oy0 = 0; s_ox0 = 0; s_TH = a.TH; s_TW = a.TW; }
    } else {
        __shared__ int khs[16], kws[16], s_nkh, s_nkw;
        const int ph = blockIdx.y / a.SW, pw = blockIdx.y % a.SW;
        if (tid == 0) {
            int nkh = 0, nkw = 0;
            for (int kh = 0; kh < a.KH; ++kh)
                if (pos_mod(ph + a.PH - kh * a.DH, a.SH) == 0) khs[nkh++] = kh;
            for (int kw = 0; kw < a.KW; ++kw)
                if (pos_mod(pw + a.PW - kw * a.DW, a.SW) == 0) kws[nkw++] = kw;
            s_nkh = nkh;
            s_nkw = nkw;
            s_K = a.Co * nkh * nkw;
            s_oy0 = ph;
            s_ox0 = pw;
            s_TH = (a.H - ph + a.SH - 1) / a.SH;
            s_TW = (a.W - pw + a.SW - 1) / a.SW;
        }
        __syncthreads();
        const int nkh = s_nkh, nkw = s_nkw, ntap = nkh * nkw;
        for (int k = tid; k < s_K; k += kThreads) {
            const int co = k / ntap, t = k - co * ntap;
            const int kh = khs[t / nkw], kw = kws[t % nkw];
            ktab[k] = KEnt{co, (ph + a.PH - kh * a.DH) / a.SH, (pw + a.PW - kw * a.DW) / a.SW,
                           co * a.Ci * KK + kh * a.KW + kw};
        }
    }
    load_vt_coefs(a.src, coef, tid, kThreads);
    load_sink_coefs(a.out, scoef, tid, kThreads);
    for (int i = tid; i < kWaves * 3 * kMaxRows; i += kThreads) (&red[0][0][0])[i] = 0.f;
    __syncthreads();

    const int K = s_K;
    const int TH = s_TH, TW = s_TW;
    const int oy0 = s_oy0, ox0 = s_ox0;
    const int64_t srcHW = (int64_t)a.SrcH * a.SrcW;
    const int64_t dstHW = (int64_t)a.DstH * a.DstW;
    const int64_t tilePix = (int64_t)TH * TW;
    const int64_t P = (int64_t)a.N * tilePix;
    const int64_t ntiles = (P + 15) / 16;
    const bool need_red = sinks_need_red(a.out);
    const float* __restrict__ w = a.w;

    for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < ntiles;
         tile += (int64_t)gridDim.x * kWaves) {
        const int64_t p = tile * 16 + pl;
        const bool pv = p < P;
        int n = 0, ty = 0, tx = 0;
        if (pv) {
            n = (int)(p / tilePix);
            int r = (int)(p - (int64_t)n * tilePix);
            ty = r / TW;
            tx = r - ty * TW;
        }
        const int sy0 = a.my * ty, sx0 = a.mx * tx;
        f32x4 acc[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 2
        for (int k0 = 0; k0 < K; k0 += 4) {
            const int k = k0 + kk;
            float bv = 0.f;
            int wk = 0;
            const bool kv = k < K;
            if (kv) {
                const KEnt e = ktab[k];
                wk = e.wk;
                const int sy = e.by + sy0, sx = e.bx + sx0;
                if (pv && sy >= 0 && sy < a.SrcH && sx >= 0 && sx < a.SrcW)
                    bv = vt_load(a.src, coef, n, e.c, srcHW, (int64_t)sy * a.SrcW + sx);
            }
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const int row = m * 16 + pl;
                const float av = (kv && row < a.M) ? w[wk + row * a.wrs] : 0.f;
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[m], 0, 0, 0);
            }
        }

        // ---- epilogue: lane holds rows m*16 + kk*4 + r at pixel p -------------
        const int dy = oy0 + a.dmy * ty, dx = ox0 + a.dmx * tx;
        const int64_t dpix = (int64_t)dy * a.DstW + dx;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m * 16 + kk * 4 + r;
                SinkRed rr = {0.f, 0.f, 0.f};
                if (row < a.M && pv) {
                    const int s = sink_of(a.out, row);
                    rr = sink_apply(a.out.s[s], scoef, row, n, dstHW, dpix, acc[m][r]);
                }
                if (need_red) {
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) {
                        rr.r0 += __shfl_xor(rr.r0, o, 64);
                        rr.r1 += __shfl_xor(rr.r1, o, 64);
                        rr.r2 += __shfl_xor(rr.r2, o, 64);
                    }
                    if (pl == 0 && row < a.M) {  // one lane of this wave owns the row
                        red[wave][0][row] += rr.r0;
                        red[wave][1][row] += rr.r1;
                        red[wave][2][row] += rr.r2;
                    }
                }
            }
        }
    }
    if (need_red) {
        __syncthreads();
        for (int i = tid; i < 3 * kMaxRows; i += kThreads) {
            float* r = &red[0][0][0] + i;
            *r = ((r[0] + r[3 * kMaxRows]) + r[6 * kMaxRows]) + r[9 * kMaxRows];
        }
        __syncthreads();
        flush_sink_red(a.out, red[0][0], red[0][1], red[0][2], a.M, tid, kThreads);
    }
}

int vt_channels(const isg_vtensor* v) {
    int c = 0;
    for (int i = 0; i < v->nseg; ++i) c += v->s[i].C;
    return c;
}

int num_blocks_for(int64_t ntiles) {
    int64_t b = (ntiles + kWaves - 1) / kWaves;
    if (b > 4096) b = 4096;
    if (b < 1) b = 1;
    return (int)b;
}

template <int MT>
void launch_gemm(const GemmArgs& a, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL(gemm_conv_kernel<MT>, grid, dim3(kThreads), 0, st, a);
}

int32_t dispatch_gemm(const GemmArgs& a, dim3 grid, hipStream_t st) {
    const int mt = (a.M + 15) / 16;
    switch (mt) {
        case 1: launch_gemm<1>(a, grid, st); break;
        case 2: launch_gemm<2>(a, grid, st); break;
        case 3: launch_gemm<3>(a, grid, st); break;
        case 4: launch_gemm<4>(a, grid, st); break;
        case 5: case 6: launch_gemm<6>(a, grid, st); break;
        case 7: case 8: launch_gemm<8>(a, grid, st); break;
        case 9: case 10: case 11: case 12: launch_gemm<12>(a, grid, st); break;
        case 13: case 14: case 15: case 16: launch_gemm<16>(a, grid, st); break;
        default: return isg_set_error(ISG_ERR_UNSUPPORTED, "gemm conv: %d rows > 256", a.M);
    }
    return isg_check_launch("gemm_conv_kernel");
}

int32_t check_sinks(const isg_sinks* s, int M, const char* what) {
    if (!s || s->nsink < 1 || s->nsink > ISG_MAX_SEGS)
        return isg_set_error(ISG_ERR_INVALID, "%s: bad sink count", what);
    int c = 0;
    for (int i = 0; i < s->nsink; ++i) {
        if (s->s[i].c0 != c) return isg_set_error(ISG_ERR_INVALID, "%s: sinks not contiguous", what);
        c += s->s[i].C;
    }
    if (c != M) return isg_set_error(ISG_ERR_INVALID, "%s: sinks cover %d of %d channels", what, c, M);
    return 0;
}

}  // namespace

int32_t isg_halo_conv_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                          const isg_sinks* out, hipStream_t st);
int32_t isg_pw_gemm(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                    const isg_sinks* out, bool dgrad, hipStream_t st);
int32_t isg_tap_conv(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                     const isg_sinks* out, bool dgrad, hipStream_t st);
int32_t isg_thin_conv(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                      const isg_sinks* out, bool dgrad, hipStream_t st);

static bool is_pointwise(const isg_conv_geom* g) {
    return g->KH == 1 && g->KW == 1 && g->SH == 1 && g->SW == 1 && g->PH == 0 && g->PW == 0 &&
           g->groups == 1 && g->Ci <= 256 && g->Co <= 256;
}

int32_t isg_down_conv_fwd(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                          const isg_sinks* out, hipStream_t st);
int32_t isg_s2k5_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                     const isg_sinks* out, hipStream_t st);
int32_t isg_sub2_dgrad(const isg_conv_geom* g, const isg_vtensor* dy, const float* w,
                       const isg_sinks* dx, hipStream_t st);

int32_t isg_dense_conv_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                           const isg_sinks* out, hipStream_t st) {
    if (vt_channels(x) != g->Ci) return isg_set_error(ISG_ERR_INVALID, "conv fwd: Ci mismatch");
    if (int32_t e = check_sinks(out, g->Co, "conv fwd")) return e;
    if (is_pointwise(g)) return isg_pw_gemm(g, x, w, out, false, st);
    {  // thin stride-1 convs on the VALU (thin_conv.hip)
        const int32_t t = isg_thin_conv(g, x, w, out, false, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    {  // k 2S, stride S: the sub-pixel convT's input gradient (down_conv.hip)
        const int32_t t = isg_down_conv_fwd(g, x, w, out, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    {  // 5x5 stride 2, <= 16 channels: the stem's second conv (down_conv.hip)
        const int32_t t = isg_s2k5_fwd(g, x, w, out, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    {  // dense spatial conv, <= 48 output channels (tap_conv.hip)
        const int32_t t = isg_tap_conv(g, x, w, out, false, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    // narrow outputs with spatial taps: LDS halo-tiled kernel (halo_conv.hip)
    {
        const int32_t h = isg_halo_conv_fwd(g, x, w, out, st);
        if (h != 0) return h < 0 ? h : 0;
    }
    if (g->Ci * g->KH * g->KW > kKtabMax)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv fwd: K=%d > %d", g->Ci * g->KH * g->KW, kKtabMax);
    if (int32_t e = check_sinks(out, g->Co, "conv fwd")) return e;
    GemmArgs a{};
    a.src = *x; a.out = *out; a.w = w; a.mode = 0; a.N = g->N;
    a.TH = g->OH; a.TW = g->OW; a.SrcH = g->H; a.SrcW = g->W; a.my = g->SH; a.mx = g->SW;
    a.DstH = g->OH; a.DstW = g->OW; a.dmy = 1; a.dmx = 1;
    a.M = g->Co; a.wrs = g->Ci * g->KH * g->KW;
    a.Ci = g->Ci; a.Co = g->Co; a.KH = g->KH; a.KW = g->KW; a.SH = g->SH; a.SW = g->SW;
    a.PH = g->PH; a.PW = g->PW; a.DH = g->DH; a.DW = g->DW; a.H = g->H; a.W = g->W;
    a.OH = g->OH; a.OW = g->OW;
    int64_t ntiles = ((int64_t)g->N * g->OH * g->OW + 15) / 16;
    return dispatch_gemm(a, dim3(num_blocks_for(ntiles)), st);
}

int32_t isg_dense_conv_dgrad(const isg_conv_geom* g, const isg_vtensor* dy, const float* w,
                             const isg_sinks* dx, hipStream_t st) {
    if (vt_channels(dy) != g->Co) return isg_set_error(ISG_ERR_INVALID, "conv dgrad: Co mismatch");
    if (int32_t e = check_sinks(dx, g->Ci, "conv dgrad")) return e;
    if (is_pointwise(g)) return isg_pw_gemm(g, dy, w, dx, true, st);
    {
        const int32_t t = isg_thin_conv(g, dy, w, dx, true, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    {  // 5x5 stride 2 as a sub-pixel transposed conv (down_conv.hip)
        const int32_t t = isg_sub2_dgrad(g, dy, w, dx, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    {
        const int32_t t = isg_tap_conv(g, dy, w, dx, true, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    if (g->KH > 16 || g->KW > 16) return isg_set_error(ISG_ERR_UNSUPPORTED, "conv dgrad: kernel > 16");
    const int maxk = g->Co * ((g->KH + g->SH - 1) / g->SH) * ((g->KW + g->SW - 1) / g->SW);
    if (maxk > kKtabMax) return isg_set_error(ISG_ERR_UNSUPPORTED, "conv dgrad: K=%d too large", maxk);
    if (int32_t e = check_sinks(dx, g->Ci, "conv dgrad")) return e;
    GemmArgs a{};
    a.src = *dy; a.out = *dx; a.w = w; a.mode = 1; a.N = g->N;
    a.TH = (g->H + g->SH - 1) / g->SH; a.TW = (g->W + g->SW - 1) / g->SW;
    a.SrcH = g->OH; a.SrcW = g->OW; a.my = 1; a.mx = 1;
    a.DstH = g->H; a.DstW = g->W; a.dmy = g->SH; a.dmx = g->SW;
    a.M = g->Ci; a.wrs = g->KH * g->KW;
    a.Ci = g->Ci; a.Co = g->Co; a.KH = g->KH; a.KW = g->KW; a.SH = g->SH; a.SW = g->SW;
    a.PH = g->PH; a.PW = g->PW; a.DH = g->DH; a.DW = g->DW; a.H = g->H; a.W = g->W;
    a.OH = g->OH; a.OW = g->OW;
    int64_t ntiles = ((int64_t)g->N * a.TH * a.TW + 15) / 16;
    return dispatch_gemm(a, dim3(num_blocks_for(ntiles), g->SH * g->SW), st);
}
