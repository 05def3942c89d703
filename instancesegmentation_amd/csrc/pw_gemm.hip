// Pointwise (1x1, stride 1) convolution as a GEMM on v_mfma_f32_16x16x4_f32 — the 50
// 1x1 convs of the reference (Conv(k=1) in every bottleneck, segment.py:59/69/89/101/
// 132/137/162/171/192/303/312/318, and the uppool 1x1s :323/:343), forward AND input
// gradient (the same GEMM with the weight read transposed).
//
//   D[m][p] = sum_k A[m][k] * Bv[k][p]     A[m][k] = w[m*rs + k*cs]
//     forward: m = co, k = ci (rs = Ci, cs = 1);  dgrad: m = ci, k = co (rs = 1, cs = Ci)
//
// A workgroup owns a BM x BP tile (BM rows = WM waves x 16*MT, BP pixels = WP waves x
// 16*GP). The activation tile is staged once into LDS in 64-channel chunks with the
// producer's BN/activation (or BN-backward rebuild) applied on load, coalesced along
// pixels; waves read B fragments from LDS and A fragments (weights, L1/L2-resident)
// from global. Sink routing per output row (segment / mode / BN coefficients) is
// resolved once per workgroup into LDS so the epilogue is branch-light.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kKC = 32;        // channels per LDS chunk
constexpr int kMaxCh = 256;    // M, K limit (larger shapes take the generic path)
constexpr int kMaxBM = 128;
constexpr int kMaxBP = 128;

struct PwArgs {
    isg_vtensor src;
    isg_sinks out;
    const float* w;
    int rs, cs;
    int N, HW, M, K;
    int WM, WP;
    int64_t P;
};

struct RowInfo {
    float* p;
    const float* y;
    int64_t ns, yns;
    int mode, act, sink;
    float bias;
    SinkCoef f;
};

ISG_DEV float row16_sum(float v) {
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

template <int MT, int GP>
__global__ __launch_bounds__(kThreads) void pw_kernel(PwArgs a) {
    constexpr int XST = kMaxBP + 4;
    __shared__ float Xs[kKC][XST];
    __shared__ ChanCoef coef[kMaxCh];
    __shared__ RowInfo ri[kMaxBM];
    __shared__ SinkCoef scoef[kMaxCh];
    __shared__ float red[3][kMaxBM];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kk = lane >> 4, pl = lane & 15;
    const int BM = a.WM * 16 * MT, BP = a.WP * 16 * GP;
    const int m0 = blockIdx.y * BM;
    const int64_t p0 = (int64_t)blockIdx.x * BP;
    const int wm = wave % a.WM, wp = wave / a.WM;
    const bool active = wp < a.WP;

    load_vt_coefs(a.src, coef, tid, kThreads);
    load_sink_coefs(a.out, scoef, tid, kThreads);
    __syncthreads();
    for (int r = tid; r < BM; r += kThreads) {
        const int m = m0 + r;
        RowInfo q = {};
        q.mode = -1;
        if (m < a.M) {
            const int s = sink_of(a.out, m);
            const isg_sink& k = a.out.s[s];
            const int cl = m - k.c0;
            q.p = k.p ? k.p + (int64_t)cl * a.HW : nullptr;
            q.y = k.y ? k.y + (int64_t)cl * a.HW : nullptr;
            q.ns = k.n_stride;
            q.yns = k.y_n_stride;
            q.mode = k.mode;
            q.act = k.act;
            q.sink = s;
            q.bias = k.bias ? k.bias[cl] : 0.f;
            q.f = scoef[m];
        }
        ri[r] = q;
        red[0][r] = red[1][r] = red[2][r] = 0.f;
    }

    f32x4 acc[GP][MT];
#pragma unroll
    for (int g = 0; g < GP; ++g)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const float* __restrict__ w = a.w;
    for (int kc = 0; kc < a.K; kc += kKC) {
        const int kn = min(kKC, a.K - kc);
        __syncthreads();
        for (int idx = tid; idx < kn * BP; idx += kThreads) {
            const int k = idx / BP, pp = idx - k * BP;
            const int64_t pg = p0 + pp;
            float v = 0.f;
            if (pg < a.P) {
                const int n = (int)(pg / a.HW);
                v = vt_load(a.src, coef, n, kc + k, a.HW, pg - (int64_t)n * a.HW);
            }
            Xs[k][pp] = v;
        }
        __syncthreads();
        if (active) {
#pragma unroll 4
            for (int k0 = 0; k0 < kn; k0 += 4) {
                const int k = k0 + kk;
                const bool kv = k < kn;
                float av[MT];
#pragma unroll
                for (int t = 0; t < MT; ++t) {
                    const int m = m0 + wm * 16 * MT + t * 16 + pl;
                    av[t] = (kv && m < a.M) ? w[(int64_t)m * a.rs + (int64_t)(kc + k) * a.cs] : 0.f;
                }
#pragma unroll
                for (int g = 0; g < GP; ++g) {
                    const float bv = kv ? Xs[k][wp * 16 * GP + g * 16 + pl] : 0.f;
#pragma unroll
                    for (int t = 0; t < MT; ++t)
                        acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], bv, acc[g][t], 0, 0, 0);
                }
            }
        }
    }

    // ---- epilogue ----------------------------------------------------------------------
    if (active) {
        float s0[MT][4], s1[MT][4], s2[MT][4];
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) s0[t][r] = s1[t][r] = s2[t][r] = 0.f;
#pragma unroll
        for (int g = 0; g < GP; ++g) {
            const int64_t pg = p0 + wp * 16 * GP + g * 16 + pl;
            const bool pv = pg < a.P;
            const int n = pv ? (int)(pg / a.HW) : 0;
            const int64_t pix = pg - (int64_t)n * a.HW;
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int rl = wm * 16 * MT + t * 16 + kk * 4 + r;
                    const RowInfo& q = ri[rl];
                    if (!pv || q.mode < 0 || q.mode == ISG_SINK_NONE) continue;
                    float v = acc[g][t][r];
                    float* dst = q.p + (int64_t)n * q.ns + pix;
                    if (q.mode == ISG_SINK_STORE) {
                        v += q.bias;
                        *dst = v;
                        s0[t][r] += v;
                        s1[t][r] += v * v;
                    } else if (q.mode == ISG_SINK_ACCUM) {
                        *dst += v;
                        s0[t][r] += v;
                        s1[t][r] += v * v;
                    } else {
                        const float y = q.y[(int64_t)n * q.yns + pix];
                        const float z = (y - q.f.mean) * q.f.scale + q.f.beta;
                        float gv = v;
                        if (q.act == ISG_ACT_RELU) {
                            gv = z > 0.f ? v : 0.f;
                        } else if (q.act == ISG_ACT_PRELU) {
                            gv = z > 0.f ? v : v * q.f.slope;
                            s2[t][r] += z > 0.f ? 0.f : z * v;
                        }
                        *dst = gv;
                        s0[t][r] += gv;
                        s1[t][r] += gv * (y - q.f.mean);
                    }
                }
        }
        if (sinks_need_red(a.out)) {
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t0 = row16_sum(s0[t][r]);
                    const float t1 = row16_sum(s1[t][r]);
                    const float t2 = row16_sum(s2[t][r]);
                    const int rl = wm * 16 * MT + t * 16 + kk * 4 + r;
                    if (pl == 0 && m0 + rl < a.M) {
                        atomicAdd(&red[0][rl], t0);
                        atomicAdd(&red[1][rl], t1);
                        atomicAdd(&red[2][rl], t2);
                    }
                }
        }
    }
    if (sinks_need_red(a.out)) {
        __syncthreads();
        for (int rl = tid; rl < BM; rl += kThreads) {
            const int m = m0 + rl;
            if (m >= a.M) continue;
            const int s = sink_of(a.out, m);
            const isg_sink& k = a.out.s[s];
            const int cl = m - k.c0;
            if (k.mode == ISG_SINK_STORE || k.mode == ISG_SINK_ACCUM) {
                if (k.stats) {
                    double* sp = rep_ptr(k.stats, 4 * k.C);
                    atomicAdd(&sp[cl], (double)red[0][rl]);
                    atomicAdd(&sp[k.C + cl], (double)red[1][rl]);
                }
            } else if (k.mode == ISG_SINK_ACTBWD) {
                if (k.bn.stats) {
                    double* sp = rep_ptr(k.bn.stats, 4 * k.C);
                    atomicAdd(&sp[2 * k.C + cl], (double)red[0][rl]);
                    atomicAdd(&sp[3 * k.C + cl], (double)red[1][rl]);
                }
                if (k.slope_grad && k.act == ISG_ACT_PRELU)
                    atomicAdd(&rep_ptr(k.slope_grad, k.C)[cl], (double)red[2][rl]);
            }
        }
    }
}

}  // namespace

// 1x1 stride-1 GEMM. dgrad=false: rows = Co (w[co][ci]); dgrad=true: rows = Ci.
int32_t isg_pw_gemm(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                    const isg_sinks* out, bool dgrad, hipStream_t st) {
    PwArgs a{};
    a.src = *src;
    a.out = *out;
    a.w = w;
    a.N = g->N;
    a.HW = g->H * g->W;
    a.M = dgrad ? g->Ci : g->Co;
    a.K = dgrad ? g->Co : g->Ci;
    a.rs = dgrad ? 1 : g->Ci;
    a.cs = dgrad ? g->Ci : 1;
    a.P = (int64_t)g->N * a.HW;
    if (a.K > kMaxCh || a.M > kMaxCh)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "pw gemm: %d x %d channels", a.M, a.K);
    // shape the workgroup: rows first (MT = 2 when there are >= 32 rows), then pixels
    const int mt = a.M > 16 ? 2 : 1;
    const int mtiles = (a.M + 16 * mt - 1) / (16 * mt);
    a.WM = mtiles >= 4 ? 4 : (mtiles >= 2 ? 2 : 1);
    a.WP = 4 / a.WM;
    // pixels per wave: 32 when the grid stays large, else 16
    const int64_t blocks32 = ((a.P + a.WP * 32 - 1) / (a.WP * 32)) *
                             ((a.M + a.WM * 16 * mt - 1) / (a.WM * 16 * mt));
    const int gp = blocks32 >= 512 ? 2 : 1;
    const int BM = a.WM * 16 * mt, BP = a.WP * 16 * gp;
    dim3 grid((unsigned)((a.P + BP - 1) / BP), (unsigned)((a.M + BM - 1) / BM));
    if (mt == 1 && gp == 1) hipLaunchKernelGGL((pw_kernel<1, 1>), grid, dim3(kThreads), 0, st, a);
    else if (mt == 1) hipLaunchKernelGGL((pw_kernel<1, 2>), grid, dim3(kThreads), 0, st, a);
    else if (gp == 1) hipLaunchKernelGGL((pw_kernel<2, 1>), grid, dim3(kThreads), 0, st, a);
    else hipLaunchKernelGGL((pw_kernel<2, 2>), grid, dim3(kThreads), 0, st, a);
    return isg_check_launch("pw_kernel");
}
