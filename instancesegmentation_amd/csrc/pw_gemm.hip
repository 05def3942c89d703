// Pointwise (1x1, stride 1) convolution as a GEMM on v_mfma_f32_16x16x4_f32 — the 50
// 1x1 convs of the reference (Conv(k=1) in every bottleneck, segment.py:59/69/89/101/
// 132/137/162/171/192/303/312/318, and the uppool 1x1s :323/:343), forward AND input
// gradient (the same GEMM with the weight read transposed).
//
//   D[m][p] = sum_k A[m][k] * Bv[k][p]     A[m][k] = w[m*rs + k*cs]
//     forward: m = co, k = ci (rs = Ci, cs = 1);  dgrad: m = ci, k = co (rs = 1, cs = Ci)
//
// A workgroup owns BM (64 or 128) rows x 64 pixels. K is processed in chunks of 32:
//   * activations: wave w stages channels w, w+4, ... of the chunk (wave-uniform channel,
//     lane = pixel, one coalesced 256-B row per load), the producer's BatchNorm/activation
//     (or BatchNorm-backward rebuild) applied on the way into LDS (stage.h records);
//   * weights: the BM x 32 slice, coalesced along whichever of m / k is contiguous.
// The MFMA loop is branch-free and reads both operands from LDS (padded strides: A rows
// = 2 mod 32 banks, B rows = 16 mod 32). The epilogue routes each output row through its
// sink (store + bias + BN statistics, accumulate, or activation backward with the
// BN-backward sums), resolved once per workgroup into LDS.
#include "stage.h"

namespace {

constexpr int kThreads = 256;
constexpr int kKC = 32;              // channels per K chunk
constexpr int kBP = 64;              // pixels per block
constexpr int kMaxBM = 128;
constexpr int kMaxK = 256;
constexpr int kWst = kKC + 2;        // Ws row stride (2 mod 32)
static_assert(kMaxBM * kWst >= 4 * 3 * kMaxBM, "BN partials alias the weight tile");
constexpr int kXst = kBP + 16;       // Xs row stride (16 mod 32)

struct PwArgs {
    isg_vtensor src;
    isg_sinks out;
    const float* w;
    int rs, cs;
    int N, HW, M, K, BM;
    int64_t P;
};

struct RowInfo {
    float* p;
    const float* y;
    int ns, yns;
    int mode, act;
    float bias;
    int pad_;
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

// TPW: 16x16 accumulator tiles per wave = (BM/16 row tiles x 4 pixel tiles) / 4 waves
template <int TPW>
__global__ __launch_bounds__(kThreads) void pw_kernel(PwArgs a) {
    __shared__ float Xs[kKC * kXst];
    __shared__ float Ws[kMaxBM * kWst];
    __shared__ ChT tab[kMaxK];
    __shared__ RowInfo ri[kMaxBM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = wave_id();
    const int kk = lane >> 4, pl = lane & 15;
    const int BM = a.BM;
    const int m0 = blockIdx.y * BM;
    const int Mb = min(BM, a.M - m0);
    const int64_t p0 = (int64_t)blockIdx.x * kBP;

    for (int c = tid; c < a.K; c += kThreads) tab[c] = ch_table_entry(a.src, c, a.HW);
    for (int r = tid; r < BM; r += kThreads) {
        const int m = m0 + r;
        RowInfo q = {};
        q.mode = -1;
        if (r < Mb) {
            const int s = sink_of(a.out, m);
            const isg_sink& k = s == 2 ? a.out.s[2] : (s == 1 ? a.out.s[1] : a.out.s[0]);
            const int cl = m - k.c0;
            q.p = k.p ? k.p + (int64_t)cl * a.HW : nullptr;
            q.y = k.y ? k.y + (int64_t)cl * a.HW : nullptr;
            q.ns = (int)k.n_stride;
            q.yns = (int)k.y_n_stride;
            q.mode = k.mode;
            q.act = k.act;
            q.bias = k.bias ? k.bias[cl] : 0.f;
            q.f = SinkCoef{0.f, 1.f, 0.f, 0.f};
            if (k.mode == ISG_SINK_ACTBWD) {
                if (k.bn.stats || !k.bn.train) {
                    const ChanCoef f = k.bn.coef ? fwd_coef(k.bn, nullptr, cl)
                                                 : coef_slow(k.bn, nullptr, cl, 0);
                    q.f.mean = f.c0; q.f.scale = f.c1; q.f.beta = f.c2;
                }
                q.f.slope = k.slope ? k.slope[cl] : 0.f;
            }
        }
        ri[r] = q;
    }

    // this lane's pixel of the block (staging) — the block never crosses an image when
    // HW % 64 == 0, otherwise per-lane image split
    const int64_t pg_l = p0 + lane;
    const bool pv_l = pg_l < a.P;
    const int n_l = pv_l ? (int)(pg_l / a.HW) : 0;
    const int pix_l = pv_l ? (int)(pg_l - (int64_t)n_l * a.HW) : 0;

    // accumulator tiles: t = wave + 4i -> row tile t>>2, pixel tile t&3
    int arow[TPW], bcol[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = wave + 4 * i;
        arow[i] = ((t >> 2) * 16 + pl) * kWst;
        bcol[i] = (t & 3) * 16 + pl;
    }
    f32x4 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

    const float* __restrict__ w = a.w;
    const bool wk_contig = a.cs == 1;  // weight row m contiguous along k (forward)
    for (int kc = 0; kc < a.K; kc += kKC) {
        const int kn = min(kKC, a.K - kc);
        __syncthreads();  // previous chunk consumed
        // activations: 8 channels per wave, all loads in flight together
        {
            float v[kKC / 4], yv[kKC / 4];
#pragma unroll
            for (int u = 0; u < kKC / 4; ++u) {
                const int k = min(wave + 4 * u, kn - 1);
                const ChT c = tab[kc + k];
                v[u] = gld(c.p, n_l * c.ns + pix_l);
                yv[u] = gld(c.y, n_l * c.yns + pix_l);
            }
#pragma unroll
            for (int u = 0; u < kKC / 4; ++u) {
                const int k = wave + 4 * u;
                const ChT c = tab[kc + min(k, kn - 1)];
                const float t = ch_xform(c.xf, c.act, c.k, v[u], yv[u]);
                Xs[k * kXst + lane] = (k < kn && pv_l) ? t : 0.f;
            }
        }
        // weights: BM x 32 slice (rows past Mb and k past kn are zero)
        for (int idx = tid; idx < BM * kKC; idx += kThreads) {
            int m, k;
            if (wk_contig) { m = idx / kKC; k = idx - m * kKC; }
            else { k = idx / BM; m = idx - k * BM; }
            float v = 0.f;
            if (m < Mb && k < kn) v = gld(w, (int64_t)(m0 + m) * a.rs + (int64_t)(kc + k) * a.cs);
            Ws[m * kWst + k] = v;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < kKC / 4; ++ks) {
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                const float av = Ws[arow[i] + ks * 4 + kk];
                const float bv = Xs[(ks * 4 + kk) * kXst + bcol[i]];
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i], 0, 0, 0);
            }
        }
    }

    // ---- epilogue: lane holds D[row = rt*16 + kk*4 + r][pixel = ct*16 + pl] ------------
    const bool need_red = sinks_need_red(a.out);
    // per-wave BN partials [4 waves][3][BM] (fixed-order sum: deterministic statistics),
    // in the weight tile's LDS, free once every wave is past the K loop
    float (*red)[3][kMaxBM] = reinterpret_cast<float (*)[3][kMaxBM]>(Ws);
    if (need_red) {
        __syncthreads();
        for (int i = tid; i < 4 * 3 * kMaxBM; i += kThreads) (&red[0][0][0])[i] = 0.f;
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = wave + 4 * i;
        const int rt = t >> 2, ct = t & 3;
        if (rt * 16 >= Mb) continue;  // wave-uniform
        const int64_t pg = p0 + ct * 16 + pl;
        const bool pv = pg < a.P;
        const int n = pv ? (int)(pg / a.HW) : 0;
        const int pix = pv ? (int)(pg - (int64_t)n * a.HW) : 0;
        float s0[4], s1[4], s2[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            s0[r] = s1[r] = s2[r] = 0.f;
            const int rl = rt * 16 + kk * 4 + r;
            const RowInfo& q = ri[rl];
            if (!pv || q.mode < 0 || q.mode == ISG_SINK_NONE) continue;
            float v = acc[i][r];
            const int off = n * q.ns + pix;
            if (q.mode == ISG_SINK_STORE) {
                v += q.bias;
                gst(q.p, off, v);
                s0[r] = v;
                s1[r] = v * v;
            } else if (q.mode == ISG_SINK_ACCUM) {
                gst(q.p, off, gld(q.p, off) + v);
                s0[r] = v;
                s1[r] = v * v;
            } else {
                const float y = gld(q.y, n * q.yns + pix);
                const float z = (y - q.f.mean) * q.f.scale + q.f.beta;
                float gv = v;
                if (q.act == ISG_ACT_RELU) {
                    gv = z > 0.f ? v : 0.f;
                } else if (q.act == ISG_ACT_PRELU) {
                    gv = z > 0.f ? v : v * q.f.slope;
                    s2[r] = z > 0.f ? 0.f : z * v;
                }
                gst(q.p, off, gv);
                s0[r] = gv;
                s1[r] = gv * (y - q.f.mean);
            }
        }
        if (need_red) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float t0 = row16_sum(s0[r]);
                const float t1 = row16_sum(s1[r]);
                const float t2 = row16_sum(s2[r]);
                const int rl = rt * 16 + kk * 4 + r;
                if (pl == 0 && rl < Mb) {
                    red[wave][0][rl] = t0;  // one tile per (wave, row)
                    red[wave][1][rl] = t1;
                    red[wave][2][rl] = t2;
                }
            }
        }
    }
    if (need_red) {
        __syncthreads();
        for (int rl = tid; rl < Mb; rl += kThreads) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
                red[0][j][rl] = ((red[0][j][rl] + red[1][j][rl]) + red[2][j][rl]) + red[3][j][rl];
            const int m = m0 + rl;
            const int s = sink_of(a.out, m);
            const isg_sink& k = s == 2 ? a.out.s[2] : (s == 1 ? a.out.s[1] : a.out.s[0]);
            const int cl = m - k.c0;
            if (k.mode == ISG_SINK_STORE || k.mode == ISG_SINK_ACCUM) {
                if (k.stats) {
                    double* sp = rep_ptr(k.stats, 4 * k.C);
                    atomicAdd(&sp[cl], (double)red[0][0][rl]);
                    atomicAdd(&sp[k.C + cl], (double)red[0][1][rl]);
                }
            } else if (k.mode == ISG_SINK_ACTBWD) {
                if (k.bn.stats) {
                    double* sp = rep_ptr(k.bn.stats, 4 * k.C);
                    atomicAdd(&sp[2 * k.C + cl], (double)red[0][0][rl]);
                    atomicAdd(&sp[3 * k.C + cl], (double)red[0][1][rl]);
                }
                if (k.slope_grad && k.act == ISG_ACT_PRELU)
                    atomicAdd(&rep_ptr(k.slope_grad, k.C)[cl], (double)red[0][2][rl]);
            }
        }
    }
    sinks_finalize(a.out);
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
    if (a.K > kMaxK)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "pw gemm: K = %d channels > %d", a.K, kMaxK);
    if (a.M > 2 * kMaxBM)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "pw gemm: M = %d rows", a.M);
    const int64_t pblocks = (a.P + kBP - 1) / kBP;
    // rows per block: up to 128, halved while that keeps more workgroups in flight
    int bm = std::min(kMaxBM, (a.M + 15) / 16 * 16);
    while (bm > 16 && pblocks * ((a.M + bm - 1) / bm) < 512) bm = (bm / 2 + 15) / 16 * 16;
    a.BM = bm;
    const int tpw = bm / 16;  // (bm/16 row tiles * 4 pixel tiles) / 4 waves
    dim3 grid((unsigned)pblocks, (unsigned)((a.M + bm - 1) / bm));
    // template tile count >= tpw; surplus tiles compute on unused rows, never stored
    switch (tpw) {
        case 1: hipLaunchKernelGGL(pw_kernel<1>, grid, dim3(kThreads), 0, st, a); break;
        case 2: hipLaunchKernelGGL(pw_kernel<2>, grid, dim3(kThreads), 0, st, a); break;
        case 3: hipLaunchKernelGGL(pw_kernel<3>, grid, dim3(kThreads), 0, st, a); break;
        case 4: hipLaunchKernelGGL(pw_kernel<4>, grid, dim3(kThreads), 0, st, a); break;
        case 5: case 6: hipLaunchKernelGGL(pw_kernel<6>, grid, dim3(kThreads), 0, st, a); break;
        default: hipLaunchKernelGGL(pw_kernel<8>, grid, dim3(kThreads), 0, st, a); break;
    }
    if (out->fin_counter) isg_fin_note_handled();
    return isg_check_launch("pw_kernel");
}
