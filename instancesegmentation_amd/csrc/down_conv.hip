// The backward of the sub-pixel ConvTranspose2d (kernel 2S, stride S, pad S/2;
// segment.py:305-306 k4 s2 p1 and the mask head's k8 s4 p2, :435-436) on the VALU. Both
// directions are "down" convolutions with kernel 2S, stride S, pad S/2 over the
// convT's output gradient dy (C channels, S x the resolution):
//
//   input gradient  dx[m][i][j] = sum_{c,kh,kw} W[m][c][kh][kw] * dy[c][S*i - S/2 + kh][S*j - S/2 + kw]
//   weight gradient dW[m][c][kh][kw] += sum_{n,i,j} x[m][i][j] * dy[c][S*i - S/2 + kh][S*j - S/2 + kw]
//
// with W = the convT weight [M = in channels][C = out channels][2S][2S], x its input.
// The plan issues them as a stride-S conv (OP_CONV_FWD) and its weight gradient
// (OP_CONV_WGRAD); tap_conv stages at most stride 2 and the generic kernels ran the head's
// pair at 67 / 90 us (1.07 GFLOP each at bs2 1024^2).
//
// down_conv_kernel: one lane per input cell (i, j), all M <= 16 outputs in registers; the
// cell's C x 2S x 2S patch is read row by row with 16-B loads (the producer's transform
// applied, zero outside the plane) and multiplied by weights kept in LDS as
// [c][kh][kw][m] (4 outputs per broadcast ds_read_b128). The epilogue routes every output
// channel through its sink (stage.h SinkRow) with the BN-backward sums reduced per
// workgroup.
// down_wgrad_kernel: persistent workgroups over tiles of TY x TX cells; per tile the x
// values (with the transform) and the dy patch region go to LDS; lane t owns GEMM column
// t = (c, kh, kw) and accumulates its M outputs across all of the workgroup's tiles; one
// atomic per dW element per workgroup into one of nrep replicas.
#include <algorithm>

#include "stage.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxM = 16;
constexpr int kMaxC = 4;

struct DownArgs {
    isg_vtensor dy;    // C channels, Hd x Wd (= S x the cell grid)
    isg_vtensor x;     // wgrad: M channels, cell grid H x W
    isg_sinks out;     // input gradient: M channels on the cell grid
    const float* w;    // [M][C][2S][2S]
    double* dw;
    int64_t rep_stride;
    int nrep;
    int N, M, C, H, W;  // cell grid
    int tiles_x, ntiles;
};

// one 2S-wide patch row of channel table entry t at source row r, columns S*j - S/2 ..
// S*j + 3S/2 - 1, transformed, zero outside the plane (after the transform)
template <int S>
ISG_DEV void patch_row(const ChT& t, int n, int r, int j, int Hd, int Wd, float (&v)[2 * S]) {
    const bool rok = (unsigned)r < (unsigned)Hd;
    const int64_t row = (int64_t)(rok ? r : 0) * Wd;
    const float* xp = t.p + (int64_t)n * t.ns + row;
    const float* yp = t.y + (int64_t)n * t.yns + row;
    const bool bwd = t.xf == ISG_XF_BN_BWD;
    // aligned 16-B / 8-B pieces covering [S*j - S, S*j + 2S): use elements S/2 .. S/2+2S-1
    const int c0 = S * j - S;
    float raw[3 * S], ry[3 * S];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int c = c0 + q * S;
        const bool cok = rok && c >= 0 && c < Wd;
        const int cc = cok ? c : 0;
        if constexpr (S == 4) {
            const f32x4 a = gld4(xp, cc);
            const f32x4 b = bwd ? gld4(yp, cc) : a;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                raw[q * 4 + e] = cok ? a[e] : 0.f;
                ry[q * 4 + e] = b[e];
            }
        } else {
            const float a0 = gld(xp, cc), a1 = gld(xp, cc + (cok ? 1 : 0));
            const float b0 = bwd ? gld(yp, cc) : a0, b1 = bwd ? gld(yp, cc + (cok ? 1 : 0)) : a1;
            raw[q * 2] = cok ? a0 : 0.f;
            raw[q * 2 + 1] = cok ? a1 : 0.f;
            ry[q * 2] = b0;
            ry[q * 2 + 1] = b1;
        }
    }
#pragma unroll
    for (int e = 0; e < 2 * S; ++e) {
        const int k = S / 2 + e;
        const int col = c0 + k;
        const bool ok = rok && col >= 0 && col < Wd;
        v[e] = ok ? ch_xform_u(t.xf, t.act, t.k, raw[k], ry[k]) : 0.f;
    }
}

template <int S, int M>
__global__ __launch_bounds__(kThreads) void down_conv_kernel(DownArgs a) {
    constexpr int K = 2 * S;
    constexpr int M4 = (M + 3) / 4;
    __shared__ f32x4 wl[kMaxC * K * K * M4];  // [c][kh][kw][m/4]
    __shared__ ChT tab[kMaxC];
    __shared__ SinkRow ri[kMaxM];
    __shared__ float red[4][3][kMaxM];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int Hd = a.H * S, Wd = a.W * S;
    if (tid < a.C) tab[tid] = ch_table_entry(a.dy, tid, (int64_t)Hd * Wd);
    if (tid < a.M) ri[tid] = sink_row(a.out, tid, (int64_t)a.H * a.W);
    float* const wf = reinterpret_cast<float*>(wl);
    for (int i = tid; i < a.C * K * K * M4 * 4; i += kThreads) {
        const int m = i % (M4 * 4), r = i / (M4 * 4);  // r = (c*K + kh)*K + kw
        const int c = r / (K * K), tap = r - c * K * K;
        wf[i] = m < a.M ? gld(a.w, ((int64_t)m * a.C + c) * K * K + tap) : 0.f;
    }
    __syncthreads();
    const int64_t hw = (int64_t)a.H * a.W;
    const int64_t cell = (int64_t)blockIdx.x * kThreads + tid;
    const bool pv = cell < (int64_t)a.N * hw;
    const int64_t cc = pv ? cell : 0;
    const int n = (int)(cc / hw);
    const int64_t pix = cc - (int64_t)n * hw;
    const int i = (int)(pix / a.W), j = (int)(pix - (int64_t)i * a.W);
    f32x4 acc[M4];
#pragma unroll
    for (int q = 0; q < M4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < a.C; ++c) {
        const ChT t = tab[c];
#pragma unroll 2
        for (int kh = 0; kh < K; ++kh) {
            float v[K];
            patch_row<S>(t, n, S * i - S / 2 + kh, j, Hd, Wd, v);
            const f32x4* wr = wl + ((c * K + kh) * K) * M4;
#pragma unroll
            for (int kw = 0; kw < K; ++kw)
#pragma unroll
                for (int q = 0; q < M4; ++q) acc[q] += wr[kw * M4 + q] * v[kw];
        }
    }
    float s0[M], s1[M], s2[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        s0[m] = s1[m] = s2[m] = 0.f;
        if (pv && m < a.M) sink_row_apply(ri[m], n, pix, acc[m >> 2][m & 3], s0[m], s1[m], s2[m]);
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
        if (tid < a.M) {
            float r3[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) r3[q] = ((red[0][q][tid] + red[1][q][tid]) + red[2][q][tid]) + red[3][q][tid];
            sink_row_flush(a.out, tid, r3[0], r3[1], r3[2]);
        }
    }
}

// weight gradient: tiles of TY x TX cells; lane t = column (c, kh, kw) < C*K*K <= 256
template <int S, int M, int TY, int TX>
__global__ __launch_bounds__(kThreads) void down_wgrad_kernel(DownArgs a) {
    constexpr int K = 2 * S;
    constexpr int M4 = (M + 3) / 4;
    constexpr int NC = TY * TX;                       // cells per tile
    constexpr int RH = S * TY + S, RW = S * TX + S;   // dy region rows / cols per channel
    __shared__ f32x4 xl[NC * M4];                     // [cell][m/4]
    __shared__ float dl[kMaxC * RH * RW];             // [c][row][col]
    __shared__ ChT tx[kMaxM], ty[kMaxC];
    const int tid = threadIdx.x;
    const int Hd = a.H * S, Wd = a.W * S;
    const int64_t hw = (int64_t)a.H * a.W;
    if (tid < a.M) tx[tid] = ch_table_entry(a.x, tid, hw);
    if (tid < a.C) ty[tid] = ch_table_entry(a.dy, tid, (int64_t)Hd * Wd);
    const int ncol = a.C * K * K;
    const int col = min(tid, ncol - 1);
    const int c = col / (K * K), tap = col - c * K * K, kh = tap / K, kw = tap - kh * K;
    const int coff = (c * RH + kh) * RW + kw;  // + S*(cy*RW + cx) per cell
    f32x4 acc[M4];
#pragma unroll
    for (int q = 0; q < M4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int tpi = a.tiles_x * ((a.H + TY - 1) / TY);
    for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
        const int n = tile / tpi, tr = tile - n * tpi;
        const int tyi = tr / a.tiles_x;
        const int i0 = tyi * TY, j0 = (tr - tyi * a.tiles_x) * TX;
        __syncthreads();  // previous tile consumed (and the channel tables written)
        // x values of the tile's cells (zero past the grid)
        float* const xf = reinterpret_cast<float*>(xl);
        for (int e = tid; e < NC * M4 * 4; e += kThreads) {
            const int cell = e / (M4 * 4), m = e - cell * (M4 * 4);
            const int ci = i0 + cell / TX, cj = j0 + cell % TX;
            float v = 0.f;
            if (m < a.M && ci < a.H && cj < a.W) {
                const ChT t = tx[m];
                const int64_t o = (int64_t)ci * a.W + cj;
                const float raw = gld(t.p, (int64_t)n * t.ns + o);
                const float yy = t.xf == ISG_XF_BN_BWD ? gld(t.y, (int64_t)n * t.yns + o) : raw;
                v = ch_xform(t.xf, t.act, t.k, raw, yy);
            }
            xf[e] = v;
        }
        // dy region rows S*i0 - S/2 .., cols S*j0 - S/2 .. (zero outside the plane)
        const int r0 = S * i0 - S / 2, q0 = S * j0 - S / 2;
        for (int e = tid; e < a.C * RH * RW; e += kThreads) {
            const int ch = e / (RH * RW), rem = e - ch * RH * RW;
            const int rr = rem / RW, qq = rem - rr * RW;
            const int r = r0 + rr, q = q0 + qq;
            float v = 0.f;
            if ((unsigned)r < (unsigned)Hd && (unsigned)q < (unsigned)Wd) {
                const ChT t = ty[ch];
                const int64_t o = (int64_t)r * Wd + q;
                const float raw = gld(t.p, (int64_t)n * t.ns + o);
                const float yy = t.xf == ISG_XF_BN_BWD ? gld(t.y, (int64_t)n * t.yns + o) : raw;
                v = ch_xform(t.xf, t.act, t.k, raw, yy);
            }
            dl[e] = v;
        }
        __syncthreads();
#pragma unroll 4
        for (int cell = 0; cell < NC; ++cell) {
            const int cy = cell / TX, cx = cell - cy * TX;
            const float d = dl[coff + S * (cy * RW + cx)];
#pragma unroll
            for (int q = 0; q < M4; ++q) acc[q] += xl[cell * M4 + q] * d;
        }
    }
    if (tid < ncol) {
        double* const dwr = a.dw + (int64_t)(blockIdx.x % (unsigned)a.nrep) * a.rep_stride;
#pragma unroll
        for (int m = 0; m < M; ++m)
            if (m < a.M) atomicAdd(&dwr[((int64_t)m * a.C + c) * K * K + tap], acc[m >> 2][m & 3]);
    }
}

// ---- input gradient of a stride-2 conv with an odd kernel K, pad K/2 (the stem's second
// 5x5 s2 conv, segment.py:26) as a sub-pixel transposed conv -----------------------------
//   dx[m][2i+a][2j+b] = sum_c sum_{kh = a+P mod 2} sum_{kw = b+P mod 2}
//                       W[c][m][kh][kw] * dy[c][(2i+a+P-kh)/2][(2j+b+P-kw)/2]
// Every output pixel of the 2x2 block of cell (i, j) reads dy inside the cell's
// (P+1)^2 neighbourhood, so one staging of dy serves all four phases (the tap_conv route
// stages the same dy once per phase, four times over: 99 us; a VALU form with a lane per
// cell and the weights broadcast from LDS: 85 us; this MFMA form: 67 us).

// sink_row_apply on two horizontally adjacent outputs (pix even, 8-B aligned): one 8-B
// load of the sink operand and one 8-B store instead of two stride-2 accesses
typedef float v2f_t __attribute__((ext_vector_type(2)));
typedef const v2f_t __attribute__((address_space(1)))* gcv2_p;
typedef v2f_t __attribute__((address_space(1)))* gv2_p;
ISG_DEV void sink_row_apply2(const SinkRow& q, int n, int64_t pix, float v0, float v1, float& s0,
                             float& s1, float& s2) {
    const int64_t off = (int64_t)n * q.ns + pix;
    if (q.mode == ISG_SINK_STORE) {
        v0 += q.bias;
        v1 += q.bias;
        *(gv2_p)((gfloat_p)q.p + off) = v2f_t{v0, v1};
        s0 = v0 + v1;
        s1 = v0 * v0 + v1 * v1;
    } else if (q.mode == ISG_SINK_ACCUM) {
        const v2f_t o = *(gcv2_p)((gcfloat_p)q.p + off);
        *(gv2_p)((gfloat_p)q.p + off) = v2f_t{o[0] + v0, o[1] + v1};
        s0 = v0 + v1;
        s1 = v0 * v0 + v1 * v1;
    } else if (q.mode == ISG_SINK_ACTBWD) {
        const v2f_t y = *(gcv2_p)((gcfloat_p)q.y + (int64_t)n * q.yns + pix);
        float g[2];
        const float v[2] = {v0, v1};
        s0 = s1 = s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float z = (y[e] - q.f.mean) * q.f.scale + q.f.beta;
            float gv = v[e];
            if (q.act == ISG_ACT_RELU) {
                gv = z > 0.f ? v[e] : 0.f;
            } else if (q.act == ISG_ACT_PRELU) {
                gv = z > 0.f ? v[e] : v[e] * q.f.slope;
                s2 += z > 0.f ? 0.f : z * v[e];
            }
            g[e] = gv;
            s0 += gv;
            s1 += gv * (y[e] - q.f.mean);
        }
        *(gv2_p)((gfloat_p)q.p + off) = v2f_t{g[0], g[1]};
    }
}

constexpr int kRowsPB = 4;  // dy rows per workgroup (measured: 1 row 81 us, 2 76, 4 67, 8 102)

// The input gradient as an MFMA GEMM (v_mfma_f32_16x16x4_f32): a wave owns 16 consecutive
// cells of one dy row and all 4 phases x 16 outputs of their 2x2 blocks; K runs over
// (channel group of 4, tap): A[m][k] = W[4g + k][m][kh][kw], B[k][cell] = the transformed
// dy value of channel 4g + k at the tap's neighbour of the cell; one MFMA per (group, tap)
// into the tap's phase accumulator. The workgroup's dy band — kRowsPB + 2 rows x (64 + 2)
// columns x 16 channels — is loaded ONCE with 16-B loads, transformed once per element
// (BatchNorm backward rebuilt from g and the saved y) and zero-padded into LDS; the MFMA
// B operands are then conflict-free ds_read_b32 (channel planes 16 mod 32 banks apart).
// (Round 2's direct form, operands straight from L2, re-read every dy element in up to 9
// lanes and re-transformed it each time: 61 % of wave cycles waiting, removed in round 5.)
constexpr int kSubRS = 72;                 // staged row: column x at x - (j0 - 4), 0..68
constexpr int kSubPL = 432;                // channel plane (>= (kRowsPB + 2) * 72, 16 mod 32)
static_assert(kSubPL >= (kRowsPB + 2) * kSubRS && kSubPL % 32 == 16, "staging plane");


// Round 5: ONE memory round trip before the MFMAs — the band's interior quads and halo
// columns (addresses straight from the kernel argument for a one-segment dy, the stem's
// case), the weight, the coefficient and sink-row tables are all issued before the first
// barrier (round 4: table + weight, then the band, then the halo columns, three trips) —
// and each dy row's sink operands (the saved forward output of the ACTBWD sink) are loaded
// before that row's MFMAs, not between them and the stores.
ISG_DEV void sink_row_apply2_pre(const SinkRow& q, int n, int64_t pix, float v0, float v1,
                                 v2f_t pre, float& s0, float& s1, float& s2) {
    const int64_t off = (int64_t)n * q.ns + pix;
    if (q.mode == ISG_SINK_STORE) {
        v0 += q.bias;
        v1 += q.bias;
        *(gv2_p)((gfloat_p)q.p + off) = v2f_t{v0, v1};
        s0 = v0 + v1;
        s1 = v0 * v0 + v1 * v1;
    } else if (q.mode == ISG_SINK_ACCUM) {
        *(gv2_p)((gfloat_p)q.p + off) = v2f_t{pre[0] + v0, pre[1] + v1};
        s0 = v0 + v1;
        s1 = v0 * v0 + v1 * v1;
    } else if (q.mode == ISG_SINK_ACTBWD) {
        float g[2];
        const float v[2] = {v0, v1};
        s0 = s1 = s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float z = (pre[e] - q.f.mean) * q.f.scale + q.f.beta;
            float gv = v[e];
            if (q.act == ISG_ACT_RELU) {
                gv = z > 0.f ? v[e] : 0.f;
            } else if (q.act == ISG_ACT_PRELU) {
                gv = z > 0.f ? v[e] : v[e] * q.f.slope;
                s2 += z > 0.f ? 0.f : z * v[e];
            }
            g[e] = gv;
            s0 += gv;
            s1 += gv * (pre[e] - q.f.mean);
        }
        *(gv2_p)((gfloat_p)q.p + off) = v2f_t{g[0], g[1]};
    }
}

__global__ __launch_bounds__(kThreads) void sub2_dgrad_lds_kernel(DownArgs a) {
    constexpr int K = 5, P = 2, R0 = 1;
    __shared__ float wl[kMaxM * kMaxM * K * K];  // [c][m][kh][kw] (the weight's own layout)
    __shared__ __attribute__((aligned(16))) float Ls[kMaxM * kSubPL];  // [c][row][col] dy band
    __shared__ XfLin lin[kMaxM];
    __shared__ SinkRow ri[kMaxM];
    __shared__ float red[4][3][kMaxM];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kq = lane >> 4, pl = lane & 15;
    const int Hs = a.H, Ws = a.W, Wd = 2 * Ws;
    const int64_t HWs = (int64_t)Hs * Ws;
    const int n = blockIdx.z, j0 = blockIdx.x * 64, i0 = blockIdx.y * kRowsPB;
    STAMP(0);
    // ---- every load of the prologue in one round trip ------------------------------------
    constexpr int NQ = kMaxM * (kRowsPB + 2) * 16;  // (c, row, quad) interior quads
    constexpr int U = NQ / kThreads;
    static_assert(NQ % kThreads == 0, "staging split");
    constexpr int NH = kMaxM * (kRowsPB + 2) * 2;   // (c, row, side) halo columns
    static_assert(NH <= kThreads, "one halo element per thread");
    const bool seg1 = a.dy.nseg == 1;
    auto chan = [&](int c, const float*& p, const float*& y, int64_t& ns, int64_t& yns) {
        if (seg1) {
            const isg_vseg& sg = a.dy.s[0];
            p = sg.p + (int64_t)c * HWs;
            y = (sg.xform == ISG_XF_BN_BWD && sg.y) ? sg.y + (int64_t)c * HWs : p;
            ns = sg.n_stride;
            yns = (sg.xform == ISG_XF_BN_BWD && sg.y) ? sg.y_n_stride : sg.n_stride;
        } else {
            const ChSrc t = ch_src(vt_lite(a.dy), c, (int)HWs);
            p = t.p; y = t.y; ns = t.ns; yns = t.yns;
        }
    };
    f32x4 xv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = tid + u * kThreads;
        const int c = e / ((kRowsPB + 2) * 16), rq = e - c * (kRowsPB + 2) * 16;
        const int rr = rq >> 4, q = rq & 15;
        const int yy = i0 - 1 + rr, xx = j0 + 4 * q;
        const bool ok = c < a.C && (unsigned)yy < (unsigned)Hs && xx < Ws;
        const float *p, *y;
        int64_t ns, yns;
        chan(c < a.C ? c : 0, p, y, ns, yns);
        const int64_t o = ok ? (int64_t)yy * Ws + xx : 0;
        xv[u] = gld4(p + (int64_t)n * ns, o);
        yv[u] = gld4(y + (int64_t)n * yns, o);  // == p unless BN_BWD (an L1 hit)
    }
    float hx, hy;
    bool hok;
    {
        const int e = min(tid, NH - 1);
        const int c = e / ((kRowsPB + 2) * 2), rs = e - c * (kRowsPB + 2) * 2;
        const int rr = rs >> 1, side = rs & 1;
        const int yy = i0 - 1 + rr, xx = side ? j0 + 64 : j0 - 1;
        hok = tid < NH && c < a.C && (unsigned)yy < (unsigned)Hs && (unsigned)xx < (unsigned)Ws;
        const float *p, *y;
        int64_t ns, yns;
        chan(c < a.C ? c : 0, p, y, ns, yns);
        const int64_t o = hok ? (int64_t)yy * Ws + xx : 0;
        hx = gld(p + (int64_t)n * ns, o);
        hy = gld(y + (int64_t)n * yns, o);
    }
    {   // the weight: every load of the thread issued before the first store (a rolled loop
        // of predicated loads paid one L2 round trip per element: 25 in a row)
        constexpr int NW = kMaxM * kMaxM * K * K, UW = NW / kThreads;
        static_assert(NW % kThreads == 0, "weight copy split");
        const int nw = a.C * a.M * K * K;
        float wv[UW];
#pragma unroll
        for (int u = 0; u < UW; ++u) {
            const int e = tid + u * kThreads;
            const int c = e / (kMaxM * K * K), r = e - c * kMaxM * K * K;
            const int m = r / (K * K), tap = r - m * K * K;
            const int src = (c * a.M + m) * K * K + tap;
            wv[u] = gld(a.w, (c < a.C && m < a.M) ? src : 0);
            wv[u] = (c < a.C && m < a.M && src < nw) ? wv[u] : 0.f;
        }
        if (tid < a.C) {
            const ChT t = ch_table_entry(a.dy, tid, HWs);
            lin[tid] = xf_lin(t.xf, t.act, t.k);
        }
        if (tid < a.M) ri[tid] = sink_row(a.out, tid, (int64_t)2 * Hs * Wd);
#pragma unroll
        for (int u = 0; u < UW; ++u) wl[tid + u * kThreads] = wv[u];
    }
    __syncthreads();
    STAMP(1);
    // ---- the band, transformed once per element, into LDS -----------------------------------
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = tid + u * kThreads;
        const int c = e / ((kRowsPB + 2) * 16), rq = e - c * (kRowsPB + 2) * 16;
        const int rr = rq >> 4, q = rq & 15;
        const int yy = i0 - 1 + rr, xx = j0 + 4 * q;
        const bool ok = c < a.C && (unsigned)yy < (unsigned)Hs && xx < Ws;
        float* d = Ls + c * kSubPL + rr * kSubRS + 4 + 4 * q;
        const XfLin l = lin[c < a.C ? c : 0];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = ok ? xf_lin_apply(l, xv[u][k], yv[u][k]) : 0.f;
    }
    if (tid < NH) {
        const int c = tid / ((kRowsPB + 2) * 2), rs = tid - c * (kRowsPB + 2) * 2;
        const int rr = rs >> 1, side = rs & 1;
        const XfLin l = lin[c < a.C ? c : 0];
        Ls[c * kSubPL + rr * kSubRS + (side ? 68 : 3)] = hok ? xf_lin_apply(l, hx, hy) : 0.f;
    }
    __syncthreads();
    STAMP(2);
    float wreg[kMaxM / 4][K * K];  // A: W[c = 4g + kq][m = pl][kh][kw], the whole launch
#pragma unroll
    for (int g = 0; g < kMaxM / 4; ++g)
#pragma unroll
        for (int t = 0; t < K * K; ++t) wreg[g][t] = wl[((4 * g + kq) * kMaxM + pl) * K * K + t];
    const int jw = j0 + wave * 16;  // this wave's first cell
    float bs0[4] = {0.f, 0.f, 0.f, 0.f}, bs1[4] = {0.f, 0.f, 0.f, 0.f}, bs2[4] = {0.f, 0.f, 0.f, 0.f};
    const int i_end = min(Hs, i0 + kRowsPB);
    const int jo = jw + pl;
    const bool cok = jo < Ws;
    const int joc = cok ? jo : 0;
    for (int i = i0; i < i_end; ++i) {
        // this row's sink operands first (ACTBWD: the saved forward output; ACCUM: the old
        // value), all 8 in flight under the row's MFMAs
        v2f_t pre[4][2];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const SinkRow& q = ri[min(4 * kq + r, a.M - 1)];
            const bool ab = q.mode == ISG_SINK_ACTBWD;
            const float* base = ab ? q.y : q.p;
            const bool live = (ab || q.mode == ISG_SINK_ACCUM) && base;  // else a dummy read
            const int64_t bns = ab ? q.yns : q.ns;
#pragma unroll
            for (int u = 0; u < 2; ++u)
                pre[r][u] = *(gcv2_p)((gcfloat_p)(live ? base : a.dy.s[0].p) +  // 16-B aligned (down_src_ok)
                                      (live ? (int64_t)n * bns + (int64_t)(2 * i + u) * Wd + 2 * joc : 0));
        }
        f32x4 acc[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < 2; ++v) acc[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* lb = Ls + kq * kSubPL + (i - i0) * kSubRS + wave * 16 + pl + 3;
        // A operands in registers (loaded once per workgroup, below), B software-pipelined:
        // kernel row (g, kh) + 1's five values are read while row (g, kh)'s MFMAs issue
        auto brow = [&](int gk, float (&b)[K]) {
            const int g = gk / K, kh = gk - g * K;
            const int au = (kh + P) & 1, rr = (au + P - kh) / 2 + R0;
            const float* lg = lb + 4 * g * kSubPL + rr * kSubRS;
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
                const int av = (kw + P) & 1, qq = (av + P - kw) / 2 + R0;
                b[kw] = lg[qq];
            }
        };
        float b0[K], b1[K];
        brow(0, b0);
#pragma unroll
        for (int gk = 0; gk < (kMaxM / 4) * K; ++gk) {
            float (&cur)[K] = (gk & 1) ? b1 : b0;
            if (gk + 1 < (kMaxM / 4) * K) {
                if (gk & 1) brow(gk + 1, b0);
                else brow(gk + 1, b1);
            }
            __builtin_amdgcn_sched_barrier(0);
            const int g = gk / K, kh = gk - g * K;
            const int au = (kh + P) & 1;
#pragma unroll
            for (int kw = 0; kw < K; ++kw) {
                const int av = (kw + P) & 1;
                acc[au][av] = __builtin_amdgcn_mfma_f32_16x16x4f32(wreg[g][kh * K + kw], cur[kw],
                                                                   acc[au][av], 0, 0, 0);
            }
        }
        // epilogue: lane holds D[m = 4kq + r][cell = pl] of every phase
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = 4 * kq + r;
            if (cok && m < a.M) {
                const SinkRow q = ri[m];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
                    sink_row_apply2_pre(q, n, (int64_t)(2 * i + u) * Wd + 2 * jo, acc[u][0][r],
                                        acc[u][1][r], pre[r][u], t0, t1, t2);
                    bs0[r] += t0;
                    bs1[r] += t1;
                    bs2[r] += t2;
                }
            }
        }
    }
    STAMP(3);
    if (sinks_need_red(a.out)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float t0 = dpp_row16_sum(bs0[r]), t1 = dpp_row16_sum(bs1[r]), t2 = dpp_row16_sum(bs2[r]);
            if (pl == 0) {
                red[wave][0][4 * kq + r] = t0;
                red[wave][1][4 * kq + r] = t1;
                red[wave][2][4 * kq + r] = t2;
            }
        }
        __syncthreads();
        if (tid < a.M) {
            float r3[3];
#pragma unroll
            for (int q3 = 0; q3 < 3; ++q3) r3[q3] = ((red[0][q3][tid] + red[1][q3][tid]) + red[2][q3][tid]) + red[3][q3][tid];
            sink_row_flush(a.out, tid, r3[0], r3[1], r3[2]);
        }
    }
    STAMP(4);
}

// ---- 5x5 stride-2 pad-2 weight gradient, LDS-staged (the stem's second conv) ------------
//   dW[m][c][kh][kw] = sum_{n,oy,ox} dy[m][n][oy][ox] * X[c][n][2oy - 2 + kh][2ox - 2 + kw]
// One v_mfma_f32_16x16x4_f32 per tap and pixel quad: D[m][c] += A[m][4 pixels] x
// B[4 pixels][c], A = dy (lane: m = l&15, pixel = l>>4), B = the band value of channel
// c = l&15 under the tap for pixel l>>4 — one A read serves the 25 taps (25 accumulators
// per lane, no dependent MFMA chain). A tile is kWgRows output rows (wave w = row w) x
// kWgX output columns of one image: its input band (2*kWgRows + 3 rows x 72 columns x 16
// channels, producer BatchNorm + activation applied once per element, split into even /
// odd column planes as in s2k5_fwd_kernel) and its dy block (BatchNorm backward rebuilt
// once per element) go to LDS with 16-B loads. Persistent workgroups walk a contiguous run
// of tiles (runs grouped per XCD so neighbouring bands share an L2), the next tile's loads
// in flight during this tile's MFMAs. Epilogue: the 4 waves' partials summed in LDS, one
// coalesced f32 atomic per dW element per workgroup into an ISG_WREP replica.
constexpr int kWgRows = 4;
constexpr int kWgX = 32;                   // output columns per tile
constexpr int kWgNR = 2 * kWgRows + 3;     // staged input rows
constexpr int kWgQ = kWgX / 2 + 2;         // 16-B quads per staged row (from column 2*ox0 - 4)
constexpr int kWgEW = 2 * kWgQ;            // columns per parity plane
constexpr int kWgRS = 2 * kWgEW;           // staged row: [even | odd]
constexpr int kWgPL = 802;                 // channel plane (>= 11 * 72; 2 mod 32: B reads conflict-free)
constexpr int kWgDQ = 130;                 // dy channel block (>= 4 * 32; 2 mod 32: A reads conflict-free)
constexpr int kWgLds = kMaxM * kWgPL + kMaxM * kWgDQ;  // floats
constexpr int kWgNW = kMaxM * kMaxM * 25;  // dW elements of one workgroup's partial
static_assert(kWgPL >= kWgNR * kWgRS && kWgPL % 32 == 2 && kWgDQ % 32 == 2 && kWgDQ >= kWgRows * kWgX,
              "s2k5 wgrad layout");
static_assert(2 * kWgNW <= kWgLds, "s2k5 wgrad epilogue regions");

struct S2wArgs {
    isg_vtensor dy;  // the conv's output gradient: M channels, OH x OW
    isg_vtensor x;   // its input: C channels, 2 OH x 2 OW
    double* dw;       // [M][wc][5][5] (the first C input channels written)
    double* dbias;
    int64_t rep_stride;
    int nrep;
    int N, M, C, wc, OH, OW;
    int tiles_x, tiles_y, ntiles, tpw;
};

// Branch-free staging record: x side v = (raw - k0) * k1 + k2, then v > 0 ? v : v * k3
// (PLAIN: identity, ReLU: k3 = 0, PReLU: k3 = slope, none: k3 = 1); dy side
// k0 * raw + k1 * (y - k2) + k3 (PLAIN: k0 = 1). A per-lane channel (the staging items
// span channels within a wave) otherwise makes every transform a divergent branch tree.
struct S2Ch {
    const float* p;
    const float* y;
    int ns, yns;
    f32x4 k;
};

ISG_DEV S2Ch s2_ch_addr(const isg_vtensor& vt, int c, int hw) {
    const ChSrc t = ch_src(vt_lite(vt), c, hw);
    return S2Ch{t.p, t.y, t.ns, t.yns, f32x4{0.f, 0.f, 0.f, 0.f}};
}

ISG_DEV f32x4 s2_coef_x(const isg_vtensor& vt, int c, int hw) {
    const ChSrc t = ch_src(vt_lite(vt), c, hw);
    f32x4 k{0.f, 1.f, 0.f, 1.f};
    const ChanCoef q = vt_coef(vt, c);
    if (t.xf == ISG_XF_BN_FWD) { k[0] = q.c0; k[1] = q.c1; k[2] = q.c2; }
    k[3] = t.act == ISG_ACT_RELU ? 0.f : t.act == ISG_ACT_PRELU ? q.c3 : 1.f;
    return k;
}

ISG_DEV f32x4 s2_coef_dy(const isg_vtensor& vt, int c, int hw) {
    const ChSrc t = ch_src(vt_lite(vt), c, hw);
    if (t.xf != ISG_XF_BN_BWD) return f32x4{1.f, 0.f, 0.f, 0.f};
    const ChanCoef q = vt_coef(vt, c);
    return f32x4{q.c0, q.c1, q.c2, q.c3};
}

// NARROW (C <= 4, the RGB layer 1): the 25 taps x C channels go into the MFMA's N dimension
// instead — B[px][n = (c, tap)], 5 N-tiles of 16 (75 used) — so a pixel quad costs 5 MFMAs,
// not 25 with 13 of every 16 columns zero.
// NT: N-tiles of the narrow form (5 for C <= 3, 7 for C = 4; 0 = the wide form)
template <bool YB, int NT>
__global__ __launch_bounds__(2 * kThreads, 1) void s2k5_wgrad_kernel(S2wArgs a) {
    extern __shared__ __attribute__((aligned(16))) float s2w_lds[];  // 2 x [Xs | Ds]
    __shared__ S2Ch tabx[kMaxM];
    __shared__ S2Ch taby[kMaxM];
    __shared__ float bred[4][64];
    typedef float f32x2 __attribute__((ext_vector_type(2)));

    // waves 0-3 consume (MFMA, wave w = tile row w), waves 4-7 produce (stage the next
    // tile into the other buffer while the consumers' MFMAs run on the same SIMDs)
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kq = lane >> 4, pl = lane & 15;
    const bool producer = wave >= 4;
    const int ptid = tid - kThreads;
    constexpr bool NARROW = NT > 0;
    constexpr int kNarN = NARROW ? NT : 1;
    constexpr int kNarNW = kMaxM * 16 * kNarN;  // the narrow form's per-workgroup partial
    const int G = gridDim.x, b = blockIdx.x;
    const int L = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;  // XCD-grouped runs
    const int t0 = L * a.tpw, t1 = min(t0 + a.tpw, a.ntiles);
    if (t0 >= t1) return;
    STAMP(0);
    const int Ho = a.OH, Wo = a.OW, Hi = 2 * Ho, Wi = 2 * Wo;
    // addresses first: the first tile's loads are in flight while the BatchNorm
    // coefficients are evaluated from the statistics (fp64, one thread per channel)
    if (tid < kMaxM) {
        tabx[tid] = s2_ch_addr(a.x, min(tid, a.C - 1), Hi * Wi);
        taby[tid] = s2_ch_addr(a.dy, min(tid, a.M - 1), Ho * Wo);
    }
    __syncthreads();
    STAMP(1);

    constexpr int NE = (NARROW ? 4 : kMaxM) * kWgNR * kWgQ;
    constexpr int UX = (NE + kThreads - 1) / kThreads;
    constexpr int ND = kMaxM * kWgRows * (kWgX / 4);
    constexpr int UD = (ND + kThreads - 1) / kThreads;
    f32x4 xv[UX], dv[UD], yv[UD];
    int n = 0, oy0 = 0, ox0 = 0;  // the tile held in xv / dv / yv
    auto load = [&](int t) {
        const int tpi = a.tiles_x * a.tiles_y;
        n = t / tpi;
        const int r = t - n * tpi, ty = r / a.tiles_x;
        oy0 = ty * kWgRows;
        ox0 = (r - ty * a.tiles_x) * kWgX;
#pragma unroll
        for (int u = 0; u < UX; ++u) {
            const int e = min(ptid + u * kThreads, NE - 1);
            const int c = e / (kWgNR * kWgQ), rq = e - c * (kWgNR * kWgQ);
            const int rr = rq / kWgQ, q = rq - rr * kWgQ;
            const int iy = 2 * oy0 - 2 + rr, ix = 2 * ox0 - 4 + 4 * q;
            const bool ok = c < a.C && (unsigned)iy < (unsigned)Hi && ix >= 0 && ix < Wi;
            const S2Ch& t = tabx[c];
            xv[u] = gld4(t.p + (int64_t)n * t.ns, ok ? (int64_t)iy * Wi + ix : 0);
        }
#pragma unroll
        for (int u = 0; u < UD; ++u) {
            const int e = min(ptid + u * kThreads, ND - 1);
            const int m = e / (kWgRows * kWgX / 4), rem = e - m * (kWgRows * kWgX / 4);
            const int r = rem / (kWgX / 4), qx = rem - r * (kWgX / 4);
            const int oy = oy0 + r, ox = ox0 + 4 * qx;
            const bool ok = m < a.M && oy < Ho && ox < Wo;
            const S2Ch& t = taby[m];
            const int64_t o = ok ? (int64_t)oy * Wo + ox : 0;
            dv[u] = gld4(t.p + (int64_t)n * t.ns, o);
            if constexpr (YB) yv[u] = gld4(t.y + (int64_t)n * t.yns, o);
        }
    };
    auto store = [&](int buf) {
        float* const Xs = s2w_lds + buf * kWgLds;
        float* const Ds = Xs + kMaxM * kWgPL;
#pragma unroll
        for (int u = 0; u < UX; ++u) {
            const int e = ptid + u * kThreads;
            if (e >= NE) continue;
            const int c = e / (kWgNR * kWgQ), rq = e - c * (kWgNR * kWgQ);
            const int rr = rq / kWgQ, q = rq - rr * kWgQ;
            const int iy = 2 * oy0 - 2 + rr, ix = 2 * ox0 - 4 + 4 * q;
            const bool ok = c < a.C && (unsigned)iy < (unsigned)Hi && ix >= 0 && ix < Wi;
            const f32x4 kk = tabx[c].k;
            f32x4 v;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float z = (xv[u][k] - kk[0]) * kk[1] + kk[2];
                v[k] = ok ? (z > 0.f ? z : z * kk[3]) : 0.f;
            }
            float* row = Xs + c * kWgPL + rr * kWgRS + 2 * q;
            *reinterpret_cast<f32x2*>(row) = f32x2{v[0], v[2]};
            *reinterpret_cast<f32x2*>(row + kWgEW) = f32x2{v[1], v[3]};
        }
#pragma unroll
        for (int u = 0; u < UD; ++u) {
            const int e = ptid + u * kThreads;
            if (e >= ND) continue;
            const int m = e / (kWgRows * kWgX / 4), rem = e - m * (kWgRows * kWgX / 4);
            const int r = rem / (kWgX / 4), qx = rem - r * (kWgX / 4);
            const bool ok = m < a.M && oy0 + r < Ho && ox0 + 4 * qx < Wo;
            const f32x4 kk = taby[m].k;
            f32x4 v;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[k] = ok ? kk[0] * dv[u][k] + kk[1] * ((YB ? yv[u][k] : dv[u][k]) - kk[2]) + kk[3] : 0.f;
            float* d = Ds + m * kWgDQ + r * kWgX + 4 * qx;
            *reinterpret_cast<f32x2*>(d) = f32x2{v[0], v[1]};
            *reinterpret_cast<f32x2*>(d + 2) = f32x2{v[2], v[3]};
        }
    };

    // the two roles run separate loops with the same barrier sequence (A, B, one per tile,
    // E1, E2), so neither role's registers are live in the other's code
    float* const R = s2w_lds;  // epilogue: two regions of [16][16][25]
    if (producer) {
        load(t0);
        __syncthreads();  // A: coefficients
        store(0);
        if (t0 + 1 < t1) load(t0 + 1);
        __syncthreads();  // B: tile t0 staged
        for (int t = t0; t < t1; ++t) {
            if (t + 1 < t1) {
                store(((t - t0) & 1) ^ 1);  // registers hold tile t + 1
                if (t + 2 < t1) load(t + 2);
            }
            __syncthreads();
        }
        __syncthreads();  // E1
        __syncthreads();  // E2
    } else {
        if (tid < kMaxM) {
            tabx[tid].k = s2_coef_x(a.x, min(tid, a.C - 1), Hi * Wi);
        } else if (tid >= 64 && tid < 64 + kMaxM) {
            taby[tid - 64].k = s2_coef_dy(a.dy, min(tid - 64, a.M - 1), Ho * Wo);
        }
        constexpr int NACC = NARROW ? kNarN : 25;
        f32x4 acc[NACC];
#pragma unroll
        for (int t = 0; t < NACC; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        float bsum = 0.f;
        // NARROW: this lane's column n = 16t + pl -> (channel, tap) as a band offset
        int noff[kNarN];
#pragma unroll
        for (int t = 0; t < kNarN; ++t) {
            const int n = 16 * t + pl, c = n / 25, tap = n - c * 25, kh = tap / 5, kw = tap - kh * 5;
            noff[t] = n < 4 * 25 ? c * kWgPL + kh * kWgRS + (kw & 1) * kWgEW + (kw >> 1) : 0;
        }
        __syncthreads();  // A
        __syncthreads();  // B
        STAMP(2);
        const int nq = kWgX / 4;
        for (int t = t0; t < t1; ++t) {
            const float* const Xs = s2w_lds + ((t - t0) & 1) * kWgLds;
            const float* const ab = Xs + kMaxM * kWgPL + pl * kWgDQ + wave * kWgX + kq;
            const float* const bb = Xs + pl * kWgPL + 2 * wave * kWgRS + kq + 1;
            // fully unrolled: every operand read is the lane's base address plus an immediate
            // offset, and the scheduler runs the reads ahead of the MFMAs (a rolled loop
            // re-derived 25 addresses per step and waited out each read)
            if (nq && NARROW) {
                const float* const nb = Xs + 2 * wave * kWgRS + kq + 1;
                // the same operand pipeline as the wide form below, two quads per stage
                float av0[2], av1[2], b0[2][kNarN], b1[2][kNarN];
                auto quads = [&](int q2, float (&av)[2], float (&b)[2][kNarN]) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        av[h] = ab[4 * (2 * q2 + h)];
#pragma unroll
                        for (int t = 0; t < kNarN; ++t) b[h][t] = nb[noff[t] + 4 * (2 * q2 + h)];
                    }
                };
                quads(0, av0, b0);
#pragma unroll
                for (int q2 = 0; q2 < kWgX / 8; ++q2) {
                    float (&av)[2] = (q2 & 1) ? av1 : av0;
                    float (&cur)[2][kNarN] = (q2 & 1) ? b1 : b0;
                    if (q2 + 1 < kWgX / 8) {
                        if (q2 & 1) quads(q2 + 1, av0, b0);
                        else quads(q2 + 1, av1, b1);
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        bsum += av[h];
#pragma unroll
                        for (int t = 0; t < kNarN; ++t)
                            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[h], cur[h][t], acc[t], 0, 0, 0);
                    }
                }
            } else if (nq) {
                // software-pipelined operands: quad q + 1's A value and 25 B values are read
                // from LDS while quad q's 25 MFMAs issue (sched_barrier keeps the reads above
                // them; the compiler's own schedule waited out each read's latency)
                float av0, av1, b0[NACC], b1[NACC];
                auto quad = [&](int q, float& av, float (&b)[NACC]) {
                    av = ab[4 * q];
#pragma unroll
                    for (int j = 0; j < NACC; ++j)
                        b[j] = bb[(j / 5) * kWgRS + ((j % 5) & 1) * kWgEW + ((j % 5) >> 1) + 4 * q];
                };
                quad(0, av0, b0);
#pragma unroll
                for (int q = 0; q < kWgX / 4; ++q) {
                    float& av = (q & 1) ? av1 : av0;
                    float (&cur)[NACC] = (q & 1) ? b1 : b0;
                    if (q + 1 < kWgX / 4) {
                        if (q & 1) quad(q + 1, av0, b0);
                        else quad(q + 1, av1, b1);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    bsum += av;
#pragma unroll
                    for (int j = 0; j < NACC; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, cur[j], acc[j], 0, 0, 0);
                }
            }
            __syncthreads();
        }
        // ---- epilogue: lane holds D[m = 4kq + i][c = pl] of every tap
        STAMP(3);
        // NARROW: R[(m * kNarN + t) * 16 + pl] = D[m][n = 16t + pl]
        auto ridx = [&](int t, int i) {
            return NARROW ? ((4 * kq + i) * kNarN + t) * 16 + pl : ((4 * kq + i) * kMaxM + pl) * 25 + t;
        };
        constexpr int NW = NARROW ? kNarNW : kWgNW;
        if (wave < 2) {
#pragma unroll
            for (int t = 0; t < NACC; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) R[wave * NW + ridx(t, i)] = acc[t][i];
        }
        bred[wave][lane] = bsum;
        __syncthreads();  // E1
        if (wave >= 2) {
#pragma unroll
            for (int t = 0; t < NACC; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) R[(wave - 2) * NW + ridx(t, i)] += acc[t][i];
        }
        __syncthreads();  // E2
    }
    double* const dwr = a.dw + (int64_t)(blockIdx.x % a.nrep) * a.rep_stride;
    if (NARROW) {
        for (int e = tid; e < kNarNW; e += 2 * kThreads) {
            const int m = e / (kNarN * 16), n = e - m * (kNarN * 16), c = n / 25, tap = n - c * 25;
            if (m < a.M && c < a.C) atomicAdd(&dwr[(m * a.wc + c) * 25 + tap], R[e] + R[kNarNW + e]);
        }
    } else {
        for (int e = tid; e < kWgNW; e += 2 * kThreads) {
            const int m = e / (kMaxM * 25), rem = e - m * (kMaxM * 25);
            const int c = rem / 25, tap = rem - c * 25;
            if (m < a.M && c < a.C) atomicAdd(&dwr[(m * a.wc + c) * 25 + tap], R[e] + R[kWgNW + e]);
        }
    }
    if (a.dbias && tid < a.M) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            s += ((bred[w][tid] + bred[w][16 + tid]) + bred[w][32 + tid]) + bred[w][48 + tid];
        atomicAdd(&(a.dbias + (int64_t)(blockIdx.x % a.nrep) * a.rep_stride)[tid], s);
    }
    STAMP(4);
}

// ---- 5x5 stride-2 pad-2 forward (the stem's second conv, segment.py:23-26: 16 -> 16
// channels, 512^2 -> 256^2 at 1024^2 input), producer / consumer like s2k5_wgrad_kernel ------
// Persistent 8-wave workgroups over tiles of kWgRows output rows x kWgX output columns (the
// wgrad kernel's tile and band layout): waves 4-7 stage the next tile's input band (11 rows
// x 72 columns x 16 channels, the producer's BatchNorm + activation applied once per element,
// split into even / odd column planes) into the other LDS buffer while waves 0-3 run this
// tile's MFMAs on the same SIMDs. The weights are the A operands, loaded ONCE per workgroup
// into 100 registers per lane: A[m][k] = W[m][4g + k][tap] (lane: m = l&15, k = l>>4);
// B[k][px] = band value of channel 4g + k under the tap for pixel px (lane: k = l>>4,
// px = l&15). Consumer wave w = output row w, two 16-pixel groups (two accumulator chains):
// 4 groups x 25 taps x 2 = 200 MFMAs per wave and tile. The output goes through the sinks
// (bias, BN statistics accumulated in registers across tiles, flushed once per workgroup).
// The previous form (one tile per workgroup, weights re-staged per tile, no overlap of
// staging and MFMA) ran 62 us against tap_conv's 65.
constexpr int kFwPL = 816;  // channel plane (>= 11 * 72; 16 mod 32: lanes k = 0 / 1 of a B read hit disjoint banks)
static_assert(kFwPL >= kWgNR * kWgRS && kFwPL % 32 == 16, "s2k5 fwd plane");
constexpr int kFwOut = kMaxM * kWgX + 4;  // one wave's output row in LDS: [16 channels][32 columns] (+4: bank shift)
constexpr int kS2fMaxWc = 32;  // weight input channels the forward's whole-weight copy takes (G < 4)
static_assert(kMaxM * kS2fMaxWc * 25 <= kMaxM * kFwPL, "s2k5 fwd weight copy fits one band buffer");

struct S2fArgs {
    isg_vtensor x;  // C channels, 2 OH x 2 OW
    const float* w;  // [M][wc][5][5], the first C input channels used (wc >= C)
    isg_sinks out;   // M channels, OH x OW
    int N, M, C, wc, OH, OW;
    int tiles_x, tiles_y, ntiles, tpw;
    int st16;  // one STORE sink over all M channels and OW % 4 == 0: 16-B epilogue stores
};

// G: channel groups of 4 (1 for the stem's RGB layer 1 with w_ci = 20, 4 for layer 2)
template <int G>
__global__ __launch_bounds__(2 * kThreads, 1) void s2k5_fwd_kernel(S2fArgs a) {
    extern __shared__ __attribute__((aligned(16))) float s2f_lds[];  // 2 x band
    __shared__ S2Ch tabx[kMaxM];
    __shared__ SinkRow ri[kMaxM];
    __shared__ float red[4][3][kMaxM];
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    constexpr int BAND = kMaxM * kFwPL;
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kq = lane >> 4, pl = lane & 15;
    const bool producer = wave >= 4;
    const int ptid = tid - kThreads;
    const int NG = gridDim.x, b = blockIdx.x;
    const int L = (NG % 8 == 0) ? (b % 8) * (NG / 8) + b / 8 : b;  // XCD-grouped runs
    const int t0 = L * a.tpw, t1 = min(t0 + a.tpw, a.ntiles);
    const int Ho = a.OH, Wo = a.OW, Hi = 2 * Ho, Wi = 2 * Wo;
    STAMP(0);
    constexpr int NE = 4 * G * kWgNR * kWgQ;
    constexpr int UX = (NE + kThreads - 1) / kThreads;
    f32x4 xv[UX];
    int n = 0, oy0 = 0, ox0 = 0;  // producers: the tile held in xv
    auto tile_of = [&](int t, int& tn, int& ty0, int& tx0) {
        const int tpi = a.tiles_x * a.tiles_y;
        tn = t / tpi;
        const int r = t - tn * tpi, ty = r / a.tiles_x;
        ty0 = ty * kWgRows;
        tx0 = (r - ty * a.tiles_x) * kWgX;
    };
    // DIRECT: the channel address from the kernel arguments (the first tile, before the
    // table in LDS exists), else from tabx
    auto load = [&](int t, auto direct) {
        tile_of(t, n, oy0, ox0);
#pragma unroll
        for (int u = 0; u < UX; ++u) {
            const int e = min(ptid + u * kThreads, NE - 1);
            const int c = e / (kWgNR * kWgQ), rq = e - c * (kWgNR * kWgQ);
            const int rr = rq / kWgQ, q = rq - rr * kWgQ;
            const int iy = 2 * oy0 - 2 + rr, ix = 2 * ox0 - 4 + 4 * q;
            const bool ok = c < a.C && (unsigned)iy < (unsigned)Hi && ix >= 0 && ix < Wi;
            const int64_t o = ok ? (int64_t)iy * Wi + ix : 0;
            if constexpr (decltype(direct)::value) {
                // one segment (the stem's input: the image / the layer-1 output): the plane
                // address from the kernel argument directly, no segment selection
                const int cc = min(c, a.C - 1);
                if (a.x.nseg == 1) {
                    xv[u] = gld4(a.x.s[0].p + (int64_t)n * a.x.s[0].n_stride + (int64_t)cc * Hi * Wi, o);
                } else {
                    const S2Ch t = s2_ch_addr(a.x, cc, Hi * Wi);
                    xv[u] = gld4(t.p + (int64_t)n * t.ns, o);
                }
            } else {
                const S2Ch& t = tabx[c];
                xv[u] = gld4(t.p + (int64_t)n * t.ns, o);
            }
        }
    };
    // ONE round trip before the first barrier (each barrier waits for every load of the
    // workgroup): the producers' first tile, the weights, the consumers' BatchNorm
    // coefficients and sink rows are all in flight together (round 4 issued the tile after
    // the weights had landed, and the coefficients after that)
    if (producer && t0 < t1) load(t0, std::true_type{});
    if (tid < kMaxM) tabx[tid] = s2_ch_addr(a.x, min(tid, a.C - 1), Hi * Wi);
    {  // the weight [M][wc][25] copied whole and linearly into buffer 1 (first written by
       // the producers after barrier B): every load of the thread in flight at once (a rolled
       // loop paid one round trip per element), no index division (the per-element (m, c,
       // tap) split by runtime divisors was most of this prologue's instructions)
        float* wl = s2f_lds + BAND;
        const int nw = a.M * a.wc * 25;
        constexpr int UW = (kMaxM * (G == 4 ? 16 : kS2fMaxWc) * 25 + 2 * kThreads - 1) / (2 * kThreads);
        float wv[UW];
#pragma unroll
        for (int u = 0; u < UW; ++u) wv[u] = gld(a.w, min(tid + u * 2 * kThreads, nw - 1));
        if (tid < kMaxM) tabx[tid].k = s2_coef_x(a.x, min(tid, a.C - 1), Hi * Wi);
        else if (tid >= 64 && tid < 64 + kMaxM) ri[tid - 64] = sink_row(a.out, tid - 64, (int64_t)Ho * Wo);
#pragma unroll
        for (int u = 0; u < UW; ++u)
            if (tid + u * 2 * kThreads < nw) wl[tid + u * 2 * kThreads] = wv[u];
    }
    STAMP(1);
    __syncthreads();  // S0: channel table, coefficients, sink rows, weight copy, tile t0 loaded
    STAMP(2);
    auto store = [&](int buf) {
        float* const Xs = s2f_lds + buf * BAND;
#pragma unroll
        for (int u = 0; u < UX; ++u) {
            const int e = ptid + u * kThreads;
            if (e >= NE) continue;
            const int c = e / (kWgNR * kWgQ), rq = e - c * (kWgNR * kWgQ);
            const int rr = rq / kWgQ, q = rq - rr * kWgQ;
            const int iy = 2 * oy0 - 2 + rr, ix = 2 * ox0 - 4 + 4 * q;
            const bool ok = c < a.C && (unsigned)iy < (unsigned)Hi && ix >= 0 && ix < Wi;
            const f32x4 kk = tabx[c].k;
            f32x4 v;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float z = (xv[u][k] - kk[0]) * kk[1] + kk[2];
                v[k] = ok ? (z > 0.f ? z : z * kk[3]) : 0.f;
            }
            float* row = Xs + c * kFwPL + rr * kWgRS + 2 * q;
            *reinterpret_cast<f32x2*>(row) = f32x2{v[0], v[2]};
            *reinterpret_cast<f32x2*>(row + kWgEW) = f32x2{v[1], v[3]};
        }
    };

    if (producer) {
        if (t0 < t1) store(0);
        if (t0 + 1 < t1) load(t0 + 1, std::false_type{});
        __syncthreads();  // B: tile t0 staged (the consumers read the weights before it)
        for (int t = t0; t < t1; ++t) {
            if (t + 1 < t1) {
                store(((t - t0) & 1) ^ 1);  // registers hold tile t + 1
                if (t + 2 < t1) load(t + 2, std::false_type{});
            }
            __syncthreads();
        }
        __syncthreads();  // E
    } else {
        float wa[G][25];
        {
            const float* wl = s2f_lds + BAND;
            const int m = pl < a.M ? pl : 0;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int c = 4 * g + kq;
                const bool ok = pl < a.M && c < a.C;
                const float* wp = wl + (m * a.wc + (c < a.C ? c : 0)) * 25;
#pragma unroll
                for (int t = 0; t < 25; ++t) wa[g][t] = ok ? wp[t] : 0.f;
            }
        }
        float bs0[4] = {0.f, 0.f, 0.f, 0.f}, bs1[4] = {0.f, 0.f, 0.f, 0.f}, bs2[4] = {0.f, 0.f, 0.f, 0.f};
        // st16: the STORE sink's base, image stride and this lane's 4 channel biases
        float* const obase = uniform_ptr(a.out.s[0].p);
        const int64_t ons = a.out.s[0].n_stride;
        float bias[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = min(4 * kq + i, a.M - 1);
            bias[i] = a.st16 && a.out.s[0].bias ? a.out.s[0].bias[m] : 0.f;
        }
        __syncthreads();  // B
        STAMP(3);
        for (int t = t0; t < t1; ++t) {
            int tn, ty0, tx0;
            tile_of(t, tn, ty0, tx0);
            const float* const bb = s2f_lds + ((t - t0) & 1) * BAND + kq * kFwPL + 2 * wave * kWgRS + pl + 1;
            f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
            // software-pipelined B operands: the next kernel row's 10 values are read from
            // LDS into a second register set while this row's 10 MFMAs issue (the compiler's
            // own schedule reused 8 registers and waited out the read latency every 4-5
            // MFMAs: ~0.5 of the MFMA rate in the loop, kbench stamps r07)
            auto rowb = [&](int gk, float (&b)[10]) {
                const int g = gk / 5, kh = gk - g * 5;
#pragma unroll
                for (int kw = 0; kw < 5; ++kw) {
                    const float* bp = bb + 4 * g * kFwPL + kh * kWgRS + (kw & 1) * kWgEW + (kw >> 1);
                    b[2 * kw] = bp[0];
                    b[2 * kw + 1] = bp[16];
                }
            };
            float b0[10], b1[10];
            rowb(0, b0);
#pragma unroll
            for (int gk = 0; gk < 5 * G; ++gk) {
                float (&cur)[10] = (gk & 1) ? b1 : b0;
                float (&nxt)[10] = (gk & 1) ? b0 : b1;
                if (gk + 1 < 5 * G) rowb(gk + 1, nxt);
                // keep those reads above this row's MFMAs (the scheduler otherwise sinks each
                // read next to its use and the loop waits out every LDS latency)
                __builtin_amdgcn_sched_barrier(0);
                const int g = gk / 5, kh = gk - g * 5;
#pragma unroll
                for (int kw = 0; kw < 5; ++kw)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[g][kh * 5 + kw], cur[2 * kw + h], acc[h], 0, 0, 0);
            }
            if (t == t0) STAMP(4);
            // epilogue: lane holds D[m = 4kq + i][px = pl] of pixel group h, row ty0 + wave
            const int oy = ty0 + wave;
            if (a.st16) {
                // bias + statistics from the registers; the row [16 channels][32 columns] goes
                // through this wave's LDS slot and leaves as 16-B stores (8 lanes = one 128-B
                // channel row) — 4-B stores of 16-lane runs made the epilogue store-issue bound
                float* ob = s2f_lds + 2 * BAND + wave * kFwOut;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const bool in = oy < Ho && tx0 + 16 * h + pl < Wo;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = 4 * kq + i;
                        const float v = acc[h][i] + bias[i];
                        ob[m * kWgX + 16 * h + pl] = v;
                        bs0[i] += in ? v : 0.f;
                        bs1[i] += in ? v * v : 0.f;
                    }
                }
                // the row is read back as f32x4 by other lanes of this wave: a compiler barrier
                // keeps those reads after the float stores (different types: no alias assumed)
                asm volatile("" ::: "memory");
                if (oy < Ho) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int m = (lane >> 3) + 8 * u, q = lane & 7, ox = tx0 + 4 * q;
                        if (m < a.M && ox < Wo)
                            gst4(obase, (int64_t)tn * ons + (int64_t)m * Ho * Wo + (int64_t)oy * Wo + ox,
                                 *reinterpret_cast<const f32x4*>(&ob[m * kWgX + 4 * q]));
                    }
                }
            } else {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int ox = tx0 + 16 * h + pl;
                    if (oy >= Ho || ox >= Wo) continue;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = 4 * kq + i;
                        if (m >= a.M) continue;
                        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
                        sink_row_apply(ri[m], tn, (int64_t)oy * Wo + ox, acc[h][i], s0, s1, s2);
                        bs0[i] += s0;
                        bs1[i] += s1;
                        bs2[i] += s2;
                    }
                }
            }
            __syncthreads();
            if (t == t0) STAMP(5);
        }
        STAMP(6);
        if (sinks_need_red(a.out)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float r0 = dpp_row16_sum(bs0[i]), r1 = dpp_row16_sum(bs1[i]), r2 = dpp_row16_sum(bs2[i]);
                if (pl == 0) {
                    red[wave][0][4 * kq + i] = r0;
                    red[wave][1][4 * kq + i] = r1;
                    red[wave][2][4 * kq + i] = r2;
                }
            }
        }
        __syncthreads();  // E
        if (sinks_need_red(a.out) && tid < a.M && t0 < t1) {
            float r3[3];
#pragma unroll
            for (int q3 = 0; q3 < 3; ++q3)
                r3[q3] = ((red[0][q3][tid] + red[1][q3][tid]) + red[2][q3][tid]) + red[3][q3][tid];
            sink_row_flush(a.out, tid, r3[0], r3[1], r3[2]);
        }
    }
    STAMP(7);
}

bool down_geom(const isg_conv_geom* g, int& S) {
    S = g->SH;
    return g->groups == 1 && (S == 2 || S == 4) && g->SW == S && g->KH == 2 * S && g->KW == 2 * S &&
           g->PH == S / 2 && g->PW == S / 2 && g->DH == 1 && g->DW == 1 && g->H == S * g->OH &&
           g->W == S * g->OW && g->W % 4 == 0 && (g->w_ci == 0 || g->w_ci == g->Ci);
}

bool down_src_ok(const isg_vtensor* v) {
    for (int i = 0; i < v->nseg; ++i) {
        const isg_vseg& s = v->s[i];
        if ((uintptr_t)s.p % 16 || s.n_stride % 4) return false;
        if (s.xform == ISG_XF_BN_BWD && ((uintptr_t)s.y % 16 || s.y_n_stride % 4)) return false;
    }
    return true;
}

}  // namespace

ISG_STAMP_ACCESSOR(isg_dbg_stamps_down)

// Returns 1 if launched, 0 if the shape is not for these kernels, <0 on error.
int32_t isg_down_conv_fwd(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                          const isg_sinks* out, hipStream_t st) {
    int S = 0;
    if (!down_geom(g, S) || g->Ci > kMaxC || g->Co > kMaxM || !down_src_ok(src)) return 0;
    // measured: S = 2 (bottle5_1up's k4 s2, 128^2 cells) ran 15.6 -> 18.2 us here against the
    // halo kernel (too few cells per lane-owned output for the VALU form); S = 4 only
    if (S != 4) return 0;
    DownArgs a{};
    a.dy = *src; a.out = *out; a.w = w;
    a.N = g->N; a.M = g->Co; a.C = g->Ci; a.H = g->OH; a.W = g->OW;
    const dim3 grid((unsigned)(((int64_t)a.N * a.H * a.W + kThreads - 1) / kThreads));
    if (S == 4) {
        if (a.M <= 4) hipLaunchKernelGGL((down_conv_kernel<4, 4>), grid, dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((down_conv_kernel<4, 16>), grid, dim3(kThreads), 0, st, a);
    } else {
        if (a.M <= 4) hipLaunchKernelGGL((down_conv_kernel<2, 4>), grid, dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((down_conv_kernel<2, 16>), grid, dim3(kThreads), 0, st, a);
    }
    const int32_t e = isg_check_launch("down_conv_kernel");
    return e ? e : 1;
}

// weight gradient of the stride-S down conv: dy = the conv's OUTPUT gradient (M channels
// on the cell grid), x = its input (C channels, S x the grid) — the plan's roles
int32_t isg_down_conv_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                            double* dw, double* dbias, int64_t rep_stride, int32_t nrep,
                            hipStream_t st) {
    int S = 0;
    if (dbias || !down_geom(g, S) || g->Ci > kMaxC || g->Co > kMaxM) return 0;
    if (g->Ci * 4 * S * S > kThreads) return 0;
    DownArgs a{};
    a.x = *dy;   // M channels on the cell grid
    a.dy = *x;   // C channels at S x the resolution
    a.dw = dw;
    a.rep_stride = nrep > 1 ? rep_stride : 0;
    a.nrep = nrep < 1 ? 1 : nrep;
    a.N = g->N; a.M = g->Co; a.C = g->Ci; a.H = g->OH; a.W = g->OW;
    constexpr int TY = 4, TX = 16;
    a.tiles_x = (a.W + TX - 1) / TX;
    a.ntiles = a.N * a.tiles_x * ((a.H + TY - 1) / TY);
    // ~2 tiles per workgroup (measured on the head's k8 s4: 4 tiles 74 us, 2 tiles 58 us,
    // 8 tiles 127 us — parallelism, not the dW atomics, bounds it)
    const int grid = std::max(1, std::min(a.ntiles, std::max(512, a.ntiles / 2)));
    if (S == 4) {
        if (a.M <= 4) hipLaunchKernelGGL((down_wgrad_kernel<4, 4, TY, TX>), dim3(grid), dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((down_wgrad_kernel<4, 16, TY, TX>), dim3(grid), dim3(kThreads), 0, st, a);
    } else {
        if (a.M <= 4) hipLaunchKernelGGL((down_wgrad_kernel<2, 4, TY, TX>), dim3(grid), dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((down_wgrad_kernel<2, 16, TY, TX>), dim3(grid), dim3(kThreads), 0, st, a);
    }
    const int32_t e = isg_check_launch("down_wgrad_kernel");
    return e ? e : 1;
}

// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
int32_t isg_sub2_dgrad(const isg_conv_geom* g, const isg_vtensor* dy, const float* w,
                       const isg_sinks* dx, hipStream_t st) {
    if (g->groups != 1 || g->SH != 2 || g->SW != 2 || g->KH != 5 || g->KW != 5 ||
        g->PH != 2 || g->PW != 2 || g->DH != 1 || g->DW != 1 || g->H != 2 * g->OH ||
        g->W != 2 * g->OW || g->Co > kMaxM || g->Ci > kMaxM || (g->w_ci && g->w_ci != g->Ci))
        return 0;
    DownArgs a{};
    a.dy = *dy; a.out = *dx; a.w = w;
    a.N = g->N; a.M = g->Ci; a.C = g->Co; a.H = g->OH; a.W = g->OW;
    const dim3 grid((unsigned)((a.W + 63) / 64), (unsigned)((a.H + kRowsPB - 1) / kRowsPB), (unsigned)a.N);
    if (a.W % 4 || !down_src_ok(dy)) return 0;  // tap_conv's stride-1 phases instead
    hipLaunchKernelGGL(sub2_dgrad_lds_kernel, grid, dim3(kThreads), 0, st, a);
    const int32_t e = isg_check_launch("sub2_dgrad_kernel");
    return e ? e : 1;
}

// 5x5 stride 2 pad 2 forward with <= 16 input / output channels (s2k5_fwd_kernel).
// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
int32_t isg_s2k5_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                     const isg_sinks* out, hipStream_t st) {
    if (g->groups != 1 || g->SH != 2 || g->SW != 2 || g->KH != 5 || g->KW != 5 ||
        g->PH != 2 || g->PW != 2 || g->DH != 1 || g->DW != 1 || g->H != 2 * g->OH ||
        g->W != 2 * g->OW || g->W % 4 || g->Co > kMaxM || g->Ci > kMaxM ||
        (g->w_ci && g->w_ci < g->Ci) || !down_src_ok(x))
        return 0;
    for (int i = 0; i < x->nseg; ++i)  // the branch-free staging transform: PLAIN / BN_FWD
        if (x->s[i].xform == ISG_XF_BN_BWD) return 0;
    if ((int64_t)g->H * g->W >= (1ll << 31)) return 0;
    S2fArgs a{};
    a.x = *x; a.w = w; a.out = *out;
    a.st16 = out->nsink == 1 && out->s[0].mode == ISG_SINK_STORE && out->s[0].c0 == 0 &&
             out->s[0].C == g->Co && g->OW % 4 == 0 && (uintptr_t)out->s[0].p % 16 == 0 &&
             out->s[0].n_stride % 4 == 0;
    a.N = g->N; a.M = g->Co; a.C = g->Ci; a.wc = g->w_ci ? g->w_ci : g->Ci; a.OH = g->OH; a.OW = g->OW;
    const int G = (a.C + 3) / 4;
    if (a.wc > (G == 4 ? 16 : kS2fMaxWc)) return 0;  // the whole-weight copy's bound
    a.tiles_x = (a.OW + kWgX - 1) / kWgX;
    a.tiles_y = (a.OH + kWgRows - 1) / kWgRows;
    const int64_t nt = (int64_t)a.N * a.tiles_x * a.tiles_y;
    if (nt >= (1ll << 31)) return 0;
    a.ntiles = (int)nt;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
    }
    const int target = cus;  // one 8-wave workgroup per CU (LDS 2 x 52 KB + 8 KB)
    a.tpw = (int)std::max<int64_t>(1, (nt + target - 1) / target);
    const int grid = (int)((nt + a.tpw - 1) / a.tpw);
    // two bands + the four consumer waves' output rows (st16 epilogue)
    const size_t lds = ((size_t)2 * kMaxM * kFwPL + 4 * kFwOut) * sizeof(float);
    auto k = G == 1 ? s2k5_fwd_kernel<1> : G == 2 ? s2k5_fwd_kernel<2> : G == 3 ? s2k5_fwd_kernel<3>
                                                                                : s2k5_fwd_kernel<4>;
    static bool attr[5] = {false, false, false, false, false};
    if (!attr[G]) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return isg_check_launch("s2k5_fwd_kernel: dynamic LDS");
        attr[G] = true;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(2 * kThreads), lds, st, a);
    const int32_t e = isg_check_launch("s2k5_fwd_kernel");
    return e ? e : 1;
}

// 5x5 stride 2 pad 2 weight gradient with <= 16 input / output channels (s2k5_wgrad_kernel).
// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
int32_t isg_s2k5_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                       double* dw, double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st) {
    if (g->groups != 1 || g->SH != 2 || g->SW != 2 || g->KH != 5 || g->KW != 5 ||
        g->PH != 2 || g->PW != 2 || g->DH != 1 || g->DW != 1 || g->H != 2 * g->OH ||
        g->W != 2 * g->OW || g->OW % 4 || g->Co > kMaxM || g->Ci > kMaxM ||
        (g->w_ci && g->w_ci < g->Ci) || !down_src_ok(x) || !down_src_ok(dy))
        return 0;
    // the kernel's branch-free transforms: x PLAIN / BN_FWD with any activation, dy PLAIN /
    // BN_BWD without one
    for (int i = 0; i < x->nseg; ++i)
        if (x->s[i].xform == ISG_XF_BN_BWD) return 0;
    for (int i = 0; i < dy->nseg; ++i)
        if (dy->s[i].xform == ISG_XF_BN_FWD || dy->s[i].act != ISG_ACT_NONE) return 0;
    if ((int64_t)g->H * g->W >= (1ll << 31)) return 0;
    S2wArgs a{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias;
    a.rep_stride = nrep > 1 ? rep_stride : 0;
    a.nrep = nrep < 1 ? 1 : nrep;
    a.N = g->N; a.M = g->Co; a.C = g->Ci; a.wc = g->w_ci ? g->w_ci : g->Ci; a.OH = g->OH; a.OW = g->OW;
    a.tiles_x = (a.OW + kWgX - 1) / kWgX;
    a.tiles_y = (a.OH + kWgRows - 1) / kWgRows;
    const int64_t nt = (int64_t)a.N * a.tiles_x * a.tiles_y;
    if (nt >= (1ll << 31)) return 0;
    a.ntiles = (int)nt;
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
    }
    const int target = cus;  // one 8-wave workgroup per CU (LDS 2 x 60 KB)
    a.tpw = (int)std::max<int64_t>(1, (nt + target - 1) / target);
    const int grid = (int)((nt + a.tpw - 1) / a.tpw);
    bool yb = false;
    for (int i = 0; i < dy->nseg; ++i) yb |= dy->s[i].xform == ISG_XF_BN_BWD && dy->s[i].y != dy->s[i].p;
    const size_t lds = (size_t)2 * kWgLds * sizeof(float);
    const int nar = a.C > 4 ? 0 : a.C <= 3 ? 1 : 2;
    auto k = yb ? (nar == 1 ? s2k5_wgrad_kernel<true, 5> : nar == 2 ? s2k5_wgrad_kernel<true, 7> : s2k5_wgrad_kernel<true, 0>)
                : (nar == 1 ? s2k5_wgrad_kernel<false, 5> : nar == 2 ? s2k5_wgrad_kernel<false, 7> : s2k5_wgrad_kernel<false, 0>);
    const int ki = 3 * yb + nar;
    static bool attr[6] = {false, false, false, false, false, false};
    if (!attr[ki]) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return isg_check_launch("s2k5_wgrad_kernel: dynamic LDS");
        attr[ki] = true;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(2 * kThreads), lds, st, a);
    const int32_t e = isg_check_launch("s2k5_wgrad_kernel");
    return e ? e : 1;
}
