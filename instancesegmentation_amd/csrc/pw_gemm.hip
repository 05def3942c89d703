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
        RowInfo q = {};
        q.mode = -1;
        if (r < Mb) {  // (sink_row: the lane's sink read at a constant index)
            const SinkRow w = sink_row(a.out, m0 + r, a.HW);
            q.p = w.p; q.y = w.y; q.ns = (int)w.ns; q.yns = (int)w.yns;
            q.mode = w.mode; q.act = w.act; q.bias = w.bias; q.f = w.f;
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
                const float t = ch_xform_u(c.xf, c.act, c.k, v[u], yv[u]);  // k is wave-uniform
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
            sink_row_flush(a.out, m0 + rl, red[0][0][rl], red[0][1][rl], red[0][2][rl]);
        }
    }
}

// ---- pwx: whole-K slab kernel (the path every aligned layer takes) ----------------------
// The chunked kernel above serialises one load round trip per 32-channel chunk behind a
// barrier, with 4-B loads: at 64 pixels x 32 channels per trip the 1x1 layers ran at
// 0.3-0.5 TB/s. This variant moves the whole problem of a workgroup into LDS at once:
//   * the BM x K weight slice (16-B loads along whichever of m / k is contiguous) and the
//     K x BP activation slab (16-B loads, lane = 4 consecutive pixels of one channel, the
//     producer's BatchNorm/activation or BatchNorm-backward applied on the way in), with
//     up to 8 loads per lane in flight per batch;
//   * then one branch-free MFMA loop over K. The A fragment is read 4 k-steps at a time
//     with one ds_read_b128: MFMA step j of k-group g gives lane slot kk the channel
//     16g + 4kk + j, for A and B alike (a permutation of the reduction order only).
// Bank layout: As row stride = 8 mod 64 floats (conflict-free b128 fragment reads), Xs row
// stride = 16 mod 32 (conflict-free b32 B reads).
constexpr int kPxMaxLds = 160 * 1024 - 256;

struct PwxArgs {
    isg_vtensor src;
    isg_sinks out;
    const float* w;
    int rs, cs;
    int HW, M, K, Kp, BM, AS, XS;
    int off_k, off_ri, off_a, off_x;  // dynamic LDS byte offsets (tabA at 0)
    int wmode;                        // 1: f32x4 along k (forward), 2: f32x4 along m (dgrad)
    int fast;                         // every record is plain loads (finalised BN coefficients)
    int wu, xu;                       // weight / activation quads per lane actually needed
    int wsh;                          // log2 of the weight quads per row, padded to a power of 2
    int stat_on;                      // some channel or sink row evaluates its BN statistics
    int pre_on;                       // some sink reads an operand (ACTBWD y / ACCUM old value)
    int res_on;                       // the one sink is ACTBWD's residual form (isg.h isg_sink)
    int rbn_in, rbn_out;              // ... with a BatchNorm'd residual (vtensor.rbn / sink rbn)
    int64_t P;
};

// Phases (each a single memory round trip; loads are never behind a branch, see stage.h):
//   1. per-channel coefficient + per-row sink loads, the BM x K weight slice (<= 8 x 16 B
//      per lane, clamped duplicates past the end) and the LDS addressing table;
//   2. barrier; the K x BP activation slab (<= 8 x 16 B per lane, + the saved forward
//      output when HY), while phase-1 results are written to LDS;
//   3. the producer transform on the way into Xs; 4. MFMA; 5. epilogue with its sink
//      operands (saved y / old value) loaded for all accumulator elements at once.
// SEG1: one source segment and one sink — the per-lane segment selection folds away (the
// prologue's address arithmetic was the first phase's cost: ~1,250 instructions per wave
// before the first barrier with three-way selects, 64-bit and runtime-divisor integer math)
// The residual term's own BatchNorm (isg.h vtensor.rbn / sink rbn) for one channel: its
// coefficient or statistics loads in the caller's round trip (`on` lane-invariant: no
// load at all on the common path), then (mean, gamma*rstd, beta)
struct RbnLoad {
    f32x4 f;
    StatLoad<2> st;
};
ISG_DEV RbnLoad rbn_issue(const isg_bn& bn, int cl, const float* any, bool on) {
    RbnLoad r;
    const float* coef = sgpr_p((const float*)bn.coef);
    r.f = f32x4{0.f, 1.f, 0.f, 0.f};
    if (on && coef) r.f = gld4(coef, 4 * (int64_t)cl);
    r.st = stat_issue<2>(coef ? nullptr : sgpr_p((const double*)bn.stats), sgpr_p(bn.gamma),
                         sgpr_p(bn.beta), sgpr_i(bn.C), cl, any, on && !coef);
    return r;
}
ISG_DEV ChanCoef rbn_finish(const isg_bn& bn, const RbnLoad& l) {
    if (bn.coef) return ChanCoef{l.f[0], l.f[1], l.f[2], 0.f};
    double mean, rstd;
    mean_rstd_of(stat_sum(l.st, 0), stat_sum(l.st, 1), sgpr_f(bn.count), sgpr_f(bn.eps), mean, rstd);
    return fwd_coef_of(mean, rstd, l.st.gamma, l.st.beta, 0.f);
}

// RES: the one sink is ACTBWD's residual form — its extra operands and reductions exist
// only in these instantiations (kept out of the common kernels, where their live registers
// cost occupancy); with SEG1 false the source is a K-stacked pair's two gradient segments
template <int TPW, int BP, bool HY, bool SEG1, bool RES>
__global__ __launch_bounds__(kThreads) void pwx_kernel(PwxArgs a) {
    constexpr bool SINK1 = SEG1 || RES;  // one sink: its operands issued in the first round trip
    extern __shared__ f32x4 pwx_smem[];
    char* const smem = reinterpret_cast<char*>(pwx_smem);
    ChSrc* const tabA = reinterpret_cast<ChSrc*>(smem);  // kThreads entries (clamped past K)
    ChanCoef* const tabK = reinterpret_cast<ChanCoef*>(smem + a.off_k);
    ChanCoef* const tabK2 = tabK + a.K;  // residual BatchNorm: per channel (fwd) / per row (dgrad)
    RowInfo* const ri = reinterpret_cast<RowInfo*>(smem + a.off_ri);
    float* const As = reinterpret_cast<float*>(smem + a.off_a);
    float* const Xs = reinterpret_cast<float*>(smem + a.off_x);
    constexpr int QPR = BP / 4;          // pixel quads per channel row
    constexpr int CPP = kThreads / QPR;  // channel rows per staging pass
    constexpr int CT = BP / 16;          // pixel tiles
    constexpr int XU = 8, WU = 8;        // activation / weight loads per lane

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = wave_id();
    const int kk = lane >> 4, pl = lane & 15;
    const int BM = a.BM, K = a.K, Kp = a.Kp, AS = a.AS, XS = a.XS;
    const int m0 = blockIdx.y * BM;
    const int Mb = min(BM, a.M - m0);
    const int64_t p0 = (int64_t)blockIdx.x * BP;
    const float* __restrict__ w = a.w;
    STAMP(0);

    if (!a.fast) {  // fp64 evaluation from the statistics (eval / direct ABI calls)
        for (int c = tid; c < K; c += kThreads) tabK[c] = vt_coef(a.src, c);
        for (int r = tid; r < Mb; r += kThreads) {
            const SinkRow q = sink_row(a.out, m0 + r, a.HW);
            RowInfo& d = ri[r];
            d.p = q.p; d.y = q.y; d.ns = (int)q.ns; d.yns = (int)q.yns;
            d.mode = q.mode; d.act = q.act; d.bias = q.bias; d.f = q.f;
        }
    }
    // ---- phase 1 ------------------------------------------------------------------------
    VtSel vs = vt_sel(a.src);
    SkSel ks = sk_sel(a.out);
    if constexpr (SEG1) vs.nseg = 1;
    if constexpr (SINK1) ks.nsink = 1;
    // ---- phase 2 first: the activation slab loads (HBM, the longest latency) lead the
    //      round trip; their channel addresses come from the kernel arguments alone, only
    //      the transform needs the coefficient table, after the barrier
    const int q = tid % QPR, cr = tid / QPR;
    const int64_t pg = p0 + 4 * q;
    const bool pv = pg < a.P;
    const int n = pv ? (int)((uint32_t)pg / (uint32_t)a.HW) : 0;  // P < 2^31 (host check)
    const int pix = pv ? (int)pg - n * a.HW : 0;
    f32x4 xv[XU], yv[XU];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        xv[u] = yv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (u >= a.xu) continue;
        const ChSrc t = ch_addr(vs, min(cr + u * CPP, K - 1), a.HW);
        xv[u] = gld4(t.p, (int64_t)n * t.ns + pix);
        if (HY) yv[u] = gld4(t.y, (int64_t)n * t.yns + pix);
    }
    const int tc = min(tid, K - 1);
    // every load below is issued only where it is needed: a lane-invariant (SGPR) guard per
    // unrolled slot — the per-CU vector-memory issue of dummy duplicates was the first round
    // trip's cost (kbench stamps: 5.2 us for ~60 load instructions per wave)
    const bool stat_on = a.stat_on != 0;
    const CoefLoad<HY ? 4 : 2> cfl = coef_issue<HY ? 4 : 2>(vs, tc, stat_on);
    const int trow = min(tid, Mb - 1);
    const SinkLoad skl = sink_issue(ks, m0 + trow, w, stat_on);
    // the residual's BatchNorm: forward per input channel, input gradient per output row
    const bool rbn_in = SEG1 && HY && a.rbn_in != 0, rbn_out = RES && a.rbn_out != 0;

    // weight slot i -> (row, quad): quads per row padded to 2^wsh, so the split is a shift
    // and a mask; forward rows are m with k contiguous, dgrad rows are k with m contiguous.
    // Padding slots load a clamped duplicate and are dropped at the LDS store.
    const int wsh = a.wsh, wmask = (1 << wsh) - 1;
    f32x4 wv[WU];
#pragma unroll
    for (int u = 0; u < WU; ++u) {
        wv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (u >= a.wu) continue;
        const int i = tid + u * kThreads;
        const int r = i >> wsh, qd = (i & wmask) * 4;
        const int o = a.wmode == 1 ? (m0 + min(r, Mb - 1)) * a.rs + min(qd, K - 4)
                                   : min(r, K - 1) * a.cs + m0 + min(qd, Mb - 4);
        wv[u] = gld4(w, o);
    }
    tabA[tid] = ch_addr(vs, tc, a.HW);
    // the epilogue's sink operands (saved forward output for ACTBWD, old value for ACCUM):
    // with one sink their addresses come from the kernel arguments, so they are issued in
    // this same round trip instead of after the MFMA loop
    constexpr int CT_ = BP / 16;
    const int nt_ = (BM / 16) * CT_;
    // sink operands: y / old value, + the residual form's old gradient, residual term and
    // p2's old value
    constexpr int TR = RES ? TPW : 1;
    float pre[TPW][4], pro[TR][4], prr[TR][4], pp2[TR][4];
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) pre[i][r] = 0.f;
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) pro[i][r] = prr[i][r] = pp2[i][r] = 0.f;
    if (SINK1 && a.pre_on) {
        const SinkLite& k0 = ks.s0;
        const bool ab = k0.mode == ISG_SINK_ACTBWD;
        const float* base = ab ? k0.y : k0.p;
        const int bns = ab ? k0.yns : k0.ns;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int t = min(wave + 4 * i, nt_ - 1);
            const int rt = t / CT_, ct = t % CT_;
            const int64_t pe = p0 + ct * 16 + pl;
            const bool pve = pe < a.P;
            const int ne = pve ? (int)((uint32_t)pe / (uint32_t)a.HW) : 0;
            const int pixe = pve ? (int)pe - ne * a.HW : 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int cl = min(rt * 16 + kk * 4 + r, Mb - 1) + m0 - k0.c0;
                pre[i][r] = gld(base, (int64_t)cl * a.HW + (int64_t)ne * bns + pixe);
            }
        }
    }
    __syncthreads();
    STAMP(1);
    // phase-1 results -> LDS (waits for phase-1 loads only)
    // the residual's own BatchNorm (two-BN tails only, 4 launches per step): its own round
    // trip inside a uniform branch, so no state of it stays live in the common kernels
    if (rbn_in) {
        const RbnLoad rbl = rbn_issue(a.src.rbn, tc, w, true);
        if (tid < K) tabK2[tid] = rbn_finish(a.src.rbn, rbl);
    } else if (rbn_out) {
        const RbnLoad rbl = rbn_issue(a.out.s[0].rbn, trow + m0 - a.out.s[0].c0, w, true);
        if (tid < Mb) tabK2[tid] = rbn_finish(a.out.s[0].rbn, rbl);
    }
    if (a.fast) {
        if (tid < K) tabK[tid] = coef_finish(vs, tid, cfl);
        if (tid < Mb) {
            const SinkRow sq = sink_finish(ks, m0 + tid, a.HW, skl);
            RowInfo& d = ri[tid];
            d.p = sq.p; d.y = sq.y; d.ns = (int)sq.ns; d.yns = (int)sq.yns;
            d.mode = sq.mode; d.act = sq.act; d.bias = sq.bias; d.f = sq.f;
        }
    }
    if (tid >= Mb && tid < BM) ri[tid].mode = -1;
#pragma unroll
    for (int u = 0; u < WU; ++u) {
        if (u >= a.wu) continue;
        const int i = tid + u * kThreads;
        const int r = i >> wsh, qd = (i & wmask) * 4;
        if (a.wmode == 1) {  // r = m, qd = k4
            if (r < BM && qd < Kp) {
                const bool ok = r < Mb && qd < K;
                *reinterpret_cast<f32x4*>(&As[r * AS + qd]) = ok ? wv[u] : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        } else if (r < Kp && qd < BM) {  // r = k, qd = m4
#pragma unroll
            for (int e = 0; e < 4; ++e) As[(qd + e) * AS + r] = (r < K && qd + e < Mb) ? wv[u][e] : 0.f;
        }
    }
    __syncthreads();
    STAMP(2);

    // ---- phase 3: producer transform into Xs[k][p] --------------------------------------
    // the materialised input (isg_vtensor.mat: a folded residual tail's block output),
    // written once per pixel by the first row block
    float* const mat = blockIdx.y == 0 ? a.src.mat : nullptr;  // host: one segment
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        const int c = cr + u * CPP;
        if (c < Kp) {
            // the channel differs between lanes: branch-free transform (XfLin)
            const bool live = c < K && pv;
            const ChSrc t = tabA[c];
            const XfLin l = xf_lin(t.xf, t.act, tabK[c]);
            f32x4 o;
            if constexpr (HY) {  // BN_FWD with a residual term (isg_vseg): y is the residual
                const float isr = t.xf == ISG_XF_BN_FWD && t.y != t.p ? 1.f : 0.f;
                f32x4 rv = yv[u];
                if (rbn_in) {  // the residual's own BatchNorm, the tail's (x - mean) * k + beta
                    const ChanCoef k2 = tabK2[c < K ? c : K - 1];
#pragma unroll
                    for (int e = 0; e < 4; ++e) rv[e] = (rv[e] - k2.c0) * k2.c1 + k2.c2;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = xf_lin_apply_r(l, xv[u][e], rv[e], isr);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = xf_lin_apply(l, xv[u][e], xv[u][e]);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = live ? o[e] : 0.f;
            *reinterpret_cast<f32x4*>(&Xs[c * XS + 4 * q]) = o;
            if (mat && live) gst4(mat, (int64_t)n * a.src.mat_n_stride + (int64_t)c * a.HW + pix, o);
        }
    }
    __syncthreads();
    STAMP(3);

    // the residual form's operands (old gradient, residual term, p2's old value): issued
    // here, once the staging registers are dead, so they are in flight during the MFMA loop
    // — held from the first round trip they kept 3 x 4 x TPW more registers live through
    // the staging (254 VGPRs: one wave per SIMD)
    if constexpr (RES) {
        if (a.pre_on) {
            const SinkLite& k0 = ks.s0;
            // lane-invariant; r is non-NULL in the residual form (host check)
            const bool res_old = k0.old != nullptr;
            const bool res_p2a = k0.p2 != nullptr && k0.p2acc != 0;
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                const int t = min(wave + 4 * i, nt_ - 1);
                const int rt = t / CT_, ct = t % CT_;
                const int64_t pe = p0 + ct * 16 + pl;
                const bool pve = pe < a.P;
                const int ne = pve ? (int)((uint32_t)pe / (uint32_t)a.HW) : 0;
                const int pixe = pve ? (int)pe - ne * a.HW : 0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t o = (int64_t)(min(rt * 16 + kk * 4 + r, Mb - 1) + m0 - k0.c0) * a.HW + pixe;
                    if (res_old) pro[i][r] = gld(k0.old, o + (int64_t)ne * k0.ons);
                    prr[i][r] = gld(k0.r, o + (int64_t)ne * k0.rns);
                    if (res_p2a) pp2[i][r] = gld(k0.p2, o + (int64_t)ne * k0.p2ns);
                }
            }
        }
    }

    // ---- phase 4: MFMA, tile t = wave + 4i -> row tile t / CT, pixel tile t % CT ---------
    const int nt = (BM / 16) * CT;
    int aoff[TPW], boff[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = min(wave + 4 * i, nt - 1);  // surplus tiles recompute the last one
        aoff[i] = ((t / CT) * 16 + pl) * AS + 4 * kk;
        boff[i] = (4 * kk) * XS + (t % CT) * 16 + pl;
    }
    f32x4 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int g = 0; g < Kp; g += 16) {
        f32x4 a4[TPW];
#pragma unroll
        for (int i = 0; i < TPW; ++i) a4[i] = *reinterpret_cast<const f32x4*>(&As[aoff[i] + g]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                const float bv = Xs[boff[i] + (g + j) * XS];
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[i][j], bv, acc[i], 0, 0, 0);
            }
    }
    STAMP(4);
    // ---- phase 5: epilogue; lane holds D[row = rt*16 + kk*4 + r][pixel = ct*16 + pl] ----
    // sink operands first (saved forward output for ACTBWD, old value for ACCUM), all in
    // flight together; other rows load a dummy word
    if (!SINK1 && a.pre_on) {
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int t = min(wave + 4 * i, nt - 1);
            const int rt = t / CT, ct = t % CT;
            const int64_t pe = p0 + ct * 16 + pl;
            const bool pve = pe < a.P;
            const int ne = pve ? (int)((uint32_t)pe / (uint32_t)a.HW) : 0;
            const int pixe = pve ? (int)pe - ne * a.HW : 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const RowInfo& qi = ri[rt * 16 + kk * 4 + r];
                const float* src = w;
                int64_t off = 0;
                if (qi.mode == ISG_SINK_ACTBWD) { src = qi.y; off = (int64_t)ne * qi.yns + pixe; }
                if (qi.mode == ISG_SINK_ACCUM) { src = qi.p; off = (int64_t)ne * qi.ns + pixe; }
                if (!pve) { src = w; off = 0; }
                pre[i][r] = gld(src, off);
            }
        }
    }
    const bool need_red = sinks_need_red(a.out);
    float (*red)[4][kMaxBM] = reinterpret_cast<float (*)[4][kMaxBM]>(Xs);
    if (need_red) {
        __syncthreads();  // every wave is past its Xs reads
        for (int i = tid; i < 4 * 4 * kMaxBM; i += kThreads) (&red[0][0][0])[i] = 0.f;
        __syncthreads();
    }
    STAMP(5);
    // one sink: its mode / activation / bases are lane-invariant (scalar), only the rows'
    // coefficients and biases come from LDS — every row's read issued before the first use.
    // (The generic loop below reads the whole row record per row behind a branch on its
    // mode: a chain of dependent LDS round trips per element.) Same arithmetic per element.
    if constexpr (SINK1) {
        const SinkLite& k0 = ks.s0;
        const int mode = k0.mode, act = k0.act;
        const bool live = mode == ISG_SINK_STORE || mode == ISG_SINK_ACCUM || mode == ISG_SINK_ACTBWD;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int t = wave + 4 * i;
            if (t >= nt || !live) continue;  // wave-uniform
            const int rt = t / CT, ct = t % CT;
            if (rt * 16 >= Mb) continue;
            const int64_t pe = p0 + ct * 16 + pl;
            const bool pve = pe < a.P;
            const int ne = pve ? (int)((uint32_t)pe / (uint32_t)a.HW) : 0;
            const int pixe = pve ? (int)pe - ne * a.HW : 0;
            SinkCoef fr[4];
            float br[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const RowInfo& qi = ri[min(rt * 16 + kk * 4 + r, Mb - 1)];
                fr[r] = qi.f;
                br[r] = qi.bias;
            }
            float s0[4], s1[4], s2[4], s3[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                s0[r] = s1[r] = s2[r] = s3[r] = 0.f;
                const int rl = rt * 16 + kk * 4 + r;
                if (!pve || rl >= Mb) continue;
                float v = acc[i][r];
                const int64_t cl = rl + m0 - k0.c0;
                const int64_t off = cl * a.HW + (int64_t)ne * k0.ns + pixe;
                if (mode == ISG_SINK_STORE) {
                    v += br[r];
                    gst(k0.p, off, v);
                    s0[r] = v;
                    s1[r] = v * v;
                } else if (mode == ISG_SINK_ACCUM) {
                    gst(k0.p, off, pre[i][r] + v);
                    s0[r] = v;
                    s1[r] = v * v;
                } else {
                    const SinkCoef& f = fr[r];
                    const float y = pre[i][r];
                    float z = (y - f.mean) * f.scale + f.beta;
                    ChanCoef k2 = {0.f, 1.f, 0.f, 0.f};
                    if constexpr (RES) {  // residual form: + old gradient, + residual term
                        v = pro[i][r] + v;
                        float rv = prr[i][r];
                        if (rbn_out) {  // the residual's own BatchNorm (two-BN tail)
                            k2 = tabK2[rl];
                            rv = (rv - k2.c0) * k2.c1 + k2.c2;
                        }
                        z = z + rv;
                    }
                    float gv = v;
                    if (act == ISG_ACT_RELU) {
                        gv = z > 0.f ? v : 0.f;
                    } else if (act == ISG_ACT_PRELU) {
                        gv = z > 0.f ? v : v * f.slope;
                        s2[r] = z > 0.f ? 0.f : z * v;
                    }
                    gst(k0.p, off, gv);
                    if constexpr (RES) {
                        if (k0.p2)
                            gst(k0.p2, cl * a.HW + (int64_t)ne * k0.p2ns + pixe, k0.p2acc ? pp2[i][r] + gv : gv);
                        if (rbn_out) s3[r] = gv * (prr[i][r] - k2.c0);  // centred on the residual's mean
                    }
                    s0[r] = gv;
                    s1[r] = gv * (y - f.mean);
                }
            }
            if (need_red) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t0 = row16_sum(s0[r]);
                    const float t1 = row16_sum(s1[r]);
                    const float t2 = row16_sum(s2[r]);
                    const float t3 = rbn_out ? row16_sum(s3[r]) : 0.f;
                    const int rl = rt * 16 + kk * 4 + r;
                    if (pl == 0 && rl < Mb) {
                        red[wave][0][rl] += t0;
                        red[wave][1][rl] += t1;
                        red[wave][2][rl] += t2;
                        red[wave][3][rl] += t3;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        if constexpr (SINK1) break;
        const int t = wave + 4 * i;
        if (t >= nt) continue;  // wave-uniform
        const int rt = t / CT, ct = t % CT;
        if (rt * 16 >= Mb) continue;
        const int64_t pe = p0 + ct * 16 + pl;
        const bool pve = pe < a.P;
        const int ne = pve ? (int)((uint32_t)pe / (uint32_t)a.HW) : 0;
        const int pixe = pve ? (int)pe - ne * a.HW : 0;
        float s0[4], s1[4], s2[4], s3[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            s0[r] = s1[r] = s2[r] = s3[r] = 0.f;
            const int rl = rt * 16 + kk * 4 + r;
            const RowInfo& qi = ri[rl];
            if (!pve || qi.mode < 0 || qi.mode == ISG_SINK_NONE) continue;
            float v = acc[i][r];
            const int64_t off = (int64_t)ne * qi.ns + pixe;
            if (qi.mode == ISG_SINK_STORE) {
                v += qi.bias;
                gst(qi.p, off, v);
                s0[r] = v;
                s1[r] = v * v;
            } else if (qi.mode == ISG_SINK_ACCUM) {
                gst(qi.p, off, pre[i][r] + v);
                s0[r] = v;
                s1[r] = v * v;
            } else {
                const float y = pre[i][r];
                float z = (y - qi.f.mean) * qi.f.scale + qi.f.beta;
                ChanCoef k2 = {0.f, 1.f, 0.f, 0.f};
                if constexpr (RES) {  // residual form: + old gradient, + residual term
                    v = pro[i][r] + v;
                    float rv = prr[i][r];
                    if (rbn_out) {  // the residual's own BatchNorm (two-BN tail)
                        k2 = tabK2[rl];
                        rv = (rv - k2.c0) * k2.c1 + k2.c2;
                    }
                    z = z + rv;
                }
                float gv = v;
                if (qi.act == ISG_ACT_RELU) {
                    gv = z > 0.f ? v : 0.f;
                } else if (qi.act == ISG_ACT_PRELU) {
                    gv = z > 0.f ? v : v * qi.f.slope;
                    s2[r] = z > 0.f ? 0.f : z * v;
                }
                gst(qi.p, off, gv);
                if constexpr (RES) {
                    if (ks.s0.p2)
                        gst(ks.s0.p2, (int64_t)(rl + m0 - ks.s0.c0) * a.HW + (int64_t)ne * ks.s0.p2ns + pixe,
                            ks.s0.p2acc ? pp2[i][r] + gv : gv);
                    if (rbn_out) s3[r] = gv * (prr[i][r] - k2.c0);  // centred on the residual's mean
                }
                s0[r] = gv;
                s1[r] = gv * (y - qi.f.mean);
            }
        }
        if (need_red) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float t0 = row16_sum(s0[r]);
                const float t1 = row16_sum(s1[r]);
                const float t2 = row16_sum(s2[r]);
                const float t3 = rbn_out ? row16_sum(s3[r]) : 0.f;
                const int rl = rt * 16 + kk * 4 + r;
                if (pl == 0 && rl < Mb) {
                    red[wave][0][rl] += t0;
                    red[wave][1][rl] += t1;
                    red[wave][2][rl] += t2;
                    red[wave][3][rl] += t3;
                }
            }
        }
    }
    if (need_red) {
        __syncthreads();
        STAMP(6);
        for (int rl = tid; rl < Mb; rl += kThreads) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                red[0][j][rl] = ((red[0][j][rl] + red[1][j][rl]) + red[2][j][rl]) + red[3][j][rl];
            if constexpr (SINK1) sink_row_flush1(a.out.s[0], m0 + rl, red[0][0][rl], red[0][1][rl], red[0][2][rl]);
            else sink_row_flush(a.out, m0 + rl, red[0][0][rl], red[0][1][rl], red[0][2][rl]);
            if (rbn_out && a.out.s[0].rbn.stats) {  // the residual BatchNorm's backward sums
                const isg_sink& k = a.out.s[0];
                double* sp = rep_ptr(k.rbn.stats, 4 * k.rbn.C);
                const int cl = m0 + rl - k.c0;
                atomicAdd(&sp[2 * k.rbn.C + cl], (double)red[0][0][rl]);
                atomicAdd(&sp[3 * k.rbn.C + cl], (double)red[0][3][rl]);
            }
        }
    }
    STAMP(7);
}

int pwx_align16(int v) { return (v + 15) & ~15; }

// (measured: 256 — one workgroup per CU, fewer and larger tiles — 3.656/3.542 -> 3.801/3.978
// ms per step)
constexpr int kPwxMinBlocks = 512;

// LDS bytes of a (BP, BM) configuration
int pwx_lds(int K, int Kp, int BM, int BP, int& off_k, int& off_ri, int& off_a, int& off_x, int& AS,
            int& XS) {
    AS = Kp + ((8 - Kp % 64) + 64) % 64;
    XS = BP + ((16 - BP % 32) + 32) % 32;  // 16 mod 32 banks
    off_k = pwx_align16(kThreads * (int)sizeof(ChSrc));
    // tabK, then the residual BatchNorm's per-channel / per-row coefficients (two-BN tails)
    off_ri = pwx_align16(off_k + (K + std::max(K, BM)) * (int)sizeof(ChanCoef));
    off_a = pwx_align16(off_ri + BM * (int)sizeof(RowInfo));
    off_x = pwx_align16(off_a + BM * AS * (int)sizeof(float));
    // the epilogue's BN partials [4][3][kMaxBM] reuse the slab
    const int xbytes = std::max(Kp * XS, 4 * 4 * kMaxBM) * (int)sizeof(float);
    return off_x + xbytes;
}

template <int TPW, int BP, bool HY, bool SEG1, bool RES>
int32_t pwx_launch(const PwxArgs& a, dim3 grid, int lds, hipStream_t st) {
    auto k = pwx_kernel<TPW, BP, HY, SEG1, RES>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, kPxMaxLds) != hipSuccess)
            return isg_check_launch("pwx_kernel: dynamic LDS");
        attr = true;
    }
    hipLaunchKernelGGL(k, grid, dim3(kThreads), lds, st, a);
    return isg_check_launch("pwx_kernel");
}

template <int BP, bool HY, bool SEG1, bool RES>
int32_t pwx_dispatch(const PwxArgs& a, dim3 grid, int lds, int tpw, hipStream_t st) {
    switch (tpw) {
        case 1: return pwx_launch<1, BP, HY, SEG1, RES>(a, grid, lds, st);
        case 2: return pwx_launch<2, BP, HY, SEG1, RES>(a, grid, lds, st);
        case 3: return pwx_launch<3, BP, HY, SEG1, RES>(a, grid, lds, st);
        case 4: return pwx_launch<4, BP, HY, SEG1, RES>(a, grid, lds, st);
        case 5: case 6: return pwx_launch<6, BP, HY, SEG1, RES>(a, grid, lds, st);
        default: return pwx_launch<8, BP, HY, SEG1, RES>(a, grid, lds, st);
    }
}
template <int BP, bool HY>
int32_t pwx_dispatch_seg(const PwxArgs& a, dim3 grid, int lds, int tpw, bool seg1, hipStream_t st) {
    if (a.res_on)  // host: one sink
        return seg1 ? pwx_dispatch<BP, HY, true, true>(a, grid, lds, tpw, st)
                    : pwx_dispatch<BP, HY, false, true>(a, grid, lds, tpw, st);
    return seg1 ? pwx_dispatch<BP, HY, true, false>(a, grid, lds, tpw, st)
                : pwx_dispatch<BP, HY, false, false>(a, grid, lds, tpw, st);
}
// weight quads per row padded to a power of two (pwx_kernel's slot split), and the rows
int pwx_wrow_quads(int wmode, int BM, int Kp) {
    int q = wmode == 1 ? Kp / 4 : BM / 4, p = 1;
    while (p < q) p *= 2;
    return p;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// host mirrors of stage.h vt_fast / sinks_fast
bool host_seg_fast(const isg_vseg& s) {
    if (s.xform == ISG_XF_BN_FWD || s.xform == ISG_XF_BN_BWD) return s.bn.coef || s.bn.train;
    return true;
}
bool host_vt_fast(const isg_vtensor& v) {
    for (int s = 0; s < v.nseg; ++s)
        if (!host_seg_fast(v.s[s])) return false;
    return true;
}
bool host_sinks_fast(const isg_sinks& sk) {
    for (int s = 0; s < sk.nsink; ++s) {
        const isg_sink& k = sk.s[s];
        if (k.mode == ISG_SINK_ACTBWD && !(k.bn.coef || k.bn.train)) return false;
    }
    return true;
}

// The slab path needs every source channel row 16-B aligned (HW % 4, n_stride % 4, base).
bool pwx_src_ok(const isg_vtensor& v, int HW) {
    if (HW % 4) return false;
    for (int s = 0; s < v.nseg; ++s) {
        const isg_vseg& g = v.s[s];
        if (!aligned16(g.p) || g.n_stride % 4) return false;
        if ((g.xform == ISG_XF_BN_BWD || g.xform == ISG_XF_BN_FWD) && g.y &&
            (!aligned16(g.y) || g.y_n_stride % 4))
            return false;
    }
    if (v.mat && (!aligned16(v.mat) || v.mat_n_stride % 4)) return false;
    return true;
}


// ---- thin pointwise (K, M <= 16) on the VALU ---------------------------------------------
// The 4 <-> 16 channel 1x1 layers of the stride-4 decoder (bottle5_*, 2 x 256^2 pixels)
// move 10-19 MB each but ran at 0.4-0.5 TB/s on the MFMA kernels: a 16-row tile pads K = 4
// to 16 and every workgroup runs the whole LDS phase chain for 64 pixels. Here one lane
// owns 4 consecutive pixels: its K channel quads are loaded with 16-B loads all at once
// (the producer's transform applied per element), the M x K weights are broadcast from LDS
// as f32x4 along m, and every output row goes through its sink with one 16-B access per
// operand. One-wave workgroups: the BN partials are a wave reduction.
struct ThinPwArgs {
    isg_vtensor src;
    isg_sinks out;
    const float* w;
    int rs, cs;
    int HW;
    int64_t Q;  // pixel quads
};

// gf32x4_p: common.h

// the row's sink operand (ACTBWD: the saved forward output, ACCUM: the old value), loaded
// branch-free before the compute (`any`: a valid address standing in for modes without one)
ISG_DEV f32x4 sink_operand4(const SinkRow& q, int n, int64_t pix, bool pv, const float* any) {
    const bool ab = q.mode == ISG_SINK_ACTBWD, ac = q.mode == ISG_SINK_ACCUM;
    const float* src = ab ? q.y : (ac ? q.p : any);
    const int64_t off = (ab || ac) && pv ? (int64_t)n * (ab ? q.yns : q.ns) + pix : 0;
    return gld4(src, off);
}

ISG_DEV void sink_row_apply4(const SinkRow& q, int n, int64_t pix, f32x4 v, f32x4 opnd, float& s0,
                             float& s1, float& s2) {
    const int64_t off = (int64_t)n * q.ns + pix;
    s0 = s1 = s2 = 0.f;
    if (q.mode == ISG_SINK_STORE) {
        v += q.bias;
        *(gf32x4_p)((gfloat_p)q.p + off) = v;
        s0 = (v[0] + v[1]) + (v[2] + v[3]);
        s1 = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
    } else if (q.mode == ISG_SINK_ACCUM) {
        const f32x4 o = opnd;
        *(gf32x4_p)((gfloat_p)q.p + off) = o + v;
        s0 = (v[0] + v[1]) + (v[2] + v[3]);
        s1 = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
    } else if (q.mode == ISG_SINK_ACTBWD) {
        const f32x4 y = opnd;
        f32x4 g;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
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
        *(gf32x4_p)((gfloat_p)q.p + off) = g;
    }
}

// kThinWaves waves per workgroup (round 3; one-wave workgroups before): the BN partials
// meet in LDS, so a launch adds (quads / 64 / kThinWaves) atomics per statistics address —
// at 4 replicas the one-wave form queued 512 atomics on each address (+10 us per op)
constexpr int kThinWaves = 4;
// PRE: some sink reads an operand (ACTBWD / ACCUM), prefetched with the activations (its
// registers exist only in these instantiations)
template <int K, int M, bool PRE>
__global__ __launch_bounds__(64 * kThinWaves) void thin_pw_kernel(ThinPwArgs a) {
    constexpr int M4 = M / 4;
    __shared__ f32x4 wl[K * M4];  // [k][m/4]
    __shared__ ChT tab[K];
    __shared__ SinkRow ri[M];
    __shared__ float part[kThinWaves][M][3];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m0 = blockIdx.y * M;  // this workgroup's M output rows
    if (tid < K) tab[tid] = ch_table_entry(a.src, tid, a.HW);
    if (tid >= 64 && tid < 64 + M) ri[tid - 64] = sink_row(a.out, m0 + tid - 64, a.HW);
    float* const wf = reinterpret_cast<float*>(wl);
    for (int i = tid; i < K * M; i += 64 * kThinWaves) {
        const int k = i / M, m = i - k * M;
        wf[i] = gld(a.w, (int64_t)(m0 + m) * a.rs + (int64_t)k * a.cs);
    }
    __syncthreads();
    const int64_t qd = (int64_t)blockIdx.x * 64 * kThinWaves + tid;
    const bool pv = qd < a.Q;
    const int64_t p = (pv ? qd : 0) * 4;
    const int n = (int)(p / a.HW);
    const int pix = (int)(p - (int64_t)n * a.HW);
    f32x4 raw[K], ry[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {  // every load in flight together (y == p unless BN-backward)
        const ChT t = tab[k];
        const int yns = t.y == t.p ? t.ns : t.yns;
        raw[k] = gld4(t.p, (int64_t)n * t.ns + pix);
        ry[k] = gld4(t.y, (int64_t)n * yns + pix);
    }
    // the sinks' operands in the same round trip (they were loaded after the compute, one
    // row at a time between the rows' reductions)
    f32x4 opnd[M];
#pragma unroll
    for (int m = 0; m < M; ++m)
        opnd[m] = PRE ? sink_operand4(ri[m], n, pix, pv, a.w) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 acc[M];
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const ChT t = tab[k];
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ch_xform_u(t.xf, t.act, t.k, raw[k][e], ry[k][e]);
#pragma unroll
        for (int q = 0; q < M4; ++q) {
            const f32x4 w4 = wl[k * M4 + q];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[q * 4 + j] += w4[j] * v;
        }
    }
    const bool red = sinks_need_red(a.out);
#pragma unroll
    for (int m = 0; m < M; ++m) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
        if (pv) sink_row_apply4(ri[m], n, pix, acc[m], opnd[m], s0, s1, s2);
        if (red) {
            s0 = wave_sum(s0);
            s1 = wave_sum(s1);
            s2 = wave_sum(s2);
            if (lane == m) {
                part[wave][m][0] = s0;
                part[wave][m][1] = s1;
                part[wave][m][2] = s2;
            }
        }
    }
    if (red) {
        __syncthreads();
        if (tid < M) {
            float r3[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                float v = 0.f;
#pragma unroll
                for (int w = 0; w < kThinWaves; ++w) v += part[w][tid][j];
                r3[j] = v;
            }
            sink_row_flush(a.out, m0 + tid, r3[0], r3[1], r3[2]);
        }
    }
}

bool sinks_aligned16(const isg_sinks& sk) {
    for (int s = 0; s < sk.nsink; ++s) {
        const isg_sink& k = sk.s[s];
        if (k.mode == ISG_SINK_NONE) continue;
        if (!aligned16(k.p) || k.n_stride % 4) return false;
        if (k.mode == ISG_SINK_ACTBWD && (!aligned16(k.y) || k.y_n_stride % 4)) return false;
    }
    return true;
}

// 1: launched, 0: not applicable, < 0: error
int32_t thin_pw(const PwArgs& a, hipStream_t st) {
    if (a.HW % 4 || !pwx_src_ok(a.src, a.HW) || !sinks_aligned16(a.out))
        return 0;
    ThinPwArgs b{};
    b.src = a.src; b.out = a.out; b.w = a.w; b.rs = a.rs; b.cs = a.cs; b.HW = a.HW;
    b.Q = a.P / 4;
    const dim3 grid((unsigned)((b.Q + 64 * kThinWaves - 1) / (64 * kThinWaves)));
    bool pre = false;
    for (int s = 0; s < a.out.nsink; ++s)
        pre |= a.out.s[s].mode == ISG_SINK_ACTBWD || a.out.s[s].mode == ISG_SINK_ACCUM;
#define ISG_THIN_PW(KK, MM)                                                                      \
    if (a.K == KK && a.M == MM) {                                                                 \
        if (pre) hipLaunchKernelGGL((thin_pw_kernel<KK, MM, true>), grid, dim3(64 * kThinWaves), 0, st, b); \
        else hipLaunchKernelGGL((thin_pw_kernel<KK, MM, false>), grid, dim3(64 * kThinWaves), 0, st, b); \
        const int32_t e = isg_check_launch("thin_pw_kernel");                                    \
        return e ? e : 1;                                                                        \
    }
    ISG_THIN_PW(4, 16)
    ISG_THIN_PW(16, 4)
    ISG_THIN_PW(4, 4)
    ISG_THIN_PW(8, 8)
    ISG_THIN_PW(16, 16)
#undef ISG_THIN_PW
    return 0;
}
}  // namespace

ISG_STAMP_ACCESSOR(isg_dbg_stamps_pw)

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
    // a folded residual tail (isg.h: BN_FWD segment with y / vtensor.mat in the forward,
    // ACTBWD sink's residual form in the input gradient) runs on the slab kernel only
    const bool rbn_src = src->rbn.stats || src->rbn.coef;
    bool res_in = src->mat != nullptr || rbn_src, res_out = false;
    for (int s = 0; s < src->nseg; ++s) res_in |= src->s[s].xform == ISG_XF_BN_FWD && src->s[s].y;
    for (int s = 0; s < out->nsink; ++s) {
        const isg_sink& k = out->s[s];
        res_out |= k.r || k.old || k.p2 || k.rbn.stats || k.rbn.coef;
    }
    const bool res = res_in || res_out;
    // forward: one source segment (the residual's own BatchNorm: also one sink), any sinks;
    // input gradient: one residual sink, any gradient segments (a stacked pair's two)
    if (res && ((res_in && dgrad) || (res_in && src->nseg != 1) ||
                (res_in && rbn_src && !(src->s[0].xform == ISG_XF_BN_FWD && src->s[0].y && out->nsink == 1)) ||
                (res_out && (!dgrad || out->nsink != 1 || out->s[0].mode != ISG_SINK_ACTBWD || !out->s[0].r))))
        return isg_set_error(ISG_ERR_UNSUPPORTED, "pw gemm: residual forms need one segment in the forward "
                             "(input residual), one ACTBWD residual sink in the input gradient");
    if (!res) {  // thin layers (K, M <= 16) on the VALU
        const int32_t t = thin_pw(a, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    int wmode = 0;
    if (aligned16(w)) {
        if (!dgrad && a.K % 4 == 0) wmode = 1;
        if (dgrad && a.M % 4 == 0) wmode = 2;
    }
    // measured (per-op tables, kbench): the slab kernel wins on the wide 256^2 forward
    // layers and on input gradients with few rows (M = Ci <= 64, K <= 128: the 48 -> 128
    // expansions' dgrads 17.1 -> 14.9 us, >= 512 workgroups); elsewhere its longer
    // per-workgroup phase chain loses to the chunked kernel (the 128 -> 48 dgrads
    // 12.2 -> 17.0 us, the 256 -> 128 resconv forward 27.6 -> 49.5 us)
    // (r02g per-op tables: the 64^2 128 -> 48 forwards 13.8 -> 12.5 us on the slab)
    // (round 3, after the single-segment prologue: the 48 -> 128 expansions and their
    // transposes, M = 128 rows over K = 48, on 32 x 64 tiles — kbench fwd 15.3 -> 14.8 us,
    // dgrad 18.4 -> 17.2 us against the chunked kernel)
    // (round 6, measured: the slab for K = 256 — bottle3_1's stacked 256 -> 176 pair at
    // 32 x 32 tiles — step 3.654 -> 3.680 ms, 3.573 -> 3.595 eager: kept on the chunked kernel)
    const bool slab_pays = res || (!dgrad && a.P >= 65536) || (dgrad && a.M <= 64 && a.K <= 128) ||
                           (!dgrad && a.M <= 64 && a.K <= 128) || (a.M <= 128 && a.K <= 64);
    if (slab_pays && wmode && pwx_src_ok(*src, a.HW) && a.P < ((int64_t)1 << 31)) {
        PwxArgs b{};
        b.src = a.src; b.out = a.out; b.w = w; b.rs = a.rs; b.cs = a.cs;
        b.HW = a.HW; b.M = a.M; b.K = a.K; b.Kp = (a.K + 15) / 16 * 16; b.P = a.P;
        b.wmode = wmode;
        b.fast = host_vt_fast(*src) && host_sinks_fast(*out);
        b.pre_on = 0;
        b.res_on = res_out ? 1 : 0;
        auto bn_on = [](const isg_bn& q) { return q.stats != nullptr || q.coef != nullptr; };
        b.rbn_in = res_in && bn_on(src->rbn) ? 1 : 0;
        b.rbn_out = res_out && bn_on(out->s[0].rbn) ? 1 : 0;
        for (int s = 0; s < out->nsink; ++s)
            if (out->s[s].mode == ISG_SINK_ACTBWD || out->s[s].mode == ISG_SINK_ACCUM) b.pre_on = 1;
        b.stat_on = 0;
        for (int s = 0; s < src->nseg; ++s) {
            const isg_vseg& g = src->s[s];
            if ((g.xform == ISG_XF_BN_FWD || g.xform == ISG_XF_BN_BWD) && !g.bn.coef && g.bn.stats) b.stat_on = 1;
        }
        for (int s = 0; s < out->nsink; ++s) {
            const isg_sink& k = out->s[s];
            if (k.mode == ISG_SINK_ACTBWD && !k.bn.coef && k.bn.stats) b.stat_on = 1;
        }
        // HY also selects the 4-group statistics loads (coef_issue<4>): a BN_BWD segment
        // finalised by the consumer needs them even when its y is its own input (ADVICE r03:
        // the 2-group form would apply identity coefficients there)
        // HY also loads a BN_FWD segment's residual term (isg_vseg residual form)
        bool hy = false;
        for (int s = 0; s < src->nseg; ++s) {
            if (src->s[s].xform == ISG_XF_BN_BWD &&
                ((src->s[s].y && src->s[s].y != src->s[s].p) || (!src->s[s].bn.coef && src->s[s].bn.stats)))
                hy = true;
            if (src->s[s].xform == ISG_XF_BN_FWD && src->s[s].y) hy = true;
        }
        // (BM, BP): rows first (fewer row blocks = fewer slab re-reads), then pixels; the
        // first configuration that fits the LDS and the per-lane load budget (8 weight and
        // 8 activation loads of 16 B), keeps >= 4 MFMA tiles per workgroup and gives >= 256
        // workgroups (one per CU), else the one with the most workgroups
        const int R = (a.M + 15) / 16;
        int best_bp = 0, best_bm = 0, best_lds = 0;
        int64_t best_blocks = -1;
        bool done = false;
        // more than 64 rows: the widest pixel tile first (fewer weight re-reads per pixel,
        // kbench (32, 64) beat (128, 16) on M = 128), else the most rows first
        const bool bp_first = a.M > 64;
        for (int it = 0; it < 8 * 3 && !done; ++it) {
            const int bm = bp_first ? std::min(R, 8) * 16 - 16 * (it % 8) : std::min(R, 8) * 16 - 16 * (it / 3);
            const int bp = bp_first ? (64 >> (it / 8)) : (64 >> (it % 3));
            if (bm < 16) continue;
            {
                const int wq = pwx_wrow_quads(wmode, bm, b.Kp) * (wmode == 1 ? bm : b.Kp);
                // (measured: 3-tile configurations when one row block covers M — the 64^2
                // 128 <-> 48 layers on 48 x 16 tiles instead of 32 x 32 — 12.6 -> 13.3 us
                // forward, 13.6 -> 15.8 us input gradient, step +0.05-0.09 ms)
                if ((bm / 16) * (bp / 16) < 4 || wq > 8 * kThreads) continue;
                if (b.Kp > 8 * (kThreads / (bp / 4))) continue;
                int o0, o1, o2, o3, as, xs;
                const int lds = pwx_lds(a.K, b.Kp, bm, bp, o0, o1, o2, o3, as, xs);
                if (lds > kPxMaxLds) continue;
                const int64_t blocks = ((a.P + bp - 1) / bp) * ((a.M + bm - 1) / bm);
                if (blocks > best_blocks) {
                    best_bp = bp; best_bm = bm; best_lds = lds; best_blocks = blocks;
                }
                if (blocks >= kPwxMinBlocks) { done = true; break; }
            }
        }
        if (best_bp) {
            b.BM = best_bm;
            const int wqp = pwx_wrow_quads(wmode, best_bm, b.Kp);
            b.wu = (wqp * (wmode == 1 ? best_bm : b.Kp) + kThreads - 1) / kThreads;
            b.wsh = 0;
            while ((1 << b.wsh) < wqp) ++b.wsh;
            b.xu = (b.Kp + kThreads / (best_bp / 4) - 1) / (kThreads / (best_bp / 4));
            pwx_lds(a.K, b.Kp, best_bm, best_bp, b.off_k, b.off_ri, b.off_a, b.off_x, b.AS, b.XS);
            const int tpw = ((best_bm / 16) * (best_bp / 16) + 3) / 4;
            const dim3 grid((unsigned)((a.P + best_bp - 1) / best_bp), (unsigned)((a.M + best_bm - 1) / best_bm));
            int32_t rc;
            const bool seg1 = src->nseg == 1 && out->nsink == 1;
            static const bool log = getenv("ISG_PWX_LOG") != nullptr;  // diagnostics: the chosen tiling
            if (log)
                fprintf(stderr, "pwx %s M %d K %d P %lld BM %d BP %d TPW %d HY %d SEG1 %d RES %d blocks %lld\n",
                        dgrad ? "dgrad" : "fwd", a.M, a.K, (long long)a.P, best_bm, best_bp, tpw, (int)hy,
                        (int)seg1, b.res_on, (long long)best_blocks);
            if (best_bp == 64) rc = hy ? pwx_dispatch_seg<64, true>(b, grid, best_lds, tpw, seg1, st)
                                       : pwx_dispatch_seg<64, false>(b, grid, best_lds, tpw, seg1, st);
            else if (best_bp == 32) rc = hy ? pwx_dispatch_seg<32, true>(b, grid, best_lds, tpw, seg1, st)
                                            : pwx_dispatch_seg<32, false>(b, grid, best_lds, tpw, seg1, st);
            else rc = hy ? pwx_dispatch_seg<16, true>(b, grid, best_lds, tpw, seg1, st)
                         : pwx_dispatch_seg<16, false>(b, grid, best_lds, tpw, seg1, st);
            return rc;
        }
    }
    if (res)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "pw gemm: residual form off the slab kernel "
                             "(16-B aligned rows and weights, HW %% 4 == 0)");
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
    return isg_check_launch("pw_kernel");
}
