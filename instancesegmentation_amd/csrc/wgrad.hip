// Weight gradient of dense convolutions (gfx950): every nn.Conv2d weight of the
// reference (segment.py) and — with the operand roles swapped — the ConvTranspose2d
// weights (segment.py:305, :435).
//
//   dW[row][col] += sum_p dy[row][p] * x[ci][p*S - P + (kh,kw)*D],  col = ci*KH*KW + kh*KW + kw
//
// A GEMM with the output pixels as the reduction (K) dimension. A workgroup owns a block
// of up to 64 rows x 128 columns of dW and a contiguous range of 64-pixel tiles
// (TR x TC output pixels, TC in {8,16,32,64}). Per tile it stages into LDS
//   * the dy rows (BatchNorm-backward rebuilt on load): wave w loads rows w, w+4, ...,
//     lane = pixel;
//   * the INPUT HALO of the tile for the block's input channels (producer BatchNorm +
//     activation applied on load): slot s = (channel, halo row) is wave-uniform, lane =
//     halo column (HC <= 64),
// so every channel quantity is scalar (stage.h) and each element costs one address add,
// one load and one fused transform. Every (kh,kw) tap reads the halo at a shifted offset
// (no im2col gather). The loads of tile t+1 are issued into registers before the MFMAs
// of tile t (register double buffer).
// MFMA v_mfma_f32_16x16x4_f32: A[i=row][k=pixel] from LDS dy, B[k=pixel][j=col] from the
// halo. Each wave keeps up to 4 16x16 accumulator tiles; blocks with fewer than 4 tiles
// split the 64 pixels of a tile across waves. A single-row dW (the 4->1 mask-head conv,
// segment.py:437) runs on the VALU instead: an MFMA there would be 15/16 padding.
// Partial sums leave the block with one f32 atomic per dW element, into one of the
// ISG_WREP replicas (include/isg.h).
#include <cstdlib>

#include "stage.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTP = 64;             // pixels per tile
constexpr int kAStride = kTP + 2;   // conflict-free A-fragment reads
constexpr int kRowsBlk = 64;        // dW rows per block (BMT <= 4)
constexpr int kColsBlk = 512;       // dW columns per block (BMT*BNT <= 32 tiles)
constexpr int kMaxXCh = 64;         // halo channels per block
constexpr int kXs = 9216;           // halo floats per block (36 KB) incl. channel padding

struct WgArgs {
    isg_vtensor dy;  // rows: N x R x OH x OW
    isg_vtensor x;   // gathered: N x Ci x H x W
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int nrep;
    int N, OH, OW, H, W, R, Ci, KH, KW, SH, SW, PH, PW, DH, DW;
    int BMT, BNT, ncb;          // 16-row / 16-col tiles per block, column blocks
    int HR, HC, hsp;            // halo rows, cols, LDS channel stride
    int lgTC;                   // log2 tile width (tile = (64>>lgTC) x (1<<lgTC))
    int tiles_x, tiles_y;
    int64_t ntiles, tiles_per_block;
    int valu;                   // R == 1 path
    int dbg;                    // ablation bits (stamp build only, tools/kbench)
};
#ifdef ISG_STAMPS
#define DBG(a, b) ((a).dbg & (b))
#else
#define DBG(a, b) 0
#endif

struct TileCtx {
    int per_img, TR, TC, apy, apx, lane, wave, Rb, nslots;
    const ChT* tA;  // LDS: dy rows of the block
    const ChT* tX;  // LDS: x channels of the block
};

ISG_DEV void tile_origin(const WgArgs& a, const TileCtx& t, int64_t tl, int& n, int& oy0,
                         int& ox0) {
    n = (int)(tl / t.per_img);
    const int r = (int)(tl - (int64_t)n * t.per_img);
    const int ty = r / a.tiles_x;
    oy0 = ty * t.TR;
    ox0 = (r - ty * a.tiles_x) * t.TC;
}

// Direct staging, groups of U slots with all their loads in flight together. The loop
// bodies stay small on purpose: fully unrolled register-prefetch variants of this kernel
// grew past 60-130 KB of code and ran 2-3x slower (instruction fetch, one wave per SIMD).
template <int U>
ISG_DEV void wg_stage(const WgArgs& a, const TileCtx& t, int64_t tl, int nrow_w, float* As,
                      float* Xs) {
    int n, oy0, ox0;
    tile_origin(a, t, tl, n, oy0, ox0);
    const int oy = oy0 + t.apy, ox = ox0 + t.apx;
    const bool pv = oy < a.OH && ox < a.OW;
    const int pix = pv ? oy * a.OW + ox : 0;
    for (int j0 = 0; j0 < nrow_w; j0 += U) {
        float v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = min(t.wave + 4 * (j0 + u), t.Rb - 1);
            const ChT c = t.tA[row];
            v[u] = gld(c.p, n * c.ns + pix);
            w[u] = gld(c.y, n * c.yns + pix);  // == p unless BatchNorm-backward
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = t.wave + 4 * (j0 + u);
            if (row < t.Rb) {
                const ChT c = t.tA[row];
                As[row * kAStride + t.lane] = pv ? ch_xform(c.xf, c.act, c.k, v[u], w[u]) : 0.f;
            }
        }
    }
    const int iy0 = oy0 * a.SH - a.PH, ix = ox0 * a.SW - a.PW + t.lane;
    const bool colok = t.lane < a.HC && ix >= 0 && ix < a.W;
    for (int s0 = t.wave; s0 < t.nslots; s0 += 4 * U) {
        float v[U], w[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int slot = min(s0 + 4 * u, t.nslots - 1);
            const int cl = slot / a.HR, iy = iy0 + slot - cl * a.HR;
            const ChT c = t.tX[cl];
            ok[u] = colok && iy >= 0 && iy < a.H;
            const int o = ok[u] ? iy * a.W + ix : 0;
            v[u] = gld(c.p, n * c.ns + o);
            w[u] = gld(c.y, n * c.yns + o);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int slot = s0 + 4 * u;
            if (slot < t.nslots) {
                const int cl = slot / a.HR, hr = slot - cl * a.HR;
                const ChT c = t.tX[cl];
                if (t.lane < a.HC)
                    Xs[cl * a.hsp + hr * a.HC + t.lane] = ok[u] ? ch_xform(c.xf, c.act, c.k, v[u], w[u]) : 0.f;
            }
        }
    }
}

// BMT: 16-row tiles of dW per block (A row slots per wave = 4*BMT); AB / XB: the dy / x
// operand has BatchNorm-backward channels (second load of the saved forward output).
template <int TPW>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(WgArgs a) {
    // TPW: accumulator tiles per wave = ceil(BMT*BNT / 4)
    // dynamic LDS sized per launch (occupancy): A tile [BMT*16][kAStride], then the halo
    extern __shared__ float smem[];
    float* const As = smem;
    float* const Xs = smem + a.BMT * 16 * kAStride;
    __shared__ ChT tA[kRowsBlk];
    __shared__ ChT tX[kMaxXCh];

    STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = wave_id();
    const int kk = lane >> 4, pl = lane & 15;
    const int KK = a.KH * a.KW;
    const int NCOL = a.Ci * KK;
    const int rb = blockIdx.y / a.ncb, cb = blockIdx.y - rb * a.ncb;
    const int r_lo = rb * kRowsBlk;
    const int Rb = min(kRowsBlk, a.R - r_lo);
    const int c_lo = cb * a.BNT * 16;
    const int c_hi = min(NCOL, c_lo + a.BNT * 16);
    const int ci_lo = c_lo / KK;
    const int nci = (c_hi - 1) / KK + 1 - ci_lo;
    const int nslots = nci * a.HR;
    const int TC = 1 << a.lgTC, TR = kTP >> a.lgTC;
    const int ohw = a.OH * a.OW, xhw = a.H * a.W;
    // this workgroup's replica of dW / dbias (include/isg.h ISG_WREP)
    const int64_t rep_off = (int64_t)((blockIdx.x + 7u * blockIdx.y) % (unsigned)a.nrep) * a.rep_stride;
    double* const dwr = a.dw + rep_off;

    for (int i = tid; i < Rb; i += kThreads) tA[i] = ch_table_entry(a.dy, r_lo + i, ohw);
    for (int i = tid; i < nci; i += kThreads) tX[i] = ch_table_entry(a.x, ci_lo + i, xhw);
    // rows Rb .. 16*BMT of the A tile stay zero (never restaged)
    for (int i = Rb * kAStride + tid; i < a.BMT * 16 * kAStride; i += kThreads) As[i] = 0.f;

    // ---- MFMA operand offsets --------------------------------------------------------
    const int nt = a.BMT * a.BNT;
    const bool ksplit = nt < 4;
    const int ks = ksplit ? 4 / nt : 1;
    const int kpart = ksplit ? wave / nt : 0;
    const bool kactive = !ksplit || kpart < ks;
    const int kq_lo = kpart * (kTP / ks), kq_hi = kq_lo + kTP / ks;
    // tv[i]: wave-uniform presence of accumulator tile i; columns past c_hi read any
    // staged value (their D columns are never stored), so no per-lane guards in the loop
    bool tv[TPW];
    int arow[TPW], xoff[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = ksplit ? (i == 0 && kactive ? wave % nt : 1 << 20) : wave + 4 * i;
        const int rt = t / a.BNT, ct = t - rt * a.BNT;
        tv[i] = t < nt;
        arow[i] = tv[i] ? (rt * 16 + pl) * kAStride : 0;
        const int col = min(c_lo + ct * 16 + pl, c_hi - 1);
        const int ci = col / KK, tap = col - ci * KK;
        const int kh = tap / a.KW, kw = tap - kh * a.KW;
        xoff[i] = tv[i] ? (ci - ci_lo) * a.hsp + kh * a.DH * a.HC + kw * a.DW : 0;
    }
    // halo offset of pixel 4*s + kk of the tile, per k-step s
    int poffs[kTP / 4];
#pragma unroll
    for (int s = 0; s < kTP / 4; ++s) {
        const int p = 4 * s + kk;
        poffs[s] = (p >> a.lgTC) * a.SH * a.HC + (p & (TC - 1)) * a.SW;
    }
    const int s_lo = kq_lo / 4, s_hi = kq_hi / 4;
    f32x4 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float vacc = 0.f;  // VALU path (R == 1): column lane, pixel quarter wave
    int vxoff = -1;
    if (a.valu) {
        const int col = c_lo + lane;
        if (col < c_hi) {
            const int ci = col / KK, tap = col - ci * KK;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            vxoff = (ci - ci_lo) * a.hsp + kh * a.DH * a.HC + kw * a.DW;
        }
    }
    float bsum = 0.f;
    const bool do_bias = a.dbias && cb == 0;
    __syncthreads();
    STAMP(1);

    const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_block;
    const int64_t t1 = min(t0 + a.tiles_per_block, a.ntiles);
    const int per_img = a.tiles_x * a.tiles_y;
    const int apy = lane >> a.lgTC, apx = lane & (TC - 1);

    const TileCtx tc{per_img, TR, TC, apy, apx, lane, wave, Rb, nslots, tA, tX};
    const int nrow_w = (Rb - wave + 3) / 4;  // this wave's dy rows
    for (int64_t tl = t0; tl < t1; ++tl) {
        __syncthreads();  // previous tile's LDS reads are done
        wg_stage<8>(a, tc, tl, nrow_w, As, Xs);
        __syncthreads();
        if (tl == t0) STAMP(2);
        if (do_bias && tid < Rb) {
            const float* rowp = As + tid * kAStride;
            float s = 0.f;
#pragma unroll 16
            for (int p = 0; p < kTP; ++p) s += rowp[p];
            bsum += s;
        }
        if (a.valu) {
            if (vxoff >= 0) {
                const int q0 = wave * 16;
#pragma unroll
                for (int p = q0; p < q0 + 16; ++p) {
                    const int poff = (p >> a.lgTC) * a.SH * a.HC + (p & (TC - 1)) * a.SW;
                    vacc = fmaf(As[p], Xs[vxoff + poff], vacc);
                }
            }
            continue;
        }
        if (!kactive || DBG(a, 4)) continue;
        if (!ksplit) {
            // every wave owns TPW tiles (absent ones compute on row 0 and are never
            // stored): branch-free, so the LDS reads batch ahead of the MFMAs
#pragma unroll
            for (int s = 0; s < kTP / 4; ++s)
#pragma unroll
                for (int i = 0; i < TPW; ++i) {
                    const float av = As[arow[i] + 4 * s + kk];
                    const float bv = Xs[xoff[i] + poffs[s]];
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i], 0, 0, 0);
                }
        } else {
            for (int s = s_lo; s < s_hi; ++s) {
                const float av = As[arow[0] + 4 * s + kk];
                const int p = 4 * s + kk;
                const float bv = Xs[xoff[0] + (p >> a.lgTC) * a.SH * a.HC + (p & (TC - 1)) * a.SW];
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[0], 0, 0, 0);
            }
        }
    }
    __syncthreads();
    STAMP(3);
    if (a.valu) {
        float* part = Xs;
        part[tid] = vacc;
        __syncthreads();
        if (tid < 64) {
            const float s = part[tid] + part[tid + 64] + part[tid + 128] + part[tid + 192];
            const int col = c_lo + tid;
            if (col < c_hi && Rb > 0) atomicAdd(&dwr[(int64_t)r_lo * NCOL + col], s);
        }
    } else {
        // k-split: waves kpart>0 hand their partial tile to wave (wave % nt) via LDS
        if (ksplit) {
            float* part = Xs;
            if (kactive && kpart > 0)
#pragma unroll
                for (int r = 0; r < 4; ++r) part[((wave - nt) * 4 + r) * 64 + lane] = acc[0][r];
            __syncthreads();
            if (kactive && kpart == 0)
                for (int j = 1; j < ks; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[0][r] += part[((wave + (j - 1) * nt) * 4 + r) * 64 + lane];
        }
        // lane holds D[row = rt*16 + kk*4 + r][col = c_lo + ct*16 + pl]
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int t = ksplit ? (i == 0 && kactive && kpart == 0 ? wave : 1 << 20) : wave + 4 * i;
            if (t >= nt) continue;
            const int rt = t / a.BNT, ct = t - rt * a.BNT;
            const int col = c_lo + ct * 16 + pl;
            if (col >= c_hi) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = rt * 16 + kk * 4 + r;
                if (row < Rb) atomicAdd(&dwr[(int64_t)(r_lo + row) * NCOL + col], acc[i][r]);
            }
        }
    }
    if (do_bias && tid < Rb) atomicAdd(&a.dbias[rep_off + r_lo + tid], bsum);
    STAMP(4);
}

// ---- 1x1 stride-1 weight gradient on pixel slabs (pwg) ----------------------------------
// dW[r][c] = sum_p dy[r][p] * x[c][p]. A workgroup owns BR rows x BC columns of dW and a
// contiguous range of 64-pixel tiles. Per tile, ALL its loads are issued together, with no
// branch around any of them (stage.h): lane = 4 consecutive pixels of one channel row
// (16-B loads), 16 channel rows per pass, the dy rows (BatchNorm backward rebuilt on load)
// and the x rows (producer BatchNorm + activation) in one slab; passes past the last row
// repeat it (L1 hits). The next tile's loads are issued before this tile's MFMAs. Both
// MFMA operands are read 4 k-steps (pixels) at a time with ds_read_b128 (step j of pixel
// group g gives lane slot kk pixel 16g + 4kk + j); row stride 72 floats = 8 mod 64.
constexpr int kGTP = 64;            // pixels per tile
constexpr int kGS = kGTP + 8;       // LDS row stride (floats)
constexpr int kGMaxRows = 192;      // BR + BC

struct PwgArgs {
    isg_vtensor dy, x;
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int nrep;
    int HW, R, C, BR, BC, ncb;
    int fast;   // finalised BatchNorm coefficients everywhere (stage.h vt_fast)
    int stat_on;  // some channel evaluates its BatchNorm statistics (consumer-side)
    int off_k, off_x;  // byte offsets: coefficient table, slab (addressing table at 0)
    int64_t P, ntiles, tiles_per_block;
};

template <int NU, bool HY>
ISG_DEV void pwg_issue(const PwgArgs& a, const ChSrc* tabA, int NR, int q, int cr, int64_t tl,
                       f32x4* v, f32x4* yv, bool& pv) {
    const int64_t pg = tl * kGTP + 4 * q;
    pv = pg < a.P;
    const int n = pv ? (int)(pg / a.HW) : 0;
    const int pix = pv ? (int)(pg - (int64_t)n * a.HW) : 0;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const ChSrc t = tabA[min(cr + 16 * u, NR - 1)];
        v[u] = gld4(t.p, (int64_t)n * t.ns + pix);
        if (HY) yv[u] = gld4(t.y, (int64_t)n * t.yns + pix);
    }
}

extern __shared__ f32x4 pwg_smem[];

// the kernel body over block (bx, by) of problem a: pwg_kernel runs one problem on its own
// 2-D grid, pwg_group_kernel several problems of one instantiation on one flat grid
template <int TPW, int NU, bool HY>
ISG_DEV void pwg_body(const PwgArgs& a, const unsigned bx, const unsigned by) {
    char* const smem = reinterpret_cast<char*>(pwg_smem);
    ChSrc* const tabA = reinterpret_cast<ChSrc*>(smem);  // kThreads entries: BR dy rows, BC x rows
    ChanCoef* const tabK = reinterpret_cast<ChanCoef*>(smem + a.off_k);
    // per row: (negative-side slope, 1 if BatchNorm backward) — the staging transform runs
    // branch-free (rows of one wave can differ in transform kind and activation)
    float2* const tabN = reinterpret_cast<float2*>(smem + a.off_k + kGMaxRows * (int)sizeof(ChanCoef));
    float* const S = reinterpret_cast<float*>(smem + a.off_x);  // [BR + BC][kGS]

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = wave_id();
    const int kk = lane >> 4, pl = lane & 15;
    const int rb = by / a.ncb, cb = by - rb * a.ncb;
    const int r0 = rb * a.BR, c0 = cb * a.BC;
    const int Rb = min(a.BR, a.R - r0), Cb = min(a.BC, a.C - c0);
    const int BR = a.BR, NR = a.BR + a.BC;
    const int64_t rep_off = (int64_t)((bx + 7u * by) % (unsigned)a.nrep) * a.rep_stride;
    double* const dwr = a.dw + rep_off;
    STAMP(0);

    // ---- tables: row j < BR is dy channel r0 + j, else x channel c0 + j - BR -------------
    const int jr = min(tid, NR - 1);
    const bool is_dy = jr < BR;
    const int cdy = r0 + min(jr, Rb - 1), cx = c0 + min(max(jr - BR, 0), Cb - 1);
    {
        const VtSel vd = vt_sel(a.dy), vx = vt_sel(a.x);
        const ChSrc ad = ch_addr(vd, cdy, a.HW), ax = ch_addr(vx, cx, a.HW);
        const CoefLoad<4> ld = coef_issue<4>(vd, cdy, a.stat_on != 0);
        const CoefLoad<2> lx = coef_issue<2>(vx, cx, a.stat_on != 0);
        ChSrc& e = tabA[tid];  // field by field: a select of whole records goes through scratch
        e.p = is_dy ? ad.p : ax.p; e.y = is_dy ? ad.y : ax.y;
        e.ns = is_dy ? ad.ns : ax.ns; e.yns = is_dy ? ad.yns : ax.yns;
        e.xf = is_dy ? ad.xf : ax.xf; e.act = is_dy ? ad.act : ax.act;
        ChanCoef kk;
        if (a.fast) {
            const ChanCoef kd = coef_finish(vd, cdy, ld), kx = coef_finish(vx, cx, lx);
            kk = ChanCoef{is_dy ? kd.c0 : kx.c0, is_dy ? kd.c1 : kx.c1, is_dy ? kd.c2 : kx.c2,
                          is_dy ? kd.c3 : kx.c3};
        } else {
            kk = tid < NR ? (is_dy ? vt_coef(a.dy, cdy) : vt_coef(a.x, cx)) : ChanCoef{0.f, 1.f, 0.f, 0.f};
        }
        if (tid < NR) {
            const int xf = e.xf, act = e.act;
            if (xf == ISG_XF_PLAIN) kk = ChanCoef{0.f, 1.f, 0.f, 0.f};
            tabK[tid] = kk;
            const float neg = (xf != ISG_XF_BN_FWD || act == ISG_ACT_NONE) ? 1.f
                              : act == ISG_ACT_RELU ? 0.f : kk.c3;
            tabN[tid] = float2{neg, xf == ISG_XF_BN_BWD ? 1.f : 0.f};
        }
    }
    __syncthreads();
    STAMP(1);

    const int CTn = a.BC / 16;
    const int nt = (BR / 16) * CTn;
    int aoff[TPW], boff[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = min(wave + 4 * i, nt - 1);  // surplus tiles recompute the last one
        aoff[i] = ((t / CTn) * 16 + pl) * kGS + 4 * kk;
        boff[i] = (BR + (t % CTn) * 16 + pl) * kGS + 4 * kk;
    }
    f32x4 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    const bool do_bias = a.dbias && cb == 0;

    const int q = tid & 15, cr = tid >> 4;
    const int64_t t0 = (int64_t)bx * a.tiles_per_block;
    const int64_t t1 = min(t0 + a.tiles_per_block, a.ntiles);
    f32x4 v[NU], yv[NU];
    bool pv;
    pwg_issue<NU, HY>(a, tabA, NR, q, cr, t0, v, yv, pv);
    for (int64_t tl = t0; tl < t1; ++tl) {
        __syncthreads();  // previous tile's fragment reads are done
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int j = cr + 16 * u;
            if (j < NR) {
                const bool live = pv && (j < BR ? j < Rb : j - BR < Cb);
                const ChanCoef k = tabK[j];
                const float2 nb = tabN[j];
                f32x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // ch_xform's three forms, evaluated unconditionally and selected
                    const float x = v[u][e], y = HY ? yv[u][e] : x;
                    float zf = (x - k.c0) * k.c1 + k.c2;
                    zf = zf > 0.f ? zf : zf * nb.x;
                    const float zb = k.c0 * x + k.c1 * (y - k.c2) + k.c3;
                    o[e] = live ? (nb.y != 0.f ? zb : zf) : 0.f;
                }
                *reinterpret_cast<f32x4*>(&S[j * kGS + 4 * q]) = o;
            }
        }
        __syncthreads();
        if (tl == t0) STAMP(2);
        // next tile's loads (a clamped repeat of the last tile past the range)
        pwg_issue<NU, HY>(a, tabA, NR, q, cr, min(tl + 1, t1 - 1), v, yv, pv);
        if (do_bias && tid < Rb) {
            const float* rowp = S + tid * kGS;
            float s = 0.f;
#pragma unroll 16
            for (int p = 0; p < kGTP; ++p) s += rowp[p];
            bsum += s;
        }
#pragma unroll
        for (int g = 0; g < kGTP; g += 16) {
            f32x4 a4[TPW], b4[TPW];
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                a4[i] = *reinterpret_cast<const f32x4*>(&S[aoff[i] + g]);
                b4[i] = *reinterpret_cast<const f32x4*>(&S[boff[i] + g]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < TPW; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[i][j], b4[i][j], acc[i], 0, 0, 0);
        }
    }
    STAMP(3);
    // lane holds D[row = rt*16 + kk*4 + r][col = ct*16 + pl]
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = wave + 4 * i;
        if (t >= nt) continue;
        const int rt = t / CTn, ct = t % CTn;
        const int col = ct * 16 + pl;
        if (col >= Cb) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = rt * 16 + kk * 4 + r;
            if (row < Rb) atomicAdd(&dwr[(int64_t)(r0 + row) * a.C + c0 + col], acc[i][r]);
        }
    }
    if (do_bias && tid < Rb) atomicAdd(&a.dbias[rep_off + r0 + tid], bsum);
    STAMP(4);
}

template <int TPW, int NU, bool HY>
__global__ __launch_bounds__(kThreads) void pwg_kernel(PwgArgs a) {
    pwg_body<TPW, NU, HY>(a, blockIdx.x, blockIdx.y);
}

// Up to kPwgGroup problems of one instantiation in one launch (the executor's side-stream
// batches, api.cpp): measured, every side-stream node costs the step ~3 us even when it
// does no work (a since-removed timing switch: 4.02 ms, 3.62 with the weight gradients as empty
// launches, 3.35 with no launches), so the 1x1 weight gradients of a batch go out grouped.
constexpr int kPwgGroup = 3;
struct PwgGroupMeta {
    int start[kPwgGroup + 1];  // flat block ranges
    int gx[kPwgGroup];
    int n;
};

// the records travel as separate kernel parameters (an array of them, indexed per branch,
// was merged by the compiler into one body reading a copied array from scratch)
template <int TPW, int NU, bool HY>
__global__ __launch_bounds__(kThreads) void pwg_group_kernel(PwgArgs p0, PwgArgs p1, PwgArgs p2,
                                                             PwgGroupMeta m) {
    const int b = blockIdx.x;
    if (m.n > 2 && b >= m.start[2]) {
        const int l = b - m.start[2];
        pwg_body<TPW, NU, HY>(p2, l % m.gx[2], l / m.gx[2]);
    } else if (m.n > 1 && b >= m.start[1]) {
        const int l = b - m.start[1];
        pwg_body<TPW, NU, HY>(p1, l % m.gx[1], l / m.gx[1]);
    } else {
        pwg_body<TPW, NU, HY>(p0, b % m.gx[0], b / m.gx[0]);
    }
}

bool g_aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

bool pwg_src_ok(const isg_vtensor& v, int HW) {
    if (HW % 4) return false;
    for (int s = 0; s < v.nseg; ++s) {
        const isg_vseg& g = v.s[s];
        if (!g_aligned16(g.p) || g.n_stride % 4) return false;
        if (g.xform == ISG_XF_BN_BWD && g.y && (!g_aligned16(g.y) || g.y_n_stride % 4)) return false;
    }
    return true;
}

bool pwg_has_y(const isg_vtensor& v) {
    for (int s = 0; s < v.nseg; ++s)
        if (v.s[s].xform == ISG_XF_BN_BWD && v.s[s].y && v.s[s].y != v.s[s].p) return true;
    return false;
}

bool pwg_fast(const isg_vtensor& v) {
    for (int s = 0; s < v.nseg; ++s) {
        const isg_vseg& g = v.s[s];
        // stage.h seg_fast: finalised coefficients or training-mode statistics
        if ((g.xform == ISG_XF_BN_FWD || g.xform == ISG_XF_BN_BWD) && !(g.bn.coef || g.bn.train))
            return false;
    }
    return true;
}

template <int TPW, int NU, bool HY>
int32_t pwg_launch(const PwgArgs& a, dim3 grid, size_t lds, hipStream_t st) {
    auto k = pwg_kernel<TPW, NU, HY>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) != hipSuccess)
            return isg_check_launch("pwg_kernel: dynamic LDS");
        attr = true;
    }
    hipLaunchKernelGGL(k, grid, dim3(kThreads), lds, st, a);
    return isg_check_launch("pwg_kernel");
}


// ---- 1x1 weight gradient of the small maps, K split over the waves (pwk) ----------------
// At 64^2 / 128^2 (bs2: 8K-32K pixels against a dW of a few thousand elements) pwg_kernel
// spent three quarters of its time in latency (kbench stamps, 48 -> 128 at 64^2: 3.1 us
// table / coefficient setup, 3.0 us first tile load, 1.5 us MFMA, 3.2 us atomics). Here a
// workgroup owns a BR x BC block of dW (BR + BC <= 64 rows: RT x CT tiles of 16 x 16) and
// super-tiles of 256 pixels. The loads of a super-tile need only kernel arguments for their
// addresses (row j = wave + 4u is wave-uniform, one 1-KB run per wave and pass), so they
// are issued BEFORE the BatchNorm coefficients are evaluated and setup shares their round
// trip. Wave w multiplies pixels [64w, 64w + 64) for ALL the block's tiles (K split over
// the waves); the four partials meet in LDS, then one atomic per dW element: 4x the pixels
// per workgroup of pwg's 64-pixel tile at the same grid size — a quarter of its atomics.
constexpr int kKTP = 256;            // pixels per super-tile
constexpr int kKS = kKTP + 8;        // LDS row stride (8 mod 64, as pwg)
constexpr int kKMaxRows = 64;        // BR + BC

struct PwkArgs {
    isg_vtensor dy, x;
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int nrep;
    int HW, R, C, ncb;
    int fast, stat_on;  // fast: always 1 here (pwk_try)
    int64_t P, ntiles, tiles_per_block;
};

// A row's staging coefficients when the lane's row may come from either tensor (pwk: the
// dy rows and the x rows of one wave): the fields are picked per lane FIRST, then ONE set
// of loads (coef_issue / coef_finish over a picked segment). Two coef_issue calls, one per
// tensor, let the compiler finish the first tensor's statistics before issuing the second's
// loads — a second memory round trip in the kernel's prologue.
ISG_DEV ChanCoef pwk_row_coef(const VtSel& vd, int cdy, const VtSel& vx, int cx, bool is_dy,
                              bool stat_on) {
    int cld, clx;
    const int sd = vt_seg(vd, cdy, cld), sx = vt_seg(vx, cx, clx);
#define PWK_PICK(f) (is_dy ? ISG_SEL3(sd, f, vd) : ISG_SEL3(sx, f, vx))
    const float* coef = PWK_PICK(coef);
    const float* slope = PWK_PICK(slope);
    const float* p = PWK_PICK(p);
    const int xf = PWK_PICK(xf), bnC = PWK_PICK(bnC);
    const double* stats = PWK_PICK(stats);
    const float* gamma = PWK_PICK(gamma);
    const float* beta = PWK_PICK(beta);
    const float count = PWK_PICK(count), eps = PWK_PICK(eps);
#undef PWK_PICK
    const int cl = is_dy ? cld : clx;
    const int idx = xf == ISG_XF_BN_BWD ? bnC + cl : cl;
    const float* cp = coef ? coef + 4 * (int64_t)idx : p;
    const float* sp = slope ? slope + cl : p;
    const bool bn = xf == ISG_XF_BN_FWD || xf == ISG_XF_BN_BWD;
    const f32x4 f = f32x4{gld(cp, 0), gld(cp, 1), gld(cp, 2), gld(cp, 3)};
    const float sl = gld(sp, 0);
    const StatLoad<4> st = stat_issue<4>(bn && !coef ? stats : nullptr, gamma, beta, bnC, cl, p, stat_on);
    ChanCoef k = {0.f, 1.f, 0.f, 0.f};
    if (xf == ISG_XF_BN_FWD) {
        if (coef) {
            k.c0 = f[0]; k.c1 = f[1]; k.c2 = f[2];
        } else if (stats) {
            double mean, rstd;
            mean_rstd_of(stat_sum(st, 0), stat_sum(st, 1), count, eps, mean, rstd);
            k = fwd_coef_of(mean, rstd, st.gamma, st.beta, 0.f);
        }
        k.c3 = slope ? sl : 0.f;
    } else if (xf == ISG_XF_BN_BWD) {
        if (coef) {
            k = ChanCoef{f[0], f[1], f[2], f[3]};
        } else {
            double mean, rstd;
            mean_rstd_of(stat_sum(st, 0), stat_sum(st, 1), count, eps, mean, rstd);
            k = bwd_coef_of(mean, rstd, st.gamma, stat_sum(st, 2), stat_sum(st, 3), count);
        }
    }
    return k;
}

template <int RT, int CT, bool HY>
__global__ __launch_bounds__(kThreads) void pwk_kernel(PwkArgs a) {
    constexpr int BR = 16 * RT, BC = 16 * CT, NR = BR + BC, NU = NR / 4, NUY = HY ? BR / 4 : 0;
    constexpr int NT = RT * CT;
    static_assert(NR <= kKMaxRows && NR % 4 == 0, "pwk block");
    __shared__ __attribute__((aligned(16))) float S[kKMaxRows * kKS];
    __shared__ ChanCoef tabK[kKMaxRows];
    __shared__ float2 tabN[kKMaxRows];
    __shared__ ChSrc tabA[kKMaxRows];
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kk = lane >> 4, pl = lane & 15;
    const int rb = blockIdx.y / a.ncb, cb = blockIdx.y - rb * a.ncb;
    const int r0 = rb * BR, c0 = cb * BC;
    const int Rb = min(BR, a.R - r0), Cb = min(BC, a.C - c0);
    STAMP(0);
    const int64_t rep_off = (int64_t)((blockIdx.x + 7u * blockIdx.y) % (unsigned)a.nrep) * a.rep_stride;
    const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_block;
    const int64_t t1 = min(t0 + a.tiles_per_block, a.ntiles);
    // ---- per-row tables, wave-local: wave w stages (and transforms) only the rows
    //      j = w + 4u, so lane u of wave w builds row j's entries and no workgroup barrier
    //      stands between the table and the first super-tile's loads
    const int ju = wave + 4 * lane;  // this lane's table row (lane < NU)
    const bool own = lane < NU;
    const bool is_dy = ju < BR;
    const int cdy = r0 + min(ju, Rb - 1), cx = c0 + min(max(ju - BR, 0), Cb - 1);
    {
        const VtSel vd = vt_sel(a.dy), vx = vt_sel(a.x);
        if (own) {
            const ChSrc ad = ch_addr(vd, cdy, a.HW), ax = ch_addr(vx, cx, a.HW);
            ChSrc& e = tabA[ju];  // field by field (a select of whole records goes through scratch)
            e.p = is_dy ? ad.p : ax.p; e.y = is_dy ? ad.y : ax.y;
            e.ns = is_dy ? ad.ns : ax.ns; e.yns = is_dy ? ad.yns : ax.yns;
            e.xf = is_dy ? ad.xf : ax.xf; e.act = is_dy ? ad.act : ax.act;
        }
    }
    // the wave's LDS operations complete in order; this keeps the compiler from hoisting
    // the table reads above the writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    f32x4 v[NU], yv[NUY > 0 ? NUY : 1];
    bool pv;
    // row j = wave + 4u of the slab (wave-uniform): j < BR dy channel r0 + j, else x channel
    // c0 + j - BR (clamped into the block: the repeats are cache hits, zeroed by `live`)
    auto issue = [&](int64_t tl) {
        const int64_t pg = tl * kKTP + 4 * lane;
        pv = pg < a.P;
        const int n = pv ? (int)(pg / a.HW) : 0;
        const int pix = pv ? (int)(pg - (int64_t)n * a.HW) : 0;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const ChSrc& t = tabA[wave + 4 * u];
            v[u] = gld4(t.p, (int64_t)n * t.ns + pix);
            if constexpr (HY)
                if (u < NUY) yv[u < NUY ? u : 0] = gld4(t.y, (int64_t)n * t.yns + pix);
        }
    };
    if (t0 < t1) issue(t0);
    // the coefficient loads go out behind the slab's (their waits may cover both: one round
    // trip either way)
    if (own) {
        const VtSel vd = vt_sel(a.dy), vx = vt_sel(a.x);
        const ChSrc& e = tabA[ju];
        const int xf = e.xf, act = e.act;
        // finalised coefficients or training-mode statistics only (host check: a.fast)
        ChanCoef k = pwk_row_coef(vd, cdy, vx, cx, is_dy, a.stat_on != 0);
        if (xf == ISG_XF_PLAIN) k = ChanCoef{0.f, 1.f, 0.f, 0.f};
        tabK[ju] = k;
        const float neg = (xf != ISG_XF_BN_FWD || act == ISG_ACT_NONE) ? 1.f : act == ISG_ACT_RELU ? 0.f : k.c3;
        tabN[ju] = float2{neg, xf == ISG_XF_BN_BWD ? 1.f : 0.f};
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    STAMP(1);

    f32x4 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool do_bias = a.dbias && cb == 0;
    float bs[BR / 4];
#pragma unroll
    for (int u = 0; u < BR / 4; ++u) bs[u] = 0.f;
    // MFMA operand bases: lane (pl, kk) reads row 16 t + pl, pixels 64 wave + 16 g + 4 kk ..
    const int kb = 64 * wave + 4 * kk;
    for (int64_t tl = t0; tl < t1; ++tl) {
        if (tl > t0) __syncthreads();  // the previous super-tile's operand reads are done
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int j = wave + 4 * u;
            const bool live = pv && (u < BR / 4 ? j < Rb : j - BR < Cb);
            const ChanCoef k = tabK[j];
            const float2 nb = tabN[j];
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = v[u][e];
                const float y = (HY && u < NUY) ? yv[u < NUY ? u : 0][e] : x;
                float zf = (x - k.c0) * k.c1 + k.c2;
                zf = zf > 0.f ? zf : zf * nb.x;
                const float zb = k.c0 * x + k.c1 * (y - k.c2) + k.c3;
                o[e] = live ? (nb.y != 0.f ? zb : zf) : 0.f;
            }
            if (u < BR / 4) bs[u] += (o[0] + o[1]) + (o[2] + o[3]);
            *reinterpret_cast<f32x4*>(&S[j * kKS + 4 * lane]) = o;
        }
        __syncthreads();
        if (tl == t0) STAMP(2);
        if (tl + 1 < t1) issue(tl + 1);  // under this super-tile's MFMAs
#pragma unroll
        for (int g = 0; g < 64; g += 16) {
            f32x4 a4[RT], b4[CT];
#pragma unroll
            for (int r = 0; r < RT; ++r) a4[r] = *reinterpret_cast<const f32x4*>(&S[(16 * r + pl) * kKS + kb + g]);
#pragma unroll
            for (int c = 0; c < CT; ++c) b4[c] = *reinterpret_cast<const f32x4*>(&S[(BR + 16 * c + pl) * kKS + kb + g]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < RT; ++r)
#pragma unroll
                    for (int c = 0; c < CT; ++c)
                        acc[r * CT + c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[r][j], b4[c][j], acc[r * CT + c], 0, 0, 0);
        }
    }
    STAMP(3);
    // ---- the four waves' partials through LDS, then one atomic per element --------------
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) S[((wave * NT + i) * 4 + r) * 64 + lane] = acc[i][r];
    __syncthreads();
    double* const dwr = a.dw + rep_off;
    {
        const int r = tid >> 6, l = tid & 63;  // element (tile i, acc slot r, lane l)
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int e = (i * 4 + r) * 64 + l;
            const float s = (S[e] + S[NT * 256 + e]) + (S[2 * NT * 256 + e] + S[3 * NT * 256 + e]);
            const int row = (i / CT) * 16 + (l >> 4) * 4 + r, col = (i % CT) * 16 + (l & 15);
            if (row < Rb && col < Cb) atomicAdd(&dwr[(int64_t)(r0 + row) * a.C + c0 + col], s);
        }
    }
    if (do_bias) {
#pragma unroll
        for (int u = 0; u < BR / 4; ++u) {
            const float s = wave_sum(bs[u]);
            const int j = wave + 4 * u;
            if (lane == 0 && j < Rb) atomicAdd(&a.dbias[rep_off + r0 + j], s);
        }
    }
    STAMP(4);
}

template <int RT, int CT, bool HY>
int32_t pwk_launch(const PwkArgs& a, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((pwk_kernel<RT, CT, HY>), grid, dim3(kThreads), 0, st, a);
    return isg_check_launch("pwk_kernel");
}

// returns 1 when launched, 0 when the shape is not for this kernel, <0 on error
int32_t pwk_try(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st) {
    // opt-in (ISG_PWK=1): faster alone (kbench 48 -> 128 at 64^2: 16.8 -> 13.1 us) but
    // slower in the step (4.01 -> 4.11 ms, 2 interleaved pairs): its 256-384 workgroups of
    // 68 KB LDS take the CUs the input-gradient chain runs on, where pwg's fewer, thinner
    // workgroups leave them free — on the side streams a thin kernel beats a fast one
    const char* pe = getenv("ISG_PWK");  // read per call: the parity test runs both paths
    const int env = pe ? atoi(pe) : 0;
    if (!env) return 0;
    const int HW = g->H * g->W;
    const int64_t P = (int64_t)g->N * HW;
    if ((int64_t)g->Co * g->Ci > 65536) return 0;
    for (int i = 0; i < x->nseg; ++i)  // the x rows' transform is loaded as BN_FWD / plain only
        if (x->s[i].xform == ISG_XF_BN_BWD) return 0;
    PwkArgs a{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias; a.rep_stride = rep_stride; a.nrep = nrep;
    a.HW = HW; a.R = g->Co; a.C = g->Ci; a.P = P;
    a.fast = pwg_fast(*dy) && pwg_fast(*x);
    if (!a.fast) return 0;  // eval-mode statistics (direct ABI calls): pwg_kernel's fp64 path
    a.stat_on = 0;
    for (const isg_vtensor* v : {dy, x})
        for (int s = 0; s < v->nseg; ++s) {
            const isg_vseg& q = v->s[s];
            if ((q.xform == ISG_XF_BN_FWD || q.xform == ISG_XF_BN_BWD) && !q.bn.coef && q.bn.stats) a.stat_on = 1;
        }
    const bool hy = pwg_has_y(*dy);
    // block shape: the fewest slab rows loaded per super-tile over the whole dW
    static const int shapes[6][2] = {{1, 3}, {3, 1}, {2, 2}, {1, 2}, {2, 1}, {1, 1}};
    int best = -1;
    int64_t best_rows = 0;
    for (int i = 0; i < 6; ++i) {
        const int br = 16 * shapes[i][0], bc = 16 * shapes[i][1];
        const int64_t rows = (int64_t)((a.R + br - 1) / br) * ((a.C + bc - 1) / bc) * (br + bc);
        if (best < 0 || rows < best_rows) { best = i; best_rows = rows; }
    }
    const int RT = shapes[best][0], CT = shapes[best][1];
    a.ncb = (a.C + 16 * CT - 1) / (16 * CT);
    const int64_t gy = (int64_t)((a.R + 16 * RT - 1) / (16 * RT)) * a.ncb;
    a.ntiles = (P + kKTP - 1) / kKTP;
    a.tiles_per_block = std::max<int64_t>(1, (gy * a.ntiles) / 384);
    const int64_t gx = (a.ntiles + a.tiles_per_block - 1) / a.tiles_per_block;
    if (gy > 65535) return 0;
    const dim3 grid((unsigned)gx, (unsigned)gy);
    int32_t rc;
#define ISG_PWK_CASE(r, c)                                                              \
    if (RT == r && CT == c)                                                             \
        rc = hy ? pwk_launch<r, c, true>(a, grid, st) : pwk_launch<r, c, false>(a, grid, st); \
    else
    ISG_PWK_CASE(1, 3) ISG_PWK_CASE(3, 1) ISG_PWK_CASE(2, 2) ISG_PWK_CASE(1, 2) ISG_PWK_CASE(2, 1)
    rc = hy ? pwk_launch<1, 1, true>(a, grid, st) : pwk_launch<1, 1, false>(a, grid, st);
#undef ISG_PWK_CASE
    return rc ? rc : 1;
}

// returns 1 when launched, 0 when the shape is not for this kernel, <0 on error
// a pwg launch, planned: its record, grid, dynamic LDS and instantiation
struct PwgPlan {
    PwgArgs a;
    dim3 grid;
    size_t lds;
    int tpw, nu;  // instantiated TPW (1, 2, 3, 4, 6, 8) and NU (4, 8, 12)
    bool hy;
    int key() const { return 1 + (tpw * 16 + nu) * 2 + (hy ? 1 : 0); }
};

// the shape and operand checks of pwg_try and the launch geometry; false: not for pwg
bool pwg_plan(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
              double* dbias, int64_t rep_stride, int32_t nrep, PwgPlan& pl) {
    if (!(g->KH == 1 && g->KW == 1 && g->SH == 1 && g->SW == 1 && g->PH == 0 && g->PW == 0))
        return false;
    if (g->OH != g->H || g->OW != g->W || g->Co < 2) return false;
    const int HW = g->H * g->W;
    if (!pwg_src_ok(*dy, HW) || !pwg_src_ok(*x, HW)) return false;
    PwgArgs& a = pl.a;
    a = PwgArgs{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias; a.rep_stride = rep_stride; a.nrep = nrep;
    a.HW = HW; a.R = g->Co; a.C = g->Ci;
    a.P = (int64_t)g->N * HW;
    a.fast = pwg_fast(*dy) && pwg_fast(*x);
    a.stat_on = 0;
    for (const isg_vtensor* v : {dy, x})
        for (int s = 0; s < v->nseg; ++s) {
            const isg_vseg& q = v->s[s];
            if ((q.xform == ISG_XF_BN_FWD || q.xform == ISG_XF_BN_BWD) && !q.bn.coef && q.bn.stats) a.stat_on = 1;
        }
    pl.hy = pwg_has_y(*dy) || pwg_has_y(*x);
    a.ntiles = (a.P + kGTP - 1) / kGTP;
    int br = std::min(64, (a.R + 15) / 16 * 16);
    int bc = std::min(kGMaxRows - br, std::min(128, (a.C + 15) / 16 * 16));
    auto gy_of = [&](int bcv) {
        return (int64_t)((a.R + br - 1) / br) * ((a.C + bcv - 1) / bcv);
    };
    // narrower column blocks while the grid would not cover the CUs
    while (bc > 32 && a.ntiles * gy_of(bc) < 256) bc = (bc / 2 + 15) / 16 * 16;
    a.BR = br; a.BC = bc;
    a.ncb = (a.C + bc - 1) / bc;
    const int64_t gy = gy_of(bc);
    int64_t gx = std::max<int64_t>(1, 512 / gy);
    if (gx > a.ntiles) gx = a.ntiles;
    a.tiles_per_block = (a.ntiles + gx - 1) / gx;
    // at least 2 tiles per workgroup: half the dW atomics, and — these kernels run on the
    // executor's side stream — half the workgroups competing with the input-gradient
    // chain (measured: 5.55 -> 5.43 ms/step; the 256->128 resconv wgrads 41 -> 35 us)
    if (a.tiles_per_block < 2) a.tiles_per_block = 2;
    gx = (a.ntiles + a.tiles_per_block - 1) / a.tiles_per_block;
    if (gx * gy >= (1ll << 31)) return false;
    a.off_k = (kThreads * (int)sizeof(ChSrc) + 15) & ~15;
    a.off_x = (a.off_k + kGMaxRows * (int)(sizeof(ChanCoef) + 2 * sizeof(float)) + 15) & ~15;
    pl.lds = (size_t)a.off_x + (size_t)(br + bc) * kGS * sizeof(float);
    const int tpw = ((br / 16) * (bc / 16) + 3) / 4;
    pl.tpw = tpw <= 4 ? tpw : tpw <= 6 ? 6 : 8;
    pl.grid = dim3((unsigned)gx, (unsigned)gy);
    const int passes = (br + bc + 15) / 16;
    pl.nu = passes <= 4 ? 4 : passes <= 8 ? 8 : 12;
    return true;
}

template <int TPW, int NU, bool HY>
int32_t pwg_group_launch_t(const PwgPlan* const* pl, int n, hipStream_t st) {
    PwgGroupMeta m{};
    size_t lds = 0;
    int64_t total = 0;
    for (int i = 0; i < n; ++i) {
        m.start[i] = (int)total;
        m.gx[i] = (int)pl[i]->grid.x;
        total += (int64_t)pl[i]->grid.x * pl[i]->grid.y;
        lds = std::max(lds, pl[i]->lds);
    }
    m.start[n] = (int)total;
    m.n = n;
    if (total >= (1ll << 31)) return isg_set_error(ISG_ERR_UNSUPPORTED, "pwg group: grid");
    auto k = pwg_group_kernel<TPW, NU, HY>;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) != hipSuccess)
            return isg_check_launch("pwg_group_kernel: dynamic LDS");
        attr = true;
    }
    const PwgArgs& a0 = pl[0]->a;
    const PwgArgs& a1 = pl[n > 1 ? 1 : 0]->a;
    const PwgArgs& a2 = pl[n > 2 ? 2 : 0]->a;
    hipLaunchKernelGGL(k, dim3((unsigned)total), dim3(kThreads), lds, st, a0, a1, a2, m);
    return isg_check_launch("pwg_group_kernel");
}

template <int TPW, int NU, bool HY>
int32_t pwg_launch_plan(const PwgPlan* const* pl, int n, hipStream_t st) {
    if (n == 1) return pwg_launch<TPW, NU, HY>(pl[0]->a, pl[0]->grid, pl[0]->lds, st);
    return pwg_group_launch_t<TPW, NU, HY>(pl, n, st);
}

// n plans of one key (same instantiation), n <= kPwgGroup
int32_t pwg_run(const PwgPlan* const* pl, int n, hipStream_t st) {
    const PwgPlan& p = *pl[0];
#define ISG_PWG_T(T)                                                                     \
    if (p.tpw == T) {                                                                    \
        if (p.nu == 4) return p.hy ? pwg_launch_plan<T, 4, true>(pl, n, st) : pwg_launch_plan<T, 4, false>(pl, n, st); \
        if (p.nu == 8) return p.hy ? pwg_launch_plan<T, 8, true>(pl, n, st) : pwg_launch_plan<T, 8, false>(pl, n, st); \
        return p.hy ? pwg_launch_plan<T, 12, true>(pl, n, st) : pwg_launch_plan<T, 12, false>(pl, n, st); \
    }
    ISG_PWG_T(1) ISG_PWG_T(2) ISG_PWG_T(3) ISG_PWG_T(4) ISG_PWG_T(6) ISG_PWG_T(8)
#undef ISG_PWG_T
    return isg_set_error(ISG_ERR_INVALID, "pwg: tpw %d", p.tpw);
}

// returns 1 when launched, 0 when the shape is not for this kernel, <0 on error
int32_t pwg_try(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st) {
    {
        if (!(g->KH == 1 && g->KW == 1 && g->SH == 1 && g->SW == 1 && g->PH == 0 && g->PW == 0))
            return 0;
        if (g->OH != g->H || g->OW != g->W || g->Co < 2) return 0;
        const int HW = g->H * g->W;
        if (!pwg_src_ok(*dy, HW) || !pwg_src_ok(*x, HW)) return 0;
        if (const int32_t k = pwk_try(g, dy, x, dw, dbias, rep_stride, nrep, st)) return k;
    }
    PwgPlan pl;
    if (!pwg_plan(g, dy, x, dw, dbias, rep_stride, nrep, pl)) return 0;
    const PwgPlan* p = &pl;
    const int32_t rc = pwg_run(&p, 1, st);
    return rc ? rc : 1;
}

int vt_channels(const isg_vtensor* v) {
    int c = 0;
    for (int i = 0; i < v->nseg; ++i) c += v->s[i].C;
    return c;
}

}  // namespace

ISG_STAMP_ACCESSOR(isg_dbg_stamps_wgrad)

int32_t isg_tap_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                      double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st);

int32_t isg_thin_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                       double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st);
int32_t isg_down_conv_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                            double* dw, double* dbias, int64_t rep_stride, int32_t nrep,
                            hipStream_t st);
int32_t isg_s2k5_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                       double* dw, double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st);

int32_t isg_dense_conv_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                             double* dw, double* dbias, int64_t rep_stride, int32_t nrep,
                             hipStream_t st) {
    if (vt_channels(dy) != g->Co || vt_channels(x) != g->Ci)
        return isg_set_error(ISG_ERR_INVALID, "conv wgrad: channel mismatch");
    if (!dw) return isg_set_error(ISG_ERR_INVALID, "conv wgrad: dw is NULL");
    if (!(g->KH == 1 && g->KW == 1)) {  // thin 3x3 (thin_conv.hip), narrow spatial (tap_wgrad.hip)
        int32_t t = isg_thin_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);
        if (t != 0) return t < 0 ? t : 0;
        t = isg_down_conv_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);  // convT weights
        if (t != 0) return t < 0 ? t : 0;
        t = isg_s2k5_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);  // the stem's layer 2
        if (t != 0) return t < 0 ? t : 0;
        t = isg_tap_wgrad(g, dy, x, dw, dbias, rep_stride, nrep, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    {
        const int32_t t = pwg_try(g, dy, x, dw, dbias, rep_stride, nrep, st);
        if (t != 0) return t < 0 ? t : 0;
    }
    WgArgs a{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias;
    a.rep_stride = rep_stride; a.nrep = nrep;
    a.N = g->N; a.OH = g->OH; a.OW = g->OW; a.H = g->H; a.W = g->W;
    a.R = g->Co; a.Ci = g->Ci; a.KH = g->KH; a.KW = g->KW; a.SH = g->SH; a.SW = g->SW;
    a.PH = g->PH; a.PW = g->PW; a.DH = g->DH; a.DW = g->DW;
    const int KK = g->KH * g->KW;
    const int ncol = g->Ci * KK;
    const int CT = (ncol + 15) / 16;
    // tile width: 64 pixels of a row for stride-1 1x1 convs on wide maps, else 16 (a
    // 4x16 tile), narrowed until the halo row fits the 64 lanes
    const bool pw = KK == 1 && g->SH == 1 && g->SW == 1;
    int tc = pw ? (g->OW >= 64 ? 64 : (g->OW >= 32 ? 32 : 16)) : 16;
    auto hc_of = [&](int t) { return (t - 1) * g->SW + (g->KW - 1) * g->DW + 1; };
    while (tc > 8 && hc_of(tc) > 64) tc /= 2;
    if (hc_of(tc) > 64)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: halo row %d > 64", hc_of(tc));
    a.lgTC = tc == 64 ? 6 : (tc == 32 ? 5 : (tc == 16 ? 4 : 3));
    const int TC = tc, TR = kTP / TC;
    a.HR = (TR - 1) * g->SH + (g->KH - 1) * g->DH + 1;
    a.HC = hc_of(tc);
    const int hs = a.HR * a.HC;
    a.hsp = hs + ((2 - hs % 32) + 32) % 32;  // channel stride = 2 mod 32 banks
    a.valu = g->Co == 1 ? 1 : 0;
    const int nrt = (std::min(g->Co, kRowsBlk) + 15) / 16;
    a.BMT = nrt;
    // widest column block whose halo fits the slot budget
    auto max_nci = [&](int bnt) {
        int m = 0;
        for (int c_lo = 0; c_lo < ncol; c_lo += bnt * 16) {
            const int c_hi = std::min(ncol, c_lo + bnt * 16);
            m = std::max(m, (c_hi - 1) / KK + 1 - c_lo / KK);
        }
        return m;
    };
    auto fits = [&](int bnt) {
        const int m = max_nci(bnt);
        return m <= kMaxXCh && m * a.hsp <= kXs;
    };
    int bnt = a.valu ? 4 : std::min(CT, std::max(1, 16 / nrt));  // <= 4 tiles per wave (VGPRs)
    bnt = std::min(bnt, kColsBlk / 16);
    while (bnt > 1 && !fits(bnt)) --bnt;
    if (!fits(bnt))
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: halo %d rows x %d too large",
                             a.HR, a.HC);
    a.BNT = bnt;
    a.ncb = (ncol + bnt * 16 - 1) / (bnt * 16);
    const int nrb = (g->Co + kRowsBlk - 1) / kRowsBlk;
    const int gy = nrb * a.ncb;
    a.tiles_x = (g->OW + TC - 1) / TC;
    a.tiles_y = (g->OH + TR - 1) / TR;
    a.ntiles = (int64_t)g->N * a.tiles_x * a.tiles_y;
    int64_t gx = std::max<int64_t>(1, 1024 / gy);
    if (gx > a.ntiles) gx = a.ntiles;
    a.tiles_per_block = (a.ntiles + gx - 1) / gx;
    gx = (a.ntiles + a.tiles_per_block - 1) / a.tiles_per_block;
#ifdef ISG_STAMPS
    { const char* e = getenv("ISG_DBG"); a.dbg = e ? atoi(e) : 0; }
#endif
    dim3 grid((unsigned)gx, (unsigned)gy);
    const int tpw = (a.BMT * a.BNT + 3) / 4;
    // halo floats (>= 768: the k-split / VALU partial sums reuse that space)
    const size_t xs = std::max<size_t>((size_t)max_nci(bnt) * a.hsp, 768);
    const size_t lds = ((size_t)a.BMT * 16 * kAStride + xs) * sizeof(float);
#define WG_LAUNCH(T) hipLaunchKernelGGL((wgrad_kernel<T>), grid, dim3(kThreads), lds, st, a)
    switch (tpw) {
        case 1: WG_LAUNCH(1); break;
        case 2: WG_LAUNCH(2); break;
        case 3: WG_LAUNCH(3); break;
        case 4: WG_LAUNCH(4); break;
        case 5: case 6: WG_LAUNCH(6); break;
        default: WG_LAUNCH(8); break;
    }
#undef WG_LAUNCH
    return isg_check_launch("wgrad_kernel");
}

// ---- executor hooks (api.cpp): the 1x1 weight gradients of a side-stream batch, grouped --
// isg_pwg_plan: > 0 (the instantiation key) when isg_conv_wgrad_rep would run this op on
// pwg_kernel, the plan written into `plan` (isg_pwg_plan_bytes() bytes); 0 otherwise.
// isg_pwg_run: launch n <= isg_pwg_group_max() plans of one key as one launch.
extern "C" int32_t isg_pwg_plan_bytes() { return (int32_t)sizeof(PwgPlan); }
extern "C" int32_t isg_pwg_group_max() { return kPwgGroup; }

extern "C" int32_t isg_pwg_plan(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                     double* dbias, int64_t rep_stride, int32_t nrep, void* plan) {
    if (isg_vt_res(dy) || isg_vt_res(x)) return 0;  // isg_conv_wgrad_rep refuses it
    const char* pe = getenv("ISG_PWK");
    if (pe && atoi(pe)) return 0;  // the opt-in pwk path stays on the per-op route
    if (!dw || nrep < 1 || (nrep > 1 && rep_stride <= 0) || g->groups != 1) return 0;
    if (g->w_ci && g->w_ci != g->Ci) return 0;
    if (vt_channels(dy) != g->Co || vt_channels(x) != g->Ci) return 0;
    PwgPlan& pl = *static_cast<PwgPlan*>(plan);
    if (!pwg_plan(g, dy, x, dw, dbias, rep_stride, nrep, pl)) return 0;
    return pl.key();
}

extern "C" int32_t isg_pwg_run(const void* const* plans, int32_t n, hipStream_t st) {
    if (n < 1 || n > kPwgGroup) return isg_set_error(ISG_ERR_INVALID, "pwg group of %d", n);
    const PwgPlan* pl[kPwgGroup];
    for (int i = 0; i < n; ++i) {
        pl[i] = static_cast<const PwgPlan*>(plans[i]);
        if (pl[i]->key() != pl[0]->key()) return isg_set_error(ISG_ERR_INVALID, "pwg group: mixed kernels");
    }
    return pwg_run(pl, n, st);
}

