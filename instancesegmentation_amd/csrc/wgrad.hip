// Weight gradient of dense convolutions (gfx950): every nn.Conv2d weight of the
// reference (segment.py) and — with the operand roles swapped — the ConvTranspose2d
// weights (segment.py:305, :435).
//
//   dW[row][col] += sum_p dy[row][p] * x[ci][p*S - P + (kh,kw)*D],  col = ci*KH*KW + kh*KW + kw
//
// A GEMM with the output pixels as the reduction (K) dimension. A workgroup owns a block
// of up to 64 rows x 128 columns of dW and a contiguous range of 64-pixel tiles (4x16,
// 2x32 or 1x64 output pixels). Per tile it stages into LDS
//   * the dy rows (BatchNorm-backward rebuilt on load), and
//   * the INPUT HALO of the tile for the block's input channels (producer BatchNorm +
//     activation applied on load),
// and every (kh,kw) tap reads the halo at a shifted offset (no im2col gather).
// The global loads of tile t+1 are issued into registers before the MFMAs of tile t
// (register double buffer): with 64-pixel tiles a block spends ~1-4k MFMA cycles per
// tile, which covers the HBM latency of the next tile's loads.
// MFMA v_mfma_f32_16x16x4_f32: A[i=row][k=pixel] from LDS dy, B[k=pixel][j=col] from the
// halo. Each wave keeps up to 4 16x16 accumulator tiles; blocks with fewer than 4 tiles
// split the 64 pixels of a tile across waves. A single-row dW (the 4->1 mask-head conv,
// segment.py:437) runs on the VALU instead: an MFMA there would be 15/16 padding.
// Partial sums leave the block with one f32 atomic per dW element.
#include "common.h"
#include <cstdlib>

namespace {

constexpr int kThreads = 256;
constexpr int kTP = 64;             // pixels per tile
constexpr int kAStride = kTP + 2;   // conflict-free A-fragment reads
constexpr int kRowsBlk = 64;        // dW rows per block (BMT <= 4)
constexpr int kColsBlk = 128;       // dW columns per block (BNT <= 8)
constexpr int kPA = kRowsBlk * kTP / kThreads;  // A elements per thread per tile (16)
constexpr int kPX = 16;             // halo elements per thread per tile (max)
constexpr int kHaloMax = kPX * kThreads;
constexpr int kMaxXCh = 128;        // halo channels per block

struct VChan {
    const float* p;
    const float* y;
    int ns, yns;  // elements between images (< 2^31 for every tensor here)
    int xf, act;
    ChanCoef k;
};

struct WgArgs {
    isg_vtensor dy;  // rows: N x R x OH x OW
    isg_vtensor x;   // gathered: N x Ci x H x W
    float* dw;
    float* dbias;
    int64_t rep_stride;
    int nrep;
    int N, OH, OW, H, W, R, Ci, KH, KW, SH, SW, PH, PW, DH, DW;
    int BMT, BNT, ncb;          // 16-row / 16-col tiles per block, column blocks
    int HR, HC, hsp;            // halo rows, cols, LDS channel stride
    int lgTC;                   // log2 tile width (tile = (64>>lgTC) x (1<<lgTC))
    int tiles_x, tiles_y;
    int64_t ntiles, tiles_per_block;
    int valu;                   // R == 1 path
    unsigned m_hs, m_hc;        // ceil(2^32 / (HR*HC)), ceil(2^32 / HC)
    int dbg;                    // ablation bits (stamp build only, tools/kbench)
};
#ifdef ISG_STAMPS
#define DBG(a, b) ((a).dbg & (b))
#else
#define DBG(a, b) 0
#endif

// Fill the per-channel source table of channels [c_lo, c_lo+nc) of a vtensor.
ISG_DEV void load_vchan(const isg_vtensor& vt, int c_lo, int nc, int64_t hw, VChan* tab,
                        int tid) {
    for (int i = tid; i < nc; i += kThreads) {
        const int c = c_lo + i;
        int s = 0, cb = 0;
        if (vt.nseg > 1 && c >= vt.s[0].C) { s = 1; cb = vt.s[0].C; }
        if (vt.nseg > 2 && c >= vt.s[0].C + vt.s[1].C) { s = 2; cb = vt.s[0].C + vt.s[1].C; }
        const isg_vseg& sg = vt.s[s];
        const int cl = c - cb;
        VChan v;
        v.p = sg.p + (int64_t)cl * hw;
        v.y = (sg.xform == ISG_XF_BN_BWD && sg.y) ? sg.y + (int64_t)cl * hw : v.p;  // always loadable
        v.ns = (int)sg.n_stride;
        v.yns = (int)sg.y_n_stride;
        v.xf = sg.xform;
        v.act = sg.act;
        ChanCoef k = {0.f, 1.f, 0.f, 0.f};
        if (sg.xform == ISG_XF_BN_FWD) {
            if (sg.bn.stats || !sg.bn.train) {
                k = fwd_coef(sg.bn, sg.slope, cl);
            } else {
                k.c3 = sg.slope ? sg.slope[cl] : 0.f;
            }
        } else if (sg.xform == ISG_XF_BN_BWD) {
            k = bwd_coef(sg.bn, cl);
        }
        v.k = k;
        tab[i] = v;
    }
}


// exact n / d for n, d < 2^16 with m = ceil(2^32 / d) (host-computed)
ISG_DEV int fdiv(int n, unsigned m) { return (int)__umulhi((unsigned)n, m); }

// Virtual-tensor transform with per-lane format (selects, no branches).
ISG_DEV float vchan_apply_sel(const VChan& c, float x, float y) {
    const float z = (x - c.k.c0) * c.k.c1 + c.k.c2;
    const float za = c.act == ISG_ACT_RELU ? fmaxf(z, 0.f)
                     : (c.act == ISG_ACT_PRELU ? (z > 0.f ? z : z * c.k.c3) : z);
    const float b = c.k.c0 * x + c.k.c1 * (y - c.k.c2) + c.k.c3;
    return c.xf == ISG_XF_PLAIN ? x : (c.xf == ISG_XF_BN_FWD ? za : b);
}

// BMT: 16-row tiles of dW per block (A loads per thread = 4*BMT); AB / XB: the dy / x
// operand has BatchNorm-backward channels (second load of the saved forward output).
template <int BMT, bool AB, bool XB>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(WgArgs a) {
    constexpr int TPW = 4;      // accumulator tiles per wave (BMT*BNT <= 16)
    constexpr int NA = 4 * BMT; // A elements per thread per tile
    __shared__ float As[kRowsBlk * kAStride];
    __shared__ float Xs[kHaloMax + 64];
    __shared__ VChan tabA[kRowsBlk];
    __shared__ VChan tabX[kMaxXCh];

    STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
    const int hs = a.HR * a.HC;
    const int TC = 1 << a.lgTC;
    const int64_t ohw = (int64_t)a.OH * a.OW, xhw = (int64_t)a.H * a.W;
    // this workgroup's replica of dW / dbias (include/isg.h ISG_WREP)
    const int64_t rep_off = (int64_t)((blockIdx.x + 7u * blockIdx.y) % (unsigned)a.nrep) * a.rep_stride;
    float* const dwr = a.dw + rep_off;

    if (!DBG(a, 1)) {
        load_vchan(a.dy, r_lo, Rb, ohw, tabA, tid);
        load_vchan(a.x, ci_lo, nci, xhw, tabX, tid);
    } else {
        for (int i = tid; i < kRowsBlk + kMaxXCh; i += kThreads) {
            VChan v = {a.dy.s[0].p, a.dy.s[0].p, 0, 0, 0, 0, {0.f, 1.f, 0.f, 0.f}};
            if (i < kRowsBlk) tabA[i] = v; else { v.p = v.y = a.x.s[0].p; tabX[i - kRowsBlk] = v; }
        }
    }

    // ---- per-thread element lists (tile-invariant) --------------------------------
    // A: pixel p = lane, rows wave + 4j (j < NA); rows >= Rb load row Rb-1, store 0
    const int ap = lane;
    const int apy = ap >> a.lgTC, apx = ap & (TC - 1);
    const int na = (Rb + 3 - wave) / 4;  // wave-uniform
    // X: halo element e = tid + 256 j, packed (cl << 20 | hr << 10 | hc); -1 past the end
    const int nxe = nci * hs;
    const int nxj = (nxe + kThreads - 1) / kThreads;  // block-uniform
    int xe[kPX];
#pragma unroll
    for (int j = 0; j < kPX; ++j) {
        const int e = tid + kThreads * j;
        const int cl = fdiv(e, a.m_hs), rem = e - cl * hs;
        const int hr = fdiv(rem, a.m_hc), hc = rem - hr * a.HC;
        xe[j] = e < nxe ? ((cl << 20) | (hr << 10) | hc) : -1;
    }

    // ---- MFMA operand offsets --------------------------------------------------------
    const int nt = BMT * a.BNT;
    const bool ksplit = nt < 4;
    const int ks = ksplit ? 4 / nt : 1;
    const int kpart = ksplit ? wave / nt : 0;
    const bool kactive = !ksplit || kpart < ks;
    const int kq_lo = kpart * (kTP / ks), kq_hi = kq_lo + kTP / ks;
    int arow[TPW], xoff[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = ksplit ? (i == 0 && kactive ? wave % nt : 1 << 20) : wave + 4 * i;
        const int rt = t / a.BNT, ct = t - rt * a.BNT;
        arow[i] = -1;
        xoff[i] = -1;
        if (t < nt) {
            arow[i] = (rt * 16 + pl) * kAStride;
            const int col = c_lo + ct * 16 + pl;
            if (col < c_hi) {
                const int ci = col / KK, tap = col - ci * KK;
                const int kh = tap / a.KW, kw = tap - kh * a.KW;
                xoff[i] = (ci - ci_lo) * a.hsp + kh * a.DH * a.HC + kw * a.DW;
            }
        }
    }
    f32x4 acc[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float vacc = 0.f;  // VALU path (R == 1): column tid&63, pixel quarter tid>>6
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
    const int TR = kTP >> a.lgTC;

    // register double buffer: raw values of the next tile; loads are unconditional
    // (clamped addresses) so the compiler issues them back to back
    float ra[NA], ry[NA], rx[kPX], rxy[kPX];
    auto tile_origin = [&](int64_t tl, int& n, int& oy0, int& ox0) {
        n = (int)(tl / per_img);
        const int r = (int)(tl - (int64_t)n * per_img);
        const int ty = r / a.tiles_x;
        oy0 = ty * TR;
        ox0 = (r - ty * a.tiles_x) * TC;
    };
    auto load_tile = [&](int64_t tl) {
        int n, oy0, ox0;
        tile_origin(tl, n, oy0, ox0);
        const int oy = oy0 + apy, ox = ox0 + apx;
        const int pix = (oy < a.OH && ox < a.OW) ? oy * a.OW + ox : 0;
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            if (j < na) {  // wave-uniform
                const VChan& c = tabA[wave + 4 * j];
                if (DBG(a, 2)) { ra[j] = 1.f; ry[j] = 1.f; continue; }
                ra[j] = gld(c.p, n * c.ns + pix);
                if (AB) ry[j] = gld(c.y, n * c.yns + pix);
            }
        }
        const int iy0 = oy0 * a.SH - a.PH, ix0 = ox0 * a.SW - a.PW;
#pragma unroll
        for (int j = 0; j < kPX; ++j) {
            if (j < nxj) {  // block-uniform
                const int v = xe[j];
                const int iy = iy0 + ((v >> 10) & 1023), ix = ix0 + (v & 1023);
                const bool ok = v >= 0 && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                const VChan& c = tabX[v >= 0 ? v >> 20 : 0];
                const int o = ok ? iy * a.W + ix : 0;
                if (DBG(a, 2)) { rx[j] = 1.f; rxy[j] = 1.f; continue; }
                rx[j] = gld(c.p, n * c.ns + o);
                if (XB) rxy[j] = gld(c.y, n * c.yns + o);
            }
        }
    };
    auto store_tile = [&](int64_t tl) {
        int n, oy0, ox0;
        tile_origin(tl, n, oy0, ox0);
        const bool pv = oy0 + apy < a.OH && ox0 + apx < a.OW;
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            float v = 0.f;
            if (j < na) {  // wave-uniform
                const VChan& c = tabA[wave + 4 * j];
                const float t = vchan_apply_sel(c, ra[j], AB ? ry[j] : 0.f);
                v = pv ? t : 0.f;
            }
            As[(wave + 4 * j) * kAStride + ap] = v;
        }
        const int iy0 = oy0 * a.SH - a.PH, ix0 = ox0 * a.SW - a.PW;
#pragma unroll
        for (int j = 0; j < kPX; ++j) {
            if (j < nxj) {  // block-uniform
                const int v = xe[j];
                const int cl = v >> 20, hr = (v >> 10) & 1023, hc = v & 1023;
                const int iy = iy0 + hr, ix = ix0 + hc;
                const bool ok = v >= 0 && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                const float t = vchan_apply_sel(tabX[v >= 0 ? cl : 0], rx[j], XB ? rxy[j] : 0.f);
                if (v >= 0) Xs[cl * a.hsp + hr * a.HC + hc] = ok ? t : 0.f;
            }
        }
    };

    if (t0 < t1) load_tile(t0);
    for (int64_t tl = t0; tl < t1; ++tl) {
        __syncthreads();  // previous tile's LDS reads are done
        store_tile(tl);
        __syncthreads();
        if (tl == t0) STAMP(2);
        if (tl + 1 < t1) load_tile(tl + 1);  // in flight during this tile's MFMAs
        if (do_bias && tid < Rb) {
            const float* rowp = As + tid * kAStride;
            float s = 0.f;
#pragma unroll 16
            for (int p = 0; p < kTP; ++p) s += rowp[p];
            bsum += s;
        }
        if (a.valu) {
            if (vxoff >= 0) {
                const int q0 = (tid >> 6) * 16;
#pragma unroll
                for (int p = q0; p < q0 + 16; ++p) {
                    const int poff = (p >> a.lgTC) * a.SH * a.HC + (p & (TC - 1)) * a.SW;
                    vacc = fmaf(As[p], Xs[vxoff + poff], vacc);
                }
            }
            continue;
        }
        if (!kactive || DBG(a, 4)) continue;
#pragma unroll 4
        for (int kq = kq_lo; kq < kq_hi; kq += 4) {
            const int p = kq + kk;
            const int poff = (p >> a.lgTC) * a.SH * a.HC + (p & (TC - 1)) * a.SW;
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                if (arow[i] >= 0) {  // wave-uniform
                    const float av = As[arow[i] + p];
                    const float bv = xoff[i] >= 0 ? Xs[xoff[i] + poff] : 0.f;
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i], 0, 0, 0);
                }
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

int vt_channels(const isg_vtensor* v) {
    int c = 0;
    for (int i = 0; i < v->nseg; ++i) c += v->s[i].C;
    return c;
}

}  // namespace

ISG_STAMP_ACCESSOR(isg_dbg_stamps_wgrad)

int32_t isg_dense_conv_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                             float* dw, float* dbias, int64_t rep_stride, int32_t nrep,
                             hipStream_t st) {
    if (vt_channels(dy) != g->Co || vt_channels(x) != g->Ci)
        return isg_set_error(ISG_ERR_INVALID, "conv wgrad: channel mismatch");
    if (!dw) return isg_set_error(ISG_ERR_INVALID, "conv wgrad: dw is NULL");
    WgArgs a{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias;
    a.rep_stride = rep_stride; a.nrep = nrep;
    a.N = g->N; a.OH = g->OH; a.OW = g->OW; a.H = g->H; a.W = g->W;
    a.R = g->Co; a.Ci = g->Ci; a.KH = g->KH; a.KW = g->KW; a.SH = g->SH; a.SW = g->SW;
    a.PH = g->PH; a.PW = g->PW; a.DH = g->DH; a.DW = g->DW;
    const int KK = g->KH * g->KW;
    const int ncol = g->Ci * KK;
    const int CT = (ncol + 15) / 16;
    // tile shape: 1x64 rows for stride-1 1x1 convs on wide maps, else 4x16
    const bool pw = KK == 1 && g->SH == 1 && g->SW == 1;
    a.lgTC = (pw && g->OW >= 64) ? 6 : (g->OW >= 32 && pw ? 5 : 4);
    const int TC = 1 << a.lgTC, TR = kTP / TC;
    a.HR = (TR - 1) * g->SH + (g->KH - 1) * g->DH + 1;
    a.HC = (TC - 1) * g->SW + (g->KW - 1) * g->DW + 1;
    if (a.HR >= 1024 || a.HC >= 1024)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: halo %dx%d", a.HR, a.HC);
    const int hs = a.HR * a.HC;
    a.hsp = hs + ((2 - hs % 32) + 32) % 32;  // channel stride = 2 mod 32 banks
    a.valu = g->Co == 1 ? 1 : 0;
    const int nrt = (std::min(g->Co, kRowsBlk) + 15) / 16;
    a.BMT = nrt;
    // widest column block whose halo fits the per-thread prefetch budget
    auto max_nci = [&](int bnt) {
        int m = 0;
        for (int c_lo = 0; c_lo < ncol; c_lo += bnt * 16) {
            const int c_hi = std::min(ncol, c_lo + bnt * 16);
            m = std::max(m, (c_hi - 1) / KK + 1 - c_lo / KK);
        }
        return m;
    };
    int bnt = a.valu ? 4 : std::min(CT, std::max(1, 16 / nrt));
    bnt = std::min(bnt, kColsBlk / 16);
    while (bnt > 1 && (max_nci(bnt) * a.hsp > kHaloMax || max_nci(bnt) > kMaxXCh)) --bnt;
    const int mnci = max_nci(bnt);
    if (mnci * a.hsp > kHaloMax || mnci > kMaxXCh || mnci * hs > kHaloMax)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: halo %d x %d too large", mnci, hs);
    if (a.valu && bnt * 16 > 64) bnt = 4;
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
    const int hs2 = a.HR * a.HC;
    a.m_hs = (unsigned)(((1ull << 32) + hs2 - 1) / hs2);
    a.m_hc = (unsigned)(((1ull << 32) + a.HC - 1) / a.HC);
    bool xb = false;
    for (int i = 0; i < x->nseg; ++i) xb = xb || x->s[i].xform == ISG_XF_BN_BWD;
    bool ab = false;
    for (int i = 0; i < dy->nseg; ++i) ab = ab || dy->s[i].xform == ISG_XF_BN_BWD;
    dim3 grid((unsigned)gx, (unsigned)gy);
#define WG_LAUNCH(M, A, B) hipLaunchKernelGGL((wgrad_kernel<M, A, B>), grid, dim3(kThreads), 0, st, a)
#define WG_LAUNCH_M(A, B)                        \
    switch (a.BMT) {                             \
        case 1: WG_LAUNCH(1, A, B); break;       \
        case 2: WG_LAUNCH(2, A, B); break;       \
        case 3: WG_LAUNCH(3, A, B); break;       \
        default: WG_LAUNCH(4, A, B); break;      \
    }
    if (ab && xb) WG_LAUNCH_M(true, true)
    else if (ab) WG_LAUNCH_M(true, false)
    else if (xb) WG_LAUNCH_M(false, true)
    else WG_LAUNCH_M(false, false)
#undef WG_LAUNCH_M
#undef WG_LAUNCH
    return isg_check_launch("wgrad_kernel");
}
