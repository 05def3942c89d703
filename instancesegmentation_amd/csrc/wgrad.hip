// Weight gradient of dense convolutions on v_mfma_f32_16x16x4_f32 (gfx950).
//
//   dW[row][col] += sum_p dy[row][p] * x[ci][p*S - P + (kh,kw)*D],  col = ci*KH*KW + kh*KW + kw
//
// (segment.py: every nn.Conv2d weight of the reference; the ConvTranspose2d weights
// run through here with the operand roles swapped.) Pixels are the MFMA K dimension.
// A workgroup owns a 4x16 tile of dy pixels at a time: it stages the dy rows (with the
// BatchNorm-backward rebuild applied on load) and the INPUT HALO of that tile (with the
// producer's BatchNorm+activation applied on load) into LDS once; every (kh,kw) tap then
// reads the halo at a shifted offset — no im2col gather, each input element is loaded
// and transformed once per tile instead of KH*KW times.
// Each wave accumulates up to 8 (16-row x 16-col) output tiles in registers across all
// pixel tiles of its workgroup; partial sums are flushed with one f32 atomic per element.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTR = 4, kTC = 16, kTP = kTR * kTC;  // pixel tile (64 pixels)
constexpr int kAStride = kTP + 2;                   // conflict-free A-fragment reads
constexpr int kMaxTiles = 8;                        // output tiles per wave

struct WgArgs {
    isg_vtensor dy;  // rows: N x R x OH x OW
    isg_vtensor x;   // gathered: N x Ci x H x W
    float* dw;
    float* dbias;
    int N, OH, OW, H, W, R, Ci, KH, KW, SH, SW, PH, PW, DH, DW;
    int RT, CTB, HR, HC;
    int64_t ntiles, tiles_per_block;
    int tiles_x, tiles_y;
};

__global__ __launch_bounds__(kThreads) void wgrad_tiled_kernel(WgArgs a) {
    extern __shared__ float smem[];
    __shared__ ChanCoef cdy[ISG_MAX_CH];
    __shared__ ChanCoef cx[ISG_MAX_CH];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int kk = lane >> 4;
    const int pl = lane & 15;
    const int KK = a.KH * a.KW;
    const int NCOL = a.Ci * KK;
    const int c_lo = blockIdx.y * a.CTB * 16;
    const int c_hi = min(NCOL, c_lo + a.CTB * 16);
    const int ci_lo = c_lo / KK;
    const int ci_hi = (c_hi - 1) / KK + 1;
    const int nci = ci_hi - ci_lo;
    const int halo = a.HR * a.HC;
    const int Rpad = a.RT * 16;
    float* As = smem;
    float* Xs = smem + Rpad * kAStride;

    load_vt_coefs(a.dy, cdy, tid, kThreads);
    load_vt_coefs(a.x, cx, tid, kThreads);

    // per-lane tile descriptors (tile t = wave + 4*i). With fewer than 4 output tiles
    // (narrow layers) the waves split the 64 pixels of each tile instead (k-split) and
    // combine their partial sums through LDS before the atomics.
    const int ntile_blk = a.RT * a.CTB;
    const bool ksplit = ntile_blk < 4;
    const int ks = ksplit ? 4 / ntile_blk : 1;          // waves per tile
    const int kpart = ksplit ? wave / ntile_blk : 0;    // this wave's pixel quarter/half
    const bool kactive = !ksplit || kpart < ks;
    const int kq_lo = kpart * (kTP / ks), kq_hi = kq_lo + kTP / ks;
    int arow[kMaxTiles], xoff[kMaxTiles];
#pragma unroll
    for (int i = 0; i < kMaxTiles; ++i) {
        const int t = ksplit ? (i == 0 ? wave % ntile_blk : 1 << 20) : wave + 4 * i;
        const int rt = t / a.CTB, ct = t - rt * a.CTB;
        arow[i] = (rt * 16 + pl) * kAStride;
        const int col = c_lo + ct * 16 + pl;
        xoff[i] = -1;
        if (t < ntile_blk && col < c_hi) {
            const int ci = col / KK, tap = col - ci * KK;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            xoff[i] = (ci - ci_lo) * halo + kh * a.DH * a.HC + kw * a.DW;
        }
    }
    f32x4 acc[kMaxTiles];
#pragma unroll
    for (int i = 0; i < kMaxTiles; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    const bool do_bias = a.dbias && blockIdx.y == 0;
    __syncthreads();

    const int64_t ohw = (int64_t)a.OH * a.OW, xhw = (int64_t)a.H * a.W;
    const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_block;
    int64_t t1 = t0 + a.tiles_per_block;
    if (t1 > a.ntiles) t1 = a.ntiles;
    const int per_img = a.tiles_x * a.tiles_y;

    for (int64_t tl = t0; tl < t1; ++tl) {
        const int n = (int)(tl / per_img);
        const int r = (int)(tl - (int64_t)n * per_img);
        const int oy0 = (r / a.tiles_x) * kTR, ox0 = (r % a.tiles_x) * kTC;
        // stage dy rows (BN backward rebuilt on load)
        for (int idx = tid; idx < Rpad * kTP; idx += kThreads) {
            const int row = idx >> 6, p = idx & 63;
            const int oy = oy0 + (p >> 4), ox = ox0 + (p & 15);
            float v = 0.f;
            if (row < a.R && oy < a.OH && ox < a.OW)
                v = vt_load(a.dy, cdy, n, row, ohw, (int64_t)oy * a.OW + ox);
            As[row * kAStride + p] = v;
        }
        // stage the input halo of the tile for channels [ci_lo, ci_hi)
        const int iy0 = oy0 * a.SH - a.PH, ix0 = ox0 * a.SW - a.PW;
        for (int idx = tid; idx < nci * halo; idx += kThreads) {
            const int cl = idx / halo, rem = idx - cl * halo;
            const int hr = rem / a.HC, hc = rem - hr * a.HC;
            const int iy = iy0 + hr, ix = ix0 + hc;
            float v = 0.f;
            if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
                v = vt_load(a.x, cx, n, ci_lo + cl, xhw, (int64_t)iy * a.W + ix);
            Xs[idx] = v;
        }
        __syncthreads();
        if (do_bias && tid < a.R) {
            const float* rowp = As + tid * kAStride;
#pragma unroll 8
            for (int p = 0; p < kTP; ++p) bsum += rowp[p];
        }
#pragma unroll 4
        for (int kq = kq_lo; kq < kq_hi; kq += 4) {
            if (!kactive) break;
            const int p = kq + kk;
            const int poff = (p >> 4) * a.SH * a.HC + (p & 15) * a.SW;
#pragma unroll
            for (int i = 0; i < kMaxTiles; ++i) {
                if (ksplit ? i == 0 : wave + 4 * i < ntile_blk) {  // wave-uniform
                    const float av = As[arow[i] + p];
                    const float bv = xoff[i] >= 0 ? Xs[xoff[i] + poff] : 0.f;
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }
    // k-split: waves kpart>0 hand their partial tile to wave (wave % ntile_blk) via LDS
    if (ksplit) {
        float* part = smem;  // the staging buffers are free now (loop ended on a barrier)
        if (kactive && kpart > 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[((wave - ntile_blk) * 4 + r) * 64 + lane] = acc[0][r];
        __syncthreads();
        if (kpart == 0)
            for (int j = 1; j < ks; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    acc[0][r] += part[((wave + (j - 1) * ntile_blk) * 4 + r) * 64 + lane];
    }
    // flush: lane holds D[row = rt*16 + kk*4 + r][col = c_lo + ct*16 + pl]
#pragma unroll
    for (int i = 0; i < kMaxTiles; ++i) {
        const int t = ksplit ? (i == 0 && kpart == 0 ? wave : 1 << 20) : wave + 4 * i;
        if (t >= ntile_blk) continue;
        const int rt = t / a.CTB, ct = t - rt * a.CTB;
        const int col = c_lo + ct * 16 + pl;
        if (col >= c_hi) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = rt * 16 + kk * 4 + r;
            if (row < a.R) atomicAdd(&a.dw[(int64_t)row * NCOL + col], acc[i][r]);
        }
    }
    if (do_bias && tid < a.R) atomicAdd(&a.dbias[tid], bsum);
}

int vt_channels(const isg_vtensor* v) {
    int c = 0;
    for (int i = 0; i < v->nseg; ++i) c += v->s[i].C;
    return c;
}

}  // namespace

int32_t isg_dense_conv_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x,
                             float* dw, float* dbias, hipStream_t st) {
    if (vt_channels(dy) != g->Co || vt_channels(x) != g->Ci)
        return isg_set_error(ISG_ERR_INVALID, "conv wgrad: channel mismatch");
    if (!dw) return isg_set_error(ISG_ERR_INVALID, "conv wgrad: dw is NULL");
    WgArgs a{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias;
    a.N = g->N; a.OH = g->OH; a.OW = g->OW; a.H = g->H; a.W = g->W;
    a.R = g->Co; a.Ci = g->Ci; a.KH = g->KH; a.KW = g->KW; a.SH = g->SH; a.SW = g->SW;
    a.PH = g->PH; a.PW = g->PW; a.DH = g->DH; a.DW = g->DW;
    const int KK = g->KH * g->KW;
    const int ncol = g->Ci * KK;
    const int CT = (ncol + 15) / 16;
    a.RT = (g->Co + 15) / 16;
    if (a.RT > 32) return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: %d rows > 512", g->Co);
    a.CTB = 32 / a.RT;
    if (a.CTB < 1) a.CTB = 1;
    if (a.CTB > CT) a.CTB = CT;
    if (a.RT * a.CTB > 4 * kMaxTiles)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: %d rows too many", g->Co);
    a.HR = (kTR - 1) * g->SH + (g->KH - 1) * g->DH + 1;
    a.HC = (kTC - 1) * g->SW + (g->KW - 1) * g->DW + 1;
    const int gy = (CT + a.CTB - 1) / a.CTB;
    int max_ci = 0;
    for (int by = 0; by < gy; ++by) {
        const int c_lo = by * a.CTB * 16;
        const int c_hi = std::min(ncol, c_lo + a.CTB * 16);
        max_ci = std::max(max_ci, (c_hi - 1) / KK + 1 - c_lo / KK);
    }
    const size_t lds = ((size_t)a.RT * 16 * kAStride + (size_t)max_ci * a.HR * a.HC) * sizeof(float);
    if (lds + 2 * ISG_MAX_CH * sizeof(ChanCoef) > 160 * 1024)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "conv wgrad: LDS %zu bytes too large", lds);
    a.tiles_x = (g->OW + kTC - 1) / kTC;
    a.tiles_y = (g->OH + kTR - 1) / kTR;
    a.ntiles = (int64_t)g->N * a.tiles_x * a.tiles_y;
    // blocks along pixels: enough to fill the chip, but every block adds its partial dW
    // with f32 atomics — cap the adders per address (contention) and the atomic bytes
    int64_t gx = (2048 + gy - 1) / gy;
    const int64_t nout = (int64_t)g->Co * ncol;
    gx = std::min<int64_t>(gx, nout < 1024 ? 128 : 512);
    if (gx > a.ntiles) gx = a.ntiles;
    if (gx < 1) gx = 1;
    a.tiles_per_block = (a.ntiles + gx - 1) / gx;
    gx = (a.ntiles + a.tiles_per_block - 1) / a.tiles_per_block;
    hipLaunchKernelGGL(wgrad_tiled_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(kThreads), lds, st, a);
    return isg_check_launch("wgrad_tiled_kernel");
}
