// Halo-tiled dense convolution forward for narrow outputs (Co <= 32) on
// v_mfma_f32_16x16x4_f32 — the stem (segment.py:23-26: 5x5 s2, 20->16 at full
// resolution, 60 % of the network's FLOPs), the 2x2 s2 down convs (:121), the dense 3x3
// (:242, :437), and the ConvTranspose2d input-gradients (8x8 s4 / 4x4 s2).
//
// A workgroup owns an output tile of THO x 32 pixels for all Co. Input channels are
// processed in chunks: the chunk's input halo ((THO-1)*S+(K-1)*D+1 rows x 31*S+(K-1)*D+1
// cols) is loaded ONCE (with the producer's BatchNorm/activation applied on load) into
// LDS, together with the chunk's weights; every (kh, kw) tap then reads the halo at a
// shifted offset. The generic implicit-GEMM path instead re-gathers every input element
// KH*KW times through the cache with per-element index arithmetic.
//
// MFMA maps (16x16x4 f32): A[i=co][k] = W (lane: co = l&15, k = l>>4),
// B[k][j=pixel] = halo (lane: k = l>>4, pixel = l&15), D lane holds co = (l>>4)*4+r.
#include "stage.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTW = 32;        // output tile width
constexpr int kKMax = 512;     // K entries per chunk (channels_in_chunk * KH * KW)
constexpr int kHaloMax = 6144; // floats of halo per chunk
constexpr int kMaxCi = 64;     // channel records per block

struct HaloArgs {
    isg_vtensor x;
    isg_sink out;
    const float* w;  // [Co][Ci][KH][KW]
    int N, Ci, H, W, Co, OH, OW, KH, KW, SH, SW, PH, PW, DH, DW;
    int HR, HC, cic;  // halo rows/cols, channels per chunk
    int tiles_x, tiles_y;
};

// sum over the 16 lanes of a DPP row (lanes sharing l>>4), result in every lane
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

template <int MT, int THO>
__global__ __launch_bounds__(kThreads) void halo_conv_kernel(HaloArgs a) {
    constexpr int G = THO / 2;  // 16-pixel groups per wave (THO*32 pixels / 16 / 4 waves)
    __shared__ float Xs[kHaloMax];
    __shared__ float Ws[MT * 16 * kKMax / 4 + 16];  // chunk weights [co][k] (k <= cic*KK)
    __shared__ int koff[kKMax];
    __shared__ ChT tab[kMaxCi];
    __shared__ float red[4][2][MT * 16];  // per-wave partials: fixed-order sum

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kk = lane >> 4, pl = lane & 15;
    const int KK = a.KH * a.KW;
    const int n = blockIdx.x / (a.tiles_x * a.tiles_y);
    const int tr = blockIdx.x - n * a.tiles_x * a.tiles_y;
    const int oy0 = (tr / a.tiles_x) * THO, ox0 = (tr % a.tiles_x) * kTW;
    const int iy0 = oy0 * a.SH - a.PH, ix0 = ox0 * a.SW - a.PW;
    const int hsz = a.HR * a.HC;
    const int wst = ((a.cic * KK + 3) & ~3) + 1;  // Ws row stride (odd), holds the k padding

    for (int c = tid; c < a.Ci; c += kThreads) tab[c] = ch_table_entry(a.x, c, a.H * a.W);
    for (int i = tid; i < MT * 16; i += kThreads)
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) red[wv][0][i] = red[wv][1][i] = 0.f;

    // per-lane pixel offsets inside the halo for each of the wave's groups
    int poff[G];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        const int p = (wave * G + gi) * 16 + pl;  // pixel index in tile, row-major 32 wide
        const int py = p >> 5, px = p & 31;
        poff[gi] = py * a.SH * a.HC + px * a.SW;
    }
    f32x4 acc[G][MT];
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[gi][m] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int npass = (a.HC + 63) >> 6;  // lane passes per halo row
    for (int c0 = 0; c0 < a.Ci; c0 += a.cic) {
        const int nc = min(a.cic, a.Ci - c0);
        const int K = nc * KK;
        const int Kp = (K + 3) & ~3;
        __syncthreads();  // previous chunk fully consumed (tab ready on the first pass)
        // halo: item = (channel, halo row, lane pass), wave-uniform; lane = column.
        // Groups of 8 items per wave with all loads in flight together.
        const int nitems = nc * a.HR * npass;
        for (int i0 = wave; i0 < nitems; i0 += 32) {
            float v[8], yv[8];
            bool ok[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int it = min(i0 + 4 * u, nitems - 1);
                const int cr = it / npass, pass = it - cr * npass;
                const int cl = cr / a.HR, hr = cr - cl * a.HR;
                const ChT c = tab[c0 + cl];
                const int iy = iy0 + hr, hc = pass * 64 + lane, ix = ix0 + hc;
                ok[u] = hc < a.HC && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
                const int o = ok[u] ? iy * a.W + ix : 0;
                v[u] = gld(c.p, n * c.ns + o);
                yv[u] = gld(c.y, n * c.yns + o);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int it = i0 + 4 * u;
                if (it < nitems) {
                    const int cr = it / npass, pass = it - cr * npass;
                    const int cl = cr / a.HR, hr = cr - cl * a.HR;
                    const ChT c = tab[c0 + cl];
                    const int hc = pass * 64 + lane;
                    if (hc < a.HC)
                        Xs[cl * hsz + hr * a.HC + hc] = ok[u] ? ch_xform(c.xf, c.act, c.k, v[u], yv[u]) : 0.f;
                }
            }
        }
        for (int idx = tid; idx < MT * 16 * Kp; idx += kThreads) {
            const int co = idx / Kp, k = idx - co * Kp;
            Ws[co * wst + k] = (co < a.Co && k < K) ? gld(a.w, ((int64_t)co * a.Ci + c0) * KK + k) : 0.f;
        }
        for (int k = tid; k < Kp; k += kThreads) {
            int o = 0;  // padding k: weight 0, any valid halo offset
            if (k < K) {
                const int cl = k / KK, t = k - cl * KK;
                const int kh = t / a.KW, kw = t - kh * a.KW;
                o = cl * hsz + kh * a.DH * a.HC + kw * a.DW;
            }
            koff[k] = o;
        }
        __syncthreads();
#pragma unroll 2
        for (int k0 = 0; k0 < Kp; k0 += 4) {
            const int k = k0 + kk;
            const int o = koff[k];
            float av[MT];
#pragma unroll
            for (int m = 0; m < MT; ++m) av[m] = Ws[(m * 16 + pl) * wst + k];
#pragma unroll
            for (int gi = 0; gi < G; ++gi) {
                const float bv = Xs[o + poff[gi]];
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    acc[gi][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv, acc[gi][m], 0, 0, 0);
            }
        }
    }

    // ---- epilogue: bias, store (64-B rows), BN statistics ---------------------------
    const isg_sink& o = a.out;
    const int64_t ohw = (int64_t)a.OH * a.OW;
    float s0[MT][4], s1[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            s0[m][r] = 0.f;
            s1[m][r] = 0.f;
        }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
        const int p = (wave * G + gi) * 16 + pl;
        const int oy = oy0 + (p >> 5), ox = ox0 + (p & 31);
        const bool pv = oy < a.OH && ox < a.OW;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = m * 16 + kk * 4 + r;
                if (co < a.Co && pv) {
                    float v = acc[gi][m][r];
                    if (o.bias) v += o.bias[co];
                    o.p[(int64_t)n * o.n_stride + (int64_t)co * ohw + (int64_t)oy * a.OW + ox] = v;
                    s0[m][r] += v;
                    s1[m][r] += v * v;
                }
            }
    }
    if (o.stats) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float t0 = row16_sum(s0[m][r]);
                const float t1 = row16_sum(s1[m][r]);
                const int co = m * 16 + kk * 4 + r;
                if (pl == 0 && co < a.Co) {
                    red[wave][0][co] = t0;
                    red[wave][1][co] = t1;
                }
            }
        __syncthreads();
        double* sp = rep_ptr(o.stats, 4 * o.C);
        for (int co = tid; co < a.Co; co += kThreads) {
            const float t0 = ((red[0][0][co] + red[1][0][co]) + red[2][0][co]) + red[3][0][co];
            const float t1 = ((red[0][1][co] + red[1][1][co]) + red[2][1][co]) + red[3][1][co];
            atomicAdd(&sp[co], (double)t0);
            atomicAdd(&sp[o.C + co], (double)t1);
        }
    }
}

}  // namespace

// Returns 1 if handled, 0 if the shape is not for this kernel, <0 on error.
int32_t isg_halo_conv_fwd(const isg_conv_geom* g, const isg_vtensor* x, const float* w,
                          const isg_sinks* out, hipStream_t st) {
    if (g->groups != 1 || g->Co > 32 || g->Ci > kMaxCi || out->nsink != 1 ||
        out->s[0].mode != ISG_SINK_STORE ||
        (g->KH == 1 && g->KW == 1 && g->SH == 1 && g->SW == 1))
        return 0;
    const int KK = g->KH * g->KW;
    if (KK > kKMax) return 0;
    int tho = 8;
    auto halo_rows = [&](int t) { return (t - 1) * g->SH + (g->KH - 1) * g->DH + 1; };
    const int HC = (kTW - 1) * g->SW + (g->KW - 1) * g->DW + 1;
    while (tho > 2 && halo_rows(tho) * HC > kHaloMax / 2) tho /= 2;
    const int HR = halo_rows(tho);
    if (HR * HC > kHaloMax) return 0;
    HaloArgs a{};
    a.x = *x; a.out = out->s[0]; a.w = w;
    a.N = g->N; a.Ci = g->Ci; a.H = g->H; a.W = g->W; a.Co = g->Co; a.OH = g->OH; a.OW = g->OW;
    a.KH = g->KH; a.KW = g->KW; a.SH = g->SH; a.SW = g->SW; a.PH = g->PH; a.PW = g->PW;
    a.DH = g->DH; a.DW = g->DW; a.HR = HR; a.HC = HC;
    const int mt = g->Co <= 16 ? 1 : 2;
    int cic = kHaloMax / (HR * HC);
    auto wfit = [&](int c) {  // padded K fits koff and the weight chunk fits Ws
        const int kp = (c * KK + 3) & ~3;
        return kp <= kKMax && mt * 16 * (kp + 1) <= mt * 16 * kKMax / 4 + 16;
    };
    while (cic > 1 && !wfit(cic)) --cic;
    cic = std::max(1, std::min(cic, g->Ci));
    a.cic = cic;
    a.tiles_x = (g->OW + kTW - 1) / kTW;
    a.tiles_y = (g->OH + tho - 1) / tho;
    dim3 grid((unsigned)(g->N * a.tiles_x * a.tiles_y));
#define HALO_LAUNCH(MT, THO) \
    hipLaunchKernelGGL((halo_conv_kernel<MT, THO>), grid, dim3(kThreads), 0, st, a)
    if (mt == 1) {
        if (tho == 8) HALO_LAUNCH(1, 8);
        else if (tho == 4) HALO_LAUNCH(1, 4);
        else HALO_LAUNCH(1, 2);
    } else {
        if (tho == 8) HALO_LAUNCH(2, 8);
        else if (tho == 4) HALO_LAUNCH(2, 4);
        else HALO_LAUNCH(2, 2);
    }
#undef HALO_LAUNCH
    const int32_t e = isg_check_launch("halo_conv_kernel");
    return e ? e : 1;
}
