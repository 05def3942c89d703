// Tap-table halo convolution on v_mfma_f32_16x16x4_f32: every dense spatial conv of the
// reference with at most 48 GEMM rows, forward AND input gradient.
//
//   forward : the stem 5x5 s2 convs (segment.py:23-26; 60 % of the network's FLOPs), the
//             2x2 s2 down convs (:121), the dense 3x3 of BottleneckDim (:242) and the
//             head 3x3 (:437);
//   dgrad   : the same convs' input gradients (stride-1 phases of dy).
//
// GEMM view: out[m][pix] = sum_{c, tap} W[m][c][tap] * src[c][pos(pix, tap)]. A stride-S
// input gradient splits into S*S PHASES: the output pixels (S*ty+ph, S*tx+pw) of one
// phase see only the taps with (ph + P - kh*D) % S == 0, each a stride-1 shift of dy —
// no lane multiplies a structural zero.
//
// Persistent workgroups walk (tile, 4-channel chunk) work items. Per workgroup, once: the
// tap tables of every phase, the channel records, the sink rows and ALL weights go to
// LDS. Per item: wave w stages channel 4*chunk + w of the tile's source halo, one halo
// ROW per load instruction (wave-uniform row, lanes = columns; for a stride-2 source
// each lane loads a column PAIR and splits it into the even / odd column planes, so the
// 16 lanes of a pixel group always read 16 consecutive LDS words). The row's bounds are
// scalar; the producer's BatchNorm / activation / BatchNorm-backward is applied on the
// way into LDS. The NEXT item's loads are issued into registers before this item's
// MFMAs. Each tap is one wave-uniform LDS offset: the MFMA loop is ds_read + MFMA.
//
// MFMA lane maps (16x16x4 f32): A[i=m][k] = W (lane: m = l&15, k = l>>4 = channel in
// the chunk), B[k][j] = halo (lane: k = l>>4, pixel j = l&15), D lane: m = (l>>4)*4+r.
#include <cstdio>

#include "stage.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxTaps = 64;  // KH*KW
constexpr int kMaxPh = 4;     // dgrad phases (stride <= 2)
constexpr int kTapTab = kMaxTaps + 3 * kMaxPh;  // per-phase tap lists padded to 4
// staged halo rows per wave per chunk (registers). 20 was tried: halo tiles of 17-20 rows
// passed every single-kernel parity test yet left 5-14 % L2 errors in Segment(20) 128^2
// gradients (root cause open; the 16-row cap is exact to 3e-5)
constexpr int kPF = 16;
constexpr int kMaxM = 48;
constexpr int kMaxC = 64;
constexpr int kLdsMax = 64 * 1024;

struct TapGeo {
    int KH, KW, SH, SW, PH, PW, DH, DW;
    int dgrad;
};

// Visit the taps of phase (ph, pw): f(i, by, bx, wofs) with the source offset (by, bx)
// relative to (my*ty, mx*tx) and the weight offset kh*KW + kw. Forward has one phase.
template <class F>
__host__ __device__ inline int for_each_tap(const TapGeo& q, int ph, int pw, F&& f) {
    int n = 0;
    for (int kh = 0; kh < q.KH; ++kh) {
        int by;
        if (q.dgrad) {
            const int r = ph + q.PH - kh * q.DH;
            if (((r % q.SH) + q.SH) % q.SH) continue;
            by = r / q.SH;  // exact
        } else {
            by = kh * q.DH - q.PH;
        }
        for (int kw = 0; kw < q.KW; ++kw) {
            int bx;
            if (q.dgrad) {
                const int r = pw + q.PW - kw * q.DW;
                if (((r % q.SW) + q.SW) % q.SW) continue;
                bx = r / q.SW;
            } else {
                bx = kw * q.DW - q.PW;
            }
            f(n, by, bx, kh * q.KW + kw);
            ++n;
        }
    }
    return n;
}

struct TapArgs {
    isg_vtensor src;  // gathered operand: x (forward) or dy (dgrad)
    isg_sinks out;
    const float* w;
    int64_t wm, wc;   // weight index = m*wm + c*wc + (kh*KW + kw)
    TapGeo q;
    int N, C, M, KK;
    int SrcH, SrcW;   // source plane
    int DstH, DstW;   // destination plane
    int OutH, OutW;   // dgrad: conv input dims (phase grids derive from them); fwd: OH, OW
    int BY, BX, tiles_x, tiles_y, nph, ntiles;  // ntiles over all phases and images
    int nchunk;       // chunks of 4 channels (one per wave)
    int HR, HCu, PS, RS, CHS;  // halo rows, units per row (cols, or col pairs), LDS layout
    int ws_floats;    // weights in LDS: [Cp][WCS] with WCS >= (KK+1)*MP (row KK zero)
    int WCS;          // per-channel weight stride (== 16 mod 32: conflict-free quads)
    uint32_t m_img, m_tpi, m_tx;  // ceil(2^32/d) for d = N*tpi, tpi, tiles_x (exact, x*d < 2^32;
                                  // 0 for d == 1)
};

template <int MT, int G, bool YB, bool PAIR>
__global__ __launch_bounds__(kThreads) void tap_conv_kernel(TapArgs a) {
    constexpr int MP = 16 * MT;
    constexpr int MX = PAIR ? 2 : 1;  // source columns per output column step
    extern __shared__ float lds[];
    float* const Ws = lds;
    float* const Xs = lds + a.ws_floats;
    __shared__ ChT tab[kMaxC];
    __shared__ SinkRow ri[kMaxM];
    __shared__ __attribute__((aligned(16))) int toff[kTapTab];
    __shared__ __attribute__((aligned(16))) int twof[kTapTab];
    __shared__ int p_beg[kMaxPh], p_n[kMaxPh], p_miny[kMaxPh], p_minx[kMaxPh];
    __shared__ float red[4][3][kMaxM];

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kq = lane >> 4, pl = lane & 15;
    const int dg = a.q.dgrad;
    const int my = dg ? 1 : a.q.SH;

    // ---- per-workgroup prologue: tap tables of every phase, channel records, sink rows,
    //      all weights (zero row KK serves the padded taps)
    if (tid == 0) {
        int beg = 0;
        for (int p = 0; p < a.nph; ++p) {
            const int ph = dg ? p / a.q.SW : 0, pw = dg ? p % a.q.SW : 0;
            int miny = 1 << 20, minx = 1 << 20;
            const int nt = for_each_tap(a.q, ph, pw, [&](int, int by, int bx, int) {
                miny = min(miny, by);
                minx = min(minx, bx);
            });
            if (MX == 2) minx &= ~1;  // column pairs start even (an odd first tap: +1 column)
            for_each_tap(a.q, ph, pw, [&](int i, int by, int bx, int wofs) {
                const int cy = by - miny, cx = bx - minx;
                toff[beg + i] = cy * a.RS + (cx % MX) * a.PS + cx / MX;
                twof[beg + i] = wofs * MP;
            });
            const int ntp = (nt + 3) & ~3;
            for (int i = nt; i < ntp; ++i) {
                toff[beg + i] = 0;
                twof[beg + i] = a.KK * MP;  // zero weight row
            }
            p_beg[p] = beg;
            p_n[p] = nt;  // taps; the table is padded to 4 for the int4 reads
            p_miny[p] = nt ? miny : 0;
            p_minx[p] = nt ? minx : 0;
            beg += ntp;
        }
    }
    for (int c = tid; c < a.C; c += kThreads) tab[c] = ch_table_entry(a.src, c, (int64_t)a.SrcH * a.SrcW);
    for (int r = tid; r < kMaxM; r += kThreads) {
        SinkRow q = {};
        q.mode = -1;
        if (r < a.M) q = sink_row(a.out, r, (int64_t)a.DstH * a.DstW);
        ri[r] = q;
    }
    coop_gather<8>(Ws, a.ws_floats, tid, kThreads, a.w, [&](int f) {
        const int c = f / a.WCS, rem = f - c * a.WCS;
        const int k = rem / MP, m = rem - k * MP;
        return (m < a.M && c < a.C && k < a.KK) ? m * a.wm + c * a.wc + k : -1;
    });
    __syncthreads();

    // per-group pixel (16 consecutive pixels of the tile in row-major order) and LDS base
    const int tpx = a.BY * a.BX;
    int xbase[G], gpix[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int q = (wave * G + g) * 16 + pl;
        const int qq = q < tpx ? q : 0;
        const int tyl = qq / a.BX, txl = qq - tyl * a.BX;
        xbase[g] = kq * a.CHS + my * tyl * a.RS + txl;
        gpix[g] = q < tpx ? (tyl << 16) | txl : -1;
    }
    const int wlane = kq * a.WCS + pl;  // lane part of the weight index
    const uint32_t plane_bytes = (uint32_t)a.SrcH * a.SrcW * 4u;

    // ---- work items: (tile, chunk), tiles strided over the grid -------------------------
    const int tpi = a.tiles_x * a.tiles_y;
    auto tile_geo = [&](int tile, int& p, int& n, int& ty0, int& tx0, bool& live) {
        // magic 0 encodes a divisor of 1
        auto qdiv = [](int x, uint32_t m) { return m ? (int)__umulhi((uint32_t)x, m) : x; };
        p = qdiv(tile, a.m_img);
        const int r = tile - p * a.N * tpi;
        n = qdiv(r, a.m_tpi);
        const int tr = r - n * tpi;
        const int tyi = qdiv(tr, a.m_tx);
        ty0 = tyi * a.BY;
        tx0 = (tr - tyi * a.tiles_x) * a.BX;
        const int ph = dg ? p / a.q.SW : 0, pw = dg ? p % a.q.SW : 0;
        const int TH = dg ? (a.OutH - ph + a.q.SH - 1) / a.q.SH : a.OutH;
        const int TW = dg ? (a.OutW - pw + a.q.SW - 1) / a.q.SW : a.OutW;
        live = ty0 < TH && tx0 < TW;
    };

    // staging registers: one halo row per entry (lane = column or column pair)
    typedef float v2f __attribute__((ext_vector_type(2)));
    v2f v[kPF], yv[kPF];
    uint32_t rowok = 0;  // wave-uniform bitmask over halo rows
    bool colok = false;  // this lane's column (pair) inside the source
    auto load_item = [&](int tile, int ch) {
        int p, n, ty0, tx0;
        bool live;
        tile_geo(tile, p, n, ty0, tx0, live);
        const int sy0 = my * ty0 + p_miny[p], sx0 = MX * tx0 + p_minx[p];
        const int c = ch * 4 + wave;
        const ChT t = tab[min(c, a.C - 1)];
        const bool cv = c < a.C;
        const float* const xp = uniform_ptr(t.p + (int64_t)n * t.ns);
        const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)xp, (short)0, (int)plane_bytes, 0x00020000);
        const float* const yp = YB ? uniform_ptr(t.y + (int64_t)n * t.yns) : xp;
        const auto yr = __builtin_amdgcn_make_buffer_rsrc((void*)yp, (short)0, (int)plane_bytes, 0x00020000);
        const int ix = sx0 + MX * lane;
        colok = cv && lane < a.HCu && ix >= 0 && ix < a.SrcW;
        const uint32_t voff = colok ? (uint32_t)ix * 4u : 0x80000000u;
        rowok = 0;
#pragma unroll
        for (int r = 0; r < kPF; ++r) {
            if (r < a.HR) {
                const int iy = sy0 + r;
                if ((unsigned)iy < (unsigned)a.SrcH) {
                    rowok |= 1u << r;
                    const uint32_t o = colok ? voff + (uint32_t)iy * (uint32_t)a.SrcW * 4u : voff;
                    if constexpr (PAIR) {
                        // whole-vector bit_cast: element access on the builtin's result
                        // lowers to ONE dword load duplicated (hipcc, ROCm 7.2)
                        v[r] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(xr, o, 0, 0));
                        if constexpr (YB)
                            yv[r] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(yr, o, 0, 0));
                    } else {
                        v[r][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o, 0, 0));
                        if constexpr (YB)
                            yv[r][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, o, 0, 0));
                    }
                }
            }
        }
    };
    auto store_item = [&](int ch) {
        const int c = ch * 4 + wave;
        const ChT t = tab[min(c, a.C - 1)];
        float* const xs = Xs + wave * a.CHS + lane;
        if (lane < a.PS) {
#pragma unroll
            for (int r = 0; r < kPF; ++r) {
                if (r < a.HR) {
                    const bool ok = ((rowok >> r) & 1u) && colok;
                    float x0 = 0.f, x1 = 0.f;
                    if (ok) {
                        x0 = ch_xform(t.xf, t.act, t.k, v[r][0], YB ? yv[r][0] : v[r][0]);
                        if constexpr (PAIR) x1 = ch_xform(t.xf, t.act, t.k, v[r][1], YB ? yv[r][1] : v[r][1]);
                    }
                    xs[r * a.RS] = x0;
                    if constexpr (PAIR) xs[r * a.RS + a.PS] = x1;
                }
            }
        }
    };

    f32x4 acc[G][MT];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[g][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    float s0[MT][4], s1[MT][4], s2[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) s0[m][r] = s1[m][r] = s2[m][r] = 0.f;

    auto next_live = [&](int tile) {
        for (; tile < a.ntiles; tile += gridDim.x) {
            int p, n, ty0, tx0;
            bool live;
            tile_geo(tile, p, n, ty0, tx0, live);
            if (live) break;
        }
        return tile;
    };
    int tile = next_live(blockIdx.x), ch = 0;
    if (tile < a.ntiles) load_item(tile, 0);
    while (tile < a.ntiles) {
        __syncthreads();  // Xs free
        store_item(ch);
        __syncthreads();
        // prefetch the next item while this one computes
        int ntile = tile, nch = ch + 1;
        if (nch == a.nchunk) {
            nch = 0;
            ntile = next_live(tile + gridDim.x);
        }
        if (ntile < a.ntiles) load_item(ntile, nch);

        int p, n, ty0, tx0;
        bool live;
        tile_geo(tile, p, n, ty0, tx0, live);
        const int tb = p_beg[p], tn = p_n[p];
        const float* const wch = Ws + ch * 4 * a.WCS + wlane;
        const int tn4 = tn & ~3;
        for (int t0 = 0; t0 < tn4; t0 += 4) {
            const int4 to = *reinterpret_cast<const int4*>(&toff[tb + t0]);
            const int4 tw = *reinterpret_cast<const int4*>(&twof[tb + t0]);
            const int tos[4] = {to.x, to.y, to.z, to.w}, tws[4] = {tw.x, tw.y, tw.z, tw.w};
            float av[4][MT], bv[4][G];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int m = 0; m < MT; ++m) av[u][m] = wch[tws[u] + m * 16];
#pragma unroll
                for (int g = 0; g < G; ++g) bv[u][g] = Xs[xbase[g] + tos[u]];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int m = 0; m < MT; ++m)
                        acc[g][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][m], bv[u][g], acc[g][m], 0, 0, 0);
        }
        for (int t = tn4; t < tn; ++t) {  // remainder taps, one at a time
            const int to = toff[tb + t], tw = twof[tb + t];
            float av[MT], bv[G];
#pragma unroll
            for (int m = 0; m < MT; ++m) av[m] = wch[tw + m * 16];
#pragma unroll
            for (int g = 0; g < G; ++g) bv[g] = Xs[xbase[g] + to];
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    acc[g][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[g], acc[g][m], 0, 0, 0);
        }

        if (ch == a.nchunk - 1) {  // tile complete: epilogue
            const int ph = dg ? p / a.q.SW : 0, pw = dg ? p % a.q.SW : 0;
            const int TH = dg ? (a.OutH - ph + a.q.SH - 1) / a.q.SH : a.OutH;
            const int TW = dg ? (a.OutW - pw + a.q.SW - 1) / a.q.SW : a.OutW;
            const int dmy = dg ? a.q.SH : 1, dmx = dg ? a.q.SW : 1;
            int64_t gp[G];
            bool gv[G];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int ty = ty0 + (gpix[g] >> 16), tx = tx0 + (gpix[g] & 0xFFFF);
                gv[g] = gpix[g] >= 0 && ty < TH && tx < TW;
                gp[g] = (int64_t)(dmy * ty + ph) * a.DstW + (dmx * tx + pw);
            }
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m * 16 + kq * 4 + r;
                    if (row < a.M) {
                        const SinkRow q = ri[row];
#pragma unroll
                        for (int g = 0; g < G; ++g) {
                            if (gv[g]) {
                                float t0 = 0.f, t1 = 0.f, t2 = 0.f;
                                sink_row_apply(q, n, gp[g], acc[g][m][r], t0, t1, t2);
                                s0[m][r] += t0;
                                s1[m][r] += t1;
                                s2[m][r] += t2;
                            }
                        }
                    }
#pragma unroll
                    for (int g = 0; g < G; ++g) acc[g][m][r] = 0.f;
                }
        }
        tile = ntile;
        ch = nch;
    }

    // ---- per-workgroup BN partial sums: waves in fixed order, one atomic per row ---------
    if (sinks_need_red(a.out)) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float t0 = dpp_row16_sum(s0[m][r]);
                const float t1 = dpp_row16_sum(s1[m][r]);
                const float t2 = dpp_row16_sum(s2[m][r]);
                const int row = m * 16 + kq * 4 + r;
                if (pl == 0 && row < kMaxM) {
                    red[wave][0][row] = t0;
                    red[wave][1][row] = t1;
                    red[wave][2][row] = t2;
                }
            }
        __syncthreads();
        for (int row = tid; row < a.M; row += kThreads) {
            float r3[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) r3[j] = ((red[0][j][row] + red[1][j][row]) + red[2][j][row]) + red[3][j][row];
            sink_row_flush(a.out, row, r3[0], r3[1], r3[2]);
        }
    }
}

template <int MT, int G, bool YB, bool PAIR>
int32_t tap_launch(const TapArgs& a, size_t lds, hipStream_t st) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
    }
    auto k = tap_conv_kernel<MT, G, YB, PAIR>;
    if (lds > 48 * 1024 &&
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return isg_check_launch("tap_conv_kernel: dynamic LDS");
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kThreads, lds) != hipSuccess || occ < 1) occ = 1;
    const int grid = std::max(1, std::min(a.ntiles, occ * cus));
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kThreads), lds, st, a);
    return isg_check_launch("tap_conv_kernel");
}

template <int MT, int G>
int32_t tap_launch_v(const TapArgs& a, size_t lds, bool yb, bool pair, hipStream_t st) {
    if (pair) return yb ? tap_launch<MT, G, true, true>(a, lds, st) : tap_launch<MT, G, false, true>(a, lds, st);
    return yb ? tap_launch<MT, G, true, false>(a, lds, st) : tap_launch<MT, G, false, false>(a, lds, st);
}

template <int MT>
int32_t tap_launch_g(const TapArgs& a, size_t lds, int G, bool yb, bool pair, hipStream_t st) {
    if (G == 1) return tap_launch_v<MT, 1>(a, lds, yb, pair, st);
    if (G == 2) return tap_launch_v<MT, 2>(a, lds, yb, pair, st);
    return tap_launch_v<MT, 4>(a, lds, yb, pair, st);
}

}  // namespace

// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
//   dgrad = 0: out[Co] = conv(x)      src = x  (C = Ci), rows M = Co
//   dgrad = 1: out[Ci] = conv^T(dy)   src = dy (C = Co), rows M = Ci, weight [Co][Ci][KH][KW]
int32_t isg_tap_conv(const isg_conv_geom* g, const isg_vtensor* src, const float* w,
                     const isg_sinks* out, bool dgrad, hipStream_t st) {
    if (g->groups != 1) return 0;
    TapArgs a{};
    a.q = TapGeo{g->KH, g->KW, g->SH, g->SW, g->PH, g->PW, g->DH, g->DW, dgrad ? 1 : 0};
    const int KK = g->KH * g->KW;
    if (KK > kMaxTaps) return 0;
    a.KK = KK;
    a.M = dgrad ? g->Ci : g->Co;
    a.C = dgrad ? g->Co : g->Ci;
    if (a.M > kMaxM || a.C > kMaxC) return 0;
    const int mx = dgrad ? 1 : g->SW, my = dgrad ? 1 : g->SH;
    a.nph = dgrad ? g->SH * g->SW : 1;
    if (a.nph > kMaxPh || mx > 2) return 0;
    a.src = *src; a.out = *out; a.w = w; a.N = g->N;
    const int64_t wci = g->w_ci > 0 ? g->w_ci : g->Ci;  // weight input channels (isg.h)
    a.wm = dgrad ? KK : wci * KK;
    a.wc = dgrad ? wci * KK : KK;
    a.SrcH = dgrad ? g->OH : g->H; a.SrcW = dgrad ? g->OW : g->W;
    a.DstH = dgrad ? g->H : g->OH; a.DstW = dgrad ? g->W : g->OW;
    a.OutH = dgrad ? g->H : g->OH; a.OutW = dgrad ? g->W : g->OW;
    if ((int64_t)a.SrcH * a.SrcW * 4 >= (1ll << 31)) return 0;  // 32-bit buffer offsets
    // tap extents over all phases (the LDS layout serves the widest)
    int ext_y = 0, ext_x = 0;
    for (int p = 0; p < a.nph; ++p) {
        int y0 = 1 << 20, y1 = -(1 << 20), x0 = 1 << 20, x1 = -(1 << 20);
        const int nt = for_each_tap(a.q, p / g->SW, p % g->SW, [&](int, int by, int bx, int) {
            y0 = std::min(y0, by); y1 = std::max(y1, by);
            x0 = std::min(x0, bx); x1 = std::max(x1, bx);
        });
        if (!nt) continue;
        ext_y = std::max(ext_y, y1 - y0);
        // a stride-2 source is staged in column pairs from an even origin: an odd first
        // tap column (the k4 s2 p1 ConvTranspose input gradients) widens the halo by one
        ext_x = std::max(ext_x, x1 - (mx == 2 ? (x0 & ~1) : x0));
    }
    if (mx == 2 && a.SrcW % 2) return 0;
    const int THm = dgrad ? (g->H + g->SH - 1) / g->SH : g->OH;
    const int TWm = dgrad ? (g->W + g->SW - 1) / g->SW : g->OW;
    const int mt = (a.M + 15) / 16;
    const int Cp = (a.C + 3) & ~3;
    a.WCS = (KK + 1) * 16 * mt;
    a.WCS += ((16 - a.WCS % 32) + 32) % 32;
    a.ws_floats = Cp * a.WCS;
    // Tile candidates (BX, BY) with BX*BY <= 64*G pixels (G groups of 16 per wave, G in
    // 4, 2, 1): the even split of the output width under the 64-lane halo-row limit, and
    // the power-of-two widths 32 / 16 (exact 64*G tiles). Cost = padded pixels (column
    // overhang + idle group lanes) + halo overfetch; at least 512 tiles when possible.
    const int bxmax = mx == 1 ? 64 - ext_x : (128 - ext_x - 1) / 2 + 1;
    if (bxmax < 8) return 0;
    int BX = 0, BY = 0, G = 0, tiles_x = 0;
    double best_cost = 1e30;
    bool best_many = false;
    int64_t best_tiles = 0;
    {
        const int tx_even = (TWm + bxmax - 1) / bxmax;
        const int bx_even = (TWm + tx_even - 1) / tx_even;
        for (int bx : {bx_even, 32, 16}) {
            if (bx > bxmax || bx < 8) continue;
            const int HC = mx * (bx - 1) + ext_x + 1;
            const int hcu = (HC + mx - 1) / mx;
            if (hcu > 64) continue;
            const int tx = (TWm + bx - 1) / bx;
            for (int gg : {4, 2, 1}) {
                const int by = std::max(1, 64 * gg / bx);
                if (by * bx > 64 * gg) continue;
                const int HR = my * (by - 1) + ext_y + 1;
                int CHS = HR * mx * hcu;
                CHS += ((16 - CHS % 32) + 32) % 32;
                if (HR > kPF || (size_t)(a.ws_floats + 4 * CHS) * 4 > kLdsMax) continue;
                const int ty = (THm + by - 1) / by;
                const int64_t tiles = (int64_t)g->N * ty * tx * a.nph;
                // work ~ padded pixels (64*G per tile) plus the staged halo per tile
                const double cost = (double)tiles * (64.0 * gg + 0.25 * HR * hcu * mx);
                const bool many = tiles >= 512;
                // below 512 tiles the chip is under-filled: more (smaller) tiles first
                // (the 48->16 2x2 s2 conv at 128^2 took 39 us on 32 tiles of 256 pixels)
                const bool more = !many && !best_many && tiles > best_tiles;
                const bool same = many == best_many && (many || tiles == best_tiles);
                if ((many && !best_many) || more || (same && cost < best_cost)) {
                    best_tiles = tiles;
                    best_cost = cost;
                    best_many = many;
                    BX = bx; BY = by; G = gg; tiles_x = tx;
                }
            }
        }
    }
    if (BX) {
        const int HC = mx * (BX - 1) + ext_x + 1;
        a.HCu = (HC + mx - 1) / mx;
        a.PS = a.HCu;
        a.RS = mx * a.PS;
    }
    if (!BY) return 0;
    a.BY = BY; a.BX = BX;
    a.HR = my * (BY - 1) + ext_y + 1;
    a.CHS = a.HR * a.RS;
    a.CHS += ((16 - a.CHS % 32) + 32) % 32;
    a.nchunk = (a.C + 3) / 4;
    a.tiles_x = tiles_x;
    a.tiles_y = (THm + BY - 1) / BY;
    a.ntiles = g->N * a.tiles_x * a.tiles_y * a.nph;
    const int64_t tpi = (int64_t)a.tiles_x * a.tiles_y;
    if ((int64_t)a.ntiles * g->N * tpi >= (1ll << 32)) return 0;  // magic-division range
    auto magic = [](int64_t d) { return d == 1 ? 0u : (uint32_t)(((1ull << 32) + d - 1) / d); };
    a.m_img = magic(g->N * tpi);
    a.m_tpi = magic(tpi);
    a.m_tx = magic(a.tiles_x);
    bool yb = false;
    for (int i = 0; i < src->nseg; ++i) yb |= src->s[i].xform == ISG_XF_BN_BWD;
    const size_t lds = (size_t)(a.ws_floats + 4 * a.CHS) * sizeof(float);
    const bool pair = mx == 2;
    int32_t e;
    if (mt == 1) e = tap_launch_g<1>(a, lds, G, yb, pair, st);
    else if (mt == 2) e = tap_launch_g<2>(a, lds, G, yb, pair, st);
    else e = tap_launch_g<3>(a, lds, G, yb, pair, st);
    return e ? e : 1;
}
