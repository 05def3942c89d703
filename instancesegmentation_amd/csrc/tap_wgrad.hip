// Weight gradient of the narrow dense spatial convs on v_mfma_f32_16x16x4_f32: the stem
// 5x5 s2 convs (segment.py:23-26; 60 % of the network's FLOPs and the largest single
// kernel of the train step), the dense 3x3 of BottleneckDim (:242), the head 3x3 (:437)
// and the 2x2 s2 down convs (:121) — every dense conv with at most 16 output channels,
// source stride 1 or 2 and at most 32 taps.
//
//   dW[co][ci][kh][kw] = sum_{n,oy,ox} dy[co][n][oy][ox] * x[ci][n][S*oy - P + kh*D][...]
//
// GEMM: rows i = co (16), columns j = (ci of a 4-channel chunk, tap), reduction over the
// output pixels in steps of 4 along an output row. blockIdx.y = the channel chunk;
// persistent workgroups walk 4 x BX output tiles (wave w owns tile row w). Per tile the
// workgroup stages the chunk's input halo (a stride-2 source as even / odd column planes,
// the producer's BatchNorm + activation applied on load; wave w stages channel
// 4*chunk + w) and the tile's dy rows (BatchNorm backward rebuilt on load; wave w stages
// tile row w of all 16 rows); the NEXT tile's loads are issued into registers before
// this tile's MFMAs. Each column's (channel, tap) halo offset is a per-lane constant and
// the pixel step a wave-uniform one, so the MFMA loop is one ds_read per MFMA plus one dy
// read per step shared by the NT column tiles. Accumulators live across all of a
// workgroup's tiles; one f32 atomic per dW element per workgroup goes to one of the
// ISG_WREP replicas.
//
// MFMA lane maps (16x16x4 f32): A[i=co][k=pixel] = dy (lane: co = l&15, pixel = l>>4),
// B[k][j] = halo (lane: pixel = l>>4, column j = l&15), D lane: co = (l>>4)*4+r, j = l&15.
#include "stage.h"

#include <cstring>
#include <mutex>
#include <vector>

namespace {

constexpr int kThreads = 256;
constexpr int kBY = 4;      // tile rows = waves
constexpr int kPF = 16;     // staged halo rows per wave (registers)
constexpr int kMaxNT = 8;   // column tiles per chunk (4 channels x taps <= 128)
constexpr int kMaxC = 64;

struct TwArgs {
    isg_vtensor dy;   // N x Co x OH x OW (Co <= 16)
    isg_vtensor x;    // N x C x H x W
    double* dw;        // [Co][C][KH][KW], replica r at dw + r*rep_stride
    double* dbias;     // [Co] or NULL
    int64_t rep_stride;
    int nrep;
    int N, C, Co, H, W, OH, OW, KH, KW, SH, SW, PH, PW, DH, DW, KK;
    int WC;  // the weight's input channels (isg_conv_geom.w_ci; == C but for the keypoint stem)
    int BX, tiles_x, tiles_y, ntiles;
    int HR, HCu, PS, RS, CHS, DQ;  // halo rows / units / LDS layout; dy LDS row stride
    uint32_t m_tpi, m_tx;          // magic divisors (0 = divide by 1)
    // column tile t, lane pl: channel pl>>2 of the chunk, tap gtap[t][pl&3] (-1: padding,
    // reads the slot-0 tap's address, result discarded). Taps are grouped so that the 32
    // lanes of a ds_read_b32 group hit 32 distinct banks (host: tw_layout).
    int8_t gtap[8][4];
};

template <int NT, bool YB, bool PAIR>
__global__ __launch_bounds__(kThreads) void tap_wgrad_kernel(TwArgs a) {
    constexpr int MX = PAIR ? 2 : 1;
    extern __shared__ float lds[];
    float* const Xs = lds;              // [4][CHS]
    float* const Ds = lds + 4 * a.CHS;  // [16][DQ]
    __shared__ ChT tabx[kMaxC];
    __shared__ ChT taby[16];

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kq = lane >> 4, pl = lane & 15;
    const int ch = blockIdx.y;  // 4-channel chunk
    for (int c = tid; c < a.C; c += kThreads) tabx[c] = ch_table_entry(a.x, c, (int64_t)a.H * a.W);
    for (int c = tid; c < a.Co; c += kThreads) taby[c] = ch_table_entry(a.dy, c, (int64_t)a.OH * a.OW);
    __syncthreads();

    // per-lane column offsets into the halo (channel pl>>2, tap of the group), pixel kq
    int boff[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        int tap = a.gtap[t][pl & 3];
        if (tap < 0) tap = a.gtap[t][0];
        if (tap < 0) tap = 0;  // an all-padding tile (NT rounded up)
        const int kh = tap / a.KW, kw = tap - kh * a.KW;
        const int cx = kw * a.DW;
        boff[t] = (pl >> 2) * a.CHS + kh * a.DH * a.RS + (cx % MX) * a.PS + cx / MX + kq;
    }
    const int aoff = pl * a.DQ + wave * a.BX + kq;  // dy row co = pl, tile row = wave

    const int tpi = a.tiles_x * a.tiles_y;
    auto qdiv = [](int x, uint32_t m) { return m ? (int)__umulhi((uint32_t)x, m) : x; };
    auto tile_geo = [&](int tile, int& n, int& oy0, int& ox0) {
        n = qdiv(tile, a.m_tpi);
        const int tr = tile - n * tpi;
        const int tyi = qdiv(tr, a.m_tx);
        oy0 = tyi * kBY;
        ox0 = (tr - tyi * a.tiles_x) * a.BX;
    };
    const uint32_t xplane = (uint32_t)a.H * a.W * 4u, yplane = (uint32_t)a.OH * a.OW * 4u;

    typedef float v2f __attribute__((ext_vector_type(2)));
    v2f v[kPF];
    float dv[16], dyy[16];
    uint32_t rowok = 0;
    bool colok = false, dok = false;
    auto load_tile = [&](int tile) {
        int n, oy0, ox0;
        tile_geo(tile, n, oy0, ox0);
        // x halo rows of channel 4*ch + wave
        {
            const int c = ch * 4 + wave;
            const ChT t = tabx[min(c, a.C - 1)];
            const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(t.p + (int64_t)n * t.ns),
                                                              (short)0, (int)xplane, 0x00020000);
            const int sy0 = oy0 * a.SH - a.PH, sx0 = ox0 * a.SW - a.PW;
            const int ix = sx0 + MX * lane;
            colok = c < a.C && lane < a.HCu && ix >= 0 && ix < a.W;
            const uint32_t voff = colok ? (uint32_t)ix * 4u : 0x80000000u;
            rowok = 0;
#pragma unroll
            for (int r = 0; r < kPF; ++r) {
                if (r < a.HR) {
                    const int iy = sy0 + r;
                    if ((unsigned)iy < (unsigned)a.H) {
                        rowok |= 1u << r;
                        const uint32_t o = colok ? voff + (uint32_t)iy * (uint32_t)a.W * 4u : voff;
                        if constexpr (PAIR)
                            v[r] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(xr, o, 0, 0));
                        else
                            v[r][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o, 0, 0));
                    }
                }
            }
        }
        // dy: tile row oy0 + wave of every row co
        {
            const int oy = oy0 + wave, ox = ox0 + lane;
            dok = lane < a.BX && ox < a.OW && oy < a.OH;
            const uint32_t o = dok ? ((uint32_t)oy * (uint32_t)a.OW + (uint32_t)ox) * 4u : 0x80000000u;
#pragma unroll
            for (int co = 0; co < 16; ++co) {
                if (co < a.Co) {
                    const ChT ty = taby[co];
                    const auto dr = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(ty.p + (int64_t)n * ty.ns),
                                                                      (short)0, (int)yplane, 0x00020000);
                    dv[co] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dr, o, 0, 0));
                    if constexpr (YB) {
                        const auto yr = __builtin_amdgcn_make_buffer_rsrc(
                            (void*)uniform_ptr(ty.y + (int64_t)n * ty.yns), (short)0, (int)yplane, 0x00020000);
                        dyy[co] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, o, 0, 0));
                    }
                }
            }
        }
    };
    auto store_tile = [&]() {
        {
            const int c = ch * 4 + wave;
            const ChT t = tabx[min(c, a.C - 1)];
            float* const xs = Xs + wave * a.CHS + lane;
            if (lane < a.PS) {
#pragma unroll
                for (int r = 0; r < kPF; ++r) {
                    if (r < a.HR) {
                        const bool ok = ((rowok >> r) & 1u) && colok;
                        float x0 = 0.f, x1 = 0.f;
                        if (ok) {
                            x0 = ch_xform(t.xf, t.act, t.k, v[r][0], v[r][0]);
                            if constexpr (PAIR) x1 = ch_xform(t.xf, t.act, t.k, v[r][1], v[r][1]);
                        }
                        xs[r * a.RS] = x0;
                        if constexpr (PAIR) xs[r * a.RS + a.PS] = x1;
                    }
                }
            }
        }
        if (lane < a.BX) {
            float* const ds = Ds + wave * a.BX + lane;
#pragma unroll
            for (int co = 0; co < 16; ++co) {
                float d = 0.f;
                if (co < a.Co && dok) {
                    const ChT ty = taby[co];
                    d = ch_xform(ty.xf, ty.act, ty.k, dv[co], YB ? dyy[co] : dv[co]);
                }
                ds[co * a.DQ] = d;
            }
        }
    };

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;  // dbias partial: sum of this lane's dy values (row co = pl)

    int tile = blockIdx.x;
    if (tile < a.ntiles) load_tile(tile);
    const int nstep = a.BX >> 2;
    const int xrow = wave * a.SH * a.RS;  // halo row of this wave's tile row
    while (tile < a.ntiles) {
        __syncthreads();  // LDS free
        store_tile();
        __syncthreads();
        const int ntile = tile + gridDim.x;
        if (ntile < a.ntiles) load_tile(ntile);
        for (int s = 0; s < nstep; ++s) {
            const float av = Ds[aoff + 4 * s];
            bsum += av;
            const int xo = xrow + 4 * s;  // 4 output pixels = 4 plane units (stride 1 or 2)
            float bv[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) bv[t] = Xs[boff[t] + xo];
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[t], acc[t], 0, 0, 0);
        }
        tile = ntile;
    }

    // ---- reduce the 4 waves' partials in LDS (fixed order), one atomic per dW element
    __syncthreads();
    float* const red = lds;  // [4][16 rows][NT*16 cols]
    const int ncol = NT * 16;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(wave * 16 + kq * 4 + r) * ncol + t * 16 + pl] = acc[t][r];
    __syncthreads();
    double* const dwr = a.dw + (int64_t)(blockIdx.x % a.nrep) * a.rep_stride;
    for (int e = tid; e < 16 * ncol; e += kThreads) {
        const int co = e / ncol, j = e - co * ncol;
        const int t = j >> 4, l16 = j & 15;
        const int tap = a.gtap[t][l16 & 3];
        const int ci = ch * 4 + (l16 >> 2);
        if (co < a.Co && tap >= 0 && ci < a.C) {
            const float s = ((red[e] + red[16 * ncol + e]) + red[32 * ncol + e]) + red[48 * ncol + e];
            atomicAdd(&dwr[((int64_t)co * a.WC + ci) * a.KK + tap], s);
        }
    }
    if (a.dbias && ch == 0) {
        // lanes with the same co (pl) in the 4 kq groups and 4 waves
        __syncthreads();
        float* const rb = lds;
        rb[wave * 64 + lane] = bsum;
        __syncthreads();
        if (tid < 16 && tid < a.Co) {
            float s = 0.f;
            for (int w = 0; w < 4; ++w)
                for (int q = 0; q < 4; ++q) s += rb[w * 64 + q * 16 + tid];
            atomicAdd(&(a.dbias + (int64_t)(blockIdx.x % a.nrep) * a.rep_stride)[tid], s);
        }
    }
}

template <int NT, bool YB, bool PAIR>
int32_t tw_launch(const TwArgs& a, int nchunk, size_t lds, hipStream_t st) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
    }
    auto k = tap_wgrad_kernel<NT, YB, PAIR>;
    if (lds > 48 * 1024 &&
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return isg_check_launch("tap_wgrad_kernel: dynamic LDS");
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kThreads, lds) != hipSuccess || occ < 1) occ = 1;
    // workgroups per chunk: fill the chip once over all chunks
    const int per = std::max(1, std::min(a.ntiles, (occ * cus + nchunk - 1) / nchunk));
    hipLaunchKernelGGL(k, dim3((unsigned)per, (unsigned)nchunk), dim3(kThreads), lds, st, a);
    return isg_check_launch("tap_wgrad_kernel");
}

template <int NT>
int32_t tw_launch_v(const TwArgs& a, int nchunk, size_t lds, bool yb, bool pair, hipStream_t st) {
    if (pair) return yb ? tw_launch<NT, true, true>(a, nchunk, lds, st) : tw_launch<NT, false, true>(a, nchunk, lds, st);
    return yb ? tw_launch<NT, true, false>(a, nchunk, lds, st) : tw_launch<NT, false, false>(a, nchunk, lds, st);
}

// Worst bank multiplicity of one column tile's B reads: lanes pl (16 columns) x kq; the
// ds_read_b32 groups are lanes 0-31 (kq 0,1) and 32-63 (kq 2,3), bank = dword % 32.
int tw_tile_conflicts(const int* off16) {
    int worst = 1;
    for (int base = 0; base < 4; base += 2) {
        int cnt[32] = {0};
        int addr[32][32];
        for (int kq = base; kq < base + 2; ++kq)
            for (int l = 0; l < 16; ++l) {
                const int ad = off16[l] + kq, b = ad % 32;
                bool dup = false;
                for (int i = 0; i < cnt[b]; ++i) dup |= addr[b][i] == ad;
                if (!dup) addr[b][cnt[b]++] = ad;
                worst = std::max(worst, cnt[b]);
            }
    }
    return worst;
}

// Choose PS / RS / CHS paddings and group the KK taps into column tiles of 4 channels x 4
// taps such that every tile's reads are bank-conflict-free (4 channels at CHS = 8 mod 32
// apart, 4 taps of one parity with distinct offsets mod 8). Falls back to the layout
// with the smallest worst case. Returns false if more than 8 tiles would be needed.
bool tw_layout(TwArgs& a, int mx, int& NT) {
    int best = 1 << 30;
    TwArgs b = a;
    for (int ps = a.HCu; ps < a.HCu + 8; ++ps) {
        for (int rs = mx * ps; rs < mx * ps + 8; ++rs) {
            int chs = a.HR * rs;
            chs += ((8 - chs % 32) + 32) % 32;
            auto toff = [&](int tap) {
                const int kh = tap / a.KW, kw = tap - kh * a.KW, cx = kw * a.DW;
                return kh * a.DH * rs + (cx % mx) * ps + cx / mx;
            };
            // greedy: per parity class, repeatedly take one tap from each residue mod 8
            int8_t grp[8][4];
            int ng = 0;
            bool used[32] = {false};
            bool ok = true;
            for (int par = 0; par < 2 && ok; ++par) {
                for (;;) {
                    int g[4], n = 0;
                    bool taken[8] = {false};
                    for (int t = 0; t < a.KK && n < 4; ++t) {
                        const int o = toff(t);
                        if (used[t] || (o & 1) != par || taken[o % 8]) continue;
                        taken[o % 8] = true;
                        g[n++] = t;
                    }
                    if (!n) break;
                    if (ng == 8) { ok = false; break; }
                    for (int i = 0; i < 4; ++i) grp[ng][i] = (int8_t)(i < n ? g[i] : -1);
                    for (int i = 0; i < n; ++i) used[g[i]] = true;
                    ++ng;
                }
            }
            if (!ok || (size_t)(4 * chs) * 4 > 40 * 1024) continue;
            int worst = 1;
            for (int t = 0; t < ng; ++t) {
                int off[16];
                for (int l = 0; l < 16; ++l) {
                    const int tap = grp[t][l & 3] >= 0 ? grp[t][l & 3] : grp[t][0];
                    off[l] = (l >> 2) * chs + toff(tap);
                }
                worst = std::max(worst, tw_tile_conflicts(off));
            }
            const int cost = worst * 16 + ng;
            if (cost < best) {
                best = cost;
                b.PS = ps; b.RS = rs; b.CHS = chs;
                for (int t = 0; t < 8; ++t)
                    for (int i = 0; i < 4; ++i) b.gtap[t][i] = t < ng ? grp[t][i] : (int8_t)-1;
                NT = ng;
                if (worst == 1) break;
            }
        }
        if (best < 32) break;  // conflict-free found
    }
    if (best == (1 << 30)) return false;
    a = b;
    NT = NT <= 4 ? NT : NT <= 6 ? 6 : 8;  // instantiated tile counts (extra tiles: padding)
    return true;
}

// ---- all-channel variant for stride-2 convs (the stem, segment.py:23-26) -----------------
// The chunked kernel above re-stages (and re-transforms) the tile's dy rows once per
// 4-channel chunk: for the stem's 20 input channels that is 5 passes over dy and the saved
// y, and its staging instructions, not the MFMAs, bounded it. Here one workgroup stages
// the halo of EVERY input channel plus dy once per tile, and the 4 waves split the
// C*KK GEMM columns (wave w owns column tiles [w*NTW, (w+1)*NTW)); each wave walks all 4
// tile rows. Waves own disjoint columns, so the epilogue needs no cross-wave reduction.
//
// Staging: a "pair item" is two consecutive halo rows of one channel (lanes 0-31 the
// first, 32-63 the second, one column pair per lane), so the channel — its pointer,
// transform and coefficients — stays wave-uniform. Items are prefetched into registers
// for the next tile while this tile's MFMAs run.
constexpr int kTwaMaxPW = 30;  // pair items per wave (C * ceil(HR/2) <= 120)
constexpr int kTwaTiles = 32;  // column tiles (C*KK <= 512)
constexpr int kDyPT = 7;       // dy tile elements per thread (16 x 4 x BX, BX <= 28)


struct TwaArgs {
    isg_vtensor dy;
    isg_vtensor x;
    double* dw;
    double* dbias;
    int64_t rep_stride;
    int nrep;
    int N, C, Co, H, W, OH, OW, KH, KW, PH, PW, KK;
    int WC;  // the weight's input channels (isg_conv_geom.w_ci)
    int BX, tiles_x, tiles_y, ntiles;
    int HR, HRP, HCu, PS, RS, CHS, DQ, KPW;
    uint32_t m_tpi, m_tx, m_4bx, m_bx, m_hrp;
    // tile t, lane pl: column id ci*KK + tap, or -1 - (a column id to read) for padding
    int16_t col[kTwaTiles][16];
};

template <int NTW, bool YB>
__global__ __launch_bounds__(kThreads, 2) void tap_wgrad_all_kernel(TwaArgs a) {
    extern __shared__ float lds[];
    float* const Xs = lds;                  // [C][CHS]: rows of RS = even plane | odd plane
    float* const Ds = lds + a.C * a.CHS;    // [16][DQ]: dy rows, 4 tile rows of BX
    __shared__ ChT tabx[kMaxC];
    __shared__ ChT taby[16];

    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    const int kq = lane >> 4, pl = lane & 15, half = lane >> 5, hl = lane & 31;
    for (int c = tid; c < a.C; c += kThreads) tabx[c] = ch_table_entry(a.x, c, (int64_t)a.H * a.W);
    for (int c = tid; c < a.Co; c += kThreads) taby[c] = ch_table_entry(a.dy, c, (int64_t)a.OH * a.OW);
    __syncthreads();

    int boff[NTW];
    bool cval[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
        int c = a.col[wave * NTW + t][pl];
        cval[t] = c >= 0;
        if (c < 0) c = -1 - c;
        const int ci = c / a.KK, tap = c - ci * a.KK;
        const int kh = tap / a.KW, kw = tap - kh * a.KW;
        boff[t] = ci * a.CHS + kh * a.RS + (kw & 1) * a.PS + (kw >> 1) + kq;
    }
    const int aoff = pl * a.DQ + kq;

    const int tpi = a.tiles_x * a.tiles_y;
    auto qdiv = [](int x, uint32_t m) { return m ? (int)__umulhi((uint32_t)x, m) : x; };
    auto tile_geo = [&](int tile, int& n, int& oy0, int& ox0) {
        n = qdiv(tile, a.m_tpi);
        const int tr = tile - n * tpi;
        const int tyi = qdiv(tr, a.m_tx);
        oy0 = tyi * kBY;
        ox0 = (tr - tyi * a.tiles_x) * a.BX;
    };
    const uint32_t xplane = (uint32_t)a.H * a.W * 4u, yplane = (uint32_t)a.OH * a.OW * 4u;

    typedef float v2f __attribute__((ext_vector_type(2)));
    v2f v[kTwaMaxPW];
    float dv[kDyPT], dyy[kDyPT];
    uint32_t okm = 0;   // bit j: item j's row and column are inside the image
    uint32_t dokm = 0;  // bit i: dy element i is inside the map
    auto load_tile = [&](int tile) {
        int n, oy0, ox0;
        tile_geo(tile, n, oy0, ox0);
        const int sy0 = oy0 * 2 - a.PH, ix = ox0 * 2 - a.PW + 2 * hl;
        const bool colok = hl < a.HCu && ix >= 0 && ix < a.W;
        okm = 0;
        // branch-free: every item slot issues its load (items past C*HRP and halo rows
        // past HR get an out-of-range offset, which the buffer load returns as 0)
#pragma unroll
        for (int j = 0; j < kTwaMaxPW; ++j) {
            const int k = 4 * j + wave;
            const int ch = (int)__umulhi((uint32_t)k, a.m_hrp), rp = k - ch * a.HRP;
            const ChT t = tabx[min(ch, a.C - 1)];
            const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)uniform_ptr(t.p + (int64_t)n * t.ns),
                                                              (short)0, (int)xplane, 0x00020000);
            const int r = 2 * rp + half, iy = sy0 + r;
            const bool ok = colok && ch < a.C && r < a.HR && (unsigned)iy < (unsigned)a.H;
            okm |= (uint32_t)ok << j;
            const uint32_t o = ok ? ((uint32_t)iy * (uint32_t)a.W + (uint32_t)ix) * 4u : 0x80000000u;
            v[j] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(xr, o, 0, 0));
        }
        // dy: kDyPT elements per thread (co, tile row, column), per-lane addresses
        dokm = 0;
#pragma unroll
        for (int i = 0; i < kDyPT; ++i) {
            const int e = tid + kThreads * i;
            const int co = qdiv(e, a.m_4bx), rem = e - co * 4 * a.BX;
            const int r = qdiv(rem, a.m_bx), px = rem - r * a.BX;
            const int oy = oy0 + r, ox = ox0 + px;
            const bool ok = co < a.Co && oy < a.OH && ox < a.OW;
            dokm |= (uint32_t)ok << i;
            const ChT& ty = taby[min(co, a.Co - 1)];
            const int64_t o = ok ? (int64_t)oy * a.OW + ox : 0;  // invalid: channel base
            dv[i] = gld(ty.p + (int64_t)n * ty.ns, o);
            if constexpr (YB) dyy[i] = gld(ty.y + (int64_t)n * ty.yns, o);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int j = 0; j < kTwaMaxPW; ++j) {
            const int k = 4 * j + wave;
            const int ch = (int)__umulhi((uint32_t)k, a.m_hrp), rp = k - ch * a.HRP;
            const int r = 2 * rp + half;
            if (ch < a.C && hl < a.PS && r < a.HR) {
                const ChT t = tabx[ch];
                float x0 = 0.f, x1 = 0.f;
                if ((okm >> j) & 1u) {
                    x0 = ch_xform(t.xf, t.act, t.k, v[j][0], v[j][0]);
                    x1 = ch_xform(t.xf, t.act, t.k, v[j][1], v[j][1]);
                }
                float* const xs = Xs + ch * a.CHS + r * a.RS + hl;
                xs[0] = x0;
                xs[a.PS] = x1;
            }
        }
#pragma unroll
        for (int i = 0; i < kDyPT; ++i) {
            const int e = tid + kThreads * i;
            const int co = qdiv(e, a.m_4bx), rem = e - co * 4 * a.BX;
            if (co < 16) {
                float d = 0.f;
                if ((dokm >> i) & 1u) {
                    const ChT& ty = taby[co];
                    d = ch_xform(ty.xf, ty.act, ty.k, dv[i], YB ? dyy[i] : dv[i]);
                }
                Ds[co * a.DQ + rem] = d;
            }
        }
    };

    f32x4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;  // dbias partial (wave 0): sum of this lane's dy values (row co = pl)

    int tile = blockIdx.x;
    if (tile < a.ntiles) load_tile(tile);
    const int nstep = a.BX >> 2;
    while (tile < a.ntiles) {
        __syncthreads();  // LDS free
        store_tile();
        __syncthreads();
        const int ntile = tile + gridDim.x;
        if (ntile < a.ntiles) load_tile(ntile);
        // kBY rows x nstep pixel quads, software-pipelined: the next quad's dy and halo
        // operands are read from LDS while this quad's MFMAs run
        const int nq = kBY * nstep;
        int r = 0, sq = 0;
        if (nq) {
        float av = Ds[aoff];
        float bv[NTW];
#pragma unroll
        for (int t = 0; t < NTW; ++t) bv[t] = Xs[boff[t]];
#pragma unroll 1
        for (int q = 0; q < nq; ++q) {
            if (++sq == nstep) { sq = 0; ++r; }
            const bool more = q + 1 < nq;
            const int xo = more ? r * 2 * a.RS + 4 * sq : 0;
            const int dq = more ? r * a.BX + 4 * sq : 0;
            const float avn = Ds[aoff + dq];
            float bn[NTW];
#pragma unroll
            for (int t = 0; t < NTW; ++t) bn[t] = Xs[boff[t] + xo];
            if (wave == 0) bsum += av;
#pragma unroll
            for (int t = 0; t < NTW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[t], acc[t], 0, 0, 0);
            av = avn;
#pragma unroll
            for (int t = 0; t < NTW; ++t) bv[t] = bn[t];
        }
        }
        tile = ntile;
    }

    // ---- epilogue: waves own disjoint columns; one atomic per dW element per workgroup
    double* const dwr = a.dw + (int64_t)(blockIdx.x % a.nrep) * a.rep_stride;
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
        if (!cval[t]) continue;
        const int c = a.col[wave * NTW + t][pl];
        const int ci = c / a.KK, tap = c - ci * a.KK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = kq * 4 + i;
            if (co < a.Co) atomicAdd(&dwr[((int64_t)co * a.WC + ci) * a.KK + tap], acc[t][i]);
        }
    }
    if (a.dbias) {
        __syncthreads();
        float* const rb = lds;
        if (wave == 0) rb[lane] = bsum;
        __syncthreads();
        if (tid < 16 && tid < a.Co) {
            const float s = ((rb[tid] + rb[16 + tid]) + rb[32 + tid]) + rb[48 + tid];
            atomicAdd(&(a.dbias + (int64_t)(blockIdx.x % a.nrep) * a.rep_stride)[tid], s);
        }
    }
}

template <int NTW>
int32_t twa_launch(const TwaArgs& a, size_t lds, bool yb, hipStream_t st) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
    }
    auto k = yb ? tap_wgrad_all_kernel<NTW, true> : tap_wgrad_all_kernel<NTW, false>;
    if (lds > 48 * 1024 &&
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return isg_check_launch("tap_wgrad_all_kernel: dynamic LDS");
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kThreads, lds) != hipSuccess || occ < 1) occ = 1;
    const int per = std::max(1, std::min(a.ntiles, occ * cus));
    hipLaunchKernelGGL(k, dim3((unsigned)per), dim3(kThreads), lds, st, a);
    return isg_check_launch("tap_wgrad_all_kernel");
}

// Bank multiplicity of one column tile's B reads (lanes 0-31: kq 0/1 x 16 columns).
int twa_conflicts(const int* off, int n) {
    int cnt[32] = {0};
    int addr[32][32];
    int worst = 1;
    for (int kq = 0; kq < 2; ++kq)
        for (int l = 0; l < n; ++l) {
            const int ad = off[l] + kq, b = ad % 32;
            bool dup = false;
            for (int i = 0; i < cnt[b]; ++i) dup |= addr[b][i] == ad;
            if (!dup) addr[b][cnt[b]++] = ad;
            worst = std::max(worst, cnt[b]);
        }
    return worst;
}

// Pads (PS, RS, CHS) and groups the C*KK columns into tiles of 16 with at most `lim`-way
// bank conflicts (2-way costs 4 LDS cycles against a 32-cycle MFMA), fewest tiles first.
bool twa_layout(TwaArgs& a, int& ntiles) {
    const int ncol = a.C * a.KK;
    int best = 1 << 30;
    TwaArgs b = a;
    const int minimal = (ncol + 15) / 16;
    for (int lim = 1; lim <= 2 && best > minimal; ++lim) {
        for (int ps = a.HCu; ps < a.HCu + 4; ++ps) {
            for (int rs = 2 * ps; rs < 2 * ps + 4; ++rs) {
                for (int pad = 0; pad < 32; pad += 4) {
                    const int chs = a.HR * rs + pad;
                    if ((size_t)(a.C * chs + 16 * a.DQ) * 4 > 64 * 1024) continue;
                    auto off = [&](int c) {
                        const int ci = c / a.KK, tap = c - ci * a.KK, kh = tap / a.KW, kw = tap - kh * a.KW;
                        return ci * chs + kh * rs + (kw & 1) * ps + (kw >> 1);
                    };
                    std::vector<char> used(ncol, 0);
                    int16_t col[kTwaTiles][16];
                    int nt = 0, left = ncol;
                    bool ok = true;
                    while (left > 0) {
                        if (nt == kTwaTiles) { ok = false; break; }
                        int o[16], ids[16], n = 0;
                        for (int c = 0; c < ncol && n < 16; ++c) {
                            if (used[c]) continue;
                            o[n] = off(c);
                            if (twa_conflicts(o, n + 1) > lim) continue;
                            ids[n++] = c;
                            used[c] = 1;
                            --left;
                        }
                        for (int l = 0; l < 16; ++l) col[nt][l] = (int16_t)(l < n ? ids[l] : -1 - ids[0]);
                        ++nt;
                    }
                    if (!ok) continue;
                    if (nt < best) {
                        best = nt;
                        b.PS = ps; b.RS = rs; b.CHS = chs;
                        for (int t = 0; t < kTwaTiles; ++t)
                            for (int l = 0; l < 16; ++l) b.col[t][l] = t < nt ? col[t][l] : (int16_t)-1;
                    }
                    if (best == minimal) break;
                }
                if (best == minimal) break;
            }
            if (best == minimal) break;
        }
    }
    if (best == (1 << 30)) return false;
    a = b;
    ntiles = best;
    return true;
}

// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
int32_t twa_try(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st) {
    if (g->SH != 2 || g->SW != 2 || g->DH != 1 || g->DW != 1) return 0;
    if (g->PW % 2 || g->W % 2) return 0;
    const int KK = g->KH * g->KW;
    // measured (kbench): the stem layer1 (20 x 25 columns) 433 -> 308 us; the 16-channel
    // layer2 (400 columns, a 4x smaller map) is faster on the chunked kernel (71 vs ~100 us)
    if (g->Ci * KK > 16 * kTwaTiles || g->Ci * KK < 448) return 0;
    TwaArgs a{};
    a.N = g->N; a.C = g->Ci; a.Co = g->Co; a.H = g->H; a.W = g->W; a.OH = g->OH; a.OW = g->OW;
    a.WC = g->w_ci > 0 ? g->w_ci : g->Ci;
    a.KH = g->KH; a.KW = g->KW; a.PH = g->PH; a.PW = g->PW; a.KK = KK;
    // tile width: a multiple of 4 whose halo (column pairs) fits one 32-lane half-wave
    const int bxmax = (32 * 2 - (g->KW - 1) - 1) / 2 + 1;
    const int bxm = std::min(bxmax, 64) & ~3;
    if (bxm < 4) return 0;
    a.tiles_x = (g->OW + bxm - 1) / bxm;
    a.BX = ((g->OW + a.tiles_x - 1) / a.tiles_x + 3) & ~3;
    if (a.BX > bxm) a.BX = bxm;
    a.tiles_x = (g->OW + a.BX - 1) / a.BX;
    a.HCu = (2 * (a.BX - 1) + g->KW + 1) / 2;
    if (a.HCu > 32 || 16 * kBY * a.BX > kThreads * kDyPT) return 0;
    a.HR = 2 * (kBY - 1) + g->KH;
    a.HRP = (a.HR + 1) / 2;
    if (a.HRP < 4) return 0;  // the item walk wraps at most once per step of 4
    a.KPW = (a.C * a.HRP + 3) / 4;
    if (a.KPW > kTwaMaxPW) return 0;
    a.DQ = kBY * a.BX;
    a.DQ += ((2 - a.DQ % 32) + 32) % 32;  // av reads (co*DQ + kq) conflict-free
    // the layout search is host work of a few ms: cache it per geometry
    struct Cached { int key[7]; int ntiles; int PS, RS, CHS; int16_t col[kTwaTiles][16]; };
    static std::mutex mu;
    static std::vector<Cached> cache;
    const int key[7] = {a.C, a.KK, a.KW, a.HR, a.HCu, a.DQ, 0};
    int ntiles = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        const Cached* hit = nullptr;
        for (const auto& c : cache)
            if (!memcmp(c.key, key, sizeof key)) hit = &c;
        if (hit) {
            ntiles = hit->ntiles; a.PS = hit->PS; a.RS = hit->RS; a.CHS = hit->CHS;
            memcpy(a.col, hit->col, sizeof a.col);
        } else {
            if (!twa_layout(a, ntiles)) ntiles = 0;
            Cached c;
            memcpy(c.key, key, sizeof key);
            c.ntiles = ntiles; c.PS = a.PS; c.RS = a.RS; c.CHS = a.CHS;
            memcpy(c.col, a.col, sizeof a.col);
            cache.push_back(c);
        }
    }
    if (ntiles < 1) return 0;
    const int NTW = (ntiles + 3) / 4;
    a.tiles_y = (g->OH + kBY - 1) / kBY;
    const int64_t tpi = (int64_t)a.tiles_x * a.tiles_y;
    a.ntiles = (int)(g->N * tpi);
    if ((int64_t)a.ntiles * tpi >= (1ll << 32)) return 0;
    auto magic = [](int64_t d) { return d == 1 ? 0u : (uint32_t)(((1ull << 32) + d - 1) / d); };
    a.m_tpi = magic(tpi);
    a.m_tx = magic(a.tiles_x);
    a.m_4bx = magic(4 * a.BX);
    a.m_bx = magic(a.BX);
    a.m_hrp = (uint32_t)(((1ull << 32) + a.HRP - 1) / a.HRP);  // k < 4*kTwaMaxPW: exact
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias;
    a.rep_stride = nrep > 1 ? rep_stride : 0;
    a.nrep = nrep < 1 ? 1 : nrep;
    const size_t lds = (size_t)(a.C * a.CHS + 16 * a.DQ) * sizeof(float);
    bool yb = false;
    for (int i = 0; i < dy->nseg; ++i) yb |= dy->s[i].xform == ISG_XF_BN_BWD;
    int32_t e;
    if (NTW <= 4) e = twa_launch<4>(a, lds, yb, st);
    else if (NTW <= 6) e = twa_launch<6>(a, lds, yb, st);
    else if (NTW <= 7) e = twa_launch<7>(a, lds, yb, st);
    else e = twa_launch<8>(a, lds, yb, st);
    return e ? e : 1;
}

}  // namespace

// Returns 1 if launched, 0 if the shape is not for this kernel, <0 on error.
int32_t isg_tap_wgrad(const isg_conv_geom* g, const isg_vtensor* dy, const isg_vtensor* x, double* dw,
                      double* dbias, int64_t rep_stride, int32_t nrep, hipStream_t st) {
    if (g->groups != 1 || g->Co > 16 || g->Ci > kMaxC) return 0;
    for (int i = 0; i < x->nseg; ++i)
        if (x->s[i].xform == ISG_XF_BN_BWD) return 0;
    if ((int64_t)g->H * g->W * 4 < (1ll << 31) && (int64_t)g->OH * g->OW * 4 < (1ll << 31)) {
        const int32_t t = twa_try(g, dy, x, dw, dbias, rep_stride, nrep, st);
        if (t != 0) return t;
    }
    if (g->SH != g->SW || (g->SH != 1 && g->SH != 2)) return 0;
    const int KK = g->KH * g->KW;
    if (KK > 32) return 0;
    if (g->SH == 2 && (g->PW % 2 || g->W % 2)) return 0;  // column pairs start even
    for (int i = 0; i < x->nseg; ++i)
        if (x->s[i].xform == ISG_XF_BN_BWD) return 0;  // the gathered side never needs y
    if ((int64_t)g->H * g->W * 4 >= (1ll << 31) || (int64_t)g->OH * g->OW * 4 >= (1ll << 31)) return 0;
    TwArgs a{};
    a.dy = *dy; a.x = *x; a.dw = dw; a.dbias = dbias;
    a.rep_stride = nrep > 1 ? rep_stride : 0;
    a.nrep = nrep < 1 ? 1 : nrep;
    a.N = g->N; a.C = g->Ci; a.Co = g->Co; a.H = g->H; a.W = g->W; a.OH = g->OH; a.OW = g->OW;
    a.WC = g->w_ci > 0 ? g->w_ci : g->Ci;
    a.KH = g->KH; a.KW = g->KW; a.SH = g->SH; a.SW = g->SW; a.PH = g->PH; a.PW = g->PW;
    a.DH = g->DH; a.DW = g->DW; a.KK = KK;
    const int mx = g->SW;
    const int ext_x = (g->KW - 1) * g->DW, ext_y = (g->KH - 1) * g->DH;
    // tile width: a multiple of 4 whose halo row fits 64 lanes, split evenly
    const int bxmax = (mx == 1 ? 64 - ext_x : (128 - ext_x - 1) / 2 + 1) & ~3;
    if (bxmax < 4) return 0;
    a.tiles_x = (g->OW + bxmax - 1) / bxmax;
    a.BX = ((g->OW + a.tiles_x - 1) / a.tiles_x + 3) & ~3;
    const int HC = mx * (a.BX - 1) + ext_x + 1;
    a.HCu = (HC + mx - 1) / mx;
    if (a.HCu > 64 || a.BX > 64) return 0;
    a.HR = g->SH * (kBY - 1) + ext_y + 1;
    if (a.HR > kPF) return 0;
    // LDS layout + tap grouping with the fewest bank conflicts (first conflict-free one)
    int NT = 0;
    if (!tw_layout(a, mx, NT)) return 0;
    a.DQ = kBY * a.BX;
    a.DQ += ((2 - a.DQ % 32) + 32) % 32;  // dy rows: lane co*DQ + kq conflict-free
    a.tiles_y = (g->OH + kBY - 1) / kBY;
    const int64_t tpi = (int64_t)a.tiles_x * a.tiles_y;
    a.ntiles = (int)(g->N * tpi);
    if ((int64_t)a.ntiles * tpi >= (1ll << 32)) return 0;
    auto magic = [](int64_t d) { return d == 1 ? 0u : (uint32_t)(((1ull << 32) + d - 1) / d); };
    a.m_tpi = magic(tpi);
    a.m_tx = magic(a.tiles_x);
    const int nchunk = (g->Ci + 3) / 4;
    size_t lds = (size_t)(4 * a.CHS + 16 * a.DQ) * sizeof(float);
    if (NT < 1) return 0;
    lds = std::max(lds, (size_t)(4 * 16 * NT * 16) * sizeof(float));  // the wave reduction
    if (lds > 64 * 1024) return 0;
    bool yb = false;
    for (int i = 0; i < dy->nseg; ++i) yb |= dy->s[i].xform == ISG_XF_BN_BWD;
    const bool pair = mx == 2;
    int32_t e;
    switch (NT) {
        case 1: e = tw_launch_v<1>(a, nchunk, lds, yb, pair, st); break;
        case 2: e = tw_launch_v<2>(a, nchunk, lds, yb, pair, st); break;
        case 3: e = tw_launch_v<3>(a, nchunk, lds, yb, pair, st); break;
        case 4: e = tw_launch_v<4>(a, nchunk, lds, yb, pair, st); break;
        case 6: e = tw_launch_v<6>(a, nchunk, lds, yb, pair, st); break;
        default: e = tw_launch_v<8>(a, nchunk, lds, yb, pair, st); break;
    }
    return e ? e : 1;
}
