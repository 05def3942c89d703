// Fused mask head (segment.py:435-438, 504-505): bottle6_1 = ConvTranspose2d(16 -> 4, k8,
// s4, p2) and bottle6_2 = Conv2d(4 -> 1, 3x3, p1), with no nonlinearity between them.
//
// Unfused, the 4-channel full-resolution intermediate (4 x 1024^2 per image, 33.5 MB at
// bs2) made several HBM round trips through six kernels (convT forward, 3x3 forward, the
// 3x3's input and weight gradients, the convT's input and weight gradients). Here it
// never leaves LDS:
//   forward : one workgroup per 32 x 64 logit tile: the 10 x 18 x 16 input region -> LDS;
//             the 34 x 66 x 4 intermediate (tile + 3x3 halo) -> LDS; the 3x3 -> logits.
//   backward: the same tile, looped over by a persistent grid: input region and the
//             38 x 70 dlogits region -> LDS; the intermediate is recomputed for the 3x3's
//             weight gradient, then overwritten by the intermediate's gradient (36 x 68 x 4,
//             stored phase-split so the stride-4 reads of the convT backward are
//             bank-conflict free), from which the input gradient (through the caller's
//             sinks) and the convT weight gradient (registers across tiles, one atomic per
//             weight per workgroup into the ISG_WREP replicas) follow.
//
// Sub-pixel form of the convT: output pixel o (per axis) receives input pixels
// i0 - 1 and i0, i0 = (o + 2) >> 2, through taps r + 4 and r, r = (o + 2) & 3 — exactly
// 2 x 2 input pixels per output pixel. Tiles start at multiples of 4 so a tile-local
// row ly (origin Y0 - 1) has phase r = (1 + ly) & 3 and local input row (1 + ly) >> 2.
#include "stage.h"

namespace {

constexpr int kThreads = 256;
constexpr int kCi = 16, kCm = 4;          // convT input / intermediate channels
constexpr int TY = 32, TX = 64;           // logit (= intermediate) tile
constexpr int RY = TY / 4 + 2, RX = TX / 4 + 2;   // input region (1-pixel halo)   10 x 18
constexpr int RXS = RX + 1;
constexpr int IY = TY + 2, IX = TX + 2;   // intermediate region (3x3 halo)     34 x 66
constexpr int IXS = IX + 1;
constexpr int DY = TY + 6, DX = TX + 6;   // dlogits region (backward)         38 x 70
constexpr int DXS = DX + 1;
constexpr int GY = TY + 4, GX = TX + 4;   // intermediate-gradient region       36 x 68
constexpr int GJY = GY / 4, GJX = GX / 4; // per phase: 9 x 17
constexpr int GPL = 16 * GJY * GJX;       // one channel, phase-split             2448
constexpr int IPL = IY * IXS;             // one channel of the intermediate      2278
constexpr int XPL = GPL > IPL ? GPL : IPL;
constexpr int kW1 = kCi * kCm * 64;       // convT weights [16][4][8][8]

// convT weights staged in LDS as Wt[co][ky][kx][ci]: every use reads 4 or 8 consecutive
// input channels of one (co, ky, kx) with one wave-uniform (broadcast) ds_read_b128
ISG_DEV void stage_w1(const float* w1, float* Wt) {
    for (int i = threadIdx.x; i < kW1; i += kThreads) {
        const int ci = i & 15, k = i >> 4;  // k = (co * 8 + ky) * 8 + kx
        const int co = k >> 6, kk = k & 63;
        Wt[i] = w1[(ci * kCm + co) * 64 + kk];
    }
}

ISG_DEV f32x4 lds4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// the input region of the tile whose top-left intermediate pixel is (Y0, X0), transformed,
// zero outside the image
ISG_DEV void load_input(const isg_mask_head& a, const ChanCoef* coef, int n, int Y0, int X0,
                        float (*Ts)[RY][RXS]) {
    const int iy0 = Y0 / 4 - 1, ix0 = X0 / 4 - 1;
    const int64_t hw = (int64_t)a.Hi * a.Wi;
    for (int i = threadIdx.x; i < kCi * RY * RX; i += kThreads) {
        const int c = i / (RY * RX), r = (i / RX) % RY, q = i % RX;
        const int iy = iy0 + r, ix = ix0 + q;
        float v = 0.f;
        if (iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi)
            v = vt_load(a.x, coef, n, c, hw, (int64_t)iy * a.Wi + ix);
        Ts[c][r][q] = v;
    }
}

// The intermediate over the tile + 1-pixel halo into Is[co][ly][lx] (zero outside the
// image: the 3x3's zero padding). Work is split into (phase, 64-pixel chunk) tasks per
// wave, so a phase's weights are wave-uniform: per half of the input channels a lane
// holds its 2 x 2 x 8 input values and reads the weights as broadcast b128 over ci.
ISG_DEV void intermediate(const isg_mask_head& a, int Y0, int X0, const float (*Ts)[RY][RXS],
                          const float* Wt, float* Is) {
    constexpr int NCH = 3;  // chunks per phase: <= 9 x 17 = 153 pixels
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int OH = 4 * a.Hi, OW = 4 * a.Wi;
    float b1[kCm];
#pragma unroll
    for (int co = 0; co < kCm; ++co) b1[co] = a.b1 ? a.b1[co] : 0.f;
    for (int task = wave; task < 16 * NCH; task += kThreads / 64) {
        const int ph = task / NCH, chunk = task - ph * NCH;
        const int r = ph >> 2, s = ph & 3;
        const int ly0 = (r + 3) & 3, lx0 = (s + 3) & 3;
        const int ny = (IY - ly0 + 3) >> 2, nx = (IX - lx0 + 3) >> 2;
        const int j = chunk * 64 + lane;
        if (chunk * 64 >= ny * nx) continue;  // wave-uniform
        const int jj = j < ny * nx ? j : ny * nx - 1;
        const int ly = ly0 + 4 * (jj / nx), lx = lx0 + 4 * (jj % nx);
        const int tr = (1 + ly) >> 2, tc = (1 + lx) >> 2;
        float acc[kCm];
#pragma unroll
        for (int co = 0; co < kCm; ++co) acc[co] = b1[co];
        const float* wt = Wt + opaque(0);  // no hoisting of weight reads out of the tile loop
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float t[4][8];  // [a * 2 + b][ci - 8h]: input pixel (tr + a, tc + b)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                t[0][c] = Ts[8 * h + c][tr][tc];
                t[1][c] = Ts[8 * h + c][tr][tc + 1];
                t[2][c] = Ts[8 * h + c][tr + 1][tc];
                t[3][c] = Ts[8 * h + c][tr + 1][tc + 1];
            }
#pragma unroll
            for (int co = 0; co < kCm; ++co) {
#pragma unroll
                for (int ab = 0; ab < 4; ++ab) {
                    // a = 0 (row tr = i0 - 1) uses tap r + 4, a = 1 tap r; same for b / s
                    const int ky = r + ((ab >> 1) ? 0 : 4), kx = s + ((ab & 1) ? 0 : 4);
                    const float* w = wt + ((co * 8 + ky) * 8 + kx) * 16 + 8 * h;
                    const f32x4 wa = lds4(w), wb = lds4(w + 4);
                    acc[co] += t[ab][0] * wa[0] + t[ab][1] * wa[1] + t[ab][2] * wa[2] + t[ab][3] * wa[3] +
                               t[ab][4] * wb[0] + t[ab][5] * wb[1] + t[ab][6] * wb[2] + t[ab][7] * wb[3];
                }
            }
        }
        if (j >= ny * nx) continue;
        const int oy = Y0 - 1 + ly, ox = X0 - 1 + lx;
        const bool in = oy >= 0 && oy < OH && ox >= 0 && ox < OW;
#pragma unroll
        for (int co = 0; co < kCm; ++co) Is[co * IPL + ly * IXS + lx] = in ? acc[co] : 0.f;
    }
}

__global__ __launch_bounds__(kThreads) void head_fwd_kernel(isg_mask_head a) {
    __shared__ float Ts[kCi][RY][RXS];
    __shared__ float Is[kCm * IPL];
    __shared__ __attribute__((aligned(16))) float Wt[kW1];
    __shared__ ChanCoef coef[kCi];
    const int n = blockIdx.z, Y0 = blockIdx.y * TY, X0 = blockIdx.x * TX;
    const int OH = 4 * a.Hi, OW = 4 * a.Wi;
    load_vt_coefs(a.x, coef, threadIdx.x, kThreads);
    stage_w1(a.w1, Wt);
    __syncthreads();
    load_input(a, coef, n, Y0, X0, Ts);
    __syncthreads();
    intermediate(a, Y0, X0, Ts, Wt, Is);
    __syncthreads();
    // 3x3 (4 -> 1): lane = column, 8 rows per thread (10 x 3 reads per channel)
    const int lx = threadIdx.x & 63, rb = threadIdx.x >> 6;
    float out[8];
    const float b2 = a.b2 ? a.b2[0] : 0.f;
#pragma unroll
    for (int o = 0; o < 8; ++o) out[o] = b2;
#pragma unroll
    for (int co = 0; co < kCm; ++co) {
#pragma unroll
        for (int rr = 0; rr < 10; ++rr) {
            const float* row = Is + co * IPL + (rb * 8 + rr) * IXS + lx;
            const float v0 = row[0], v1 = row[1], v2 = row[2];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const int o = rr - dy;
                if (o < 0 || o >= 8) continue;
                const float* w = a.w2 + (co * 3 + dy) * 3;
                out[o] += w[0] * v0 + w[1] * v1 + w[2] * v2;
            }
        }
    }
    const int ox = X0 + lx;
#pragma unroll
    for (int o = 0; o < 8; ++o) {
        const int oy = Y0 + rb * 8 + o;
        if (oy < OH && ox < OW) a.out[(int64_t)n * a.out_n_stride + (int64_t)oy * OW + ox] = out[o];
    }
}

__global__ __launch_bounds__(kThreads, 2) void head_bwd_kernel(isg_mask_head a, int ntx, int nty,
                                                            int ntiles) {
    __shared__ float Ts[kCi][RY][RXS];
    __shared__ __attribute__((aligned(16))) float Ds[DY * DXS];  // then the own input pixels [px][ci]
    __shared__ float Xs[kCm * XPL];
    __shared__ __attribute__((aligned(16))) float Wt[kW1];
    __shared__ ChanCoef coef[kCi];
    __shared__ SinkRow sk[kCi];
    __shared__ float red[42 * 4];
    static_assert(DY * DXS >= (TY / 4) * (TX / 4) * kCi, "own-pixel table aliases Ds");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const int OH = 4 * a.Hi, OW = 4 * a.Wi;
    const int64_t hw = (int64_t)a.Hi * a.Wi;
    load_vt_coefs(a.x, coef, tid, kThreads);
    stage_w1(a.w1, Wt);
    if (tid < kCi) {
        SinkRow q = {};
        q.mode = ISG_SINK_NONE;
        if (a.dx.nsink > 0) q = sink_row(a.dx, tid, hw);
        sk[tid] = q;
    }
    // convT weight gradient: thread <-> (co, ky, kx), all 16 input channels, across tiles
    const int wco = tid >> 6, wky = (tid >> 3) & 7, wkx = tid & 7;
    const int woff = (((wky & 3) * 4 + (wkx & 3)) * GJY + (wky >> 2)) * GJX + (wkx >> 2);
    float dw1[kCi];
#pragma unroll
    for (int c = 0; c < kCi; ++c) dw1[c] = 0.f;
    float dw2[kCm * 9], db2 = 0.f, db1[kCm];
#pragma unroll
    for (int i = 0; i < kCm * 9; ++i) dw2[i] = 0.f;
#pragma unroll
    for (int co = 0; co < kCm; ++co) db1[co] = 0.f;

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int n = tile / (ntx * nty), t2 = tile - n * ntx * nty;
        const int Y0 = (t2 / ntx) * TY, X0 = (t2 % ntx) * TX;
        __syncthreads();  // previous tile's LDS consumed (and the coefficient table ready)
        load_input(a, coef, n, Y0, X0, Ts);
        for (int i = tid; i < DY * DX; i += kThreads) {
            const int r = i / DX, q = i - r * DX;
            const int oy = Y0 - 3 + r, ox = X0 - 3 + q;
            float v = 0.f;
            if (oy >= 0 && oy < OH && ox >= 0 && ox < OW)
                v = a.dout[(int64_t)n * a.dout_n_stride + (int64_t)oy * OW + ox];
            Ds[r * DXS + q] = v;
        }
        __syncthreads();
        intermediate(a, Y0, X0, Ts, Wt, Xs);
        __syncthreads();
        // ---- 3x3 weight / bias gradient over the tile's own logit pixels
        {
            const int lx = tid & 63, rb = tid >> 6;
            float dl[8];
#pragma unroll
            for (int o = 0; o < 8; ++o) {
                dl[o] = Ds[(rb * 8 + o + 3) * DXS + lx + 3];  // zero outside the image
                db2 += dl[o];
            }
#pragma unroll
            for (int co = 0; co < kCm; ++co) {
#pragma unroll
                for (int rr = 0; rr < 10; ++rr) {
                    const float* row = Xs + co * IPL + (rb * 8 + rr) * IXS + lx;
                    const float v0 = row[0], v1 = row[1], v2 = row[2];
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy) {
                        const int o = rr - dy;
                        if (o < 0 || o >= 8) continue;
                        dw2[(co * 3 + dy) * 3 + 0] += dl[o] * v0;
                        dw2[(co * 3 + dy) * 3 + 1] += dl[o] * v1;
                        dw2[(co * 3 + dy) * 3 + 2] += dl[o] * v2;
                    }
                }
            }
        }
        __syncthreads();
        // ---- intermediate gradient over the tile + 2-pixel halo, phase-split
        for (int p = tid; p < GY * GX; p += kThreads) {
            const int qy = p / GX, qx = p - qy * GX;
            const int oy = Y0 - 2 + qy, ox = X0 - 2 + qx;
            const bool in = oy >= 0 && oy < OH && ox >= 0 && ox < OW;
            const bool own = qy >= 2 && qy < 2 + TY && qx >= 2 && qx < 2 + TX;
            const float* d = Ds + qy * DXS + qx;  // d[(2 - dy) * DXS + 2 - dx] = dl[oy+1-dy][ox+1-dx]
            const int dst = (((qy & 3) * 4 + (qx & 3)) * GJY + (qy >> 2)) * GJX + (qx >> 2);
#pragma unroll
            for (int co = 0; co < kCm; ++co) {
                float v = 0.f;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx)
                        v += a.w2[(co * 3 + dy) * 3 + dx] * d[(2 - dy) * DXS + 2 - dx];
                v = in ? v : 0.f;
                if (own) db1[co] += v;
                Xs[co * XPL + dst] = v;
            }
        }
        __syncthreads();
        // own input pixels as [px][ci] (into the free dlogits buffer): broadcast b128 reads
        for (int i = tid; i < (TY / 4) * (TX / 4) * kCi; i += kThreads) {
            const int c = i & 15, px = i >> 4;
            Ds[i] = Ts[c][(px >> 4) + 1][(px & 15) + 1];
        }
        // ---- input gradient: thread <-> (own input pixel, 8 input channels)
        {
            const int px = tid & 127, c0 = (wave >> 1) * 8;
            const int ly = px >> 4, lx = px & 15;
            float acc[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[c] = 0.f;
            // (the weights are the same for every tile: an opaque base keeps the compiler
            // from hoisting all 2 x 256 of their reads out of the tile loop into registers)
            const float* wt = Wt + opaque(c0);
#pragma unroll 1
            for (int co = 0; co < kCm; ++co) {
#pragma unroll 1
                for (int ky = 0; ky < 8; ++ky) {
#pragma unroll
                    for (int kx = 0; kx < 8; ++kx) {
                        const float v = Xs[co * XPL + (((ky & 3) * 4 + (kx & 3)) * GJY + ly + (ky >> 2)) * GJX +
                                           lx + (kx >> 2)];
                        const float* w = wt + ((co * 8 + ky) * 8 + kx) * 16;
                        const f32x4 wa = lds4(w), wb = lds4(w + 4);
                        acc[0] += wa[0] * v; acc[1] += wa[1] * v; acc[2] += wa[2] * v; acc[3] += wa[3] * v;
                        acc[4] += wb[0] * v; acc[5] += wb[1] * v; acc[6] += wb[2] * v; acc[7] += wb[3] * v;
                    }
                }
            }
            const int iy = Y0 / 4 + ly, ix = X0 / 4 + lx;
            if (iy < a.Hi && ix < a.Wi) {
                const int64_t pix = (int64_t)iy * a.Wi + ix;
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const SinkRow& q = sk[c0 + c];  // wave-uniform channel
                    if (q.mode != ISG_SINK_STORE && q.mode != ISG_SINK_ACCUM) continue;
                    float* p = q.p + (int64_t)n * q.ns + pix;
                    *p = q.mode == ISG_SINK_ACCUM ? *p + acc[c] : acc[c];
                }
            }
        }
        __syncthreads();  // the own-pixel table is complete
        // ---- convT weight gradient (the own input pixels; zero outside the image)
        for (int ly = 0; ly < TY / 4; ++ly) {
#pragma unroll 2
            for (int lx = 0; lx < TX / 4; ++lx) {
                const float v = Xs[wco * XPL + woff + ly * GJX + lx];
                const float* t = Ds + (ly * (TX / 4) + lx) * kCi;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 t4 = lds4(t + 4 * q);
                    dw1[4 * q + 0] += t4[0] * v; dw1[4 * q + 1] += t4[1] * v;
                    dw1[4 * q + 2] += t4[2] * v; dw1[4 * q + 3] += t4[3] * v;
                }
            }
        }
    }
    // ---- fold the partial weight gradients into this workgroup's replica
    const int rep = blockIdx.x % a.nrep;
    if (a.dw1) {
        float* d = a.dw1 + (int64_t)rep * a.rep_stride;
#pragma unroll
        for (int c = 0; c < kCi; ++c) atomicAdd(&d[((c * kCm + wco) * 8 + wky) * 8 + wkx], dw1[c]);
    }
    float v[kCm * 9 + 1 + kCm];
#pragma unroll
    for (int i = 0; i < kCm * 9; ++i) v[i] = wave_sum(dw2[i]);
    v[kCm * 9] = wave_sum(db2);
#pragma unroll
    for (int co = 0; co < kCm; ++co) v[kCm * 9 + 1 + co] = wave_sum(db1[co]);
    constexpr int NV = kCm * 9 + 1 + kCm;
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) red[i * 4 + wave] = v[i];
    __syncthreads();
    if (tid < NV) {
        const float s = (red[tid * 4] + red[tid * 4 + 1]) + (red[tid * 4 + 2] + red[tid * 4 + 3]);
        const int64_t ro = (int64_t)rep * a.rep_stride;
        float* dst = nullptr;
        if (tid < kCm * 9) dst = a.dw2 ? a.dw2 + ro + tid : nullptr;
        else if (tid == kCm * 9) dst = a.db2 ? a.db2 + ro : nullptr;
        else dst = a.db1 ? a.db1 + ro + (tid - kCm * 9 - 1) : nullptr;
        if (dst) atomicAdd(dst, s);
    }
}

int32_t check_head(const isg_mask_head* a, bool bwd) {
    if (!a || !a->w1 || !a->w2 || a->N < 1 || a->Hi < 1 || a->Wi < 1)
        return isg_set_error(ISG_ERR_INVALID, "mask head: NULL weights or bad size");
    int C = 0;
    for (int s = 0; s < a->x.nseg; ++s) C += a->x.s[s].C;
    if (a->x.nseg < 1 || a->x.nseg > ISG_MAX_SEGS || C != kCi || a->x.H != a->Hi || a->x.W != a->Wi)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "mask head: input must be %d channels of %dx%d",
                             kCi, a->Hi, a->Wi);
    if ((int64_t)a->N * 16 * a->Hi * a->Wi >= ((int64_t)1 << 31))
        return isg_set_error(ISG_ERR_UNSUPPORTED, "mask head: output exceeds 32-bit offsets");
    if (!bwd) return a->out ? ISG_OK : isg_set_error(ISG_ERR_INVALID, "mask head: NULL output");
    if (!a->dout) return isg_set_error(ISG_ERR_INVALID, "mask head bwd: NULL dlogits");
    for (int s = 0; s < a->dx.nsink; ++s) {
        const isg_sink& k = a->dx.s[s];
        if (k.mode == ISG_SINK_ACTBWD || (k.mode != ISG_SINK_NONE && (k.stats || !k.p)))
            return isg_set_error(ISG_ERR_UNSUPPORTED, "mask head bwd: input-gradient sinks must be "
                                 "STORE / ACCUM without statistics");
    }
    if (a->nrep < 1 || (a->nrep > 1 && a->rep_stride <= 0))
        return isg_set_error(ISG_ERR_INVALID, "mask head bwd: bad replicas");
    return ISG_OK;
}

}  // namespace

extern "C" int32_t isg_mask_head_fwd(const isg_mask_head* a, isg_stream_t st) {
    if (int32_t e = check_head(a, false)) return e;
    const int OH = 4 * a->Hi, OW = 4 * a->Wi;
    const dim3 grid((unsigned)((OW + TX - 1) / TX), (unsigned)((OH + TY - 1) / TY), (unsigned)a->N);
    hipLaunchKernelGGL(head_fwd_kernel, grid, dim3(kThreads), 0, st, *a);
    return isg_check_launch("head_fwd_kernel");
}

extern "C" int32_t isg_mask_head_bwd(const isg_mask_head* a, isg_stream_t st) {
    if (int32_t e = check_head(a, true)) return e;
    const int OH = 4 * a->Hi, OW = 4 * a->Wi;
    const int ntx = (OW + TX - 1) / TX, nty = (OH + TY - 1) / TY;
    const int ntiles = ntx * nty * a->N;
    static const int env = getenv("ISG_HEAD_BWD_GRID") ? atoi(getenv("ISG_HEAD_BWD_GRID")) : 0;
    const int grid = std::min(ntiles, env > 0 ? env : 512);  // 2 workgroups per CU
    hipLaunchKernelGGL(head_bwd_kernel, dim3(grid), dim3(kThreads), 0, st, *a, ntx, nty, ntiles);
    return isg_check_launch("head_bwd_kernel");
}
