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
constexpr int RXS = RX;
constexpr int IY = TY + 2, IX = TX + 2;   // intermediate region (3x3 halo)     34 x 66
constexpr int IXS = IX + 1;
constexpr int DY = TY + 6, DX = TX + 6;   // dlogits region (backward)         38 x 70
constexpr int DXS = DX;
constexpr int GY = TY + 4, GX = TX + 4;   // intermediate-gradient region       36 x 68
constexpr int GJY = GY / 4, GJX = GX / 4; // per phase: 9 x 17
constexpr int GPL = 16 * GJY * GJX;       // one channel, phase-split             2448
constexpr int IPL = IY * IXS;             // one channel of the intermediate      2278
constexpr int XPL = GPL > IPL ? GPL : IPL;
constexpr int kW1 = kCi * kCm * 64;       // convT weights [16][4][8][8]

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

// ---- MFMA form of the convT (v_mfma_f32_16x16x4_f32) ----------------------------------
// A "cell" (by, bx) is the 4 x 4 block of intermediate pixels (4by - 2 + r, 4bx - 2 + s) that
// share the same 2 x 2 input neighbourhood (by - 1 + a, bx - 1 + b): per cell the convT is
// a 64 x 64 matrix product, out[(co, r, s)] = sum_{(a, b, ci)} W1[ci][co][r + 4(1-a)][s + 4(1-b)]
// * T[ci][by - 1 + a][bx - 1 + b]. One MFMA per (co, ci): A[m = (r, s)][k = (a, b)] (lane: m =
// l & 15, k = l >> 4, registers for the whole workgroup), B[k = (a, b)][n = cell] (an LDS
// read of the staged input), D lane: (r, s) = (l >> 4, i) of cell l & 15 — 4 consecutive
// intermediate pixels of one row, one 16-B LDS store.
constexpr int CY = TY / 4 + 1, CX = TX / 4 + 1;  // cells covering the tile + halo: 9 x 17
constexpr int NCELL = CY * CX;
constexpr int IRS = 4 * CX;                      // cell-region row stride (16-B rows) 68
constexpr int IRP = 4 * CY * IRS;                // one channel of the cell region   2448

// The convT weight copied into LDS scratch (>= kW1 floats) with coalesced 16-B loads; a
// per-lane gather straight from global memory (64 scattered loads per lane) bound the
// kernels on the address unit. Caller: barrier before reading `scratch`.
ISG_DEV void copy_w1(const float* w1, float* scratch) {
    for (int e = threadIdx.x; e < kW1 / 4; e += kThreads)
        reinterpret_cast<f32x4*>(scratch)[e] = gld4(w1, 4 * e);
}

// A fragments of the cell GEMM for this lane, from the LDS copy of W1: wf[co][ci]
ISG_DEV void cell_afrag(const float* w1s, float (&wf)[kCm][kCi]) {
    const int lane = threadIdx.x & 63;
    const int m = lane & 15, k = lane >> 4;
    const int r = m >> 2, s = m & 3, aa = k >> 1, bb = k & 1;
    const int ky = r + 4 * (1 - aa), kx = s + 4 * (1 - bb);
#pragma unroll
    for (int co = 0; co < kCm; ++co)
#pragma unroll
        for (int ci = 0; ci < kCi; ++ci) wf[co][ci] = w1s[((ci * kCm + co) * 8 + ky) * 8 + kx];
}

// The intermediate over the cells of the tile region (rows Y0 - 2 .. Y0 + 34, columns
// X0 - 2 .. X0 + 66) into Ic[co][row][col] (origin (Y0 - 2, X0 - 2)), + bias, zero outside
// the image.
ISG_DEV void intermediate_mfma(const isg_mask_head& a, int Y0, int X0, const float (*Ts)[RY][RXS],
                               const float (&wf)[kCm][kCi], float* Ic) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int kq = lane >> 4, aa = kq >> 1, bb = kq & 1;
    const int OH = 4 * a.Hi, OW = 4 * a.Wi;
    float b1[kCm];
#pragma unroll
    for (int co = 0; co < kCm; ++co) b1[co] = a.b1 ? a.b1[co] : 0.f;
    for (int grp = wave; grp * 16 < NCELL; grp += kThreads / 64) {
        const int cell = grp * 16 + (lane & 15);
        const int cl = cell < NCELL ? cell : NCELL - 1;
        const int cy = cl / CX, cx = cl - cy * CX;
        f32x4 acc[kCm];
#pragma unroll
        for (int co = 0; co < kCm; ++co) acc[co] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ci = 0; ci < kCi; ++ci) {
            const float bv = Ts[ci][cy + aa][cx + bb];
#pragma unroll
            for (int co = 0; co < kCm; ++co)
                acc[co] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[co][ci], bv, acc[co], 0, 0, 0);
        }
        // D: (r, s) = (kq, i) of cell `cl`: pixel (Y0 - 2 + 4cy + kq, X0 - 2 + 4cx + i)
        const int oy = Y0 - 2 + 4 * cy + kq, ox = X0 - 2 + 4 * cx;
        const bool rok = cell < NCELL && oy >= 0 && oy < OH;
#pragma unroll
        for (int co = 0; co < kCm; ++co) {
            f32x4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = (rok && ox + i >= 0 && ox + i < OW) ? acc[co][i] + b1[co] : 0.f;
            if (cell < NCELL) *reinterpret_cast<f32x4*>(&Ic[co * IRP + (4 * cy + kq) * IRS + 4 * cx]) = v;
        }
    }
}

__global__ __launch_bounds__(kThreads, 2) void head_fwd_kernel(isg_mask_head a) {
    __shared__ float Ts[kCi][RY][RXS];
    __shared__ __attribute__((aligned(16))) float Ic[kCm * IRP];
    __shared__ ChanCoef coef[kCi];
    const int n = blockIdx.z, Y0 = blockIdx.y * TY, X0 = blockIdx.x * TX;
    const int OH = 4 * a.Hi, OW = 4 * a.Wi;
    load_vt_coefs(a.x, coef, threadIdx.x, kThreads);
    copy_w1(a.w1, Ic);
    __syncthreads();
    float wf[kCm][kCi];
    cell_afrag(Ic, wf);
    __syncthreads();
    load_input(a, coef, n, Y0, X0, Ts);
    __syncthreads();
    intermediate_mfma(a, Y0, X0, Ts, wf, Ic);
    __syncthreads();
    // 3x3 (4 -> 1): lane = column, 8 rows per thread (10 x 3 reads per channel); the
    // intermediate's origin is (Y0 - 2, X0 - 2)
    const int lx = threadIdx.x & 63, rb = threadIdx.x >> 6;
    float out[8];
    const float b2 = a.b2 ? a.b2[0] : 0.f;
#pragma unroll
    for (int o = 0; o < 8; ++o) out[o] = b2;
#pragma unroll
    for (int co = 0; co < kCm; ++co) {
#pragma unroll
        for (int rr = 0; rr < 10; ++rr) {
            const float* row = Ic + co * IRP + (rb * 8 + rr + 1) * IRS + lx + 1;
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

// dT GEMM A operand in LDS: Wd[o = (co, r, s)][k = (a, b)][ci] = W1[ci][co][r + 4(1-a)][s + 4(1-b)]
// (a lane reads word o * 64 + lane: conflict-free)
ISG_DEV void stage_wd(const float* w1s, float* Wd) {
    for (int e = threadIdx.x; e < kW1; e += kThreads) {
        const int ci = e & 15, k = (e >> 4) & 3, o = e >> 6;
        const int co = o >> 4, r = (o >> 2) & 3, s = o & 3, aa = k >> 1, bb = k & 1;
        Wd[e] = w1s[((ci * kCm + co) * 8 + r + 4 * (1 - aa)) * 8 + s + 4 * (1 - bb)];
    }
}

constexpr int XPP = NCELL;        // phase-split intermediate gradient: one (co, r, s) plane
constexpr int XCF = kCm * 16 * XPP > kCm * IRP ? kCm * 16 * XPP : kCm * IRP;

__global__ __launch_bounds__(kThreads, 2) void head_bwd_kernel(isg_mask_head a, int ntx, int nty,
                                                               int ntiles) {
    __shared__ float Ts[kCi][RY][RXS];
    __shared__ float Ds[DY * DXS];
    __shared__ __attribute__((aligned(16))) float Xc[XCF];  // intermediate, then its gradient
    __shared__ float Wd[kW1];
    __shared__ ChanCoef coef[kCi];
    __shared__ SinkRow sk[kCi];
    __shared__ float red[kCm * 4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const int kq = lane >> 4, nl = lane & 15;
    const int OH = 4 * a.Hi, OW = 4 * a.Wi;
    const int64_t hw = (int64_t)a.Hi * a.Wi;
    load_vt_coefs(a.x, coef, tid, kThreads);
    copy_w1(a.w1, Xc);
    __syncthreads();
    stage_wd(Xc, Wd);
    if (tid < kCi) {
        SinkRow q = {};
        q.mode = ISG_SINK_NONE;
        if (a.dx.nsink > 0) q = sink_row(a.dx, tid, hw);
        sk[tid] = q;
    }
    float wf[kCm][kCi];
    cell_afrag(Xc, wf);
    // convT weight gradient: this wave's 4 N-tiles of the [16 ci] x [256 (co, ky, kx)] GEMM
    f32x4 dw1[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) dw1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 3x3 weight / bias gradient: per-tile partials wave-reduced into LDS (acc2[37])
    __shared__ float acc2[kCm * 9 + 1];
    if (tid < kCm * 9 + 1) acc2[tid] = 0.f;
    float db1[kCm];
#pragma unroll
    for (int co = 0; co < kCm; ++co) db1[co] = 0.f;

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int n = tile / (ntx * nty), t2 = tile - n * ntx * nty;
        const int Y0 = (t2 / ntx) * TY, X0 = (t2 % ntx) * TX;
        __syncthreads();  // previous tile's LDS consumed (and the tables ready)
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
        intermediate_mfma(a, Y0, X0, Ts, wf, Xc);  // origin (Y0 - 2, X0 - 2)
        __syncthreads();
        // ---- 3x3 weight / bias gradient over the tile's own logit pixels
        {
            const int lx = tid & 63, rb = tid >> 6;
            float dl[8], dw2[kCm * 9], db2 = 0.f;
#pragma unroll
            for (int i = 0; i < kCm * 9; ++i) dw2[i] = 0.f;
#pragma unroll
            for (int o = 0; o < 8; ++o) {
                dl[o] = Ds[(rb * 8 + o + 3) * DXS + lx + 3];  // zero outside the image
                db2 += dl[o];
            }
#pragma unroll
            for (int co = 0; co < kCm; ++co) {
#pragma unroll
                for (int rr = 0; rr < 10; ++rr) {
                    const float* row = Xc + co * IRP + (rb * 8 + rr + 1) * IRS + lx + 1;
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
#pragma unroll
            for (int i = 0; i < kCm * 9; ++i) {
                const float w = wave_sum(dw2[i]);
                if (lane == 0) atomicAdd(&acc2[i], w);
            }
            const float b = wave_sum(db2);
            if (lane == 0) atomicAdd(&acc2[kCm * 9], b);
        }
        __syncthreads();
        // ---- intermediate gradient over the cell region (origin (Y0 - 2, X0 - 2)), stored
        //      phase-split: Xc[((co * 4 + r) * 4 + s) * NCELL + cy * CX + cx]
        for (int p = tid; p < GY * GX; p += kThreads) {
            const int qy = p / GX, qx = p - qy * GX;
            const int oy = Y0 - 2 + qy, ox = X0 - 2 + qx;
            const bool in = oy >= 0 && oy < OH && ox >= 0 && ox < OW;
            const bool own = qy >= 2 && qy < 2 + TY && qx >= 2 && qx < 2 + TX;
            const float* d = Ds + qy * DXS + qx;  // d[(2 - dy) * DXS + 2 - dx] = dl[oy+1-dy][ox+1-dx]
            const int dst = ((qy & 3) * 4 + (qx & 3)) * NCELL + (qy >> 2) * CX + (qx >> 2);
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
                Xc[co * 16 * NCELL + dst] = v;
            }
        }
        __syncthreads();
        // ---- input gradient (MFMA): D[ci][px] = sum_{o, (a,b)} Wd[o][(a,b)][ci] *
        //      dI[o][cell (ly + 1 - a, lx + 1 - b)]; wave w: own input rows w and w + 4
        {
            const int aa = kq >> 1, bb = kq & 1;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ly = wave + 4 * h;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                const float* bp = Xc + (ly + 1 - aa) * CX + (nl + 1 - bb);
                const float* ap = Wd + lane;
#pragma unroll 8
                for (int o = 0; o < 64; ++o)
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[o * 64], bp[o * NCELL], acc, 0, 0, 0);
                // D lane: ci = 4kq + i, px = (ly, nl)
                const int iy = Y0 / 4 + ly, ix = X0 / 4 + nl;
                if (iy < a.Hi && ix < a.Wi) {
                    const int64_t pix = (int64_t)iy * a.Wi + ix;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const SinkRow& q = sk[4 * kq + i];
                        if (q.mode != ISG_SINK_STORE && q.mode != ISG_SINK_ACCUM) continue;
                        float* p = q.p + (int64_t)n * q.ns + pix;
                        *p = q.mode == ISG_SINK_ACCUM ? *p + acc[i] : acc[i];
                    }
                }
            }
        }
        // ---- convT weight gradient (MFMA): K = the 128 own input pixels, 4 per step;
        //      A[ci][px] = input, B[px][(co, ky, kx)] = dI under tap (ky, kx) of px
        {
#pragma unroll 2
            for (int st = 0; st < (TY / 4) * (TX / 4) / 4; ++st) {
                const int P = st * 4 + kq;
                const int ly = P >> 4, lx = P & 15;
                const float av = Ts[nl][ly + 1][lx + 1];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int col = (wave * 4 + t) * 16 + nl;  // (co, ky, kx), kx fastest
                    const int co = col >> 6, ky = (col >> 3) & 7, kx = col & 7;
                    const float bv = Xc[((co * 4 + (ky & 3)) * 4 + (kx & 3)) * NCELL +
                                        (ly + (ky >> 2)) * CX + lx + (kx >> 2)];
                    dw1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, dw1[t], 0, 0, 0);
                }
            }
        }
    }
    // ---- fold the partial weight gradients into this workgroup's replica
    const int rep = blockIdx.x % a.nrep;
    if (a.dw1) {
        float* d = a.dw1 + (int64_t)rep * a.rep_stride;
        // D lane: ci = 4kq + i, column (co, ky, kx) = (wave * 4 + t) * 16 + nl
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                atomicAdd(&d[(4 * kq + i) * (kCm * 64) + (wave * 4 + t) * 16 + nl], dw1[t][i]);
    }
    float v[kCm];
#pragma unroll
    for (int co = 0; co < kCm; ++co) v[co] = wave_sum(db1[co]);
    constexpr int NV = kCm * 9 + 1 + kCm;
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int co = 0; co < kCm; ++co) red[co * 4 + wave] = v[co];
    __syncthreads();
    if (tid < NV) {
        const int j = tid - (kCm * 9 + 1);
        const float s = tid <= kCm * 9 ? acc2[tid]
                                       : (red[j * 4] + red[j * 4 + 1]) + (red[j * 4 + 2] + red[j * 4 + 3]);
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
