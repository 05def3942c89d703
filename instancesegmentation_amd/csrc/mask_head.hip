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

#include <type_traits>

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
// the image. ring (this image's [4][ISG_HEAD_RING] block, NULL off the image border): the
// un-cropped values on the one-pixel ring outside the image are stored there as well
// (isg.h isg_mask_head); a ring pixel two tiles both cover gets the same bits from each.
ISG_DEV void intermediate_mfma(const isg_mask_head& a, int Y0, int X0, const float (*Ts)[RY][RXS],
                               const float (&wf)[kCm][kCi], float* Ic, float* ring = nullptr) {
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
        if (ring && cell < NCELL) {
            const int64_t rn = ISG_HEAD_RING(a.Hi, a.Wi);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int px = ox + i;
                int idx = -1;
                if ((oy == -1 || oy == OH) && px >= -1 && px <= OW) idx = (oy == OH ? OW + 2 : 0) + px + 1;
                else if ((px == -1 || px == OW) && oy >= 0 && oy < OH) idx = 2 * (OW + 2) + (px == OW ? OH : 0) + oy;
                if (idx >= 0) {
#pragma unroll
                    for (int co = 0; co < kCm; ++co) ring[co * rn + idx] = acc[co][i] + b1[co];
                }
            }
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
    const bool border = Y0 == 0 || Y0 + TY >= OH || X0 == 0 || X0 + TX >= OW;
    intermediate_mfma(a, Y0, X0, Ts, wf, Ic,
                      a.ring && border ? a.ring + (int64_t)n * kCm * ISG_HEAD_RING(a.Hi, a.Wi) : nullptr);
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

// ---- backward, round 4 (head_bwd_kernel) ----------------------------------------------
// Per 32 x 64 logit tile (8 x 16 own input pixels), on a persistent grid:
//   staging  : dlogits rows Y0-3 .. Y0+34, cols X0-4 .. X0+67 and the input rows iy0-1 ..
//              iy0+8, cols ix0-4 .. ix0+19 (transformed) -> LDS, 16-B loads;
//   VALU     : the intermediate gradient dI = 3x3^T(dlogits) over the 9 x 17 cells
//              (phase-split, as head_bwd_v1) and its per-channel sums (convT bias);
//   MFMA     : dx = convT^T(dI) (A operands = the convT weights, kept in 64 registers per
//              lane for the whole launch), dW1 = x (x) dI (this wave's output channel), and
//              Z'[ci][d] = sum_i x[ci][i] * dl[4i + d - 2], d in [-1, 8]^2 (100 offsets);
//   epilogue : dx staged in LDS and written with 16-B stores at the next tile's top.
// The intermediate itself is never recomputed (head_bwd_v1 spent 640 of its 1664 MFMAs
// per tile and ~40 % of its VALU on that, for the 3x3 weight gradient only): with
// I_full = b1 + convT(x) WITHOUT the output crop,
//     dW2[co][t] = sum_{p in image} dl[p] * I[co][p + t - 1]
//                = b1[co] * sum(dl) + sum_{ci,k} W1[ci][co][k] * Z'[ci][k - t + 1] - C[co][t]
// where C removes the (p, t) pairs whose intermediate pixel q = p + t - 1 lies just
// outside the cropped image (q row -1 / OH, column -1 / OW: I there is zero in the
// reference, segment.py:435-438 with padding 2). C needs I_full only on that one-pixel
// ring, computed by the tiles on the image border. Z' and C are reduced once per
// workgroup, then dW2 = W1 . Z' (1024 MACs per output) — the same sum as the reference's
// sum_q I(q) dl(q - t'), reassociated.
namespace hb {
constexpr int IH = TY / 4, IW = TX / 4;     // own input pixels per tile: 8 x 16
constexpr int TSH = IH + 2, TSW = IW + 8;   // staged input: rows iy0-1.., cols ix0-4.. (16-B quads)
constexpr int TSP = TSH * TSW;              // one channel: 240
constexpr int DSH = TY + 6, DSW = TX + 8;   // staged dlogits: rows Y0-3.., cols X0-4..
constexpr int DNQ = DSW / 4;                // 18 quads per dlogits row
constexpr int ZD = 10, ZN = 112;            // Z' offsets per axis (d = -1 .. 8); columns padded
constexpr int RT = TX + 2, RL = TY + 2;     // ring lengths: top/bottom (cols X0-1 .. X0+TX), left/right
constexpr int RING = 2 * RT + 2 * RL;       // per output channel
constexpr int NDI = GY * CX;                // dI items: one intermediate row x one cell column (4 px)
static_assert(IW == 16 && IH == 8, "lane mappings below assume 8 x 16 own input pixels");
static_assert(TX == 64, "the ring correction maps one lane per tile column");
}  // namespace hb

// the dx of one finished tile (LDS [16 ci][IH][IW]) through the caller's STORE / ACCUM sinks
template <bool VX>
ISG_DEV void hb_store_dx(const isg_mask_head& a, const SinkRow* sk, const float* dxs, int n, int iy0,
                         int ix0, int tid) {
    using namespace hb;
    if (VX) {
        for (int i = tid; i < kCi * IH * IW / 4; i += kThreads) {
            const int ci = i >> 5, r = (i >> 2) & 7, qd = i & 3;
            const int iy = iy0 + r, ix = ix0 + 4 * qd;
            const SinkRow& q = sk[ci];
            if (iy >= a.Hi || ix >= a.Wi || (q.mode != ISG_SINK_STORE && q.mode != ISG_SINK_ACCUM)) continue;
            const f32x4 v = *reinterpret_cast<const f32x4*>(&dxs[(ci * IH + r) * IW + 4 * qd]);
            const int64_t off = (int64_t)n * q.ns + (int64_t)iy * a.Wi + ix;
            gst4(q.p, off, q.mode == ISG_SINK_ACCUM ? gld4(q.p, off) + v : v);
        }
    } else {
        for (int i = tid; i < kCi * IH * IW; i += kThreads) {
            const int ci = i >> 7, r = (i >> 4) & 7, c = i & 15;
            const int iy = iy0 + r, ix = ix0 + c;
            const SinkRow& q = sk[ci];
            if (iy >= a.Hi || ix >= a.Wi || (q.mode != ISG_SINK_STORE && q.mode != ISG_SINK_ACCUM)) continue;
            const float v = dxs[(ci * IH + r) * IW + c];
            const int64_t off = (int64_t)n * q.ns + (int64_t)iy * a.Wi + ix;
            gst(q.p, off, q.mode == ISG_SINK_ACCUM ? gld(q.p, off) + v : v);
        }
    }
}

// Staging of one tile into registers (16-B loads, issued together so their latencies
// overlap) and from registers into LDS. Lane items: 3 dlogits quads and 4 input quads
// (channel, row, quad) per thread; the input transform is the branch-free per-lane form
// (stage.h XfLin: PLAIN / BN_FWD + activation).
struct HbPrefetch {
    f32x4 dl[3], x[4];
    int ok;  // bit k: dl[k] in range, bit 3 + k: x[k] in range (else the load read a dummy)
};

// Branch-free: every lane issues its 7 loads unconditionally (an out-of-range item reads
// the first element of its tensor instead and its bit in `ok` is clear). A load under a
// branch makes the compiler drain the whole memory queue (s_waitcnt vmcnt(0)) at the join,
// which turned the prefetch into a synchronous load.
struct HbSrc {  // the input's segments as element offsets from segment 0 (opaque scalars)
    const float* p0;
    int64_t d1, d2;
    int ns0, ns1, ns2, c1, c2, Hi, Wi;
};

ISG_DEV HbSrc hb_src(const VtLite& l, int Hi, int Wi) {
    HbSrc r;
    r.p0 = sgpr_p(l.p0);
    // per-lane segment selection as integer selects: a select between pointers was
    // lowered to an indexed load from a stack copy of the candidates
    const int64_t d1 = l.p1 ? l.p1 - l.p0 : 0, d2 = l.p2 ? l.p2 - l.p0 : 0;
    r.d1 = ((int64_t)sgpr_i((int)(d1 >> 32)) << 32) | (uint32_t)sgpr_i((int)d1);
    r.d2 = ((int64_t)sgpr_i((int)(d2 >> 32)) << 32) | (uint32_t)sgpr_i((int)d2);
    r.ns0 = sgpr_i(l.ns0); r.ns1 = sgpr_i(l.ns1); r.ns2 = sgpr_i(l.ns2);
    r.c1 = sgpr_i(l.c1); r.c2 = sgpr_i(l.c2);
    r.Hi = sgpr_i(Hi); r.Wi = sgpr_i(Wi);
    return r;
}

ISG_DEV void hb_issue(const HbSrc& hs, const float* dout0, int64_t dns, int n, int Y0, int X0,
                      HbPrefetch& f, int tid) {
    using namespace hb;
    const int OH = 4 * hs.Hi, OW = 4 * hs.Wi, iy0 = Y0 / 4, ix0 = X0 / 4;
    const int hw = hs.Hi * hs.Wi;
    const float* dout = dout0 + (int64_t)n * dns;
    int ok = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int i = tid + k * kThreads;
        const int r = i / DNQ, qd = i - r * DNQ;
        const int oy = Y0 - 3 + r, ox = X0 - 4 + 4 * qd;
        const bool in = (i < DSH * DNQ) & (oy >= 0) & (oy < OH) & (ox >= 0) & (ox < OW);
        f.dl[k] = gld4(dout, in ? oy * OW + ox : 0);
        ok |= in ? 1 << k : 0;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // opaque: recompute the per-lane channel addressing per tile instead of keeping 4
        // 64-bit offsets live across the whole tile loop (they spilled)
        const int i = opaque(tid + k * kThreads);
        const int ci = i / (TSH * TSW / 4), rem = i - ci * (TSH * TSW / 4);
        const int r = rem / (TSW / 4), qd = rem - r * (TSW / 4);
        const int iy = iy0 - 1 + r, ix = ix0 - 4 + 4 * qd;
        const bool in = (i < kCi * TSH * TSW / 4) & (iy >= 0) & (iy < hs.Hi) & (ix >= 0) & (ix < hs.Wi);
        // segment by masks, not selects: a select chain over the three candidates was
        // turned into a lookup table in scratch memory
        const int m2 = -(int)(ci >= hs.c2), m1 = -(int)(ci >= hs.c1) & ~m2;
        const int cl = ci - (hs.c1 & m1) - (hs.c2 & m2);
        const int ns = hs.ns0 + ((hs.ns1 - hs.ns0) & m1) + ((hs.ns2 - hs.ns0) & m2);
        const int64_t off = (hs.d1 & (int64_t)m1) + (hs.d2 & (int64_t)m2) + (int64_t)n * ns +
                            (int64_t)cl * hw + iy * hs.Wi + ix;
        f.x[k] = gld4(hs.p0, in ? off : 0);
        ok |= in ? 1 << (3 + k) : 0;
    }
    f.ok = ok;
}

ISG_DEV void hb_commit(const HbPrefetch& f, const XfLin* xl, float* Ts, float* Ds, float& db2, int tid) {
    using namespace hb;
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int i = tid + k * kThreads;
        if (i < DSH * DNQ) {
            const int r = i / DNQ, qd = i - r * DNQ;
            const f32x4 v = (f.ok >> k) & 1 ? f.dl[k] : zero;
            *reinterpret_cast<f32x4*>(&Ds[r * DSW + 4 * qd]) = v;
            if (r >= 3 && r < 3 + TY && qd >= 1 && qd <= TX / 4) db2 += (v[0] + v[1]) + (v[2] + v[3]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = tid + k * kThreads;
        if (i < kCi * TSH * TSW / 4) {
            const int ci = i / (TSH * TSW / 4), rem = i - ci * (TSH * TSW / 4);
            // outside the image the convT input is zero padding, not transform(0)
            const bool in = (f.ok >> (3 + k)) & 1;
            const XfLin l = xl[ci];
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = in ? xf_lin_apply(l, f.x[k][e], 0.f) : 0.f;
            *reinterpret_cast<f32x4*>(&Ts[ci * TSP + 4 * rem]) = v;
        }
    }
}

// One 512-thread workgroup per CU: two halves of 4 waves, each with its own tile in flight
// and its own LDS tile buffers (2 x 77 KB), sharing the tables and combining their dW1 / Z'
// / bias partials in LDS before the atomics — half the replica atomics of two 256-thread
// workgroups (4096 per workgroup: ~6 us of chip-wide atomic throughput at 512 of them)
// and one weight / table setup per 4 tiles instead of per 2.
template <bool VX>
__global__ __launch_bounds__(2 * kThreads, 1) void head_bwd_kernel(isg_mask_head a, int ntx, int nty,
                                                                   int ntiles) {
    using namespace hb;
    __shared__ __attribute__((aligned(16))) float Ts_[2][kCi * TSP];
    __shared__ __attribute__((aligned(16))) float Ds_[2][DSH * DSW];
    __shared__ __attribute__((aligned(16))) float Xc_[2][kCm * 16 * NCELL];  // dI, phase-split
    __shared__ __attribute__((aligned(16))) float dxs_[2][kCi * IH * IW];
    __shared__ float ring_[2][kCm * RING];
    __shared__ float Cs_[2][kCm * 9];
    __shared__ float red_[2][kCm * 4 + 4];
    __shared__ __attribute__((aligned(16))) float w2s[kCm * 9];
    __shared__ ChanCoef coef[kCi];
    __shared__ XfLin xl[kCi];
    __shared__ SinkRow sk[kCi];
    const int tid = threadIdx.x, lane = tid & 63;
    const int h = __builtin_amdgcn_readfirstlane((int)(tid >> 8)), ht = tid & (kThreads - 1);
    const int wave = __builtin_amdgcn_readfirstlane((int)((tid >> 6) & 3));
    float* const Ts = Ts_[h];
    float* const Ds = Ds_[h];
    float* const Xc = Xc_[h];
    float* const dxs = dxs_[h];
    float* const ring = ring_[h];
    float* const Cs = Cs_[h];
    float* const red = red_[h];
    const int kq = lane >> 4, nl = lane & 15, aa = kq >> 1, bb = kq & 1;
    const int OH = 4 * a.Hi, OW = 4 * a.Wi;
    const int64_t hw = (int64_t)a.Hi * a.Wi;
    const int64_t rn = ISG_HEAD_RING(a.Hi, a.Wi);
    const int nb = 2 * (int)gridDim.x;                                  // tile stride
    const int nk = (ntiles - 2 * (int)blockIdx.x + nb - 1) / nb;        // half 0's count (>= half 1's)
    STAMP(0);
    const VtLite vl = vt_lite(a.x);
    const HbSrc hs = hb_src(vl, a.Hi, a.Wi);
    const float* dout0 = sgpr_p(a.dout);
    const int64_t dns = a.dout_n_stride;
    constexpr int NW1 = kW1 / 4 / (2 * kThreads);
    f32x4 w1r[NW1];  // the convT weight, issued first: its LDS copy below waits for these only
#pragma unroll
    for (int k = 0; k < NW1; ++k) w1r[k] = gld4(a.w1, 4 * (tid + k * 2 * kThreads));
    HbPrefetch pf;
    const int tile0 = 2 * (int)blockIdx.x + h;
    if (VX && tile0 < ntiles) {  // the first tile's loads overlap the setup below
        const int t2 = tile0 % (ntx * nty);
        hb_issue(hs, dout0, dns, tile0 / (ntx * nty), (t2 / ntx) * TY, (t2 % ntx) * TX, pf, ht);
    }
    load_vt_coefs(a.x, coef, tid, 2 * kThreads);
#pragma unroll
    for (int k = 0; k < NW1; ++k) reinterpret_cast<f32x4*>(Xc_[0])[tid + k * 2 * kThreads] = w1r[k];
    if (tid < kCi) {
        SinkRow q = {};
        q.mode = ISG_SINK_NONE;
        if (a.dx.nsink > 0) q = sink_row(a.dx, tid, hw);
        sk[tid] = q;
    }
    if (tid < kCm * 9) w2s[tid] = a.w2[tid];
    if (tid < 2 * kCm * 9) Cs_[tid / (kCm * 9)][tid % (kCm * 9)] = 0.f;
    __syncthreads();
    if (tid < kCi) {
        const int c1 = vl.c1, c2 = vl.c2;
        const int xf = tid >= c2 ? vl.xf2 : tid >= c1 ? vl.xf1 : vl.xf0;
        const int act = tid >= c2 ? vl.act2 : tid >= c1 ? vl.act1 : vl.act0;
        xl[tid] = xf_lin(xf, act, coef[tid]);
    }
    // dx GEMM A operands, constant for the launch: A[m = ci][k = (a, b)] of plane o = (co, r, s)
    // = W1[ci][co][r + 4(1 - a)][s + 4(1 - b)]
    float wdA[64];
#pragma unroll
    for (int o = 0; o < 64; ++o) {
        const int co = o >> 4, r = (o >> 2) & 3, s = o & 3;
        wdA[o] = Xc_[0][((nl * kCm + co) * 8 + r + 4 * (1 - aa)) * 8 + s + 4 * (1 - bb)];
    }
    // Z' N-tiles of this wave: 2 wave, 2 wave + 1 (of 7); column d = (dy, dx) of this lane
    // as a Ds offset
    int zoff[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int j = 16 * (2 * wave + t) + nl;
        zoff[t] = j < ZD * ZD ? (j / ZD - 1) * DSW + (j % ZD - 1) : 0;
    }
    const bool z2 = 2 * wave + 1 < ZN / 16;  // wave 3 has one N-tile
    // dW1 N-tiles of this wave's output channel co = wave: column (ky, kx) = 16t + nl
    int w1off[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int ky = 2 * t + (nl >> 3), kx = nl & 7;
        w1off[t] = ((wave * 4 + (ky & 3)) * 4 + (kx & 3)) * NCELL + (ky >> 2) * CX + (kx >> 2);
    }
    f32x4 dw1[4], zp[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) dw1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    zp[0] = zp[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db1[kCm] = {0.f, 0.f, 0.f, 0.f}, db2 = 0.f;
    int pn = -1, piy0 = 0, pix0 = 0;  // the tile whose dx sits in dxs
    STAMP(1);

    int tile = tile0;
    for (int kt = 0; kt < nk; ++kt, tile += nb) {
        // both halves run nk iterations (the workgroup-wide barriers); half 1's last one
        // may have no tile
        const bool act = tile < ntiles;
        const int tc = act ? tile : 0;
        const int n = tc / (ntx * nty), t2 = tc - n * ntx * nty;
        const int Y0 = (t2 / ntx) * TY, X0 = (t2 % ntx) * TX;
        const int iy0 = Y0 / 4, ix0 = X0 / 4;
        const bool top = Y0 == 0, bot = Y0 + TY >= OH, lft = X0 == 0, rgt = X0 + TX >= OW;
        const bool border = top || bot || lft || rgt;
        __syncthreads();  // the previous tile's LDS reads are done (tables and wdA ready)
        if (pn >= 0) hb_store_dx<VX>(a, sk, dxs, pn, piy0, pix0, ht);
        pn = -1;
        // ---- staging: dlogits (+ own sum), input region, the ring (border tiles)
        if (!act) {
        } else if (VX) {
            hb_commit(pf, xl, Ts, Ds, db2, ht);
        } else {
            const float* dout = a.dout + (int64_t)n * a.dout_n_stride;
            for (int i = ht; i < DSH * DSW; i += kThreads) {
                const int r = i / DSW, c = i - r * DSW;
                const int oy = Y0 - 3 + r, ox = X0 - 4 + c;
                float v = 0.f;
                if (oy >= 0 && oy < OH && ox >= 0 && ox < OW) v = dout[(int64_t)oy * OW + ox];
                Ds[i] = v;
                if (r >= 3 && r < 3 + TY && c >= 4 && c < 4 + TX) db2 += v;
            }
            for (int i = ht; i < kCi * TSP; i += kThreads) {
                const int ci = i / TSP, r = (i / TSW) % TSH, c = i % TSW;
                const int iy = iy0 - 1 + r, ix = ix0 - 4 + c;
                float v = 0.f;
                if (iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi)
                    v = vt_load(a.x, coef, n, ci, hw, (int64_t)iy * a.Wi + ix);
                Ts[i] = v;
            }
        }
        if (act && border) {
            const float* rg = a.ring + (int64_t)n * kCm * rn;
            for (int it = ht; it < kCm * RING; it += kThreads) {
                const int co = it / RING, e = it - co * RING;
                float v = 0.f;
                if (e < 2 * RT) {  // top / bottom rows, corners included
                    const bool b = e >= RT;
                    const int qx = X0 - 1 + (e - (b ? RT : 0));
                    if ((b ? bot : top) && qx <= OW) v = rg[co * rn + (b ? OW + 2 : 0) + qx + 1];
                } else {  // left / right columns, rows inside the image only
                    const bool rr = e >= 2 * RT + RL;
                    const int qy = Y0 - 1 + (e - 2 * RT - (rr ? RL : 0));
                    if ((rr ? rgt : lft) && qy >= 0 && qy < OH) v = rg[co * rn + 2 * (OW + 2) + (rr ? OH : 0) + qy];
                }
                ring[it] = v;
            }
        }
        __syncthreads();
        if (kt == 0) STAMP(2);
        // ---- the next tile's loads, in flight during this tile's compute
        if (VX && tile + nb < ntiles) {
            const int nt = tile + nb, nn = nt / (ntx * nty), nt2 = nt - nn * ntx * nty;
            hb_issue(hs, dout0, dns, nn, (nt2 / ntx) * TY, (nt2 % ntx) * TX, pf, ht);
        }
        if (kt == 0) STAMP(3);
        // ---- intermediate gradient over the cell region (origin (Y0 - 2, X0 - 2)):
        //      dI[co][q] = sum_{ty,tx} w2[co][ty][tx] dl[q + 1 - ty][q + 1 - tx], zero outside
        //      the image, stored phase-split Xc[((co * 4 + r) * 4 + s) * NCELL + cy * CX + cx]
        for (int it = act ? ht : NDI; it < NDI; it += kThreads) {
            const int ql = it / CX, cx = it - ql * CX;
            const int cy = ql >> 2, r = ql & 3;
            const int qy = Y0 - 2 + ql;
            float d[3][8];  // Ds rows ql .. ql + 2, columns 4cx .. 4cx + 7
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const f32x4 lo = *reinterpret_cast<const f32x4*>(&Ds[(ql + k) * DSW + 4 * cx]);
                const f32x4 hi = *reinterpret_cast<const f32x4*>(&Ds[(ql + k) * DSW + 4 * cx + 4]);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    d[k][e] = lo[e];
                    d[k][4 + e] = hi[e];
                }
            }
            const bool rin = qy >= 0 && qy < OH;
            const bool rown = ql >= 2 && ql < 2 + TY;
#pragma unroll
            for (int co = 0; co < kCm; ++co) {
                float w[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) w[k] = w2s[co * 9 + k];
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int qxl = 4 * cx + s, qx = X0 - 2 + qxl;
                    const bool in = rin && qx >= 0 && qx < OW;
                    const bool own = rown && qxl >= 2 && qxl < 2 + TX;
                    float v = 0.f;
#pragma unroll
                    for (int ty = 0; ty < 3; ++ty)
#pragma unroll
                        for (int tx = 0; tx < 3; ++tx) v += w[ty * 3 + tx] * d[2 - ty][s + 3 - tx];
                    v = in ? v : 0.f;
                    db1[co] += own ? v : 0.f;
                    Xc[((co * 4 + r) * 4 + s) * NCELL + cy * CX + cx] = v;
                }
            }
        }
        __syncthreads();
        if (kt == 0) STAMP(4);
        if (!act) continue;
        // ---- border tiles: C[co][t] += dl[p] * I_full[p + t - 1] over the pairs whose
        //      intermediate pixel is outside the image (wave = co, lane = tile column / row)
        if (border) {
            const int co = wave;
            const float* rg = ring + co * RING;
            float c[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) c[t] = 0.f;
            if (top && X0 + lane < OW) {
                const float dv = Ds[3 * DSW + lane + 4];
#pragma unroll
                for (int tx = 0; tx < 3; ++tx) c[tx] += dv * rg[lane + tx];
            }
            if (bot && X0 + lane < OW) {
                const float dv = Ds[(OH - 1 - Y0 + 3) * DSW + lane + 4];
#pragma unroll
                for (int tx = 0; tx < 3; ++tx) c[6 + tx] += dv * rg[RT + lane + tx];
            }
            if (lane < TY && Y0 + lane < OH) {
                if (lft) {
                    const float dv = Ds[(lane + 3) * DSW + 4];
#pragma unroll
                    for (int ty = 0; ty < 3; ++ty) c[ty * 3] += dv * rg[2 * RT + lane + ty];
                }
                if (rgt) {
                    const float dv = Ds[(lane + 3) * DSW + OW - 1 - X0 + 4];
#pragma unroll
                    for (int ty = 0; ty < 3; ++ty) c[ty * 3 + 2] += dv * rg[2 * RT + RL + lane + ty];
                }
            }
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const float v = wave_sum(c[t]);
                if (lane == 0) Cs[co * 9 + t] += v;
            }
        }
        // ---- input gradient: rows ly = wave, wave + 4 of the tile; D lane: ci = 4kq + i, px nl
        {
            const int ly0 = wave, ly1 = wave + 4;
            const float* b0 = Xc + (ly0 + 1 - aa) * CX + (nl + 1 - bb);
            const float* b1p = Xc + (ly1 + 1 - aa) * CX + (nl + 1 - bb);
            f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int o = 0; o < 64; ++o) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wdA[o], b0[o * NCELL], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wdA[o], b1p[o * NCELL], acc1, 0, 0, 0);
                // bound how far the scheduler hoists the B reads (each a live register)
                if ((o & 15) == 15) asm volatile("" ::: "memory");
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dxs[((4 * kq + i) * IH + ly0) * IW + nl] = acc0[i];
                dxs[((4 * kq + i) * IH + ly1) * IW + nl] = acc1[i];
            }
        }
        // ---- convT weight gradient of output channel co = wave and this wave's Z' N-tiles:
        //      K = the 128 own pixels, 4 per step (A = the input, shared by both GEMMs)
        {
            const float* ap = Ts + nl * TSP + TSW + 4 + kq;
            const float* zb = Ds + DSW + 4 * kq + 2;
#pragma unroll
            for (int st = 0; st < IH * IW / 4; ++st) {
                const int ly = st >> 2, lx4 = 4 * (st & 3);
                const float av = ap[ly * TSW + lx4];
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    dw1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Xc[w1off[t] + ly * CX + lx4 + kq],
                                                                  dw1[t], 0, 0, 0);
                // Z' B[px][d] = dl[4 px + d - 2]: Ds row 4 ly + 1 + dy, column 4 lx + 2 + dx
                const float* zr = zb + 4 * ly * DSW + 4 * lx4;
                zp[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, zr[zoff[0]], zp[0], 0, 0, 0);
                if (z2) zp[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, zr[zoff[1]], zp[1], 0, 0, 0);
                if ((st & 3) == 3) asm volatile("" ::: "memory");
            }
        }
        if (kt == 0) STAMP(5);
        pn = n; piy0 = iy0; pix0 = ix0;
    }
    __syncthreads();
    STAMP(6);
    if (pn >= 0) hb_store_dx<VX>(a, sk, dxs, pn, piy0, pix0, ht);
    // ---- once per workgroup: the halves' partials combined in LDS, then dW1, Z' -> dW2 and
    //      the bias gradients into replica rep (half 0)
    const int rep = blockIdx.x % a.nrep;
    const int64_t ro = (int64_t)rep * a.rep_stride;
    float* const P1 = Xc_[1];            // half 1's dW1 partial [4096]
    float* const Zs = Xc_[0];            // half 0's Z' [16 ci][ZN]
    float* const Z1 = Xc_[1] + kW1;      // half 1's Z'
    float v1[kCm];
#pragma unroll
    for (int co = 0; co < kCm; ++co) v1[co] = wave_sum(db1[co]);
    const float v2 = wave_sum(db2);
    auto dw1_idx = [&](int t, int i) { return (4 * kq + i) * (kCm * 64) + wave * 64 + t * 16 + nl; };
    float* const zdst = h ? Z1 : Zs;
#pragma unroll
    for (int t = 0; t < 2; ++t)
        if (t == 0 || z2)
#pragma unroll
            for (int i = 0; i < 4; ++i) zdst[(4 * kq + i) * ZN + 16 * (2 * wave + t) + nl] = zp[t][i];
    if (h) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) P1[dw1_idx(t, i)] = dw1[t][i];
    }
    if (lane == 0) {
#pragma unroll
        for (int co = 0; co < kCm; ++co) red[co * 4 + wave] = v1[co];
        red[kCm * 4 + wave] = v2;
    }
    __syncthreads();
    if (h) {
        __syncthreads();
        STAMP(7);
        return;
    }
    if (a.dw1_part) {  // the partial slab, folded later by isg_mask_head_fold (plain stores)
        float* d = a.dw1_part + (int64_t)blockIdx.x * kW1;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) d[dw1_idx(t, i)] = dw1[t][i] + P1[dw1_idx(t, i)];
    } else if (a.dw1) {
        double* d = a.dw1 + ro;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(&d[dw1_idx(t, i)], dw1[t][i] + P1[dw1_idx(t, i)]);
    }
    auto red2 = [&](int j) {
        return ((red_[0][j] + red_[0][j + 1]) + (red_[0][j + 2] + red_[0][j + 3])) +
               ((red_[1][j] + red_[1][j + 1]) + (red_[1][j + 2] + red_[1][j + 3]));
    };
    const float sdl = red2(kCm * 4);
    // dW2[co][t] = sum_{ci, ky, kx} W1[ci][co][ky][kx] Z'[ci][(ky - ty + 1, kx - tx + 1)] from
    // the W1 values already in wdA: lane (ci = nl, (a, b) = kq) holds, for plane o = (co, r,
    // s), W1[ci][co][r + 4(1 - a)][s + 4(1 - b)]; wave = co, the 9 taps summed over the wave
    {
        float zr[6][6];  // Z' rows / columns 4(1-a) .. 4(1-a) + 5 of this lane's input channel
        const int zo = nl * ZN + 4 * (1 - aa) * ZD + 4 * (1 - bb);
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = 0; c < 6; ++c) zr[r][c] = Zs[zo + r * ZD + c] + Z1[zo + r * ZD + c];
        float c9[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) c9[t] = 0.f;
        auto dw2_co = [&](auto cot) {
            constexpr int co = decltype(cot)::value;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int r = j >> 2, s2 = j & 3;
                const float wv = wdA[co * 16 + j];
#pragma unroll
                for (int ty = 0; ty < 3; ++ty)
#pragma unroll
                    for (int tx = 0; tx < 3; ++tx) c9[ty * 3 + tx] += wv * zr[r + 2 - ty][s2 + 2 - tx];
            }
        };
        if (wave == 0) dw2_co(std::integral_constant<int, 0>{});
        else if (wave == 1) dw2_co(std::integral_constant<int, 1>{});
        else if (wave == 2) dw2_co(std::integral_constant<int, 2>{});
        else dw2_co(std::integral_constant<int, 3>{});
        const int co = wave;
        const float b1 = a.b1 ? a.b1[co] : 0.f;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const float v = wave_sum(c9[t]);
            if (lane == 0 && a.dw2)
                atomicAdd(a.dw2 + ro + co * 9 + t, v + b1 * sdl - (Cs_[0][co * 9 + t] + Cs_[1][co * 9 + t]));
        }
        if (lane == 1 && a.db1) atomicAdd(a.db1 + ro + co, red2(co * 4));
        if (tid == 2 && a.db2) atomicAdd(a.db2 + ro, sdl);
    }
    __syncthreads();
    STAMP(7);
}

int32_t check_head(const isg_mask_head* a, bool bwd) {
    if (!a || !a->w1 || !a->w2 || a->N < 1 || a->Hi < 1 || a->Wi < 1)
        return isg_set_error(ISG_ERR_INVALID, "mask head: NULL weights or bad size");
    if (isg_vt_res(&a->x) || (bwd && isg_sinks_res(&a->dx)))
        return isg_set_error(ISG_ERR_UNSUPPORTED, "mask head: residual form");
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
    if (!a->ring)
        return isg_set_error(ISG_ERR_INVALID, "mask head bwd: NULL ring (the forward writes it)");
    return ISG_OK;
}

// 16-B staging and dx stores: the input width a multiple of 4 and every base pointer and
// image stride 16-B aligned (the network's H, W = 0 mod 16 always give that)
bool head_bwd_vec(const isg_mask_head* a) {
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (a->Wi % 4 || !al(a->dout) || a->dout_n_stride % 4) return false;
    for (int s = 0; s < a->x.nseg; ++s) {
        const isg_vseg& g = a->x.s[s];
        if (!al(g.p) || g.n_stride % 4 || g.xform == ISG_XF_BN_BWD) return false;
    }
    for (int s = 0; s < a->dx.nsink; ++s) {
        const isg_sink& k = a->dx.s[s];
        if (k.mode != ISG_SINK_NONE && (!al(k.p) || k.n_stride % 4)) return false;
    }
    return true;
}

}  // namespace

ISG_STAMP_ACCESSOR(isg_dbg_stamps_head)

extern "C" int32_t isg_mask_head_fwd(const isg_mask_head* a, isg_stream_t st) {
    if (int32_t e = check_head(a, false)) return e;
    const int OH = 4 * a->Hi, OW = 4 * a->Wi;
    const dim3 grid((unsigned)((OW + TX - 1) / TX), (unsigned)((OH + TY - 1) / TY), (unsigned)a->N);
    hipLaunchKernelGGL(head_fwd_kernel, grid, dim3(kThreads), 0, st, *a);
    return isg_check_launch("head_fwd_kernel");
}

// the backward's workgroup count (1 two-tile workgroup per CU at most)
static int head_bwd_blocks(int N, int Hi, int Wi) {
    const int OH = 4 * Hi, OW = 4 * Wi;
    const int ntiles = ((OW + TX - 1) / TX) * ((OH + TY - 1) / TY) * N;
    return std::min((ntiles + 1) / 2, 256);
}

extern "C" int64_t isg_mask_head_part_floats(int32_t N, int32_t Hi, int32_t Wi) {
    if (N < 1 || Hi < 1 || Wi < 1) return 0;
    return (int64_t)head_bwd_blocks(N, Hi, Wi) * kW1;
}

// dw1[replica r][e] += sum of the rows of its row chunk r' (r = r' % nrep): a thread per
// (element, 16-row chunk), fp64 sums of fp32 partials (exact, order-free)
__global__ __launch_bounds__(256) void head_fold_kernel(const float* __restrict__ part, int rows,
                                                        double* dw1, int64_t rep_stride, int nrep) {
    const int e = blockIdx.x * 256 + threadIdx.x;  // < kW1 (grid.x = kW1 / 256)
    const int r0 = blockIdx.y * 16;
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += r0 + r < rows ? (double)part[(int64_t)(r0 + r) * kW1 + e] : 0.0;
    atomicAdd(&dw1[(int64_t)(blockIdx.y % (unsigned)nrep) * rep_stride + e], s);
}

extern "C" int32_t isg_mask_head_fold(const isg_mask_head* a, isg_stream_t st) {
    if (!a || !a->dw1_part || !a->dw1 || a->N < 1 || a->Hi < 1 || a->Wi < 1)
        return isg_set_error(ISG_ERR_INVALID, "mask head fold: NULL slab / dw1 or bad size");
    if (a->nrep < 1 || (a->nrep > 1 && a->rep_stride <= 0))
        return isg_set_error(ISG_ERR_INVALID, "mask head fold: bad replicas");
    const int rows = head_bwd_blocks(a->N, a->Hi, a->Wi);
    static_assert(kW1 % 256 == 0, "fold grid");
    hipLaunchKernelGGL(head_fold_kernel, dim3(kW1 / 256, (rows + 15) / 16), dim3(256), 0, st, a->dw1_part,
                       rows, a->dw1, a->nrep > 1 ? a->rep_stride : 0, a->nrep);
    return isg_check_launch("head_fold_kernel");
}

extern "C" int32_t isg_mask_head_bwd(const isg_mask_head* a, isg_stream_t st) {
    if (int32_t e = check_head(a, true)) return e;
    const int OH = 4 * a->Hi, OW = 4 * a->Wi;
    const int ntx = (OW + TX - 1) / TX, nty = (OH + TY - 1) / TY;
    const int ntiles = ntx * nty * a->N;
    const int grid = head_bwd_blocks(a->N, a->Hi, a->Wi);
    if (head_bwd_vec(a))
        hipLaunchKernelGGL(head_bwd_kernel<true>, dim3(grid), dim3(2 * kThreads), 0, st, *a, ntx, nty, ntiles);
    else
        hipLaunchKernelGGL(head_bwd_kernel<false>, dim3(grid), dim3(2 * kThreads), 0, st, *a, ntx, nty, ntiles);
    return isg_check_launch("head_bwd_kernel");
}
