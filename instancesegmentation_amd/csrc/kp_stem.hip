// Keypoint stem: the first layer of Segment(20)'s init_head_s4
// (segment.py:19-31) over cat(image, heatmaps) (segment.py:531-532), with the 17 keypoint
// heatmaps of train_instance.py:33-68 synthesised on the fly and never written to HBM.
//
// A heatmap is zero outside its keypoint's window (about 43 x 43 pixels at sigma 10), so
// the stem splits into
//   * the dense conv over the RGB channels (tap_conv / tap_wgrad with w_ci = 20, isg.h);
//   * kp_fwd_kernel: per 16x16 output tile that any window reaches, the heatmap
//     channels' contribution is added to the raw conv output and the BatchNorm sum /
//     sum-of-squares statistics are corrected by the change of every pixel it touched;
//   * kp_wgrad_kernel: per (image, part, row band) the weight gradient of that part's
//     channel over the output pixels its window reaches;
//   * kp_pool_kernel: the stem's max_pool(x, 4) shortcut (segment.py:31) of the heatmap
//     channels, written densely into their channels of init_down.
// Heatmap value (train_instance.py:50-64): inside [max(0,int(kx-r)), min(W-1,int(kx+r+1)))
// x (same in y), e = exp(-((x-kx)^2+(y-ky)^2)/sigma^2) in double, stored as float where
// e > threshold; 0 elsewhere and for keypoints that are not visible. Contraction is off so
// the double arithmetic is numpy's, operation for operation.
#include <algorithm>
#include <cmath>

#include "stage.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTile = 16;       // fwd: output tile edge (one thread per output pixel)
constexpr int kMaxParts = 32;   // one wave ballots the parts
constexpr int kMaxCo = 16;
constexpr int kMaxKK = 49;
constexpr int kMaxFoot = 64;    // fwd: footprint edge of a 16x16 output tile
constexpr int kMaxWl = 8192;    // fwd: Co x parts x KK weights of the heatmap channels
constexpr int kMaxWgPix = 256;  // wgrad: output pixels per staged chunk
constexpr int kMaxWgFoot = 4096;

struct KpArgs {
    const double* kp;
    int nparts, c_kp0;
    double s2, thr, r;
    int N, Ci, H, W, Co, OH, OW, KH, KW, SH, SW, PH, PW, DH, DW, KK;
    const float* w;
    float* y;
    int64_t y_ns;
    double* stats;
    isg_vtensor dy;
    double* dw;
    int64_t rep_stride;
    int nrep;
    int k;
    float* out;
    int64_t out_ns;
    int tiles_x, FH, FW;
};

struct Win {
    int x0, y0, x1, y1;  // [x0,x1) x [y0,y1); empty when not visible
    double kx, ky;
};

// the keypoint's window (train_instance.py:52-58; python int() truncates toward zero)
ISG_DEV Win part_window(const KpArgs& a, int n, int j) {
    const double* q = a.kp + ((int64_t)n * a.nparts + j) * 3;
    Win w;
    w.kx = q[0];
    w.ky = q[1];
    if (!(q[2] > 0.0) || !kp_coord(w.kx, a.r, a.W) || !kp_coord(w.ky, a.r, a.H)) {
        w.x0 = w.y0 = 0;
        w.x1 = w.y1 = 0;
        return w;
    }
    w.x0 = max(0, (int)(w.kx - a.r));
    w.x1 = min(a.W - 1, (int)(w.kx + a.r + 1.0));
    w.y0 = max(0, (int)(w.ky - a.r));
    w.y1 = min(a.H - 1, (int)(w.ky + a.r + 1.0));
    return w;
}

ISG_DEV float heat(const KpArgs& a, const Win& w, int iy, int ix) {
#pragma clang fp contract(off)
    if (ix < w.x0 || ix >= w.x1 || iy < w.y0 || iy >= w.y1) return 0.f;
    const double dx = (double)ix - w.kx, dy = (double)iy - w.ky;
    const double e = exp(-(dx * dx + dy * dy) / a.s2);
    return e > a.thr ? (float)e : 0.f;
}

ISG_DEV int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
ISG_DEV int ceil_div(int a, int b) { return -floor_div(-a, b); }

// ---- forward: add the heatmap channels' contribution to the raw conv output -----------
__global__ __launch_bounds__(kThreads) void kp_fwd_kernel(KpArgs a) {
    // weights of the active parts' channels, [slot][tap][16 co] (co past Co zero): one
    // broadcast ds_read_b128 per 4 output channels
    __shared__ f32x4 wl[kMaxWl / 4];
    __shared__ float hl[kMaxFoot * kMaxFoot];
    __shared__ int toff[kMaxKK];
    __shared__ Win wins[kMaxParts];
    __shared__ uint32_t act_mask;
    __shared__ int jofs[32];
    __shared__ float red[2][4][kMaxCo];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = blockIdx.y;
    const int ty = blockIdx.x / a.tiles_x, tx = blockIdx.x - ty * a.tiles_x;
    const int oy0 = ty * kTile, ox0 = tx * kTile;
    const int iy0 = oy0 * a.SH - a.PH, ix0 = ox0 * a.SW - a.PW;
    if (wave == 0) {
        bool hit = false;
        if (lane < a.nparts) {
            const Win w = part_window(a, n, lane);
            wins[lane] = w;
            hit = w.x1 > w.x0 && w.y1 > w.y0 && w.y0 < iy0 + a.FH && w.y1 > iy0 &&
                  w.x0 < ix0 + a.FW && w.x1 > ix0;
        }
        const uint64_t m = __ballot(hit);
        if (lane == 0) act_mask = (uint32_t)m;
    }
    __syncthreads();
    uint32_t mask = act_mask;
    if (!mask) return;  // block-uniform: no window reaches this tile
    const int KK = a.KK;
    {
        float* const wf = reinterpret_cast<float*>(wl);
        int s = 0;
        // every part's weights in one gather (their loads in flight together); slot s =
        // the s-th set bit j of the visible-part mask (table in LDS: a register array with
        // a runtime index lives in scratch memory)
        if (tid < 32 && ((mask >> tid) & 1u)) jofs[__popc(mask & ((1u << tid) - 1u))] = tid;
        __syncthreads();
        s = __popc(mask);
        coop_gather<8>(wf, s * KK * kMaxCo, tid, kThreads, a.w, [&](int i) {
            const int co = i % kMaxCo, r = i / kMaxCo, tap = r % KK, sl = r / KK;
            return co < a.Co ? (co * a.Ci + a.c_kp0 + jofs[sl]) * KK + tap : -1;
        });
        for (int t = tid; t < KK; t += kThreads) {
            const int kh = t / a.KW, kw = t - kh * a.KW;
            toff[t] = kh * a.DH * a.FW + kw * a.DW;
        }
    }
    const int py = tid / kTile, px = tid - py * kTile;
    const int hbase = py * a.SH * a.FW + px * a.SW;
    f32x4 acc[kMaxCo / 4];
#pragma unroll
    for (int c = 0; c < kMaxCo / 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (uint32_t m = mask; m; m &= m - 1, ++s) {
        const int j = __ffs(m) - 1;
        const Win w = wins[j];
        __syncthreads();  // previous part's map consumed (and wl / toff written, first time)
        for (int i = tid; i < a.FH * a.FW; i += kThreads) {
            const int r = i / a.FW, c = i - r * a.FW;
            hl[i] = heat(a, w, iy0 + r, ix0 + c);
        }
        __syncthreads();
        const f32x4* wp = wl + s * KK * (kMaxCo / 4);
        int t = 0;
        for (; t + 5 <= KK; t += 5) {
            float h[5];
#pragma unroll
            for (int u = 0; u < 5; ++u) h[u] = hl[hbase + toff[t + u]];
#pragma unroll
            for (int u = 0; u < 5; ++u)
#pragma unroll
                for (int c = 0; c < kMaxCo / 4; ++c) acc[c] += wp[(t + u) * (kMaxCo / 4) + c] * h[u];
        }
        for (; t < KK; ++t) {
            const float h = hl[hbase + toff[t]];
#pragma unroll
            for (int c = 0; c < kMaxCo / 4; ++c) acc[c] += wp[t * (kMaxCo / 4) + c] * h;
        }
    }
    // apply + statistics change (sum, sum of squares) of the stored values
    const int oy = oy0 + py, ox = ox0 + px;
    const bool in = oy < a.OH && ox < a.OW;
    float d0[kMaxCo], d1[kMaxCo];
#pragma unroll
    for (int c = 0; c < kMaxCo; ++c) {
        d0[c] = d1[c] = 0.f;
        if (c < a.Co && in) {
            const int64_t o = (int64_t)n * a.y_ns + ((int64_t)c * a.OH + oy) * a.OW + ox;
            const float v = gld(a.y, o);
            const float nv = v + acc[c >> 2][c & 3];
            gst(a.y, o, nv);
            d0[c] = nv - v;
            d1[c] = (nv - v) * (nv + v);
        }
    }
    if (!a.stats) return;
#pragma unroll
    for (int c = 0; c < kMaxCo; ++c) {
        if (c >= a.Co) break;
        const float t0 = wave_sum(d0[c]), t1 = wave_sum(d1[c]);
        if (lane == 0) {
            red[0][wave][c] = t0;
            red[1][wave][c] = t1;
        }
    }
    __syncthreads();
    if (tid < a.Co) {
        double* sp = rep_ptr(a.stats, 4 * a.Co);
        const float t0 = ((red[0][0][tid] + red[0][1][tid]) + red[0][2][tid]) + red[0][3][tid];
        const float t1 = ((red[1][0][tid] + red[1][1][tid]) + red[1][2][tid]) + red[1][3][tid];
        atomicAdd(&sp[tid], (double)t0);
        atomicAdd(&sp[a.Co + tid], (double)t1);
    }
}

// ---- weight gradient of the heatmap channels -----------------------------------------
// block (image * nparts + part, row band): dw[co][c_kp0+part][tap] over the output pixels
// of its band whose taps reach the window, staged in chunks of <= 256 pixels
__global__ __launch_bounds__(kThreads) void kp_wgrad_kernel(KpArgs a) {
    __shared__ float hl[kMaxWgFoot];
    __shared__ float dyl[kMaxCo * kMaxWgPix];
    __shared__ ChT taby[kMaxCo];
    const int tid = threadIdx.x;
    const int n = blockIdx.x / a.nparts, j = blockIdx.x - n * a.nparts;
    const Win w = part_window(a, n, j);
    if (w.x1 <= w.x0 || w.y1 <= w.y0) return;
    // output pixels with a tap in the window
    const int oy_lo = max(0, ceil_div(w.y0 + a.PH - a.DH * (a.KH - 1), a.SH));
    const int oy_hi = min(a.OH - 1, floor_div(w.y1 - 1 + a.PH, a.SH));
    const int ox_lo = max(0, ceil_div(w.x0 + a.PW - a.DW * (a.KW - 1), a.SW));
    const int ox_hi = min(a.OW - 1, floor_div(w.x1 - 1 + a.PW, a.SW));
    if (oy_hi < oy_lo || ox_hi < ox_lo) return;
    const int nrow = oy_hi - oy_lo + 1, ncol = ox_hi - ox_lo + 1;
    const int band = (nrow + gridDim.y - 1) / gridDim.y;
    const int r_lo = oy_lo + blockIdx.y * band, r_hi = min(oy_hi + 1, r_lo + band);
    if (r_lo >= r_hi) return;
    for (int c = tid; c < a.Co; c += kThreads) taby[c] = ch_table_entry(a.dy, c, a.OH * a.OW);
    const int rows_per = max(1, kMaxWgPix / ncol);
    const int fw = (ncol - 1) * a.SW + a.DW * (a.KW - 1) + 1;
    const int ix0 = ox_lo * a.SW - a.PW;
    const int npair = a.Co * a.KK;
    float acc[2] = {0.f, 0.f};
    for (int r0 = r_lo; r0 < r_hi; r0 += rows_per) {
        const int nr = min(rows_per, r_hi - r0);
        const int np = nr * ncol;
        const int fh = (nr - 1) * a.SH + a.DH * (a.KH - 1) + 1;
        const int iy0 = r0 * a.SH - a.PH;
        __syncthreads();  // previous chunk consumed (and taby written)
        for (int i = tid; i < fh * fw; i += kThreads) {
            const int r = i / fw, c = i - r * fw;
            hl[i] = heat(a, w, iy0 + r, ix0 + c);
        }
        // 4 items per thread with their loads in flight together (ChT.y == p unless
        // BatchNorm backward, so the second load needs no branch)
        for (int i0 = tid; i0 < a.Co * np; i0 += 4 * kThreads) {
            float g[4], yv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = min(i0 + u * kThreads, a.Co * np - 1);
                const int co = i / np, p = i - co * np;
                const int pr = p / ncol, pc = p - pr * ncol;
                const int64_t pix = (int64_t)(r0 + pr) * a.OW + ox_lo + pc;
                const ChT& t = taby[co];
                g[u] = gld(t.p, (int64_t)n * t.ns + pix);
                yv[u] = gld(t.y, (int64_t)n * t.yns + pix);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + u * kThreads;
                if (i >= a.Co * np) continue;
                const int co = i / np, p = i - co * np;
                const ChT& t = taby[co];
                dyl[co * kMaxWgPix + p] = ch_xform(t.xf, t.act, t.k, g[u], yv[u]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + u * kThreads;
            if (e >= npair) continue;
            const int co = e / a.KK, tap = e - co * a.KK;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            const float* dr = dyl + co * kMaxWgPix;
            const float* hr = hl + kh * a.DH * fw + kw * a.DW;
            float s4[4] = {0.f, 0.f, 0.f, 0.f};
            for (int pr = 0; pr < nr; ++pr) {
                const float* d = dr + pr * ncol;
                const float* hh = hr + pr * a.SH * fw;
                int pc = 0;
                for (; pc + 4 <= ncol; pc += 4)
#pragma unroll
                    for (int q = 0; q < 4; ++q) s4[q] += d[pc + q] * hh[(pc + q) * a.SW];
                for (; pc < ncol; ++pc) s4[0] += d[pc] * hh[pc * a.SW];
            }
            acc[u] += (s4[0] + s4[1]) + (s4[2] + s4[3]);
        }
    }
    double* const dwr = a.dw + (int64_t)((blockIdx.x + 7u * blockIdx.y) % (unsigned)a.nrep) * a.rep_stride;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = tid + u * kThreads;
        if (e >= npair) continue;
        const int co = e / a.KK, tap = e - co * a.KK;
        atomicAdd(&dwr[((int64_t)co * a.Ci + a.c_kp0 + j) * a.KK + tap], acc[u]);
    }
}

// ---- max_pool(k) of the heatmap channels (segment.py:31), dense ------------------------
// The map decreases with the distance to the keypoint, so the maximum over a k x k cell is
// the value at the cell pixel inside the window nearest to the keypoint (one exp per
// pooled pixel; a distance tie gives the same value either way).
__global__ __launch_bounds__(kThreads) void kp_pool_kernel(KpArgs a) {
    __shared__ Win ws;
    const int j = blockIdx.y, n = blockIdx.z;
    if (threadIdx.x == 0) ws = part_window(a, n, j);
    __syncthreads();
    const Win w = ws;
    const int PH = a.H / a.k, PW = a.W / a.k;
    const int64_t o = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (o >= (int64_t)PH * PW) return;
    const int py = (int)(o / PW), px = (int)(o - (int64_t)py * PW);
    const int xl = max(px * a.k, w.x0), xh = min(px * a.k + a.k, w.x1) - 1;
    const int yl = max(py * a.k, w.y0), yh = min(py * a.k + a.k, w.y1) - 1;
    float m = 0.f;
    if (xl <= xh && yl <= yh) {
        const int ix = min(max((int)floor(w.kx + 0.5), xl), xh);
        const int iy = min(max((int)floor(w.ky + 0.5), yl), yh);
        m = heat(a, w, iy, ix);
    }
    gst(a.out, (int64_t)n * a.out_ns + (int64_t)j * PH * PW + o, m);
}

int32_t kp_args(const isg_kp_stem* s, KpArgs& a, bool conv) {
    if (!s || !s->kp || s->nparts < 1 || s->nparts > kMaxParts || !(s->sigma > 0.0) ||
        !(s->threshold > 0.0) || !(s->threshold < 1.0))
        return isg_set_error(ISG_ERR_INVALID, "kp_stem: bad keypoint arguments");
    const isg_conv_geom& g = s->g;
    a = KpArgs{};
    a.kp = s->kp;
    a.nparts = s->nparts;
    a.c_kp0 = s->c_kp0;
    a.s2 = s->sigma * s->sigma;
    a.thr = s->threshold;
    a.r = std::sqrt(std::log(s->threshold) * (-a.s2));  // train_instance.py:35
    a.N = g.N; a.Ci = g.Ci; a.H = g.H; a.W = g.W; a.Co = g.Co; a.OH = g.OH; a.OW = g.OW;
    a.KH = g.KH; a.KW = g.KW; a.SH = g.SH; a.SW = g.SW; a.PH = g.PH; a.PW = g.PW;
    a.DH = g.DH; a.DW = g.DW; a.KK = g.KH * g.KW;
    if (a.N < 1 || a.H < 1 || a.W < 1)
        return isg_set_error(ISG_ERR_INVALID, "kp_stem: bad geometry");
    if (a.r > 120.0)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "kp_stem: keypoint radius %.1f > 120", a.r);
    if (!conv) return ISG_OK;
    if (g.groups != 1 || a.Co < 1 || a.Co > kMaxCo || a.KK > kMaxKK || a.SH < 1 || a.SW < 1 ||
        a.DH < 1 || a.DW < 1 || a.c_kp0 < 0 || a.c_kp0 + a.nparts != a.Ci)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "kp_stem: conv Co %d Ci %d (keypoint channels %d+%d) k%dx%d",
                             a.Co, a.Ci, a.c_kp0, a.nparts, a.KH, a.KW);
    a.FH = a.SH * (kTile - 1) + a.DH * (a.KH - 1) + 1;
    a.FW = a.SW * (kTile - 1) + a.DW * (a.KW - 1) + 1;
    if (a.FH > kMaxFoot || a.FW > kMaxFoot)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "kp_stem: footprint %dx%d", a.FH, a.FW);
    return ISG_OK;
}

}  // namespace

extern "C" {

int32_t isg_kp_stem_fwd(const isg_kp_stem* s, isg_stream_t st) {
    KpArgs a;
    if (int32_t e = kp_args(s, a, true)) return e;
    if (!s->w || !s->y) return isg_set_error(ISG_ERR_INVALID, "kp_stem_fwd: NULL weight / output");
    a.w = s->w; a.y = s->y; a.y_ns = s->y_n_stride; a.stats = s->stats;
    // the active parts' weights: Co x nact x KK floats in LDS
    if (kMaxCo * a.nparts * a.KK > kMaxWl)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "kp_stem_fwd: %d parts x %d taps", a.nparts, a.KK);
    a.tiles_x = (a.OW + kTile - 1) / kTile;
    const int tiles_y = (a.OH + kTile - 1) / kTile;
    hipLaunchKernelGGL(kp_fwd_kernel, dim3((unsigned)(a.tiles_x * tiles_y), (unsigned)a.N),
                       dim3(kThreads), 0, st, a);
    return isg_check_launch("kp_fwd_kernel");
}

int32_t isg_kp_stem_wgrad(const isg_kp_stem* s, isg_stream_t st) {
    KpArgs a;
    if (int32_t e = kp_args(s, a, true)) return e;
    if (isg_vt_res(&s->dy)) return isg_set_error(ISG_ERR_UNSUPPORTED, "kp stem wgrad: residual form");
    if (!s->dw || s->dy.nseg != 1 || s->dy.s[0].C != a.Co)
        return isg_set_error(ISG_ERR_INVALID, "kp_stem_wgrad: dw / dy (one segment of Co channels)");
    if (s->nrep < 1 || (s->nrep > 1 && s->rep_stride <= 0))
        return isg_set_error(ISG_ERR_INVALID, "kp_stem_wgrad: bad replicas");
    if (a.Co * a.KK > 2 * kThreads)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "kp_stem_wgrad: %d x %d taps", a.Co, a.KK);
    // the widest window reaches (2r+2)/SW + KW output columns; its footprint must fit
    const int wmax = (int)(2.0 * a.r) + 2;
    const int ncol = wmax / a.SW + a.KW + 1;
    const int rows_per = std::max(1, kMaxWgPix / ncol);
    const int fw = (ncol - 1) * a.SW + a.DW * (a.KW - 1) + 1;
    const int fh = (rows_per - 1) * a.SH + a.DH * (a.KH - 1) + 1;
    if (ncol > kMaxWgPix || fw * fh > kMaxWgFoot)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "kp_stem_wgrad: window footprint %dx%d", fh, fw);
    a.dy = s->dy; a.dw = s->dw;
    a.rep_stride = s->nrep > 1 ? s->rep_stride : 0;
    a.nrep = s->nrep;
    hipLaunchKernelGGL(kp_wgrad_kernel, dim3((unsigned)(a.N * a.nparts), 4u), dim3(kThreads), 0, st, a);
    return isg_check_launch("kp_wgrad_kernel");
}

int32_t isg_kp_pool(const isg_kp_stem* s, isg_stream_t st) {
    KpArgs a;
    if (int32_t e = kp_args(s, a, false)) return e;
    if (!s->out || s->k < 1 || a.H % s->k || a.W % s->k)
        return isg_set_error(ISG_ERR_INVALID, "kp_pool: output / window %d for %dx%d", s->k, a.H, a.W);
    a.k = s->k; a.out = s->out; a.out_ns = s->out_n_stride;
    const int64_t np = (int64_t)(a.H / a.k) * (a.W / a.k);
    hipLaunchKernelGGL(kp_pool_kernel, dim3((unsigned)((np + kThreads - 1) / kThreads), (unsigned)a.nparts, (unsigned)a.N),
                       dim3(kThreads), 0, st, a);
    return isg_check_launch("kp_pool_kernel");
}

}  // extern "C"
