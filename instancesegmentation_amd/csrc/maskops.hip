// Infer post-process: per-instance mask paste-back (A13) and greedy mask-NMS (A14).
//
// The reference has no implementation (infer.py:32-36 is a stub);
// the contract is frozen in oracle/maskops_oracle.py and these kernels are bit-exact
// to it: every float op is a single IEEE op in the oracle's order (contraction off,
// correctly rounded division), everything after the paste is integer.
#include <algorithm>

#include "common.h"

namespace {

constexpr int kThreads = 256;

// Writes the instance's window only (the canvas is zeroed by isg_mask_paste first):
// blocks of instance k walk the clipped window [cx0,cx1) x [cy0,cy1).
constexpr int kPasteBlocks = 64;  // blocks per instance (grid-stride over the window)

// The A13 contract for canvas pixel (x, y) of instance window (x0, y0, x1, y1) with
// scales (sx, sy) = S / window size: one fp32 IEEE op at a time, oracle order.
ISG_DEV uint8_t paste_px(const float* __restrict__ p, int S, int x0, int y0, float sx, float sy,
                         int x, int y) {
#pragma clang fp contract(off)
    float fx = ((float)(x - x0) + 0.5f) * sx - 0.5f;
    float fy = ((float)(y - y0) + 0.5f) * sy - 0.5f;
    fx = fx < 0.f ? 0.f : fx;
    fy = fy < 0.f ? 0.f : fy;
    const int ix = (int)fx, iy = (int)fy;
    const float ax = fx - (float)ix, ay = fy - (float)iy;
    const int ix1 = ix + 1 < S ? ix + 1 : S - 1;
    const int iy1 = iy + 1 < S ? iy + 1 : S - 1;
    const float p00 = p[(int64_t)iy * S + ix], p01 = p[(int64_t)iy * S + ix1];
    const float p10 = p[(int64_t)iy1 * S + ix], p11 = p[(int64_t)iy1 * S + ix1];
    const float bx = 1.f - ax, by = 1.f - ay;
    const float top = (bx * p00) + (ax * p01);
    const float bot = (bx * p10) + (ax * p11);
    const float v = (by * top) + (ay * bot);
    return (uint8_t)(int)(v * 255.f);
}

__global__ __launch_bounds__(kThreads) void paste_kernel(const float* __restrict__ prob, int S,
                                                          const int32_t* __restrict__ boxes, int H,
                                                          int W, uint8_t* __restrict__ out) {
#pragma clang fp contract(off)
    const int k = blockIdx.y;
    const int x0 = boxes[4 * k], y0 = boxes[4 * k + 1], x1 = boxes[4 * k + 2], y1 = boxes[4 * k + 3];
    if (x1 <= x0 || y1 <= y0) return;
    const int cx0 = max(x0, 0), cx1 = min(x1, W), cy0 = max(y0, 0), cy1 = min(y1, H);
    if (cx1 <= cx0 || cy1 <= cy0) return;
    const int ww = cx1 - cx0;
    const int64_t area = (int64_t)ww * (cy1 - cy0);
    const float sx = (float)S / (float)(x1 - x0);
    const float sy = (float)S / (float)(y1 - y0);
    const float* p = prob + (int64_t)k * S * S;
    uint8_t* o = out + (int64_t)k * H * W;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < area;
         i += (int64_t)kPasteBlocks * kThreads) {
        const int y = cy0 + (int)(i / ww), x = cx0 + (int)(i % ww);
        o[(int64_t)y * W + x] = paste_px(p, S, x0, y0, sx, sy, x, y);
    }
}

struct NmsWork {
    unsigned long long* bits;  // [K][words]
    unsigned long long* cnt;   // [K]
    unsigned long long* sum;   // [K]
    int64_t* inter;            // [K][K]
};

NmsWork carve(void* work, int K, int64_t words) {
    char* p = (char*)work;
    NmsWork w;
    w.bits = (unsigned long long*)p;
    p += (size_t)K * words * 8;
    w.cnt = (unsigned long long*)p;
    p += (size_t)K * 8;
    w.sum = (unsigned long long*)p;
    p += (size_t)K * 8;
    w.inter = (int64_t*)p;
    return w;
}

// Bit-packing of mask >= 128, coalesced: a wave reads 256 consecutive bytes (4 per lane)
// and ballots them into 4 words; word 4g+j holds byte j of every lane of 256-pixel
// group g. The bit order is internal to the workspace (every mask uses the same one, so
// AND-popcount intersections are unchanged); counts and sums are exact integers.
__global__ __launch_bounds__(kThreads) void pack_kernel(const uint8_t* __restrict__ m, int64_t hw,
                                                         int64_t words, NmsWork w) {
    __shared__ unsigned long long sc[4], ss[4];
    const int k = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint8_t* src = m + (int64_t)k * hw;
    const int64_t groups = words / 4;
    unsigned long long cnt = 0, sum = 0;
    for (int64_t g = (int64_t)blockIdx.x * 4 + wave; g < groups; g += (int64_t)gridDim.x * 4) {
        const int64_t base = g * 256 + 4 * lane;
        uint32_t v4 = 0;
        if (base + 3 < hw && ((hw & 3) == 0)) {
            v4 = *reinterpret_cast<const uint32_t*>(src + base);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (base + j < hw) v4 |= (uint32_t)src[base + j] << (8 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned v = (v4 >> (8 * j)) & 0xffu;
            const bool on = v >= 128u;
            const unsigned long long b = __ballot(on);
            if (lane == 0) w.bits[(int64_t)k * words + 4 * g + j] = b;
            if (on) {
                cnt += 1;
                sum += v;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
        sum += __shfl_xor(sum, o, 64);
    }
    if (lane == 0) {
        sc[wave] = cnt;
        ss[wave] = sum;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&w.cnt[k], sc[0] + sc[1] + sc[2] + sc[3]);
        atomicAdd(&w.sum[k], ss[0] + ss[1] + ss[2] + ss[3]);
    }
}

// Paste-back and NMS bit-packing in one pass over the canvas (the product path): a wave
// owns 256-pixel groups of instance k's canvas, lane l the 4 pixels 256g + 4l .. + 3; it
// writes them (0 outside the clipped window) as one 4-B store and ballots mask >= 128 into
// words 4g + j exactly as pack_kernel does, with the exact integer count and sum. This
// replaces the canvas memset, paste_kernel and pack_kernel's re-read of the canvases
// (16 MB at K = 16, 1024^2). Groups whose rows miss the window skip the resampling.
__global__ __launch_bounds__(kThreads) void paste_pack_kernel(const float* __restrict__ prob, int S,
                                                               const int32_t* __restrict__ boxes,
                                                               int H, int W, int64_t words,
                                                               uint8_t* __restrict__ out, NmsWork w) {
    __shared__ unsigned long long sc[4], ss[4];
    const int k = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x0 = boxes[4 * k], y0 = boxes[4 * k + 1], x1 = boxes[4 * k + 2], y1 = boxes[4 * k + 3];
    const bool any = x1 > x0 && y1 > y0;
    const int cx0 = max(x0, 0), cx1 = min(x1, W), cy0 = max(y0, 0), cy1 = min(y1, H);
    const bool win = any && cx1 > cx0 && cy1 > cy0;
    const float sx = any ? (float)S / (float)(x1 - x0) : 0.f;
    const float sy = any ? (float)S / (float)(y1 - y0) : 0.f;
    const float* p = prob + (int64_t)k * S * S;
    const int64_t hw = (int64_t)H * W;
    uint8_t* o = out + (int64_t)k * hw;
    const int64_t groups = words / 4;
    const bool aligned = (hw & 3) == 0;
    unsigned long long cnt = 0, sum = 0;
    for (int64_t g = (int64_t)blockIdx.x * 4 + wave; g < groups; g += (int64_t)gridDim.x * 4) {
        const int64_t base = g * 256 + 4 * lane;
        // rows of the group: uniform test against the window
        const int64_t gy0 = (g * 256) / W, gy1 = min((int64_t)H - 1, (g * 256 + 255) / W);
        uint32_t v4 = 0;
        if (win && gy1 >= cy0 && gy0 < cy1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t px = base + j;
                if (px >= hw) continue;
                const int y = (int)(px / W), x = (int)(px - (int64_t)y * W);
                if (y >= cy0 && y < cy1 && x >= cx0 && x < cx1)
                    v4 |= (uint32_t)paste_px(p, S, x0, y0, sx, sy, x, y) << (8 * j);
            }
        }
        if (aligned && base + 3 < hw) {
            *reinterpret_cast<uint32_t*>(o + base) = v4;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (base + j < hw) o[base + j] = (uint8_t)(v4 >> (8 * j));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned v = (v4 >> (8 * j)) & 0xffu;
            const bool on = v >= 128u;
            const unsigned long long b = __ballot(on);
            if (lane == 0) w.bits[(int64_t)k * words + 4 * g + j] = b;
            if (on) {
                cnt += 1;
                sum += v;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        cnt += __shfl_xor(cnt, off, 64);
        sum += __shfl_xor(sum, off, 64);
    }
    if (lane == 0) {
        sc[wave] = cnt;
        ss[wave] = sum;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&w.cnt[k], sc[0] + sc[1] + sc[2] + sc[3]);
        atomicAdd(&w.sum[k], ss[0] + ss[1] + ss[2] + ss[3]);
    }
}

__global__ __launch_bounds__(kThreads) void inter_kernel(int K, int64_t words, NmsWork w) {
    __shared__ unsigned long long sh[4];
    const int i = blockIdx.x, j = blockIdx.y;
    if (j <= i) return;
    const unsigned long long* a = w.bits + (int64_t)i * words;
    const unsigned long long* b = w.bits + (int64_t)j * words;
    unsigned long long c = 0;
    for (int64_t t = threadIdx.x; t < words; t += kThreads) c += __popcll(a[t] & b[t]);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) sh[wave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int64_t v = (int64_t)(sh[0] + sh[1] + sh[2] + sh[3]);
        w.inter[(int64_t)i * K + j] = v;
        w.inter[(int64_t)j * K + i] = v;
    }
}

// one workgroup: scores, stable rank sort, greedy suppression (K <= kMaxNms)
constexpr int kMaxNms = 256;

__global__ __launch_bounds__(kMaxNms) void nms_kernel(int K, float thr, NmsWork w, float* scores_out,
                                                      int32_t* keep, int32_t* nkeep) {
#pragma clang fp contract(off)
    __shared__ float sc[kMaxNms];
    __shared__ int order[kMaxNms];
    __shared__ int sup[kMaxNms];
    const int t = threadIdx.x;
    float s = 0.f;
    if (t < K) {
        const unsigned long long c = w.cnt[t];
        if (c > 0) s = (float)w.sum[t] / ((float)c * 255.f);
        sc[t] = s;
        scores_out[t] = s;
        sup[t] = 0;
    }
    __syncthreads();
    int rank = 0;  // this instance's position in the (-score, index) order
    if (t < K) {
        for (int j = 0; j < K; ++j) {
            const float sj = sc[j];
            rank += (sj > s || (sj == s && j < t)) ? 1 : 0;
        }
        order[rank] = t;
    }
    __syncthreads();
    int nk = 0;
    for (int a = 0; a < K; ++a) {
        const int i = order[a];
        const bool alive = sup[i] == 0;  // uniform: read before any write this step
        __syncthreads();
        if (!alive) continue;
        if (t == 0) keep[nk] = i;
        ++nk;
        if (t < K && rank > a && sup[t] == 0) {
            const int64_t in = w.inter[(int64_t)i * K + t];
            const int64_t u = (int64_t)w.cnt[i] + (int64_t)w.cnt[t] - in;
            const float iou = u > 0 ? (float)in / (float)u : 0.f;
            if (iou > thr) sup[t] = 1;
        }
        __syncthreads();
    }
    if (t == 0) *nkeep = nk;
}

}  // namespace

extern "C" {

int32_t isg_mask_paste(const float* prob, int32_t K, int32_t S, const int32_t* boxes, int32_t H,
                       int32_t W, uint8_t* out, isg_stream_t st) {
    if (K <= 0) return 0;
    if (S <= 0 || H <= 0 || W <= 0) return isg_set_error(ISG_ERR_INVALID, "paste: bad sizes");
    if (hipMemsetAsync(out, 0, (size_t)K * H * W, st) != hipSuccess)
        return isg_check_launch("paste memset");
    dim3 grid((unsigned)kPasteBlocks, (unsigned)K);
    hipLaunchKernelGGL(paste_kernel, grid, dim3(kThreads), 0, st, prob, S, boxes, H, W, out);
    return isg_check_launch("paste_kernel");
}

// packed words per mask: 4 per 256-pixel group (pack_kernel)
static int64_t nms_words(int64_t hw) { return (hw + 255) / 256 * 4; }

int64_t isg_mask_nms_workspace(int32_t K, int32_t H, int32_t W) {
    const int64_t words = nms_words((int64_t)H * W);
    return (int64_t)K * words * 8 + (int64_t)K * 16 + (int64_t)K * K * 8;
}

int32_t isg_mask_paste_nms(const float* prob, int32_t K, int32_t S, const int32_t* boxes, int32_t H,
                           int32_t W, float iou_thr, uint8_t* masks, void* work, float* scores_out,
                           int32_t* keep, int32_t* nkeep, isg_stream_t st) {
    if (K < 0 || K > kMaxNms)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "paste+nms: K=%d (max %d)", K, kMaxNms);
    if (K == 0) {
        (void)hipMemsetAsync(nkeep, 0, sizeof(int32_t), st);
        return isg_check_launch("nms memset");
    }
    if (S <= 0 || H <= 0 || W <= 0) return isg_set_error(ISG_ERR_INVALID, "paste+nms: bad sizes");
    const int64_t hw = (int64_t)H * W;
    const int64_t words = nms_words(hw);
    NmsWork w = carve(work, K, words);
    (void)hipMemsetAsync(w.cnt, 0, (size_t)K * 16, st);
    (void)hipMemsetAsync(w.inter, 0, (size_t)K * K * 8, st);
    const int64_t gblocks = std::min<int64_t>((words / 4 + 3) / 4, 256);
    hipLaunchKernelGGL(paste_pack_kernel, dim3((unsigned)gblocks, K), dim3(kThreads), 0, st, prob, S,
                       boxes, H, W, words, masks, w);
    hipLaunchKernelGGL(inter_kernel, dim3(K, K), dim3(kThreads), 0, st, K, words, w);
    hipLaunchKernelGGL(nms_kernel, dim3(1), dim3(kMaxNms), 0, st, K, iou_thr, w, scores_out, keep,
                       nkeep);
    return isg_check_launch("paste+nms kernels");
}

int32_t isg_mask_nms(const uint8_t* masks, int32_t K, int32_t H, int32_t W, float iou_thr,
                     void* work, float* scores_out, int32_t* keep, int32_t* nkeep,
                     isg_stream_t st) {
    if (K < 0 || K > kMaxNms)
        return isg_set_error(ISG_ERR_UNSUPPORTED, "nms: K=%d (max %d)", K, kMaxNms);
    if (K == 0) {
        (void)hipMemsetAsync(nkeep, 0, sizeof(int32_t), st);
        return isg_check_launch("nms memset");
    }
    const int64_t hw = (int64_t)H * W;
    const int64_t words = nms_words(hw);
    NmsWork w = carve(work, K, words);
    (void)hipMemsetAsync(w.cnt, 0, (size_t)K * 16, st);
    (void)hipMemsetAsync(w.inter, 0, (size_t)K * K * 8, st);
    const int64_t gblocks = std::min<int64_t>((words / 4 + 3) / 4, 256);
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)gblocks, K), dim3(kThreads), 0, st, masks, hw,
                       words, w);
    hipLaunchKernelGGL(inter_kernel, dim3(K, K), dim3(kThreads), 0, st, K, words, w);
    hipLaunchKernelGGL(nms_kernel, dim3(1), dim3(kMaxNms), 0, st, K, iou_thr, w, scores_out, keep,
                       nkeep);
    return isg_check_launch("nms kernels");
}

}  // extern "C"
