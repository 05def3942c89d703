// Infer post-process: per-instance mask paste-back (A13) and greedy mask-NMS (A14).
//
// The reference has no implementation (infer.py:32-36 is a stub);
// the contract is frozen in oracle/maskops_oracle.py and these kernels are bit-exact
// to it: every float op is a single IEEE op in the oracle's order (contraction off,
// correctly rounded division), everything after the paste is integer.
#include "common.h"

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void paste_kernel(const float* __restrict__ prob, int S,
                                                          const int32_t* __restrict__ boxes, int H,
                                                          int W, uint8_t* __restrict__ out) {
#pragma clang fp contract(off)
    const int k = blockIdx.y;
    const int64_t hw = (int64_t)H * W;
    const int64_t pix = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (pix >= hw) return;
    const int y = (int)(pix / W), x = (int)(pix - (int64_t)y * W);
    const int x0 = boxes[4 * k], y0 = boxes[4 * k + 1], x1 = boxes[4 * k + 2], y1 = boxes[4 * k + 3];
    uint8_t r = 0;
    if (x1 > x0 && y1 > y0 && x >= x0 && x < x1 && y >= y0 && y < y1) {
        const float sx = (float)S / (float)(x1 - x0);
        const float sy = (float)S / (float)(y1 - y0);
        float fx = ((float)(x - x0) + 0.5f) * sx - 0.5f;
        float fy = ((float)(y - y0) + 0.5f) * sy - 0.5f;
        fx = fx < 0.f ? 0.f : fx;
        fy = fy < 0.f ? 0.f : fy;
        const int ix = (int)fx, iy = (int)fy;
        const float ax = fx - (float)ix, ay = fy - (float)iy;
        const int ix1 = ix + 1 < S ? ix + 1 : S - 1;
        const int iy1 = iy + 1 < S ? iy + 1 : S - 1;
        const float* p = prob + (int64_t)k * S * S;
        const float p00 = p[(int64_t)iy * S + ix], p01 = p[(int64_t)iy * S + ix1];
        const float p10 = p[(int64_t)iy1 * S + ix], p11 = p[(int64_t)iy1 * S + ix1];
        const float bx = 1.f - ax, by = 1.f - ay;
        const float top = (bx * p00) + (ax * p01);
        const float bot = (bx * p10) + (ax * p11);
        const float v = (by * top) + (ay * bot);
        r = (uint8_t)(int)(v * 255.f);
    }
    out[(int64_t)k * hw + pix] = r;
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

__global__ __launch_bounds__(kThreads) void pack_kernel(const uint8_t* __restrict__ m, int64_t hw,
                                                         int64_t words, NmsWork w) {
    __shared__ unsigned long long sc[4], ss[4];
    const int k = blockIdx.y;
    const int64_t wd = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    unsigned long long bits = 0, cnt = 0, sum = 0;
    if (wd < words) {
        const uint8_t* src = m + (int64_t)k * hw + wd * 64;
        const int64_t lim = hw - wd * 64;
        const int n = lim < 64 ? (int)lim : 64;
        for (int i = 0; i < n; ++i) {
            const unsigned v = src[i];
            if (v >= 128u) {
                bits |= 1ull << i;
                cnt += 1;
                sum += v;
            }
        }
        w.bits[(int64_t)k * words + wd] = bits;
    }
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
        sum += __shfl_xor(sum, o, 64);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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

// one wave: scores, stable rank sort, greedy suppression (K <= 64)
__global__ __launch_bounds__(64) void nms_kernel(int K, float thr, NmsWork w, float* scores_out,
                                                 int32_t* keep, int32_t* nkeep) {
#pragma clang fp contract(off)
    __shared__ float sc[64];
    __shared__ int order[64];
    __shared__ int sup[64];
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
    if (t < K) {
        int r = 0;
        for (int j = 0; j < K; ++j) {
            const float sj = sc[j];
            r += (sj > s || (sj == s && j < t)) ? 1 : 0;
        }
        order[r] = t;
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
        if (t < K) {
            int pos = 0;
            for (int b = 0; b < K; ++b) pos = (order[b] == t) ? b : pos;
            if (pos > a && sup[t] == 0) {
                const int64_t in = w.inter[(int64_t)i * K + t];
                const int64_t u = (int64_t)w.cnt[i] + (int64_t)w.cnt[t] - in;
                const float iou = u > 0 ? (float)in / (float)u : 0.f;
                if (iou > thr) sup[t] = 1;
            }
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
    dim3 grid((unsigned)(((int64_t)H * W + kThreads - 1) / kThreads), K);
    hipLaunchKernelGGL(paste_kernel, grid, dim3(kThreads), 0, st, prob, S, boxes, H, W, out);
    return isg_check_launch("paste_kernel");
}

int64_t isg_mask_nms_workspace(int32_t K, int32_t H, int32_t W) {
    const int64_t words = ((int64_t)H * W + 63) / 64;
    return (int64_t)K * words * 8 + (int64_t)K * 16 + (int64_t)K * K * 8;
}

int32_t isg_mask_nms(const uint8_t* masks, int32_t K, int32_t H, int32_t W, float iou_thr,
                     void* work, float* scores_out, int32_t* keep, int32_t* nkeep,
                     isg_stream_t st) {
    if (K < 0 || K > 64) return isg_set_error(ISG_ERR_UNSUPPORTED, "nms: K=%d (max 64)", K);
    if (K == 0) {
        hipMemsetAsync(nkeep, 0, sizeof(int32_t), st);
        return isg_check_launch("nms memset");
    }
    const int64_t hw = (int64_t)H * W;
    const int64_t words = (hw + 63) / 64;
    NmsWork w = carve(work, K, words);
    hipMemsetAsync(w.cnt, 0, (size_t)K * 16, st);
    hipMemsetAsync(w.inter, 0, (size_t)K * K * 8, st);
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((words + kThreads - 1) / kThreads), K),
                       dim3(kThreads), 0, st, masks, hw, words, w);
    hipLaunchKernelGGL(inter_kernel, dim3(K, K), dim3(kThreads), 0, st, K, words, w);
    hipLaunchKernelGGL(nms_kernel, dim3(1), dim3(64), 0, st, K, iou_thr, w, scores_out, keep, nkeep);
    return isg_check_launch("nms kernels");
}

}  // extern "C"
