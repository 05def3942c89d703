// Infer pre-process on the GPU: the per-instance crop and the keypoint heatmaps that feed
// Segment(20).
//
// Crop (reference: train_instance.py:139-196, test branch). The reference translates the
// image so the person box is centred, crops/pads it to the instance box +/- 16 px and
// resizes that window to 480x480 (imgaug + cv2, both absent here: "parity unpinned";
// the contract is frozen in oracle/infer_oracle.py). Translation, crop and pad are integer
// moves, so the three collapse into one resampling of the window [x0,x1)x[y0,y1) of the
// ORIGINAL image: half-pixel-centre bilinear (cv2 INTER_LINEAR's mapping), sample
// coordinates clamped into the window (cv2's border on the materialised crop), pixels
// outside the instance's valid rectangle (the image, minus what the centring translation
// pushed out of the frame) are the fill value 0, the result rounded to uint8 and normalised like
// ToTensor + Normalize(0.5, 0.5) (train_instance.py:80-85). Every float op is one IEEE
// op in the oracle's order (contraction off).
//
// Heatmaps (train_instance.py:33-68): 17 maps per instance, exp(-(dx^2+dy^2)/sigma^2)
// evaluated in DOUBLE precision (numpy's float64 e_table) and stored as float32, only for
// 'vis' keypoints, only inside [max(0,int(x-r)), min(w-1,int(x+r+1))) (the last row and
// column are never written), only where the value exceeds the threshold. The launch
// writes the windows only; the caller's buffer is zeroed first (isg_keypoint_heatmaps).
#include <cmath>

#include "common.h"

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void crop_kernel(const uint8_t* __restrict__ img, int H, int W,
                                                         const int32_t* __restrict__ win,
                                                         const int32_t* __restrict__ valid, int S,
                                                         float* __restrict__ out) {
#pragma clang fp contract(off)
    const int k = blockIdx.y;
    const int64_t ss = (int64_t)S * S;
    const int64_t o = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (o >= ss) return;
    const int v = (int)(o / S), u = (int)(o - (int64_t)v * S);
    const int x0 = win[4 * k], y0 = win[4 * k + 1], x1 = win[4 * k + 2], y1 = win[4 * k + 3];
    float* dst = out + (int64_t)k * 3 * ss + o;
    if (x1 <= x0 || y1 <= y0) {
        dst[0] = -1.f; dst[ss] = -1.f; dst[2 * ss] = -1.f;  // empty window: all padding
        return;
    }
    const float sx = (float)(x1 - x0) / (float)S;
    const float sy = (float)(y1 - y0) / (float)S;
    const float fx = (((float)u + 0.5f) * sx - 0.5f) + (float)x0;
    const float fy = (((float)v + 0.5f) * sy - 0.5f) + (float)y0;
    const float flx = floorf(fx), fly = floorf(fy);
    const float ax = fx - flx, ay = fy - fly;
    const int ix = (int)flx, iy = (int)fly;
    const int cx0 = min(max(ix, x0), x1 - 1), cx1 = min(max(ix + 1, x0), x1 - 1);
    const int cy0 = min(max(iy, y0), y1 - 1), cy1 = min(max(iy + 1, y0), y1 - 1);
    const int vx0 = max(valid[4 * k], 0), vy0 = max(valid[4 * k + 1], 0);
    const int vx1 = min(valid[4 * k + 2], W), vy1 = min(valid[4 * k + 3], H);
    const bool ox0 = cx0 >= vx0 && cx0 < vx1, ox1 = cx1 >= vx0 && cx1 < vx1;
    const bool oy0 = cy0 >= vy0 && cy0 < vy1, oy1 = cy1 >= vy0 && cy1 < vy1;
    const float bx = 1.f - ax, by = 1.f - ay;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float s00 = (oy0 && ox0) ? (float)img[((int64_t)cy0 * W + cx0) * 3 + c] : 0.f;
        const float s01 = (oy0 && ox1) ? (float)img[((int64_t)cy0 * W + cx1) * 3 + c] : 0.f;
        const float s10 = (oy1 && ox0) ? (float)img[((int64_t)cy1 * W + cx0) * 3 + c] : 0.f;
        const float s11 = (oy1 && ox1) ? (float)img[((int64_t)cy1 * W + cx1) * 3 + c] : 0.f;
        const float top = (bx * s00) + (ax * s01);
        const float bot = (bx * s10) + (ax * s11);
        const float val = (by * top) + (ay * bot);
        int q = (int)(val + 0.5f);
        q = q < 0 ? 0 : (q > 255 ? 255 : q);
        dst[c * ss] = ((float)q / 255.f - 0.5f) / 0.5f;
    }
}

// one block per (instance, part): the keypoint's window only
__global__ __launch_bounds__(kThreads) void heatmap_kernel(const double* __restrict__ kp, int nparts,
                                                            int H, int W, double sigma2, double thr,
                                                            double r, float* __restrict__ out) {
#pragma clang fp contract(off)  // numpy's double arithmetic, operation for operation
    const int kpart = blockIdx.x;  // instance * nparts + part
    const double* q = kp + (int64_t)kpart * 3;
    if (!(q[2] > 0.0)) return;  // not 'vis'
    double x = q[0], y = q[1];
    if (!kp_coord(x, r, W) || !kp_coord(y, r, H)) return;  // non-finite: not visible
    // python int() truncates toward zero
    const int xmin = max(0, (int)(x - r)), xmax = min(W - 1, (int)(x + r + 1.0));
    const int ymin = max(0, (int)(y - r)), ymax = min(H - 1, (int)(y + r + 1.0));
    const int ww = xmax - xmin, wh = ymax - ymin;
    if (ww <= 0 || wh <= 0) return;
    float* dst = out + (int64_t)kpart * H * W;
    for (int i = threadIdx.x; i < ww * wh; i += kThreads) {
        const int yy = ymin + i / ww, xx = xmin + i % ww;
        const double dx = (double)xx - x, dy = (double)yy - y;
        const double e = exp(-(dx * dx + dy * dy) / sigma2);
        if (e > thr) dst[(int64_t)yy * W + xx] = (float)e;
    }
}

}  // namespace

extern "C" {

int32_t isg_instance_crop(const uint8_t* image, int32_t H, int32_t W, const int32_t* windows,
                          const int32_t* valid, int32_t K, int32_t S, float* out,
                          isg_stream_t st) {
    if (K <= 0) return 0;
    if (!image || !windows || !valid || !out || H <= 0 || W <= 0 || S <= 0)
        return isg_set_error(ISG_ERR_INVALID, "instance_crop: bad arguments");
    dim3 grid((unsigned)(((int64_t)S * S + kThreads - 1) / kThreads), (unsigned)K);
    hipLaunchKernelGGL(crop_kernel, grid, dim3(kThreads), 0, st, image, H, W, windows, valid, S,
                       out);
    return isg_check_launch("crop_kernel");
}

int32_t isg_keypoint_heatmaps(const double* keypoints, int32_t K, int32_t nparts, int32_t H,
                              int32_t W, double sigma, double threshold, float* out,
                              isg_stream_t st) {
    if (K <= 0 || nparts <= 0) return 0;
    if (!keypoints || !out || H <= 0 || W <= 0 || !(sigma > 0.0) || !(threshold > 0.0) ||
        !(threshold < 1.0))
        return isg_set_error(ISG_ERR_INVALID, "keypoint_heatmaps: bad arguments");
    if (hipMemsetAsync(out, 0, (size_t)K * nparts * H * W * sizeof(float), st) != hipSuccess)
        return isg_check_launch("keypoint_heatmaps memset");
    // r = sqrt(log(threshold) * (-sigma^2)) in double (train_instance.py:35)
    const double s2 = sigma * sigma;
    const double r = std::sqrt(std::log(threshold) * (-s2));
    hipLaunchKernelGGL(heatmap_kernel, dim3((unsigned)(K * nparts)), dim3(kThreads), 0, st,
                       keypoints, nparts, H, W, s2, threshold, r, out);
    return isg_check_launch("heatmap_kernel");
}

}  // extern "C"
