// Kernel micro-benchmark harness: times one libisg op in isolation on synthetic data and
// dumps per-workgroup s_memrealtime stamps (libisg_stamp.so, built with -DISG_STAMPS).
//   kbench wgrad|fwd|dgrad N Ci H W Co k s p d [reps]
// Output: avg us per launch (hipEvent over reps), then stamp statistics of the last launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/isg.h"

#include <dlfcn.h>

// stamp buffers exist only in libisg_stamp.so (-DISG_STAMPS); against libisg.so the
// harness times launches only
static void* stamps(const char* name) {
    auto f = (void* (*)(void))dlsym(RTLD_DEFAULT, name);
    return f ? f() : nullptr;
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

static float* dalloc(size_t n, float v = 0.f, unsigned seed = 1) {
    std::vector<float> h(n);
    srand(seed);
    for (size_t i = 0; i < n; ++i) h[i] = v != 0.f ? v : (float)rand() / RAND_MAX - 0.5f;
    float* d;
    CK(hipMalloc(&d, n * sizeof(float)));
    CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    return d;
}

int main(int argc, char** argv) {
    if (argc < 11) {
        fprintf(stderr, "usage: kbench wgrad|fwd|dgrad N Ci H W Co k s p d [reps]\n");
        return 2;
    }
    const int N = atoi(argv[2]), Ci = atoi(argv[3]), H = atoi(argv[4]), W = atoi(argv[5]),
              Co = atoi(argv[6]), k = atoi(argv[7]), s = atoi(argv[8]), p = atoi(argv[9]),
              d = atoi(argv[10]);
    const int reps = argc > 11 ? atoi(argv[11]) : 50;
    const char* op = argv[1];
    isg_conv_geom g{};
    g.N = N; g.Ci = Ci; g.H = H; g.W = W; g.Co = Co; g.KH = g.KW = k; g.SH = g.SW = s;
    g.PH = g.PW = p; g.DH = g.DW = d; g.groups = 1;
    g.OH = (H + 2 * p - d * (k - 1) - 1) / s + 1;
    g.OW = (W + 2 * p - d * (k - 1) - 1) / s + 1;
    const size_t nx = (size_t)N * Ci * H * W, ny = (size_t)N * Co * g.OH * g.OW;
    float* x = dalloc(nx, 0.f, 1);
    float* dy = dalloc(ny, 0.f, 2);
    float* yraw = dalloc(ny, 0.f, 3);
    float* gam = dalloc(std::max(Ci, Co), 1.f);
    float* bet = dalloc(std::max(Ci, Co), 0.1f);
    float* slope = dalloc(std::max(Ci, Co), 0.25f);
    double* stats;
    const int C4 = 4 * std::max(Ci, Co) * ISG_STAT_REP;
    CK(hipMalloc(&stats, C4 * sizeof(double)));
    std::vector<double> hs(C4, 0.5);
    CK(hipMemcpy(stats, hs.data(), C4 * sizeof(double), hipMemcpyHostToDevice));
    const int64_t nw = (int64_t)Co * Ci * k * k;
    double* dw;  // fp64 weight-gradient replicas (isg.h ISG_WREP)
    CK(hipMalloc(&dw, ISG_WREP * nw * sizeof(double)));
    float* wt = dalloc(nw, 0.f, 4);
    float* out;
    CK(hipMalloc(&out, std::max(nx, ny) * sizeof(float)));
    double* ostats;
    CK(hipMalloc(&ostats, C4 * sizeof(double)));
    double* sgrad;
    CK(hipMalloc(&sgrad, std::max(Ci, Co) * ISG_STAT_REP * sizeof(double)));
    // dy: BN backward rebuilt (the common case); x: BN fwd + PReLU
    isg_vtensor vdy{}, vx{};
    vdy.nseg = 1; vdy.N = N; vdy.H = g.OH; vdy.W = g.OW;
    vdy.s[0].p = dy; vdy.s[0].y = yraw; vdy.s[0].n_stride = (int64_t)Co * g.OH * g.OW;
    vdy.s[0].y_n_stride = vdy.s[0].n_stride; vdy.s[0].C = Co; vdy.s[0].xform = ISG_XF_BN_BWD;
    vdy.s[0].bn = isg_bn{gam, bet, nullptr, nullptr, stats, Co, 1, (float)(N * g.OH * g.OW), 1e-5f};
    vx.nseg = 1; vx.N = N; vx.H = H; vx.W = W;
    vx.s[0].p = x; vx.s[0].n_stride = (int64_t)Ci * H * W; vx.s[0].C = Ci;
    vx.s[0].xform = ISG_XF_BN_FWD; vx.s[0].act = ISG_ACT_PRELU; vx.s[0].slope = slope;
    vx.s[0].bn = isg_bn{gam, bet, nullptr, nullptr, stats, Ci, 1, (float)(N * H * W), 1e-5f};
    // KB_COEF=1: finalised BatchNorm coefficients (isg_bn.coef), as the training graph has them
    if (getenv("KB_COEF")) {
        const int Cm = std::max(Ci, Co);
        std::vector<float> hc(8 * Cm);
        for (int c = 0; c < Cm; ++c) {
            float* f = &hc[4 * c];
            f[0] = 0.1f; f[1] = 1.0f; f[2] = 0.1f; f[3] = 0.f;
            float* b = &hc[4 * (Cm + c)];
            b[0] = 1.0f; b[1] = -0.01f; b[2] = 0.1f; b[3] = 0.001f;
        }
        float* coef;
        CK(hipMalloc(&coef, hc.size() * sizeof(float)));
        CK(hipMemcpy(coef, hc.data(), hc.size() * sizeof(float), hipMemcpyHostToDevice));
        vdy.s[0].bn.coef = coef; vdy.s[0].bn.C = Cm;
        vx.s[0].bn.coef = coef; vx.s[0].bn.C = Cm;
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    // forward: STORE sink with BN statistics; dgrad: ACTBWD sink (BN + PReLU backward)
    isg_sinks sk{};
    sk.nsink = 1;
    isg_sink& s0 = sk.s[0];
    if (!strcmp(op, "fwd")) {
        s0.p = out; s0.n_stride = (int64_t)Co * g.OH * g.OW; s0.C = Co; s0.mode = ISG_SINK_STORE;
        s0.bias = bet; s0.stats = ostats;
    } else {
        s0.p = out; s0.n_stride = (int64_t)Ci * H * W; s0.C = Ci; s0.mode = ISG_SINK_ACTBWD;
        s0.act = ISG_ACT_PRELU; s0.y = x; s0.y_n_stride = s0.n_stride; s0.slope = slope;
        s0.slope_grad = sgrad;
        s0.bn = isg_bn{gam, bet, nullptr, nullptr, ostats, Ci, 1, (float)(N * H * W), 1e-5f};
        if (getenv("KB_COEF")) { s0.bn.coef = vx.s[0].bn.coef; s0.bn.C = vx.s[0].bn.C; }
    }
    // mask head (isg_mask_head_*): x = Ci(16) x H x W plain, logits 4H x 4W
    isg_mask_head mh{};
    float *hw1 = nullptr, *hw2 = nullptr, *hdl = nullptr, *hdx = nullptr;
    double* hrep = nullptr;
    if (!strncmp(op, "head", 4)) {
        vx.s[0].xform = ISG_XF_PLAIN;
        mh.x = vx;
        hw1 = dalloc(16 * 4 * 64, 0.f, 7);
        hw2 = dalloc(36, 0.f, 8);
        hdl = dalloc((size_t)N * 16 * H * W, 0.f, 9);
        CK(hipMalloc(&hdx, (size_t)N * 16 * H * W * sizeof(float)));
        CK(hipMalloc(&hrep, (size_t)ISG_WREP * 4200 * sizeof(double)));
        mh.w1 = hw1; mh.b1 = bet; mh.w2 = hw2; mh.b2 = bet;
        mh.out = out; mh.out_n_stride = (int64_t)16 * H * W;
        mh.dout = hdl; mh.dout_n_stride = (int64_t)16 * H * W;
        mh.dx.nsink = 1;
        mh.dx.s[0].p = hdx; mh.dx.s[0].n_stride = (int64_t)16 * H * W; mh.dx.s[0].C = 16;
        mh.dx.s[0].mode = ISG_SINK_STORE;
        mh.dw1 = hrep; mh.db1 = hrep + 4096; mh.dw2 = hrep + 4100; mh.db2 = hrep + 4136;
        mh.rep_stride = 4200; mh.nrep = ISG_WREP;
        mh.N = N; mh.Hi = H; mh.Wi = W;
        CK(hipMalloc(&mh.ring, (size_t)N * 4 * ISG_HEAD_RING(H, W) * sizeof(float)));
    }
    auto run = [&]() {
        int rc;
        if (!strcmp(op, "headf")) rc = isg_mask_head_fwd(&mh, (isg_stream_t)st);
        else if (!strcmp(op, "headb")) rc = isg_mask_head_bwd(&mh, (isg_stream_t)st);
        else if (!strcmp(op, "fwd")) rc = isg_conv_fwd(&g, &vx, wt, &sk, (isg_stream_t)st);
        else if (!strcmp(op, "dgrad")) rc = isg_conv_dgrad(&g, &vdy, wt, &sk, (isg_stream_t)st);
        else rc = isg_conv_wgrad_rep(&g, &vdy, &vx, dw, nullptr, nw, ISG_WREP, (isg_stream_t)st);
        if (rc) {
            fprintf(stderr, "isg error %d: %s\n", rc, isg_last_error());
            exit(1);
        }
    };
    if (!strcmp(op, "headb") && isg_mask_head_fwd(&mh, (isg_stream_t)st)) {  // writes the ring
        fprintf(stderr, "isg error: %s\n", isg_last_error());
        exit(1);
    }
    for (int i = 0; i < 5; ++i) run();
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) run();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // stamped single launch
    unsigned long long* sp = (unsigned long long*)stamps(
        getenv("KB_STAMPS") ? getenv("KB_STAMPS") : getenv("KB_STAMPS_DOWN") ? "isg_dbg_stamps_down"
        : strcmp(op, "wgrad") ? "isg_dbg_stamps_pw" : "isg_dbg_stamps_wgrad");
    if (!sp) {
        printf("%s N%d Ci%d %dx%d -> Co%d %dx%d k%d s%d p%d d%d: %.2f us/launch (%d reps)\n", op, N,
               Ci, H, W, Co, g.OH, g.OW, k, s, p, d, 1e3 * ms / reps, reps);
        return 0;
    }
    CK(hipMemset(sp, 0, 65536 * 8 * sizeof(unsigned long long)));
    run();
    CK(hipStreamSynchronize(st));
    std::vector<unsigned long long> h(65536 * 8);
    CK(hipMemcpy(h.data(), sp, h.size() * 8, hipMemcpyDeviceToHost));
    int nb = 0;
    unsigned long long t0 = ~0ull, tend = 0;
    for (int b = 0; b < 65536 && h[b * 8]; ++b) {
        nb = b + 1;
        t0 = std::min(t0, h[b * 8]);
        for (int k = 4; k < 8; ++k) tend = std::max(tend, h[b * 8 + k]);
    }
    if (nb == 0) {
        printf("%s N%d Ci%d %dx%d -> Co%d %dx%d k%d s%d p%d d%d: %.2f us/launch (%d reps)\n", op, N,
               Ci, H, W, Co, g.OH, g.OW, k, s, p, d, 1e3 * ms / reps, reps);
        return 0;
    }
    printf("%s N%d Ci%d %dx%d -> Co%d %dx%d k%d s%d p%d d%d: %.2f us/launch (%d reps); "
           "stamped launch %d blocks, span %.2f us\n",
           op, N, Ci, H, W, Co, g.OH, g.OW, k, s, p, d, 1e3 * ms / reps, reps, nb,
           (tend - t0) / 100.0);
    // per-segment medians (10 ns ticks)
    for (int seg = 0; seg < 7; ++seg) {
        std::vector<double> v;
        for (int b = 0; b < nb; ++b)
            if (h[b * 8 + seg + 1] && h[b * 8 + seg]) v.push_back((h[b * 8 + seg + 1] - h[b * 8 + seg]) / 100.0);
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        printf("  seg %d->%d: median %.2f us  p90 %.2f  max %.2f\n", seg, seg + 1, v[v.size() / 2],
               v[v.size() * 9 / 10], v.back());
    }
    std::vector<double> starts;
    for (int b = 0; b < nb; ++b) starts.push_back((h[b * 8] - t0) / 100.0);
    std::sort(starts.begin(), starts.end());
    printf("  block start offsets: p10 %.2f p50 %.2f p90 %.2f max %.2f us\n", starts[nb / 10],
           starts[nb / 2], starts[nb * 9 / 10], starts.back());
    return 0;
}
