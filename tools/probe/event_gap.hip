// Probe: main-queue idle around a fork event. Kernel chains on one stream with
//   mode 0: nothing between kernels
//   mode 1: hipEventRecord(ev, main) + hipStreamWaitEvent(side, ev) + a small side kernel
//   mode 2: the event bound to the kernel itself (hipExtLaunchKernelGGL stop event)
//   mode 3: hipStreamWaitEvent(main, ev_side) on an already-complete side event (a join)
// Per-kernel durations/gaps come from rocprofv3 --kernel-trace; the wall time per chain
// from hipEvents around it.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>

__global__ void busy(float* p, int n, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = p[i];
    for (int k = 0; k < iters; ++k) v = v * 0.999f + 0.5f;
    p[i] = v;
}

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

int main(int argc, char** argv) {
    const int chain = 64, n = 256 * 512;
    float *a, *b;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    hipStream_t m, s;
    CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev0[chain], ev4[chain], ev5[chain], t0, t1;
    for (int i = 0; i < chain; ++i) {
        CK(hipEventCreateWithFlags(&ev0[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev4[i], hipEventDisableTiming | hipEventDisableSystemFence));
        CK(hipEventCreateWithFlags(&ev5[i], hipEventDisableTiming | hipEventReleaseToDevice));
    }
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int mode = 0; mode < 9; ++mode) {
        hipEvent_t* ev = mode == 4 ? ev4 : (mode == 5 ? ev5 : ev0);
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(t0, m));
            for (int i = 0; i < chain; ++i) {
                if (mode == 2) {
                    hipExtLaunchKernelGGL(busy, dim3(n / 256), dim3(256), 0, m, nullptr, ev[i], 0, a, n, 200);
                } else {
                    hipLaunchKernelGGL(busy, dim3(n / 256), dim3(256), 0, m, a, n, 200);
                }
                if (mode == 1 || mode >= 4) CK(hipEventRecord(ev[i], m));
                if (mode == 7 || mode == 8) CK(hipStreamWaitEvent(s, ev[i], 0));
                if (mode == 8 && i % 8 == 7) hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, b, 64, 10);
                if (mode == 1 || mode == 2 || mode == 4 || mode == 5) {
                    CK(hipStreamWaitEvent(s, ev[i], 0));
                    hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, b, 64, 10);
                }
                if (mode == 3) {
                    if (i == 0) {
                        hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, b, 64, 10);
                        CK(hipEventRecord(ev[0], s));
                        CK(hipStreamSynchronize(s));
                    }
                    CK(hipStreamWaitEvent(m, ev[0], 0));
                }
            }
            CK(hipEventRecord(t1, m));
            CK(hipDeviceSynchronize());
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            printf("mode %d rep %d: %.2f us per kernel\n", mode, rep, 1e3f * ms / chain);
        }
    }
    return 0;
}
