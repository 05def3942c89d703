// Instruction-fetch probe: the same 8192 dependent-free FMAs per lane as one straight-line
// block (64 KB of code) or as a 512-FMA block looped 16 times (4 KB of code), one wave per
// workgroup, timed with hip events over back-to-back launches. If straight-line code costs
// more than issue time, kernel duration grows with code size (instruction cache refills).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

// straight-line FMA blocks by macro expansion (a loop would be re-rolled by the compiler)
#define F(k) x[k] = __builtin_fmaf(x[k], a, 1.0f);
#define S1 F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(8) F(9) F(10) F(11) F(12) F(13) F(14) F(15)
#define S8 S1 S1 S1 S1 S1 S1 S1 S1
#define S32 S8 S8 S8 S8
#define S256 S32 S32 S32 S32 S32 S32 S32 S32
#define S512 S256 S256

__global__ __launch_bounds__(64) void straight(float* out, float a) {
    float x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = threadIdx.x + k;
    S512
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += x[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ __launch_bounds__(64) void looped(float* out, float a, int n) {
    float x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = threadIdx.x + k;
    for (int r = 0; r < n; ++r) {
        S32
        asm volatile("" ::: "memory");
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += x[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

__global__ void empty(float* out) { if (threadIdx.x == 1000) out[0] = 0.f; }

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 1;
    float* out;
    hipMalloc(&out, 4096 * 64 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto time = [&](const char* name, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 50;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s blocks %4d: %8.2f us/launch\n", name, blocks, 1e3 * ms / reps);
    };
    time("empty", [&] { hipLaunchKernelGGL(empty, dim3(blocks), dim3(64), 0, 0, out); });
    time("straight", [&] { hipLaunchKernelGGL(straight, dim3(blocks), dim3(64), 0, 0, out, 0.999f); });
    time("looped", [&] { hipLaunchKernelGGL(looped, dim3(blocks), dim3(64), 0, 0, out, 0.999f, 16); });
    time("looped1", [&] { hipLaunchKernelGGL(looped, dim3(blocks), dim3(64), 0, 0, out, 0.999f, 1); });
    return 0;
}
