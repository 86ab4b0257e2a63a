// ubench_launch.hip -- how long the dispatcher takes to start every wave of a grid (the "start spread"
// of the env-step kernels, tools/exp_stamps_split.py: 1.35-1.5 us for 256 x 512-thread workgroups against
// 0.5-0.7 us for the one-wave kernel's 1024 x 256).  Each wave stores s_memrealtime (100 MHz) as its first
// instruction and again after a fixed amount of dependent VALU work; the program prints, per geometry and
// register footprint, the spread of the start stamps and the time from the first start to the last end.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ub/ubench_launch tools/ubench_launch.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int NV, int LDS_DOUBLES>
__global__ void k_probe(unsigned long long *out, int work)
{
    unsigned long long t0;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    __shared__ double lds[LDS_DOUBLES > 0 ? LDS_DOUBLES : 1];
    double v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = threadIdx.x * 0.5 + j;
    for (int it = 0; it < work; ++it) {
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = fma(v[j], 1.0000001, 0.5);
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NV; ++j) s += v[j];
    if (LDS_DOUBLES > 0) {
        lds[threadIdx.x % (LDS_DOUBLES > 0 ? LDS_DOUBLES : 1)] = s;
        __syncthreads();
        s += lds[(threadIdx.x + 1) % (LDS_DOUBLES > 0 ? LDS_DOUBLES : 1)];
    }
    unsigned long long t1;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) {
        out[3 * w] = t0;
        out[3 * w + 1] = t1;
        out[3 * w + 2] = (unsigned long long)(s != 12345.0);
    }
}

template <int NV, int LDS>
int run(const char *tag, int blocks, int threads, int work, unsigned long long *d, int reps)
{
    const int waves = blocks * threads / 64;
    std::vector<unsigned long long> h(3 * waves);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    double spread = 0, span = 0;
    float ms_total = 0;
    for (int r = 0; r < reps + 2; ++r) {
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((k_probe<NV, LDS>), dim3(blocks), dim3(threads), 0, 0, d, work);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipDeviceSynchronize());
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        CHECK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 3 * waves, hipMemcpyDeviceToHost));
        if (r < 2) continue;
        unsigned long long s0 = ~0ull, s1 = 0, e1v = 0;
        for (int w = 0; w < waves; ++w) {
            s0 = std::min(s0, h[3 * w]);
            s1 = std::max(s1, h[3 * w]);
            e1v = std::max(e1v, h[3 * w + 1]);
        }
        spread += (s1 - s0) / 100.0;   // 100 MHz realtime -> us
        span += (e1v - s0) / 100.0;
        ms_total += ms;
    }
    std::printf("%-34s blocks %5d x %4d thr (%5d waves) VGPR~%3d LDS %6d B: start spread %6.3f us, first start -> last end %7.3f us, event %7.3f us\n",
                tag, blocks, threads, waves, 2 * NV, LDS * 8, spread / reps, span / reps, 1e3 * ms_total / reps);
    return 0;
}

int main()
{
    unsigned long long *d;
    CHECK(hipMalloc(&d, sizeof(unsigned long long) * 3 * 65536));
    const int reps = 20, work = 40;
    run<8, 0>("small regs, no LDS", 1024, 256, work, d, reps);
    run<8, 0>("small regs, no LDS", 256, 512, work, d, reps);
    run<8, 0>("small regs, no LDS", 512, 256, work, d, reps);
    run<8, 0>("small regs, no LDS", 256, 256, work, d, reps);
    run<96, 0>("~200 VGPRs, no LDS", 256, 512, work, d, reps);
    run<96, 0>("~200 VGPRs, no LDS", 1024, 256, work, d, reps);
    run<96, 9000>("~200 VGPRs, 72 KB LDS", 256, 512, work, d, reps);
    run<96, 9000>("~200 VGPRs, 72 KB LDS", 1024, 256, work, d, reps);
    run<8, 9000>("small regs, 72 KB LDS", 256, 512, work, d, reps);
    CHECK(hipFree(d));
    return 0;
}
