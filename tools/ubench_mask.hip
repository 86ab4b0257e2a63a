// ubench_mask.hip -- does a wave with only some lanes active issue fp64 VALU faster (gfx950)?
// Lanes >= ACTIVE leave before the timed loop, so the loop runs with a constant exec mask.  Reports
// cycles per fp64 FMA per wave (median over waves) for 1 and 2 waves per SIMD, ILP 1 and 8, plus the
// same for a mixed chain (fma + mul + add) -- the question behind a 32-envs-per-wave launch of the env
// step (two waves per SIMD for the same 65,536 envs).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ub/ubench_mask tools/ubench_mask.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

#define REP 512

template <int ACTIVE, int ILP>
__global__ void kern(double *out, long long *cyc, double seed)
{
    const int lane = threadIdx.x & 63;
    double a[8], b = seed * 1.0000001 + threadIdx.x * 1e-9, c = 0.999999;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = b + j;
    if (lane >= ACTIVE) return;   // exec = lanes [0, ACTIVE) from here on
    long long t0 = clock64();
#pragma unroll 1
    for (int r = 0; r < REP / 8; ++r) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
#pragma unroll
            for (int j = 0; j < ILP; ++j) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
        }
    }
    long long t1 = clock64();
    double s = 0;
    for (int j = 0; j < 8; ++j) s += a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int ACTIVE, int ILP>
static void run(int waves_per_simd)
{
    const int blocks = 256, threads = 256 * waves_per_simd;
    double *out; long long *cyc;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
    hipMemset(cyc, 0, sizeof(long long) * blocks * threads / 64);
    hipLaunchKernelGGL((kern<ACTIVE, ILP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((kern<ACTIVE, ILP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(blocks * threads / 64);
    hipMemcpy(h.data(), cyc, sizeof(long long) * h.size(), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("active %2d lanes  ILP%d  waves/SIMD %d : %6.2f cyc/fma per wave (median), kernel %.2f us\n", ACTIVE, ILP,
           waves_per_simd, h[h.size() / 2] / (double)(REP * ILP), ms * 1e3);
    hipFree(out); hipFree(cyc);
}

#define ALL(A) run<A, 8>(1); run<A, 8>(2); run<A, 1>(1); run<A, 1>(2); run<A, 8>(4);

int main()
{
    ALL(64) ALL(32) ALL(16) ALL(8)
    return 0;
}
