// ubench_trans.hip -- does a transcendental (v_exp_f32 / v_rcp_f32) overlap with independent VALU work of the same
// or another wave on a gfx950 SIMD?  Each wave times REP groups with s_memtime; a group is one transcendental per
// chain (8 independent chains) plus F v_fma_f32 on 8 rotating accumulators (a dependent FMA 8 FMAs later).  If the transcendental unit runs beside
// the VALU, cycles per group stay near max(trans, F x fma); if they share the issue, they add.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/build/ubench_trans tools/ubench_trans.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

#define REP 256

template <int TR, int F>   // TR: 0 none, 1 v_exp_f32, 2 v_rcp_f32, 3 exp + rcp (a sigmoid's pair)
__global__ void kern(float *out, long long *cyc, float seed)
{
    float t[8], a[8];
    const float b = seed * 1.0000001f + threadIdx.x * 1e-9f, c = 0.999999f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { t[j] = 0.001f * j + b * 1e-3f; a[j] = b + j; }
    long long t0 = clock64();
#pragma unroll 1
    for (int r = 0; r < REP; ++r) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (TR == 1 || TR == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(t[j]));
            if (TR == 2 || TR == 3) asm volatile("v_rcp_f32 %0, %0" : "+v"(t[j]));
#pragma unroll
            for (int q = 0; q < F; ++q) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[(j * F + q) & 7]) : "v"(b), "v"(c));
        }
    }
    long long t1 = clock64();
    float s = 0;
    for (int j = 0; j < 8; ++j) s += a[j] + t[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int TR, int F>
static void run(const char *name, int waves_per_simd)
{
    const int blocks = 256, threads = 256 * waves_per_simd;   // 256 CUs x 4 SIMDs x w
    float *out; long long *cyc;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
    hipLaunchKernelGGL((kern<TR, F>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0f);
    hipLaunchKernelGGL((kern<TR, F>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0f);
    hipDeviceSynchronize();
    std::vector<long long> h(blocks * threads / 64);
    hipMemcpy(h.data(), cyc, sizeof(long long) * h.size(), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-22s waves/SIMD %d : %7.2f cyc per chain-group (median wave)\n", name, waves_per_simd,
           h[h.size() / 2] / (double)(REP * 8));
    hipFree(out); hipFree(cyc);
}

int main()
{
    for (int w = 1; w <= 2; ++w) {
        run<1, 0>("exp", w);
        run<2, 0>("rcp", w);
        run<3, 0>("exp+rcp", w);
        run<0, 1>("1 fma", w);
        run<0, 2>("2 fma", w);
        run<0, 4>("4 fma", w);
        run<1, 1>("exp + 1 fma", w);
        run<1, 2>("exp + 2 fma", w);
        run<1, 4>("exp + 4 fma", w);
        run<3, 2>("exp+rcp + 2 fma", w);
        run<3, 4>("exp+rcp + 4 fma", w);
        run<3, 8>("exp+rcp + 8 fma", w);
    }
    return 0;
}
