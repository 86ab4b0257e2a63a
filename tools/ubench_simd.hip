// ubench_simd.hip -- which SIMD does each wave of a 512-thread workgroup land on (gfx950)?  Reads
// HW_REG_HW_ID (SIMD_ID = bits 5:4, CU_ID = bits 11:8) per wave for a grid of 256 workgroups (one per CU)
// and prints the wave -> SIMD map of the first workgroups and a census of the maps seen.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <map>
#include <string>
#include <vector>

__global__ __launch_bounds__(512) void k(unsigned *out)
{
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    __shared__ double pad[12000];   // ~94 KB of LDS: one workgroup per CU
    pad[threadIdx.x] = 1.0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = id + (unsigned)pad[(threadIdx.x + 1) % 512] * 0u;
}

int main()
{
    const int nb = 256;
    unsigned *d;
    hipMalloc(&d, nb * 8 * sizeof(unsigned));
    hipLaunchKernelGGL(k, dim3(nb), dim3(512), 0, 0, d);
    std::vector<unsigned> h(nb * 8);
    hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::map<std::string, int> census;
    for (int b = 0; b < nb; ++b) {
        std::string s;
        for (int w = 0; w < 8; ++w) s += std::to_string((h[b * 8 + w] >> 4) & 3);
        census[s]++;
        if (b < 4) printf("block %d: wave->simd %s (cu %u)\n", b, s.c_str(), (h[b * 8] >> 8) & 15);
    }
    for (auto &kv : census) printf("map %s: %d blocks\n", kv.first.c_str(), kv.second);
    return 0;
}
