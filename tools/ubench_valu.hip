// ubench_valu.hip -- issue cost and dependent latency of the VALU instructions the env-step kernel
// is made of, for one and two waves per SIMD (gfx950).  Each wave times a fixed instruction
// stream with s_memtime; the host reports cycles per instruction (median over waves).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/build/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define REP 256

// 8 independent chains (ILP 8) or one chain (ILP 1), REP instructions per chain
template <int OP, int ILP>
__global__ void kern(double *out, long long *cyc, double seed)
{
    double a[8], b = seed * 1.0000001 + threadIdx.x * 1e-9, c = 0.999999;
    float f[8], fb = (float)b, fc = 0.99999f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = b + j; f[j] = fb + j; }
    __shared__ double sh[1024];
    sh[threadIdx.x] = b;
    __syncthreads();
    long long t0 = clock64();
#pragma unroll 1
    for (int r = 0; r < REP / 8; ++r) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
#pragma unroll
            for (int j = 0; j < ILP; ++j) {
                if (OP == 0) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[j]) : "v"(fb), "v"(fc));
                if (OP == 2) asm volatile("v_rsq_f64 %0, %0" : "+v"(a[j]));
                if (OP == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(f[j]));
                if (OP == 4) asm volatile("v_cmp_le_f64 vcc, %0, %1\n\tv_cndmask_b32 %2, 0, 1, vcc" : "+v"(a[j]) : "v"(b), "v"(f[j]) : "vcc");
                if (OP == 5) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[j]) : "v"(b));
                if (OP == 6) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == 7) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[j]) : "v"(b));
                if (OP == 8) asm volatile("s_mov_b32 s40, 0x3ff00001\n\ts_mov_b32 s41, 0x3ff00002\n\tv_fma_f64 %0, %0, s[40:41], %1" : "+v"(a[j]) : "v"(c) : "s40", "s41");
                if (OP == 9 && (threadIdx.x & 63) < 32) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == 10) asm volatile("v_fma_f64 %0, %0, s[40:41], %1" : "+v"(a[j]) : "v"(c) : "s40", "s41");
                if (OP == 11) asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(a[j]) : "v"((unsigned)(threadIdx.x * 8)));
            }
        }
    }
    long long t1 = clock64();
    double s = 0;
    for (int j = 0; j < 8; ++j) s += a[j] + f[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + sh[(threadIdx.x + 1) & 1023];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP, int ILP>
static void run(const char *name, int waves_per_simd)
{
    const int blocks = 256, threads = 256 * waves_per_simd;   // 256 CUs x 4 SIMDs x w
    double *out; long long *cyc;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
    hipLaunchKernelGGL((kern<OP, ILP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((kern<OP, ILP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(blocks * threads / 64);
    hipMemcpy(h.data(), cyc, sizeof(long long) * h.size(), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double n = (double)REP * ILP;
    printf("%-10s ILP%d waves/SIMD %d : %6.2f cyc/instr per wave (median), wall %.2f us\n", name, ILP, waves_per_simd,
           h[h.size() / 2] / n, ms * 1e3);
    hipFree(out); hipFree(cyc);
}


// blocks of 8 independent instructions: constant-supply strategies for an fp64 FMA stream
template <int OP>
__global__ void kblk(double *out, long long *cyc, double seed)
{
    __shared__ double sh[1024];
    double a0 = seed + threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7, c = 0.999999;
    double k0, k1, k2, k3, k4, k5, k6, k7;
    int cnt = 0;
    sh[threadIdx.x] = a0;
    __syncthreads();
    long long t0 = clock64();
#pragma unroll 1
    for (int r = 0; r < 32; ++r) {
        if (OP == 0) {   // SGPR operand, 8 distinct pairs, set once (outside timing would be ideal; cheap here)
            asm volatile(
                "v_fma_f64 %0, %0, s[40:41], %8\n\tv_fma_f64 %1, %1, s[42:43], %8\n\tv_fma_f64 %2, %2, s[44:45], %8\n\t"
                "v_fma_f64 %3, %3, s[46:47], %8\n\tv_fma_f64 %4, %4, s[48:49], %8\n\tv_fma_f64 %5, %5, s[50:51], %8\n\t"
                "v_fma_f64 %6, %6, s[52:53], %8\n\tv_fma_f64 %7, %7, s[54:55], %8"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c)
                : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");
        }
        if (OP == 1) {   // 16 s_mov (hoisted), then 8 FMAs reading them
            asm volatile(
                "s_mov_b32 s40, 0x3ff00001\n\ts_mov_b32 s41, 0x3ff00002\n\ts_mov_b32 s42, 0x3ff00003\n\ts_mov_b32 s43, 0x3ff00004\n\t"
                "s_mov_b32 s44, 0x3ff00001\n\ts_mov_b32 s45, 0x3ff00002\n\ts_mov_b32 s46, 0x3ff00003\n\ts_mov_b32 s47, 0x3ff00004\n\t"
                "s_mov_b32 s48, 0x3ff00001\n\ts_mov_b32 s49, 0x3ff00002\n\ts_mov_b32 s50, 0x3ff00003\n\ts_mov_b32 s51, 0x3ff00004\n\t"
                "s_mov_b32 s52, 0x3ff00001\n\ts_mov_b32 s53, 0x3ff00002\n\ts_mov_b32 s54, 0x3ff00003\n\ts_mov_b32 s55, 0x3ff00004\n\t"
                "v_fma_f64 %0, %0, s[40:41], %8\n\tv_fma_f64 %1, %1, s[42:43], %8\n\tv_fma_f64 %2, %2, s[44:45], %8\n\t"
                "v_fma_f64 %3, %3, s[46:47], %8\n\tv_fma_f64 %4, %4, s[48:49], %8\n\tv_fma_f64 %5, %5, s[50:51], %8\n\t"
                "v_fma_f64 %6, %6, s[52:53], %8\n\tv_fma_f64 %7, %7, s[54:55], %8"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c)
                : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");
        }
        if (OP == 2) {   // 8 uniform ds_read_b64 -> 8 VGPR constants, wait, 8 FMAs
            asm volatile(
                "ds_read_b64 %8, %16\n\tds_read_b64 %9, %16 offset:8\n\tds_read_b64 %10, %16 offset:16\n\tds_read_b64 %11, %16 offset:24\n\t"
                "ds_read_b64 %12, %16 offset:32\n\tds_read_b64 %13, %16 offset:40\n\tds_read_b64 %14, %16 offset:48\n\tds_read_b64 %15, %16 offset:56\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "v_fma_f64 %0, %0, %8, %17\n\tv_fma_f64 %1, %1, %9, %17\n\tv_fma_f64 %2, %2, %10, %17\n\t"
                "v_fma_f64 %3, %3, %11, %17\n\tv_fma_f64 %4, %4, %12, %17\n\tv_fma_f64 %5, %5, %13, %17\n\t"
                "v_fma_f64 %6, %6, %14, %17\n\tv_fma_f64 %7, %7, %15, %17"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                  "=&v"(k0), "=&v"(k1), "=&v"(k2), "=&v"(k3), "=&v"(k4), "=&v"(k5), "=&v"(k6), "=&v"(k7)
                : "v"(0u), "v"(c));
        }
        if (OP == 3) {   // 16 v_mov_b32 literals -> 8 VGPR pairs, then 8 FMAs
            asm volatile(
                "v_mov_b32 %8, 0x3ff00001\n\tv_mov_b32 %9, 0x3ff00001\n\tv_mov_b32 %10, 0x3ff00001\n\tv_mov_b32 %11, 0x3ff00001\n\t"
                "v_fma_f64 %0, %0, %12, %13\n\tv_fma_f64 %1, %1, %12, %13\n\tv_fma_f64 %2, %2, %12, %13\n\tv_fma_f64 %3, %3, %12, %13\n\t"
                "v_fma_f64 %4, %4, %12, %13\n\tv_fma_f64 %5, %5, %12, %13\n\tv_fma_f64 %6, %6, %12, %13\n\tv_fma_f64 %7, %7, %12, %13"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=v"(cnt), "=v"(cnt), "=v"(cnt), "=v"(cnt)
                : "v"(c), "v"(c));
        }
        if (OP == 4) {   // fp32 compare against a literal + carry add, 8 of them
            asm volatile(
                "v_cmp_le_f32 vcc, 0x3e99999a, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f32 vcc, 0x3f4ccccd, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f32 vcc, 0x3f570a3d, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f32 vcc, 0x3f7851ec, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f32 vcc, 0x3e99999a, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f32 vcc, 0x3f4ccccd, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f32 vcc, 0x3f570a3d, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f32 vcc, 0x3f7851ec, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc"
                : "+v"(cnt) : "v"((float)a0) : "vcc");
        }
        if (OP == 5) {   // fp64 compare against SGPR pairs + carry add, 8 of them
            asm volatile(
                "v_cmp_le_f64 vcc, s[40:41], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f64 vcc, s[42:43], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f64 vcc, s[44:45], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f64 vcc, s[46:47], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f64 vcc, s[48:49], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f64 vcc, s[50:51], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f64 vcc, s[52:53], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t"
                "v_cmp_le_f64 vcc, s[54:55], %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc"
                : "+v"(cnt) : "v"(a0) : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");
        }
        if (OP == 6) {   // fp64 compares into 8 distinct SGPR masks, then 8 cndmask + add (no VCC chain)
            asm volatile(
                "v_cmp_le_f64 s[60:61], s[40:41], %1\n\tv_cmp_le_f64 s[62:63], s[42:43], %1\n\t"
                "v_cmp_le_f64 s[64:65], s[44:45], %1\n\tv_cmp_le_f64 s[66:67], s[46:47], %1\n\t"
                "v_cmp_le_f64 s[68:69], s[48:49], %1\n\tv_cmp_le_f64 s[70:71], s[50:51], %1\n\t"
                "v_cmp_le_f64 s[72:73], s[52:53], %1\n\tv_cmp_le_f64 s[74:75], s[54:55], %1\n\t"
                "v_addc_co_u32 %0, vcc, 0, %0, s[60:61]\n\tv_addc_co_u32 %0, vcc, 0, %0, s[62:63]\n\t"
                "v_addc_co_u32 %0, vcc, 0, %0, s[64:65]\n\tv_addc_co_u32 %0, vcc, 0, %0, s[66:67]\n\t"
                "v_addc_co_u32 %0, vcc, 0, %0, s[68:69]\n\tv_addc_co_u32 %0, vcc, 0, %0, s[70:71]\n\t"
                "v_addc_co_u32 %0, vcc, 0, %0, s[72:73]\n\tv_addc_co_u32 %0, vcc, 0, %0, s[74:75]"
                : "+v"(cnt) : "v"(a0) : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55",
                  "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75");
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + k0 + k1 + k2 + k3 + k4 + k5 + k6 + k7 + cnt + sh[(threadIdx.x + 1) & 1023];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
static void runblk(const char *name, int waves_per_simd)
{
    const int blocks = 256, threads = 256 * waves_per_simd;
    double *out; long long *cyc;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
    hipLaunchKernelGGL((kblk<OP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0);
    hipLaunchKernelGGL((kblk<OP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, 1.0);
    hipDeviceSynchronize();
    std::vector<long long> h(blocks * threads / 64);
    hipMemcpy(h.data(), cyc, sizeof(long long) * h.size(), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-28s waves/SIMD %d : %7.1f cyc per block of 8 (median)\n", name, waves_per_simd, h[h.size() / 2] / 32.0);
    hipFree(out); hipFree(cyc);
}

#define RUN(OP, NAME) \
    run<OP, 8>(NAME, 1); run<OP, 1>(NAME, 1); run<OP, 8>(NAME, 2); run<OP, 1>(NAME, 2); run<OP, 1>(NAME, 4);

int main()
{
    RUN(0, "fma_f64");
    RUN(7, "mul_f64");
    RUN(5, "add_f64");
    RUN(1, "fma_f32");
    RUN(6, "pk_fma_f32");
    RUN(2, "rsq_f64");
    RUN(3, "exp_f32");
    RUN(4, "cmp64+cnd");
    RUN(8, "smov2+fma64");
    RUN(10, "fma64 sgpr");
    RUN(9, "fma64 half");
    RUN(11, "ds_read lat");
    const char *bn[] = {"fma64 x8 sgpr distinct", "16 s_mov + fma64 x8", "4 ds_read_b128 + fma64 x8", "4 v_mov + fma64 x8 (vgpr k)",
                        "cmp_f32 lit + addc x8", "cmp_f64 sgpr + addc x8 (vcc)", "cmp_f64 x8 -> masks, addc x8"};
    runblk<0>(bn[0], 1); runblk<0>(bn[0], 2);
    runblk<1>(bn[1], 1); runblk<1>(bn[1], 2);
    runblk<2>(bn[2], 1); runblk<2>(bn[2], 2);
    runblk<3>(bn[3], 1); runblk<3>(bn[3], 2);
    runblk<4>(bn[4], 1); runblk<4>(bn[4], 2);
    runblk<5>(bn[5], 1); runblk<5>(bn[5], 2);
    runblk<6>(bn[6], 1); runblk<6>(bn[6], 2);
    return 0;
}
