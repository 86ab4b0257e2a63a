// ubench_budget.hip -- the launch and memory terms of the per-step kernel's budget (profiles/<round>/env_step_budget.json,
// tools/budget_summary.py), measured with standalone kernels of the SAME geometry as k_env_step_split
// (b747_rl_ctrl_amd/csrc/b747_split.h: 65,536 envs, 256 workgroups of 768 threads = flight / ahead / control waves of
// 256 envs, the same LDS footprint) replayed like the bench, K launches in one HIP graph:
//   launch   every wave reaches a workgroup barrier and ends: dispatch ramp + the kernel boundary alone;
//   memory   each role loads exactly the fields the product's role loads for one env step (fp64 SoA, the same
//            per-field arrays, the FAST table image staged into LDS by the flight waves) and writes back what the
//            product writes (write-through stores, as st_state), with no arithmetic between: the launch plus the
//            step's HBM traffic in the order the product issues it.
// The product's own time (rocprofv3 kernel trace / the bench's HIP events) minus `memory` is the compute it adds.
// No product code is built into this tool; it reads and writes its own buffers only.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ub/ubench_budget tools/ubench_budget.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kEnvs = 256, kBlock = 3 * kEnvs;
constexpr int kLdsBytes = 69696;               // k_env_step_split's group segment (tools/kernel_resources.py)
constexpr int kTable = 768;                    // FAST table image entries staged per workgroup (<= 3 per flight lane)

struct Bufs {
    double *X;         // [18][n]
    double *aero;      // [5][n]
    uint32_t *k;
    double *disc;      // [9][n]
    uint8_t *flags, *mem, *done;
    float *action, *obs, *reward;
    double *ref, *h_zh;
    float *ep_ret;   // (float since ABI 10)
    const double *table;
};

template <typename T>
__device__ __forceinline__ void st_wt(T *p, T v)   // write-through store (b747_lanes.h st_state)
{
    using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned>::type;
    U bits;
    __builtin_memcpy(&bits, &v, sizeof(T));
    __hip_atomic_store((U *)p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kBlock) void k_launch(int *sink)
{
    __shared__ double lds[kLdsBytes / 8];
    if (threadIdx.x == 0) lds[0] = 1.0;
    __syncthreads();
    if (lds[0] != 1.0) sink[0] = 1;
}

__global__ __launch_bounds__(kBlock) void k_memory(int64_t n, Bufs b)
{
    __shared__ double lds[kLdsBytes / 8];
    const int el = threadIdx.x % kEnvs, role = threadIdx.x / kEnvs;
    const int64_t i = (int64_t)blockIdx.x * kEnvs + el;
    if (role == 0) {                                        // flight: tables, X0..X2, X5..X8, aero_err, k
        double tv[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) tv[q] = b.table[el + q * kEnvs];
        constexpr int fx[7] = {0, 1, 2, 5, 6, 7, 8};
        double x[7], s = 0.0;
#pragma unroll
        for (int j = 0; j < 7; ++j) x[j] = b.X[fx[j] * n + i];
#pragma unroll
        for (int j = 0; j < 5; ++j) s += b.aero[j * n + i];
        s += (double)b.k[i];
#pragma unroll
        for (int q = 0; q < 3; ++q) lds[el + q * kEnvs] = tv[q];
        __syncthreads();
        s += lds[(el + 1) % kTable];
#pragma unroll
        for (int j = 0; j < 7; ++j) st_wt(&b.X[fx[j] * n + i], x[j] + 1e-300 * s);
    } else if (role == 1) {                                 // ahead: X1, X2, X5, X7, X8 (no stores)
        constexpr int ax[5] = {1, 2, 5, 7, 8};
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < 5; ++j) s += b.X[ax[j] * n + i];
        __syncthreads();
        if (s == 12345.678) b.done[i] = 2;                  // (never: keeps the loads)
    } else {                                                // control
        const uint32_t k = b.k[i];
        double d[5], s = 0.0;
#pragma unroll
        for (int j = 0; j < 5; ++j) d[j] = b.disc[j * n + i];
#pragma unroll
        for (int q = 0; q < 3; ++q) s += b.disc[(int64_t)(5u + ((k + q) & 3u)) * n + i];
        const uint8_t fl = b.flags[i];
        s += b.X[1 * n + i] + b.X[2 * n + i] + b.X[5 * n + i];
        const float a = b.action[i];
        double x[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) x[j] = b.X[(9 + j) * n + i];
        __syncthreads();
        const uint8_t m = b.mem[i];
        s += b.ref[i] + b.h_zh[i];
        const float er = b.ep_ret[i];
        s += (double)a + (double)fl + (double)m;
#pragma unroll
        for (int j = 2; j < 5; ++j) st_wt(&b.disc[j * n + i], d[j] + 1e-300 * s);
        st_wt(&b.disc[(int64_t)(5u + (k & 3u)) * n + i], d[0] + 1e-300 * s);
        b.k[i] = k;
        b.mem[i] = m;
#pragma unroll
        for (int j = 0; j < 3; ++j) b.obs[i * 3 + j] = (float)(s * 1e-300);
        b.reward[i] = a;
        b.done[i] = 0;
        b.ep_ret[i] = er;
#pragma unroll
        for (int j = 0; j < 9; ++j) st_wt(&b.X[(9 + j) * n + i], x[j] + 1e-300 * s);
    }
}

template <class L>
int graph_us(const char *tag, L launch, int k, int reps, hipStream_t st)
{
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < k; ++r) launch();
    CHECK(hipStreamEndCapture(st, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipGraphLaunch(ge, st));                          // upload
    CHECK(hipStreamSynchronize(st));
    std::vector<float> us;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0, st));
        CHECK(hipGraphLaunch(ge, st));
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        us.push_back(ms * 1e3f / k);
    }
    std::sort(us.begin(), us.end());
    std::printf("{\"term\": \"%s\", \"us_per_launch_median\": %.3f, \"min\": %.3f, \"max\": %.3f, \"launches_per_graph\": %d, "
                "\"replays\": %d}\n", tag, us[us.size() / 2], us.front(), us.back(), k, reps);
    std::fflush(stdout);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
    return 0;
}

int main()
{
    const int64_t n = 65536;
    const unsigned grid = (unsigned)(n / kEnvs);
    Bufs b{};
    CHECK(hipMalloc(&b.X, 18 * n * 8));
    CHECK(hipMalloc(&b.aero, 5 * n * 8));
    CHECK(hipMalloc(&b.k, n * 4));
    CHECK(hipMalloc(&b.disc, 9 * n * 8));
    CHECK(hipMalloc(&b.flags, n));
    CHECK(hipMalloc(&b.mem, n));
    CHECK(hipMalloc(&b.done, n));
    CHECK(hipMalloc(&b.action, n * 4));
    CHECK(hipMalloc(&b.obs, 3 * n * 4));
    CHECK(hipMalloc(&b.reward, n * 4));
    CHECK(hipMalloc(&b.ref, n * 8));
    CHECK(hipMalloc(&b.h_zh, n * 8));
    CHECK(hipMalloc(&b.ep_ret, n * 4));
    double *table;
    CHECK(hipMalloc(&table, kTable * 8));
    b.table = table;
    CHECK(hipMemset(b.X, 0, 18 * n * 8));
    CHECK(hipMemset(b.aero, 0, 5 * n * 8));
    CHECK(hipMemset(b.k, 0, n * 4));
    CHECK(hipMemset(b.disc, 0, 9 * n * 8));
    CHECK(hipMemset(b.flags, 0, n));
    CHECK(hipMemset(b.mem, 0, n));
    CHECK(hipMemset(b.action, 0, n * 4));
    CHECK(hipMemset(b.ref, 0, n * 8));
    CHECK(hipMemset(b.h_zh, 0, n * 8));
    CHECK(hipMemset(b.ep_ret, 0, n * 4));
    CHECK(hipMemset(table, 0, kTable * 8));
    int *sink;
    CHECK(hipMalloc(&sink, 4));
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int K = 20, REPS = 200;                           // the driver's --steps 20
    for (int round = 0; round < 2; ++round) {
        if (graph_us("launch", [&] { hipLaunchKernelGGL(k_launch, dim3(grid), dim3(kBlock), 0, st, sink); }, K, REPS, st)) return 1;
        if (graph_us("memory", [&] { hipLaunchKernelGGL(k_memory, dim3(grid), dim3(kBlock), 0, st, n, b); }, K, REPS, st)) return 1;
    }
    CHECK(hipStreamSynchronize(st));
    return 0;
}
