// ubench_geometry.hip -- what the launch-alone term of the per-step kernel's budget (2.18 us, tools/ubench_budget.hip)
// depends on: the same do-nothing kernel (every wave reaches a workgroup barrier and ends) over grids of different
// workgroup size, workgroup count and LDS footprint, replayed as in the bench (K launches per HIP graph, median of
// replays).  Rows: the per-step kernel's geometry (256 x 768 threads, 69.7 KB LDS), the same without LDS, the same
// 3,072 waves in other workgroup shapes, and a third of the waves.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ub/ubench_geometry tools/ubench_geometry.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int LDS_BYTES>
__global__ __launch_bounds__(1024) void k_nothing(int *sink)
{
    if constexpr (LDS_BYTES > 0) {
        __shared__ double lds[LDS_BYTES / 8];
        if (threadIdx.x == 0) lds[0] = 1.0;
        __syncthreads();
        if (lds[0] != 1.0) sink[0] = 1;
    } else {
        __syncthreads();
        if (threadIdx.x == 1u << 30) sink[0] = 1;
    }
}

template <typename L>
int graph_us(const char *tag, int wgs, int threads, int lds, L launch, int k, int reps, hipStream_t st)
{
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < k; ++r) launch();
    CHECK(hipStreamEndCapture(st, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipGraphLaunch(ge, st));
    CHECK(hipStreamSynchronize(st));
    std::vector<float> us;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a, st));
        CHECK(hipGraphLaunch(ge, st));
        CHECK(hipEventRecord(b, st));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        us.push_back(ms * 1e3f / k);
    }
    std::sort(us.begin(), us.end());
    std::printf("{\"geometry\": \"%s\", \"workgroups\": %d, \"threads\": %d, \"waves\": %d, \"lds_bytes\": %d, "
                "\"us_per_launch_median\": %.3f, \"min\": %.3f}\n",
                tag, wgs, threads, wgs * threads / 64, lds, us[us.size() / 2], us[0]);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
    return 0;
}

int main()
{
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int *sink;
    CHECK(hipMalloc(&sink, 4));
    constexpr int K = 20, REPS = 200;
#define ROW(tag, WG, T, LDS) \
    if (graph_us(tag, WG, T, LDS, [&] { hipLaunchKernelGGL(k_nothing<LDS>, dim3(WG), dim3(T), 0, st, sink); }, K, REPS, st)) return 1
    for (int round = 0; round < 2; ++round) {
        ROW("per-step kernel: 256 x 768, its LDS", 256, 768, 69696);
        ROW("256 x 768, no LDS", 256, 768, 0);
        ROW("256 x 768, 32 KB LDS", 256, 768, 32768);
        ROW("768 x 256 (the same waves), 23 KB LDS", 768, 256, 23232);
        ROW("3072 x 64 (the same waves), no LDS", 3072, 64, 0);
        ROW("256 x 512 (2/3 of the waves), its LDS", 256, 512, 69696);
        ROW("256 x 256 (1/3 of the waves), no LDS", 256, 256, 0);
        ROW("256 x 64 (one wave per CU), no LDS", 256, 64, 0);
        ROW("1 x 64", 1, 64, 0);
    }
    return 0;
}
