// b747_kernels.hip -- MI355X (gfx950) kernels + C ABI of libb747.so.
//
// One lane = one environment = one copy of the reference DLL's static model state
// (core/model_simple_win64.dll; the reference loads a file copy of the DLL per env,
// core/model.py:99-110).  State is structure-of-arrays in HBM ([field][N]) so that each
// wave64 load/store of a field is one contiguous 256 B (fp32) / 512 B (fp64) transaction.
// The 241 lookup-table doubles (CYa, CXa, dCm/ddeltaz, mz, K_alpha) are staged into LDS once
// per workgroup; per-lane table gathers then hit LDS, not L1/L2.
//
// Roofline: with n_steps == 1 a step moves the whole compact state through HBM
// (algorithmic bytes in DESIGN.md); with n_steps > 1 state stays in VGPRs and the kernel is
// fp64-VALU bound (4 output passes x ~11 transcendentals per step).
#include <hip/hip_runtime.h>

#include <stdio.h>

#include "../../include/b747.h"
#include "b747_dynamics.h"

using namespace b747;

namespace {

thread_local char g_err[256] = "";

int32_t fail(hipError_t e, const char *where)
{
    snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
    return -(int32_t)e;
}

int32_t bad_arg(const char *what)
{
    snprintf(g_err, sizeof(g_err), "invalid argument: %s", what);
    return -(int32_t)hipErrorInvalidValue;
}

constexpr int kBlock = 256;

template <typename XT>
__device__ __forceinline__ void load_x(const XT *__restrict__ X, int64_t n, int64_t i, double *x)
{
#pragma unroll
    for (int j = 0; j < NX; ++j) x[j] = (double)X[j * n + i];
}

template <typename XT>
__device__ __forceinline__ void store_x(XT *__restrict__ X, int64_t n, int64_t i, const double *x)
{
#pragma unroll
    for (int j = 0; j < NX; ++j) X[j * n + i] = (XT)x[j];
}

__device__ __forceinline__ void load_params(const b747_model_batch &b, int64_t i, Params &P)
{
    const int64_t n = b.n;
    P.deltaz = b.deltaz[i];
    P.vartheta = b.vartheta[i];
    P.h_zh = b.h_zh[i];
    P.flags = b.flags[i];
    P.kCX = (double)b.aero_err[0 * n + i] + B747_F_ONE;
    P.kCY = (double)b.aero_err[1 * n + i] + B747_F_ONE;
    P.kmz = (double)b.aero_err[2 * n + i] + B747_M_ONE;
    P.kdCm = (double)b.aero_err[3 * n + i] + B747_M_ONE;
    P.kKa = (double)b.aero_err[4 * n + i] + B747_M_ONE;
}

__device__ __forceinline__ void load_disc(const double *__restrict__ disc, int64_t n, int64_t i, Disc &D)
{
    D.x_dss = disc[0 * n + i];
    D.y_dss = disc[1 * n + i];
    D.rl_prevY = disc[2 * n + i];
    D.e_prev = disc[3 * n + i];
    D.ed_prev = disc[4 * n + i];
#pragma unroll
    for (int j = 0; j < 4; ++j) D.u_hist[j] = disc[(5 + j) * n + i];
}

__device__ __forceinline__ void store_disc(double *__restrict__ disc, int64_t n, int64_t i, const Disc &D)
{
    disc[0 * n + i] = D.x_dss;
    disc[1 * n + i] = D.y_dss;
    disc[2 * n + i] = D.rl_prevY;
    disc[3 * n + i] = D.e_prev;
    disc[4 * n + i] = D.ed_prev;
#pragma unroll
    for (int j = 0; j < 4; ++j) disc[(5 + j) * n + i] = D.u_hist[j];
}

// ---------------------------------------------------------------- model-level kernels ----

template <typename XT>
__global__ __launch_bounds__(kBlock) void k_model_step(b747_model_batch b, Consts C, int32_t n_steps)
{
    __shared__ double tb[T_N];
    __shared__ double scr[2 * NX][kBlock];   // RK4 y / acc, [field][lane]: conflict-free ds_*_b64
    stage_tables(tb, threadIdx.x, blockDim.x);
    __syncthreads();
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x[NX];
    load_x((const XT *)b.X, n, i, x);
    Disc D;
    load_disc(b.disc, n, i, D);
    uint32_t k = b.k[i];
    uint32_t mem = b.mem[i];
    Params P;
    load_params(b, i, P);
    for (int32_t s = 0; s < n_steps; ++s) {
        double *sig = (b.sig && s == n_steps - 1) ? b.sig + i : nullptr;
        major_step(x, D, k, mem, C, P, tb, sig, n, &scr[0][threadIdx.x], kBlock);
    }
    store_x((XT *)b.X, n, i, x);
    store_disc(b.disc, n, i, D);
    b.k[i] = k;
    b.mem[i] = (uint8_t)mem;
}

template <typename XT>
__global__ __launch_bounds__(kBlock) void k_model_init(b747_model_batch b, const uint8_t *mask)
{
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mask && !mask[i]) return;
    double s0[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) s0[j] = b.state0[j * n + i];
    double x[NX];
    Disc D;
    uint32_t k, mem;
    initialize(x, D, k, mem, s0);
    store_x((XT *)b.X, n, i, x);
    store_disc(b.disc, n, i, D);
    b.k[i] = k;
    b.mem[i] = (uint8_t)mem;
    if (b.sig) {
#pragma unroll
        for (int j = 0; j < NSIG; ++j) b.sig[j * n + i] = 0.0;
    }
}

int32_t check_batch(const b747_model_batch *b, bool need_params)
{
    if (!b) return bad_arg("batch is NULL");
    if (b->n < 0) return bad_arg("n < 0");
    if (b->n == 0) return 0;
    if (!b->X || !b->disc || !b->k || !b->mem) return bad_arg("state pointer is NULL");
    if (need_params && (!b->deltaz || !b->vartheta || !b->h_zh || !b->flags || !b->aero_err))
        return bad_arg("parameter pointer is NULL");
    return 1;
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

// ------------------------------------------------------------------------------ C ABI ----
extern "C" {

__attribute__((visibility("default"))) int32_t b747_abi_version(void) { return B747_ABI_VERSION; }

__attribute__((visibility("default"))) const char *b747_last_error(void) { return g_err; }

__attribute__((visibility("default"))) int32_t b747_consts_default(b747_consts *c)
{
    if (!c) return bad_arg("consts is NULL");
    c->Iz = B747_DEF_IZ;
    c->P = B747_DEF_P;
    c->S = B747_DEF_S;
    c->c_ = B747_DEF_C;
    c->g = B747_DEF_G;
    c->m0 = B747_DEF_M0;
    for (int j = 0; j < 4; ++j) { c->PID_CS[j] = B747_DEF_PID_CS[j]; c->PID_SS[j] = B747_DEF_PID_SS[j]; }
    return 0;
}

__attribute__((visibility("default"))) int32_t b747_model_initialize(const b747_model_batch *b,
                                                                       const uint8_t *mask, void *stream)
{
    int32_t r = check_batch(b, false);
    if (r <= 0) return r;
    if (!b->state0) return bad_arg("state0 is NULL");
    hipStream_t s = (hipStream_t)stream;
    if (b->x_f64) hipLaunchKernelGGL(k_model_init<double>, dim3(grid_for(b->n)), dim3(kBlock), 0, s, *b, mask);
    else hipLaunchKernelGGL(k_model_init<float>, dim3(grid_for(b->n)), dim3(kBlock), 0, s, *b, mask);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_model_initialize");
}

__attribute__((visibility("default"))) int32_t b747_model_step(const b747_model_batch *b,
                                                                 const b747_consts *c, int32_t n_steps,
                                                                 void *stream)
{
    int32_t r = check_batch(b, true);
    if (r <= 0) return r;
    if (!c) return bad_arg("consts is NULL");
    if (n_steps < 0) return bad_arg("n_steps < 0");
    if (n_steps == 0) return 0;
    Consts C;
    C.Iz = c->Iz; C.P = c->P; C.S = c->S; C.c_ = c->c_; C.g = c->g; C.m0 = c->m0;
    for (int j = 0; j < 4; ++j) { C.PID_CS[j] = c->PID_CS[j]; C.PID_SS[j] = c->PID_SS[j]; }
    hipStream_t s = (hipStream_t)stream;
    if (b->x_f64) hipLaunchKernelGGL(k_model_step<double>, dim3(grid_for(b->n)), dim3(kBlock), 0, s, *b, C, n_steps);
    else hipLaunchKernelGGL(k_model_step<float>, dim3(grid_for(b->n)), dim3(kBlock), 0, s, *b, C, n_steps);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_model_step");
}

}  // extern "C"
