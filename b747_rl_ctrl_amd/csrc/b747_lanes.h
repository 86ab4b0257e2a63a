// b747_lanes.h -- the per-lane kernels of libb747.so (state load/store, env step, model step)
// and their launchers.  Included by two translation units: b747_kernels.hip instantiates the
// FAITHFUL variant (no FMA contraction: the DLL's roundings) and b747_fast.hip the FAST variant
// under `#pragma clang fp contract(fast)` (mul+add pairs become v_fma_f64: fewer VALU issues and
// shorter dependency chains).  Device code of each translation unit is its own code object, so
// the two instantiations never mix.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/b747.h"
#include "b747_dynamics.h"
#include "b747_karg.h"
#include "b747_env.h"

namespace b747 {
// FAST launchers, defined in b747_fast.hip (hidden: not part of the C ABI)
__attribute__((visibility("hidden"))) void launch_env_steps_fast(const b747_env_batch &b, const b747_env_config &cfg,
                                                                 const Consts &C, int kind, const float *actions,
                                                                 int32_t n_env_steps, float *obs_seq, float *reward_seq,
                                                                 uint8_t *done_seq, hipStream_t s);
__attribute__((visibility("hidden"))) void launch_ppo_rollout_fast(const b747_env_batch &b, const b747_env_config &cfg,
                                                                   const float *params, uint64_t seed,
                                                                   const uint64_t *step_base, int32_t T, float *obs_buf,
                                                                   float *act_buf, float *logp_buf, float *val_buf,
                                                                   float *rew_buf, uint8_t *done_buf, float act_lo,
                                                                   float act_hi, hipStream_t s);
__attribute__((visibility("hidden"))) void launch_model_step_fast(const b747_model_batch &b, const Consts &C,
                                                                  int32_t n_steps, bool split, hipStream_t s);
}  // namespace b747

namespace {

using namespace b747;

// The fp64 kernels are compiled without v_fmac_f64: its addend is tied to the destination, so every
// a*b + K with a constant K (the polynomial steps of the FAST math, table interpolation) cost two
// v_mov_b32 copying K into VGPRs; v_fma_f64 reads K from an SGPR pair instead (~60 fewer VALU per
// output pass).
#if defined(__HIP_DEVICE_COMPILE__)
#define B747_NO_FMAC __attribute__((target("no-fmacf64-inst")))
#else
#define B747_NO_FMAC
#endif

// __syncthreads() is not always-inline, and a callee whose target features differ from its caller's
// is never inlined: it would become a real call (with a scratch spill) in the B747_NO_FMAC kernels.
__device__ __forceinline__ void wg_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// some lane of the wave has p (HIP's __ballot is not always-inline: in the B747_NO_FMAC kernels it became a real
// call, with its register save / restore, after the prologue barrier)
__device__ __forceinline__ bool wave_any(bool p)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(p) != 0;
#else
    return p;
#endif
}
constexpr int kBlock = 256;

// Diagnostic build only (-DB747_STAMPS, the one diagnostic switch; tools/exp_stamps_split.py, tools/exp_stamps_ppo.py):
// per-wave s_memtime stamps of a kernel's phases in a buffer of their own.  Never compiled into the product library.
#ifdef B747_STAMPS
constexpr int kStampWaves = 4096, kStampSlots = 16;   // 0-7 phases, 8-15 end of env steps 0-7
__device__ unsigned long long g_b747_stamps[kStampWaves * kStampSlots];
__device__ __forceinline__ void stamp(int slot, bool real = false)
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    if (real) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    else asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && w < (unsigned)kStampWaves) g_b747_stamps[w * kStampSlots + slot] = t;
}
#define B747_STAMP(...) stamp(__VA_ARGS__)
#else
#define B747_STAMP(...) ((void)0)
#endif

// Stores of the per-step state: write-through (sc1) -- the lines leave the XCD's L2 during the launch instead of as
// dirty lines at the kernel boundary (MI355X_MICROARCH.md "boundary": + dirty bytes / 6 TB/s).  Two-wave per-step
// kernel: 9.9 us against 10.5 with write-back stores and 10.6 with non-temporal ones (tools/ab_bench.sh; the K-step
// and PPO rollout kernels, which store once per launch, unchanged).
template <typename T>
__device__ __forceinline__ void st_state(T *p, T v)
{
    static_assert(sizeof(T) == 8 || sizeof(T) == 4, "write-through state stores are 4 or 8 bytes");
    using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned>::type;
    U bits;
    __builtin_memcpy(&bits, &v, sizeof(T));
    __hip_atomic_store((U *)p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// PQ: the FAST pitch-plane quaternion (kPitchPlane, b747_dynamics.h): q1 = X[3] and q2 = X[4] are the
// constant +0 that initialize() stored, so the per-step path neither loads nor stores them (32 B/env).
template <typename XT, bool PQ = false>
__device__ __forceinline__ void load_x(const XT *__restrict__ X, int64_t n, int64_t i, double *x)
{
#pragma unroll
    for (int j = 0; j < NX; ++j) x[j] = (PQ && (j == 3 || j == 4)) ? 0.0 : (double)X[j * n + i];
}

template <typename XT, bool PQ = false>
__device__ __forceinline__ void store_x(XT *__restrict__ X, int64_t n, int64_t i, const double *x)
{
#pragma unroll
    for (int j = 0; j < NX; ++j)
        if (!(PQ && (j == 3 || j == 4))) st_state(&X[j * n + i], (XT)x[j]);
}

__device__ __forceinline__ void load_params(const b747_model_batch &b, int64_t i, Params &P)
{
    const int64_t n = b.n;
    P.deltaz = b.deltaz[i];
    P.vartheta = b.vartheta[i];
    P.h_zh = b.h_zh[i];
    P.flags = b.flags[i];
    P.kCX = b.aero_err[0 * n + i] + B747_F_ONE;    // fp64, as the DLL's parameter (core/model.py:164)
    P.kCY = b.aero_err[1 * n + i] + B747_F_ONE;
    P.kmz = b.aero_err[2 * n + i] + B747_M_ONE;
    P.kdCm = b.aero_err[3 * n + i] + B747_M_ONE;
    P.kKa = b.aero_err[4 * n + i] + B747_M_ONE;
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
    st_state(&disc[0 * n + i], D.x_dss);
    st_state(&disc[1 * n + i], D.y_dss);
    st_state(&disc[2 * n + i], D.rl_prevY);
    st_state(&disc[3 * n + i], D.e_prev);
    st_state(&disc[4 * n + i], D.ed_prev);
#pragma unroll
    for (int j = 0; j < 4; ++j) st_state(&disc[(5 + j) * n + i], D.u_hist[j]);
}

// ---------------------------------------------------------------- model-level kernels ----

template <typename XT, bool FAST, int BS = kBlock>
__global__ __launch_bounds__(BS) B747_NO_FMAC void k_model_step(b747_model_batch b, Consts C, int32_t n_steps)
{
    __shared__ __attribute__((aligned(16))) double tb[T_TOTAL];
    const unsigned kpd = prefetch_kernargs_issue<sizeof(b747_model_batch) + sizeof(Consts) + 8>();
    // As k_env_steps: this variant's table entries (Q per lane, all issued at once -- a load / LDS-write loop waits
    // out one memory round trip per iteration: 11 of them with config 2's 64-lane workgroups), then the lane's state,
    // then the LDS writes, one barrier: the prologue costs one round trip
    constexpr int lo = FAST ? T_FAST_LO : 0, hi = FAST ? T_TOTAL : T_N;
    constexpr int Q = (hi - lo + BS - 1) / BS;
    double tv[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = lo + (int)threadIdx.x + q * BS;
        tv[q] = (j < hi) ? kTableImage.v[j] : 0.0;
    }
    prefetch_kernargs_wait(kpd);
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
    const int64_t il = i < n ? i : n - 1;   // (lanes past n load env n - 1 and exit after the barrier)
    double x[NX];
    load_x((const XT *)b.X, n, il, x);
    Disc D;
    load_disc(b.disc, n, il, D);
    uint32_t k = b.k[il];
    uint32_t mem = b.mem[il];
    Params P;
    load_params(b, il, P);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = lo + (int)threadIdx.x + q * BS;
        if (j < hi) tb[j] = tv[q];
    }
    wg_barrier();
    if (i >= n) return;
    SigWriter wr{b.sig + i, n};
    for (int32_t s = 0; s < n_steps; ++s) {
        major_step<FAST>(x, D, k, mem, C, P, tb, wr, b.sig && s == n_steps - 1);
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


// ------------------------------------------------------------------ env-level kernels ----

// The reference's training configuration (main.py / env/ctrl_env.py defaults; BASELINE configs 3-5):
// PID_LIKE observation, CLASSIC reward, MANUAL control with DIRECT_CONTROL actions, CONST reference
// resets, AERO disturbance with drawn errors, normalised obs/action, no limiter, auto-reset.  Only the
// fields that select code paths are fixed; values (tk, limits, reward weights, seed, n_sub) stay
// run-time.  spec_config_matches is the launch-time test for kind 3.
constexpr int kSpecObs = OBS_PID_LIKE, kSpecRew = REW_CLASSIC, kSpecLimiter = 0;
__host__ __device__ __forceinline__ void spec_config(EnvCfg &c)
{
    c.obs_type = kSpecObs; c.reward_type = kSpecRew; c.ctrl_type = CT_MANUAL; c.ctrl_mode = CM_DIRECT;
    c.reset_ref_mode = RM_CONST; c.disturbance_mode = 0; c.norm_obs = 1; c.norm_act = 1; c.use_limiter = kSpecLimiter;
    c.auto_reset = 1; c.aero_fixed = 0;
}
inline bool spec_config_matches(const EnvCfg &c)
{
    EnvCfg s = c;
    spec_config(s);
    return s.obs_type == c.obs_type && s.reward_type == c.reward_type && s.ctrl_type == c.ctrl_type &&
           s.ctrl_mode == c.ctrl_mode && s.reset_ref_mode == c.reset_ref_mode && s.disturbance_mode == c.disturbance_mode &&
           s.norm_obs == c.norm_obs && s.norm_act == c.norm_act && s.use_limiter == c.use_limiter &&
           s.auto_reset == c.auto_reset && s.aero_fixed == c.aero_fixed;
}

struct EnvLane {
    double x[NX];
    Disc D;
    uint32_t k, mem;
    EnvSlot s;
    double aero[5];   // the DLL's double aero_err[5]
    double vartheta, h_zh;
};

// Per-step loads: only the slots this configuration uses (include/b747.h).  Every condition is
// uniform (batch config), never a loaded per-env value, so all loads of a lane issue at once and
// the kernel pays ONE memory round trip before the first output pass.  full = true (reset kernel)
// loads everything.
template <typename XT, bool PQ = false>
__device__ __forceinline__ void env_load(const b747_env_batch &b, const EnvCfg &cfg, int64_t i, EnvLane &L,
                                         bool full)
{
    const int64_t n = b.n;
    // issue order = first-use order (loads return in order): the MAJOR step starts with k, the delay
    // history and the DSS state, then the output pass reads X
    L.k = b.k[i];
    load_disc(b.disc, n, i, L.D);
    load_x<XT, PQ>((const XT *)b.X, n, i, L.x);
    L.mem = b.mem[i];
    // deltaz persists only through ANG_VEL integration; every other manual mode overwrites it from
    // the action, and with the SS PID on it keeps the 0 of Model.initialize
    L.s.deltaz = (full || cfg.ctrl_mode == CM_ANG_VEL) ? b.deltaz[i] : 0.0;
    L.s.flags = b.flags[i];
    // oscillating references only come from OSCILLATING resets or set_reference (reset mode NONE):
    // under CONST / HYBRID resets every reference is constant and ref_kind is not read;
    // the altitude command only matters where the CS PID can be on
    const bool osc = cfg.reset_ref_mode == RM_OSCILLATING || cfg.reset_ref_mode == RM_NONE;
    L.s.ref_kind = (full || osc) ? b.ref_kind[i] : (uint32_t)REF_CONST;
    const bool may_ctrl = cfg.ctrl_type == CT_FULL_AUTO || cfg.ctrl_type == CT_SEMI_MANUAL ||
                          cfg.reset_ref_mode == RM_HYBRID;
    const bool add = cfg.ctrl_mode == CM_ADD_PROC || cfg.ctrl_mode == CM_ADD_DIRECT;
    L.s.upid = (full || add) ? b.upid[i] : 0.0;
    L.s.tp = (full || cfg.reward_type == REW_TF_REFERENCE) ? b.tp[i] : 0.0;
    L.s.ep_ret = (double)b.ep_return[i];
    // env steps since the reset: each env step moves k to the next multiple of n_sub, so after a step ep_len =
    // ceil(k / n_sub) = floor(k_before / n_sub) + 1 -- a function of k alone, also for a counter that was not aligned
    L.s.ep_len = full ? b.ep_len[i] : (int32_t)(L.k / (uint32_t)cfg.n_sub);
    L.s.episode = full ? b.episode[i] : 0u;            // the reset path loads it when needed
    L.s.ref[0] = b.ref[i];
#pragma unroll
    for (int j = 1; j < 7; ++j) L.s.ref[j] = (full || osc) ? b.ref[j * n + i] : 0.0;
    L.s.ref[7] = (full || may_ctrl) ? b.ref[7 * n + i] : 0.0;
#pragma unroll
    for (int j = 0; j < 5; ++j) L.aero[j] = b.aero_err[j * n + i];
    L.vartheta = 0.0;                                   // recomputed by every step (see env_step_lane)
    L.h_zh = b.h_zh[i];
}

// ctrl0 = the env had the CS PID on when it was loaded.
// The dynamics state is stored with the rest at the end of the launch: storing it before the read-out
// (to drain during it) measured 0.8 us SLOWER -- a wave whose env resets then waits for its own stores
// (one vmcnt counter for loads and stores on gfx950) before the reset's loads, and some wave resets in
// every launch.
// EARLY: the env step already stored X / disc / k / mem (env_step_lane<..., EARLY>); only a reset in this
// launch (slot_params) rewrites them here.
template <typename XT, bool PQ = false, bool EARLY = false>
__device__ __forceinline__ void env_store(const b747_env_batch &b, const EnvCfg &cfg, int64_t i, const EnvLane &L,
                                          bool slot_params, bool ctrl0)
{
    const int64_t n = b.n;
    if (!EARLY || slot_params) {
        store_x<XT, PQ>((XT *)b.X, n, i, L.x);
        if (PQ && slot_params) {   // a reset in this launch: write initialize()'s q1 = q2 = +0 back as well
            st_state(&((XT *)b.X)[3 * n + i], (XT)L.x[3]);
            st_state(&((XT *)b.X)[4 * n + i], (XT)L.x[4]);
        }
        store_disc(b.disc, n, i, L.D);
        b.k[i] = L.k;
        b.mem[i] = (uint8_t)L.mem;
    }
    if (slot_params || cfg.ctrl_mode == CM_ANG_VEL) b.deltaz[i] = L.s.deltaz;
    if (slot_params || cfg.ctrl_mode == CM_ADD_PROC || cfg.ctrl_mode == CM_ADD_DIRECT) b.upid[i] = L.s.upid;
    if (slot_params || cfg.reward_type == REW_TF_REFERENCE) b.tp[i] = L.s.tp;
    b.ep_return[i] = (float)L.s.ep_ret;
    if (slot_params) b.ep_len[i] = L.s.ep_len;
    const bool ctrl = (L.s.flags & F_PID_CS) != 0u;
    if (slot_params) b.vartheta[i] = L.vartheta;
    if (slot_params || ctrl || ctrl0) b.h_zh[i] = L.h_zh;
    if (slot_params) {   // only resets change these
        b.flags[i] = (uint8_t)L.s.flags;
        b.episode[i] = L.s.episode;
#pragma unroll
        for (int j = 0; j < 8; ++j) b.ref[j * n + i] = L.s.ref[j];
        b.ref_kind[i] = (uint8_t)L.s.ref_kind;
#pragma unroll
        for (int j = 0; j < 5; ++j) b.aero_err[j * n + i] = L.aero[j];
    }
}

// Where an episode ends: the VecMonitor info (ep_final_*) and the device-side episode accumulators
// (ep_stats, include/b747.h).  Runs on done lanes only, so the per-step path pays nothing for it.
__device__ __forceinline__ void record_episode_end(const b747_env_batch &b, int64_t i, const EnvLane &L)
{
    if (b.ep_final_return) b.ep_final_return[i] = L.s.ep_ret;
    if (b.ep_final_len) b.ep_final_len[i] = L.s.ep_len;
    if (b.ep_stats) {
        b.ep_stats[i] += 1.0;
        b.ep_stats[b.n + i] += L.s.ep_ret;
        b.ep_stats[2 * b.n + i] += (double)L.s.ep_len;
    }
}

// Controller.reset + Model.initialize (core/controller.py:134-201, core/model.py:238-244)
// reload: the lane's episode / ref slots are not in registers yet (the per-step load skips them;
// a reset stores all of them, and the draws write subsets of ref).  False after an earlier reset
// in the same launch, which left the current values in L.
// owner: the lane owns env i.  Idle lanes of a partial last wave (k_ppo_rollout steps them on a copy
// of env n-1) must not write env n-1's state0 slot while that env's own lane is live.
__device__ __forceinline__ void env_reset_lane(const b747_env_batch &b, const EnvCfg &cfg, int64_t i, EnvLane &L,
                                               bool reload, bool owner = true)
{
    if (reload) {
        L.s.episode = b.episode[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) L.s.ref[j] = b.ref[j * b.n + i];
    }
    double s0[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) s0[j] = b.state0 ? b.state0[j * b.n + i] : (j == 1 ? 11000.0 : (j == 2 ? 259.1667 : 0.0));
    draw_reset(cfg, (uint64_t)(b.env_offset + i), L.s, s0, L.aero);
    if (owner && b.state0 && cfg.reset_ref_mode != RM_NONE) {   // Model.set_initial writes the state0 parameter
#pragma unroll
        for (int j = 0; j < 6; ++j) b.state0[j * b.n + i] = s0[j];
    }
    L.s.episode += 1u;
    initialize(L.x, L.D, L.k, L.mem, s0);
    L.s.deltaz = 0.0;      // Model.initialize: deltaz = vartheta_zh = 0
    L.vartheta = 0.0;
    L.s.upid = 0.0;        // all signals are 0 after initialize (A.6)
    L.s.ep_ret = 0.0;
    L.s.ep_len = 0;
}

// One ControllerEnv.step for this lane; returns done.  ONE: the caller guarantees n_sub == 1 (sample_time
// = dt), so the sub-step loop is a single straight-line DLL step.
// EARLY (with ONE, per-step kernel only): the discrete state / k / mem are stored right after the MAJOR
// pass and X right after the RK4 combine, before the read-out -- their stores drain while the wave still
// computes instead of in one burst at the end of every wave (env_store<..., EARLY> skips them).
template <bool FAST, bool REC, uint32_t SIGMASK = kAllSignals, bool ONE = false, bool EARLY = false,
          typename XT = double>
__device__ __forceinline__ bool env_step_lane(const b747_env_batch &b, const EnvCfg &cfg, const Consts &C,
                                              int64_t i, EnvLane &L, float a, float *obs_row, float *obs_row2,
                                              float *term_row, float &reward_out, const double *tb, double *sg,
                                              int sst, int step_ix = 0)
{
    static_assert(!EARLY || ONE, "early state stores need the single-DLL-step path");
    // env/ctrl_env.py:262-264: action *= action_max, in place on a float32 array
    const float a32 = cfg.norm_act ? (float)((double)a * cfg.action_max) : a;
    const double act = (double)a32;
    const double t = t_of(L.k);                        // Model.time read-out
    const bool use_ctrl = (L.s.flags & F_PID_CS) != 0u;
    const bool manual = (L.s.flags & F_PID_SS) == 0u;
    // core/controller.py:234-239: command injection.  With the CS PID on, the DLL parameter
    // vartheta keeps the 0 that Model.initialize wrote (core/model.py:243-244); with it off, h_zh
    // keeps its last value (only the unobservable CS-loop states read it).
    const double pref = use_ctrl ? 0.0 : pitch_ref(L.s, t);          // (both fields written on both
    const double href = use_ctrl ? L.s.ref[7] : L.h_zh;               //  paths: keeps L out of scratch)
    L.vartheta = pref;
    L.h_zh = href;
    // core/controller.py:240-250: action modes
    const double lim = 17 * PI / 180;
    if (manual) {
        double dz;
        switch (cfg.ctrl_mode) {
        case CM_ADD_PROC: dz = (1 + act) * L.s.upid; break;
        case CM_ADD_DIRECT: dz = act + L.s.upid; break;
        case CM_ANG_VEL: dz = L.s.deltaz + act * cfg.sample_time; break;
        default: dz = act; break;                      // DIRECT_CONTROL or None
        }
        if (cfg.ctrl_mode == CM_ADD_PROC || cfg.ctrl_mode == CM_ADD_DIRECT || cfg.ctrl_mode == CM_ANG_VEL)
            dz = dz < -lim ? -lim : (dz > lim ? lim : dz);   // np.clip
        L.s.deltaz = dz;
    }
    Params P;
    P.deltaz = L.s.deltaz;
    P.vartheta = L.vartheta;
    P.h_zh = L.h_zh;
    P.flags = L.s.flags;
    P.kCX = L.aero[0] + B747_F_ONE;
    P.kCY = L.aero[1] + B747_F_ONE;
    P.kmz = L.aero[2] + B747_M_ONE;
    P.kdCm = L.aero[3] + B747_M_ONE;
    P.kKa = L.aero[4] + B747_M_ONE;
    // core/controller.py:258-264: step until round(t/dt) is a multiple of round(sample_time/dt);
    // the last sub-step's stage-4 signals go to the LDS stash sg
    const SigStash<REC ? kAllSignals : SIGMASK> stash{sg, sst};
    const uint32_t nsub = (uint32_t)cfg.n_sub;
    const uint32_t steps = ONE ? 1u : nsub - (L.k % nsub);
    const bool rec = REC && b.sig != nullptr;          // Storage recording: every DLL step's signals
    const int64_t n = b.n;
    // Only what this DLL step changed is written back: the U_com history slot k & 3 (the ring of
    // b747_dynamics.h hist_put; the other three slots are unchanged) and the DSS pair only on its 0.05 s
    // tick (k % 5 == 0, dll@0x2711) -- 37 of the 230 bytes a step would otherwise write per env.
    auto early_disc = [&](const Disc &D, uint32_t k1, uint32_t mem) {
        if (EARLY) {
            const uint32_t k0 = k1 - 1u;
            if (k0 % 5u == 0u) {
                st_state(&b.disc[0 * n + i], D.x_dss);
                st_state(&b.disc[1 * n + i], D.y_dss);
            }
            st_state(&b.disc[2 * n + i], D.rl_prevY);
            st_state(&b.disc[3 * n + i], D.e_prev);
            st_state(&b.disc[4 * n + i], D.ed_prev);
            st_state(&b.disc[(int64_t)(5u + (k0 & 3u)) * n + i], hist_get(D.u_hist, k0));
            b.k[i] = k1;
            b.mem[i] = (uint8_t)mem;
        }
    };
    for (uint32_t q = 0; q < steps; ++q) {
        major_step<FAST>(L.x, L.D, L.k, L.mem, C, P, tb, stash, rec || q + 1u == steps, early_disc);
        if (rec) {
            double *row = b.sig + (int64_t)(nsub - steps + q) * NSIG * b.n;
#pragma unroll
            for (int j = 0; j < NSIG; ++j) row[j * b.n + i] = sg[j * sst];
        }
    }
    if (rec && b.rec_params) {   // the parameters this env step ran with (Storage columns vartheta_ref, hzh)
        b.rec_params[i] = L.vartheta;
        b.rec_params[n + i] = L.h_zh;
        b.rec_params[2 * n + i] = L.s.deltaz;
    }
    if (EARLY) store_x<XT, FAST && kPitchPlane>((XT *)b.X, n, i, L.x);
    EnvReadOut<FAST, REC ? kAllSignals : SIGMASK> ro{cfg, L.s.flags, L.s.deltaz, L.vartheta, obs_row, term_row, obs_row2, 0.0, L.s.upid, L.s.tp, false};
    ro(sg, sst);
    L.s.upid = ro.upid;
    L.s.tp = ro.tp;
    const float r32 = (float)ro.reward;
    reward_out = r32;
    L.s.ep_ret = vecmonitor_add(L.s.ep_ret, ro.reward);
    L.s.ep_len += 1;
    return ro.done;
}

// n_env_steps env steps per launch.  actions: [n_env_steps][N] (or b.action for 1 step);
// obs/reward/done of step t go to the *_seq buffers at offset t (nullable) and the last step's
// also to b.obs / b.reward / b.done.
// KIND: 0 = generic constants, 1 = the DLL's default constants as literals (DEFC),
// 2 = generic constants + per-DLL-step signal recording (b.sig; evaluation / Storage path),
// 3 = DEFC + the branch-selecting fields of the reference's training configuration as compile-time
//     values (spec_config_matches): the read-out, controller and reset code of every other
//     configuration folds away instead of sitting behind uniform branches.
// K1: one env step of one DLL step per launch (n_env_steps == 1, n_sub == 1: the per-step API at
//     sample_time = dt) -- no loop anywhere on the path, so the compiler's memory-wait placement is exact
//     and the first output pass starts on the fields it needs while the rest of the state still streams in.
template <typename XT, bool FAST, int KIND, bool K1 = false>
__global__ __launch_bounds__(kBlock) B747_NO_FMAC void k_env_steps(b747_env_batch b, b747_env_config cfgc, Consts Cin,
                                                      const float *actions, int32_t n_env_steps,
                                                      float *obs_seq, float *reward_seq, uint8_t *done_seq)
{
    __shared__ __attribute__((aligned(16))) double tb[T_TOTAL];
    constexpr uint32_t kSigMask = KIND == 3 ? readout_signal_mask(kSpecObs, kSpecRew, kSpecLimiter) : kAllSignals;
    __shared__ double sg[sig_rows(kSigMask)][kBlock];   // stage-4 signal stash, [row][lane]: conflict-free ds_*_b64
    unsigned kpd = prefetch_kernargs_issue<sizeof(b747_env_batch) + sizeof(b747_env_config) + sizeof(Consts) + 48>();
#if defined(__HIP_DEVICE_COMPILE__)
    if (FAST) prefetch_const_lines<sizeof(FitCoefs)>(kfit(0), kpd);
#endif
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    EnvCfg cfgk = cfgc;
    if (KIND == 3) spec_config(cfgk);
    const EnvCfg &cfg = cfgk;
    B747_STAMP(0, true);
    B747_STAMP(1);
    // Table image first (up to 3 entries per lane), then the lane's state: loads return in order, so
    // the LDS writes of the table wait only for the first loads and the whole prologue costs one
    // memory round trip.
    constexpr int lo = FAST ? T_FAST_LO : 0, hi = FAST ? T_TOTAL : T_N;   // this variant's part (stage_tables)
    static_assert(hi - lo <= 3 * kBlock, "table image must fit three entries per lane");
    const int j0 = lo + threadIdx.x, j1 = j0 + kBlock, j2 = j0 + 2 * kBlock;
    const double tv0 = (j0 < hi) ? kTableImage.v[j0] : 0.0;
    const double tv1 = (j1 < hi) ? kTableImage.v[j1] : 0.0;
    const double tv2 = (j2 < hi) ? kTableImage.v[j2] : 0.0;
    prefetch_kernargs_wait(kpd);
    // lanes past n load env n-1 (n >= 1 here) and exit after the barrier: no branch around the
    // loads, so the wait for the table entries can count outstanding loads precisely
    const int64_t il = i < n ? i : n - 1;
    EnvLane L;
    env_load<XT, FAST && kPitchPlane>(b, cfg, il, L, false);
    const float a0 = actions[il];          // step 0's action travels with the state loads
    if (j0 < hi) tb[j0] = tv0;
    if (j1 < hi) tb[j1] = tv1;
    if (j2 < hi) tb[j2] = tv2;
    wg_barrier();
    B747_STAMP(2);
    B747_STAMP(3);
    if (i >= n) return;
    const int od = b.obs_dim;
    const bool ctrl0 = (L.s.flags & F_PID_CS) != 0u;
    const Consts &C = (KIND == 1 || KIND == 3) ? kDefaultConsts : Cin;   // DEFC: the 14 constants become literals
    bool any_reset = false;
    const int32_t n_st = K1 ? 1 : n_env_steps;
    for (int32_t st = 0; st < n_st; ++st) {
        const float a = (st == 0) ? a0 : actions[(int64_t)st * n + i];
        const bool last = st == n_st - 1;
        float *seq_row = obs_seq ? obs_seq + ((int64_t)st * n + i) * od : nullptr;
        float *orow = last ? b.obs + i * od : seq_row;   // the last step's row goes to both
        float *orow2 = last ? seq_row : nullptr;
        float *trow = b.terminal_obs ? b.terminal_obs + i * od : nullptr;
        float r;
        const bool done = env_step_lane<FAST, KIND == 2, kSigMask, K1, K1, XT>(b, cfg, C, i, L, a, orow ? orow : b.obs + i * od, orow2,
                                                         trow, r, tb, &sg[0][threadIdx.x], kBlock, st);
        if (last) {
            b.reward[i] = r;
            b.done[i] = done ? 1 : 0;
        }
        if (reward_seq) reward_seq[(int64_t)st * n + i] = r;
        if (done_seq) done_seq[(int64_t)st * n + i] = done ? 1 : 0;
        if (done) {
            record_episode_end(b, i, L);
            if (cfg.auto_reset) {
                env_reset_lane(b, cfg, i, L, !any_reset);
                any_reset = true;
            }
        }
        if (st < 8) B747_STAMP(8 + st);
    }
    B747_STAMP(4);
    env_store<XT, FAST && kPitchPlane, K1>(b, cfg, i, L, any_reset, ctrl0);
    B747_STAMP(5);
    B747_STAMP(6);
    B747_STAMP(7, true);
}

template <typename XT>
__global__ __launch_bounds__(kBlock) void k_env_reset(b747_env_batch b, b747_env_config cfgc, const uint8_t *mask)
{
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mask && !mask[i]) return;
    const EnvCfg &cfg = cfgc;
    EnvLane L;
    env_load<XT>(b, cfg, i, L, true);
    env_reset_lane(b, cfg, i, L, false);
    env_store<XT>(b, cfg, i, L, true, true);
    for (int j = 0; j < b.obs_dim; ++j) b.obs[i * b.obs_dim + j] = 0.0f;
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// kind: 0 = generic constants, 1 = the DLL's defaults as literals, 2 = signal recording
template <bool FAST>
void launch_env_steps(const b747_env_batch &b, const b747_env_config &cfg, const Consts &C, int kind,
                      const float *actions, int32_t n_env_steps, float *obs_seq, float *reward_seq, uint8_t *done_seq,
                      hipStream_t s)
{
    const dim3 g(grid_for(b.n)), blk(kBlock);
#define B747_LAUNCH_ENV(XT, D) \
    hipLaunchKernelGGL((k_env_steps<XT, FAST, D>), g, blk, 0, s, b, cfg, C, actions, n_env_steps, obs_seq, reward_seq, \
                       done_seq)
    const bool k1 = n_env_steps == 1 && cfg.n_sub == 1;
#define B747_LAUNCH_ENV2(XT) \
    if (kind == 2) B747_LAUNCH_ENV(XT, 2); \
    else if (FAST && kind == 3 && k1) \
        hipLaunchKernelGGL((k_env_steps<XT, FAST, (FAST ? 3 : 1), true>), g, blk, 0, s, b, cfg, C, actions, 1, obs_seq, \
                           reward_seq, done_seq); \
    else if (FAST && kind == 3) B747_LAUNCH_ENV(XT, (FAST ? 3 : 1)); \
    else if (kind == 1) B747_LAUNCH_ENV(XT, 1); else B747_LAUNCH_ENV(XT, 0)
    if (b.x_f64) B747_LAUNCH_ENV2(double);
    else B747_LAUNCH_ENV2(float);
#undef B747_LAUNCH_ENV2
#undef B747_LAUNCH_ENV
}

template <bool FAST>
void launch_model_step(const b747_model_batch &b, const Consts &C, int32_t n_steps, hipStream_t s)
{
    // small batches (config 2: 4,096 envs): one wave per workgroup, so that the waves spread over n / 64 CUs instead of
    // sharing n / 256 (each then has a CU's LDS, instruction and scalar caches to itself): 9.36 against 10.25 us per
    // one-step launch at 4,096 envs, 5.30 against 5.38 us per step at 100 steps a launch (profiles/r06/config2_geometry.txt)
    if (b.n <= 16384) {
        const dim3 g((unsigned)((b.n + 63) / 64)), blk(64);
        if (b.x_f64) hipLaunchKernelGGL((k_model_step<double, FAST, 64>), g, blk, 0, s, b, C, n_steps);
        else hipLaunchKernelGGL((k_model_step<float, FAST, 64>), g, blk, 0, s, b, C, n_steps);
        return;
    }
    const dim3 g(grid_for(b.n)), blk(kBlock);
    if (b.x_f64) hipLaunchKernelGGL((k_model_step<double, FAST>), g, blk, 0, s, b, C, n_steps);
    else hipLaunchKernelGGL((k_model_step<float, FAST>), g, blk, 0, s, b, C, n_steps);
}

}  // namespace
