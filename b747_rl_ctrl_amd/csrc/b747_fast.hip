// b747_fast.hip -- the FAST variant's kernels (b747_lanes.h instantiated with FAST = true).
// A separate translation unit so that FMA contraction applies to FAST only: the FAITHFUL
// kernels in b747_kernels.hip keep the DLL's separate mul/add roundings (-ffp-contract=off),
// while here every a*b+c of the dynamics becomes one v_fma_f64 (one rounding instead of two:
// within FAST's per-step tolerance).
#pragma clang fp contract(fast)

#include "b747_lanes.h"
#include "b747_split.h"
#include "b747_split_steps.h"
#define B747_POLICY_NO_KERNELS   // the policy kernels live in b747_kernels.hip; this unit reuses actor_critic
#include "b747_policy.h"
#ifndef B747_STEPS_PAIR
#define B747_STEPS_PAIR 1        // K env steps per launch (b747_env_rollout) on that kernel's pair protocol, not k_env_steps_split
#endif
#if B747_PPO_SPLIT
#include "b747_ppo_split.h"
#endif

namespace {

using namespace b747;

// Fused config-5 rollout (BASELINE configs[4]): T steps of SB3 collect_rollouts for every env in ONE
// launch -- policy forward (actor_critic, the k_policy_act math), Gaussian sample (policy_noise, the
// same Philox draws), clip, then the env step of the kind-3 kernel -- with the env state, the
// observation and the action in registers across steps instead of a policy launch and an env launch
// per step with their HBM round trips and kernel boundaries.  Training configuration only (kind 3:
// spec_config, default constants, fp64 state, PID_LIKE obs_dim 3); n a multiple of 64 (every wave
// runs the matrix-core layers with all 64 lanes).  Outputs per step t, row t*n + i: obs_buf (the
// observation the policy saw), act_buf (unclipped sample), logp_buf, val_buf, rew_buf, done_buf;
// afterwards b.obs / b.reward / b.done hold the last step's.
__global__ __launch_bounds__(kBlock) B747_NO_FMAC void k_ppo_rollout(b747_env_batch b, b747_env_config cfgc,
                                                                    const float *__restrict__ params, uint64_t seed,
                                                                    const uint64_t *step_base, int32_t T,
                                                                    float *obs_buf, float *act_buf, float *logp_buf,
                                                                    float *val_buf, float *rew_buf, uint8_t *done_buf,
                                                                    float act_lo, float act_hi)
{
    constexpr int OD = 3;
    constexpr PolicyDerived PD = PolicyDerived::of(OD);
    __shared__ __attribute__((aligned(16))) double tb[T_TOTAL];
    constexpr uint32_t sigmask = readout_signal_mask(kSpecObs, kSpecRew, kSpecLimiter);
    __shared__ double sg[sig_rows(sigmask)][kBlock];   // the read-out's 8 signals
    __shared__ float w[PD.total];
    // the env's continuous and discrete state waits here while the policy runs: the policy's
    // activations and matrix fragments then have the register file (no scratch spills)
    constexpr int kPark = NX + NDISC + 4 + 5 + 8;   // + aero_err, ref (float64, ABI v7)
    __shared__ double park[kPark][kBlock];
#ifndef B747_PPO_GLOBAL_FRAGS
    // the policy's matrix-core A fragments (36 KB, the same for every wave): staged once per launch, read
    // from LDS every rollout step instead of from L2 (actor_critic fr)
    __shared__ uint4 frag[kPolicyFragUint4];
#endif
    unsigned kpd = prefetch_kernargs_issue<sizeof(b747_env_batch) + sizeof(b747_env_config) + 96>();
#if defined(__HIP_DEVICE_COMPILE__)
    prefetch_const_lines<sizeof(FitCoefs)>(kfit(0), kpd);
#endif
    const int64_t n = b.n;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    EnvCfg cfgk = cfgc;
    spec_config(cfgk);
    const EnvCfg &cfg = cfgk;
    // table image (FAST part) and the policy's small parameters, all loads issued before the LDS writes
    constexpr int lo = T_FAST_LO, hi = T_TOTAL;
    const int j0 = lo + threadIdx.x, j1 = j0 + kBlock, j2 = j0 + 2 * kBlock;
    const double tv0 = (j0 < hi) ? kTableImage.v[j0] : 0.0;
    const double tv1 = (j1 < hi) ? kTableImage.v[j1] : 0.0;
    const double tv2 = (j2 < hi) ? kTableImage.v[j2] : 0.0;
    prefetch_kernargs_wait(kpd);
    PolicyStage<OD, kBlock> stage;
    stage.load(params, threadIdx.x);
    const bool valid = i < n;
    const int64_t il = valid ? i : n - 1;
    EnvLane L;
    env_load<double, kPitchPlane>(b, cfg, il, L, false);
    float o[OD];
#pragma unroll
    for (int k = 0; k < OD; ++k) o[k] = b.obs[il * OD + k];
    if (j0 < hi) tb[j0] = tv0;
    if (j1 < hi) tb[j1] = tv1;
    if (j2 < hi) tb[j2] = tv2;
    stage.store(w, threadIdx.x);
#ifndef B747_PPO_GLOBAL_FRAGS
    {
        static_assert(OD <= kL1MaxOD, "LDS fragments: the matrix-core layer 1");
        const uint4 *gl1 = reinterpret_cast<const uint4 *>(params + policy_l1pack_offset(OD));
        const uint4 *gpk = reinterpret_cast<const uint4 *>(params + policy_packed_offset(OD));
        for (int q = threadIdx.x; q < kPolicyFragUint4; q += kBlock) frag[q] = q < 4 * 64 ? gl1[q] : gpk[q - 4 * 64];
    }
    const uint4 *fr = frag;
#else
    const uint4 *fr = nullptr;
#endif
    wg_barrier();
    const int lane = threadIdx.x & 63;
    const bool ctrl0 = (L.s.flags & F_PID_CS) != 0u;
    const Consts &C = kDefaultConsts;
    const float log_std = w[PD.log_std];
    const float sdev = expf(log_std);
    const uint64_t ctr0 = step_base ? *step_base : 0u;
    bool any_reset = false, done = false;
    float r = 0.0f;
    for (int32_t t = 0; t < T; ++t) {
        double *pk = &park[0][threadIdx.x];
#pragma unroll
        for (int j = 0; j < NX; ++j) pk[j * kBlock] = L.x[j];
        pk[(NX + 0) * kBlock] = L.D.x_dss; pk[(NX + 1) * kBlock] = L.D.y_dss; pk[(NX + 2) * kBlock] = L.D.rl_prevY;
        pk[(NX + 3) * kBlock] = L.D.e_prev; pk[(NX + 4) * kBlock] = L.D.ed_prev;
#pragma unroll
        for (int j = 0; j < 4; ++j) pk[(NX + 5 + j) * kBlock] = L.D.u_hist[j];
        pk[(NX + 9) * kBlock] = L.s.ep_ret; pk[(NX + 10) * kBlock] = L.h_zh; pk[(NX + 11) * kBlock] = L.vartheta;
        pk[(NX + 12) * kBlock] = L.s.deltaz;
        double *pf = pk + (NX + 13) * kBlock;
#pragma unroll
        for (int j = 0; j < 5; ++j) pf[j * kBlock] = L.aero[j];
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[(5 + j) * kBlock] = L.s.ref[j];
        asm volatile("" ::: "memory");                  // the registers holding them are free from here
        float mean, value;
        // the value head is deferred to k_policy_value over the whole obs_buf (B747_PPO_VALUE_PASS)
        actor_critic<OD, false, B747_PPO_VALUE_PASS ? 1 : 3>(w, params, params + policy_derived_offset(OD), o, lane, mean,
                                                             value, fr);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < NX; ++j) L.x[j] = pk[j * kBlock];
        L.D.x_dss = pk[(NX + 0) * kBlock]; L.D.y_dss = pk[(NX + 1) * kBlock]; L.D.rl_prevY = pk[(NX + 2) * kBlock];
        L.D.e_prev = pk[(NX + 3) * kBlock]; L.D.ed_prev = pk[(NX + 4) * kBlock];
#pragma unroll
        for (int j = 0; j < 4; ++j) L.D.u_hist[j] = pk[(NX + 5 + j) * kBlock];
        L.s.ep_ret = pk[(NX + 9) * kBlock]; L.h_zh = pk[(NX + 10) * kBlock]; L.vartheta = pk[(NX + 11) * kBlock];
        L.s.deltaz = pk[(NX + 12) * kBlock];
#pragma unroll
        for (int j = 0; j < 5; ++j) L.aero[j] = pf[j * kBlock];
#pragma unroll
        for (int j = 0; j < 8; ++j) L.s.ref[j] = pf[(5 + j) * kBlock];
        const float z = policy_noise(seed, ctr0 + (uint64_t)t, (uint64_t)(b.env_offset + il));
        const float a = __fadd_rn(mean, __fmul_rn(sdev, z));                   // k_policy_act: mean + std z
        const float aenv = fminf(fmaxf(a, act_lo), act_hi);
        const int64_t row = (int64_t)t * n + i;
        if (valid) {
#pragma unroll
            for (int k = 0; k < OD; ++k) obs_buf[row * OD + k] = o[k];
            act_buf[row] = a;
            logp_buf[row] = __fsub_rn(__fsub_rn(__fmul_rn(__fmul_rn(-0.5f, z), z), log_std), 0.918938533204672742f);
            if (!B747_PPO_VALUE_PASS) val_buf[row] = value;
        }
        float onew[OBS_MAX_DIM];
        float *trow = (valid && b.terminal_obs) ? b.terminal_obs + i * OD : nullptr;
        done = env_step_lane<true, false, sigmask>(b, cfg, C, il, L, aenv, onew, nullptr, trow, r, tb,
                                                    &sg[0][threadIdx.x], kBlock, t);
        if (valid) {
            rew_buf[row] = r;
            done_buf[row] = done ? 1 : 0;
        }
        if (done) {
            if (valid) record_episode_end(b, i, L);
            env_reset_lane(b, cfg, il, L, !any_reset, valid);
            any_reset = true;
        }
#pragma unroll
        for (int k = 0; k < OD; ++k) o[k] = onew[k];
    }
    if (!valid) return;
#pragma unroll
    for (int k = 0; k < OD; ++k) b.obs[i * OD + k] = o[k];
    b.reward[i] = r;
    b.done[i] = done ? 1 : 0;
    env_store<double, kPitchPlane>(b, cfg, i, L, any_reset, ctrl0);
}

}  // namespace

namespace b747 {

void launch_env_steps_fast(const b747_env_batch &b, const b747_env_config &cfg, const Consts &C, int kind,
                           const float *actions, int32_t n_env_steps, float *obs_seq, float *reward_seq,
                           uint8_t *done_seq, hipStream_t s)
{
#ifndef B747_NO_SPLIT
    // the per-step API of the training configuration: each env over a flight and a control wave
    // MIXED: the same kernels with the flight aerodynamics in fp32 (include/b747.h B747_VARIANT_MIXED)
    const bool mix = b.variant == B747_VARIANT_MIXED;
    if (kind == 4 && n_env_steps == 1 && cfg.n_sub == 1) {
        const dim3 grid((unsigned)((b.n + kSplitEnvs - 1) / kSplitEnvs));
#define B747_STEP_SPLIT(XT, MIX) hipLaunchKernelGGL((k_env_step_split<XT, MIX>), grid, dim3(kSplitBlock), 0, s, b, cfg, \
                                                    actions, obs_seq, reward_seq, done_seq)
        if (b.x_f64) { if (mix) B747_STEP_SPLIT(double, true); else B747_STEP_SPLIT(double, false); }
        else { if (mix) B747_STEP_SPLIT(float, true); else B747_STEP_SPLIT(float, false); }
#undef B747_STEP_SPLIT
        return;
    }
#ifndef B747_NO_SPLIT_STEPS
    // K steps per launch (b747_env_rollout), or one env step of n_sub > 1 DLL steps: the same two-wave step in a
    // loop, state in registers
    if (kind == 4 && (n_env_steps > 1 || cfg.n_sub > 1)) {
        const dim3 grid((unsigned)((b.n + kSplitEnvs - 1) / kSplitEnvs));
#if B747_PPO_SPLIT && B747_STEPS_PAIR
        // the rollout kernel of b747_ppo_rollout without the policy: the two roles hand off per wave pair and the
        // flight wave never waits for the next step's controller (b747_ppo_split.h)
        const RolloutArgs ra{nullptr, 0, nullptr, actions, n_env_steps, obs_seq, nullptr, nullptr, reward_seq, done_seq,
                             0.0f, 0.0f, nullptr};
        const bool sub = cfg.n_sub > 1;
#define B747_ROLL(XT, SUB, MIX) hipLaunchKernelGGL((k_rollout_split<false, XT, SUB, MIX>), grid, dim3(kSplitBlock), 0, s, b, \
                                                   cfg, ra)
        if (b.x_f64) {
            if (sub) { if (mix) B747_ROLL(double, true, true); else B747_ROLL(double, true, false); }
            else { if (mix) B747_ROLL(double, false, true); else B747_ROLL(double, false, false); }
        } else {
            if (sub) { if (mix) B747_ROLL(float, true, true); else B747_ROLL(float, true, false); }
            else { if (mix) B747_ROLL(float, false, true); else B747_ROLL(float, false, false); }
        }
#undef B747_ROLL
        return;
#else
        if (cfg.n_sub == 1) {
            if (b.x_f64)
                hipLaunchKernelGGL(k_env_steps_split<double>, grid, dim3(kSplitBlock), 0, s, b, cfg, actions, n_env_steps,
                                   obs_seq, reward_seq, done_seq);
            else
                hipLaunchKernelGGL(k_env_steps_split<float>, grid, dim3(kSplitBlock), 0, s, b, cfg, actions, n_env_steps,
                                   obs_seq, reward_seq, done_seq);
            return;
        }
#endif
    }
#endif
#endif
    launch_env_steps<true>(b, cfg, C, kind == 4 ? 3 : kind, actions, n_env_steps, obs_seq, reward_seq, done_seq, s);
}

void launch_model_step_fast(const b747_model_batch &b, const Consts &C, int32_t n_steps, hipStream_t s)
{
    launch_model_step<true>(b, C, n_steps, s);
}

void launch_ppo_rollout_fast(const b747_env_batch &b, const b747_env_config &cfg, const float *params, uint64_t seed,
                             const uint64_t *step_base, int32_t T, float *obs_buf, float *act_buf, float *logp_buf,
                             float *val_buf, float *rew_buf, uint8_t *done_buf, float act_lo, float act_hi,
                             hipStream_t s)
{
#if B747_PPO_SPLIT
    const RolloutArgs ra{params, seed, step_base, nullptr, T, obs_buf, act_buf, logp_buf, rew_buf, done_buf, act_lo, act_hi,
                         val_buf};
    const dim3 grid((unsigned)((b.n + kSplitEnvs - 1) / kSplitEnvs));
    const bool mix = b.variant == B747_VARIANT_MIXED;
#define B747_PPO(SUB, MIX) hipLaunchKernelGGL((k_rollout_split<true, double, SUB, MIX>), grid, dim3(kSplitBlock), 0, s, b, cfg, ra)
    // sample_time > dt (main.py's 0.05): n_sub DLL steps per env step (core/controller.py:258-264)
    if (cfg.n_sub > 1) { if (mix) B747_PPO(true, true); else B747_PPO(true, false); }
    else { if (mix) B747_PPO(false, true); else B747_PPO(false, false); }
#undef B747_PPO
#else
    hipLaunchKernelGGL(k_ppo_rollout, dim3(grid_for(b.n)), dim3(kBlock), 0, s, b, cfg, params, seed, step_base, T,
                       obs_buf, act_buf, logp_buf, val_buf, rew_buf, done_buf, act_lo, act_hi);
#endif
}

}  // namespace b747

#ifdef B747_STAMPS
// diagnostic build only: copy the per-wave phase stamps of the last FAST env-step launch to the host
extern "C" __attribute__((visibility("default"))) int b747_debug_stamps(unsigned long long *out, int n)
{
    const size_t bytes = sizeof(unsigned long long) * (size_t)(n < kStampWaves * kStampSlots ? n : kStampWaves * kStampSlots);
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_b747_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
