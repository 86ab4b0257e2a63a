// b747_fast.hip -- the FAST variant's kernels (b747_lanes.h instantiated with FAST = true).
// A separate translation unit so that FMA contraction applies to FAST only: the FAITHFUL
// kernels in b747_kernels.hip keep the DLL's separate mul/add roundings (-ffp-contract=off),
// while here every a*b+c of the dynamics becomes one v_fma_f64 (one rounding instead of two:
// within FAST's per-step tolerance).
#pragma clang fp contract(fast)

#include "b747_lanes.h"
#include "b747_split.h"
#include "b747_model_split.h"


#define B747_POLICY_NO_KERNELS   // the policy kernels live in b747_kernels.hip; this unit reuses actor_critic
#include "b747_policy.h"
#include "b747_ppo_split.h"

namespace b747 {

void launch_env_steps_fast(const b747_env_batch &b, const b747_env_config &cfg, const Consts &C, int kind,
                           const float *actions, int32_t n_env_steps, float *obs_seq, float *reward_seq,
                           uint8_t *done_seq, hipStream_t s)
{
    // the training configuration (kind 4): each env over a flight and a control wave.  MIXED: the same kernels with
    // the flight aerodynamics in fp32 (include/b747.h B747_VARIANT_MIXED)
    const bool mix = b.variant == B747_VARIANT_MIXED;
    const dim3 grid((unsigned)((b.n + kSplitEnvs - 1) / kSplitEnvs));
    if (kind == 4 && n_env_steps == 1 && cfg.n_sub == 1) {   // the per-step API (b747_split.h)
        // 256 envs per workgroup (four wave triples, the three waves of a triple on one SIMD); small batches 64 (one
        // triple: its three waves run on three SIMDs of a CU, and n / 64 CUs work instead of n / 256) -- faster up to
        // 32,768 envs, slower at 65,536 (profiles/r06/small_batch_env_step.txt)
        const bool small = b.n <= 32768;
        const dim3 g64((unsigned)((b.n + 63) / 64));
#define B747_STEP_SPLIT(XT, MIX) do { \
            if (small) hipLaunchKernelGGL((k_env_step_split<XT, MIX, 64>), g64, dim3(3 * 64), 0, s, b.n, (const void *)b.X, \
                                          (const double *)b.aero_err, (const uint32_t *)b.k, (const double *)b.disc, \
                                          (const uint8_t *)b.flags, actions, b, cfg, obs_seq, reward_seq, done_seq); \
            else hipLaunchKernelGGL((k_env_step_split<XT, MIX>), grid, dim3(kStepBlock), 0, s, b.n, (const void *)b.X, \
                                    (const double *)b.aero_err, (const uint32_t *)b.k, (const double *)b.disc, \
                                    (const uint8_t *)b.flags, actions, b, cfg, obs_seq, reward_seq, done_seq); \
        } while (0)
        if (b.x_f64) { if (mix) B747_STEP_SPLIT(double, true); else B747_STEP_SPLIT(double, false); }
        else { if (mix) B747_STEP_SPLIT(float, true); else B747_STEP_SPLIT(float, false); }
#undef B747_STEP_SPLIT
        return;
    }
    if (kind == 4) {
        // K steps per launch (b747_env_rollout), or one env step of n_sub > 1 DLL steps: the rollout kernel of
        // b747_ppo_rollout without the policy -- the two roles hand off per wave pair and the flight wave never waits
        // for the next step's controller (b747_ppo_split.h)
        const RolloutArgs ra{nullptr, 0, nullptr, actions, n_env_steps, obs_seq, nullptr, nullptr, reward_seq, done_seq,
                             0.0f, 0.0f, nullptr};
        const bool sub = cfg.n_sub > 1;
        // (small batches: one flight / control pair per 64-env workgroup, the two waves on two SIMDs, as the per-step
        // kernel; faster up to 16,384 envs, slower from 24,576)
        const bool small = b.n <= 16384;
        const dim3 g64((unsigned)((b.n + 63) / 64));
#define B747_ROLL(XT, SUB, MIX) do { \
            if (small) hipLaunchKernelGGL((k_rollout_split<false, XT, SUB, MIX, 64>), g64, dim3(2 * 64), 0, s, b, cfg, ra); \
            else hipLaunchKernelGGL((k_rollout_split<false, XT, SUB, MIX>), grid, dim3(kSplitBlock), 0, s, b, cfg, ra); \
        } while (0)
        if (b.x_f64) {
            if (sub) { if (mix) B747_ROLL(double, true, true); else B747_ROLL(double, true, false); }
            else { if (mix) B747_ROLL(double, false, true); else B747_ROLL(double, false, false); }
        } else {
            if (sub) { if (mix) B747_ROLL(float, true, true); else B747_ROLL(float, true, false); }
            else { if (mix) B747_ROLL(float, false, true); else B747_ROLL(float, false, false); }
        }
#undef B747_ROLL
        return;
    }
    launch_env_steps<true>(b, cfg, C, kind == 4 ? 3 : kind, actions, n_env_steps, obs_seq, reward_seq, done_seq, s);
}

void launch_model_step_fast(const b747_model_batch &b, const Consts &C, int32_t n_steps, bool split, hipStream_t s)
{
    // the DLL's default constants: each env over three waves (b747_model_split.h) -- one step (BASELINE config 2's
    // per-step calls), or K steps with the state in registers for small batches (config 2's 100-step launches; above
    // 16,384 envs the one-wave kernel, whose single wave per env keeps every SIMD at one wave per 64 envs)
    const dim3 g((unsigned)((b.n + kMsEnvs - 1) / kMsEnvs)), blk(kMsBlock);
    if (split && n_steps == 1) {
        if (b.x_f64) hipLaunchKernelGGL((k_model_step_split<double>), g, blk, 0, s, b);
        else hipLaunchKernelGGL((k_model_step_split<float>), g, blk, 0, s, b);
        return;
    }
    if (split && b.n <= 16384) {
        if (b.x_f64) hipLaunchKernelGGL((k_model_steps_split<double>), g, blk, 0, s, b, n_steps);
        else hipLaunchKernelGGL((k_model_steps_split<float>), g, blk, 0, s, b, n_steps);
        return;
    }
    launch_model_step<true>(b, C, n_steps, s);
}

void launch_ppo_rollout_fast(const b747_env_batch &b, const b747_env_config &cfg, const float *params, uint64_t seed,
                             const uint64_t *step_base, int32_t T, float *obs_buf, float *act_buf, float *logp_buf,
                             float *val_buf, float *rew_buf, uint8_t *done_buf, float act_lo, float act_hi,
                             hipStream_t s)
{
    const RolloutArgs ra{params, seed, step_base, nullptr, T, obs_buf, act_buf, logp_buf, rew_buf, done_buf, act_lo, act_hi,
                         val_buf};
    const dim3 grid((unsigned)((b.n + kSplitEnvs - 1) / kSplitEnvs));
    const bool mix = b.variant == B747_VARIANT_MIXED;
    const bool small = b.n <= 32768;   // (one flight / control pair per 64-env workgroup, as b747_env_rollout; the policy
                                       //  then fits without spilling: faster up to 32,768 envs, slower at 65,536)
    const dim3 g64((unsigned)((b.n + 63) / 64));
#define B747_PPO(SUB, MIX) do { \
        if (small) hipLaunchKernelGGL((k_rollout_split<true, double, SUB, MIX, 64>), g64, dim3(2 * 64), 0, s, b, cfg, ra); \
        else hipLaunchKernelGGL((k_rollout_split<true, double, SUB, MIX>), grid, dim3(kSplitBlock), 0, s, b, cfg, ra); \
    } while (0)
    // sample_time > dt (main.py's 0.05): n_sub DLL steps per env step (core/controller.py:258-264)
    if (cfg.n_sub > 1) { if (mix) B747_PPO(true, true); else B747_PPO(true, false); }
    else { if (mix) B747_PPO(false, true); else B747_PPO(false, false); }
#undef B747_PPO
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
