// b747_fast.hip -- the FAST variant's kernels (b747_lanes.h instantiated with FAST = true).
// A separate translation unit so that FMA contraction applies to FAST only: the FAITHFUL
// kernels in b747_kernels.hip keep the DLL's separate mul/add roundings (-ffp-contract=off),
// while here every a*b+c of the dynamics becomes one v_fma_f64 (one rounding instead of two:
// within FAST's per-step tolerance).
#pragma clang fp contract(fast)

#include "b747_lanes.h"

namespace b747 {

void launch_env_steps_fast(const b747_env_batch &b, const b747_env_config &cfg, const Consts &C, int kind,
                           const float *actions, int32_t n_env_steps, float *obs_seq, float *reward_seq,
                           uint8_t *done_seq, hipStream_t s)
{
    launch_env_steps<true>(b, cfg, C, kind, actions, n_env_steps, obs_seq, reward_seq, done_seq, s);
}

void launch_model_step_fast(const b747_model_batch &b, const Consts &C, int32_t n_steps, hipStream_t s)
{
    launch_model_step<true>(b, C, n_steps, s);
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
