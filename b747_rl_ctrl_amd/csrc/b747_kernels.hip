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

#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../../include/b747.h"
#include "b747_dynamics.h"
#include "b747_env.h"
#include "b747_lanes.h"
#include "b747_policy.h"

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

int32_t check_env(const b747_env_batch *b, const b747_env_config *cfg)
{
    if (!b || !cfg) return bad_arg("env batch/config is NULL");
    if (b->n < 0) return bad_arg("n < 0");
    if (b->n == 0) return 0;
    if (!b->X || !b->disc || !b->k || !b->mem || !b->deltaz || !b->vartheta || !b->h_zh || !b->upid ||
        !b->tp || !b->flags || !b->aero_err || !b->ref || !b->ref_kind || !b->episode || !b->ep_return ||
        !b->ep_len || !b->obs || !b->reward || !b->done)
        return bad_arg("env batch pointer is NULL");
    if (cfg->obs_type < 0 || cfg->obs_type > 4) return bad_arg("obs_type");
    if (b->obs_dim != obs_dim_of(cfg->obs_type)) return bad_arg("obs_dim does not match obs_type");
    if (cfg->reward_type < 0 || cfg->reward_type > 4) return bad_arg("reward_type");
    if (cfg->n_sub < 1) return bad_arg("n_sub < 1 (sample_time < dt)");
    if (cfg->ctrl_mode < -1 || cfg->ctrl_mode > 3) return bad_arg("ctrl_mode");
    if (cfg->reset_ref_mode < -1 || cfg->reset_ref_mode > 2) return bad_arg("reset_ref_mode");
    return 1;
}

Consts consts_of(const b747_consts *c)
{
    return make_consts(c->Iz, c->P, c->S, c->c_, c->g, c->m0, c->PID_CS, c->PID_SS);
}

// The DLL's default constants (bitwise): such batches run the kernels specialised on them.
// kind 3 (config-specialised env kernel): on unless b747_set_specialization switches it off
static int32_t g_spec_kind = 1;

bool is_default(const b747_consts *c)
{
    const Consts &d = kDefaultConsts;
    bool same = c->Iz == d.Iz && c->P == d.P && c->S == d.S && c->c_ == d.c_ && c->g == d.g && c->m0 == d.m0;
    for (int j = 0; j < 4; ++j) same = same && c->PID_CS[j] == d.PID_CS[j] && c->PID_SS[j] == d.PID_SS[j];
    return same;
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

}  // namespace

// ------------------------------------------------------------------------------ C ABI ----
extern "C" {

__attribute__((visibility("default"))) int32_t b747_abi_version(void) { return B747_ABI_VERSION; }

__attribute__((visibility("default"))) int64_t b747_struct_size(int32_t which)
{
    switch (which) {
    case B747_STRUCT_CONSTS: return (int64_t)sizeof(b747_consts);
    case B747_STRUCT_MODEL_BATCH: return (int64_t)sizeof(b747_model_batch);
    case B747_STRUCT_ENV_CONFIG: return (int64_t)sizeof(b747_env_config);
    case B747_STRUCT_ENV_BATCH: return (int64_t)sizeof(b747_env_batch);
    default: return -1;
    }
}

__attribute__((visibility("default"))) const char *b747_last_error(void) { return g_err; }

__attribute__((visibility("default"))) int32_t b747_policy_num_params(int32_t obs_dim)
{
    if (obs_dim < 1 || obs_dim > 10) return bad_arg("obs_dim");
    return policy_total_params(obs_dim);
}

__attribute__((visibility("default"))) int32_t b747_policy_pack(float *params, int32_t obs_dim, void *stream)
{
    if (!params) return bad_arg("params is NULL");
    if (obs_dim < 1 || obs_dim > 10) return bad_arg("obs_dim");
    hipLaunchKernelGGL(k_policy_pack, dim3((policy_pack_threads(obs_dim) + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       params, (int)obs_dim);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_policy_pack");
}

__attribute__((visibility("default"))) int32_t b747_policy_act(const float *params, int32_t obs_dim, int64_t n,
                                                                 const float *obs, const float *noise, uint64_t seed,
                                                                 const uint64_t *step_base, uint32_t step,
                                                                 int64_t env_offset, float *obs_out,
                                                                 float *act_out, float *logp_out, float *value_out,
                                                                 float *env_action, float act_lo, float act_hi,
                                                                 void *stream)
{
    if (n < 0) return bad_arg("n < 0");
    if (n == 0) return 0;
    if (!params || !obs || !act_out || !logp_out || !value_out || !env_action) return bad_arg("NULL buffer");
    if (!(act_lo <= act_hi)) return bad_arg("act_lo > act_hi");
    hipStream_t s = (hipStream_t)stream;
    const dim3 g(grid_for(n)), blk(kBlock);
#define B747_LAUNCH_POLICY(OD)                                                                               \
    hipLaunchKernelGGL(k_policy_act<OD>, g, blk, 0, s, params, n, obs, noise, seed, step_base, step, env_offset, \
                       obs_out, \
                       act_out, logp_out, value_out, env_action, act_lo, act_hi)
    switch (obs_dim) {
    case 3: B747_LAUNCH_POLICY(3); break;
    case 5: B747_LAUNCH_POLICY(5); break;
    case 7: B747_LAUNCH_POLICY(7); break;
    case 8: B747_LAUNCH_POLICY(8); break;
    case 10: B747_LAUNCH_POLICY(10); break;
    default: return bad_arg("obs_dim (PID_LIKE 3, SPEED_MODE 5, MODEL_STATE 7, PID_AERO 8, PID_SPEED_AERO 10)");
    }
#undef B747_LAUNCH_POLICY
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_policy_act");
}

__attribute__((visibility("default"))) int32_t b747_ppo_rollout(const b747_env_batch *b, const b747_env_config *cfg,
                                                                 const b747_consts *c, const float *params,
                                                                 uint64_t seed, uint64_t *step_base, int32_t T,
                                                                 float *obs_buf, float *act_buf, float *logp_buf,
                                                                 float *val_buf, float *rew_buf, uint8_t *done_buf,
                                                                 float act_lo, float act_hi, void *stream)
{
    int32_t r = check_env(b, cfg);
    if (r <= 0) return r;
    if (!c || !params || !obs_buf || !act_buf || !logp_buf || !val_buf || !rew_buf || !done_buf)
        return bad_arg("NULL buffer");
    if (T < 0) return bad_arg("T < 0");
    if (!(act_lo <= act_hi)) return bad_arg("act_lo > act_hi");
    if (!is_default(c) || !spec_config_matches(*cfg) || !b->x_f64 || b->variant == B747_VARIANT_FAITHFUL ||
        b->obs_dim != 3 || b->n % 64 != 0 || b->sig)
        return bad_arg("b747_ppo_rollout: the fused kernel covers the training configuration only (default "
                       "constants, PID_LIKE/CLASSIC/MANUAL-DIRECT/CONST/AERO, fp64 state, FAST, n % 64 == 0); "
                       "use b747_policy_act + b747_env_step");
    if (T == 0) return 0;
    launch_ppo_rollout_fast(*b, *cfg, params, seed, step_base, T, obs_buf, act_buf, logp_buf, val_buf, rew_buf, done_buf,
                            act_lo, act_hi, (hipStream_t)stream);
    // the value head of every observation the rollout stored (V(obs_t), the rollout's parameters): one batched
    // launch after the rollout instead of inside its latency-bound step loop; it also advances *step_base by T
    const int64_t rows = (int64_t)T * b->n;
    hipLaunchKernelGGL(k_policy_value<3>, dim3((unsigned)policy_value_blocks(rows)), dim3(256), 0, (hipStream_t)stream,
                       params, rows, obs_buf, val_buf, step_base, (uint32_t)T);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_ppo_rollout");
}

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
    Consts C = consts_of(c);
    hipStream_t s = (hipStream_t)stream;
    // the three-wave one-step kernel where the specialised kernels are on (b747_set_specialization) and the constants
    // are the DLL's defaults (its control and flight sides take them as literals)
    if (b->variant != B747_VARIANT_FAITHFUL) launch_model_step_fast(*b, C, n_steps, g_spec_kind != 0 && is_default(c), s);
    else launch_model_step<false>(*b, C, n_steps, s);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_model_step");
}


__attribute__((visibility("default"))) int32_t b747_env_obs_dim(int32_t obs_type)
{
    if (obs_type < 0 || obs_type > 4) return bad_arg("obs_type");
    return obs_dim_of(obs_type);
}

__attribute__((visibility("default"))) int32_t b747_env_config_default(b747_env_config *cfg, int32_t obs_type,
                                                                         int32_t reward_type)
{
    if (!cfg) return bad_arg("cfg is NULL");
    memset(cfg, 0, sizeof(*cfg));
    cfg->obs_type = obs_type;
    cfg->reward_type = reward_type;
    cfg->ctrl_type = B747_CTRL_MANUAL;             // main.py:91
    cfg->ctrl_mode = B747_MODE_DIRECT;
    cfg->reset_ref_mode = B747_RESET_CONST;
    cfg->disturbance_mode = B747_DIST_NONE;
    cfg->norm_obs = 1;                             // main.py:15-16
    cfg->norm_act = 1;
    cfg->use_limiter = 0;
    cfg->auto_reset = 1;                           // SB3 VecEnv semantics
    cfg->sample_time = 0.05;                       // main.py:18
    cfg->n_sub = 5;
    cfg->tk = 20.0;                                // main.py:95
    cfg->action_max = 17 * PI / 180;               // Controller default / DIRECT_CONTROL
    cfg->vartheta_max = 10 * PI / 180;
    switch (reward_type) {
    case B747_REW_CLASSIC: {                       // env/ctrl_env.py:112-123
        double k1 = 2, k2 = 2, k3 = 1, s = k1 + k2 + k3;
        cfg->rew[0] = k1 / s; cfg->rew[1] = k2 / s; cfg->rew[2] = k3 / s;
        cfg->rew[3] = 0.1;                         // kf
        cfg->rew[4] = 0.3;                         // kITSE
        cfg->rew[5] = 2;                           // k0
        cfg->rew[6] = -log(0.8) / 10;              // kt = calc_exp_k(0.8, 10), tools/general.py:32
        cfg->rew[7] = -log(0.75) / 0.15;           // ko = calc_exp_k(0.75, 0.15)
        break;
    }
    case B747_REW_PID_LIKE: cfg->rew[0] = 10; break;                       // :146
    case B747_REW_MINIMAL: cfg->rew[0] = 0.2; cfg->rew[1] = 2; cfg->rew[2] = 0.5; break;  // :157-160
    case B747_REW_TF_REFERENCE: cfg->rew[0] = 2; cfg->rew[1] = 5; cfg->rew[2] = 0.1; break;  // :177-179
    default: break;
    }
    cfg->seed = 0;
    return 0;
}

__attribute__((visibility("default"))) int32_t b747_env_reset(const b747_env_batch *b, const b747_env_config *cfg,
                                                                const b747_consts *c, const uint8_t *mask,
                                                                void *stream)
{
    int32_t r = check_env(b, cfg);
    if (r <= 0) return r;
    (void)c;
    hipStream_t s = (hipStream_t)stream;
    if (b->x_f64) hipLaunchKernelGGL(k_env_reset<double>, dim3(grid_for(b->n)), dim3(kBlock), 0, s, *b, *cfg, mask);
    else hipLaunchKernelGGL(k_env_reset<float>, dim3(grid_for(b->n)), dim3(kBlock), 0, s, *b, *cfg, mask);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_env_reset");
}

__attribute__((visibility("default"))) int32_t b747_env_rollout(const b747_env_batch *b, const b747_env_config *cfg,
                                                                  const b747_consts *c, const float *actions,
                                                                  int32_t n_env_steps, float *obs_seq,
                                                                  float *reward_seq, uint8_t *done_seq, void *stream)
{
    int32_t r = check_env(b, cfg);
    if (r <= 0) return r;
    if (!c) return bad_arg("consts is NULL");
    if (!actions) return bad_arg("actions is NULL");
    if (n_env_steps < 0) return bad_arg("n_env_steps < 0");
    if (n_env_steps == 0) return 0;
    Consts C = consts_of(c);
    hipStream_t s = (hipStream_t)stream;
    // kind 4 = kind 3 where the FAST launcher may take the two-wave single-step kernel (b747_split.h)
    const int kind = b->sig ? 2 : (is_default(c) ? (g_spec_kind && spec_config_matches(*cfg) ? (g_spec_kind == 2 ? 3 : 4) : 1) : 0);
    if (b->variant != B747_VARIANT_FAITHFUL)
        launch_env_steps_fast(*b, *cfg, C, kind, actions, n_env_steps, obs_seq, reward_seq, done_seq, s);
    else launch_env_steps<false>(*b, *cfg, C, kind >= 3 ? 1 : kind, actions, n_env_steps, obs_seq, reward_seq, done_seq, s);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(e, "b747_env_rollout");
}

__attribute__((visibility("default"))) int32_t b747_env_kernel(const b747_env_batch *b, const b747_env_config *cfg,
                                                                 const b747_consts *c, int32_t n_env_steps)
{
    int32_t r = check_env(b, cfg);
    if (r <= 0) return r < 0 ? r : bad_arg("empty batch");
    if (!c) return bad_arg("consts is NULL");
    // the dispatch of b747_env_rollout / launch_env_steps_fast
    const int kind = b->sig ? 2 : (is_default(c) ? (g_spec_kind && spec_config_matches(*cfg) ? (g_spec_kind == 2 ? 3 : 4) : 1) : 0);
    if (b->variant == B747_VARIANT_FAITHFUL) return kind >= 3 ? B747_KERNEL_DEFC : kind;
    if (kind == 4) return (n_env_steps == 1 && cfg->n_sub == 1) ? B747_KERNEL_STEP_SPLIT : B747_KERNEL_ROLLOUT_SPLIT;
    return kind;
}

__attribute__((visibility("default"))) int32_t b747_set_specialization(int32_t on)
{
    const int32_t prev = g_spec_kind;
    g_spec_kind = (on == 2) ? 2 : (on ? 1 : 0);
    return prev;
}

__attribute__((visibility("default"))) int32_t b747_env_step(const b747_env_batch *b, const b747_env_config *cfg,
                                                               const b747_consts *c, void *stream)
{
    if (b && b->n > 0 && !b->action) return bad_arg("action is NULL");
    return b747_env_rollout(b, cfg, c, b ? b->action : nullptr, 1, nullptr, nullptr, nullptr, stream);
}

__attribute__((visibility("default"))) int32_t b747_env_step_seq(const b747_env_batch *b, const b747_env_config *cfg,
                                                                   const b747_consts *c, const float *actions,
                                                                   int32_t n_env_steps, void *stream)
{
    if (n_env_steps < 0 || (n_env_steps > 0 && !actions)) return bad_arg("actions/n_env_steps");
    for (int32_t t = 0; t < n_env_steps; ++t) {   // one per-step launch each, as n_env_steps b747_env_step calls
        const int32_t rc = b747_env_rollout(b, cfg, c, actions + (int64_t)t * (b ? b->n : 0), 1, nullptr, nullptr,
                                            nullptr, stream);
        if (rc != 0) return rc;
    }
    return 0;
}

__attribute__((visibility("default"))) int32_t b747_env_time_steps(const b747_env_batch *b,
                                                                     const b747_env_config *cfg,
                                                                     const b747_consts *c, const float *actions,
                                                                     int32_t n_env_steps, float *ms_out, void *stream)
{
    if (!ms_out || !actions || n_env_steps <= 0) return bad_arg("actions/ms_out/n_env_steps");
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t e0, e1;
    hipError_t e = hipEventCreateWithFlags(&e0, hipEventDisableSystemFence);
    if (e != hipSuccess) return fail(e, "hipEventCreateWithFlags");
    e = hipEventCreateWithFlags(&e1, hipEventDisableSystemFence);
    if (e != hipSuccess) { (void)hipEventDestroy(e0); return fail(e, "hipEventCreateWithFlags"); }
    int32_t rc = 0;
    for (int32_t t = 0; t < n_env_steps && rc == 0; ++t) {
        (void)hipEventRecord(e0, s);
        rc = b747_env_rollout(b, cfg, c, actions + (int64_t)t * b->n, 1, nullptr, nullptr, nullptr, stream);
        (void)hipEventRecord(e1, s);
        e = hipEventSynchronize(e1);
        if (e != hipSuccess) { rc = fail(e, "hipEventSynchronize"); break; }
        e = hipEventElapsedTime(&ms_out[t], e0, e1);
        if (e != hipSuccess) rc = fail(e, "hipEventElapsedTime");
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

}  // extern "C"
