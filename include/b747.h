/* b747.h -- C ABI of libb747.so, the MI355X-native batched B747 pitch-control environment.
 *
 * Drop-in boundary.  The reference drives ONE aircraft per process through the Simulink
 * "exported globals" ABI of core/model_simple_win64.dll via ctypes:
 *     model_simple_initialize()   core/model.py:124 (bound), :238-244 (Model.initialize)
 *     model_simple_step()         core/model.py:125,          :247-250 (Model.step)
 *     model_simple_terminate()    core/model.py:126,          :253-256
 *     parameter / signal globals  core/model.py:129-164 (in_dll bindings)
 * and the env loop on top of it (core/controller.py:134-264, env/ctrl_env.py:237-278).
 * This library replaces that whole chain for N environments at once:
 *   - b747_model_*  : the DLL ABI, batched.  Every exported global becomes a [N] (or [k][N])
 *                     device array; initialize/step act on all envs (or a masked subset).
 *   - b747_env_*    : ControllerEnv.step/reset (obs -> action -> reward -> done, sub-stepping,
 *                     action modes, random resets) fused into one launch per env step.
 * All pointers are DEVICE pointers (e.g. torch.Tensor.data_ptr() of ROCm tensors), laid out
 * structure-of-arrays: field-major, env-minor ("[F][N]").  Every call is asynchronous on the
 * given HIP stream (NULL = default stream) and returns 0 or a negative hipError_t; no call
 * allocates, synchronises or throws.  Calls on different batches are re-entrant; calls on the
 * same batch must be stream-ordered (like the reference, one model instance is not thread-safe).
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define B747_ABI_VERSION 10  /* 1: round 1; 2: + b747_set_specialization, b747_policy_*, b747_ppo_rollout;
                                * 3: + b747_env_batch.rec_params, b747_struct_size; 4: + b747_env_batch.ep_stats;
                                * 5: + b747_env_step_seq; 6: b747_model_batch.aero_err is double (the DLL's
                                * `double aero_err[5]`, core/model.py:164), the policy buffer gains the layer-1
                                * matrix-core fragments (b747_policy_num_params); 7: b747_env_batch.aero_err and
                                * .ref are double (the reference's float64 draws and references reach the DLL
                                * unrounded: core/controller.py:153-193); 8: B747_VARIANT_MIXED, and b747_ppo_rollout /
                                * the two-wave kernels run sample_time > dt (n_sub DLL steps per env step); 9: + b747_env_kernel,
                                * and ep_return / ep_final_return accumulate as SB3's VecMonitor (float32); 10:
                                * b747_ppo_rollout advances *step_base by T on the device, b747_env_batch.ep_return is float
                                * (it holds float32 values; 8 B less per env step) */

#define B747_NX 18   /* continuous states, SURVEY A.1 (dll.data@0x2b380) */
#define B747_NDISC 9 /* compact discrete state, see b747_model_batch.disc */
#define B747_NSIG 31 /* exported signals, see B747_SIG_* */
#define B747_NAERO 5 /* aero_err components (CXa, CYa, mz, dCm/ddeltaz, K_alpha) */

/* Arithmetic variant of the dynamics (all parity-tested against the oracle):
 *   FAST     fp64: sin/cos(theta) from the quaternion, sin/cos(alpha) from (u, v)/V, pow via exp/log,
 *            reciprocals instead of divisions -- each a few ulp from the DLL's operations;
 *   FAITHFUL fp64: the DLL's operations in the DLL's order (bit-exact vs the CPU oracle on one libm);
 *   MIXED    FAST, except that the two-wave env kernels of the training configuration compute the flight
 *            aerodynamics (ISA atmosphere, speed, alpha, the table lookups, forces, pitching moment) in fp32;
 *            the state, the attitude, the RK4 integration and the whole control side stay fp64.  Per step from
 *            the oracle's state: within 2e-6 |oracle| + 1e-7 + 1e-7 x the batch's largest |value| (absolute ~1e-7
 *            at full scale for the normalised observations and the reward, relative above it); free-running over
 *            a 20 s episode: median deviation 6e-8 of scale, 99th percentile 1.8e-5 (tests/test_gpu_mixed.py,
 *            DESIGN.md 5).  Every other kernel runs FAST.  (round 4, ABI v8) */
#define B747_VARIANT_FAST 0
#define B747_VARIANT_FAITHFUL 1
#define B747_VARIANT_MIXED 2

/* flags[i] bits = the DLL's use_* parameters (each tested as `>= 1.0`, dll@0x1ee9 etc.) */
#define B747_F_PID_SS 1u /* use_PID_SS: SS (pitch) PID drives U_com          */
#define B747_F_PID_CS 2u /* use_PID_CS: CS (altitude) PID drives the pitch reference */
#define B747_F_RP 4u     /* use_RP: actuator model (delay, lag, rate limit, saturation) */
#define B747_F_RL 8u     /* use_RL: PID output with +-10 deg dead zone      */

/* Exported-signal order of b747_model_batch.sig ([B747_NSIG][N] doubles). */
enum {
    B747_SIG_SIM_TIME = 0, B747_SIG_DVARTHETA, B747_SIG_U_COM, B747_SIG_ALPHA, B747_SIG_V,
    B747_SIG_STATE /* 6 entries: x, y, Vx, Vy, vartheta, wz */,
    B747_SIG_MACH = B747_SIG_STATE + 6, B747_SIG_DVARTHETA_DT, B747_SIG_DVARTHETA_DT_DT,
    B747_SIG_DVARTHETA_INT, B747_SIG_AE, B747_SIG_ITAE, B747_SIG_IAE, B747_SIG_ISE, B747_SIG_ITSE,
    B747_SIG_SE, B747_SIG_TAE, B747_SIG_TSE, B747_SIG_K_ALPHA, B747_SIG_MZ, B747_SIG_DCM_DDELTAZ,
    B747_SIG_CXA, B747_SIG_CYA, B747_SIG_DELTAZ_RP, B747_SIG_U_COM_PID, B747_SIG_VARTHETA_ZH
};

/* Batch-wide model parameters (the DLL's scalar model parameters, dll.data@0x24000...). */
typedef struct b747_consts {
    double Iz, P, S, c_, g, m0;
    double PID_CS[4]; /* [Kp, Ki, Kd, N] of the CS (altitude-hold) loop */
    double PID_SS[4]; /* [Kp, Ki, Kd, N] of the SS (pitch-stabilisation) loop */
} b747_consts;

/* One batch of N independent models = N copies of the reference DLL's static data.
 * State (read+write):
 *   X     [18][N]  float (x_f64 == 0) or double (x_f64 == 1): continuous states, SURVEY A.1
 *   disc  [9][N]   double: x_dss, y_dss (held), rate-limiter PrevY, Derivative inputs at the
 *                  last major step (dvartheta, dvartheta_dt), U_com history (slot j&3 = step j)
 *   k     [N]      uint32: major step counter (time = k * 0.01 s)
 *   mem   [N]      uint8 : anti-windup Memory blocks (bit0 SS loop, bit1 CS loop)
 * Parameters (read):
 *   deltaz, vartheta, h_zh [N] double; flags [N] uint8 (B747_F_*); aero_err [5][N] double (the DLL's
 *   parameter precision: core/model.py:164 binds `(real_T*5).in_dll(dll, "aero_err")`, real_T = c_double);
 *   state0 [6][N] double (read by initialize only)
 * Read-out (write, nullable): sig [31][N] double = every exported signal after the call, i.e.
 *   what core/model.py's properties return after Model.step()/initialize(). */
typedef struct b747_model_batch {
    int64_t n;
    int32_t x_f64;
    int32_t variant;   /* B747_VARIANT_FAST (0, default), B747_VARIANT_FAITHFUL (MIXED runs FAST here) */
    void *X;
    double *disc;
    uint32_t *k;
    uint8_t *mem;
    const double *deltaz;
    const double *vartheta;
    const double *h_zh;
    const uint8_t *flags;
    const double *aero_err;
    const double *state0;
    double *sig;
} b747_model_batch;

/* ABI version (B747_ABI_VERSION) -- lets a ctypes binding check it loaded the right library. */
int32_t b747_abi_version(void);
/* sizeof of the ABI structs (B747_STRUCT_*), or -1: a binding checks its struct mirrors against these. */
enum { B747_STRUCT_CONSTS = 0, B747_STRUCT_MODEL_BATCH = 1, B747_STRUCT_ENV_CONFIG = 2, B747_STRUCT_ENV_BATCH = 3 };
int64_t b747_struct_size(int32_t which);
/* Fill *c with the DLL's defaults (Iz = 6.73e7, P = 275000, PID gains, ...). */
int32_t b747_consts_default(b747_consts *c);

/* model_simple_initialize (dll@0x12a0) for every env with mask[i] != 0 (mask NULL = all).
 * Replaces core/model.py:238-241.  Signals (if sig != NULL) are zeroed, as in the DLL. */
int32_t b747_model_initialize(const b747_model_batch *b, const uint8_t *mask, void *stream);

/* n_steps consecutive model_simple_step calls (dll@0x16d0) on every env: one ode4 step of
 * h = 0.01 s each.  Replaces core/model.py:247-250 (x N envs, x n_steps).  n_steps = 1 with the DLL's
 * default constants (FAST) runs each env over three waves (k_model_step_split); otherwise one wave per env
 * with the state in registers across the n_steps (k_model_step): the same operations, agreeing to a few ulp
 * (FMA contraction); b747_set_specialization(0) keeps every call on the one-wave kernel. */
int32_t b747_model_step(const b747_model_batch *b, const b747_consts *c, int32_t n_steps,
                        void *stream);

/* ------------------------------------------------------------------ env level ---------
 * ControllerEnv (env/ctrl_env.py) + Controller (core/controller.py) for N envs.
 * Enum values equal the reference's Python Enum values. */
enum { B747_OBS_PID_LIKE = 0, B747_OBS_SPEED_MODE = 1, B747_OBS_PID_AERO = 2,
       B747_OBS_PID_SPEED_AERO = 3, B747_OBS_MODEL_STATE = 4 };
enum { B747_REW_CLASSIC = 0, B747_REW_PID_LIKE = 1, B747_REW_QUALITY = 2, B747_REW_MINIMAL = 3,
       B747_REW_TF_REFERENCE = 4 };
enum { B747_CTRL_FULL_AUTO = 0, B747_CTRL_AUTO = 1, B747_CTRL_SEMI_MANUAL = 2, B747_CTRL_MANUAL = 3 };
enum { B747_MODE_NONE = -1, B747_MODE_DIRECT = 0, B747_MODE_ADD_PROC = 1, B747_MODE_ANG_VEL = 2,
       B747_MODE_ADD_DIRECT = 3 };
enum { B747_RESET_NONE = -1, B747_RESET_CONST = 0, B747_RESET_OSCILLATING = 1, B747_RESET_HYBRID = 2 };
enum { B747_DIST_NONE = -1, B747_DIST_AERO = 0 };
enum { B747_REF_CONST = 0, B747_REF_OSC = 1 };

/* Batch-wide env configuration = the ControllerEnv(...) / Controller(...) constructor args. */
typedef struct b747_env_config {
    int32_t obs_type, reward_type, ctrl_type, ctrl_mode, reset_ref_mode, disturbance_mode;
    int32_t norm_obs, norm_act, use_limiter, auto_reset;
    int32_t n_sub;        /* DLL steps per env step: round(sample_time / 0.01) */
    int32_t aero_fixed;   /* AERO disturbance with the fixed vector aero_err_fixed */
    double sample_time, tk, action_max, vartheta_max;
    double rew[8];        /* reward constants (b747_env_config_default documents each type) */
    double aero_err_fixed[5];
    uint64_t seed;        /* Philox key of the random resets */
} b747_env_config;

/* N environments.  Model state as in b747_model_batch, plus the controller's per-env state.
 * obs / terminal_obs are row-major [N][obs_dim] (what a policy consumes). */
typedef struct b747_env_batch {
    int64_t n;
    int64_t env_offset;   /* global id of env 0 (GPU shard offset); RNG stream = seed x global id */
    int32_t x_f64, obs_dim;
    int32_t variant;      /* B747_VARIANT_* */
    int32_t reserved;
    void *X; double *disc; uint32_t *k; uint8_t *mem;
    double *deltaz;       /* DLL parameter deltaz: read/written by a step only in ANG_VEL mode
                           * (the one mode that integrates it; the others derive it from the action) */
    /* The next four are controller-internal slots.  A step reads/writes each only where the
     * configuration uses it (keeps the per-step HBM traffic to what the path needs):
     *   vartheta  written by resets only: a step recomputes it (CS PID on: the 0 that
     *             Model.initialize wrote; off: the pitch reference at t)
     *   h_zh      read every step, written where the CS PID is on (it persists); ref[7] is read
 *             only when the configuration can turn the CS PID on
     *   upid      only in ADD_PROC / ADD_DIRECT ctrl modes
     *   tp        only with the TF_REFERENCE reward                                        */
    double *vartheta;     /* DLL parameter vartheta */
    double *h_zh;         /* DLL parameter h_zh */
    double *upid;         /* U_com_PID read-out of the last step (Model.deltaz_ref) */
    double *tp;           /* TF_REFERENCE reward state */
    uint8_t *flags;       /* B747_F_* per env (HYBRID resets switch the CS PID per env) */
    double *aero_err;     /* [5][N]: the DLL's double aero_err[5] (core/model.py:164), which Controller.reset
                           * fills with float64 normal draws (core/controller.py:181-193) */
    double *ref;          /* [8][N], float64 as the reference's Python floats (core/controller.py:153-177):
                           * [0] const pitch, [1..3] A1..A3, [4..6] f1..f3 (Hz), [7] altitude;
                           * a step reads [0], [7], and [1..6] when the reset mode can give
                           * oscillating references (OSCILLATING or NONE) */
    uint8_t *ref_kind;    /* B747_REF_*; read by a step only when the reset mode can give oscillating
                           * references (OSCILLATING or NONE): CONST / HYBRID treat every ref as constant */
    double *state0;       /* [6][N] initial state used when reset_ref_mode == NONE */
    uint32_t *episode;    /* resets done so far (Philox counter) */
    float *ep_return; int32_t *ep_len;               /* running episode statistics: the return accumulated as
                                                      * SB3's VecMonitor does (float32(return + float64 reward)
                                                      * per step; float since ABI 10); a step derives ep_len from k
                                                      * (ceil(k / n_sub)), resets write it */
    double *ep_final_return; int32_t *ep_final_len;  /* written where done (VecMonitor's episode "r", "l") */
    const float *action;  /* [N] action (action dim 1) */
    float *obs;           /* [N][obs_dim] */
    float *reward;        /* [N] */
    uint8_t *done;        /* [N] */
    float *terminal_obs;  /* [N][obs_dim], nullable: last obs of an episode that ended */
    double *sig;          /* [n_sub][31][N], nullable: every exported signal (B747_SIG_* rows)
                           * after each DLL step of the env step -- what Controller._post_step
                           * records into its Storage (core/controller.py:209-228) and what
                           * core/model.py's properties read; slot q = DLL step q of the env
                           * step (slots before an unaligned first step are left untouched);
                           * for an env that finished, the values before its auto-reset */
    double *rec_params;   /* [3][N], nullable, written only with sig: the DLL parameters vartheta, h_zh
                           * and deltaz in effect during the last env step (before an auto-reset) --
                           * the Controller values _post_step records beside the signals
                           * (vartheta_ref when the CS PID is off, hzh; core/controller.py:209-228) */
    double *ep_stats;     /* [3][N], nullable: per-env episode accumulators, added to where an episode ends
                           * (a step's done): [0] += 1, [1] += its return, [2] += its length -- what SB3's
                           * VecMonitor logs (neural/agent.py:63-82 wraps the env in it), kept on the device
                           * so a caller can reduce them across envs and ranks every M steps
                           * instead of copying every step's info to the host */
} b747_env_batch;

/* Defaults of ControllerEnv/Controller for the given obs/reward types (reward constants of
 * env/ctrl_env.py:109-192 with reward_config = {}; main.py settings for the rest). */
int32_t b747_env_config_default(b747_env_config *cfg, int32_t obs_type, int32_t reward_type);
int32_t b747_env_obs_dim(int32_t obs_type);

/* ControllerEnv.reset (env/ctrl_env.py:273-278) for envs with mask[i] != 0 (NULL = all):
 * random ICs / reference / aero errors per the config, Model.initialize, obs <- zeros. */
int32_t b747_env_reset(const b747_env_batch *b, const b747_env_config *cfg, const b747_consts *c,
                       const uint8_t *mask, void *stream);

/* ControllerEnv.step (env/ctrl_env.py:260-270) for every env, fused in one launch: action
 * scaling, command injection, action mode, round(sample_time/dt) DLL steps, obs, reward,
 * done, and (auto_reset) the SB3 VecEnv auto-reset with terminal_obs. */
int32_t b747_env_step(const b747_env_batch *b, const b747_env_config *cfg, const b747_consts *c,
                      void *stream);

/* n_env_steps consecutive env steps in ONE launch with actions[t][N] given up front (open-loop
 * or pre-sampled actions; obs/reward/done of every step are written to obs_seq[t][N][obs_dim],
 * reward_seq[t][N], done_seq[t][N], each nullable).  State stays in registers between steps. */
int32_t b747_env_rollout(const b747_env_batch *b, const b747_env_config *cfg, const b747_consts *c,
                         const float *actions, int32_t n_env_steps, float *obs_seq, float *reward_seq,
                         uint8_t *done_seq, void *stream);

/* n_env_steps consecutive ControllerEnv.step calls with actions[t][N] given up front, as n_env_steps
 * launches of the per-step kernel (the b747_env_step launch, one per step: the same kernel and the
 * same results as a host loop of b747_env_step with b->action = actions + t*N); obs/reward/done and
 * the episode buffers hold the last step's.  Stream-ordered and graph-capturable; what it saves
 * over such a loop, or over a replayed graph of it, is host-side latency only. */
int32_t b747_env_step_seq(const b747_env_batch *b, const b747_env_config *cfg, const b747_consts *c,
                          const float *actions, int32_t n_env_steps, void *stream);

/* Measurement helper (synchronous; not for graph capture): runs n_env_steps b747_env_step
 * launches on `stream` (actions[t][N]) with a HIP event pair recorded directly around each
 * launch (events created with hipEventDisableSystemFence so they add no cache flush), and
 * writes each launch's duration in milliseconds to ms_out[t] (host memory). */
int32_t b747_env_time_steps(const b747_env_batch *b, const b747_env_config *cfg, const b747_consts *c,
                            const float *actions, int32_t n_env_steps, float *ms_out, void *stream);

/* Kernel specialisation switch (diagnostic; process-wide, not thread-safe).  With on != 0 (the
 * default) an env step whose configuration has the branch-selecting fields of the reference's
 * training setup (PID_LIKE obs, CLASSIC reward, MANUAL/DIRECT control, CONST resets, drawn AERO
 * errors, normalised obs/action, no limiter, auto-reset) and the DLL's default constants runs a
 * kernel compiled for exactly that configuration; with on == 1 a single step of it (sample_time = dt)
 * runs each env over three waves (flight / ahead / control), on == 2 keeps one wave per env; on == 0
 * forces the generic kernel (tests compare them), and b747_model_step's one-step calls the one-wave kernel.
 * Returns the previous setting.  No reference counterpart (the reference has no kernels). */
int32_t b747_set_specialization(int32_t on);

/* Which kernel b747_env_rollout(b, cfg, c, ..., n_env_steps) launches for this batch and configuration (b747_env_step
 * is n_env_steps = 1): B747_KERNEL_* below.  Lets a caller (and the tests) confirm that a configuration runs the
 * two-wave kernels of the bench.  No reference counterpart.  Returns < 0 on a bad argument. */
#define B747_KERNEL_GENERIC 0        /* k_env_steps, run-time constants */
#define B747_KERNEL_DEFC 1           /* k_env_steps, the DLL's default constants as literals */
#define B747_KERNEL_RECORDING 2      /* k_env_steps with per-DLL-step signal recording (b747_env_batch.sig) */
#define B747_KERNEL_SPEC_ONE_WAVE 3  /* k_env_steps specialised on the training configuration, one wave per env */
#define B747_KERNEL_STEP_SPLIT 4     /* k_env_step_split: the per-step two-wave kernel (the bench headline) */
#define B747_KERNEL_ROLLOUT_SPLIT 5  /* k_rollout_split<false>: K env steps / n_sub DLL steps, two waves per env */
int32_t b747_env_kernel(const b747_env_batch *b, const b747_env_config *cfg, const b747_consts *c, int32_t n_env_steps);

/* ---- on-GPU PPO rollout (BASELINE config 5) ----
 * One step of stable-baselines3's collect_rollouts for every env (neural/agent.py:167-171 ->
 * SB3 1.4 PPO.collect_rollouts with the default MlpPolicy): policy forward through separate
 * pi / vf extractors [64, 64] tanh, Gaussian sample with a state-independent log_std, log-prob,
 * value, and the clipped action handed to the env.  params = the policy's parameters flattened
 * in this order (torch Linear weights are [out][in] row-major): pi_net.0.{weight,bias},
 * pi_net.2.{weight,bias}, vf_net.0.{weight,bias}, vf_net.2.{weight,bias}, action_net.{weight,bias},
 * value_net.{weight,bias}, log_std -- fp32, device memory (b747_rl_ctrl_amd/ppo.py flat_params),
 * followed by 2 x 4096 floats that b747_policy_pack fills with the 64x64 layers (scaled by -4/ln 2)
 * repacked for the matrix cores as f16 hi/lo pairs, 2*64*(obs_dim+1) + 4*64 + 3 floats of
 * derived parameters with tanh's scale and affine part folded in, and (from a 16-byte boundary) 1024
 * floats of layer-1 matrix-core fragments (obs_dim <= 4: the first layer of both heads as one
 * v_mfma_f32_32x32x16_f16 per 32-unit tile, its f16 hi/lo split and bias folded into K) -- call it after
 * every parameter update; b747_policy_num_params counts all four parts.  Outputs agree with the f32 torch policy within 2e-5 (f16 hi/lo split products, tests/test_gpu_ppo.py). */
int32_t b747_policy_num_params(int32_t obs_dim);
/* T rollout steps (policy forward + sample + clip + env step, as b747_policy_act followed by
 * b747_env_step with the same Philox noise) for every env in ONE launch -- each env on two waves, the policy
 * head on one beside the other's RK4 stages, the env state and observation kept in registers across steps --
 * then ONE batched launch of the value head over the T*N rows of obs_buf into val_buf; both on `stream`
 * (SB3 collect_rollouts, neural/agent.py:167-171 -> PPO.collect_rollouts).  Row t*N + i of obs_buf[T][N][3], act_buf, logp_buf, val_buf, rew_buf,
 * done_buf; the env's obs / reward / done hold the last step's afterwards.  Covers the reference's
 * training configuration only (default constants; PID_LIKE, CLASSIC, MANUAL/DIRECT, CONST resets,
 * AERO errors, normalised obs/action, no limiter, auto-reset; fp64 state; FAST; N % 64 == 0) and
 * returns -hipErrorInvalidValue for anything else.  step_base (device, nullable = 0): the Philox counter base of
 * step 0, read by the rollout and advanced by T on the device after it (ABI 10), so that consecutive calls -- or
 * replays of one captured graph -- draw fresh noise with no host or extra kernel in between. */
int32_t b747_ppo_rollout(const b747_env_batch *b, const b747_env_config *cfg, const b747_consts *c, const float *params,
                         uint64_t seed, uint64_t *step_base, int32_t T, float *obs_buf, float *act_buf,
                         float *logp_buf, float *val_buf, float *rew_buf, uint8_t *done_buf, float act_lo, float act_hi,
                         void *stream);
int32_t b747_policy_pack(float *params, int32_t obs_dim, void *stream);
/* noise [N] (nullable): standard-normal draws; NULL = Philox4x32-10 keyed by seed with counter
 * (env_offset + i, *step_base + step); step_base (device, nullable = 0) lets a captured rollout
 * graph draw fresh noise on every replay.  obs_out (nullable) receives a copy of obs. */
int32_t b747_policy_act(const float *params, int32_t obs_dim, int64_t n, const float *obs, const float *noise,
                        uint64_t seed, const uint64_t *step_base, uint32_t step, int64_t env_offset,
                        float *obs_out, float *act_out,
                        float *logp_out, float *value_out, float *env_action, float act_lo, float act_hi,
                        void *stream);

/* Human-readable text of the last error returned on this thread. */
const char *b747_last_error(void);

#ifdef __cplusplus
}
#endif
