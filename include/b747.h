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

#define B747_ABI_VERSION 1

#define B747_NX 18   /* continuous states, SURVEY A.1 (dll.data@0x2b380) */
#define B747_NDISC 9 /* compact discrete state, see b747_model_batch.disc */
#define B747_NSIG 31 /* exported signals, see B747_SIG_* */
#define B747_NAERO 5 /* aero_err components (CXa, CYa, mz, dCm/ddeltaz, K_alpha) */

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
 *   deltaz, vartheta, h_zh [N] double; flags [N] uint8 (B747_F_*); aero_err [5][N] float;
 *   state0 [6][N] double (read by initialize only)
 * Read-out (write, nullable): sig [31][N] double = every exported signal after the call, i.e.
 *   what core/model.py's properties return after Model.step()/initialize(). */
typedef struct b747_model_batch {
    int64_t n;
    int32_t x_f64;
    int32_t reserved;
    void *X;
    double *disc;
    uint32_t *k;
    uint8_t *mem;
    const double *deltaz;
    const double *vartheta;
    const double *h_zh;
    const uint8_t *flags;
    const float *aero_err;
    const double *state0;
    double *sig;
} b747_model_batch;

/* ABI version (B747_ABI_VERSION) -- lets a ctypes binding check it loaded the right library. */
int32_t b747_abi_version(void);
/* Fill *c with the DLL's defaults (Iz = 6.73e7, P = 275000, PID gains, ...). */
int32_t b747_consts_default(b747_consts *c);

/* model_simple_initialize (dll@0x12a0) for every env with mask[i] != 0 (mask NULL = all).
 * Replaces core/model.py:238-241.  Signals (if sig != NULL) are zeroed, as in the DLL. */
int32_t b747_model_initialize(const b747_model_batch *b, const uint8_t *mask, void *stream);

/* n_steps consecutive model_simple_step calls (dll@0x16d0) on every env: one ode4 step of
 * h = 0.01 s each.  Replaces core/model.py:247-250 (x N envs, x n_steps). */
int32_t b747_model_step(const b747_model_batch *b, const b747_consts *c, int32_t n_steps,
                        void *stream);

/* Human-readable text of the last error returned on this thread. */
const char *b747_last_error(void);

#ifdef __cplusplus
}
#endif
