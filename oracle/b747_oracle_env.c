/* b747_oracle_env.c -- batched ControllerEnv restatement over the CPU oracle.
 *
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY (the product path never links or calls it).
 *
 * Each env is one DLL-faithful model instance (b747o_model, oracle/b747_oracle.c) driven by a C
 * restatement of the reference's Python loop around the DLL:
 *   core/model.py:238-250        Model.initialize (deltaz = vartheta_zh = 0 after the DLL init) / step
 *   core/controller.py:134-201   Controller.reset (draws supplied by the caller, see b747oe_reset)
 *   core/controller.py:231-264   Controller.step: command injection, action modes, sub-stepping
 *   core/controller.py:268-270   Controller.vartheta_ref;  :336 quality()
 *   env/ctrl_env.py:109-192      rewards;  :200-247 observations;  :255-270 done / step
 * operation for operation as oracle/ref_env.py states them in Python (IEEE double, libm exp/sin,
 * no FMA contraction: -ffp-contract=off), so the two agree bit for bit (tests/test_oracle_env.py).
 * It lets the GPU tests check EVERY env of a 65,536-env batch (ref_env covers a subset), and with
 * OpenMP over envs it is the all-cores CPU baseline of the bench's env workload.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "b747_oracle.h"

#define EXPORT __attribute__((visibility("default")))

enum { F_PID_SS = 1, F_PID_CS = 2, F_RP = 4, F_RL = 8 };
enum { OBS_PID_LIKE = 0, OBS_SPEED_MODE = 1, OBS_PID_AERO = 2, OBS_PID_SPEED_AERO = 3, OBS_MODEL_STATE = 4 };
enum { REW_CLASSIC = 0, REW_PID_LIKE = 1, REW_QUALITY = 2, REW_MINIMAL = 3, REW_TF_REFERENCE = 4 };

static const double PI = 3.141592653589793;   /* math.pi */
/* Python's float ** float is libm pow(), which for an exponent of 2 is not always x*x (1 ulp on ~0.1 % of
 * arguments); called through a volatile pointer so that the compiler cannot fold pow(x, 2.0) into x*x */
static double (*volatile py_pow)(double, double) = pow;

/* Batch-wide ControllerEnv / Controller settings. */
typedef struct b747oe_cfg {
    int32_t obs_type, reward_type, ctrl_mode;   /* ctrl_mode -1 = None */
    int32_t norm_obs, norm_act, use_limiter;
    double sample_time, tk, action_max, vartheta_max;
    /* reward_config (env/ctrl_env.py:109-192): CLASSIC k1, k2, k3 (raw), kf, kITSE, k0;
     * PID_LIKE k; TF_REFERENCE overshoot_ref, tp_ref, k */
    double rew[6];
} b747oe_cfg;

/* One ControllerEnv. */
typedef struct b747oe_env {
    b747o_model m;
    int32_t ref_kind;       /* 0 constant pitch reference, 1 oscillating */
    double ref, osc[6], h1; /* Controller.vartheta_func / h_func */
    double tp;              /* TF_REFERENCE state (never reset, as in the reference) */
} b747oe_env;

EXPORT int64_t b747oe_sizeof_env(void) { return (int64_t)sizeof(b747oe_env); }

static void model_initialize(b747o_model *m)   /* core/model.py:238-244 */
{
    b747o_initialize(m);
    m->deltaz = 0.0;
    m->vartheta = 0.0;
}

/* A fresh ControllerEnv: the DLL's defaults with the control type's use_* flags
 * (core/controller.py:128-131) and initialize(). */
EXPORT void b747oe_create(int64_t n, b747oe_env *envs, const uint8_t *flags)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        b747oe_env *e = &envs[i];
        memset(e, 0, sizeof(*e));
        b747o_defaults(&e->m);
        e->m.use_PID_SS = (flags[i] & F_PID_SS) ? 1.0 : 0.0;
        e->m.use_PID_CS = (flags[i] & F_PID_CS) ? 1.0 : 0.0;
        e->m.use_RP = (flags[i] & F_RP) ? 1.0 : 0.0;
        e->h1 = 11000.0;
        model_initialize(&e->m);
    }
}

/* Controller.reset for envs with mask[i] != 0 (NULL = all), with the draws given in the device's
 * SoA layout: state0[6][n] f64, ref[8][n] f64 ([0] constant pitch, [1..6] A1..A3, f1..f3,
 * [7] altitude command), ref_kind[n], aero_err[5][n] f64 (NULL = keep the model's), fresh_flags[n]
 * (NULL = keep the model; else HYBRID: a fresh model with these use_* flags, core/controller.py:172-178). */
EXPORT void b747oe_reset(int64_t n, b747oe_env *envs, const uint8_t *mask, const double *state0, const double *ref,
                         const uint8_t *ref_kind, const double *aero_err, const uint8_t *fresh_flags)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        b747oe_env *e = &envs[i];
        if (fresh_flags) {
            const double tp = e->tp;
            b747oe_create(1, e, &fresh_flags[i]);
            e->tp = tp;
        }
        e->ref_kind = ref_kind[i];
        e->ref = ref[0 * n + i];
        for (int j = 0; j < 6; ++j) e->osc[j] = ref[(1 + j) * n + i];
        e->h1 = ref[7 * n + i];
        for (int j = 0; j < 6; ++j) e->m.state0[j] = state0[j * n + i];   /* Model.set_initial */
        if (aero_err)
            for (int j = 0; j < 5; ++j) e->m.aero_err[j] = aero_err[j * n + i];
        model_initialize(&e->m);
    }
}

static double vartheta_func(const b747oe_env *e, double t)   /* core/controller.py:153-177 */
{
    if (e->ref_kind == 1) {
        const double *o = e->osc;
        return o[0] * sin(2 * PI * o[3] * t) + o[1] * sin(2 * PI * o[4] * t) + o[2] * sin(2 * PI * o[5] * t);
    }
    return e->ref;
}

static double clip17(double x)   /* np.clip(x, -17 pi/180, 17 pi/180) */
{
    const double lim = 17 * PI / 180;
    return x < -lim ? -lim : (x > lim ? lim : x);
}

static double nan_to_num(double x)
{
    if (isnan(x)) return 0.0;
    if (isinf(x)) return x > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308;
    return x;
}

static int obs_dim_of(int t)
{
    return t == OBS_PID_LIKE ? 3 : t == OBS_SPEED_MODE ? 5 : t == OBS_PID_AERO ? 8 : t == OBS_PID_SPEED_AERO ? 10 : 7;
}

static double obs_max(int t, int j)   /* env/ctrl_env.py:200-214 */
{
    static const double pl[3] = {60 * PI, PI, PI};
    static const double sm[5] = {60 * PI, PI, PI, 500, 100};
    static const double psa[10] = {60 * PI, PI, PI, 500, 100, 0.5, 2, 0.6, 0.05, 1.0};
    static const double pa[8] = {60 * PI, PI, PI, 0.5, 2, 0.6, 0.05, 1.0};
    static const double ms[7] = {10 * PI / 180, 12000, 15000, 500, 100, PI, PI};
    switch (t) {
    case OBS_PID_LIKE: return pl[j];
    case OBS_SPEED_MODE: return sm[j];
    case OBS_PID_SPEED_AERO: return psa[j];
    case OBS_PID_AERO: return pa[j];
    default: return ms[j];
    }
}

static double vartheta_ref(const b747o_model *m)   /* core/controller.py:268-270 */
{
    return m->use_PID_CS ? m->vartheta_zh : m->vartheta;
}

static double reward(b747oe_env *e, const b747oe_cfg *c)   /* env/ctrl_env.py:109-192 */
{
    const b747o_model *m = &e->m;
    const double vref = vartheta_ref(m);
    const double vf = vref != 0.0 ? vref : c->vartheta_max;
    const double t = m->sim_time;
    switch (c->reward_type) {
    case REW_CLASSIC: {
        double k1 = c->rew[0], k2 = c->rew[1], k3 = c->rew[2];
        const double kf = c->rew[3], kITSE = c->rew[4], k0 = c->rew[5];
        const double kt = -log(0.8) / 10, ko = -log(0.75) / 0.15;   /* tools/general.py:32-33 */
        const double s = k1 + k2 + k3;
        k1 = k1 / s; k2 = k2 / s; k3 = k3 / s;
        const double r1 = 0.50 * exp(-k0 * (k1 * fabs(m->dvartheta) + k2 * 1 * fabs(m->dvartheta_dt) +
                                            k3 * fabs(m->dvartheta_dt_dt)) / fabs(vf));
        const double r2 = vref * m->dvartheta < 0 ? 0.20 * exp(-ko * fabs(m->dvartheta / vf)) : 0.20;
        const double r3 = fabs(m->dvartheta / vf) > 0.05 ? 0.20 * exp(-kt * t) : 0.20;
        const double r4 = 0.1 * exp(-kITSE * m->ITSE / py_pow(vf, 2.0));   /* vf**2 */
        const double rf = c->ctrl_mode == 0
                              ? -kf * fabs(m->dvartheta / (2 * vf)) * (fabs(m->deltaz - m->U_com_PID)) / (34 * PI / 180)
                              : 0.0;
        return r1 + r2 + r3 + r4 + rf;
    }
    case REW_PID_LIKE:
        return exp(-c->rew[0] * fabs(m->U_com - m->U_com_PID) / (34 * PI / 180));
    case REW_QUALITY:
    case REW_MINIMAL:   /* Controller.quality(), core/controller.py:336 */
        return exp(-60 * 0.1 * m->ITSE / (c->tk * py_pow(vref, 2.0)));   /* vartheta_ref**2 */
    default: {           /* TF_REFERENCE */
        const double overshoot = fabs(m->dvartheta / vf) * 100;
        if (overshoot > 5) e->tp = t;
        return exp(-c->rew[2] * fabs(overshoot - c->rew[0]) * fabs(c->rew[1] - e->tp));
    }
    }
}

static void observation(const b747oe_env *e, const b747oe_cfg *c, float *out)   /* env/ctrl_env.py:217-247 */
{
    const b747o_model *m = &e->m;
    double s[6], o[10];
    for (int j = 0; j < 6; ++j) s[j] = nan_to_num(m->state[j]);   /* state getter, core/model.py:200 */
    const double base[3] = {m->dvartheta_int, m->dvartheta, m->dvartheta_dt};
    const double aero[5] = {m->CXa, m->CYa, m->mz, m->dCm_ddeltaz, m->K_alpha};
    int d = 0;
    switch (c->obs_type) {
    case OBS_MODEL_STATE:
        o[d++] = vartheta_ref(m);
        for (int j = 0; j < 6; ++j) o[d++] = s[j];
        break;
    default:
        for (int j = 0; j < 3; ++j) o[d++] = base[j];
        if (c->obs_type == OBS_SPEED_MODE || c->obs_type == OBS_PID_SPEED_AERO) { o[d++] = s[2]; o[d++] = s[3]; }
        if (c->obs_type == OBS_PID_AERO || c->obs_type == OBS_PID_SPEED_AERO)
            for (int j = 0; j < 5; ++j) o[d++] = aero[j];
    }
    for (int j = 0; j < d; ++j) out[j] = (float)(c->norm_obs ? o[j] / obs_max(c->obs_type, j) : o[j]);
}

/* ControllerEnv.step (env/ctrl_env.py:260-270) for every env: actions[n] as the policy produced
 * them (float32); obs[n][obs_dim] f32, reward[n] (float64, as the reference returns it), done[n].
 * No auto-reset: the caller resets finished envs with b747oe_reset (draws from the device). */
EXPORT void b747oe_step(int64_t n, b747oe_env *envs, const b747oe_cfg *c, const float *actions, float *obs,
                        double *rew, uint8_t *done)
{
    const int od = obs_dim_of(c->obs_type);
    const double dt = 0.01;
    const long long nsub = llrint(c->sample_time / dt);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        b747oe_env *e = &envs[i];
        b747o_model *m = &e->m;
        /* action *= action_max in place on a float32 array (the product is formed in float64) */
        const float a32 = c->norm_act ? (float)((double)actions[i] * c->action_max) : actions[i];
        const double a = (double)a32;
        if (!m->use_PID_CS) m->vartheta = vartheta_func(e, m->sim_time);
        else m->h_zh = e->h1;
        if (!m->use_PID_SS) {
            switch (c->ctrl_mode) {
            case 1: m->deltaz = clip17((1 + a) * m->U_com_PID); break;
            case 3: m->deltaz = clip17(a + m->U_com_PID); break;
            case 2: m->deltaz = clip17(m->deltaz + a * c->sample_time); break;
            default: m->deltaz = a; break;                 /* DIRECT_CONTROL or None */
            }
        }
        b747o_step(m);
        while (llrint(m->sim_time / dt) % nsub != 0) b747o_step(m);
        observation(e, c, obs + i * od);
        rew[i] = reward(e, c);
        int d = m->sim_time >= c->tk;
        if (c->use_limiter)
            d = d || fabs(nan_to_num(m->state[4])) > 5 * PI / 180 + c->vartheta_max || m->deltaz > c->action_max;
        done[i] = (uint8_t)d;
    }
}

/* The compact state of env i (to compare with the HIP path's HBM state). */
EXPORT void b747oe_export(int64_t n, const b747oe_env *envs, double *X, uint32_t *k)
{
    for (int64_t i = 0; i < n; ++i) {
        b747o_compact cs;
        b747o_export_compact(&envs[i].m, &cs);
        for (int j = 0; j < B747O_NX; ++j) X[j * n + i] = cs.X[j];
        k[i] = cs.k;
    }
}

/* The whole compact model state of every env in the HIP path's SoA layout (include/b747.h: X[18][n],
 * disc[9][n], k[n], mem[n]): the shadow scheme of the GPU tests loads it into a device batch so that a
 * long episode is checked step by step from the oracle's own state (tests/test_gpu_fullsize.py). */
EXPORT void b747oe_export_full(int64_t n, const b747oe_env *envs, double *X, double *disc, uint32_t *k, uint8_t *mem)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        b747o_compact cs;
        b747o_export_compact(&envs[i].m, &cs);
        for (int j = 0; j < B747O_NX; ++j) X[j * n + i] = cs.X[j];
        disc[0 * n + i] = cs.x_dss; disc[1 * n + i] = cs.y_dss; disc[2 * n + i] = cs.rl_prevY;
        disc[3 * n + i] = cs.e_prev; disc[4 * n + i] = cs.ed_prev;
        for (int j = 0; j < 4; ++j) disc[(5 + j) * n + i] = cs.u_hist[j];
        k[i] = cs.k;
        mem[i] = (uint8_t)cs.mem;
    }
}
