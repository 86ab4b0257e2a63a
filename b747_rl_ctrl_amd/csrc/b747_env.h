/* b747_env.h -- per-lane ControllerEnv / Controller semantics on top of b747_dynamics.h.
 *
 * Re-derives, for one environment held in registers, the Python hot loop that the reference
 * runs around the DLL for every env step:
 *   env/ctrl_env.py:260-270   ControllerEnv.step: action scaling, obs, reward, done
 *   core/controller.py:231-264 Controller.step: command injection, action modes, sub-stepping
 *   core/controller.py:134-201 Controller.reset: random ICs / references / aero errors
 *   env/ctrl_env.py:109-247   reward functions, observation layouts and normalisation
 * Random resets draw from a counter-based Philox4x32-10 stream keyed by (seed, env id) with the
 * per-env episode number as counter, so every env's sequence is reproducible and independent
 * of the batch size and of how envs are sharded over GPUs.  Distributions match the reference
 * (Python `random` / numpy streams are not reproduced bit for bit).
 */
#pragma once

#include "../../include/b747.h"
#include "b747_dynamics.h"

namespace b747 {

/* ---- enums: values equal to the reference's Python Enum values ---- */
enum ObsType { OBS_PID_LIKE = 0, OBS_SPEED_MODE = 1, OBS_PID_AERO = 2, OBS_PID_SPEED_AERO = 3, OBS_MODEL_STATE = 4 };
enum RewType { REW_CLASSIC = 0, REW_PID_LIKE = 1, REW_QUALITY = 2, REW_MINIMAL = 3, REW_TF_REFERENCE = 4 };
enum CtrlType { CT_FULL_AUTO = 0, CT_AUTO = 1, CT_SEMI_MANUAL = 2, CT_MANUAL = 3 };
enum CtrlMode { CM_NONE = -1, CM_DIRECT = 0, CM_ADD_PROC = 1, CM_ANG_VEL = 2, CM_ADD_DIRECT = 3 };
enum ResetMode { RM_NONE = -1, RM_CONST = 0, RM_OSCILLATING = 1, RM_HYBRID = 2 };
enum RefKind { REF_CONST = 0, REF_OSC = 1 };

constexpr double PI = 3.141592653589793;  /* math.pi */
constexpr int OBS_MAX_DIM = 10;

/* np.nan_to_num (core/model.py:167-168): NaN -> 0, +-inf -> +-DBL_MAX */
B747_HD double nan_to_num(double x)
{
    if (isnan(x)) return 0.0;
    if (isinf(x)) return x > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308;
    return x;
}

B747_HD int obs_dim_of(int obs_type)
{
    switch (obs_type) {
    case OBS_PID_LIKE: return 3;
    case OBS_SPEED_MODE: return 5;
    case OBS_PID_AERO: return 8;
    case OBS_PID_SPEED_AERO: return 10;
    default: return 7;  /* OBS_MODEL_STATE */
    }
}

/* obs_max of env/ctrl_env.py:200-214 */
B747_HD double obs_max(int obs_type, int j)
{
    switch (obs_type) {
    case OBS_PID_LIKE: { const double m[3] = {60 * PI, PI, PI}; return m[j]; }
    case OBS_SPEED_MODE: { const double m[5] = {60 * PI, PI, PI, 500, 100}; return m[j]; }
    case OBS_PID_SPEED_AERO: { const double m[10] = {60 * PI, PI, PI, 500, 100, 0.5, 2, 0.6, 0.05, 1.0}; return m[j]; }
    case OBS_PID_AERO: { const double m[8] = {60 * PI, PI, PI, 0.5, 2, 0.6, 0.05, 1.0}; return m[j]; }
    default: { const double m[7] = {10 * PI / 180, 12000, 15000, 500, 100, PI, PI}; return m[j]; }
    }
}

/* Batch-wide env configuration = include/b747.h b747_env_config (kernels read it straight from
 * the kernel-argument segment: scalar loads, no per-lane copy). */
typedef b747_env_config EnvCfg;

/* ------------------------------------------------------------- Philox4x32-10 ---- */
struct Rng {
    uint32_t k0, k1, c0, c1, c2, c3;   /* key = seed; counter = (env id, episode, block) */
    uint32_t buf[4];
    int left;

    B747_HD void init(uint64_t seed, uint64_t env_id, uint32_t episode)
    {
        k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32);
        c0 = (uint32_t)env_id; c1 = (uint32_t)(env_id >> 32); c2 = episode; c3 = 0u;
        left = 0;
    }
    B747_HD void refill()
    {
        uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = c3, a = k0, b = k1;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
            uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ a, y1 = (uint32_t)p1;
            uint32_t y2 = (uint32_t)(p0 >> 32) ^ x3 ^ b, y3 = (uint32_t)p0;
            x0 = y0; x1 = y1; x2 = y2; x3 = y3;
            a += 0x9E3779B9u; b += 0xBB67AE85u;
        }
        buf[0] = x0; buf[1] = x1; buf[2] = x2; buf[3] = x3;
        left = 4;
        c3++;
    }
    B747_HD uint32_t u32()
    {
        if (left == 0) refill();
        --left;
        return left == 3 ? buf[0] : (left == 2 ? buf[1] : (left == 1 ? buf[2] : buf[3]));
    }
    /* uniform double in [0, 1) with 53 random bits (Python random.random resolution) */
    B747_HD double u01()
    {
        uint64_t hi = u32(), lo = u32();
        return (double)(((hi << 32) | lo) >> 11) * (1.0 / 9007199254740992.0);
    }
    /* The draws are rounded exactly as written (no FMA contraction, also in the FAST translation
     * unit): a reset draws the same numbers whichever kernel runs it (k_env_reset, the auto-reset
     * inside k_env_steps / k_ppo_rollout) and the host build (tests) reproduces them bit for bit. */
    B747_HD double uniform(double a, double b)                               /* random.uniform */
    {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
        return a + (b - a) * u01();
    }
    B747_HD double normal(double mean, double std)                           /* Box-Muller */
    {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
        double u1 = 1.0 - u01(), u2 = u01();
        return mean + std * (sqrt(-2.0 * log(u1)) * cos(2.0 * PI * u2));
    }
};

/* Per-env controller state that survives between env steps. */
struct EnvSlot {
    double deltaz, upid, tp, ep_ret;
    int32_t ep_len;
    uint32_t flags, episode;
    double ref[8];         /* [0] const pitch, [1..3] A, [4..6] f, [7] altitude command (float64 as the
                            * reference's Python floats, core/controller.py:153-177) */
    uint32_t ref_kind;
};

/* Reference functions (core/controller.py:153-177): pitch command at time t. */
B747_HD double pitch_ref(const EnvSlot &s, double t)
{
    if (s.ref_kind == REF_OSC) {
        double A1 = s.ref[1], A2 = s.ref[2], A3 = s.ref[3], f1 = s.ref[4], f2 = s.ref[5], f3 = s.ref[6];
        return A1 * sin(2 * PI * f1 * t) + A2 * sin(2 * PI * f2 * t) + A3 * sin(2 * PI * f3 * t);
    }
    return s.ref[0];
}

/* Controller.reset random part (core/controller.py:144-193).  Writes state0 and the env's
 * reference, ctrl flags and aero errors.  Returns false when reset_mode == NONE (keep state0). */
B747_HD void draw_reset(const EnvCfg &cfg, uint64_t env_id, EnvSlot &s, double *state0, double *aero)
{
    Rng rng;
    rng.init(cfg.seed, env_id, s.episode);
    if (cfg.reset_ref_mode != RM_NONE) {
        double h0 = rng.uniform(1000, 11000);
        double Vx = rng.uniform(100, 265);
        double Vy = rng.uniform(-20, 20);
        double wz0 = rng.uniform(-0.001, 0.001);
        double vmax = cfg.vartheta_max;
        s.ref_kind = REF_CONST;
        if (cfg.reset_ref_mode == RM_CONST) {
            double r = rng.uniform(-vmax, -1 * PI / 180);
            r *= (rng.u01() < 0.5) ? 1.0 : -1.0;                        /* random.choice([1,-1]) */
            s.ref[0] = r;
        } else if (cfg.reset_ref_mode == RM_OSCILLATING) {
            double A1 = rng.uniform(0, vmax);
            double A2 = rng.uniform(0, vmax - A1);
            double A3 = rng.uniform(0, vmax - A1 - A2);
            s.ref[1] = A1; s.ref[2] = A2; s.ref[3] = A3;
            s.ref[4] = rng.uniform(0.01, 0.5);
            s.ref[5] = rng.uniform(0.01, 0.5);
            s.ref[6] = rng.uniform(0.01, 0.5);
            s.ref_kind = REF_OSC;
        } else {                                                         /* HYBRID */
            const bool use_ctrl = rng.u01() < 0.5;
            const double draw = use_ctrl ? rng.uniform(-1000, 1000) : rng.uniform(-vmax, vmax);
            /* both fields written on both paths: a store with a select()ed offset would force
             * the whole lane state into scratch */
            s.ref[7] = use_ctrl ? h0 + draw : s.ref[7];                 /* SEMI_MANUAL: h1 */
            s.ref[0] = use_ctrl ? s.ref[0] : draw;                      /* MANUAL: pitch ref */
            s.flags = use_ctrl ? (F_RP | F_PID_CS) : F_RP;
            /* a fresh Model: aero_err back to the DLL default 0 (core/controller.py:178) */
#pragma unroll
            for (int j = 0; j < 5; ++j) aero[j] = 0.0;
        }
        state0[0] = 0.0; state0[1] = h0; state0[2] = Vx; state0[3] = Vy; state0[4] = 0.0; state0[5] = wz0;
    }
    if (cfg.disturbance_mode == 0) {                                          /* AERO_DISTURBANCE */
        if (cfg.aero_fixed) {
#pragma unroll
            for (int j = 0; j < 5; ++j) aero[j] = cfg.aero_err_fixed[j];
        } else {
            const double mean[5] = {-0.1, 0.1, -0.1, -0.1, 0.1};
#pragma unroll
            for (int j = 0; j < 5; ++j) aero[j] = rng.normal(mean[j], 0.5);
        }
    }
}

/* exp() of the reward terms.  FAST: the hardware 2^x in f32 (v_exp_f32, ~1 ulp of f32) on the
 * f64 product x log2(e) -- the reward leaves the env as float32 (the SB3 buffers), and every CLASSIC
 * / PID_LIKE / QUALITY argument is <= 0, so the term is within ~2e-7 relative of the f64 exp (tests
 * hold obs and reward to 2e-6); FAITHFUL: libm / ocml exp. */
template <bool FAST>
B747_HD double rexp(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if (FAST) return (double)__builtin_amdgcn_exp2f((float)(x * 1.4426950408889634));
#endif
    return exp(x);
}

/* The episode return as SB3's VecMonitor accumulates it (neural/agent.py:77-78 wraps the SubprocVecEnv in
 * VecMonitor): `episode_returns += rewards` on a float32 array with the workers' float64 rewards, i.e. each step
 * float32(float64(return) + reward).  The return stays float32-valued in its double slot; SB3's ep_rew_mean is the
 * float32 mean of these (tests/tb_transfer.py: with these semantics 16 of the 17 recorded first-rollout means are
 * reproduced bit for bit). */
B747_HD double vecmonitor_add(double ret, double reward) { return (double)(float)(ret + reward); }

/* 1 / obs_max (FAST normalisation multiplies; the f64 quotient and product differ by at most 1 ulp,
 * below the float32 rounding of the observation) */
B747_HD double inv_obs_max(int obs_type, int j)
{
    switch (obs_type) {
    case OBS_PID_LIKE: { const double m[3] = {1 / (60 * PI), 1 / PI, 1 / PI}; return m[j]; }
    case OBS_SPEED_MODE: { const double m[5] = {1 / (60 * PI), 1 / PI, 1 / PI, 1.0 / 500, 1.0 / 100}; return m[j]; }
    case OBS_PID_SPEED_AERO: {
        const double m[10] = {1 / (60 * PI), 1 / PI, 1 / PI, 1.0 / 500, 1.0 / 100, 1 / 0.5, 1.0 / 2, 1 / 0.6, 1 / 0.05, 1.0};
        return m[j];
    }
    case OBS_PID_AERO: { const double m[8] = {1 / (60 * PI), 1 / PI, 1 / PI, 1 / 0.5, 1.0 / 2, 1 / 0.6, 1 / 0.05, 1.0}; return m[j]; }
    default: { const double m[7] = {1 / (10 * PI / 180), 1.0 / 12000, 1.0 / 15000, 1.0 / 500, 1.0 / 100, 1 / PI, 1 / PI}; return m[j]; }
    }
}

/* The stashed signals EnvReadOut reads for a configuration (SigStash's MASK), as a constexpr function of
 * the fields that select its code paths; must cover every SV() the read-out evaluates for that
 * configuration (tests/test_gpu_env.py compares a kernel stashing only these with one stashing all). */
constexpr uint32_t sig_bit(int j) { return 1u << j; }
constexpr uint32_t readout_signal_mask(int obs_type, int reward_type, int use_limiter)
{
    uint32_t m = sig_bit(S_SIM_TIME) | sig_bit(S_DVARTHETA) | sig_bit(S_VARTHETA_ZH) | sig_bit(S_U_COM_PID);
    if (reward_type == REW_CLASSIC) m |= sig_bit(S_DVARTHETA_DT) | sig_bit(S_DVARTHETA_DT_DT) | sig_bit(S_ITSE);
    else if (reward_type == REW_PID_LIKE) m |= sig_bit(S_U_COM);
    else if (reward_type == REW_QUALITY || reward_type == REW_MINIMAL) m |= sig_bit(S_ITSE);
    if (use_limiter) m |= sig_bit(S_STATE4);
    m |= sig_bit(S_DVARTHETA_INT) | sig_bit(S_DVARTHETA_DT);
    if (obs_type == OBS_SPEED_MODE || obs_type == OBS_PID_SPEED_AERO) m |= sig_bit(S_STATE2) | sig_bit(S_STATE3);
    if (obs_type == OBS_PID_AERO || obs_type == OBS_PID_SPEED_AERO)
        m |= sig_bit(S_CXA) | sig_bit(S_CYA) | sig_bit(S_MZ) | sig_bit(S_DCM) | sig_bit(S_K_ALPHA);
    if (obs_type == OBS_MODEL_STATE)
        for (int j = 0; j < 6; ++j) m |= sig_bit(S_STATE0 + j);
    return m;
}

/* Read-out of the env step: turns the stage-4 signals of the last sub-step (stashed by the
 * output pass at sg[j*sst], LDS on the GPU) into the observation (env/ctrl_env.py:217-247),
 * reward (:109-192) and done (:255-257).  Runs once per env step, after the RK4 stages, so none
 * of its configuration-dependent code sits inside the stage loop. */
template <bool FAST, uint32_t MASK = kAllSignals>   /* MASK: the stash layout (SigStash<MASK>) */
struct EnvReadOut {
    const EnvCfg &c;
    uint32_t flags;
    double deltaz;             /* DLL parameter deltaz used this step */
    double vartheta_param;     /* DLL parameter vartheta set for this step */
    float *obs;                /* this env's row */
    float *term_obs;           /* nullable */
    float *obs2;               /* nullable: second copy of the row (rollout obs_seq at the last step) */
    mutable double reward;
    mutable double upid;       /* U_com_PID read-out (Model.deltaz_ref) for the next ADD_* step */
    mutable double tp;         /* TF_REFERENCE state (in/out) */
    mutable bool done;

    B747_HD void operator()(const double *sg, int sst) const
    {
#define SV(j) sg[sig_row(MASK, (j)) * sst]
        const double t = SV(S_SIM_TIME);
        const double e = SV(S_DVARTHETA);
        /* Controller.vartheta_ref (core/controller.py:268-270) */
        const double vref = (flags & F_PID_CS) ? SV(S_VARTHETA_ZH) : vartheta_param;
        const double vf = (vref != 0.0) ? vref : c.vartheta_max;
        const double th = nan_to_num(SV(S_STATE4));   /* state getter nan_to_num */
        double r;
        /* FAST: one reciprocal of vf instead of five divisions */
        const double ivf = FAST ? 1.0 / vf : 0.0;
        const double e_vf = FAST ? fabs(e * ivf) : fabs(e / vf);
        if (c.reward_type == REW_CLASSIC) {
            /* rew[0..2] = normalised k1,k2,k3; rew[3]=kf, [4]=kITSE, [5]=k0, [6]=kt, [7]=ko */
            const double sum = c.rew[0] * fabs(e) + c.rew[1] * 1 * fabs(SV(S_DVARTHETA_DT)) +
                               c.rew[2] * fabs(SV(S_DVARTHETA_DT_DT));
            double r1 = 0.50 * rexp<FAST>(FAST ? -c.rew[5] * sum * fabs(ivf) : -c.rew[5] * sum / fabs(vf));
            double r2 = (vref * e < 0) ? 0.20 * rexp<FAST>(-c.rew[7] * e_vf) : 0.20;
            double r3 = (e_vf > 0.05) ? 0.20 * rexp<FAST>(-c.rew[6] * t) : 0.20;
            double r4 = 0.1 * rexp<FAST>(FAST ? -c.rew[4] * SV(S_ITSE) * (ivf * ivf) : -c.rew[4] * SV(S_ITSE) / (vf * vf));
            double rf = (c.ctrl_mode == CM_DIRECT)
                            ? (FAST ? -c.rew[3] * (0.5 * e_vf) * (fabs(deltaz - SV(S_U_COM_PID))) * (1 / (34 * PI / 180))
                                    : -c.rew[3] * fabs(e / (2 * vf)) * (fabs(deltaz - SV(S_U_COM_PID))) / (34 * PI / 180))
                            : 0.0;
            r = r1 + r2 + r3 + r4 + rf;
        } else if (c.reward_type == REW_PID_LIKE) {
            r = rexp<FAST>(-c.rew[0] * fabs(SV(S_U_COM) - SV(S_U_COM_PID)) / (34 * PI / 180));
        } else if (c.reward_type == REW_QUALITY || c.reward_type == REW_MINIMAL) {
            /* quality() (core/controller.py:336); MINIMAL returns Qmax * quality(), Qmax = 1 */
            r = rexp<FAST>(-60 * 0.1 * SV(S_ITSE) / (c.tk * (vref * vref)));
        } else {   /* REW_TF_REFERENCE: rew[0]=overshoot_ref, [1]=tp_ref, [2]=k */
            double overshoot = e_vf * 100;
            if (overshoot > 5) tp = t;
            r = exp(-c.rew[2] * fabs(overshoot - c.rew[0]) * fabs(c.rew[1] - tp));
        }
        reward = r;
        upid = SV(S_U_COM_PID);
        bool d = t >= c.tk;
        if (c.use_limiter)
            d = d || fabs(th) > 5 * PI / 180 + c.vartheta_max || deltaz > c.action_max;
        done = d;
        /* observation: entries in the reference's order, unrolled so they stay in registers */
        double o[OBS_MAX_DIM];
        const double Vx = nan_to_num(SV(S_STATE2)), Vy = nan_to_num(SV(S_STATE3));
        const int ot = c.obs_type;
        o[0] = SV(S_DVARTHETA_INT); o[1] = e; o[2] = SV(S_DVARTHETA_DT);
        o[3] = (ot == OBS_PID_AERO) ? SV(S_CXA) : Vx;
        o[4] = (ot == OBS_PID_AERO) ? SV(S_CYA) : Vy;
        o[5] = (ot == OBS_PID_AERO) ? SV(S_MZ) : SV(S_CXA);
        o[6] = (ot == OBS_PID_AERO) ? SV(S_DCM) : SV(S_CYA);
        o[7] = (ot == OBS_PID_AERO) ? SV(S_K_ALPHA) : SV(S_MZ);
        o[8] = SV(S_DCM);
        o[9] = SV(S_K_ALPHA);
        if (ot == OBS_MODEL_STATE) {
            o[0] = vref;
#pragma unroll
            for (int j = 0; j < 6; ++j) o[1 + j] = nan_to_num(SV(S_STATE0 + j));
        }
        const int nd = obs_dim_of(ot);
        const bool reset_now = d && c.auto_reset;
#pragma unroll
        for (int j = 0; j < OBS_MAX_DIM; ++j) {
            if (j < nd) {
                double v = c.norm_obs ? (FAST ? o[j] * inv_obs_max(ot, j) : o[j] / obs_max(ot, j)) : o[j];
                if (term_obs && d) term_obs[j] = (float)v;
                obs[j] = reset_now ? 0.0f : (float)v;   /* reset obs is all zeros (A.6) */
                if (obs2) obs2[j] = reset_now ? 0.0f : (float)v;
            }
        }
#undef SV
    }
};

}  // namespace b747
