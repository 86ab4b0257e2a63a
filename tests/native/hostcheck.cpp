// hostcheck.cpp -- TEST-ONLY host build of the product's per-lane dynamics
// (b747_rl_ctrl_amd/csrc/b747_dynamics.h) behind the oracle's batched signature.
//
// It lets the CPU test suite prove, without a GPU, that the compact-state reformulation used by
// the HIP kernels (k, last-4 U_com, last-major Derivative inputs, ...) reproduces the faithful
// DLL restatement (oracle/b747_oracle.c) step for step.  Never loaded by the product package.
#include <stdint.h>
#include <string.h>

#include "../../b747_rl_ctrl_amd/csrc/b747_dynamics.h"

using namespace b747;

template <bool FAST>
static void batch_step(
    int64_t n, int32_t n_steps, const double *consts, int32_t x64, void *X, double *disc,
    uint32_t *kk, uint8_t *memv, const double *deltaz, const double *vartheta, const double *h_zh,
    const uint8_t *flags, const double *aero_err, double *sig)
{
    Consts C = make_consts(consts[0], consts[1], consts[2], consts[3], consts[4], consts[5], consts + 6, consts + 10);
    double tb[T_TOTAL];
    stage_tables<FAST>(tb, 0, 1);
    for (int64_t i = 0; i < n; ++i) {
        double x[NX];
        for (int j = 0; j < NX; ++j) x[j] = x64 ? ((double *)X)[j * n + i] : (double)((float *)X)[j * n + i];
        Disc D;
        D.x_dss = disc[0 * n + i]; D.y_dss = disc[1 * n + i]; D.rl_prevY = disc[2 * n + i];
        D.e_prev = disc[3 * n + i]; D.ed_prev = disc[4 * n + i];
        for (int j = 0; j < 4; ++j) D.u_hist[j] = disc[(5 + j) * n + i];
        uint32_t k = kk[i], mem = memv[i];
        Params P;
        P.deltaz = deltaz[i]; P.vartheta = vartheta[i]; P.h_zh = h_zh[i]; P.flags = flags[i];
        P.kCX = aero_err[0 * n + i] + B747_F_ONE;
        P.kCY = aero_err[1 * n + i] + B747_F_ONE;
        P.kmz = aero_err[2 * n + i] + B747_M_ONE;
        P.kdCm = aero_err[3 * n + i] + B747_M_ONE;
        P.kKa = aero_err[4 * n + i] + B747_M_ONE;
        SigWriter wr{sig + i, n};
        for (int s = 0; s < n_steps; ++s)
            major_step<FAST>(x, D, k, mem, C, P, tb, wr, sig && s == n_steps - 1);
        for (int j = 0; j < NX; ++j) {
            if (x64) ((double *)X)[j * n + i] = x[j];
            else ((float *)X)[j * n + i] = (float)x[j];
        }
        disc[0 * n + i] = D.x_dss; disc[1 * n + i] = D.y_dss; disc[2 * n + i] = D.rl_prevY;
        disc[3 * n + i] = D.e_prev; disc[4 * n + i] = D.ed_prev;
        for (int j = 0; j < 4; ++j) disc[(5 + j) * n + i] = D.u_hist[j];
        kk[i] = k;
        memv[i] = (uint8_t)mem;
    }
}

extern "C" {

// DLL-faithful variant (must be bit-exact vs the oracle)
__attribute__((visibility("default"))) void b747h_batch_step(
    int64_t n, int32_t n_steps, const double *consts, int32_t x64, void *X, double *disc, uint32_t *kk,
    uint8_t *memv, const double *deltaz, const double *vartheta, const double *h_zh, const uint8_t *flags,
    const double *aero_err, const double * /*state0*/, double *sig)
{
    batch_step<false>(n, n_steps, consts, x64, X, disc, kk, memv, deltaz, vartheta, h_zh, flags, aero_err, sig);
}

// FAST variant (the GPU default): within a few ulp per step of the oracle
__attribute__((visibility("default"))) void b747h_batch_step_fast(
    int64_t n, int32_t n_steps, const double *consts, int32_t x64, void *X, double *disc, uint32_t *kk,
    uint8_t *memv, const double *deltaz, const double *vartheta, const double *h_zh, const uint8_t *flags,
    const double *aero_err, const double * /*state0*/, double *sig)
{
    batch_step<true>(n, n_steps, consts, x64, X, disc, kk, memv, deltaz, vartheta, h_zh, flags, aero_err, sig);
}

}  // extern "C"

extern "C" {
// FAST-variant math kernels on the host (the same B747_HD code the GPU runs)
__attribute__((visibility("default"))) double b747h_isa_powfit(double thr) { return isa_powfit(thr); }
__attribute__((visibility("default"))) double b747h_isa_expfit(double dhc) { return isa_expfit(dhc); }
__attribute__((visibility("default"))) double b747h_unit_atan2(double s, double c) { return unit_atan2(s, c); }
// interval index of the cell-grid axes: cell = 1 -> the FAST cell-grid search, 0 -> bp_index (the
// DLL's binary search restated); axis 0 CXa(CYa), 1 dCm(M), 2 mz(alpha), 3 K_alpha(alpha)
__attribute__((visibility("default"))) int b747h_axis_index(int axis, int cell, double u)
{
    const double *tb = kTableImage.v;
    switch (axis) {
    case 0: return cell ? cell_index(tb + T_CELL_CXA1, kCellCXa1, u) : bp_index<B747_CXA_MAX1>(B747_CXA_BP1, u);
    case 1: return cell ? cell_index(tb + T_CELL_DCM1, kCellDCm1, u) : bp_index<B747_DCM_MAX1>(B747_DCM_BP1, u);
    case 2: return cell ? cell_index(tb + T_CELL_MZ1, kCellMz1, u) : bp_index<B747_MZ_MAX1>(B747_MZ_BP1, u);
    default: return cell ? cell_index(tb + T_CELL_KA, kCellKa, u) : bp_index<B747_KA_MAX>(B747_KA_BP, u);
    }
}
__attribute__((visibility("default"))) int b747h_axis_cells(int axis)
{
    const CellGrid g[4] = {kCellCXa1, kCellDCm1, kCellMz1, kCellKa};
    return g[axis & 3].nc;
}
}

#include "../../b747_rl_ctrl_amd/csrc/b747_env.h"

extern "C" {

// Host build of the env reset draws (Philox keyed by seed x global env id): lets the CPU suite
// check sharding independence (gloo, world size 2) and the draw distributions.
__attribute__((visibility("default"))) void b747h_draw_resets(uint64_t seed, int64_t env_offset, int64_t n,
                                                               uint32_t episode, int32_t reset_mode,
                                                               int32_t disturbance, double vmax,
                                                               double *state0 /*[n][6]*/, double *ref /*[n][8]*/,
                                                               double *aero /*[n][5]*/, uint8_t *flags)
{
    b747_env_config cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.seed = seed;
    cfg.reset_ref_mode = reset_mode;
    cfg.disturbance_mode = disturbance;
    cfg.vartheta_max = vmax;
    for (int64_t i = 0; i < n; ++i) {
        EnvSlot s;
        memset(&s, 0, sizeof(s));
        s.episode = episode;
        s.flags = F_RP;
        double s0[6] = {0, 11000, 259.1667, 0, 0, 0};
        double ae[5] = {0, 0, 0, 0, 0};
        draw_reset(cfg, (uint64_t)(env_offset + i), s, s0, ae);
        for (int j = 0; j < 6; ++j) state0[i * 6 + j] = s0[j];
        for (int j = 0; j < 8; ++j) ref[i * 8 + j] = s.ref[j];
        for (int j = 0; j < 5; ++j) aero[i * 5 + j] = ae[j];
        flags[i] = (uint8_t)s.flags;
    }
}

}  // extern "C"

extern "C" {

// Host build of one env shard of the bench workload (BASELINE configs[2]/[3]: PID_LIKE obs, CLASSIC
// reward, MANUAL / DIRECT control, CONST resets, AERO errors, normalised obs/action, auto-reset) from
// the product's per-lane pieces (b747_dynamics.h major_step<FAST>, b747_env.h EnvReadOut / draw_reset /
// initialize); only the controller glue of env_step_lane (b747_lanes.h, device-only) is restated.
// Lets the gloo test step real shards on N CPU ranks.  All arrays are SoA [field][n] like the device
// batch; the envs are global ids env_offset..env_offset+n-1; state starts from the first reset inside.
__attribute__((visibility("default"))) void b747h_bench_shard(
    int64_t n, int64_t env_offset, uint64_t seed, double tk, int32_t n_steps, const float *actions /*[n_steps][n]*/,
    double *X /*[18][n]*/, uint32_t *kk, uint32_t *episode, float *obs /*[n][3]*/, float *reward, uint8_t *done,
    double *ep_ret)
{
    b747_env_config cfg;   // b747_env_config_default(PID_LIKE, CLASSIC) + the bench's settings
    memset(&cfg, 0, sizeof(cfg));
    cfg.obs_type = OBS_PID_LIKE; cfg.reward_type = REW_CLASSIC; cfg.norm_obs = 1; cfg.norm_act = 1;
    cfg.action_max = 17 * PI / 180; cfg.vartheta_max = 10 * PI / 180;
    cfg.rew[0] = 2.0 / 5; cfg.rew[1] = 2.0 / 5; cfg.rew[2] = 1.0 / 5; cfg.rew[3] = 0.1; cfg.rew[4] = 0.3; cfg.rew[5] = 2;
    cfg.rew[6] = -log(0.8) / 10; cfg.rew[7] = -log(0.75) / 0.15;
    cfg.ctrl_type = CT_MANUAL; cfg.ctrl_mode = CM_DIRECT; cfg.reset_ref_mode = RM_CONST; cfg.disturbance_mode = 0;
    cfg.n_sub = 1; cfg.sample_time = 0.01; cfg.tk = tk; cfg.seed = seed; cfg.auto_reset = 1;
    const Consts C = kDefaultConsts;
    double tb[T_TOTAL];
    stage_tables<true>(tb, 0, 1);
    double sg[NSIG];
    for (int64_t i = 0; i < n; ++i) {
        double x[NX], s0[6] = {0, 11000, 259.1667, 0, 0, 0};
        double aero[5] = {0, 0, 0, 0, 0};
        Disc D;
        uint32_t k, mem;
        EnvSlot s;
        memset(&s, 0, sizeof(s));
        s.flags = F_RP;
        s.episode = 0;
        draw_reset(cfg, (uint64_t)(env_offset + i), s, s0, aero);      // ControllerEnv.reset
        s.episode += 1u;
        initialize(x, D, k, mem, s0);
        double ret = 0.0;
        for (int32_t t = 0; t < n_steps; ++t) {
            const float a32 = (float)((double)actions[(int64_t)t * n + i] * cfg.action_max);   // env/ctrl_env.py:262
            Params P;
            P.deltaz = (double)a32;                                  // DIRECT_CONTROL (core/controller.py:242)
            P.vartheta = pitch_ref(s, t_of(k));                      // vartheta_func(t) (:235)
            P.h_zh = 11000.0;
            P.flags = s.flags;
            P.kCX = aero[0] + B747_F_ONE; P.kCY = aero[1] + B747_F_ONE;
            P.kmz = aero[2] + B747_M_ONE; P.kdCm = aero[3] + B747_M_ONE;
            P.kKa = aero[4] + B747_M_ONE;
            major_step<true>(x, D, k, mem, C, P, tb, SigStash<>{sg, 1}, true);
            EnvReadOut<true> ro{cfg, s.flags, P.deltaz, P.vartheta, obs + i * 3, nullptr, nullptr, 0.0, 0.0, 0.0, false};
            ro(sg, 1);
            const float r32 = (float)ro.reward;
            reward[i] = r32;
            ret = vecmonitor_add(ret, ro.reward);
            done[i] = ro.done ? 1 : 0;
            if (ro.done) {                                           // SB3 auto-reset (b747_lanes.h env_reset_lane)
                draw_reset(cfg, (uint64_t)(env_offset + i), s, s0, aero);
                s.episode += 1u;
                initialize(x, D, k, mem, s0);
                ret = 0.0;
            }
        }
        for (int j = 0; j < NX; ++j) X[j * n + i] = x[j];
        kk[i] = k;
        episode[i] = s.episode;
        ep_ret[i] = ret;
    }
}

}  // extern "C"
