/* b747_oracle_batch.c -- batched driver of the CPU oracle over the HIP path's SoA layout.
 *
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY.  For every env it rebuilds a DLL-faithful model
 * (b747o_model) from the compact SoA state (include/b747.h layout), runs `n_steps` calls of
 * model_simple_step (dll@0x16d0) and writes the compact state and the exported-signal read-out
 * back.  OpenMP over envs provides the "all host cores" CPU baseline.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "b747_oracle.h"

#define EXPORT __attribute__((visibility("default")))

/* keep in sync with include/b747.h */
#define NDISC 9
#define NSIG 31
enum { F_PID_SS = 1, F_PID_CS = 2, F_RP = 4, F_RL = 8 };

typedef struct {
    double Iz, P, S, c_, g, m0, PID_CS[4], PID_SS[4];
} consts_t;

static void set_params(b747o_model *m, const consts_t *c, int64_t n, int64_t i, const double *deltaz,
                       const double *vartheta, const double *h_zh, const uint8_t *flags,
                       const double *aero_err, const double *state0)
{
    m->Iz = c->Iz; m->P = c->P; m->S = c->S; m->c_ = c->c_; m->g = c->g; m->m0 = c->m0;
    for (int j = 0; j < 4; ++j) { m->PID_CS[j] = c->PID_CS[j]; m->PID_SS[j] = c->PID_SS[j]; }
    m->deltaz = deltaz[i];
    m->vartheta = vartheta[i];
    m->h_zh = h_zh[i];
    uint8_t f = flags[i];
    m->use_PID_SS = (f & F_PID_SS) ? 1.0 : 0.0;
    m->use_PID_CS = (f & F_PID_CS) ? 1.0 : 0.0;
    m->use_RP = (f & F_RP) ? 1.0 : 0.0;
    m->use_RL = (f & F_RL) ? 1.0 : 0.0;
    for (int j = 0; j < 5; ++j) m->aero_err[j] = aero_err[j * n + i];
    for (int j = 0; j < 6; ++j) m->state0[j] = state0[j * n + i];
}

static void signals_to_soa(const b747o_model *m, double *sig, int64_t n, int64_t i)
{
    const double v[NSIG] = {
        m->sim_time, m->dvartheta, m->U_com, m->alpha, m->V,
        m->state[0], m->state[1], m->state[2], m->state[3], m->state[4], m->state[5],
        m->Mach, m->dvartheta_dt, m->dvartheta_dt_dt, m->dvartheta_int, m->AE, m->ITAE, m->IAE,
        m->ISE, m->ITSE, m->SE, m->TAE, m->TSE, m->K_alpha, m->mz, m->dCm_ddeltaz, m->CXa, m->CYa,
        m->deltaz_RP, m->U_com_PID, m->vartheta_zh};
    for (int j = 0; j < NSIG; ++j) sig[j * n + i] = v[j];
}

/* X64 != 0: X is double[18][n]; else float[18][n] (promoted to double on import). */
EXPORT void b747o_batch_step(int64_t n, int32_t n_steps, const double *consts, int32_t x64, void *X,
                             double *disc, uint32_t *k, uint8_t *mem, const double *deltaz,
                             const double *vartheta, const double *h_zh, const uint8_t *flags,
                             const double *aero_err, const double *state0, double *sig)
{
    const consts_t *c = (const consts_t *)consts;
#pragma omp parallel
    {
        b747o_model *m = (b747o_model *)malloc(sizeof(b747o_model));
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            b747o_defaults(m);
            set_params(m, c, n, i, deltaz, vartheta, h_zh, flags, aero_err, state0);
            b747o_compact cs;
            memset(&cs, 0, sizeof(cs));
            cs.k = k[i];
            cs.mem = mem[i];
            for (int j = 0; j < B747O_NX; ++j)
                cs.X[j] = x64 ? ((double *)X)[j * n + i] : (double)((float *)X)[j * n + i];
            cs.x_dss = disc[0 * n + i]; cs.y_dss = disc[1 * n + i]; cs.rl_prevY = disc[2 * n + i];
            cs.e_prev = disc[3 * n + i]; cs.ed_prev = disc[4 * n + i];
            for (int j = 0; j < 4; ++j) cs.u_hist[j] = disc[(5 + j) * n + i];
            b747o_import_compact(m, &cs);
            for (int s = 0; s < n_steps; ++s) b747o_step(m);
            b747o_export_compact(m, &cs);
            k[i] = cs.k;
            mem[i] = (uint8_t)cs.mem;
            for (int j = 0; j < B747O_NX; ++j) {
                if (x64) ((double *)X)[j * n + i] = cs.X[j];
                else ((float *)X)[j * n + i] = (float)cs.X[j];
            }
            disc[0 * n + i] = cs.x_dss; disc[1 * n + i] = cs.y_dss; disc[2 * n + i] = cs.rl_prevY;
            disc[3 * n + i] = cs.e_prev; disc[4 * n + i] = cs.ed_prev;
            for (int j = 0; j < 4; ++j) disc[(5 + j) * n + i] = cs.u_hist[j];
            if (sig) signals_to_soa(m, sig, n, i);
        }
        free(m);
    }
}

/* model_simple_initialize for every env with mask[i] != 0 (mask may be NULL = all). */
EXPORT void b747o_batch_initialize(int64_t n, const double *consts, int32_t x64, void *X, double *disc,
                                   uint32_t *k, uint8_t *mem, const double *deltaz,
                                   const double *vartheta, const double *h_zh, const uint8_t *flags,
                                   const double *aero_err, const double *state0, double *sig,
                                   const uint8_t *mask)
{
    const consts_t *c = (const consts_t *)consts;
#pragma omp parallel
    {
        b747o_model *m = (b747o_model *)malloc(sizeof(b747o_model));
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            if (mask && !mask[i]) continue;
            b747o_defaults(m);
            set_params(m, c, n, i, deltaz, vartheta, h_zh, flags, aero_err, state0);
            b747o_initialize(m);
            b747o_compact cs;
            b747o_export_compact(m, &cs);
            k[i] = cs.k;
            mem[i] = (uint8_t)cs.mem;
            for (int j = 0; j < B747O_NX; ++j) {
                if (x64) ((double *)X)[j * n + i] = cs.X[j];
                else ((float *)X)[j * n + i] = (float)cs.X[j];
            }
            disc[0 * n + i] = cs.x_dss; disc[1 * n + i] = cs.y_dss; disc[2 * n + i] = cs.rl_prevY;
            disc[3 * n + i] = cs.e_prev; disc[4 * n + i] = cs.ed_prev;
            for (int j = 0; j < 4; ++j) disc[(5 + j) * n + i] = cs.u_hist[j];
            if (sig) signals_to_soa(m, sig, n, i);
        }
        free(m);
    }
}

/* Faithful single-model trajectory (no compact round trip): runs one env from initialize for
 * n_steps and records the 31 exported signals after every step -> sig[n_steps][31].
 * deltaz_seq (nullable) sets the `deltaz` parameter before each step, vartheta_seq likewise. */
EXPORT void b747o_trajectory(const double *consts, double deltaz, double vartheta, double h_zh,
                             uint8_t flags, const double *aero_err5, const double *state0_6,
                             int32_t n_steps, const double *deltaz_seq, const double *vartheta_seq,
                             double *sig_out)
{
    b747o_model *m = (b747o_model *)malloc(sizeof(b747o_model));
    const consts_t *c = (const consts_t *)consts;
    b747o_defaults(m);
    set_params(m, c, 1, 0, &deltaz, &vartheta, &h_zh, &flags, aero_err5, state0_6);
    b747o_initialize(m);
    for (int s = 0; s < n_steps; ++s) {
        if (deltaz_seq) m->deltaz = deltaz_seq[s];
        if (vartheta_seq) m->vartheta = vartheta_seq[s];
        b747o_step(m);
        signals_to_soa(m, sig_out + (size_t)s * NSIG, 1, 0);
    }
    free(m);
}

EXPORT double b747o_lookup(int which, double u0, double u1) { return b747o_test_lookup(which, u0, u1); }
EXPORT void b747o_pass(const double *X, uint32_t k, double deltaz, double vartheta, double use_pid_ss,
                       double *sig31, double *isa4)
{
    b747o_test_pass(X, k, deltaz, vartheta, use_pid_ss, sig31, isa4);
}

EXPORT int32_t b747o_nsig(void) { return NSIG; }
EXPORT int32_t b747o_ndisc(void) { return NDISC; }
