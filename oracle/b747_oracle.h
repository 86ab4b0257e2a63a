/* b747_oracle.h -- CPU restatement of the reference dynamics (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X path.  It restates, block for block and in the
 * same floating-point operation order, the Simulink-ERT model compiled into the reference's
 * core/model_simple_win64.dll (`model_simple_initialize` dll@0x12a0, `model_simple_step`
 * dll@0x16d0, `model_simple_derivatives` dll@0x11a0, ode4 update dll@0x2c60,
 * `look2_binlx` dll@0x1000, `rt_TDelayInterpolate` dll@0x29e0, `rt_powd_snf` dll@0x3530).
 * Derived by reading the DLL's disassembly as text; the DLL itself was
 * never executed (executing it is denied in this environment).
 * Parity status: pinned to the DLL's own constant tables (gen/params.json, extracted from
 * its .data bytes) and, at trajectory level, to the closed-loop test results the reference
 * recorded on the DLL (tensorboard.xlsx transfer_custom/*, tests/golden/tb_transfer_first_log.json:
 * 48 of 51 closed-loop test metrics reproduced bit for bit in float32, the rest within 5e-7;
 * tests/test_tb_transfer_pin.py).  The reference ships no per-step golden vectors.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this code.
 * The product path (b747_rl_ctrl_amd/) never links or calls it.
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define B747O_NX 18

typedef struct b747o_model {
    /* ---- model parameters (exported globals; persist across initialize) ---- */
    double Iz, P, PID_CS[4], PID_SS[4], S, aero_err[5], c_, deltaz, g, h_zh, m0, state0[6];
    double use_PID_CS, use_PID_SS, use_RL, use_RP, vartheta;

    /* ---- exported block signals (what core/model.py reads) ---- */
    double sim_time, dvartheta, U_com, alpha, V, state[6], Mach;
    double dvartheta_dt, dvartheta_dt_dt, dvartheta_int, AE, ITAE, IAE, ISE, ITSE, SE, TAE, TSE;
    double K_alpha, mz, dCm_ddeltaz, CXa, CYa, deltaz_RP, U_com_PID, vartheta_zh;

    /* ---- internal block outputs (B struct) ---- */
    double rdot[2], acc[2], qdot[4], wdot;
    double in_CS, Np_CS, in_SS, Np_SS;      /* integrator inputs (Switch) and filter inputs */
    double k_CX, k_CY, k_mz, k_dCm, k_Ka;   /* 1 + aero_err, held in minor steps */
    double ud;                              /* transport-delay output */
    double T_isa, a_isa, rho, qq;           /* ISA block internals (kept for known-answer tests) */
    double y_dss;                           /* discrete state-space output (held) */
    double rl_out;                          /* rate-limiter output */
    uint8_t and3_SS, and3_CS, mem_SS, mem_CS;

    /* ---- DWork ---- */
    double x_dss, ic_firstT, rl_prevY, rl_lastT;
    double d1_TA, d1_uA, d1_TB, d1_uB, d2_TA, d2_uA, d2_TB, d2_uB;
    uint8_t dw_mem_SS, dw_mem_CS;
    int32_t dl_tail, dl_head, dl_last, dl_bufsz;
    double dl_buf[2 * 1024];                /* [0,bufsz) = u, [bufsz,2*bufsz) = t */

    /* ---- continuous states + timing ---- */
    double X[B747O_NX];
    double t, stop_time;
    uint32_t clock_tick0, clock_tick1;
    int major;                              /* 1 = MAJOR_TIME_STEP, 0 = MINOR */
    uint8_t tid2;                           /* 0.05 s rate counter (k mod 5) */
    uint8_t first_step;
} b747o_model;

/* Parameter defaults exactly as the DLL's .data. */
void b747o_defaults(b747o_model *m);
/* model_simple_initialize (dll@0x12a0). */
void b747o_initialize(b747o_model *m);
/* model_simple_step (dll@0x16d0): one major step + ode4. */
void b747o_step(b747o_model *m);

/* ---- compact state (the layout the HIP kernels keep in HBM; see include/b747.h) ----
 * k, X[18], x_dss, y_dss, rl_prevY, e_prev, ed_prev, u_hist[4] (slot j&3 = U_com at major
 * step j), mem bits.  Valid for any state reached by initialize + steps. */
typedef struct b747o_compact {
    uint32_t k;
    uint32_t mem;          /* bit0 = Memory (SS loop), bit1 = Memory (CS loop) */
    double X[B747O_NX];
    double x_dss, y_dss, rl_prevY, e_prev, ed_prev;
    double u_hist[4];
} b747o_compact;

void b747o_export_compact(const b747o_model *m, b747o_compact *c);
/* Rebuild the full DLL-faithful DWork (delay ring, Derivative time stamps, IC, TID) from a
 * compact state; parameters in *m are left untouched. */
void b747o_import_compact(b747o_model *m, const b747o_compact *c);

/* ---- test hooks (known-answer tests of single blocks) ---- */
/* which: 0 CYa(M, alpha_deg), 1 CXa(M, CYa), 2 dCm(h, M), 3 mz(M, alpha_deg), 4 K_alpha(alpha_deg) */
double b747o_test_lookup(int which, double u0, double u1);
/* one MAJOR output pass at step k on state X (parameters = DLL defaults + the given flags/commands);
 * writes the 31 exported signals (B747_SIG_* order) and ISA internals {T, a, rho, qq} */
void b747o_test_pass(const double *X, uint32_t k, double deltaz, double vartheta, double use_pid_ss,
                     double *sig31, double *isa4);

#ifdef __cplusplus
}
#endif
