/* model_simple_abi.c -- the reference DLL's exported-globals C ABI over the CPU oracle.
 *
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY.  Exposes exactly the symbol set that
 * core/model.py binds (core/model.py:124-164): model_simple_initialize/step/terminate plus the
 * exported `double` signals and parameters, so that a ctypes harness mimicking core/model.py
 * (or core/model.py itself on Linux, core/model.py:104-113) can drive it as
 * `model_simple.so`.  Used for BASELINE config 1 (the reference-equivalent single-env ctypes
 * path) and by the parity tests.  Built into oracle/build/model_simple.so by oracle/Makefile.
 */
#include <string.h>

#include "b747_oracle.h"

#define EXPORT __attribute__((visibility("default")))

/* ---- exported model parameters (dll.data / .bss) ---- */
EXPORT double Iz, P, PID_CS[4], PID_SS[4], S, aero_err[5], c_, deltaz, g, h_zh, m0, state0[6];
EXPORT double use_PID_CS, use_PID_SS, use_RL, use_RP, vartheta;
/* ---- exported block signals ---- */
EXPORT double sim_time, dvartheta, U_com, alpha, V, state[6], Mach;
EXPORT double dvartheta_dt, dvartheta_dt_dt, dvartheta_int, AE, ITAE, IAE, ISE, ITSE, SE, TAE, TSE;
EXPORT double K_alpha, mz, dCm_ddeltaz, CXa, CYa, deltaz_RP, U_com_PID, vartheta_zh;

static b747o_model M;
static int loaded;

static void params_in(void)
{
    M.Iz = Iz; M.P = P; memcpy(M.PID_CS, PID_CS, sizeof(PID_CS)); memcpy(M.PID_SS, PID_SS, sizeof(PID_SS));
    M.S = S; memcpy(M.aero_err, aero_err, sizeof(aero_err)); M.c_ = c_; M.deltaz = deltaz; M.g = g;
    M.h_zh = h_zh; M.m0 = m0; memcpy(M.state0, state0, sizeof(state0));
    M.use_PID_CS = use_PID_CS; M.use_PID_SS = use_PID_SS; M.use_RL = use_RL; M.use_RP = use_RP;
    M.vartheta = vartheta;
}

static void signals_out(void)
{
    sim_time = M.sim_time; dvartheta = M.dvartheta; U_com = M.U_com; alpha = M.alpha; V = M.V;
    memcpy(state, M.state, sizeof(state)); Mach = M.Mach;
    dvartheta_dt = M.dvartheta_dt; dvartheta_dt_dt = M.dvartheta_dt_dt; dvartheta_int = M.dvartheta_int;
    AE = M.AE; ITAE = M.ITAE; IAE = M.IAE; ISE = M.ISE; ITSE = M.ITSE; SE = M.SE; TAE = M.TAE; TSE = M.TSE;
    K_alpha = M.K_alpha; mz = M.mz; dCm_ddeltaz = M.dCm_ddeltaz; CXa = M.CXa; CYa = M.CYa;
    deltaz_RP = M.deltaz_RP; U_com_PID = M.U_com_PID; vartheta_zh = M.vartheta_zh;
}

/* Load-time defaults = the DLL image's .data. */
__attribute__((constructor)) static void load_defaults(void)
{
    b747o_defaults(&M);
    Iz = M.Iz; P = M.P; memcpy(PID_CS, M.PID_CS, sizeof(PID_CS)); memcpy(PID_SS, M.PID_SS, sizeof(PID_SS));
    S = M.S; memcpy(aero_err, M.aero_err, sizeof(aero_err)); c_ = M.c_; deltaz = M.deltaz; g = M.g;
    h_zh = M.h_zh; m0 = M.m0; memcpy(state0, M.state0, sizeof(state0));
    use_PID_CS = M.use_PID_CS; use_PID_SS = M.use_PID_SS; use_RL = M.use_RL; use_RP = M.use_RP;
    vartheta = M.vartheta;
    loaded = 1;
}

EXPORT void model_simple_initialize(void)
{
    params_in();
    b747o_initialize(&M);
    signals_out();
}

EXPORT void model_simple_step(void)
{
    params_in();
    b747o_step(&M);
    signals_out();
}

EXPORT void model_simple_terminate(void) { /* dll@0x29d0 is a bare `ret` */ }

/* ---- test hooks (not part of the reference ABI) ---- */
EXPORT void b747o_abi_export_compact(b747o_compact *c) { b747o_export_compact(&M, c); }
EXPORT void b747o_abi_import_compact(const b747o_compact *c) { params_in(); b747o_import_compact(&M, c); }
