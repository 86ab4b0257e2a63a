// model_simple_gpu.cpp -- the reference DLL's exported-globals ABI on the MI355X model kernels.
//
// core/model.py binds core/model_simple_win64.dll (core/model.py:104-113 loads `model_simple.so` on
// Linux) through exactly this surface: model_simple_initialize / model_simple_step /
// model_simple_terminate (core/model.py:238-250) and the exported `double` parameters and block
// signals it reads and writes with ctypes `in_dll` (core/model.py:124-164).  This library exports the
// same symbols; behind them one aircraft lives on the GPU as a 1-env b747_model_batch (include/b747.h)
// and every call is b747_model_initialize / b747_model_step on it: the parameter globals go to the
// device before the call, the 31 signals (B747_SIG_* order = the globals' order) come back after it.
// So the unmodified reference Model runs on the HIP dynamics -- one env per loaded copy, like the DLL;
// batches belong to b747_model_step / BatchModel.
//
// Variant: FAITHFUL (the DLL's operations in its order; parity vs the CPU oracle's DLL-ABI library at
// 1e-9 of each signal's range, tests/test_model_simple_shim.py); B747_MODEL_VARIANT=fast selects FAST.
// Every parameter crosses as the DLL's double, aero_err included (b747_model_batch.aero_err is double[5][N]).
// There is no CPU fallback: a HIP error aborts with its text, as the DLL has no error channel.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "b747.h"
#include "b747_tables.h"

#define EXPORT extern "C" __attribute__((visibility("default")))
#define EXPORT_VAR __attribute__((visibility("default")))   // inside extern "C" { }: definitions, not declarations

extern "C" {
// ---- exported model parameters (the DLL's .data; defaults = B747_DEF_*) ----
EXPORT_VAR double Iz = B747_DEF_IZ, P = B747_DEF_P, S = B747_DEF_S, c_ = B747_DEF_C, g = B747_DEF_G, m0 = B747_DEF_M0;
EXPORT_VAR double PID_CS[4] = {B747_DEF_PID_CS[0], B747_DEF_PID_CS[1], B747_DEF_PID_CS[2], B747_DEF_PID_CS[3]};
EXPORT_VAR double PID_SS[4] = {B747_DEF_PID_SS[0], B747_DEF_PID_SS[1], B747_DEF_PID_SS[2], B747_DEF_PID_SS[3]};
EXPORT_VAR double aero_err[5] = {B747_DEF_AERO_ERR[0], B747_DEF_AERO_ERR[1], B747_DEF_AERO_ERR[2], B747_DEF_AERO_ERR[3],
                             B747_DEF_AERO_ERR[4]};
EXPORT_VAR double deltaz = B747_DEF_DELTAZ, h_zh = B747_DEF_H_ZH, vartheta = B747_DEF_VARTHETA;
EXPORT_VAR double state0[6] = {B747_DEF_STATE0[0], B747_DEF_STATE0[1], B747_DEF_STATE0[2],
                           B747_DEF_STATE0[3], B747_DEF_STATE0[4], B747_DEF_STATE0[5]};
EXPORT_VAR double use_PID_CS = B747_DEF_USE_PID_CS, use_PID_SS = B747_DEF_USE_PID_SS, use_RL = B747_DEF_USE_RL,
              use_RP = B747_DEF_USE_RP;
// ---- exported block signals, B747_SIG_* order (zero until the first call, as in the DLL image) ----
EXPORT_VAR double sim_time, dvartheta, U_com, alpha, V, state[6], Mach;
EXPORT_VAR double dvartheta_dt, dvartheta_dt_dt, dvartheta_int, AE, ITAE, IAE, ISE, ITSE, SE, TAE, TSE;
EXPORT_VAR double K_alpha, mz, dCm_ddeltaz, CXa, CYa, deltaz_RP, U_com_PID, vartheta_zh;
}

namespace {

// the device parameter block (15 doubles, one copy per call): deltaz, vartheta, h_zh, state0[6],
// aero_err[5] (doubles 9-13), flags in the first byte of double 14
constexpr int kParDoubles = 15;

struct Device {
    b747_model_batch b{};
    b747_consts c{};
    void *mem = nullptr;   // one allocation: X, disc, k, mem, parameters, signals
    double *p_deltaz, *p_vartheta, *p_h_zh, *p_state0, *p_aero;
    uint8_t *p_flags;
    bool ready = false;
};
Device D;

void die(const char *what, int rc)
{
    std::fprintf(stderr, "model_simple (MI355X): %s failed (%d): %s\n", what, rc, b747_last_error());
    std::abort();
}
void hip_check(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        std::fprintf(stderr, "model_simple (MI355X): %s: %s\n", what, hipGetErrorString(e));
        std::abort();
    }
}

constexpr double kSwitch = 1.0;   // use_* >= 1.0 (dll@0x1ee9)

void params_in(bool defaults_only)
{
    double hb[kParDoubles] = {};
    hb[0] = defaults_only ? B747_DEF_DELTAZ : deltaz;
    hb[1] = defaults_only ? B747_DEF_VARTHETA : vartheta;
    hb[2] = defaults_only ? B747_DEF_H_ZH : h_zh;
    for (int j = 0; j < 6; ++j) hb[3 + j] = defaults_only ? B747_DEF_STATE0[j] : state0[j];
    for (int j = 0; j < 5; ++j) hb[9 + j] = defaults_only ? B747_DEF_AERO_ERR[j] : aero_err[j];
    const double u_ss = defaults_only ? B747_DEF_USE_PID_SS : use_PID_SS, u_cs = defaults_only ? B747_DEF_USE_PID_CS : use_PID_CS;
    const double u_rp = defaults_only ? B747_DEF_USE_RP : use_RP, u_rl = defaults_only ? B747_DEF_USE_RL : use_RL;
    *reinterpret_cast<uint8_t *>(hb + 14) = (uint8_t)((u_ss >= kSwitch ? B747_F_PID_SS : 0u) | (u_cs >= kSwitch ? B747_F_PID_CS : 0u) |
                                                      (u_rp >= kSwitch ? B747_F_RP : 0u) | (u_rl >= kSwitch ? B747_F_RL : 0u));
    hip_check(hipMemcpy(D.p_deltaz, hb, sizeof(hb), hipMemcpyHostToDevice), "parameters");
    D.c.Iz = defaults_only ? B747_DEF_IZ : Iz;
    D.c.P = defaults_only ? B747_DEF_P : P;
    D.c.S = defaults_only ? B747_DEF_S : S;
    D.c.c_ = defaults_only ? B747_DEF_C : c_;
    D.c.g = defaults_only ? B747_DEF_G : g;
    D.c.m0 = defaults_only ? B747_DEF_M0 : m0;
    for (int j = 0; j < 4; ++j) {
        D.c.PID_CS[j] = defaults_only ? B747_DEF_PID_CS[j] : PID_CS[j];
        D.c.PID_SS[j] = defaults_only ? B747_DEF_PID_SS[j] : PID_SS[j];
    }
}

void signals_out()
{
    double s[B747_NSIG];
    hip_check(hipMemcpy(s, D.b.sig, sizeof(s), hipMemcpyDeviceToHost), "signals");
    double *dst[B747_NSIG] = {&sim_time, &dvartheta, &U_com, &alpha, &V, &state[0], &state[1], &state[2],
                              &state[3], &state[4], &state[5], &Mach, &dvartheta_dt, &dvartheta_dt_dt,
                              &dvartheta_int, &AE, &ITAE, &IAE, &ISE, &ITSE, &SE, &TAE, &TSE, &K_alpha, &mz,
                              &dCm_ddeltaz, &CXa, &CYa, &deltaz_RP, &U_com_PID, &vartheta_zh};
    for (int j = 0; j < B747_NSIG; ++j) *dst[j] = s[j];
}

// First call: the device copy of the DLL image.  The DLL is loaded already initialised from its
// default parameters (.data), whatever the globals hold by now, so this initialize runs on B747_DEF_*.
void ensure_ready()
{
    if (D.ready) return;
    if (b747_abi_version() != B747_ABI_VERSION) die("b747_abi_version", b747_abi_version());
    const size_t off_disc = 18 * sizeof(double), off_k = off_disc + B747_NDISC * sizeof(double);
    const size_t off_par = off_k + 16, off_sig = off_par + kParDoubles * sizeof(double);
    const size_t total = off_sig + B747_NSIG * sizeof(double);
    hip_check(hipMalloc(&D.mem, total), "hipMalloc");
    hip_check(hipMemset(D.mem, 0, total), "hipMemset");
    char *m = static_cast<char *>(D.mem);
    double *par = reinterpret_cast<double *>(m + off_par);
    D.p_deltaz = par + 0;
    D.p_vartheta = par + 1;
    D.p_h_zh = par + 2;
    D.p_state0 = par + 3;                                    // [6][1]
    D.p_aero = par + 9;                                      // [5][1] double
    D.p_flags = reinterpret_cast<uint8_t *>(par + 14);
    D.b.n = 1;
    D.b.x_f64 = 1;
    const char *v = std::getenv("B747_MODEL_VARIANT");
    D.b.variant = (v && (v[0] == 'f' || v[0] == 'F') && (v[1] == 'a' || v[1] == 'A') && (v[2] == 's' || v[2] == 'S'))
                      ? B747_VARIANT_FAST : B747_VARIANT_FAITHFUL;
    D.b.X = m;
    D.b.disc = reinterpret_cast<double *>(m + off_disc);
    D.b.k = reinterpret_cast<uint32_t *>(m + off_k);
    D.b.mem = reinterpret_cast<uint8_t *>(m + off_k + 8);
    D.b.deltaz = D.p_deltaz;
    D.b.vartheta = D.p_vartheta;
    D.b.h_zh = D.p_h_zh;
    D.b.flags = D.p_flags;
    D.b.aero_err = D.p_aero;
    D.b.state0 = D.p_state0;
    D.b.sig = reinterpret_cast<double *>(m + off_sig);
    params_in(true);
    int rc = b747_model_initialize(&D.b, nullptr, nullptr);
    if (rc) die("b747_model_initialize", rc);
    D.ready = true;
}

}  // namespace

// model_simple_initialize (dll@0x12a0; core/model.py:238-241)
EXPORT void model_simple_initialize(void)
{
    ensure_ready();
    params_in(false);
    int rc = b747_model_initialize(&D.b, nullptr, nullptr);
    if (rc) die("b747_model_initialize", rc);
    signals_out();
}

// model_simple_step (dll@0x16d0; core/model.py:247-250): one ode4 step of 0.01 s
EXPORT void model_simple_step(void)
{
    ensure_ready();
    params_in(false);
    int rc = b747_model_step(&D.b, &D.c, 1, nullptr);
    if (rc) die("b747_model_step", rc);
    signals_out();
}

// model_simple_terminate (dll@0x29d0 is a bare `ret`); the device copy lives until unload
EXPORT void model_simple_terminate(void) {}
