// b747_split_steps.h -- K env steps per launch with every env on TWO waves (b747_env_rollout / b747_env_step
// with n_env_steps > 1, FAST, kind 3).
//
// The step of k_env_step_split (b747_split.h: flight wave -- attitude, air data, ISA, lookups, forces, the
// flight states; control wave -- actuator, PIDs, Derivative blocks, controller, discrete state, resets)
// inside a loop over the K pre-sampled actions, with the state kept in registers across the steps and
// stored once at the end, as k_env_steps does for one wave per env:
//   per step  control: controller from action t, delay / DSS, delta of the four stages | flight: stage 0
//             up to the moment; barrier; the pipelined (or lock-step) stages; barrier; flight: read-out
//             into row t of obs_seq / reward_seq / done_seq, episode bookkeeping; barrier; resets.
// Action t + 1 is loaded during step t.  The end-of-launch store is env_store's with slot_params = "this env
// reset in the launch".  Training configuration only (kind 3: spec_config, default constants; CONST resets
// never change the flags, so lock step is decided once per launch).
#pragma once

#include "b747_split.h"

namespace {

using namespace b747;

template <typename XT>
__global__ __launch_bounds__(kSplitBlock) B747_NO_FMAC void k_env_steps_split(b747_env_batch b, b747_env_config cfgc,
                                                                             const float *actions, int32_t K,
                                                                             float *obs_seq, float *reward_seq,
                                                                             uint8_t *done_seq)
{
    __shared__ __attribute__((aligned(16))) double tb[kSplitTbEnd];
    __shared__ double sg[sig_rows(kSplitSigMask)][kSplitEnvs];   // stage-4 read-out stash (control wave)
    __shared__ double xth[4][kSplitEnvs], xct[4][kSplitEnvs];    // flight -> control: sin, cos theta per stage
    __shared__ double xh[4][kSplitEnvs];                         // flight -> control: h per stage
    __shared__ double xdl[4][kSplitEnvs];                        // control -> flight: delta per stage
    __shared__ double xr[6][kSplitEnvs];                         // control -> flight: state0 of a reset
    __shared__ double xra[5][kSplitEnvs];                         // control -> flight: aero errors of a reset
    __shared__ double xcv[2][kSplitEnvs];                        // control -> flight: deltaz, vartheta
    __shared__ uint32_t xcu[2][kSplitEnvs];                      // control -> flight: flags, k
    __shared__ uint8_t xdone[kSplitEnvs];                        // flight -> control: reset this env
    __shared__ unsigned lockstep, any_reset;
    unsigned kpd = prefetch_kernargs_issue<sizeof(b747_env_batch) + sizeof(b747_env_config) + 48>();
#if defined(__HIP_DEVICE_COMPILE__)
    prefetch_const_lines<sizeof(FitCoefs)>(split_kfit(0), kpd);
#endif
    const int64_t n = b.n;
    const int el = threadIdx.x & (kSplitEnvs - 1);
    const bool flight = threadIdx.x < kSplitEnvs;                // waves 0-3 (wave-uniform)
    const int64_t i = (int64_t)blockIdx.x * kSplitEnvs + el;
    const bool valid = i < n;
    const int64_t il = valid ? i : n - 1;
    EnvCfg cfgk = cfgc;
    spec_config(cfgk);
    const EnvCfg &cfg = cfgk;
    constexpr int lo = T_FAST_LO, hi = kSplitTbEnd;
    double tv[kSplitTbQ];
#pragma unroll
    for (int q = 0; q < kSplitTbQ; ++q) {
        const int jq = lo + (int)threadIdx.x + q * kSplitBlock;
        tv[q] = (jq < hi) ? split_image<false>(jq) : 0.0;
    }
    prefetch_kernargs_wait(kpd);
    if (threadIdx.x == 0) { lockstep = 0u; any_reset = 0u; }

    // ---- the env state, loaded once (roles as k_env_step_split)
    const XT *Xg = (const XT *)b.X;
    double x[kNC], y[kNC], acc[kNC];
    double km[5];
    Disc D;
    uint32_t k = 0u, mem = 0u, flags = 0u;
    double ref0 = 0.0;
    float a = 0.0f;
    double ep_ret = 0.0, h_zh = 0.0;
    if (flight) {
#pragma unroll
        for (int j = 0; j < kNF; ++j) x[j] = (double)Xg[kFX[j] * n + il];
        x[7] = x[8] = 0.0;
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = b.aero_err[j * n + il] + (j < 2 ? B747_F_ONE : B747_M_ONE);
        ep_ret = b.ep_return[il];
    } else {
        k = b.k[il];
        load_disc(b.disc, n, il, D);
        flags = b.flags[il];
        a = actions[il];
#pragma unroll
        for (int j = 0; j < kNC; ++j) x[j] = (double)Xg[(9 + j) * n + il];
        mem = b.mem[il];
        ref0 = b.ref[il];
        h_zh = b.h_zh[il];
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = 0.0;
    }
    const bool ctrl0 = (flags & F_PID_CS) != 0u;
    #pragma unroll

    for (int q = 0; q < kSplitTbQ; ++q) {

        const int jq = lo + (int)threadIdx.x + q * kSplitBlock;

        if (jq < hi) tb[jq] = tv[q];

    }
    wg_barrier();
    // delta of a stage needs the pitch error (SS PID, dead zone): lock step (decided once: see above)
    if (!flight && (flags & (F_PID_SS | F_RL)))
        __hip_atomic_fetch_or(&lockstep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    bool any_reset_env = false, done = false;
    float r = 0.0f;
    double deltaz = 0.0, vartheta = 0.0, upid = 0.0;   // upid: the U_com_PID read-out (Model.deltaz_ref)
    wg_barrier();
    const bool lock = lockstep != 0u;                   // workgroup-uniform, for the whole launch
    const int od = b.obs_dim;

    const FlightK fk = flight_consts<false>();   // K-step kernel: no VGPRs to spare (250 of 256)
    for (int32_t t = 0; t < K; ++t) {
        // the lane's env index, opaque per step: its address arithmetic is redone per use instead of
        // per-buffer addresses being hoisted out of the loop into registers (and spilled)
        int64_t iv = i, ilv = il;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(iv), "+v"(ilv));
#endif
        const int64_t row = (int64_t)t * n + iv;
        const bool last = t == K - 1;
        float a_next = 0.0f;
        if (!flight && !last) a_next = actions[(int64_t)(t + 1) * n + ilv];   // in flight during this step
        // ---- controller (core/controller.py:231-264 as env_step_lane; kind 3: MANUAL/DIRECT, CONST refs)
        Params P{};
        const double tk = t_of(k);
        const double tnew = (double)(k + 1u) * H;
        const double temp = 0.5 * H;
        const bool dss_hit = (k % 5u) == 0u;
        double ud = 0.0;
        PassRef R{};
        const uint32_t mem_held = mem;
        if (!flight) {
            const float a32 = cfg.norm_act ? (float)((double)a * cfg.action_max) : a;
            const double act = (double)a32;
            const bool use_ctrl = (flags & F_PID_CS) != 0u;
            const bool manual = (flags & F_PID_SS) == 0u;
            vartheta = use_ctrl ? 0.0 : ref0;
            h_zh = use_ctrl ? (double)0.0f : h_zh;
            deltaz = manual ? act : 0.0;
            P.deltaz = deltaz; P.vartheta = vartheta; P.h_zh = h_zh; P.flags = flags;
            xcv[0][el] = deltaz; xcv[1][el] = vartheta;
            xcu[0][el] = flags; xcu[1][el] = k;
            ud = delay_out(k, D.u_hist);
            D.y_dss = dss_hit ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
            R.has_ref = (k != 0u);
            R.t_ref = R.has_ref ? t_of(k - 1u) : 0.0;
            R.e_ref = D.e_prev; R.ed_ref = D.ed_prev; R.rl_prevY = D.rl_prevY;
            R.y_dss = D.y_dss; R.mem = mem;
            if (!lock) {
                double r0, d0, r1, d1, r3, d3;
                actuator(tk, R, r0, d0);
                PassRef R1 = R;
                R1.has_ref = true; R1.t_ref = tk; R1.rl_prevY = r0;
                actuator(temp + tk, R1, r1, d1);
                actuator(tnew, R1, r3, d3);
                const bool rp = (flags & F_RP) != 0u;
                xdl[0][el] = rp ? d0 : P.deltaz;
                xdl[1][el] = rp ? d1 : P.deltaz;
                xdl[2][el] = rp ? d1 : P.deltaz;
                xdl[3][el] = rp ? d3 : P.deltaz;
            }
        }
#pragma unroll
        for (int j = 0; j < kNC; ++j) { y[j] = x[j]; acc[j] = 0.0; }
        FlightPass fp{};
        if (flight) {
            flight_pre(x, tb, split_kfit(0), km, fp, fk, flight_ahead(x, split_kfit(0), fk, tb));
            xth[0][el] = fp.sth; xct[0][el] = fp.cth;
            xh[0][el] = x[1];
        }
        wg_barrier();                                // stage 0's (theta, h), the delta table
        if (threadIdx.x == 0) any_reset = 0u;        // (everyone read it before this barrier)
        PassOut po{};
        double thPID = 0.0;
        auto combine = [&](int st, const double *dX, int ns) __attribute__((always_inline)) {
            const double c = (st == 2) ? H : temp;
            const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
            for (int j = 0; j < ns; ++j) {
                const double fj = dX[j];
                acc[j] = acc[j] + wm * fj;
                x[j] = c * fj + y[j];
            }
        };
        auto control_stage = [&](int st, double theta, double h, double *dX) __attribute__((always_inline)) -> double {
            const double ts = (st == 0) ? tk : (st == 3 ? tnew : temp + tk);
            const double delta = control_pass(x, ts, theta, h, P, R, dX, po, thPID);
            if (st == 3) {
                SigVals sv;
                sv.v[S_SIM_TIME] = ts;
                sv.v[S_DVARTHETA] = po.e;
                sv.v[S_VARTHETA_ZH] = thPID;
                sv.v[S_U_COM_PID] = po.UPID;
                sv.v[S_DVARTHETA_DT] = po.ed;
                sv.v[S_DVARTHETA_DT_DT] = po.edd;
                sv.v[S_ITSE] = x[8];
                sv.v[S_DVARTHETA_INT] = x[4];
                SigStash<kSplitSigMask>{&sg[0][el], kSplitEnvs}(sv);
            }
            if (st == 0) {   // MAJOR-only updates (dll@0x271a)
                D.x_dss = dss_hit ? B747_DSS_A * D.x_dss + B747_DSS_B * ud : D.x_dss;
                hist_put(D.u_hist, k, po.Ucom);
                D.rl_prevY = po.r;
                D.e_prev = po.e;
                D.ed_prev = po.ed;
                mem = po.and3_bits;
                R.has_ref = true; R.t_ref = tk; R.e_ref = po.e; R.ed_ref = po.ed; R.rl_prevY = po.r;
                R.mem = mem_held;
            }
            return delta;
        };
        if (!lock) {
#pragma unroll
            for (int j = 1; j <= 4; ++j) {
                int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
                asm volatile("" : "+s"(zoff));
#endif
                double dX[kNC];
                if (flight) {
                    flight_post(x, xdl[j - 1][el], fp, dX, fk);
                    combine(j - 1, dX, kNF);
                    if (j < 4) {
                        flight_pre(x, tb + zoff, split_kfit(zoff), km, fp, fk, flight_ahead(x, split_kfit(zoff), fk, tb + zoff));
                        xth[j][el] = fp.sth; xct[j][el] = fp.cth;
                        xh[j][el] = x[1];
                    }
                } else {
                    control_stage(j - 1, unit_atan2(xth[j - 1][el], xct[j - 1][el], split_kfit(zoff)), xh[j - 1][el], dX);
                    combine(j - 1, dX, kNC);
                }
                if (j < 4) wg_barrier();
            }
        } else {
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
                asm volatile("" : "+s"(zoff));
#endif
                double dX[kNC];
                if (st > 0) {
                    if (flight) {
                        flight_pre(x, tb + zoff, split_kfit(zoff), km, fp, fk, flight_ahead(x, split_kfit(zoff), fk, tb + zoff));
                        xth[st][el] = fp.sth; xct[st][el] = fp.cth;
                        xh[st][el] = x[1];
                    }
                    wg_barrier();
                }
                if (!flight) {
                    xdl[st][el] = control_stage(st, unit_atan2(xth[st][el], xct[st][el], split_kfit(zoff)), xh[st][el], dX);
                    combine(st, dX, kNC);
                }
                wg_barrier();
                if (flight) {
                    flight_post(x, xdl[st][el], fp, dX, fk);
                    combine(st, dX, kNF);
                }
            }
        }
        const double t6 = H / 6.0;
#pragma unroll
        for (int j = 0; j < kNC; ++j)
            if (j < kNF || !flight) x[j] = acc[j] * t6 + y[j];
        if (!flight) {
            k += 1u;
            upid = po.UPID;                          // stage 3's, the read-out's
        }
        wg_barrier();                                // the stage-4 stash is complete
        if (flight) {   // read-out (EnvReadOut of the kind-3 configuration) into row t, episode bookkeeping
            float *seq_row = obs_seq ? obs_seq + row * od : nullptr;
            float *orow = last ? b.obs + iv * od : seq_row;   // the last step's row goes to both (k_env_steps)
            float *orow2 = last ? seq_row : nullptr;
            float scratch[OBS_MAX_DIM];
            float *trow = (valid && b.terminal_obs) ? b.terminal_obs + iv * od : nullptr;
            EnvReadOut<true, kSplitSigMask> ro{cfg, xcu[0][el], xcv[0][el], xcv[1][el],
                                               (valid && orow) ? orow : scratch, trow, valid ? orow2 : nullptr,
                                               0.0, 0.0, 0.0, false};
            ro(&sg[0][el], kSplitEnvs);
            r = (float)ro.reward;
            ep_ret += (double)r;
            done = ro.done;
            const int32_t ep_len = (int32_t)(xcu[1][el] + 1u);
            if (valid) {
                if (reward_seq) reward_seq[row] = r;
                if (done_seq) done_seq[row] = done ? 1 : 0;
                if (done) {   // record_episode_end
                    if (b.ep_final_return) b.ep_final_return[iv] = ep_ret;
                    if (b.ep_final_len) b.ep_final_len[iv] = ep_len;
                    if (b.ep_stats) {
                        b.ep_stats[iv] += 1.0;
                        b.ep_stats[n + iv] += ep_ret;
                        b.ep_stats[2 * n + iv] += (double)ep_len;
                    }
                }
            }
            const bool reset = done && cfg.auto_reset;
            xdone[el] = reset ? 1 : 0;
            if (reset) __hip_atomic_fetch_or(&any_reset, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        wg_barrier();
        if (any_reset != 0u) {                       // workgroup-uniform
            const bool rs = xdone[el] != 0;
            if (!flight && rs) {   // env_reset_lane, control side (idle lanes past N draw for env N-1, store nothing)
                EnvSlot s{};
                s.episode = b.episode[ilv];
#pragma unroll
                for (int j = 0; j < 8; ++j) s.ref[j] = b.ref[j * n + ilv];
                s.flags = flags;
                s.ref_kind = REF_CONST;
                double aero[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) aero[j] = b.aero_err[j * n + ilv];
                double s0[6];
#pragma unroll
                for (int j = 0; j < 6; ++j)
                    s0[j] = b.state0 ? b.state0[j * n + ilv] : (j == 1 ? 11000.0 : (j == 2 ? 259.1667 : 0.0));
                draw_reset(cfg, (uint64_t)(b.env_offset + ilv), s, s0, aero);
                if (valid && b.state0 && cfg.reset_ref_mode != RM_NONE) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) b.state0[j * n + iv] = s0[j];
                }
                s.episode += 1u;
                double xi[NX];
                uint32_t k0, m0;
                initialize(xi, D, k0, m0, s0);
#pragma unroll
                for (int j = 0; j < kNC; ++j) x[j] = xi[9 + j];
                k = k0;
                mem = m0;
                deltaz = 0.0;      // Model.initialize: deltaz = vartheta_zh = 0, every signal 0
                vartheta = 0.0;
                upid = 0.0;
                flags = s.flags;
                ref0 = s.ref[0];
                if (valid) {   // the slots only a reset changes (the per-step ones are stored at the end)
                    b.flags[iv] = (uint8_t)s.flags;
                    b.episode[iv] = s.episode;
#pragma unroll
                    for (int j = 0; j < 8; ++j) b.ref[j * n + iv] = s.ref[j];
                    b.ref_kind[iv] = (uint8_t)s.ref_kind;
#pragma unroll
                    for (int j = 0; j < 5; ++j) b.aero_err[j * n + iv] = aero[j];
                }
#pragma unroll
                for (int j = 0; j < 6; ++j) xr[j][el] = s0[j];
#pragma unroll
                for (int j = 0; j < 5; ++j) xra[j][el] = aero[j];
                any_reset_env = true;
            }
            wg_barrier();
            if (flight && rs) {   // the reset's initialize(), flight side
                double sf[6], xi[NX];
#pragma unroll
                for (int j = 0; j < 6; ++j) sf[j] = xr[j][el];
                Disc Dd;
                uint32_t k0, m0;
                initialize(xi, Dd, k0, m0, sf);
#pragma unroll
                for (int j = 0; j < kNF; ++j) x[j] = xi[kFX[j]];
#pragma unroll
                for (int j = 0; j < 5; ++j) km[j] = xra[j][el] + (j < 2 ? B747_F_ONE : B747_M_ONE);
                ep_ret = 0.0;
                any_reset_env = true;
            }
        }
        a = a_next;
    }
    // ---- store the env state once (env_store with slot_params = a reset in this launch)
    if (!valid) return;
    XT *Xw = (XT *)b.X;
    if (flight) {
#pragma unroll
        for (int j = 0; j < kNF; ++j) st_state(&Xw[kFX[j] * n + i], (XT)x[j]);
        if (any_reset_env) {   // initialize()'s q1 = q2 = +0
            st_state(&Xw[3 * n + i], (XT)0.0);
            st_state(&Xw[4 * n + i], (XT)0.0);
        }
        b.reward[i] = r;
        b.done[i] = done ? 1 : 0;
        b.ep_return[i] = ep_ret;
    } else {
#pragma unroll
        for (int j = 0; j < kNC; ++j) st_state(&Xw[(9 + j) * n + i], (XT)x[j]);
        store_disc(b.disc, n, i, D);
        b.k[i] = k;
        b.mem[i] = (uint8_t)mem;
        if (any_reset_env) {
            b.deltaz[i] = deltaz;
            b.upid[i] = upid;
            b.tp[i] = 0.0;
            b.ep_len[i] = (int32_t)k;
            b.vartheta[i] = vartheta;
        }
        if (any_reset_env || ctrl0 || (flags & F_PID_CS)) b.h_zh[i] = h_zh;
    }
}

}  // namespace
