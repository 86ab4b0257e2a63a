// b747_ppo_split.h -- k_rollout_split: T env steps per launch with every env on TWO waves that hand off per wave
// pair, for the fused config-5 rollout (POLICY: b747_ppo_rollout, the policy head on the control wave beside the
// flight wave's RK4 stages) and for K pre-sampled actions (!POLICY: b747_env_rollout in the training configuration).
//
// k_ppo_rollout (b747_fast.hip) runs policy and env step one after the other on one wave per env: the policy
// head is VALU / transcendental work, the env step a latency-bound fp64 chain, and neither fills the SIMD while
// the other runs.  Here each env has a lane in a flight wave and a control wave of a 512-thread workgroup (the
// roles of k_env_step_split, b747_split.h).  Under MANUAL control with the rate limiter in the loop (flags F_RP
// [| F_PID_CS], every env of the training configuration) the elevator delta of all four RK4 stages of step t is
// a function of the discrete state after step t - 1's MAJOR update alone (the 0.03 s transport delay keeps the
// current command out of it), so the control wave computes step t + 1's delta table right after its own stage 0
// of step t: the flight wave never waits for the control wave's controller (nor for the policy), and the action
// of step t enters only the control wave's delay history and the read-out.
//
// Per step t and wave pair (flight wave w, control wave w + 4: one SIMD, the same 64 envs), hand-offs through
// LDS counters (pair_post / pair_wait, b747_split.h) instead of workgroup barriers, since the two roles are in
// different phases of the step:
//   control: [resets of step t - 1] policy(obs_t) or action t -> rollout rows -> controller -> stage 0 (theta_0)
//            -> delta table of step t + 1 (posted) -> stages 1-3 (theta_j) -> read-out stash (posted)
//   flight:  [reset init] stages 0-3 (each posts its theta and h as soon as the attitude is known) -> wait for
//            the stash -> the next observation and the resets (posted), then reward / done / obs rows
// A workgroup holding an env whose delta depends on the stage (SS PID, dead zone) or on the current action (no
// rate limiter) runs lock step instead: the action first, then per stage flight pre -> control (delta) -> flight
// post, with the same counters.
// SUB (sample_time > dt, main.py's 0.05 s: n_sub DLL steps per env step, core/controller.py:258-264): the policy /
// action, the command injection and the read-out once per env step, the stages of every DLL step in between; the
// stage and delta counters count DLL steps (u = t n_sub + s), the stash / observation / reset counters env steps.
// Controller.step stops at the next multiple of n_sub, so only an env whose counter k is not aligned when the launch
// starts (a batch stepped before with another sample_time) takes fewer DLL steps: it sits out the first k % n_sub
// DLL steps of the launch's first env step (its state kept by selects on both waves).
// POLICY evaluates the policy head only; the value head is the deferred
// k_policy_value pass.  Every expression is the one k_env_steps_split / k_ppo_rollout
// evaluate; tests/test_gpu_ppo.py and tests/test_gpu_split.py hold the two instantiations to the two-launch
// rollout and to the one-wave K-step kernel, tests/test_gpu_fullsize.py and tests/test_gpu_episode_replay.py replay
// them through the C env oracle.
#pragma once

#include "b747_split.h"

// The control wave runs the policy of step t at wave priority 3 (s_setprio; 0: 9.28-9.38 us/step, 2: 8.70-8.76, 3:
// -0.2 more), before its stages; step t + 1's delta table after it has posted the read-out stash; the flight wave
// posts theta itself and the next observation before it computes the reward (profiles/EXPERIMENTS.md, round 3).
constexpr int kPpoPolicyPrio = 3;

namespace {

using namespace b747;

// One head of actor_critic (matrix-core layer 1; head 0 policy -> mean, 1 value) with its A fragments read from LDS
// where they are used instead of held in registers (fr: [f][64 lanes] uint4, f 0-1 layer 1 (mt), 2-17 layer 2
// (mt, s, part); the value head's 18 blocks follow the policy head's).
constexpr int kHeadFrag = (2 + 16) * 64;   // uint4 per head (18 KB)
template <int OD>
__device__ __forceinline__ float head_lds(const float *__restrict__ w, const uint4 *fr, const float *obs, int lane, int head)
{
    static_assert(OD <= kL1MaxOD, "the matrix-core layer 1");
    constexpr PolicyDerived D = PolicyDerived::of(OD);
    const int hb = 4 * (lane >> 5);
    fr += head * kHeadFrag;
    H8 a0, a1;
    a0.v = fr[0 * 64 + lane];
    a1.v = fr[1 * 64 + lane];
    H8 ob0, ob1;
    l1_obs_frags<OD>(obs, ob0, ob1);
    f32x16 rp[2][2];
    layer1_mfma(a0, a1, ob0, ob1, rp);
    f32x16 c0, c1, d00, d01, d10, d11;
    bias_tiles(w, D.acc0 + head * PH, hb, c0, c1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        H8 b0h, b0l, b1h, b1l;
        b_frags_d(rp, s, b0h, b0l, b1h, b1l);
        H8 a0h, a0l, a1h, a1l;   // A[(mt * 4 + s) * 2 + part]
        a0h.v = fr[(2 + (0 * 4 + s) * 2) * 64 + lane];
        a0l.v = fr[(2 + (0 * 4 + s) * 2 + 1) * 64 + lane];
        a1h.v = fr[(2 + (1 * 4 + s) * 2) * 64 + lane];
        a1l.v = fr[(2 + (1 * 4 + s) * 2 + 1) * 64 + lane];
        if (s == 0) {
            d00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h.h, b0h.h, c0, 0, 0, 0);
            d01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h.h, b1h.h, c0, 0, 0, 0);
            d10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h.h, b0h.h, c1, 0, 0, 0);
            d11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h.h, b1h.h, c1, 0, 0, 0);
        } else {
            B747_MFMA16(d00, a0h, b0h); B747_MFMA16(d01, a0h, b1h); B747_MFMA16(d10, a1h, b0h); B747_MFMA16(d11, a1h, b1h);
        }
        B747_MFMA16(d00, a0h, b0l); B747_MFMA16(d01, a0h, b1l); B747_MFMA16(d10, a1h, b0l); B747_MFMA16(d11, a1h, b1l);
        B747_MFMA16(d00, a0l, b0h); B747_MFMA16(d01, a0l, b1h); B747_MFMA16(d10, a1l, b0h); B747_MFMA16(d11, a1l, b1h);
    }
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) head_slice(w, D.hw + head * PH, d00, d01, d10, d11, r, hb, p0, p1);
    swap_halves(p0, p1);
    return (p0 + p1) + w[D.c + head];
}

constexpr int kPpoFragUint4 = kHeadFrag;   // the policy head's A fragments in LDS

// B747_STAMPS (diagnostic builds, tools/exp_stamps_ppo.py): s_memtime stamps of rollout step kPpoStampStep (and
// the start of the next one, slot 15) per wave
#ifdef B747_STAMPS
constexpr int kPpoStampStep = 32;
#define B747_PSTAMP(slot) do { if (t == kPpoStampStep || ((slot) == 1 && t == kPpoStampStep + 1)) B747_STAMP(t == kPpoStampStep ? (slot) : 15); } while (0)
#else
#define B747_PSTAMP(slot) ((void)0)
#endif

// The arguments of both instantiations: POLICY (b747_ppo_rollout) -- params, seed, step_base, T; the rollout rows
// obs_buf (the observation the policy saw at step t), act_buf, logp_buf, rew_buf, done_buf; act_lo / act_hi.
// !POLICY (b747_env_rollout with pre-sampled actions [T][N]) -- actions, T; obs_buf = obs_seq (the observation
// after step t), rew_buf = reward_seq, done_buf = done_seq, each nullable.
struct RolloutArgs {
    const float *params;
    uint64_t seed;
    const uint64_t *step_base;
    const float *actions;
    int32_t T;
    float *obs_buf, *act_buf, *logp_buf, *rew_buf;
    uint8_t *done_buf;
    float act_lo, act_hi;
    float *val_buf;   // (the value head is the separate k_policy_value pass)
};

template <bool POLICY, typename XT, bool SUB, bool MIX = false, int ENVS = kSplitEnvs>
__global__ __launch_bounds__(2 * ENVS) B747_NO_FMAC void k_rollout_split(b747_env_batch b, b747_env_config cfgc,
                                                                           RolloutArgs ra)
{
    const float *__restrict__ params = ra.params;
    const uint64_t seed = ra.seed;
    const int32_t T = ra.T;
    float *obs_buf = ra.obs_buf, *act_buf = ra.act_buf, *logp_buf = ra.logp_buf, *rew_buf = ra.rew_buf;
    uint8_t *done_buf = ra.done_buf;
    const float act_lo = ra.act_lo, act_hi = ra.act_hi;
    constexpr int OD = 3;
    constexpr PolicyDerived PD = PolicyDerived::of(OD);
    // the stratosphere branch of flight_ahead: taken around the fit where the policy's registers are live (without it
    // the PPO kernel spills), evaluated branch-free in the rollouts (measured: K = 100 5.74-5.86 against 5.94-6.02
    // us per step, sample_time 0.05 24.9-25.3 against 26.6-27.0)
    constexpr bool kSkipStrat = POLICY && !SUB;
    __shared__ __attribute__((aligned(16))) double tb[kSplitTbEnd];
    __shared__ double sg[sig_rows(kSplitSigMask)][ENVS];   // read-out stash (control -> flight)
    __shared__ double xth[4][ENVS];                        // flight -> control: theta per stage
    __shared__ double xh[4][ENVS];                         // flight -> control: h per stage
    __shared__ double xdl[2][4][ENVS];                     // control -> flight: delta per stage (step parity)
    __shared__ double xr[6][ENVS];                         // control -> flight: state0 of a reset
    __shared__ double xra[5][ENVS];                        // control -> flight: aero errors of a reset
    __shared__ double xcv[2][ENVS];                        // control -> flight: deltaz, vartheta
    __shared__ uint32_t xcu[2][ENVS];                      // control -> flight: flags, k
    __shared__ float xobs[OD][ENVS];                       // flight -> control: the next observation
    __shared__ uint8_t xdone[ENVS];                        // flight -> control: reset this env
    __shared__ uint32_t xr0[SUB ? ENVS : 1];               // control -> flight: k % n_sub at the launch (SUB)
    __shared__ float w[PD.total];                                // the policy's derived section
    __shared__ uint4 frag[kPpoFragUint4];                        // the policy head's A fragments
    __shared__ unsigned lockstep;
    // per pair, over the DLL steps u = t n_sub + s: f_th flight stage posts (4 u + st + 1), c_dl control delta posts
    // (free: u + 1 = delta of DLL step u written; lock step: 4 u + st + 1); over the env steps t: c_st stash of step t
    // (t + 1), f_ob read-out of step t (t + 1), c_rs resets of step t - 1 done (t)
    constexpr int kPairs = ENVS / 64;               // flight / control wave pairs per workgroup
    constexpr int BLK = 2 * ENVS;
    __shared__ unsigned f_th[kPairs], c_dl[kPairs], c_st[kPairs], f_ob[kPairs], c_rs[kPairs];
    unsigned kpd = prefetch_kernargs_issue<sizeof(b747_env_batch) + sizeof(b747_env_config) + sizeof(RolloutArgs)>();
#if defined(__HIP_DEVICE_COMPILE__)
    prefetch_const_lines<sizeof(FitCoefs)>(split_kfit(0), kpd);
#endif
    const int64_t n = b.n;
    const int el = threadIdx.x & (ENVS - 1);
    const bool flight = threadIdx.x < ENVS;                      // waves 0 .. kPairs - 1 (wave-uniform)
    const int wv = (threadIdx.x >> 6) & (kPairs - 1);
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * ENVS + el;
    const bool valid = i < n;
    const int64_t il = valid ? i : n - 1;
    EnvCfg cfgk = cfgc;
    spec_config(cfgk);
    const EnvCfg &cfg = cfgk;
    constexpr int lo = T_FAST_LO, hi = kSplitTbEnd;
    constexpr int kTbQ = (hi - lo + BLK - 1) / BLK;   // table entries per lane
    double tv[kTbQ];
#pragma unroll
    for (int q = 0; q < kTbQ; ++q) {
        const int jq = lo + (int)threadIdx.x + q * BLK;
        tv[q] = (jq < hi) ? split_image<MIX>(jq) : 0.0;
    }
    prefetch_kernargs_wait(kpd);
    if (threadIdx.x == 0) lockstep = 0u;
    if (threadIdx.x < kPairs) {
        f_th[threadIdx.x] = 0u; c_dl[threadIdx.x] = 0u; c_st[threadIdx.x] = 0u; f_ob[threadIdx.x] = 0u; c_rs[threadIdx.x] = 0u;
    }
    PolicyStage<OD, BLK> stage;
    if (POLICY) stage.load(params, threadIdx.x);

    // ---- the env state, loaded once (roles as k_env_steps_split)
    const XT *Xg = (const XT *)b.X;
    double x[kNC], y[kNC], acc[kNC];
    double km[5];
    Disc D;
    uint32_t k = 0u, mem = 0u, flags = 0u;
    double ref0 = 0.0;
    double ep_ret = 0.0, h_zh = 0.0;
    float o[OD];
    if (flight) {
#pragma unroll
        for (int j = 0; j < kNF; ++j) x[j] = (double)Xg[kFX[j] * n + il];
        x[7] = x[8] = 0.0;
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = b.aero_err[j * n + il] + (j < 2 ? B747_F_ONE : B747_M_ONE);
        ep_ret = (double)b.ep_return[il];
#pragma unroll
        for (int q = 0; q < OD; ++q) o[q] = 0.0f;
    } else {
        k = b.k[il];
        load_disc(b.disc, n, il, D);
        flags = b.flags[il];
#pragma unroll
        for (int j = 0; j < kNC; ++j) x[j] = (double)Xg[(9 + j) * n + il];
        mem = b.mem[il];
        ref0 = b.ref[il];
        h_zh = b.h_zh[il];
#pragma unroll
        for (int j = 0; j < 5; ++j) km[j] = 0.0;
#pragma unroll
        for (int q = 0; q < OD; ++q) o[q] = b.obs[il * OD + q];
    }
    const uint32_t nsub = SUB ? (uint32_t)cfg.n_sub : 1u;   // DLL steps per env step
    if (SUB && !flight) xr0[el] = k % nsub;
    const bool ctrl0 = (flags & F_PID_CS) != 0u;
#pragma unroll
    for (int q = 0; q < kTbQ; ++q) {
        const int jq = lo + (int)threadIdx.x + q * BLK;
        if (jq < hi) tb[jq] = tv[q];
    }
    if (POLICY) {
        stage.store(w, threadIdx.x);
        const uint4 *gl1 = reinterpret_cast<const uint4 *>(params + policy_l1pack_offset(OD));
        const uint4 *gpk = reinterpret_cast<const uint4 *>(params + policy_packed_offset(OD));
        for (int q = threadIdx.x; q < kPpoFragUint4; q += BLK) {
            const int h = q / kHeadFrag, f = q % kHeadFrag;
            frag[q] = f < 2 * 64 ? gl1[h * 2 * 64 + f] : gpk[h * (kPackPerHead / 4) + f - 2 * 64];
        }
    }
    // delta of a stage depends on the stage (SS PID, dead zone) or on the action (no rate limiter): lock step,
    // decided once per launch (CONST resets never change the flags)
    if (!flight && flags != F_RP && flags != (F_RP | F_PID_CS))
        __hip_atomic_fetch_or(&lockstep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    wg_barrier();
#if defined(__HIP_DEVICE_COMPILE__)
    // Every loop-carried value loaded above is waited for here, once.  Otherwise the first use inside the step loop
    // carries the wait, and since the loop body issues stores (the rollout rows) the compiler's count of outstanding
    // operations there is vmcnt(0): every step would drain all of the previous step's stores first.
    {
#pragma unroll
        for (int j = 0; j < kNC; ++j) asm volatile("" : "+v"(x[j]));
#pragma unroll
        for (int j = 0; j < 5; ++j) asm volatile("" : "+v"(km[j]));
#pragma unroll
        for (int q = 0; q < OD; ++q) asm volatile("" : "+v"(o[q]));
        asm volatile("" : "+v"(ep_ret), "+v"(h_zh), "+v"(ref0));
        asm volatile("" : "+v"(D.x_dss), "+v"(D.y_dss), "+v"(D.rl_prevY), "+v"(D.e_prev), "+v"(D.ed_prev));
        asm volatile("" : "+v"(D.u_hist[0]), "+v"(D.u_hist[1]), "+v"(D.u_hist[2]), "+v"(D.u_hist[3]));
        asm volatile("" : "+v"(k), "+v"(mem), "+v"(flags));
    }
#endif
    const bool lock = lockstep != 0u;                   // workgroup-uniform, for the whole launch
    // where the control wave runs the policy (above); with sub-steps always first, before the env step's DLL steps
    const uint32_t r0 = SUB ? xr0[el] : 0u;             // DLL steps this env sits out at the launch's first env step
    if (!flight && !lock) {                             // delta table of DLL step 0
        double d[4];
        delta_table(k, D, d);
#pragma unroll
        for (int st = 0; st < 4; ++st) xdl[0][st][el] = d[st];
        pair_post(&c_dl[wv], 1u);
    }
    bool any_reset_env = false, done = false, pair_reset = false;
    float r = 0.0f;
    double deltaz = 0.0, vartheta = 0.0, upid = 0.0;
    // record_episode_end (flight)
    // (the step's opaque copy of i: addresses derived from i itself are hoisted out of the loop and spilled)
    auto record_end = [&](int32_t ep_len, int64_t ie) __attribute__((always_inline)) {
        if (b.ep_final_return) b.ep_final_return[ie] = ep_ret;
        if (b.ep_final_len) b.ep_final_len[ie] = ep_len;
        if (b.ep_stats) {
            b.ep_stats[ie] += 1.0;
            b.ep_stats[n + ie] += ep_ret;
            b.ep_stats[2 * n + ie] += (double)ep_len;
        }
    };
    const float log_std = POLICY ? w[PD.log_std] : 0.0f;
    const float sdev = expf(log_std);
    uint64_t ctr0 = (POLICY && ra.step_base) ? *ra.step_base : 0u;
    ctr0 = ((uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(ctr0 >> 32)) << 32)   // uniform: SGPRs, not a
           | (uint64_t)__builtin_amdgcn_readfirstlane((unsigned)ctr0);              // spilled VGPR pair
    float a_in = 0.0f;                                  // !POLICY: this step's action (prefetched one step ahead)
    if (!POLICY && !flight && T > 0) a_in = ra.actions[il];
    const FlightK fk = flight_consts();
    const double t6 = H / 6.0;

    for (int32_t t = 0; t < T; ++t) {
        int64_t iv = i, ilv = il;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(iv), "+v"(ilv));
#endif
        const int64_t row = (int64_t)t * n + iv;
        const unsigned ut = (unsigned)t;
        const unsigned u0 = ut * nsub;                  // the env step's first DLL step in the launch
        B747_PSTAMP(1);
        if (flight) {
            // ---- the resets of step t - 1 (initialize(), flight side), then the four stages of every DLL step
            if (pair_reset) {
                pair_wait<1>(&c_rs[wv], ut);
                if (xdone[el]) {
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
            for (uint32_t s = 0; s < nsub; ++s) {
                const unsigned u = u0 + s;
                const int par = (int)(u & 1u);
                const bool act = !SUB || t > 0 || s >= r0;
#pragma unroll
                for (int j = 0; j < kNC; ++j) { y[j] = x[j]; acc[j] = 0.0; }
                if (!lock) pair_wait<1>(&c_dl[wv], u + 1u);   // delta of DLL step u (posted during step u - 1)
                B747_PSTAMP(2);
                FlightPass fp{};
                auto post = [&](int st) __attribute__((always_inline)) {
                    if (lock) pair_wait<0>(&c_dl[wv], 4u * u + (unsigned)st + 1u);
                    double dX[kNF];
                    flight_post(x, xdl[par][st][el], fp, dX, fk);
                    const double c = (st == 2) ? H : 0.5 * H;
                    const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
                    for (int j = 0; j < kNF; ++j) {
                        acc[j] = acc[j] + wm * dX[j];
                        x[j] = c * dX[j] + y[j];
                    }
                };
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
                    asm volatile("" : "+s"(zoff));
#endif
                    if (st > 0) post(st - 1);
                    const FlightAhead a = flight_ahead<MIX, kSkipStrat>(x, split_kfit(zoff), fk);
                    xth[st][el] = unit_atan2(a.sth, a.cth, split_kfit(zoff));   // theta itself (off the control's chain)
                    xh[st][el] = x[1];
                    pair_post(&f_th[wv], 4u * u + (unsigned)st + 1u);
                    flight_pre<MIX>(x, tb + zoff, split_kfit(zoff), km, fp, fk, a);
                    B747_PSTAMP(3 + st);
                }
                post(3);
#pragma unroll
                for (int j = 0; j < kNF; ++j) x[j] = (SUB && !act) ? y[j] : acc[j] * t6 + y[j];
            }
            // ---- read-out of step t (EnvReadOut of the kind-3 configuration): obs_{t+1} to the policy.  The control
            // wave rewrites xcv / xcu only after this wave's next stage-0 post, so they are read here in any order.
            B747_PSTAMP(7);
            pair_wait<0>(&c_st[wv], ut + 1u);
            B747_PSTAMP(8);
            float onew[OBS_MAX_DIM];
            float *trow = (valid && b.terminal_obs) ? b.terminal_obs + iv * OD : nullptr;
            const uint32_t fl = xcu[0][el];
            {   // the policy's next observation first (EnvReadOut's PID_LIKE rows and done, kind 3: no limiter), so
                // that the control wave starts the next policy while the reward is computed
                static_assert(kSpecObs == OBS_PID_LIKE && kSpecLimiter == 0, "the kind-3 read-out's observation and done");
                constexpr uint32_t M = kSplitSigMask;
                const double tr = sg[sig_row(M, S_SIM_TIME)][el];
                const bool rs = (tr >= cfg.tk) && cfg.auto_reset;
                xobs[0][el] = rs ? 0.0f : (float)(sg[sig_row(M, S_DVARTHETA_INT)][el] * inv_obs_max(OBS_PID_LIKE, 0));
                xobs[1][el] = rs ? 0.0f : (float)(sg[sig_row(M, S_DVARTHETA)][el] * inv_obs_max(OBS_PID_LIKE, 1));
                xobs[2][el] = rs ? 0.0f : (float)(sg[sig_row(M, S_DVARTHETA_DT)][el] * inv_obs_max(OBS_PID_LIKE, 2));
#pragma unroll
                for (int q = 0; q < OD; ++q) o[q] = xobs[q][el];   // (the flight wave's value head of the next step)
                xdone[el] = rs ? 1 : 0;
                pair_post(&f_ob[wv], ut + 1u);
            }
            EnvReadOut<true, kSplitSigMask> ro{cfg, fl, xcv[0][el], xcv[1][el], onew, trow, nullptr, 0.0, 0.0, 0.0, false};
            ro(&sg[0][el], ENVS);
            done = ro.done;
            // env steps of the episode: ceil(k / n_sub) after the step = floor(k / n_sub) before it + 1 (env_load)
            const uint32_t kst = xcu[1][el];
            const int32_t ep_len = (int32_t)(SUB ? kst / nsub + 1u : kst + 1u);
            const bool reset = done && cfg.auto_reset;
            B747_PSTAMP(9);
            pair_reset = wave_any(reset);   // (wave-uniform: every lane of the pair is active here)
            r = (float)ro.reward;
            ep_ret = vecmonitor_add(ep_ret, ro.reward);
            if (valid) {
                if (done_buf) done_buf[row] = done ? 1 : 0;
                if (rew_buf) rew_buf[row] = r;
                if (!POLICY && obs_buf) {   // obs_seq: the observation after step t
#pragma unroll
                    for (int q = 0; q < OD; ++q) obs_buf[row * OD + q] = onew[q];
                }
                if (done) record_end(ep_len, iv);
            }
            if (valid) {
                if (t == T - 1) {
#pragma unroll
                    for (int q = 0; q < OD; ++q) b.obs[iv * OD + q] = onew[q];
                }
            }
        } else {
            const int par0 = (int)(u0 & 1u);
            // ---- the resets of step t - 1 (Controller.reset / env_reset_lane, control side)
            if (t > 0) {
                pair_wait<1>(&f_ob[wv], ut);
#pragma unroll
                for (int q = 0; q < OD; ++q) o[q] = xobs[q][el];
                const bool rs = xdone[el] != 0;
                if (wave_any(rs)) {
                    if (rs) {   // idle lanes past N draw for env N - 1 and store nothing
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
                        deltaz = 0.0;
                        vartheta = 0.0;
                        upid = 0.0;
                        flags = s.flags;
                        ref0 = s.ref[0];
                        if (valid) {
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
                        if (!lock) {   // the delta table of the step's first DLL step from the reset state
                            double d[4];
                            delta_table(k, D, d);
#pragma unroll
                            for (int st = 0; st < 4; ++st) xdl[par0][st][el] = d[st];
                        }
                        any_reset_env = true;
                    }
                    pair_post(&c_rs[wv], ut);
                }
            }
            // ---- policy head on obs_t, Gaussian sample (the k_policy_act / k_ppo_rollout stream), rollout rows.
            // Lock step: first (the stages' delta needs the action); otherwise after stage 0 -- nothing of step t
            // before the read-out reads the action but the delay history, which takes it after stage 0 (below)
            const bool use_ctrl = (flags & F_PID_CS) != 0u;
            const bool manual = (flags & F_PID_SS) == 0u;
            auto policy = [&]() __attribute__((always_inline)) -> double {
                if (!POLICY) {   // the pre-sampled action of step t (k_env_steps_split's controller)
                    const float a = a_in;
                    if (t + 1 < T) a_in = ra.actions[(int64_t)(t + 1) * n + ilv];   // in flight during this step
                    const float a32 = cfg.norm_act ? (float)((double)a * cfg.action_max) : a;
                    return manual ? (double)a32 : 0.0;
                }
                const float mean = head_lds<OD>(w, frag, o, lane, 0);
                const float z = policy_noise(seed, ctr0 + (uint64_t)t, (uint64_t)(b.env_offset + ilv));
                const float a = __fadd_rn(mean, __fmul_rn(sdev, z));
                const float aenv = fminf(fmaxf(a, act_lo), act_hi);
                if (valid) {
#pragma unroll
                    for (int q = 0; q < OD; ++q) obs_buf[row * OD + q] = o[q];
                    act_buf[row] = a;
                    logp_buf[row] = __fsub_rn(__fsub_rn(__fmul_rn(__fmul_rn(-0.5f, z), z), log_std), 0.918938533204672742f);
                }
                const float a32 = cfg.norm_act ? (float)((double)aenv * cfg.action_max) : aenv;
                return manual ? (double)a32 : 0.0;   // Model.deltaz
            };
            B747_PSTAMP(2);
            if (POLICY) __builtin_amdgcn_s_setprio(kPpoPolicyPrio);
            deltaz = policy();
            if (POLICY) __builtin_amdgcn_s_setprio(0);
            B747_PSTAMP(3);
            // ---- controller (core/controller.py:231-264 as k_env_steps_split): the command injection and the
            // action once per env step, then the DLL steps up to the next multiple of n_sub
            Params P{};
            vartheta = use_ctrl ? 0.0 : ref0;
            h_zh = use_ctrl ? (double)0.0f : h_zh;
            P.deltaz = deltaz; P.vartheta = vartheta; P.h_zh = h_zh; P.flags = flags;   // (free: deltaz set below)
            const uint32_t k_start = k;
            PassOut po{};
            for (uint32_t s = 0; s < nsub; ++s) {
                const unsigned u = u0 + s;
                const int par = (int)(u & 1u);
                const bool act = !SUB || t > 0 || s >= r0;   // (SUB: the misaligned env's skipped DLL steps keep its state)
#pragma unroll
                for (int j = 0; j < kNC; ++j) { y[j] = x[j]; acc[j] = 0.0; }
                const double tk = t_of(k);
                const double tnew = (double)(k + 1u) * H;
                const double temp = 0.5 * H;
                const bool dss_hit = (k % 5u) == 0u;
                const uint32_t mem_held = mem;
                const double ud = delay_out(k, D.u_hist);
                D.y_dss = (dss_hit && act) ? D.x_dss * B747_DSS_C + B747_DSS_D * ud : D.y_dss;
                PassRef R{};
                R.has_ref = (k != 0u);
                R.t_ref = R.has_ref ? t_of(k - 1u) : 0.0;
                R.e_ref = D.e_prev; R.ed_ref = D.ed_prev; R.rl_prevY = D.rl_prevY;
                R.y_dss = D.y_dss; R.mem = mem;
                double thPID = 0.0;
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    int zoff = 0;
#if defined(__HIP_DEVICE_COMPILE__)
                    asm volatile("" : "+s"(zoff));
#endif
                    (void)zoff;
                    pair_wait<1>(&f_th[wv], 4u * u + (unsigned)st + 1u);
                    if (st == 0) B747_PSTAMP(4);
                    const double ts = (st == 0) ? tk : (st == 3 ? tnew : temp + tk);
                    double dX[kNC];
                    const double theta = xth[st][el];
                    const double delta = control_pass(x, ts, theta, xh[st][el],
                                                      P, R, dX, po, thPID);
                    if (lock) {
                        xdl[par][st][el] = delta;
                        pair_post(&c_dl[wv], 4u * u + (unsigned)st + 1u);
                    }
                    if (st == 3) {
                        if (s + 1u == nsub) {   // the read-out's stage-4 signals of the env step's last DLL step
                            SigVals sv;
                            sv.v[S_SIM_TIME] = ts;
                            sv.v[S_DVARTHETA] = po.e;
                            sv.v[S_VARTHETA_ZH] = thPID;
                            sv.v[S_U_COM_PID] = po.UPID;
                            sv.v[S_DVARTHETA_DT] = po.ed;
                            sv.v[S_DVARTHETA_DT_DT] = po.edd;
                            sv.v[S_ITSE] = x[8];
                            sv.v[S_DVARTHETA_INT] = x[4];
                            SigStash<kSplitSigMask>{&sg[0][el], ENVS}(sv);
                            pair_post(&c_st[wv], ut + 1u);
                        }
                        if (!lock) {   // DLL step u + 1's delta table once the stash is out (D: stage 0's)
                            double d[4];
                            delta_table(act ? k + 1u : k, D, d);
#pragma unroll
                            for (int q = 0; q < 4; ++q) xdl[par ^ 1][q][el] = d[q];
                            pair_post(&c_dl[wv], u + 2u);
                        }
                    }
                    if (st == 0) {   // MAJOR-only updates (dll@0x271a), then DLL step u + 1's delta table
                        D.x_dss = (dss_hit && act) ? B747_DSS_A * D.x_dss + B747_DSS_B * ud : D.x_dss;
                        hist_put(D.u_hist, k, act ? po.Ucom : hist_get(D.u_hist, k));
                        D.rl_prevY = act ? po.r : D.rl_prevY;
                        D.e_prev = act ? po.e : D.e_prev;
                        D.ed_prev = act ? po.ed : D.ed_prev;
                        mem = act ? po.and3_bits : mem;
                        R.has_ref = true; R.t_ref = tk; R.e_ref = po.e; R.ed_ref = po.ed; R.rl_prevY = po.r;
                        R.mem = mem_held;
                        if (s == 0u) {
                            // the read-out's inputs of this env step: written only now, after this DLL step's stage-0
                            // wait, i.e. after the flight wave has read the previous step's (its read-out precedes its
                            // next stage-0 post in program order, and one wave's LDS operations are performed in order)
                            xcv[0][el] = deltaz; xcv[1][el] = vartheta;
                            xcu[0][el] = flags; xcu[1][el] = k_start;
                        }
                    }
                    const double c = (st == 2) ? H : temp;
                    const double wm = (st == 1 || st == 2) ? 2.0 : 1.0;
#pragma unroll
                    for (int j = 0; j < kNC; ++j) {
                        acc[j] = acc[j] + wm * dX[j];
                        x[j] = c * dX[j] + y[j];
                    }
                    B747_PSTAMP(5 + st);
                }
#pragma unroll
                for (int j = 0; j < kNC; ++j) x[j] = (SUB && !act) ? y[j] : acc[j] * t6 + y[j];
                k += act ? 1u : 0u;
            }
            upid = po.UPID;
        }
    }
    // ---- the resets of the last step, then the env state stored once (env_store, slot_params = a reset)
    if (T > 0) {
        if (flight) {
            if (pair_reset) {
                pair_wait<1>(&c_rs[wv], (unsigned)T);
                if (xdone[el]) {
                    double sf[6], xi[NX];
#pragma unroll
                    for (int j = 0; j < 6; ++j) sf[j] = xr[j][el];
                    Disc Dd;
                    uint32_t k0, m0;
                    initialize(xi, Dd, k0, m0, sf);
#pragma unroll
                    for (int j = 0; j < kNF; ++j) x[j] = xi[kFX[j]];
                    ep_ret = 0.0;
                    any_reset_env = true;
                }
            }
        } else {
            pair_wait<1>(&f_ob[wv], (unsigned)T);
            const bool rs = xdone[el] != 0;
            if (wave_any(rs)) {
                if (rs) {
                    EnvSlot s{};
                    s.episode = b.episode[il];
#pragma unroll
                    for (int j = 0; j < 8; ++j) s.ref[j] = b.ref[j * n + il];
                    s.flags = flags;
                    s.ref_kind = REF_CONST;
                    double aero[5];
#pragma unroll
                    for (int j = 0; j < 5; ++j) aero[j] = b.aero_err[j * n + il];
                    double s0[6];
#pragma unroll
                    for (int j = 0; j < 6; ++j)
                        s0[j] = b.state0 ? b.state0[j * n + il] : (j == 1 ? 11000.0 : (j == 2 ? 259.1667 : 0.0));
                    draw_reset(cfg, (uint64_t)(b.env_offset + il), s, s0, aero);
                    if (valid && b.state0 && cfg.reset_ref_mode != RM_NONE) {
#pragma unroll
                        for (int j = 0; j < 6; ++j) b.state0[j * n + i] = s0[j];
                    }
                    s.episode += 1u;
                    double xi[NX];
                    uint32_t k0, m0;
                    initialize(xi, D, k0, m0, s0);
#pragma unroll
                    for (int j = 0; j < kNC; ++j) x[j] = xi[9 + j];
                    k = k0;
                    mem = m0;
                    deltaz = 0.0;
                    vartheta = 0.0;
                    upid = 0.0;
                    flags = s.flags;
                    if (valid) {
                        b.flags[i] = (uint8_t)s.flags;
                        b.episode[i] = s.episode;
#pragma unroll
                        for (int j = 0; j < 8; ++j) b.ref[j * n + i] = s.ref[j];
                        b.ref_kind[i] = (uint8_t)s.ref_kind;
#pragma unroll
                        for (int j = 0; j < 5; ++j) b.aero_err[j * n + i] = aero[j];
                    }
#pragma unroll
                    for (int j = 0; j < 6; ++j) xr[j][el] = s0[j];
                    any_reset_env = true;
                }
                pair_post(&c_rs[wv], (unsigned)T);
            }
        }
    }
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
        b.ep_return[i] = (float)ep_ret;
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
            b.ep_len[i] = (int32_t)(k / nsub);   // env steps since the reset in this launch
            b.vartheta[i] = vartheta;
        }
        if (any_reset_env || ctrl0 || (flags & F_PID_CS)) b.h_zh[i] = h_zh;
    }
}

}  // namespace
