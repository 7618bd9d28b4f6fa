// Rollout for WIDE observations (48 < obs_dim <= 512: Humanoid's 376) -- one 256-thread workgroup per task
// (one wave per SIMD, 512 registers per lane), every one of the T steps on one CU with three workgroup
// barriers.  Same semantics as the lane kernel of
// pgm_rollout_lanes.hip (reference sites listed there: Policy.act, DiagGaussian, DummyVecEnv auto-reset,
// TimeLimitMask, VecNormalize.step_wait, RunningMeanStd, RolloutStorage.insert / after_update); the critic is
// off the step chain here too (value_kernel afterwards).
//
// Work split of one step (NN envs, 4 waves, lane l):
//   1. layer 1 (O x 64 per env, the dominant MACs): wave w owns the k-slice [w*KW, w*KW + KW) of the inputs
//      and contracts it for all envs on the f32 MFMA (16x16x4: envs on rows, W1 slice as register-resident B
//      operands); per-wave partial sums go to LDS.                                                  barrier A
//   2. env n on wave n % 4: sums the 4 partials (fixed order) + bias, tanh -> h1 row (wave-local), layer 2
//      with its W2 column in registers, the mean head as transposing DPP sums, then the Gaussian draw,
//      log-prob and clipped action with lane a = action a; clipped actions (fp64) to LDS.          barrier C
//   3. feature slots (thread t: features t and t + 256, every env in registers): fp64 SynthMO dynamics, time limit /
//      auto-reset, per-wave transposing fp64 sums of V_k . s'[n] for the objectives, ob_rms Chan merge of the
//      feature (all envs are in the thread: no cross-thread reduction), normalised fp32 obs -> LDS + HBM.
//      The last wave (fewest features) then finishes the PREVIOUS step's objectives: objective sums,
//      VecNormalize.obj accumulators, obj_rms / ret_rms merges and the scaled rewards.             barrier D
#include "pgm_dispatch.hpp"
#include "pgm_rollout.hpp"

PGM_STAMP_UNIT(wide)

namespace pgm {

namespace {

constexpr int WW = 4;          // waves per workgroup (one per SIMD: 512 registers per lane)
constexpr int WTH = 64 * WW;   // threads
constexpr int WNCH = 32;       // rollout steps per staged noise chunk

template <int O>
constexpr int wkw() { return ((O + WW - 1) / WW + 3) & ~3; }  // inputs per wave slice (multiple of 4)
template <int O>
constexpr int wrow() { return WW * wkw<O>(); }               // padded LDS input row
template <int O, int K, int NN>
constexpr bool wide_fit() { return O > 48 && O <= 2 * WTH && NN * K <= 16 && (K & (K - 1)) == 0; }

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int O, int A, int K, int NN>
struct WideSmem {
    alignas(16) float x[NN][wrow<O>() + 4];  // normalised fp32 obs rows (zero padding beyond O; +4: bank stagger)
    alignas(16) float zp[WW][NN][H];     // layer-1 partial sums, one k-slice per wave
    alignas(16) float h1[NN][H];         // per-env layer-1 row (written / read by wave n)
    float mu[NN][32];                    // per-env action means (lane-distribution staging)
    double ac[NN][A];                    // clipped actions of this step
    double e2[2][NN];                    // |clip(a)|^2, by step parity (read one step later)
    double objp[2][WW][16];              // per-wave sums of V_k . s'[n] (index n*K + k), by step parity
    alignas(16) float eps[2][NN][WNCH * A];
    double U[A][2 * WTH];                // SynthMO U^T, feature-contiguous (conflict-free per-thread reads)
    double t2[32];                       // 2^(j/32): tanh_d3's exp table
};

// 16 simultaneous fp64 64-lane sums: after the folds, row R of y[j] holds value j + 4R; lane 16R writes it
__device__ __forceinline__ void wave_sum16_d(const double (&v)[16], double* out) {
    double x[8], y[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = pl32_fold_d(v[i], v[i + 8]);  // rows 0,1: v_i   rows 2,3: v_{i+8}
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = row_sum16_d(pl16_fold_d(x[j], x[j + 4]));  // rows: j, j+4, j+8, j+12
    const int l = threadIdx.x & 63;
    if ((l & 15) == 0) {
        const int R = l >> 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) out[j + 4 * R] = y[j];
    }
}

template <int N_>
__device__ __forceinline__ int sel_lane_i(const int (&v)[N_], int i) {
    int r = 0;
#pragma unroll
    for (int q = 0; q < N_; ++q) r = i == q ? v[q] : r;
    return r;
}

// 17-wide (or any A <= 24) action-mean sums: groups of 8 through wave_sum64_multi
template <int A>
__device__ __forceinline__ void head_sums(const float (&pr)[A], float (&mu)[A]) {
#pragma unroll
    for (int g = 0; g < A; g += 8) {
        constexpr int G = 8;
        float in[G], out[G];
#pragma unroll
        for (int i = 0; i < G; ++i) in[i] = g + i < A ? pr[g + i] : 0.f;
        wave_sum64_multi<G>(in, out);
#pragma unroll
        for (int i = 0; i < G; ++i)
            if (g + i < A) mu[g + i] = out[i];
    }
}

template <int O, int A, int K, int NN>
__global__ __launch_bounds__(WTH) void rollout_wide_kernel(RolloutArgs a) {
    static_assert(wide_fit<O, K, NN>(), "wide rollout envelope");
    static_assert(A <= 32, "action lanes");
    constexpr int KW = wkw<O>(), OR = wrow<O>();
    constexpr int FPL = (O + WTH - 1) / WTH;  // features per lane (thread t: t, t + WTH)
    constexpr int EPW = (NN + WW - 1) / WW;   // env slots per wave (env n on wave n % WW, slot n / WW)
    constexpr int SW = WW - 1;                // statistics wave (fewest features)
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<WideSmem<O, A, K, NN>*>(smem_raw);
    const int p = blockIdx.x, t = threadIdx.x, l = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int T = a.T;
    const NormCfg nc = norm_cfg(a.ns);
    const Layout& L = a.L;
    const float* prm = a.params + (size_t)p * L.total;
    float* obs = a.rb.obs + (size_t)p * (T + 1) * NN * O;
    float* act = a.rb.actions + (size_t)p * T * NN * A;
    float* logp = a.rb.logp + (size_t)p * T * NN;
    float* rew = a.rb.rewards + (size_t)p * T * NN * K;
    float* masks = a.rb.masks + (size_t)p * (T + 1) * NN;
    float* bad = a.rb.bad_masks + (size_t)p * (T + 1) * NN;
    const int maxs = a.spec.max_episode_steps;

    // ---- policy registers: the B operands of this wave's layer-1 MFMAs (v_mfma_f32_16x16x4_f32: lane (j, g) =
    // (l & 15, l >> 4) holds W1^T[k][16 jb + j] for k = w*KW + g*KQ + kk: k-slot g of step kk covers a contiguous
    // KQ-feature run, so the A operand (the env rows) is three float4 LDS reads per lane per 12 steps),
    // the W2 column and head row of unit l
    constexpr int KQ = KW / 4;
    const int lj = l & 15, lg = l >> 4;
    float wb[KQ][4];
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk) {
        const int k = w * KW + lg * KQ + kk;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) wb[kk][jb] = k < O ? prm[L.off[PGM_P_ACTOR_W1] + k * H + 16 * jb + lj] : 0.f;
    }
    float w2[H], wm[A];
#pragma unroll
    for (int k = 0; k < H; ++k) w2[k] = prm[L.off[PGM_P_ACTOR_W2] + k * H + l];
#pragma unroll
    for (int j = 0; j < A; ++j) wm[j] = prm[L.off[PGM_P_MEAN_W] + l * A + j];
    const float b1 = prm[L.off[PGM_P_ACTOR_B1] + l], b2 = prm[L.off[PGM_P_ACTOR_B2] + l];
    const int la = l < A ? l : 0;  // action lane a = l < A
    const float bm_l = prm[L.off[PGM_P_MEAN_B] + la], ls_l = prm[L.off[PGM_P_LOGSTD] + la];
    const float sd_l = expf(ls_l), rsd_l = 1.0f / sd_l;
    const double lo_l = a.spec.act_lo[la], hi_l = a.spec.act_hi[la];

    // ---- feature slots j: feature o = t + WTH*j (< O): env constants, every env's state, ob_rms of o
    // SPL (O - WTH <= 128, e.g. Humanoid's 376 = 256 + 120): the features beyond WTH are split by env halves
    // over lane pairs (l, l + 32) of wave w (feature WTH + 32 w + (l & 31), envs NH (l >> 5) .. + NH - 1), so every
    // thread steps 8 + 4 (feature, env) pairs instead of 16 on half the threads and 8 on the rest; the pair's
    // ob_rms batch moments meet through one lane swap
    constexpr bool SPL = FPL == 2 && O - WTH <= WTH / 2 && NN >= 2;
    constexpr int NH = SPL ? NN / 2 : NN;
    const int hb = l >> 5;
    bool fv[FPL];
    int fo[FPL];
    double V[FPL][K], dd[FPL], cc[FPL], s[FPL][NN], mean[FPL], var[FPL], inv[FPL];
#pragma unroll
    for (int j = 0; j < FPL; ++j) {
        if (SPL && j == 1) {
            const int i1 = w * 32 + (l & 31);
            fv[j] = i1 < O - WTH;
            fo[j] = fv[j] ? WTH + i1 : 0;
        } else {
            fv[j] = t + WTH * j < O;
            fo[j] = fv[j] ? t + WTH * j : 0;
        }
        const int o = fo[j];
#pragma unroll
        for (int k = 0; k < K; ++k) V[j][k] = fv[j] ? a.spec.V[k * O + o] : 0.0;
        dd[j] = fv[j] ? a.spec.d[o] : 0.0;
        cc[j] = fv[j] ? a.spec.c[o] : 0.0;
#pragma unroll
        for (int n = 0; n < NN; ++n) {
            const int ne = SPL && j == 1 ? hb * NH + n : n;
            s[j][n] = fv[j] && (!(SPL && j == 1) || n < NH) ? a.st.s[((size_t)p * NN + ne) * O + o] : 0.0;
        }
        mean[j] = fv[j] ? a.ns.ob_mean[(size_t)p * O + o] : 0.0;
        var[j] = fv[j] ? a.ns.ob_var[(size_t)p * O + o] : 1.0;
        inv[j] = 1.0;
    }
    for (int i = t; i < A * O; i += WTH) {
        const int q = i / O, f = i - q * O;
        S.U[q][f] = a.spec.U[f * A + q];
    }
    if (t < 32) S.t2[t] = exp2((double)t / 32.0);
    double cnt = a.ns.ob_count[p];
    int elapsed[NN];
#pragma unroll
    for (int n = 0; n < NN; ++n) elapsed[n] = a.st.elapsed[p * NN + n];

    // ---- statistics wave: lane i = n*K + k < NN*K (objective accumulator + obj_rms of objective k),
    // lane 32 + n*K (ret of env n + ret_rms): both groups are the lanes of one residue mod K in a 16-lane row,
    // so one set of DPP row rotations forms every batch moment
    const bool olane = w == SW && l < NN * K;
    const bool rlane = w == SW && l >= 32 && l < 32 + NN * K && ((l - 32) % K) == 0;
    const int on = olane ? l / K : 0, ok = olane ? l % K : 0, rn = rlane ? (l - 32) / K : 0;
    double objacc = olane ? a.st.obj_acc[((size_t)p * NN + on) * K + ok] : 0.0;
    double retv = rlane ? a.st.ret[p * NN + rn] : 0.0;
    double smean = 0.0, svar = 1.0, scnt = 1.0, sinv = 1.0;
    if (olane) {
        smean = a.ns.obj_mean[p * K + ok];
        svar = a.ns.obj_var[p * K + ok];
        scnt = a.ns.obj_count[p];
    } else if (rlane) {
        smean = a.ns.ret_mean[p];
        svar = a.ns.ret_var[p];
        scnt = a.ns.ret_count[p];
    }
    int obj_valid = a.st.obj_acc_valid[p];
    const double ebase = a.spec.ebase[ok], ecoef = a.spec.ecoef[ok];

    // ---- slot 0: after_update() carry (storage.py:71-75) and the first policy input
    for (int i = t; i < NN * OR; i += WTH) {
        const int n = i / OR, k = i - n * OR;
        float v = 0.f;
        if (k < O) {
            v = obs[(size_t)(a.carry ? T : 0) * NN * O + n * O + k];
            if (a.carry) obs[n * O + k] = v;
        }
        S.x[n][k] = v;
    }
    if (a.carry && t < NN) {
        masks[t] = masks[(size_t)T * NN + t];
        bad[t] = bad[(size_t)T * NN + t];
    }
    // action noise of this wave's envs in LDS chunks of WNCH steps (as the lane kernel), a chunk ahead in
    // registers
    constexpr int CA = WNCH * A, CR = (CA + 63) / 64;
    float nreg[EPW][CR];
    auto load_eps = [&](int c) {
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = min(w + WW * e, NN - 1);
            size_t idx[CR];
#pragma unroll
            for (int r = 0; r < CR; ++r) {
                const int i = min(64 * r + l, CA - 1);
                const int st = min(c * WNCH + i / A, T - 1), j = i % A;
                idx[r] = ((size_t)st * NN + n) * A + j;
            }
            if (a.noise) {
#pragma unroll
                for (int r = 0; r < CR; ++r) nreg[e][r] = a.noise[idx[r]];
            } else {
#pragma unroll
                for (int r = 0; r < CR; ++r) nreg[e][r] = counter_normal(a.seed, idx[r]);
            }
        }
    };
    auto store_eps = [&](int cb) {
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = w + WW * e;
            if (n >= NN) break;
#pragma unroll
            for (int r = 0; r < CR; ++r)
                if (64 * r + l < CA) S.eps[cb][n][64 * r + l] = nreg[e][r];
        }
    };
    load_eps(0);
    store_eps(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): preamble loads retired before the step loop
    if (WNCH < T) load_eps(1);
    __syncthreads();

    int done_prev[NN];  // done flags of the previous step (the statistics wave runs one step behind)
#pragma unroll
    for (int n = 0; n < NN; ++n) done_prev[n] = 0;

    // statistics of step st (objective sums in objp[par], e2[par]) -> rewards, accumulators, obj/ret_rms
    // sum over the lanes of this lane's residue mod K in its 16-lane row (the batch of one statistic)
    auto group_sum = [&](double v) {
        if constexpr (K <= 8) v += dpp_d<0x128>(v);  // row_ror:8
        if constexpr (K <= 4) v += dpp_d<0x124>(v);
        if constexpr (K <= 2) v += dpp_d<0x122>(v);
        if constexpr (K <= 1) v += dpp_d<0x121>(v);
        return v;
    };
    auto finish_step = [&](int st, int par) {  // wave SW only (wave-uniform call): every lane runs the DPP folds
        double x = 0.0, raw = 0.0;
        if (olane) {
            double sum = 0.0;
#pragma unroll
            for (int ww = 0; ww < WW; ++ww) sum += S.objp[par][ww][l];
            raw = sum + ebase - ecoef * S.e2[par][on];
            objacc = obj_valid ? objacc * nc.gamma + raw : raw;
            x = objacc;
        }
        if (rlane) {  // ret = ret * gamma + 0 (SynthMO's scalar reward)
            retv = retv * nc.gamma + 0.0;
            x = retv;
        }
        const bool mrg = (olane && nc.use_obj) || rlane;  // obj_rms (if used) / ret_rms over the envs
        const double bmean = group_sum(mrg ? x : 0.0) * (1.0 / NN);
        const double bsq = group_sum(mrg ? (x - bmean) * (x - bmean) : 0.0);
        if (mrg) {
            chan_merge_i(smean, svar, scnt, bmean, bsq * (1.0 / NN), (double)NN, rcp_d(scnt + (double)NN));
            scnt += (double)NN;
        }
        if (olane) {
            double r = raw;
            if (nc.use_obj) {
                sinv = rsqrt_d(svar + nc.eps);
                r = clipd(r * sinv, -nc.cliprew, nc.cliprew);
            }
            rew[(size_t)st * NN * K + l] = (float)r;
            if (sel_lane_i(done_prev, on)) objacc = 0.0;
        }
        if (rlane && sel_lane_i(done_prev, rn)) retv = 0.0;
        obj_valid = 1;
    };

    PGM_STAMP_DECL
    for (int step = 0; step < T; ++step) {
        const int par = step & 1;
        const int cs = step % WNCH, cb = (step / WNCH) & 1;
        if (cs == 0 && step > 0) {
            store_eps(cb);
            if (step + WNCH < T) load_eps(step / WNCH + 1);
        }
        // ---- 1. layer-1 partial sums of this wave's k-slice for every env on the f32 matrix cores: rows = envs
        // (16-row tiles, rows >= NN zero), 4 column blocks of 16 units, KQ k-steps; the operands come from
        // registers (W1) and one contiguous LDS run per lane (x), not 64-lane broadcasts of every input
        {
            f32x4 acc[4];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) acc[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
            const bool arow = lj < NN;
            const float* xrow = &S.x[arow ? lj : 0][w * KW + lg * KQ];
#pragma unroll
            for (int q = 0; q < KQ; q += 4) {
                float4 xv = *reinterpret_cast<const float4*>(xrow + q);
                if (!arow) xv = make_float4(0.f, 0.f, 0.f, 0.f);
                const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb)
                        acc[jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[e], wb[q + e][jb], acc[jb], 0, 0, 0);
            }
            // C layout: lane (j, g), register r = Z1[row 4g + r][16 jb + j]
            if (4 * lg < NN) {
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (4 * lg + r < NN) S.zp[w][4 * lg + r][16 * jb + lj] = acc[jb][r];
            }
        }
        PGM_STAMP(0);
        lds_sync();  // A
        PGM_STAMP(1);
        // ---- 2. this wave's envs: layer-1 sum + tanh, layer 2, mean head, Gaussian draw, clipped action
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = w + WW * e;
            if (n >= NN) break;
            float z = b1;
#pragma unroll
            for (int ww = 0; ww < WW; ++ww) z += S.zp[ww][n][l];
            S.h1[n][l] = tanh_fast(z);
        }
        wave_lds_fence_r();
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = w + WW * e;
            if (n >= NN) break;
            f2 a01 = f2{b2, 0.f}, a23 = f2{0.f, 0.f};  // packed fp32 FMAs over unit pairs
#pragma unroll
            for (int k = 0; k < H; k += 4) {
                const float4 hv = *reinterpret_cast<const float4*>(&S.h1[n][k]);
                a01 = __builtin_elementwise_fma(f2{hv.x, hv.y}, f2{w2[k], w2[k + 1]}, a01);
                a23 = __builtin_elementwise_fma(f2{hv.z, hv.w}, f2{w2[k + 2], w2[k + 3]}, a23);
            }
            const float h2 = tanh_fast((a01.x + a01.y) + (a23.x + a23.y));
            float pr[A], mu[A];
#pragma unroll
            for (int j = 0; j < A; ++j) pr[j] = h2 * wm[j];
            head_sums<A>(pr, mu);
            if (l == 0) {
#pragma unroll
                for (int j = 0; j < A; ++j) S.mu[n][j] = mu[j];
            }
        }
        wave_lds_fence_r();
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = w + WW * e;
            if (n >= NN) break;
            const bool al = l < A;
            const float m = S.mu[n][la] + bm_l;
            const float ej = S.eps[cb][n][cs * A + la];
            const float av = fmaf(ej, sd_l, m);
            const float dz = (av - m) * rsd_l;
            const float lpt = al ? -0.5f * dz * dz - ls_l - LOG_SQRT_2PI : 0.f;
            const double acd = clipd_hw((double)av, lo_l, hi_l);
            const float lp = wave_sum64(lpt);
            const double e2 = wave_sum64_d(al ? acd * acd : 0.0);
            if (al) {
                S.ac[n][l] = acd;
                act[((size_t)step * NN + n) * A + l] = av;
            }
            if (l == 0) {
                S.e2[par][n] = e2;
                logp[(size_t)step * NN + n] = lp;
            }
        }
        PGM_STAMP(2);
        lds_sync();  // C
        PGM_STAMP(3);
        // ---- 3. time limit, fp64 dynamics, objective partial sums, auto-reset, ob_rms, normalised obs
        int done[NN];
#pragma unroll
        for (int n = 0; n < NN; ++n) {
            const int el = elapsed[n] + 1;
            done[n] = el >= maxs;
            if (t == 0) {
                masks[(size_t)(step + 1) * NN + n] = done[n] ? 0.f : 1.f;
                bad[(size_t)(step + 1) * NN + n] = (done[n] && el == maxs) ? 0.f : 1.f;
            }
            elapsed[n] = done[n] ? 0 : el;
        }
        {
            double vk[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) vk[i] = 0.0;
            double vk1[NH * K];  // SPL: slot 1's partial sums of its env half (compile-time slots)
#pragma unroll
            for (int i = 0; i < NH * K; ++i) vk1[i] = 0.0;
#pragma unroll
            for (int j = 0; j < FPL; ++j) {
                if (j > 0 && !fv[j]) continue;
                double u[A];  // U row of the feature, once per step; clipped actions are LDS broadcasts
#pragma unroll
                for (int q = 0; q < A; ++q) u[q] = S.U[q][fo[j]];
                const bool half = SPL && j == 1;
#pragma unroll
                for (int n = 0; n < (half ? NH : NN); ++n) {
                    const int ne = half ? hb * NH + n : n;
                    double pu[A];
                    // one compiler fence per feature slot: the action rows are re-read from LDS per (feature, env)
                    // instead of all hoisted into registers, while the envs' dynamics chains (and their tanh table
                    // loads) interleave (a fence per env serialised them: Humanoid 52.9 -> 51.4 ms per iteration)
                    if (n == 0) asm volatile("" ::: "memory");
#pragma unroll
                    for (int q = 0; q < A; ++q) pu[q] = u[q] * S.ac[ne][q];
                    const double sn = tanh_d3(dd[j] * s[j][n] + tree_sum(pu) + cc[j], S.t2);
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        if (half) vk1[n * K + k] = fma(V[j][k], sn, vk1[n * K + k]);
                        else vk[n * K + k] = fma(V[j][k], sn, vk[n * K + k]);
                    }
                    s[j][n] = sn;
                }
            }
            if constexpr (SPL) {
#pragma unroll
                for (int i = 0; i < NH * K; ++i) {
                    vk[i] += hb == 0 ? vk1[i] : 0.0;
                    vk[NH * K + i] += hb == 1 ? vk1[i] : 0.0;
                }
            }
            PGM_STAMP(4);
            wave_sum16_d(vk, &S.objp[par][w][0]);
            PGM_STAMP(5);
        }
        const double itot = rcp_d(cnt + (double)NN);  // shared by every feature's merge of this step
        if constexpr (SPL) {  // slot 1: this lane's env half; the pair's batch moments in fixed (half) order
            constexpr int j = 1;
#pragma unroll
            for (int n = 0; n < NH; ++n) {
                const int dn = hb ? done[NH + n] : done[n];
                if (dn && fv[j]) s[j][n] = a.st.s0[(size_t)(hb * NH + n) * O + fo[j]];  // auto-reset
            }
            if (nc.use_ob) {
                double ls = 0.0;
#pragma unroll
                for (int n = 0; n < NH; ++n) ls += s[j][n];
                const double lo_ = __shfl_xor(ls, 32, 64);
                const double sum = hb == 0 ? ls + lo_ : lo_ + ls;
                const double bmean = sum * (1.0 / NN);
                double lq = 0.0;
#pragma unroll
                for (int n = 0; n < NH; ++n) lq = fma(s[j][n] - bmean, s[j][n] - bmean, lq);
                const double oq = __shfl_xor(lq, 32, 64);
                const double sq = hb == 0 ? lq + oq : oq + lq;
                chan_merge_i(mean[j], var[j], cnt, bmean, sq * (1.0 / NN), (double)NN, itot);
                inv[j] = rsqrt_d(var[j] + nc.eps);
            }
            if (fv[j]) {
#pragma unroll
                for (int n = 0; n < NH; ++n) {
                    double v = s[j][n];
                    if (nc.use_ob) v = clipd((v - mean[j]) * inv[j], -nc.clipob, nc.clipob);
                    const float f = (float)v;  // VecPyTorch .float() (envs.py:192)
                    S.x[hb * NH + n][fo[j]] = f;
                    obs[((size_t)(step + 1) * NN + hb * NH + n) * O + fo[j]] = f;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < (SPL ? 1 : FPL); ++j) {
            if (j > 0 && !fv[j]) continue;
#pragma unroll
            for (int n = 0; n < NN; ++n)
                if (done[n]) s[j][n] = a.st.s0[(size_t)n * O + fo[j]];  // auto-reset (dummy_vec_env.py:45-56)
            if (nc.use_ob) {  // ob_rms.update over the envs of this feature (numpy: divide by N)
                double sum = 0.0;
#pragma unroll
                for (int n = 0; n < NN; ++n) sum += s[j][n];
                const double bmean = sum * (1.0 / NN);
                double sq = 0.0;
#pragma unroll
                for (int n = 0; n < NN; ++n) sq = fma(s[j][n] - bmean, s[j][n] - bmean, sq);
                chan_merge_i(mean[j], var[j], cnt, bmean, sq * (1.0 / NN), (double)NN, itot);
                inv[j] = rsqrt_d(var[j] + nc.eps);
            }
            if (fv[j]) {
#pragma unroll
                for (int n = 0; n < NN; ++n) {
                    double v = s[j][n];
                    if (nc.use_ob) v = clipd((v - mean[j]) * inv[j], -nc.clipob, nc.clipob);
                    const float f = (float)v;  // VecPyTorch .float() (envs.py:192)
                    S.x[n][fo[j]] = f;
                    obs[((size_t)(step + 1) * NN + n) * O + fo[j]] = f;
                }
            }
        }
        if (nc.use_ob) cnt += (double)NN;
        PGM_STAMP(6);
        if (w == SW && step > 0) finish_step(step - 1, par ^ 1);
#pragma unroll
        for (int n = 0; n < NN; ++n) done_prev[n] = done[n];
        lds_sync();  // D
        PGM_STAMP(7);
    }
    PGM_STAMP_FLUSH;
    if (w == SW) finish_step(T - 1, (T - 1) & 1);

    // ---- env state and statistics back to HBM
#pragma unroll
    for (int j = 0; j < FPL; ++j) {
        if (!fv[j]) continue;
        const bool half = SPL && j == 1;
#pragma unroll
        for (int n = 0; n < (half ? NH : NN); ++n)
            a.st.s[((size_t)p * NN + (half ? hb * NH + n : n)) * O + fo[j]] = s[j][n];
        if (!half || hb == 0) {
            a.ns.ob_mean[(size_t)p * O + fo[j]] = mean[j];
            a.ns.ob_var[(size_t)p * O + fo[j]] = var[j];
        }
    }
    if (t == 0) a.ns.ob_count[p] = cnt;
#pragma unroll
    for (int n = 0; n < NN; ++n)
        if (t == n) a.st.elapsed[p * NN + n] = elapsed[n];
    if (olane) {
        a.st.obj_acc[((size_t)p * NN + on) * K + ok] = objacc;
        if (on == 0) {
            a.ns.obj_mean[p * K + ok] = smean;
            a.ns.obj_var[p * K + ok] = svar;
            if (ok == 0) a.ns.obj_count[p] = scnt;
        }
    }
    if (rlane) {
        a.st.ret[p * NN + rn] = retv;
        if (rn == 0) {
            a.ns.ret_mean[p] = smean;
            a.ns.ret_var[p] = svar;
            a.ns.ret_count[p] = scnt;
            a.st.obj_acc_valid[p] = obj_valid;
        }
    }
}

// evaluation() (morl/mopg.py:25-46) for WIDE observations: the eval_num deterministic episodes of a task
// run as the envs of one workgroup with the rollout's step structure (layer 1 on the f32 MFMA over the four
// waves' k-slices, env n's layer 2 / mean head on wave n % 4, feature-slot fp64 dynamics), actions = the
// clipped means, observations normalised in fp64 by the snapshot ob_rms (eps 1e-8, clip 10) and rounded to
// fp32 as the policy input, raw objective sums discounted unless --raw; episodes end at the time limit.
// Objective partial sums of step t are finished during step t + 1 by the statistics wave (lane n*K + k).
template <int O, int A, int K, int NE>
struct WideEvalSmem {
    alignas(16) float x[NE][wrow<O>() + 4];
    alignas(16) float zp[WW][NE][H];
    alignas(16) float h1[NE][H];
    float mu[NE][32];
    double ac[NE][A];
    double e2[2][NE];
    double objp[2][WW][16];
    double U[A][2 * WTH];
    double acc[16];
    double t2[32];
};

template <int O, int A, int K, int NE>
__global__ __launch_bounds__(WTH) void eval_wide_kernel(EvalArgs a) {
    static_assert(O > 48 && O <= 2 * WTH && NE * K <= 16, "wide eval envelope");
    constexpr int KW = wkw<O>(), OR = wrow<O>();
    constexpr int FPL = (O + WTH - 1) / WTH;
    constexpr int EPW = (NE + WW - 1) / WW;
    constexpr int SW = WW - 1;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<WideEvalSmem<O, A, K, NE>*>(smem_raw);
    const int p = blockIdx.x, t = threadIdx.x, l = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const Layout& L = a.L;
    const float* prm = a.params + (size_t)p * L.total;
    const int maxs = a.spec.max_episode_steps;
    const int ne = a.eval_num;  // live episodes (rows >= ne run a copy of episode 0 and are not counted)

    constexpr int KQ = KW / 4;
    const int lj = l & 15, lg = l >> 4;
    float wb[KQ][4];
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk) {
        const int k = w * KW + lg * KQ + kk;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) wb[kk][jb] = k < O ? prm[L.off[PGM_P_ACTOR_W1] + k * H + 16 * jb + lj] : 0.f;
    }
    float w2[H], wm[A];
#pragma unroll
    for (int k = 0; k < H; ++k) w2[k] = prm[L.off[PGM_P_ACTOR_W2] + k * H + l];
#pragma unroll
    for (int j = 0; j < A; ++j) wm[j] = prm[L.off[PGM_P_MEAN_W] + l * A + j];
    const float b1 = prm[L.off[PGM_P_ACTOR_B1] + l], b2 = prm[L.off[PGM_P_ACTOR_B2] + l];
    const int la = l < A ? l : 0;
    const float bm_l = prm[L.off[PGM_P_MEAN_B] + la];
    const double lo_l = a.spec.act_lo[la], hi_l = a.spec.act_hi[la];

    bool fv[FPL];
    int fo[FPL];
    double V[FPL][K], dd[FPL], cc[FPL], s[FPL][NE], mean[FPL], inv[FPL];
#pragma unroll
    for (int j = 0; j < FPL; ++j) {
        fv[j] = t + WTH * j < O;
        fo[j] = fv[j] ? t + WTH * j : 0;
        const int o = fo[j];
#pragma unroll
        for (int k = 0; k < K; ++k) V[j][k] = fv[j] ? a.spec.V[k * O + o] : 0.0;
        dd[j] = fv[j] ? a.spec.d[o] : 0.0;
        cc[j] = fv[j] ? a.spec.c[o] : 0.0;
#pragma unroll
        for (int n = 0; n < NE; ++n) s[j][n] = fv[j] ? a.s0_eval[(size_t)(n < ne ? n : 0) * O + o] : 0.0;
        // mopg.py:37-38: fp64 normalisation with the snapshot ob_rms, fixed eps 1e-8
        mean[j] = a.use_ob && fv[j] ? a.ob_mean[(size_t)p * O + o] : 0.0;
        inv[j] = a.use_ob && fv[j] ? 1.0 / sqrt(a.ob_var[(size_t)p * O + o] + 1e-8) : 1.0;
    }
    for (int i = t; i < A * O; i += WTH) {
        const int q = i / O, f = i - q * O;
        S.U[q][f] = a.spec.U[f * A + q];
    }
    if (t < 32) S.t2[t] = exp2((double)t / 32.0);
    auto norm_x = [&]() {  // normalised fp32 policy inputs of every episode (row padding stays zero)
#pragma unroll
        for (int j = 0; j < FPL; ++j) {
            if (!fv[j]) continue;
#pragma unroll
            for (int n = 0; n < NE; ++n) {
                double v = s[j][n];
                if (a.use_ob) v = clipd((v - mean[j]) * inv[j], -10.0, 10.0);
                S.x[n][fo[j]] = (float)v;
            }
        }
    };
    for (int i = t; i < NE * OR; i += WTH) (&S.x[0][0])[(i / OR) * (OR + 4) + i % OR] = 0.f;
    __syncthreads();
    norm_x();
    // statistics wave: lane n*K + k accumulates episode n's objective k
    const bool olane = w == SW && l < NE * K;
    const int on = olane ? l / K : 0, ok = olane ? l % K : 0;
    const double ebase = a.spec.ebase[ok], ecoef = a.spec.ecoef[ok];
    double acc = 0.0, g = 1.0;
    auto finish_step = [&](int par) {
        if (olane) {
            double sum = 0.0;
#pragma unroll
            for (int ww = 0; ww < WW; ++ww) sum += S.objp[par][ww][l];
            const double raw = sum + ebase - ecoef * S.e2[par][on];
            acc += g * raw;
            if (!a.raw) g *= a.gamma;
        }
    };
    __syncthreads();

    for (int step = 0; step < maxs; ++step) {
        const int par = step & 1;
        {  // 1. layer-1 partial sums of this wave's k-slice (envs on MFMA rows)
            f32x4 z4[4];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) z4[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
            const bool arow = lj < NE;
            const float* xrow = &S.x[arow ? lj : 0][w * KW + lg * KQ];
#pragma unroll
            for (int q = 0; q < KQ; q += 4) {
                float4 xv = *reinterpret_cast<const float4*>(xrow + q);
                if (!arow) xv = make_float4(0.f, 0.f, 0.f, 0.f);
                const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb)
                        z4[jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[e], wb[q + e][jb], z4[jb], 0, 0, 0);
            }
            if (4 * lg < NE) {
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (4 * lg + r < NE) S.zp[w][4 * lg + r][16 * jb + lj] = z4[jb][r];
            }
        }
        lds_sync();  // A
        // 2. this wave's episodes: layer 1 sum + tanh, layer 2, mean head, clipped deterministic action
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = w + WW * e;
            if (n >= NE) break;
            float z = b1;
#pragma unroll
            for (int ww = 0; ww < WW; ++ww) z += S.zp[ww][n][l];
            S.h1[n][l] = tanh_fast(z);
        }
        wave_lds_fence_r();
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = w + WW * e;
            if (n >= NE) break;
            f2 a01 = f2{b2, 0.f}, a23 = f2{0.f, 0.f};
#pragma unroll
            for (int k = 0; k < H; k += 4) {
                const float4 hv = *reinterpret_cast<const float4*>(&S.h1[n][k]);
                a01 = __builtin_elementwise_fma(f2{hv.x, hv.y}, f2{w2[k], w2[k + 1]}, a01);
                a23 = __builtin_elementwise_fma(f2{hv.z, hv.w}, f2{w2[k + 2], w2[k + 3]}, a23);
            }
            const float h2 = tanh_fast((a01.x + a01.y) + (a23.x + a23.y));
            float pr[A], mu[A];
#pragma unroll
            for (int j = 0; j < A; ++j) pr[j] = h2 * wm[j];
            head_sums<A>(pr, mu);
            if (l == 0) {
#pragma unroll
                for (int j = 0; j < A; ++j) S.mu[n][j] = mu[j];
            }
        }
        wave_lds_fence_r();
#pragma unroll
        for (int e = 0; e < EPW; ++e) {
            const int n = w + WW * e;
            if (n >= NE) break;
            const bool al = l < A;
            const double acd = clipd_hw((double)(S.mu[n][la] + bm_l), lo_l, hi_l);
            const double e2 = wave_sum64_d(al ? acd * acd : 0.0);
            if (al) S.ac[n][l] = acd;
            if (l == 0) S.e2[par][n] = e2;
        }
        lds_sync();  // C
        // 3. fp64 dynamics of every episode per feature slot, objective partial sums, next inputs
        {
            double vk[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) vk[i] = 0.0;
#pragma unroll
            for (int j = 0; j < FPL; ++j) {
                if (j > 0 && !fv[j]) continue;
                double u[A];
#pragma unroll
                for (int q = 0; q < A; ++q) u[q] = S.U[q][fo[j]];
#pragma unroll
                for (int n = 0; n < NE; ++n) {
                    if (n == 0) asm volatile("" ::: "memory");  // one fence per feature slot (as in the rollout)
                    double pu[A];
#pragma unroll
                    for (int q = 0; q < A; ++q) pu[q] = u[q] * S.ac[n][q];
                    const double sn = tanh_d3(dd[j] * s[j][n] + tree_sum(pu) + cc[j], S.t2);
#pragma unroll
                    for (int k = 0; k < K; ++k) vk[n * K + k] = fma(V[j][k], sn, vk[n * K + k]);
                    s[j][n] = sn;
                }
            }
            wave_sum16_d(vk, &S.objp[par][w][0]);
        }
        norm_x();
        if (w == SW && step > 0) finish_step(par ^ 1);
        lds_sync();  // D
    }
    if (w == SW) finish_step((maxs - 1) & 1);
    if (olane) S.acc[l] = acc;
    __syncthreads();
    if (t < K) {  // objs /= eval_num, episodes summed in order
        double sum = 0.0;
        for (int n = 0; n < ne; ++n) sum += S.acc[n * K + t];
        a.objs[(size_t)p * K + t] = sum / (double)ne;
    }
}

}  // namespace

bool eval_wide_supported(const pgm_dims* d, int eval_num) {
    return d->O > 48 && d->O <= 2 * WTH && eval_num >= 1 && eval_num <= 8 && eval_num * d->K <= 16 && d->A <= 32;
}

int launch_eval_wide(const pgm_dims* d, const EvalArgs& a, hipStream_t stream) {
    return dispatch_dims(d->O, d->A, d->K, "pgm_eval", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (O <= 48 || O > 2 * WTH || A > 32) {
            set_error("pgm_eval: obs_dim %d outside the wide eval kernel", O);
            return PGM_E_UNSUPPORTED;
        } else {
            auto go = [&](auto kern, size_t smem) -> int {
                if (smem > 160 * 1024) {
                    set_error("pgm_eval: LDS image %zu bytes exceeds 160 KiB", smem);
                    return PGM_E_UNSUPPORTED;
                }
                hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
                if (e != hipSuccess) return hip_fail(e, "pgm_eval");
                hipLaunchKernelGGL(kern, dim3(d->P), dim3(WTH), smem, stream, a);
                return launch_status("pgm_eval");
            };
            const int en = a.eval_num;
            if (en <= 1) return go(eval_wide_kernel<O, A, K, 1>, sizeof(WideEvalSmem<O, A, K, 1>));
            if (en <= 2) return go(eval_wide_kernel<O, A, K, 2>, sizeof(WideEvalSmem<O, A, K, 2>));
            if (en <= 4) return go(eval_wide_kernel<O, A, K, 4>, sizeof(WideEvalSmem<O, A, K, 4>));
            if constexpr (8 * K <= 16) return go(eval_wide_kernel<O, A, K, 8>, sizeof(WideEvalSmem<O, A, K, 8>));
            set_error("pgm_eval: eval_num %d outside the wide eval kernel", en);
            return PGM_E_UNSUPPORTED;
        }
    });
}

bool rollout_wide_supported(const pgm_dims* d) {
    return d->O > 48 && d->O <= 2 * WTH && (d->N == 1 || d->N == 2 || d->N == 4 || d->N == 8) &&
           d->N * d->K <= 16 && (d->K & (d->K - 1)) == 0;
}

template <int O, int A, int K, int NN>
static int launch_wide_n(const pgm_dims* d, const RolloutArgs& a, hipStream_t s) {
    auto kern = rollout_wide_kernel<O, A, K, NN>;
    const size_t smem = sizeof(WideSmem<O, A, K, NN>);
    if (smem > 160 * 1024) {
        set_error("pgm_rollout: LDS image %zu bytes exceeds 160 KiB", smem);
        return PGM_E_UNSUPPORTED;
    }
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return hip_fail(e, "pgm_rollout");
    hipLaunchKernelGGL(kern, dim3(d->P), dim3(WTH), smem, s, a);
    if (int rc = launch_status("pgm_rollout")) return rc;
    return launch_critic_values(d, a, s);
}

int launch_rollout_wide(const pgm_dims* d, const RolloutArgs& a, hipStream_t stream) {
    return dispatch_dims(d->O, d->A, d->K, "pgm_rollout", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (O <= 48 || O > 2 * WTH || (K & (K - 1)) != 0 || A > 32) {
            set_error("pgm_rollout: obs_dim %d outside the wide rollout kernel", O);
            return PGM_E_UNSUPPORTED;
        } else {
            switch (d->N) {
                case 1: return launch_wide_n<O, A, K, 1>(d, a, stream);
                case 2: return launch_wide_n<O, A, K, 2>(d, a, stream);
                case 4: return launch_wide_n<O, A, K, 4>(d, a, stream);
                case 8:
                    if constexpr (8 * K <= 16) return launch_wide_n<O, A, K, 8>(d, a, stream);
                    break;
            }
            set_error("pgm_rollout: N=%d outside the wide rollout kernel (1, 2, 4, 8 with N*K <= 16)", d->N);
            return PGM_E_UNSUPPORTED;
        }
    });
}

}  // namespace pgm
