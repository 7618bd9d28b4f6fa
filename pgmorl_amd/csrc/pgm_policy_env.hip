// Policy forward, synthetic env + VecNormalize, the fused rollout and the deterministic
// evaluation.  One workgroup (256 threads) per task; everything a task touches per step lives
// in LDS (weights, env constants, env state, running statistics, the current obs rows), so a
// T-step rollout is one launch whose steps synchronise with LDS-only barriers: the per-step
// rollout-storage stores to HBM stay in flight across barriers instead of being drained.
//
// Reference semantics (paths relative to the reference tree):
//   Policy.act / get_value                 a2c_ppo_acktr/model.py:57-73, 237-246
//   DiagGaussian sample + log_prob         a2c_ppo_acktr/distributions.py:29-40,71-90
//   DummyVecEnv auto-reset                 baselines/common/vec_env/dummy_vec_env.py:45-56
//   TimeLimitMask bad_transition           a2c_ppo_acktr/envs.py:122-131
//   VecNormalize.step_wait / reset         baselines/common/vec_env/vec_normalize.py:29-66
//   RunningMeanStd Chan merge              baselines/common/running_mean_std.py:3-31
//   masks / bad_masks / obj_tensor         morl/mopg.py:110-130
//   RolloutStorage.insert / after_update   a2c_ppo_acktr/storage.py:50-75
//   evaluation()                           morl/mopg.py:25-46
#include <stdlib.h>

#include "pgm_dispatch.hpp"
#include "pgm_rollout.hpp"

PGM_STAMP_UNIT(rollout)

namespace pgm {


template <int O>
constexpr bool w1_in_lds() { return O <= 128; }
template <int O>
constexpr bool spec_in_lds() { return O <= 128; }


// ------------------------------------------------------------------------------------------
// LDS images
template <int O, int A, int K>
struct PolSmem {
    float bv[K];
    float bm[A];
    float logstd[A];
    alignas(16) float x[NMAX][opad<O>()];   // fp32 policy input rows
    alignas(16) float h1[NMAX][H2];
    float val[NMAX][K];
    float mu[NMAX][A];
    float lp[NMAX][A];
};

template <int O, int A, int K>
struct SpecSmem {  // fp64 env constants (only for O <= 128; Humanoid reads them from HBM/L2)
    static constexpr int OL = spec_in_lds<O>() ? O : 1;
    double U[OL][A], V[K][OL], d[OL], c[OL], s0[NMAX][OL];
    double ebase[K], ecoef[K], lo[A], hi[A];
};

template <int O, int A, int K>
struct EnvSmem {
    SpecSmem<O, A, K> sp;
    double s[NMAX][O];        // env state
    double snew[NMAX][O];     // observation returned by step (post auto-reset)
    double ac[NMAX][A];       // clipped action
    double objraw[NMAX][K];   // info['obj'] before obj_rms scaling
    double obj_acc[NMAX][K];  // VecNormalize.obj
    double ret[NMAX];         // VecNormalize.ret
    double ob_mean[O], ob_var[O], ob_inv[O];
    double obj_mean[K], obj_var[K], obj_inv[K];
    double ob_count, obj_count, ret_mean, ret_var, ret_count;
    double objsum[K];         // evaluation accumulator
    int elapsed[NMAX], done[NMAX], bad[NMAX];
    int obj_valid;
};


// env-constant accessors: LDS copy when it fits, HBM otherwise
template <int O, int A, int K>
struct Spec {
    const EnvSmem<O, A, K>& E;
    const pgm_env_spec& g;
    const double* s0g;
    __device__ double U(int o, int a) const { if constexpr (spec_in_lds<O>()) return E.sp.U[o][a]; else return g.U[o * A + a]; }
    __device__ double V(int k, int o) const { if constexpr (spec_in_lds<O>()) return E.sp.V[k][o]; else return g.V[k * O + o]; }
    __device__ double d(int o) const { if constexpr (spec_in_lds<O>()) return E.sp.d[o]; else return g.d[o]; }
    __device__ double c(int o) const { if constexpr (spec_in_lds<O>()) return E.sp.c[o]; else return g.c[o]; }
    __device__ double s0(int n, int o) const { if constexpr (spec_in_lds<O>()) return E.sp.s0[n][o]; else return s0g[n * O + o]; }
    __device__ double ebase(int k) const { return E.sp.ebase[k]; }
    __device__ double ecoef(int k) const { return E.sp.ecoef[k]; }
    __device__ double lo(int a) const { return E.sp.lo[a]; }
    __device__ double hi(int a) const { return E.sp.hi[a]; }
};

template <int O, int A, int K>
__device__ void load_spec(EnvSmem<O, A, K>& E, const pgm_env_spec& g, const double* s0, int N) {
    const int t = threadIdx.x;
    if constexpr (spec_in_lds<O>()) {
        for (int i = t; i < O * A; i += RT) E.sp.U[i / A][i % A] = g.U[i];
        for (int i = t; i < K * O; i += RT) E.sp.V[i / O][i % O] = g.V[i];
        for (int i = t; i < O; i += RT) {
            E.sp.d[i] = g.d[i];
            E.sp.c[i] = g.c[i];
        }
        for (int i = t; i < N * O; i += RT) E.sp.s0[i / O][i % O] = s0[i];
    }
    if (t < K) {
        E.sp.ebase[t] = g.ebase[t];
        E.sp.ecoef[t] = g.ecoef[t];
    }
    if (t < A) {
        E.sp.lo[t] = g.act_lo[t];
        E.sp.hi[t] = g.act_hi[t];
    }
}

// ------------------------------------------------------------------------------------------
// policy
template <int O, int A, int K>
__device__ void load_policy(PolSmem<O, A, K>& S, const float* __restrict__ prm, const Layout& L) {
    const int t = threadIdx.x;
    if (t < K) S.bv[t] = prm[L.off[PGM_P_VALUE_B] + t];
    if (t < A) {
        S.bm[t] = prm[L.off[PGM_P_MEAN_B] + t];
        S.logstd[t] = prm[L.off[PGM_P_LOGSTD] + t];
    }
}

// Per-thread register image of the weights one lane needs: column c = (tower m, unit j) of both
// tower layers and unit j's head row.  Loaded once per launch (weights are constant inside a rollout).
template <int O>
constexpr bool w1_in_regs() { return O <= 32; }

template <int O, int A, int K>
struct PolReg {
    float w1[w1_in_regs<O>() ? O : 1];
    float w2[H];
    float wh[A > K ? A : K];
    float b1, b2;
};

template <int O, int A, int K>
__device__ void load_polreg(PolReg<O, A, K>& R, const float* __restrict__ prm, const Layout& L) {
    const int t = threadIdx.x, lane = t & 63, m = (t >> 6) & 1;  // m: 0 critic, 1 actor
    const int offW1 = m == 0 ? L.off[PGM_P_CRITIC_W1] : L.off[PGM_P_ACTOR_W1];
    const int offW2 = m == 0 ? L.off[PGM_P_CRITIC_W2] : L.off[PGM_P_ACTOR_W2];
    if constexpr (w1_in_regs<O>()) {
#pragma unroll
        for (int k = 0; k < O; ++k) R.w1[k] = prm[offW1 + k * H + lane];
    }
#pragma unroll
    for (int k = 0; k < H; ++k) R.w2[k] = prm[offW2 + k * H + lane];
    constexpr int NQ = A > K ? A : K;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
        R.wh[q] = m == 0 ? (q < K ? prm[L.off[PGM_P_VALUE_W] + lane * K + q] : 0.f)
                         : (q < A ? prm[L.off[PGM_P_MEAN_W] + lane * A + q] : 0.f);
    R.b1 = prm[(m == 0 ? L.off[PGM_P_CRITIC_B1] : L.off[PGM_P_ACTOR_B1]) + lane];
    R.b2 = prm[(m == 0 ? L.off[PGM_P_CRITIC_B2] : L.off[PGM_P_ACTOR_B2]) + lane];
}

// value [N][K] -> S.val, action mean [N][A] -> S.mu, from S.x.  Wave-local: wave w computes tower
// m = w & 1 for rows r = (w >> 1) + 2i; layer 1 -> layer 2 exchanges h1 inside the wave through LDS
// (no workgroup barrier), the heads are 64-lane butterfly sums of h2 * W_head over the tower's units.
// Ends with one barrier (val/mu visible to every wave).
template <int O, int A, int K>
__device__ void policy_forward(PolSmem<O, A, K>& S, const PolReg<O, A, K>& R, int N, const float* __restrict__ prm,
                               const Layout& L) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, m = w & 1, rg = w >> 1, c = m * H + lane;
    constexpr int RPT = NMAX / 2;
    const float* gw = prm + (m == 0 ? L.off[PGM_P_CRITIC_W1] : L.off[PGM_P_ACTOR_W1]) + lane;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {  // tower layer 1
        const int r = rg + 2 * i;
        if (r < N) {
            float acc = R.b1;
            if constexpr (w1_in_regs<O>()) {
#pragma unroll
                for (int k = 0; k < opad<O>(); k += 4) {
                    const float4 x = *reinterpret_cast<const float4*>(&S.x[r][k]);
                    acc = fmaf(x.x, R.w1[k], acc);
                    if (k + 1 < O) acc = fmaf(x.y, R.w1[k + 1], acc);
                    if (k + 2 < O) acc = fmaf(x.z, R.w1[k + 2], acc);
                    if (k + 3 < O) acc = fmaf(x.w, R.w1[k + 3], acc);
                }
            } else {
#pragma unroll 8
                for (int k = 0; k < O; ++k) acc = fmaf(S.x[r][k], gw[k * H], acc);
            }
            S.h1[r][c] = tanh_f(acc);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // h1 row visible to this wave (lockstep)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < RPT; ++i) {  // tower layer 2 + heads
        const int r = rg + 2 * i;
        if (r < N) {
            float a0 = R.b2, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // four short chains instead of one of 64
#pragma unroll
            for (int k = 0; k < H; k += 4) {
                const float4 h = *reinterpret_cast<const float4*>(&S.h1[r][m * H + k]);
                a0 = fmaf(h.x, R.w2[k], a0);
                a1 = fmaf(h.y, R.w2[k + 1], a1);
                a2 = fmaf(h.z, R.w2[k + 2], a2);
                a3 = fmaf(h.w, R.w2[k + 3], a3);
            }
            const float h2 = tanh_f((a0 + a1) + (a2 + a3));
            if (m == 0) {
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    const float v = wave_sum64(h2 * R.wh[q]);
                    if (lane == 0) S.val[r][q] = v + S.bv[q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < A; ++q) {
                    const float v = wave_sum64(h2 * R.wh[q]);
                    if (lane == 0) S.mu[r][q] = v + S.bm[q];
                }
            }
        }
    }
    lds_sync();
}

// ------------------------------------------------------------------------------------------
// env
template <int O, int A, int K>
__device__ void load_env(EnvSmem<O, A, K>& E, const pgm_env_state& st, const pgm_norm_state& ns, int p, int N) {
    const int t = threadIdx.x;
    for (int i = t; i < N * O; i += RT) E.s[i / O][i % O] = st.s[(size_t)p * N * O + i];
    for (int i = t; i < N * K; i += RT) E.obj_acc[i / K][i % K] = st.obj_acc[(size_t)p * N * K + i];
    if (t < N) {
        E.elapsed[t] = st.elapsed[p * N + t];
        E.ret[t] = st.ret[p * N + t];
    }
    for (int o = t; o < O; o += RT) {
        E.ob_mean[o] = ns.ob_mean[(size_t)p * O + o];
        E.ob_var[o] = ns.ob_var[(size_t)p * O + o];
    }
    if (t < K) {
        E.obj_mean[t] = ns.obj_mean[p * K + t];
        E.obj_var[t] = ns.obj_var[p * K + t];
    }
    if (t == 0) {
        E.ob_count = ns.ob_count[p];
        E.obj_count = ns.obj_count[p];
        E.ret_mean = ns.ret_mean[p];
        E.ret_var = ns.ret_var[p];
        E.ret_count = ns.ret_count[p];
        E.obj_valid = st.obj_acc_valid[p];
    }
}

template <int O, int A, int K>
__device__ void store_env(const EnvSmem<O, A, K>& E, const pgm_env_state& st, const pgm_norm_state& ns, int p, int N) {
    const int t = threadIdx.x;
    for (int i = t; i < N * O; i += RT) st.s[(size_t)p * N * O + i] = E.s[i / O][i % O];
    for (int i = t; i < N * K; i += RT) st.obj_acc[(size_t)p * N * K + i] = E.obj_acc[i / K][i % K];
    if (t < N) {
        st.elapsed[p * N + t] = E.elapsed[t];
        st.ret[p * N + t] = E.ret[t];
    }
    for (int o = t; o < O; o += RT) {
        ns.ob_mean[(size_t)p * O + o] = E.ob_mean[o];
        ns.ob_var[(size_t)p * O + o] = E.ob_var[o];
    }
    if (t < K) {
        ns.obj_mean[p * K + t] = E.obj_mean[t];
        ns.obj_var[p * K + t] = E.obj_var[t];
    }
    if (t == 0) {
        ns.ob_count[p] = E.ob_count;
        ns.obj_count[p] = E.obj_count;
        ns.ret_mean[p] = E.ret_mean;
        ns.ret_var[p] = E.ret_var;
        ns.ret_count[p] = E.ret_count;
        st.obj_acc_valid[p] = E.obj_valid;
    }
}




// s' = tanh(d*s + U a_c + c); objectives; time limit (E.ac filled, E.s current).  Two barriers.
template <int O, int A, int K>
__device__ void env_dynamics(EnvSmem<O, A, K>& E, const Spec<O, A, K>& sp, int N, int max_steps) {
    const int t = threadIdx.x;
    for (int i = t; i < N * O; i += RT) {
        const int n = i / O, o = i % O;
        double ua = 0.0;
#pragma unroll
        for (int a = 0; a < A; ++a) ua += sp.U(o, a) * E.ac[n][a];
        E.snew[n][o] = tanh_d(sp.d(o) * E.s[n][o] + ua + sp.c(o));
    }
    lds_sync();
    for (int i = t; i < N * K; i += RT) {
        const int n = i / K, k = i % K;
        double v = 0.0, e2 = 0.0;
        for (int o = 0; o < O; ++o) v += sp.V(k, o) * E.snew[n][o];
#pragma unroll
        for (int a = 0; a < A; ++a) e2 += E.ac[n][a] * E.ac[n][a];
        E.objraw[n][k] = v + sp.ebase(k) - sp.ecoef(k) * e2;
    }
    if (t >= RT - N) {
        const int n = t - (RT - N);
        const int el = E.elapsed[n] + 1;
        const int d = el >= max_steps;
        E.done[n] = d;
        E.bad[n] = d && (el == max_steps);
        E.elapsed[n] = d ? 0 : el;
    }
    lds_sync();
}

// Auto-reset + VecNormalize statistics: ob_rms on feature threads (bottom of the block), obj
// accumulators + obj_rms on objective threads (top), ret_rms on one thread; all with the counts
// from before this step (they advance in vecnorm_emit).  One barrier.
template <int O, int A, int K>
__device__ void vecnorm_stats(EnvSmem<O, A, K>& E, const Spec<O, A, K>& sp, int N, const NormCfg& nc) {
    const int t = threadIdx.x;
    const double dn = (double)N;
    // numpy's x.mean(0) / x.var(0) divide by N; for N a power of two the reciprocal is exact
    const bool pow2 = (N & (N - 1)) == 0;
    const double rn = 1.0 / dn;
    auto divn = [&](double x) { return pow2 ? x * rn : x / dn; };
    for (int o = t; o < O; o += RT) {
        double sum = 0.0;
        for (int n = 0; n < N; ++n) {
            const double v = E.done[n] ? sp.s0(n, o) : E.snew[n][o];
            E.snew[n][o] = v;
            E.s[n][o] = v;
            sum += v;
        }
        if (nc.use_ob) {
            const double bm = divn(sum);
            double sq = 0.0;
            for (int n = 0; n < N; ++n) {
                const double dd = E.snew[n][o] - bm;
                sq += dd * dd;
            }
            chan_merge(E.ob_mean[o], E.ob_var[o], E.ob_count, bm, divn(sq), dn);
            E.ob_inv[o] = 1.0 / sqrt(E.ob_var[o] + nc.eps);
        }
    }
    const int k = RT - 1 - t;
    if (k < K) {
        for (int n = 0; n < N; ++n)
            E.obj_acc[n][k] = E.obj_valid ? E.obj_acc[n][k] * nc.gamma + E.objraw[n][k] : E.objraw[n][k];
        if (nc.use_obj) {
            double sum = 0.0;
            for (int n = 0; n < N; ++n) sum += E.obj_acc[n][k];
            const double bm = divn(sum);
            double sq = 0.0;
            for (int n = 0; n < N; ++n) {
                const double dd = E.obj_acc[n][k] - bm;
                sq += dd * dd;
            }
            chan_merge(E.obj_mean[k], E.obj_var[k], E.obj_count, bm, divn(sq), dn);
            E.obj_inv[k] = 1.0 / sqrt(E.obj_var[k] + nc.eps);
        }
    }
    if (t == RT - 1 - K) {  // ret_rms on the (always zero-reward) discounted return, vec_normalize.py:32,41-43
        double sum = 0.0;
        for (int n = 0; n < N; ++n) {
            E.ret[n] = E.ret[n] * nc.gamma + 0.0;
            sum += E.ret[n];
        }
        const double bm = divn(sum);
        double sq = 0.0;
        for (int n = 0; n < N; ++n) sq += (E.ret[n] - bm) * (E.ret[n] - bm);
        chan_merge(E.ret_mean, E.ret_var, E.ret_count, bm, divn(sq), dn);
        E.ret_count += dn;
    }
    lds_sync();
}

// Normalised fp32 obs (-> xs rows and obs_out), scaled objectives, masks; zero the accumulators of
// done envs; advance the counts.  One barrier.
template <int O, int A, int K, int XS>
__device__ void vecnorm_emit(EnvSmem<O, A, K>& E, int N, const NormCfg& nc, float (*xs)[XS], float* obs_out,
                             float* rew_out, float* mask_out, float* bad_out) {
    const int t = threadIdx.x;
    for (int i = t; i < N * O; i += RT) {
        const int n = i / O, o = i % O;
        double v = E.snew[n][o];
        if (nc.use_ob) v = clipd((v - E.ob_mean[o]) * E.ob_inv[o], -nc.clipob, nc.clipob);
        const float f = (float)v;  // VecPyTorch .float() (envs.py:192)
        xs[n][o] = f;
        if (obs_out) obs_out[i] = f;
    }
    const int i = RT - 1 - t;
    if (i < N * K) {
        const int n = i / K, k = i % K;
        double r = E.objraw[n][k];
        if (nc.use_obj) r = clipd(r * E.obj_inv[k], -nc.cliprew, nc.cliprew);
        if (rew_out) rew_out[i] = (float)r;
        if (E.done[n]) E.obj_acc[n][k] = 0.0;
    }
    const int n = RT - 1 - N * K - t;
    if (n >= 0 && n < N) {
        if (mask_out) mask_out[n] = E.done[n] ? 0.f : 1.f;
        if (bad_out) bad_out[n] = E.bad[n] ? 0.f : 1.f;
        if (E.done[n]) E.ret[n] = 0.0;
    }
    if (t == 0) {
        if (nc.use_ob) E.ob_count += (double)N;
        if (nc.use_obj) E.obj_count += (double)N;
        E.obj_valid = 1;
    }
    lds_sync();
}

// Draw actions (torch.normal(mean, std) = z*std + mean), log-prob terms, clipped env action.
template <int O, int A, int K>
__device__ void sample_actions(PolSmem<O, A, K>& P, EnvSmem<O, A, K>& E, const Spec<O, A, K>& sp, int N, float eps,
                               float* act_out) {
    const int t = threadIdx.x;
    if (t < N * A) {
        const int n = t / A, j = t % A;
        const float mu = P.mu[n][j], ls = P.logstd[j], sd = expf(ls);
        const float av = fmaf(eps, sd, mu);
        const float dz = (av - mu) / sd;
        P.lp[n][j] = -0.5f * dz * dz - ls - LOG_SQRT_2PI;
        if (act_out) act_out[t] = av;
        E.ac[n][j] = clipd((double)av, sp.lo(j), sp.hi(j));
    }
    lds_sync();
}

// ------------------------------------------------------------------------------------------
// kernels
template <int O, int A, int K>
struct StepSmem {
    PolSmem<O, A, K> pol;
    EnvSmem<O, A, K> env;
};

struct ActArgs {
    int P, N;
    Layout L;
    const float* params;
    const float* obs;
    const float* noise;
    int deterministic;
    float *value, *action, *logp;
};

template <int O, int A, int K>
__global__ __launch_bounds__(RT) void act_forward_kernel(ActArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<PolSmem<O, A, K>*>(smem_raw);
    const int p = blockIdx.x, t = threadIdx.x, N = a.N;
    const float* prm = a.params + (size_t)p * a.L.total;
    PolReg<O, A, K> R;
    load_policy(S, prm, a.L);
    load_polreg(R, prm, a.L);
    for (int i = t; i < N * O; i += RT) S.x[i / O][i % O] = a.obs[(size_t)p * N * O + i];
    __syncthreads();
    policy_forward(S, R, N, prm, a.L);
    for (int i = t; i < N * K; i += RT) a.value[(size_t)p * N * K + i] = S.val[i / K][i % K];
    for (int i = t; i < N * A; i += RT) {
        const int n = i / A, j = i % A;
        const float mu = S.mu[n][j], ls = S.logstd[j], sd = expf(ls);
        const float act = a.deterministic ? mu : fmaf(a.noise[i], sd, mu);
        const float dz = (act - mu) / sd;
        S.lp[n][j] = -0.5f * dz * dz - ls - LOG_SQRT_2PI;
        a.action[(size_t)p * N * A + i] = act;
    }
    __syncthreads();
    if (t < N) {
        float s = 0.f;
        for (int j = 0; j < A; ++j) s += S.lp[t][j];
        a.logp[(size_t)p * N + t] = s;
    }
}

struct EnvArgs {
    int P, N;
    pgm_env_spec spec;
    pgm_env_state st;
    pgm_norm_state ns;
    const float* action;
    float *obs_out, *rew_out, *mask_out, *bad_out;
    int reset;
};

template <int O, int A, int K>
__global__ __launch_bounds__(RT) void env_kernel(EnvArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<StepSmem<O, A, K>*>(smem_raw);
    auto& E = S.env;
    const int p = blockIdx.x, t = threadIdx.x, N = a.N;
    const NormCfg nc = norm_cfg(a.ns);
    const Spec<O, A, K> sp{E, a.spec, a.st.s0};
    load_spec(E, a.spec, a.st.s0, N);
    load_env(E, a.st, a.ns, p, N);
    __syncthreads();
    if (a.reset) {  // fresh make_vec_envs + reset(): vec_normalize.py:10-27,63-66
        if (t < N) {
            E.elapsed[t] = 0;
            E.ret[t] = 0.0;
        }
        if (t == 0) E.obj_valid = 0;
        const double dn = (double)N;
        for (int o = t; o < O; o += RT) {
            double sum = 0.0;
            for (int n = 0; n < N; ++n) {
                const double v = sp.s0(n, o);
                E.snew[n][o] = v;
                E.s[n][o] = v;
                sum += v;
            }
            if (nc.use_ob) {
                const double bm = sum / dn;
                double sq = 0.0;
                for (int n = 0; n < N; ++n) sq += (E.snew[n][o] - bm) * (E.snew[n][o] - bm);
                chan_merge(E.ob_mean[o], E.ob_var[o], E.ob_count, bm, sq / dn, dn);
                E.ob_inv[o] = 1.0 / sqrt(E.ob_var[o] + nc.eps);
            }
        }
        __syncthreads();
        if (t == 0 && nc.use_ob) E.ob_count += dn;
        for (int i = t; i < N * O; i += RT) {
            const int o = i % O;
            double v = E.snew[i / O][o];
            if (nc.use_ob) v = clipd((v - E.ob_mean[o]) * E.ob_inv[o], -nc.clipob, nc.clipob);
            a.obs_out[(size_t)p * N * O + i] = (float)v;
        }
    } else {
        for (int i = t; i < N * A; i += RT) {
            const int j = i % A;
            E.ac[i / A][j] = clipd((double)a.action[(size_t)p * N * A + i], sp.lo(j), sp.hi(j));
        }
        __syncthreads();
        env_dynamics(E, sp, N, a.spec.max_episode_steps);
        vecnorm_stats(E, sp, N, nc);
        vecnorm_emit<O, A, K, opad<O>()>(E, N, nc, S.pol.x, a.obs_out + (size_t)p * N * O,
                                         a.rew_out + (size_t)p * N * K, a.mask_out + (size_t)p * N,
                                         a.bad_out + (size_t)p * N);
    }
    __syncthreads();
    store_env(E, a.st, a.ns, p, N);
}


template <int O, int A, int K>
__global__ __launch_bounds__(RT) void rollout_kernel(RolloutArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<StepSmem<O, A, K>*>(smem_raw);
    auto& P = S.pol;
    auto& E = S.env;
    const int p = blockIdx.x, t = threadIdx.x, N = a.N, T = a.T;
    const NormCfg nc = norm_cfg(a.ns);
    const Spec<O, A, K> sp{E, a.spec, a.st.s0};
    const float* prm = a.params + (size_t)p * a.L.total;
    float* obs = a.rb.obs + (size_t)p * (T + 1) * N * O;
    float* act = a.rb.actions + (size_t)p * T * N * A;
    float* logp = a.rb.logp + (size_t)p * T * N;
    float* val = a.rb.values + (size_t)p * (T + 1) * N * K;
    float* rew = a.rb.rewards + (size_t)p * T * N * K;
    float* masks = a.rb.masks + (size_t)p * (T + 1) * N;
    float* bad = a.rb.bad_masks + (size_t)p * (T + 1) * N;

    PolReg<O, A, K> R;
    load_policy(P, prm, a.L);
    load_polreg(R, prm, a.L);
    load_spec(E, a.spec, a.st.s0, N);
    load_env(E, a.st, a.ns, p, N);
    if (a.carry) {  // after_update(): slot T -> slot 0 (storage.py:71-75); each thread re-reads its own writes
        for (int i = t; i < N * O; i += RT) obs[i] = obs[(size_t)T * N * O + i];
        if (t < N) {
            masks[t] = masks[(size_t)T * N + t];
            bad[t] = bad[(size_t)T * N + t];
        }
    }
    for (int i = t; i < N * O; i += RT) P.x[i / O][i % O] = obs[i];
    __syncthreads();

    // the lane drawing (n, a) of each step keeps its noise one step ahead in a register
    const bool drawer = t < N * A;
    float eps_next = 0.f;
    if (drawer) eps_next = a.noise ? a.noise[t] : counter_normal(a.seed, (uint64_t)t);
    PGM_STAMP_DECL
    for (int step = 0; step < T; ++step) {
        const float eps = eps_next;
        if (drawer && step + 1 < T) {
            const size_t idx = (size_t)(step + 1) * N * A + t;
            eps_next = a.noise ? a.noise[idx] : counter_normal(a.seed, idx);
        }
        PGM_STAMP(0);
        policy_forward(P, R, N, prm, a.L);
        PGM_STAMP(1);
        for (int i = t; i < N * K; i += RT) val[(size_t)step * N * K + i] = P.val[i / K][i % K];
        sample_actions(P, E, sp, N, eps, act + (size_t)step * N * A);
        PGM_STAMP(2);
        if (t < N) {
            float s = 0.f;
            for (int j = 0; j < A; ++j) s += P.lp[t][j];
            logp[(size_t)step * N + t] = s;
        }
        env_dynamics(E, sp, N, a.spec.max_episode_steps);
        PGM_STAMP(3);
        vecnorm_stats(E, sp, N, nc);
        PGM_STAMP(4);
        vecnorm_emit<O, A, K, opad<O>()>(E, N, nc, P.x, obs + (size_t)(step + 1) * N * O,
                                         rew + (size_t)step * N * K, masks + (size_t)(step + 1) * N,
                                         bad + (size_t)(step + 1) * N);
        PGM_STAMP(5);
    }
    // bootstrap value (mopg.py:132-135) -> value_preds[T] (storage.py:85)
    policy_forward(P, R, N, prm, a.L);
    for (int i = t; i < N * K; i += RT) val[(size_t)T * N * K + i] = P.val[i / K][i % K];
    __syncthreads();
    store_env(E, a.st, a.ns, p, N);
    PGM_STAMP_FLUSH;
}

template <int O, int A, int K>
__global__ __launch_bounds__(RT) void eval_kernel(EvalArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<StepSmem<O, A, K>*>(smem_raw);
    auto& P = S.pol;
    auto& E = S.env;
    const int p = blockIdx.x, t = threadIdx.x;
    const float* prm = a.params + (size_t)p * a.L.total;
    PolReg<O, A, K> R;
    load_policy(P, prm, a.L);
    load_polreg(R, prm, a.L);
    load_spec(E, a.spec, a.s0_eval, 1);
    for (int o = t; o < O; o += RT) {  // mopg.py:37-38: fp64 normalisation with fixed eps/clip
        E.ob_mean[o] = a.use_ob ? a.ob_mean[(size_t)p * O + o] : 0.0;
        E.ob_inv[o] = a.use_ob ? 1.0 / sqrt(a.ob_var[(size_t)p * O + o] + 1e-8) : 1.0;
    }
    if (t < K) E.objsum[t] = 0.0;
    __syncthreads();
    for (int e = 0; e < a.eval_num; ++e) {
        const double* s0 = a.s0_eval + (size_t)e * O;
        const Spec<O, A, K> sp{E, a.spec, s0};
        for (int o = t; o < O; o += RT) E.s[0][o] = s0[o];
        if (t == 0) E.elapsed[0] = 0;
        double g = 1.0;
        __syncthreads();
        while (true) {
            for (int o = t; o < O; o += RT) {  // obs is NOT rounded through fp32 before normalising
                double v = E.s[0][o];
                if (a.use_ob) v = clipd((v - E.ob_mean[o]) * E.ob_inv[o], -10.0, 10.0);
                P.x[0][o] = (float)v;
            }
            lds_sync();
            policy_forward(P, R, 1, prm, a.L);
            if (t < A) E.ac[0][t] = clipd((double)P.mu[0][t], sp.lo(t), sp.hi(t));
            lds_sync();
            env_dynamics(E, sp, 1, a.spec.max_episode_steps);
            if (t < K) E.objsum[t] += g * E.objraw[0][t];
            if (!a.raw) g *= a.gamma;
            const int done = E.done[0];
            for (int o = t; o < O; o += RT) E.s[0][o] = E.snew[0][o];
            lds_sync();
            if (done) break;
        }
    }
    if (t < K) a.objs[(size_t)p * K + t] = E.objsum[t] / (double)a.eval_num;
}

// ------------------------------------------------------------------------------------------
template <class Kern, class Args>
static int launch_smem(Kern k, int grid, size_t smem, hipStream_t s, const Args& args, const char* what) {
    if (smem > 160 * 1024) {
        set_error("%s: LDS image %zu bytes exceeds 160 KiB", what, smem);
        return PGM_E_UNSUPPORTED;
    }
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return hip_fail(e, what);
    hipLaunchKernelGGL(k, dim3(grid), dim3(RT), smem, s, args);
    return launch_status(what);
}

static bool spec_ok(const pgm_env_spec* sp) {
    return sp && sp->d && sp->U && sp->c && sp->V && sp->ebase && sp->ecoef && sp->act_lo && sp->act_hi &&
           sp->max_episode_steps > 0;
}
static bool state_ok(const pgm_env_state* st) {
    return st && st->s && st->elapsed && st->obj_acc && st->obj_acc_valid && st->ret && st->s0;
}
static bool norm_ok(const pgm_norm_state* ns) {
    return ns && ns->ob_mean && ns->ob_var && ns->ob_count && ns->ret_mean && ns->ret_var && ns->ret_count &&
           ns->obj_mean && ns->obj_var && ns->obj_count;
}

}  // namespace pgm

using namespace pgm;

extern "C" {

int pgm_act_forward(const pgm_dims* d, const float* params, const float* obs, const float* noise,
                    int32_t deterministic, float* value, float* action, float* logp, pgm_stream_t stream) {
    if (int rc = check_dims(d, "pgm_act_forward")) return rc;
    if (!params || !obs || !value || !action || !logp || (!deterministic && !noise)) {
        set_error("pgm_act_forward: null pointer (noise is required unless deterministic)");
        return PGM_E_INVALID_ARG;
    }
    ActArgs a{d->P, d->N, make_layout(d->O, d->A, d->K, d->H), params, obs, noise, deterministic, value, action, logp};
    return dispatch_dims(d->O, d->A, d->K, "pgm_act_forward", [&](auto o, auto aa, auto k) {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        return launch_smem(act_forward_kernel<O, A, K>, d->P, sizeof(PolSmem<O, A, K>), (hipStream_t)stream, a,
                           "pgm_act_forward");
    });
}

static int env_common(const pgm_dims* d, const pgm_env_spec* spec, const pgm_env_state* st,
                      const pgm_norm_state* ns, const char* what) {
    if (int rc = check_dims(d, what)) return rc;
    if (!spec_ok(spec) || !state_ok(st) || !norm_ok(ns)) {
        set_error("%s: null pointer in spec/state/norm structs", what);
        return PGM_E_INVALID_ARG;
    }
    return PGM_OK;
}

int pgm_env_reset(const pgm_dims* d, const pgm_env_spec* spec, const pgm_env_state* st,
                  const pgm_norm_state* ns, float* obs_out, pgm_stream_t stream) {
    if (int rc = env_common(d, spec, st, ns, "pgm_env_reset")) return rc;
    if (!obs_out) {
        set_error("pgm_env_reset: null obs_out");
        return PGM_E_INVALID_ARG;
    }
    EnvArgs a{d->P, d->N, *spec, *st, *ns, nullptr, obs_out, nullptr, nullptr, nullptr, 1};
    return dispatch_dims(d->O, d->A, d->K, "pgm_env_reset", [&](auto o, auto aa, auto k) {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        return launch_smem(env_kernel<O, A, K>, d->P, sizeof(StepSmem<O, A, K>), (hipStream_t)stream, a,
                           "pgm_env_reset");
    });
}

int pgm_env_step(const pgm_dims* d, const pgm_env_spec* spec, const pgm_env_state* st,
                 const pgm_norm_state* ns, const float* action, float* obs_out, float* reward_out,
                 float* masks_out, float* bad_masks_out, pgm_stream_t stream) {
    if (int rc = env_common(d, spec, st, ns, "pgm_env_step")) return rc;
    if (!action || !obs_out || !reward_out || !masks_out || !bad_masks_out) {
        set_error("pgm_env_step: null pointer");
        return PGM_E_INVALID_ARG;
    }
    EnvArgs a{d->P, d->N, *spec, *st, *ns, action, obs_out, reward_out, masks_out, bad_masks_out, 0};
    return dispatch_dims(d->O, d->A, d->K, "pgm_env_step", [&](auto o, auto aa, auto k) {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        return launch_smem(env_kernel<O, A, K>, d->P, sizeof(StepSmem<O, A, K>), (hipStream_t)stream, a,
                           "pgm_env_step");
    });
}

int pgm_rollout(const pgm_dims* d, const float* params, const pgm_env_spec* spec, const pgm_env_state* st,
                const pgm_norm_state* ns, const pgm_rollout_buf* rb, const float* noise, uint64_t seed,
                int32_t carry, const pgm_launch_opts* opts, pgm_stream_t stream) {
    if (int rc = env_common(d, spec, st, ns, "pgm_rollout")) return rc;
    pgm_launch_opts o;
    if (int rc = read_opts(opts, &o, "pgm_rollout")) return rc;
    if (!params || !rb || !rb->obs || !rb->actions || !rb->logp || !rb->values || !rb->rewards || !rb->masks ||
        !rb->bad_masks) {
        set_error("pgm_rollout: null pointer");
        return PGM_E_INVALID_ARG;
    }
    if (d->T <= 0) {
        set_error("pgm_rollout: T must be positive");
        return PGM_E_SHAPE;
    }
    RolloutArgs a{d->P, d->N, d->T, make_layout(d->O, d->A, d->K, d->H), params, *spec, *st, *ns, *rb,
                  noise, seed, carry};
    const bool block = o.rollout_kernel == 1;  // the workgroup-per-step kernel (A/B, tests)
    if (!block && rollout_lanes_supported(d)) return launch_rollout_lanes(d, a, (hipStream_t)stream);
    if (!block && rollout_wide_supported(d)) return launch_rollout_wide(d, a, (hipStream_t)stream);
    return dispatch_dims(d->O, d->A, d->K, "pgm_rollout", [&](auto o, auto aa, auto k) {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        return launch_smem(rollout_kernel<O, A, K>, d->P, sizeof(StepSmem<O, A, K>), (hipStream_t)stream, a,
                           "pgm_rollout");
    });
}

int pgm_eval(const pgm_dims* d, const float* params, const pgm_env_spec* spec, const double* ob_mean,
             const double* ob_var, const double* s0_eval, int32_t eval_num, int32_t use_ob_rms, int32_t raw,
             double gamma, double* objs_out, const pgm_launch_opts* opts, pgm_stream_t stream) {
    if (int rc = check_dims(d, "pgm_eval")) return rc;
    pgm_launch_opts o;
    if (int rc = read_opts(opts, &o, "pgm_eval")) return rc;
    if (!params || !spec_ok(spec) || !s0_eval || !objs_out || eval_num <= 0 || (use_ob_rms && (!ob_mean || !ob_var))) {
        set_error("pgm_eval: bad arguments");
        return PGM_E_INVALID_ARG;
    }
    EvalArgs a{d->P, make_layout(d->O, d->A, d->K, d->H), params, *spec, ob_mean, ob_var, s0_eval,
               eval_num, use_ob_rms, raw, gamma, objs_out};
    const bool block = o.eval_kernel == 1;  // the workgroup-per-step kernel (A/B, tests)
    if (!block && eval_waves_supported(d, eval_num)) return launch_eval_waves(d, a, (hipStream_t)stream);
    if (!block && eval_wide_supported(d, eval_num)) return launch_eval_wide(d, a, (hipStream_t)stream);
    return dispatch_dims(d->O, d->A, d->K, "pgm_eval", [&](auto o, auto aa, auto k) {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        return launch_smem(eval_kernel<O, A, K>, d->P, sizeof(StepSmem<O, A, K>), (hipStream_t)stream, a,
                           "pgm_eval");
    });
}

}  // extern "C"
