// Shared pieces of the rollout / evaluation kernels: argument blocks, fp64 VecNormalize helpers and the
// launchers of the lane-parallel kernels (pgm_rollout_lanes.hip) used by the entry points in
// pgm_policy_env.hip.
#pragma once
#include "pgm_common.hpp"

namespace pgm {

constexpr int NMAX = 8;  // envs per task handled by one workgroup
constexpr int RT = 256;  // threads per workgroup of the block-per-task kernels

template <int O>
constexpr int opad() { return (O + 3) & ~3; }

// LDS-only barrier: waits for this wave's LDS traffic, not for its outstanding HBM stores
// (__syncthreads() would also drain vmcnt, i.e. wait for every rollout-storage store).
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// this wave's LDS writes visible to its own lanes
__device__ __forceinline__ void wave_lds_fence_r() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

struct NormCfg {
    double gamma, clipob, cliprew, eps;
    int use_ob, use_obj;
};
__host__ __device__ inline NormCfg norm_cfg(const pgm_norm_state& ns) {
    return NormCfg{ns.gamma, ns.clipob, ns.cliprew, ns.epsilon, ns.use_ob_rms, ns.use_obj_rms};
}

// Chan merge of a batch (bm, bv, n) into (mean, var, count) -- running_mean_std.py:20-31
// (one fp64 division: the reference's three divisions by tot_count become a multiply by 1/tot)
// 1 / x in fp64: hardware reciprocal + two Newton steps (~1 ulp; no IEEE divide sequence on a step chain)
__device__ __forceinline__ double rcp_d(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    return fma(r, fma(-x, r, 1.0), r);
}
// chan_merge with 1 / (count + n) supplied (formed once per step for every statistic that shares the count)
__device__ __forceinline__ void chan_merge_i(double& mean, double& var, double count, double bm, double bv, double n,
                                             double inv_tot) {
    const double delta = bm - mean;
    const double new_mean = mean + delta * n * inv_tot;
    const double m2 = var * count + bv * n + delta * delta * count * n * inv_tot;
    mean = new_mean;
    var = m2 * inv_tot;
}
__device__ __forceinline__ void chan_merge(double& mean, double& var, double count, double bm, double bv, double n) {
    const double delta = bm - mean;
    const double inv_tot = 1.0 / (count + n);
    const double new_mean = mean + delta * n * inv_tot;
    const double m2 = var * count + bv * n + delta * delta * count * n * inv_tot;
    mean = new_mean;
    var = m2 * inv_tot;
}

__device__ __forceinline__ double clipd(double x, double lo, double hi) { return fmin(fmax(x, lo), hi); }
// the same clip as two bare v_max_f64 / v_min_f64: fmin / fmax on values the compiler cannot prove canonical
// (bounds loaded from memory) cost two extra canonicalising v_max_f64 per call inside the step loop
__device__ __forceinline__ double clipd_hw(double x, double lo, double hi) {
    double r;
    asm volatile("v_max_f64 %0, %1, %2\n\tv_min_f64 %0, %0, %3" : "=&v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

// fp64 tanh as expm1(2y) / (expm1(2y) + 2): a few ulp (the env state's precision is fp64, the
// observation leaves as fp32), half the instructions of the double-double libm tanh.  |y| is clamped at
// 20, where tanh is 1 to fp64 precision.
__device__ __forceinline__ double tanh_d(double y) {
    const double e = expm1(2.0 * fmin(fmax(y, -20.0), 20.0));
    return e / (e + 2.0);
}

// pairwise (tree) sum of a short register array: log2(M) dependent adds instead of M
template <class V, int M>
__device__ __forceinline__ V tree_sum(const V (&x)[M]) {
    if constexpr (M == 1) {
        return x[0];
    } else {
        constexpr int H0 = M / 2;
        V lo[H0], hi[M - H0];
#pragma unroll
        for (int i = 0; i < H0; ++i) lo[i] = x[i];
#pragma unroll
        for (int i = 0; i < M - H0; ++i) hi[i] = x[H0 + i];
        return tree_sum(lo) + tree_sum(hi);
    }
}

// Newton steps after the hardware fp64 rcp / rsq estimates on the rollout's step chain.  Measured on gfx950
// (tests/hip/f64_rcp_rsq_probe.hip, profiles/r03d_f64_rcp_rsq_probe.txt): the estimates are good to ~5e-8, one
// step to <= 2.2e-15 (rcp) / 4.3e-15 (rsq) relative, two steps to <= 1.2 ulp.  Two steps: one step measured no
// faster (Walker P = 40 iteration 8.036 vs 8.028 ms, profiles/r03e_*), so the chain keeps full fp64 precision.

// 1 / sqrt(x) in fp64: hardware estimate + two Newton steps (the IEEE sqrt + divide pair is a ~25-instruction
// dependent chain on the per-step critical path)
__device__ __forceinline__ double rsqrt_d(double x) {
    double r = __builtin_amdgcn_rsq(x);
    double e = fma(-x * r, r, 1.0);
    r = fma(r * e, 0.5, r);
    e = fma(-x * r, r, 1.0);
    return fma(r * e, 0.5, r);
}

// fp64 tanh for the SynthMO dynamics: 1 - 2 / (exp(2|y|) + 1) with the sign restored; exp through
// 2^(j/64) table-free range reduction is ocml's, the division is rcp + two Newton steps (~1 ulp).  Absolute
// error ~1e-16 (relative error grows as |y| -> 0, where the state's absolute precision is what matters).
__device__ __forceinline__ double tanh_d2(double y) {
    const double ay = fmin(fabs(y), 20.0);
    const double e = exp(2.0 * ay) + 1.0;
    double r = __builtin_amdgcn_rcp(e);
    r = fma(r, fma(-e, r, 1.0), r);
    r = fma(r, fma(-e, r, 1.0), r);
    return copysign(fma(-2.0, r, 1.0), y);
}

// fp64 tanh with a table-driven exp: exp(x) = 2^m 2^(j/32) p(r), x = (32 m + j) ln2/32 + r, |r| <= ln2/64,
// p = the degree-6 Taylor polynomial (error < 4e-18) in Estrin form (4 dependent steps); t2[j] = 2^(j/32)
// from LDS.  Max |error| vs the IEEE tanh ~3e-16 (host-checked over [-25, 25]) with two Newton steps on the
// reciprocal (~4e-15 with one); about half the dependent fp64 chain of tanh_d2.
__device__ __forceinline__ double tanh_d3(double y, const double* t2) {
    const double x = 2.0 * fmin(fabs(y), 20.0);
    const double kf = __builtin_rint(x * 46.16624130844683);  // 32 / ln 2
    const int k = (int)kf;
    double r = fma(-kf, 0.021660849392496573, x);  // ln2/32, high 42 bits (k ln2/32 exact)
    r = fma(-kf, 1.718100943346366e-15, r);        // ... low part
    const double tj = t2[k & 31];
    const double r2 = r * r;
    const double p = (1.0 + r) + r2 * (fma(r, 1.0 / 6.0, 0.5) + r2 * (fma(r, 1.0 / 120.0, 1.0 / 24.0) + r2 * (1.0 / 720.0)));
    const double e = __builtin_ldexp(tj * p, k >> 5) + 1.0;
    double q = __builtin_amdgcn_rcp(e);
    q = fma(q, fma(-e, q, 1.0), q);
    q = fma(q, fma(-e, q, 1.0), q);
    return copysign(fma(-2.0, q, 1.0), y);
}

// fp64 lane-half / row folds of the transposing multi-value sum (pgm_common.hpp has the fp32 forms)
__device__ __forceinline__ double pl32_fold_d(double a, double b) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double pl16_fold_d(double a, double b) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double row_sum16_d(double v) {
    v += dpp_d<0x128>(v);
    v += dpp_d<0x124>(v);
    v += dpp_d<0x122>(v);
    v += dpp_d<0x121>(v);
    return v;
}
// M <= 4 simultaneous fp64 64-lane sums, results wave-uniform (the fp64 form of wave_sum64_multi): one
// permlane32 fold per pair, one permlane16 fold of the pairs, one 16-lane row sum, one readlane pair per value
template <int M>
__device__ __forceinline__ void wave_sum64_d_multi(const double (&v)[M], double (&out)[M]) {
    static_assert(M >= 1 && M <= 4, "1..4 values");
    if constexpr (M == 1) {
        out[0] = wave_sum64_d(v[0]);
    } else {
        auto at = [&](int i) { return i < M ? v[i] : 0.0; };
        const double r = row_sum16_d(pl16_fold_d(pl32_fold_d(at(0), at(1)), M > 2 ? pl32_fold_d(at(2), at(3)) : 0.0));
        const int lane_of[4] = {0, 32, 16, 48};  // value i sits in row {0, 2, 1, 3}[i]
#pragma unroll
        for (int i = 0; i < M; ++i) out[i] = readlane_d(r, lane_of[i]);
    }
}

template <int N_>
__device__ __forceinline__ float sel_lane(const float (&v)[N_], int l) {
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < N_; ++q) r = l == q ? v[q] : r;
    return r;
}
template <int N_>
__device__ __forceinline__ double sel_lane_d(const double (&v)[N_], int l) {
    double r = 0.0;
#pragma unroll
    for (int q = 0; q < N_; ++q) r = l == q ? v[q] : r;
    return r;
}

struct RolloutArgs {
    int P, N, T;
    Layout L;
    const float* params;
    pgm_env_spec spec;
    pgm_env_state st;
    pgm_norm_state ns;
    pgm_rollout_buf rb;
    const float* noise;
    uint64_t seed;
    int carry;
};

struct EvalArgs {
    int P;
    Layout L;
    const float* params;
    pgm_env_spec spec;
    const double *ob_mean, *ob_var, *s0_eval;
    int eval_num, use_ob, raw;
    double gamma;
    double* objs;
};

// Lane-parallel kernels (pgm_rollout_lanes.hip).  Each returns PGM_E_UNSUPPORTED without launching when
// the dims are outside its envelope (the caller then uses the block-per-task kernel).
int launch_rollout_lanes(const pgm_dims* d, const RolloutArgs& a, hipStream_t stream);
int launch_eval_waves(const pgm_dims* d, const EvalArgs& a, hipStream_t stream);
bool rollout_lanes_supported(const pgm_dims* d);
bool eval_waves_supported(const pgm_dims* d, int eval_num);
// critic values of every stored observation (value_kernel, after an actor-only rollout)
int launch_critic_values(const pgm_dims* d, const RolloutArgs& a, hipStream_t stream);
// wide-observation rollout (pgm_rollout_wide.hip): 48 < obs_dim <= 448, N in {1, 2, 4, 8}, N*K <= 16
bool rollout_wide_supported(const pgm_dims* d);
int launch_rollout_wide(const pgm_dims* d, const RolloutArgs& a, hipStream_t stream);
// wide-observation evaluation (pgm_rollout_wide.hip): 48 < obs_dim <= 512, eval_num <= 8, eval_num*K <= 16
bool eval_wide_supported(const pgm_dims* d, int eval_num);
int launch_eval_wide(const pgm_dims* d, const EvalArgs& a, hipStream_t stream);

}  // namespace pgm
