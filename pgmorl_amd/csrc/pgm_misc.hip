// Return sweep (GAE), advantage scalarisation + normalisation, and the perf-mode RNG streams.
//
// Reference semantics:
//   RolloutStorage.compute_returns          a2c_ppo_acktr/storage.py:77-116
//   PPO.update advantage prologue           a2c_ppo_acktr/algo/ppo.py:41-56
//   WeightedSumScalarization.evaluate       morl/scalarization_methods.py:28-29
//   SubsetRandomSampler randperm / Normal.sample draws (replaced by counter-based streams in perf mode)
#include "pgm_dispatch.hpp"

namespace pgm {

// ------------------------------------------------------------------------------------------
// GAE / returns.  Every (env n, objective k) lane obeys the affine reverse recurrence
//     y_t = A_t * y_{t+1} + B_t,       R_t = y_t + (use_gae ? V_t : 0)
//   use_gae:  A_t = g*lam*m_{t+1}*(b_{t+1} if proper), B_t = delta_t*(b_{t+1} if proper), y_T = 0
//             delta_t = r_t + g*V_{t+1}*m_{t+1} - V_t
//   !use_gae: A_t = g*m_{t+1}*(b_{t+1} if proper), B_t = r_t*b + (1-b)*V_t (proper) or r_t, y_T = V_T
// Split T into C chunks per lane: pass 1 composes each chunk's affine map, a per-lane sweep over
// the C chunk maps gives every chunk's incoming y, pass 2 re-walks the chunk and writes R.
constexpr int GT = 1024;  // threads per task: N*K lanes x GT/(N*K) chunks (Walker: 128 chunks of 16 steps)

struct GaeArgs {
    int N, T, K;
    const float *rew, *val, *mask, *bad;
    float* ret;
    float gamma, lam;
    int use_gae, proper;
};

__device__ __forceinline__ void gae_coef(const GaeArgs& a, const float* rew, const float* val, const float* mask,
                                         const float* bad, int t, int n, int k, double& A, double& B) {
    const int N = a.N, K = a.K;
    const double r = rew[((size_t)t * N + n) * K + k];
    const double v = val[((size_t)t * N + n) * K + k];
    const double v1 = val[((size_t)(t + 1) * N + n) * K + k];
    const double m1 = mask[(size_t)(t + 1) * N + n];
    const double b1 = bad[(size_t)(t + 1) * N + n];
    const double g = a.gamma;
    if (a.use_gae) {
        const double delta = r + g * v1 * m1 - v;
        A = g * (double)a.lam * m1;
        B = delta;
        if (a.proper) {
            A *= b1;
            B *= b1;
        }
    } else {
        A = g * m1;
        B = r;
        if (a.proper) {
            A *= b1;
            B = r * b1 + (1.0 - b1) * v;
        }
    }
}

__global__ __launch_bounds__(GT) void gae_kernel(GaeArgs a) {
    __shared__ double yin[GT];
    const int p = blockIdx.x, t = threadIdx.x, N = a.N, T = a.T, K = a.K;
    const int lanes = N * K;
    const int C = GT / lanes;                 // chunks per lane (>= 1: N*K <= 64 checked on host)
    const int len = (T + C - 1) / C;
    const int lane = t % lanes, ch = t / lanes;
    const bool active = ch < C;
    const int n = lane / K, k = lane % K;
    const float* rew = a.rew + (size_t)p * T * N * K;
    const float* val = a.val + (size_t)p * (T + 1) * N * K;
    const float* mask = a.mask + (size_t)p * (T + 1) * N;
    const float* bad = a.bad + (size_t)p * (T + 1) * N;
    float* ret = a.ret + (size_t)p * (T + 1) * N * K;
    const int t0 = ch * len, t1 = min(T, t0 + len);
    double cA = 1.0, cB = 0.0;  // y_{t0} = cA * y_{t1} + cB
    if (active) {
        for (int s = t1 - 1; s >= t0; --s) {
            double A, B;
            gae_coef(a, rew, val, mask, bad, s, n, k, A, B);
            cB = A * cB + B;
            cA = A * cA;
        }
    }
    __shared__ double mapA[GT], mapB[GT];
    mapA[t] = cA;
    mapB[t] = cB;
    __syncthreads();
    if (t < lanes) {  // sequential sweep over the chunk maps of this lane
        double y = a.use_gae ? 0.0 : (double)val[(size_t)T * N * K + lane];
        for (int c = C - 1; c >= 0; --c) {
            yin[c * lanes + t] = y;  // y at the END of chunk c
            y = mapA[c * lanes + t] * y + mapB[c * lanes + t];
        }
    }
    __syncthreads();
    if (active) {
        double y = yin[t];
        for (int s = t1 - 1; s >= t0; --s) {
            double A, B;
            gae_coef(a, rew, val, mask, bad, s, n, k, A, B);
            y = A * y + B;
            const double vt = a.use_gae ? (double)val[((size_t)s * N + n) * K + k] : 0.0;
            ret[((size_t)s * N + n) * K + k] = (float)(y + vt);
        }
        if (ch == 0 && t < lanes) {  // returns[T]: GAE leaves it untouched, the plain sweep sets next_value
            if (!a.use_gae) ret[(size_t)T * N * K + lane] = val[(size_t)T * N * K + lane];
        }
    }
}

// ------------------------------------------------------------------------------------------
// advantages: x[t,n] = sum_k w_k s_k (R - V)[t,n,k], s_k = sqrt(obj_var_k + 1e-8);
// adv = (x - mean) / (std_unbiased + 1e-5)
constexpr int AT = 1024;

__device__ double block_sum_d(double v, double* red) {
    v = group_sum_d<64>(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    return s;
}

struct AdvArgs {
    int N, T, K;
    const float *ret, *val;
    const double *w, *obj_var;
    float* adv;
};

__global__ __launch_bounds__(AT) void adv_kernel(AdvArgs a) {
    __shared__ double red[AT / 64];
    __shared__ double coef[8];
    const int p = blockIdx.x, t = threadIdx.x, N = a.N, T = a.T, K = a.K;
    if (t < K) {
        const double s = a.obj_var ? sqrt(a.obj_var[p * K + t] + 1e-8) : 1.0;
        coef[t] = s * a.w[p * K + t];
    }
    __syncthreads();
    const float* R = a.ret + (size_t)p * (T + 1) * N * K;
    const float* V = a.val + (size_t)p * (T + 1) * N * K;
    const int B = T * N;
    auto x_of = [&](int i) {
        double r = 0.0, v = 0.0;
        for (int k = 0; k < K; ++k) {
            r += (double)R[(size_t)i * K + k] * coef[k];
            v += (double)V[(size_t)i * K + k] * coef[k];
        }
        return r - v;
    };
    double s = 0.0;
    for (int i = t; i < B; i += AT) s += x_of(i);
    const double mean = block_sum_d(s, red) / (double)B;
    double q = 0.0;
    for (int i = t; i < B; i += AT) {
        const double d = x_of(i) - mean;
        q += d * d;
    }
    const double var = block_sum_d(q, red) / (double)(B - 1);
    const double denom = sqrt(var) + 1e-5;
    float* adv = a.adv + (size_t)p * B;
    for (int i = t; i < B; i += AT) adv[i] = (float)((x_of(i) - mean) / denom);
}

// ------------------------------------------------------------------------------------------
// permutations: bitonic sort of (hash << 32 | index) keys in LDS, one workgroup per permutation
constexpr int PT = 1024;

__global__ __launch_bounds__(PT) void randperm_kernel(int n, int npow2, uint64_t seed, int32_t* out) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];
    const int c = blockIdx.x, t = threadIdx.x;
    const uint64_t s = splitmix64(seed * 0x9E3779B97F4A7C15ull + (uint64_t)c * 0xD1B54A32D192ED03ull + 1);
    for (int i = t; i < npow2; i += PT)
        keys[i] = i < n ? ((splitmix64(s ^ (uint64_t)i) & 0xFFFFFFFF00000000ull) | (uint64_t)i) : ~0ull;
    __syncthreads();
    for (int size = 2; size <= npow2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < npow2 / 2; i += PT) {
                const int lo = 2 * i - (i & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long x = keys[lo], y = keys[hi];
                if ((x > y) == up) {
                    keys[lo] = y;
                    keys[hi] = x;
                }
            }
            __syncthreads();
        }
    }
    for (int i = t; i < n; i += PT) out[(size_t)c * n + i] = (int32_t)(keys[i] & 0xFFFFFFFFull);
}

__global__ void normal_kernel(int64_t n, uint64_t seed, float* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = counter_normal(seed, (uint64_t)i);
}

}  // namespace pgm

using namespace pgm;

extern "C" {

int pgm_gae(const pgm_dims* d, const pgm_rollout_buf* rb, float gamma, float lam, int32_t use_gae,
            int32_t use_proper_time_limits, pgm_stream_t stream) {
    if (!d || !rb || !rb->rewards || !rb->values || !rb->masks || !rb->bad_masks || !rb->returns) {
        set_error("pgm_gae: null pointer");
        return PGM_E_INVALID_ARG;
    }
    if (d->P <= 0 || d->N <= 0 || d->T <= 0 || d->K <= 0 || d->N * d->K > 64) {
        set_error("pgm_gae: bad dims P=%d N=%d T=%d K=%d (need N*K <= 64)", d->P, d->N, d->T, d->K);
        return PGM_E_SHAPE;
    }
    GaeArgs a{d->N, d->T, d->K, rb->rewards, rb->values, rb->masks, rb->bad_masks, rb->returns, gamma, lam,
              use_gae, use_proper_time_limits};
    hipLaunchKernelGGL(gae_kernel, dim3(d->P), dim3(GT), 0, (hipStream_t)stream, a);
    return launch_status("pgm_gae");
}

int pgm_adv_normalize(const pgm_dims* d, const pgm_rollout_buf* rb, const double* weights,
                      const double* obj_var, pgm_stream_t stream) {
    if (!d || !rb || !rb->returns || !rb->values || !rb->adv || !weights) {
        set_error("pgm_adv_normalize: null pointer");
        return PGM_E_INVALID_ARG;
    }
    if (d->P <= 0 || d->N <= 0 || d->T <= 0 || d->K <= 0 || d->K > 8 || d->T * d->N < 2) {
        set_error("pgm_adv_normalize: bad dims P=%d N=%d T=%d K=%d", d->P, d->N, d->T, d->K);
        return PGM_E_SHAPE;
    }
    AdvArgs a{d->N, d->T, d->K, rb->returns, rb->values, weights, obj_var, rb->adv};
    hipLaunchKernelGGL(adv_kernel, dim3(d->P), dim3(AT), 0, (hipStream_t)stream, a);
    return launch_status("pgm_adv_normalize");
}

int pgm_randperm(int32_t n, int32_t count, uint64_t seed, int32_t* out, pgm_stream_t stream) {
    if (!out || n <= 0 || count <= 0) {
        set_error("pgm_randperm: bad arguments n=%d count=%d", n, count);
        return PGM_E_INVALID_ARG;
    }
    int npow2 = 1;
    while (npow2 < n) npow2 <<= 1;
    if (npow2 > 16384) {
        set_error("pgm_randperm: n=%d > 16384 unsupported (LDS sort)", n);
        return PGM_E_UNSUPPORTED;
    }
    const size_t smem = (size_t)npow2 * sizeof(unsigned long long);
    hipError_t e = hipFuncSetAttribute((const void*)randperm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)smem);
    if (e != hipSuccess) return hip_fail(e, "pgm_randperm");
    hipLaunchKernelGGL(randperm_kernel, dim3(count), dim3(PT), smem, (hipStream_t)stream, n, npow2, seed, out);
    return launch_status("pgm_randperm");
}

int pgm_normal_noise(int64_t n, uint64_t seed, float* out, pgm_stream_t stream) {
    if (!out || n < 0) {
        set_error("pgm_normal_noise: bad arguments");
        return PGM_E_INVALID_ARG;
    }
    if (n == 0) return PGM_OK;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(normal_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, seed, out);
    return launch_status("pgm_normal_noise");
}

}  // extern "C"
