// Scalarised clipped-PPO update: ppo_epoch x num_mini_batch Adam steps per task inside ONE launch,
// one 512-thread workgroup per task.  Per minibatch: gather the permuted rows (64 at a time) into
// LDS, forward both towers, loss gradients per row, backward through heads / layer 2 / layer 1 with
// gradient accumulators held in registers by the thread that owns each parameter element, then the
// global-norm clip and Adam on the owned elements (global master copy + the LDS working copy).
//
// Reference semantics:
//   PPO.update loop + losses                 a2c_ppo_acktr/algo/ppo.py:58-115
//   feed_forward_generator                   a2c_ppo_acktr/storage.py:118-154
//   Policy.evaluate_actions                  a2c_ppo_acktr/model.py:75-82
//   FixedNormal log_probs / entropy          a2c_ppo_acktr/distributions.py:29-40
//   clip_grad_norm_ (coef = max/(norm+1e-6), clamp 1)   torch.nn.utils.clip_grad
//   Adam (lerp m, v*b2 + (1-b2) g^2, bias-corrected step, eps outside sqrt)   torch.optim.adam
// torch.min / torch.max / clamp backward (ties split the gradient in half) are reproduced exactly.
#include <stdio.h>
#include <stdlib.h>

#include <mutex>
#include <unordered_map>

#include "pgm_dispatch.hpp"

PGM_STAMP_UNIT(update)

namespace pgm {

constexpr int UT = 512;  // threads: column c = t & 127 (critic < 64 <= actor), row group g = t >> 7
constexpr int UR = 64;   // rows per chunk
constexpr int UG = 16;   // rows per row group

template <int O>
constexpr int upad() { return (O + 3) & ~3; }
template <int A, int K>
constexpr int hq() { return A > K ? A : K; }

template <int O, int A, int K>
struct UpdSmem {
    float W1t[O][H2];
    float b1[H2], b2[H2];
    float W2t[2][H][H + 1];
    float Wv[H][K];
    float Wm[H][A];
    float bv[K], bm[A], logstd[A];
    alignas(16) float X[UR][upad<O>()];
    alignas(16) float H1[UR][H2];   // tanh(layer 1), then dZ1; reused as reduction scratch at minibatch end
    alignas(16) float H2[UR][H2];   // tanh(layer 2), then dZ2
    float act[UR][A];
    float dls[UR][A];
    float mu[UR][A];    // action mean, then dL/dmu
    float v[UR][K];     // value, then dL/dV
    float vold[UR][K], ret[UR][K];
    float oldlp[UR], adv[UR];
    float rowloss[UR][2];
    float red[UT / 64];
};

struct UpdArgs {
    int N, T;
    Layout L;
    pgm_ppo_hparams hp;
    float *params, *m, *v;
    int32_t* step;
    const float* lr;
    const int32_t* perms;
    const float *obs, *actions, *logp, *values, *returns, *adv;
    float* stats;
};

// LDS-only barrier: HBM stores (Adam state) stay in flight; every HBM re-read is by the writing thread
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float block_sum_f(float x, float* red) {
    x = group_sum<64>(x);
    lds_sync();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
    lds_sync();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < UT / 64; ++i) s += red[i];
    return s;
}

// torch.min(a,b) / torch.max(a,b) backward weights for the first argument (ties: half)
__device__ __forceinline__ float wmin(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }
__device__ __forceinline__ float wmax(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }

// Adam on one owned element; returns the new parameter value.
__device__ __forceinline__ float adam_elem(float* P, float* M, float* V, int idx, float g, float b1, float b2,
                                           float step_size, float bc2_sqrt, float eps) {
    float m = M[idx], v = V[idx];
    m = m + (1.f - b1) * (g - m);         // exp_avg.lerp_(grad, 1 - beta1)
    v = v * b2 + (1.f - b2) * (g * g);    // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    const float p = P[idx] - step_size * (m / denom);
    M[idx] = m;
    V[idx] = v;
    P[idx] = p;
    return p;
}

// LDS working-copy slot of flat parameter index i (nullptr for alignment padding)
template <int O, int A, int K>
__device__ __forceinline__ float* lds_slot(UpdSmem<O, A, K>& S, const Layout& L, int i) {
    auto in = [&](int tsr, int n) { return i >= L.off[tsr] && i < L.off[tsr] + n; };
    if (in(PGM_P_CRITIC_W2, H * H)) { const int r = i - L.off[PGM_P_CRITIC_W2]; return &S.W2t[0][r / H][r % H]; }
    if (in(PGM_P_ACTOR_W2, H * H)) { const int r = i - L.off[PGM_P_ACTOR_W2]; return &S.W2t[1][r / H][r % H]; }
    if (in(PGM_P_CRITIC_W1, O * H)) { const int r = i - L.off[PGM_P_CRITIC_W1]; return &S.W1t[r / H][r % H]; }
    if (in(PGM_P_ACTOR_W1, O * H)) { const int r = i - L.off[PGM_P_ACTOR_W1]; return &S.W1t[r / H][H + r % H]; }
    if (in(PGM_P_CRITIC_B1, H)) return &S.b1[i - L.off[PGM_P_CRITIC_B1]];
    if (in(PGM_P_ACTOR_B1, H)) return &S.b1[H + i - L.off[PGM_P_ACTOR_B1]];
    if (in(PGM_P_CRITIC_B2, H)) return &S.b2[i - L.off[PGM_P_CRITIC_B2]];
    if (in(PGM_P_ACTOR_B2, H)) return &S.b2[H + i - L.off[PGM_P_ACTOR_B2]];
    if (in(PGM_P_VALUE_W, H * K)) return &S.Wv[0][0] + (i - L.off[PGM_P_VALUE_W]);
    if (in(PGM_P_MEAN_W, H * A)) return &S.Wm[0][0] + (i - L.off[PGM_P_MEAN_W]);
    if (in(PGM_P_VALUE_B, K)) return &S.bv[i - L.off[PGM_P_VALUE_B]];
    if (in(PGM_P_MEAN_B, A)) return &S.bm[i - L.off[PGM_P_MEAN_B]];
    if (in(PGM_P_LOGSTD, A)) return &S.logstd[i - L.off[PGM_P_LOGSTD]];
    return nullptr;
}

template <int O, int A, int K>
__global__ __launch_bounds__(UT) void ppo_update_kernel(UpdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<UpdSmem<O, A, K>*>(smem_raw);
    constexpr int OP = upad<O>();
    constexpr int NW1 = (O + 3) / 4;
    constexpr int HQ = hq<A, K>();
    const int p = blockIdx.x, t = threadIdx.x, c = t & (H2 - 1), g = t >> 7, m = c >> 6, j = c & (H - 1);
    const int N = a.N, T = a.T, B = T * N;
    const int E = a.hp.ppo_epoch, M = a.hp.num_mini_batch;
    const int mb = B / M, nb = B / mb;
    const float clip = a.hp.clip_param;
    const Layout& L = a.L;
    float* P = a.params + (size_t)p * L.total;
    float* Mo = a.m + (size_t)p * L.total;
    float* Vo = a.v + (size_t)p * L.total;
    const float* obs = a.obs + (size_t)p * (T + 1) * N * O;
    const float* actions = a.actions + (size_t)p * B * A;
    const float* logp = a.logp + (size_t)p * B;
    const float* values = a.values + (size_t)p * (T + 1) * N * K;
    const float* returns = a.returns + (size_t)p * (T + 1) * N * K;
    const float* advs = a.adv + (size_t)p * B;

    // owned parameter offsets
    const int offW1 = (m == 0 ? L.off[PGM_P_CRITIC_W1] : L.off[PGM_P_ACTOR_W1]);
    const int offB1 = (m == 0 ? L.off[PGM_P_CRITIC_B1] : L.off[PGM_P_ACTOR_B1]);
    const int offW2 = (m == 0 ? L.off[PGM_P_CRITIC_W2] : L.off[PGM_P_ACTOR_W2]);
    const int offB2 = (m == 0 ? L.off[PGM_P_CRITIC_B2] : L.off[PGM_P_ACTOR_B2]);

    // load the LDS working copy of the parameters
    for (int i = t; i < O * H2; i += UT) {
        const int k = i / H2, cc = i % H2;
        S.W1t[k][cc] = P[(cc < H ? L.off[PGM_P_CRITIC_W1] : L.off[PGM_P_ACTOR_W1]) + k * H + (cc & (H - 1))];
    }
    for (int cc = t; cc < H2; cc += UT) {
        S.b1[cc] = P[(cc < H ? L.off[PGM_P_CRITIC_B1] : L.off[PGM_P_ACTOR_B1]) + (cc & (H - 1))];
        S.b2[cc] = P[(cc < H ? L.off[PGM_P_CRITIC_B2] : L.off[PGM_P_ACTOR_B2]) + (cc & (H - 1))];
    }
    for (int i = t; i < 2 * H * H; i += UT) {
        const int mm = i / (H * H), k = (i / H) % H, jj = i % H;
        S.W2t[mm][k][jj] = P[(mm == 0 ? L.off[PGM_P_CRITIC_W2] : L.off[PGM_P_ACTOR_W2]) + k * H + jj];
    }
    for (int i = t; i < H * K; i += UT) (&S.Wv[0][0])[i] = P[L.off[PGM_P_VALUE_W] + i];
    for (int i = t; i < H * A; i += UT) (&S.Wm[0][0])[i] = P[L.off[PGM_P_MEAN_W] + i];
    if (t < K) S.bv[t] = P[L.off[PGM_P_VALUE_B] + t];
    if (t < A) {
        S.bm[t] = P[L.off[PGM_P_MEAN_B] + t];
        S.logstd[t] = P[L.off[PGM_P_LOGSTD] + t];
    }
    __syncthreads();

    const int step0 = a.step[p];
    const double lr = a.lr[p];
    const float b1c = a.hp.beta1, b2c = a.hp.beta2, eps = a.hp.adam_eps;
    const float vscale = a.hp.value_loss_coef * 0.5f / (float)(mb * K);
    const float ascale = -1.f / (float)mb;
    float st_v = 0.f, st_a = 0.f, st_e = 0.f;
    int nstep = 0;

    PGM_STAMP_DECL
    for (int e = 0; e < E; ++e) {
        const int32_t* perm = a.perms + (size_t)e * B;
        for (int bb = 0; bb < nb; ++bb) {
            float accW2[UG], accW1[NW1], accH[HQ];
            float accB1 = 0.f, accB2 = 0.f, accS = 0.f;
            float lsum_v = 0.f, lsum_a = 0.f;
#pragma unroll
            for (int i = 0; i < UG; ++i) accW2[i] = 0.f;
#pragma unroll
            for (int i = 0; i < NW1; ++i) accW1[i] = 0.f;
#pragma unroll
            for (int i = 0; i < HQ; ++i) accH[i] = 0.f;

            for (int r0 = 0; r0 < mb; r0 += UR) {
                // ---- gather rows perm[bb*mb + r0 + r]
                for (int i = t; i < UR * OP; i += UT) {
                    const int r = i / OP, o = i % OP;
                    float x = 0.f;
                    if (r0 + r < mb && o < O) x = obs[(size_t)perm[bb * mb + r0 + r] * O + o];
                    S.X[r][o] = x;
                }
                if (t < UR) {
                    const int r = t;
                    const bool ok = r0 + r < mb;
                    const int idx = ok ? perm[bb * mb + r0 + r] : 0;
                    S.oldlp[r] = ok ? logp[idx] : 0.f;
                    S.adv[r] = ok ? advs[idx] : 0.f;
#pragma unroll
                    for (int q = 0; q < A; ++q) S.act[r][q] = ok ? actions[(size_t)idx * A + q] : 0.f;
#pragma unroll
                    for (int q = 0; q < K; ++q) {
                        S.vold[r][q] = ok ? values[(size_t)idx * K + q] : 0.f;
                        S.ret[r][q] = ok ? returns[(size_t)idx * K + q] : 0.f;
                    }
                }
                lds_sync();
                PGM_STAMP(20);
                // ---- layer 1 forward
                {
                    float acc[UG];
                    const float bias = S.b1[c];
#pragma unroll
                    for (int i = 0; i < UG; ++i) acc[i] = bias;
#pragma unroll 1
                    for (int k = 0; k < OP; k += 4) {  // X rows are zero-padded to OP
                        float w[4];
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk) w[kk] = (k + kk < O) ? S.W1t[k + kk][c] : 0.f;
#pragma unroll
                        for (int i = 0; i < UG; ++i) {
                            const float4 x = *reinterpret_cast<const float4*>(&S.X[g * UG + i][k]);
                            acc[i] = fmaf(x.x, w[0], acc[i]);
                            acc[i] = fmaf(x.y, w[1], acc[i]);
                            acc[i] = fmaf(x.z, w[2], acc[i]);
                            acc[i] = fmaf(x.w, w[3], acc[i]);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < UG; ++i) S.H1[g * UG + i][c] = tanh_f(acc[i]);
                }
                lds_sync();
                PGM_STAMP(21);
                // ---- layer 2 forward
                {
                    float acc[UG];
                    const float bias = S.b2[c];
#pragma unroll
                    for (int i = 0; i < UG; ++i) acc[i] = bias;
#pragma unroll 1
                    for (int k = 0; k < H; k += 4) {
                        const float w0 = S.W2t[m][k][j], w1 = S.W2t[m][k + 1][j];
                        const float w2 = S.W2t[m][k + 2][j], w3 = S.W2t[m][k + 3][j];
#pragma unroll
                        for (int i = 0; i < UG; ++i) {
                            const float4 h = *reinterpret_cast<const float4*>(&S.H1[g * UG + i][m * H + k]);
                            acc[i] = fmaf(h.x, w0, acc[i]);
                            acc[i] = fmaf(h.y, w1, acc[i]);
                            acc[i] = fmaf(h.z, w2, acc[i]);
                            acc[i] = fmaf(h.w, w3, acc[i]);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < UG; ++i) S.H2[g * UG + i][c] = tanh_f(acc[i]);
                }
                lds_sync();
                PGM_STAMP(22);
                // ---- heads: value [UR][K], mean [UR][A] (8 lanes per dot)
                {
                    const int sub = t & 7;
                    for (int o = t >> 3; o < UR * (K + A); o += UT / 8) {
                        const int r = o / (K + A), q = o % (K + A);
                        float s = 0.f;
                        if (q < K) {
#pragma unroll
                            for (int hh = 0; hh < 8; ++hh) s = fmaf(S.H2[r][sub * 8 + hh], S.Wv[sub * 8 + hh][q], s);
                        } else {
#pragma unroll
                            for (int hh = 0; hh < 8; ++hh)
                                s = fmaf(S.H2[r][H + sub * 8 + hh], S.Wm[sub * 8 + hh][q - K], s);
                        }
                        s = group_sum<8>(s);
                        if (sub == 0) {
                            if (q < K) S.v[r][q] = s + S.bv[q];
                            else S.mu[r][q - K] = s + S.bm[q - K];
                        }
                    }
                }
                lds_sync();
                PGM_STAMP(23);
                // ---- per-row loss gradients (ppo.py:80-96)
                if (t < UR) {  // policy (actor) rows
                    const int r = t;
                    const bool ok = r0 + r < mb;
                    float lp = 0.f;
#pragma unroll
                    for (int q = 0; q < A; ++q) {
                        const float sd = expf(S.logstd[q]);
                        const float dz = (S.act[r][q] - S.mu[r][q]) / sd;
                        lp += -0.5f * dz * dz - S.logstd[q] - LOG_SQRT_2PI;
                    }
                    const float ratio = expf(lp - S.oldlp[r]);
                    const float ad = S.adv[r];
                    const float s1 = ratio * ad;
                    const float rc = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip);
                    const float s2 = rc * ad;
                    const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
                    const float gr = ad * (wmin(s1, s2) + wmin(s2, s1) * inr);   // d min(s1,s2) / d ratio
                    const float dlp = ok ? ascale * gr * ratio : 0.f;            // dL/dlogp
                    S.rowloss[r][1] = ok ? -fminf(s1, s2) : 0.f;
#pragma unroll
                    for (int q = 0; q < A; ++q) {
                        const float sd = expf(S.logstd[q]);
                        const float diff = S.act[r][q] - S.mu[r][q];
                        const float z2 = diff * diff / (sd * sd);
                        S.mu[r][q] = dlp * diff / (sd * sd);      // dL/dmu
                        S.dls[r][q] = dlp * (z2 - 1.f);           // dL/dlogstd (row part)
                    }
                } else if (t < 2 * UR) {  // value (critic) rows
                    const int r = t - UR;
                    const bool ok = r0 + r < mb;
                    float ls = 0.f;
#pragma unroll
                    for (int q = 0; q < K; ++q) {
                        const float V = S.v[r][q], Vo = S.vold[r][q], R = S.ret[r][q];
                        float gv;
                        if (a.hp.use_clipped_value_loss) {
                            const float dv = V - Vo;
                            const float vc = Vo + fminf(fmaxf(dv, -clip), clip);
                            const float l1 = (V - R) * (V - R), l2 = (vc - R) * (vc - R);
                            const float inr = (dv >= -clip && dv <= clip) ? 1.f : 0.f;
                            gv = wmax(l1, l2) * 2.f * (V - R) + wmax(l2, l1) * 2.f * (vc - R) * inr;
                            ls += fmaxf(l1, l2);
                        } else {
                            gv = 2.f * (V - R);
                            ls += (R - V) * (R - V);
                        }
                        S.v[r][q] = ok ? vscale * gv : 0.f;  // dL/dV
                    }
                    S.rowloss[r][0] = ok ? ls : 0.f;
                }
                lds_sync();
                PGM_STAMP(24);
                // ---- head-weight grads (row group 0 owns them, all rows), bias/logstd grads, loss sums
                if (g == 0) {
#pragma unroll 2
                    for (int r = 0; r < UR; ++r) {
                        const float h = S.H2[r][c];
                        if (m == 0) {
#pragma unroll
                            for (int q = 0; q < K; ++q) accH[q] = fmaf(S.v[r][q], h, accH[q]);
                        } else {
#pragma unroll
                            for (int q = 0; q < A; ++q) accH[q] = fmaf(S.mu[r][q], h, accH[q]);
                        }
                    }
                }
                if (t < K + 2 * A) {  // bias / logstd gradients owned by threads 0 .. K+2A-1
                    float s = 0.f;
#pragma unroll 4
                    for (int r = 0; r < UR; ++r)
                        s += t < K ? S.v[r][t] : (t < K + A ? S.mu[r][t - K] : S.dls[r][t - K - A]);
                    accS += s;
                }
                if (t == 0) {
#pragma unroll 4
                    for (int r = 0; r < UR; ++r) {
                        lsum_v += S.rowloss[r][0];
                        lsum_a += S.rowloss[r][1];
                    }
                }
                lds_sync();
                PGM_STAMP(25);
                // ---- dZ2 = (dOut . W_head) * (1 - h2^2)
#pragma unroll 4
                for (int i = 0; i < UG; ++i) {
                    const int r = g * UG + i;
                    const float h = S.H2[r][c];
                    float dh = 0.f;
                    if (m == 0) {
#pragma unroll
                        for (int q = 0; q < K; ++q) dh = fmaf(S.v[r][q], S.Wv[j][q], dh);
                    } else {
#pragma unroll
                        for (int q = 0; q < A; ++q) dh = fmaf(S.mu[r][q], S.Wm[j][q], dh);
                    }
                    S.H2[r][c] = dh * (1.f - h * h);
                }
                lds_sync();
                PGM_STAMP(26);
                // ---- dW2^T[k][j] += sum_r H1[r][k] dZ2[r][j]  (k in [16g, 16g+16)), db2
#pragma unroll 2
                for (int r = 0; r < UR; ++r) {
                    const float dz = S.H2[r][c];
                    if (g == 0) accB2 += dz;
#pragma unroll
                    for (int i = 0; i < UG; i += 4) {
                        const float4 h = *reinterpret_cast<const float4*>(&S.H1[r][m * H + g * UG + i]);
                        accW2[i] = fmaf(h.x, dz, accW2[i]);
                        accW2[i + 1] = fmaf(h.y, dz, accW2[i + 1]);
                        accW2[i + 2] = fmaf(h.z, dz, accW2[i + 2]);
                        accW2[i + 3] = fmaf(h.w, dz, accW2[i + 3]);
                    }
                }
                lds_sync();
                PGM_STAMP(27);
                // ---- dH1 = dZ2 W2 -> dZ1 = dH1 * (1 - h1^2)   (this thread: tower m, input unit j)
                {
                    float dh[UG];
#pragma unroll
                    for (int i = 0; i < UG; ++i) dh[i] = 0.f;
#pragma unroll 1
                    for (int q = 0; q < H; q += 4) {
                        const float w0 = S.W2t[m][j][q], w1 = S.W2t[m][j][q + 1];
                        const float w2 = S.W2t[m][j][q + 2], w3 = S.W2t[m][j][q + 3];
#pragma unroll
                        for (int i = 0; i < UG; ++i) {
                            const float4 z = *reinterpret_cast<const float4*>(&S.H2[g * UG + i][m * H + q]);
                            dh[i] = fmaf(z.x, w0, dh[i]);
                            dh[i] = fmaf(z.y, w1, dh[i]);
                            dh[i] = fmaf(z.z, w2, dh[i]);
                            dh[i] = fmaf(z.w, w3, dh[i]);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < UG; ++i) {
                        const int r = g * UG + i;
                        const float h = S.H1[r][c];
                        S.H1[r][c] = dh[i] * (1.f - h * h);
                    }
                }
                lds_sync();
                PGM_STAMP(28);
                // ---- dW1^T[k][c] += sum_r X[r][k] dZ1[r][c]  (k = g + 4i), db1
#pragma unroll 2
                for (int r = 0; r < UR; ++r) {
                    const float dz = S.H1[r][c];
                    if (g == 0) accB1 += dz;
#pragma unroll
                    for (int i = 0; i < NW1; ++i)
                        if (g + 4 * i < O) accW1[i] = fmaf(S.X[r][g + 4 * i], dz, accW1[i]);
                }
                lds_sync();
                PGM_STAMP(29);
            }  // chunks

            // ---- stage the owned gradients in parameter layout (G aliases H1|H2, free after the chunks)
            float* G = &S.H1[0][0];
            for (int i = t; i < L.total; i += UT) G[i] = 0.f;
            float ent = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) ent += 0.5f + LOG_SQRT_2PI + S.logstd[q];
            lds_sync();
            PGM_STAMP(30);
#pragma unroll
            for (int i = 0; i < UG; ++i) G[offW2 + (g * UG + i) * H + j] = accW2[i];
#pragma unroll
            for (int i = 0; i < NW1; ++i)
                if (g + 4 * i < O) G[offW1 + (g + 4 * i) * H + j] = accW1[i];
            if (g == 0) {
                G[offB1 + j] = accB1;
                G[offB2 + j] = accB2;
                if (m == 0) {
#pragma unroll
                    for (int q = 0; q < K; ++q) G[L.off[PGM_P_VALUE_W] + j * K + q] = accH[q];
                } else {
#pragma unroll
                    for (int q = 0; q < A; ++q) G[L.off[PGM_P_MEAN_W] + j * A + q] = accH[q];
                }
            }
            if (t < K) G[L.off[PGM_P_VALUE_B] + t] = accS;
            else if (t < K + A) G[L.off[PGM_P_MEAN_B] + t - K] = accS;
            else if (t < K + 2 * A) G[L.off[PGM_P_LOGSTD] + t - K - A] = accS - a.hp.entropy_coef;
            lds_sync();
            PGM_STAMP(31);
            // ---- clip_grad_norm_ over every parameter
            float sq = 0.f;
            for (int i = t; i < L.total; i += UT) sq = fmaf(G[i], G[i], sq);
            const float total = block_sum_f(sq, S.red);
            const float coef = fminf(a.hp.max_grad_norm / (sqrtf(total) + 1e-6f), 1.f);
            // ---- Adam (coalesced over the flat parameter vector; padding slots stay 0)
            ++nstep;
            const int stepi = step0 + nstep;
            const double bc1 = 1.0 - pow((double)b1c, (double)stepi);
            const double bc2 = 1.0 - pow((double)b2c, (double)stepi);
            const float step_size = (float)(lr / bc1);
            const float bc2s = (float)sqrt(bc2);
            for (int i = t; i < L.total; i += UT) {
                const float pn = adam_elem(P, Mo, Vo, i, G[i] * coef, b1c, b2c, step_size, bc2s, eps);
                float* slot = lds_slot<O, A, K>(S, L, i);
                if (slot) *slot = pn;
            }
            if (t == 0) {
                st_v += 0.5f * lsum_v / (float)(mb * K);
                st_a += lsum_a / (float)mb;
                st_e += ent;
            }
            lds_sync();
            PGM_STAMP(32);
        }  // minibatches
    }      // epochs
    if (t == 0) {
        a.step[p] = step0 + nstep;
        const float n = (float)(E * M);
        a.stats[p * 3 + 0] = st_v / n;
        a.stats[p * 3 + 1] = st_a / n;
        a.stats[p * 3 + 2] = st_e / n;
    }
    PGM_STAMP_FLUSH;
}

}  // namespace pgm

namespace pgm {
int ppo_update_mfma(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m, float* adam_v,
                    int32_t* adam_step, const float* lr, const int32_t* perms, const pgm_rollout_buf* rb, float* stats,
                    void* workspace, const pgm_launch_opts& o, hipStream_t stream);
int ppo_update_wide(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m, float* adam_v,
                    int32_t* adam_step, const float* lr, const int32_t* perms, const pgm_rollout_buf* rb, float* stats,
                    void* workspace, const pgm_launch_opts& o, hipStream_t stream);
}

using namespace pgm;

extern "C" size_t pgm_ppo_update_workspace_bytes(const pgm_dims* d) { return d ? ppo_workspace_bytes(d) : 0; }

namespace pgm {
int describe_update_mfma(const pgm_dims* d, const pgm_ppo_hparams* hp, const pgm_launch_opts& o, char* buf, int n);
int describe_update_wide(const pgm_dims* d, const pgm_launch_opts& o, char* buf, int n);
}
extern "C" int pgm_ppo_update_variant(const pgm_dims* d, const pgm_ppo_hparams* hp, const pgm_launch_opts* opts,
                                      char* buf, int n) {
    if (int rc = check_dims(d, "pgm_ppo_update_variant")) return rc;
    if (!hp || !buf || n <= 0 || hp->num_mini_batch <= 0) {
        set_error("pgm_ppo_update_variant: null pointer or empty buffer");
        return PGM_E_INVALID_ARG;
    }
    pgm_launch_opts o;
    if (int rc = read_opts(opts, &o, "pgm_ppo_update_variant")) return rc;
    if (o.update_kernel == PGM_UPDATE_VALU)
        return snprintf(buf, n, "ppo_update_kernel (VALU, A/B)") > 0 ? PGM_OK : PGM_E_INVALID_ARG;
    if (d->O <= 32) return describe_update_mfma(d, hp, o, buf, n) > 0 ? PGM_OK : PGM_E_INVALID_ARG;
    return describe_update_wide(d, o, buf, n) > 0 ? PGM_OK : PGM_E_INVALID_ARG;
}

// workspaces zeroed ahead of their next launch by pgm_ppo_update_reset: pointer -> zeroed bytes
static std::mutex g_zeroed_mu;
static std::unordered_map<const void*, size_t> g_zeroed;

bool pgm::ws_take_zeroed(const void* ws, size_t need) {
    std::lock_guard<std::mutex> lk(g_zeroed_mu);
    auto it = g_zeroed.find(ws);
    if (it == g_zeroed.end()) return false;
    const bool ok = it->second >= need;
    g_zeroed.erase(it);  // consumed either way: the next launch reuses the workspace
    return ok;
}

extern "C" int pgm_ppo_update_reset(const pgm_dims* d, void* workspace, pgm_stream_t stream) {
    if (int rc = check_dims(d, "pgm_ppo_update_reset")) return rc;
    if (!workspace) {
        set_error("pgm_ppo_update_reset: null workspace");
        return PGM_E_INVALID_ARG;
    }
    const size_t n = ppo_reset_bytes(d);
    hipError_t e = hipMemsetAsync(workspace, 0, n, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update_reset");
    std::lock_guard<std::mutex> lk(g_zeroed_mu);
    g_zeroed[workspace] = n;
    return PGM_OK;
}

extern "C" int pgm_ppo_update(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m,
                              float* adam_v, int32_t* adam_step, const float* lr, const int32_t* perms,
                              const pgm_rollout_buf* rb, float* stats, void* workspace, const pgm_launch_opts* opts,
                              pgm_stream_t stream) {
    if (int rc = check_dims(d, "pgm_ppo_update")) return rc;
    pgm_launch_opts o;
    if (int rc = read_opts(opts, &o, "pgm_ppo_update")) return rc;
    if (!hp || !params || !adam_m || !adam_v || !adam_step || !lr || !perms || !rb || !rb->obs || !rb->actions ||
        !rb->logp || !rb->values || !rb->returns || !rb->adv || !stats) {
        set_error("pgm_ppo_update: null pointer");
        return PGM_E_INVALID_ARG;
    }
    const int B = d->T * d->N;
    if (hp->ppo_epoch <= 0 || hp->num_mini_batch <= 0 || B < hp->num_mini_batch) {
        set_error("pgm_ppo_update: need T*N (%d) >= num_mini_batch (%d) > 0 and ppo_epoch > 0", B, hp->num_mini_batch);
        return PGM_E_SHAPE;
    }
    // f32-MFMA kernels: obs_dim <= 32 (Walker, Cheetah, Hopper, Ant, Swimmer) with LDS-resident towers, wider
    // observations (Humanoid) with layer 1 in L2; the VALU kernel is kept for A/B measurements
    // (opts.update_kernel = PGM_UPDATE_VALU) and covers obs_dim <= 64
    const bool valu = o.update_kernel == PGM_UPDATE_VALU;
    if (!valu && d->O <= 32)
        return ppo_update_mfma(d, hp, params, adam_m, adam_v, adam_step, lr, perms, rb, stats, workspace, o,
                               (hipStream_t)stream);
    if (!valu && d->O > 64)
        return ppo_update_wide(d, hp, params, adam_m, adam_v, adam_step, lr, perms, rb, stats, workspace, o,
                               (hipStream_t)stream);
    if (d->O > 64) {
        set_error("pgm_ppo_update: obs_dim %d > 64 not supported by the update kernels", d->O);
        return PGM_E_UNSUPPORTED;
    }
    UpdArgs a{d->N, d->T, make_layout(d->O, d->A, d->K, d->H), *hp, params, adam_m, adam_v, adam_step, lr, perms,
              rb->obs, rb->actions, rb->logp, rb->values, rb->returns, rb->adv, stats};
    return dispatch_dims(d->O, d->A, d->K, "pgm_ppo_update", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (O > 64) {
            return PGM_E_UNSUPPORTED;
        } else {
            const size_t smem = sizeof(UpdSmem<O, A, K>);
            if ((size_t)a.L.total > 2 * UR * H2) {
                set_error("pgm_ppo_update: %d parameters exceed the LDS gradient image", a.L.total);
                return PGM_E_UNSUPPORTED;
            }
            if (smem > 160 * 1024) {
                set_error("pgm_ppo_update: LDS image %zu bytes exceeds 160 KiB", smem);
                return PGM_E_UNSUPPORTED;
            }
            auto kern = ppo_update_kernel<O, A, K>;
            hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update");
            if (workspace && !ws_take_zeroed(workspace, ppo_flag_bytes(d->P))) {
                // no exchange in this kernel: the timeout word (2P) reads 0 for this call
                e = hipMemsetAsync(workspace, 0, ppo_flag_bytes(d->P), (hipStream_t)stream);
                if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update (workspace reset)");
            }
            hipLaunchKernelGGL(kern, dim3(d->P), dim3(UT), smem, (hipStream_t)stream, a);
            return launch_status("pgm_ppo_update");
        }
    });
}
