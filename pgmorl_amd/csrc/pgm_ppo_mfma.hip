// Scalarised clipped-PPO update on the f32 matrix cores (v_mfma_f32_32x32x2_f32, exact fp32).
//
// One 256-thread workgroup per task, 4 waves: wave w runs tower m = w & 1 (0 critic, 1 actor) on
// the sample tiles (32 samples each) t = (w >> 1) + 2i of the minibatch.  Orientation: samples are
// the accumulator ROWS (registers), features the COLUMNS (lanes), i.e. for a 32-sample tile every
// activation H1, H2, dZ2, dZ1 lives in the standard C layout
//     lane l, register r  <->  (sample rowof(r, l>>5), feature l & 31),  rowof(r,h) = (r&3)+8(r>>2)+4h.
// Consequences:
//   * every weight gradient (dW2^T = H1^T dZ2, dW1^T = X^T dZ1) sums over the sample index, i.e.
//     over registers: MFMA(A = H1 reg r, B = dZ2 reg r) with no data movement at all;
//   * the two products that sum over a FEATURE index (Z2 = H1 W2^T and dH1 = dZ2 W2) take their A
//     operand from a per-wave [32][65] LDS tile written from the C layout (one ds_write per register);
//   * the value / mean heads and the per-sample losses run on the VALU, one sample per lane.
// Gradients accumulate in registers over the minibatch; the two waves of a tower then add theirs
// into an LDS gradient image in parameter layout (fixed order => deterministic), followed by
// clip_grad_norm_ and Adam as one coalesced pass over the flat parameter vector.
//
// Reference semantics: a2c_ppo_acktr/algo/ppo.py:58-115 (losses, clip_grad_norm_, Adam),
// a2c_ppo_acktr/storage.py:118-154 (minibatch rows), a2c_ppo_acktr/model.py:75-82,
// a2c_ppo_acktr/distributions.py:29-40 (log_probs / entropy).  torch.min/max/clamp backward
// (ties split the gradient in half) are reproduced exactly.
#include <stdlib.h>

#include "pgm_dispatch.hpp"

PGM_STAMP_UNIT(mfma)

namespace pgm {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MT = 256;     // threads: 4 waves
constexpr int SB = 256;     // samples staged per pass (minibatches larger than this loop over passes)
constexpr int TS = 32;      // samples per MFMA tile
constexpr int SCR = H + 1;  // per-wave transpose tile row stride (conflict-free column reads)

template <int O>
constexpr int ox() { return O | 1; }  // odd X-image stride: conflict-free A-operand reads
template <int A, int K>
constexpr int qmax() { return A > K ? A : K; }

__device__ __forceinline__ int rowof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void wave_lds_fence() {  // this wave's LDS writes are visible to its own lanes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void lds_sync_m() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ float xhalf(float v) {  // value of lane l ^ 32
    return __shfl_xor(v, 32, 64);
}

template <int O, int A, int K>
struct MSmem {
    static constexpr int Q = qmax<A, K>();
    // parameter working copy (LDS images, fp32)
    float W1t[2][O][H];        // [tower][in][out]
    float W2t[2][H][SCR];      // [tower][in][out], padded rows
    float Wh[2][Q][H];         // [tower][head output][unit]  (critic: value, actor: mean)
    float b1[2][H], b2[2][H], bh[2][Q], logstd[A];
    // per-pass staged rows
    float act[SB][A];
    float oldlp[SB], adv[SB];
    float vold[SB][K], ret[SB][K];
    float dout[4][TS][Q];      // per-wave dL/d(head output) of the current tile
    float red[16];
    // big region: X image + per-wave transpose tiles during the passes, gradient image at the end
    union Big {
        struct {
            float X[SB][ox<O>()];
            float scr[4][TS][SCR];
        } s;
        float G[1];
    } big;
};

template <int O, int A, int K>
constexpr size_t big_floats() { return sizeof(typename MSmem<O, A, K>::Big) / sizeof(float); }

struct MArgs {
    int N, T;
    Layout L;
    pgm_ppo_hparams hp;
    float *params, *m, *v;
    int32_t* step;
    const float* lr;
    const int32_t* perms;
    const float *obs, *actions, *logp, *values, *returns, *adv;
    float* stats;
    unsigned long long* ws;  // SPLIT: [2P] tagged granules + [1] timeout flag, zeroed before the launch
    int P;
};

__device__ __forceinline__ float wmin2(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }
__device__ __forceinline__ float wmax2(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }

// Visit every parameter tensor with its LDS working-copy slot: f(tensor id, count, slot(j)).
template <int O, int A, int K, class F>
__device__ __forceinline__ void for_each_tensor(MSmem<O, A, K>& S, F&& f) {
    f(PGM_P_ACTOR_W1, O * H, [&](int j) { return &S.W1t[1][0][0] + j; });
    f(PGM_P_ACTOR_B1, H, [&](int j) { return &S.b1[1][j]; });
    f(PGM_P_ACTOR_W2, H * H, [&](int j) { return &S.W2t[1][j / H][j % H]; });
    f(PGM_P_ACTOR_B2, H, [&](int j) { return &S.b2[1][j]; });
    f(PGM_P_CRITIC_W1, O * H, [&](int j) { return &S.W1t[0][0][0] + j; });
    f(PGM_P_CRITIC_B1, H, [&](int j) { return &S.b1[0][j]; });
    f(PGM_P_CRITIC_W2, H * H, [&](int j) { return &S.W2t[0][j / H][j % H]; });
    f(PGM_P_CRITIC_B2, H, [&](int j) { return &S.b2[0][j]; });
    f(PGM_P_VALUE_W, H * K, [&](int j) { return &S.Wh[0][j % K][j / K]; });
    f(PGM_P_VALUE_B, K, [&](int j) { return &S.bh[0][j]; });
    f(PGM_P_MEAN_W, H * A, [&](int j) { return &S.Wh[1][j % A][j / A]; });
    f(PGM_P_MEAN_B, A, [&](int j) { return &S.bh[1][j]; });
    f(PGM_P_LOGSTD, A, [&](int j) { return &S.logstd[j]; });
}

template <int O, int A, int K, bool SPLIT>
__global__ __launch_bounds__(MT) void ppo_update_mfma_kernel(MArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<MSmem<O, A, K>*>(smem_raw);
    constexpr int Q = qmax<A, K>();
    constexpr int OX = ox<O>();
    constexpr int KS1 = (O + 1) / 2;  // k-steps of layer 1
    // SPLIT: two workgroups per task (blockIdx = 2 task + tower), all 4 waves on one tower, exchanging
    // only the squared gradient norm per minibatch.  Otherwise one workgroup: waves 0/2 critic, 1/3 actor.
    constexpr int NWT = SPLIT ? 4 : 2;  // waves per tower
    const int t = threadIdx.x, w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int p = SPLIT ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const int m = SPLIT ? (int)(blockIdx.x & 1) : (w & 1);  // tower
    const int sh = SPLIT ? w : (w >> 1);                      // wave index within the tower
    const int NQ = m == 0 ? K : A;
    const int N = a.N, T = a.T, B = T * N;
    const int E = a.hp.ppo_epoch, M = a.hp.num_mini_batch;
    const int mb = B / M, nb = B / mb;
    const float clip = a.hp.clip_param;
    const Layout& L = a.L;
    float* __restrict__ P = a.params + (size_t)p * L.total;
    float* __restrict__ Mo = a.m + (size_t)p * L.total;
    float* __restrict__ Vo = a.v + (size_t)p * L.total;
    const float* obs = a.obs + (size_t)p * (T + 1) * N * O;
    const float* actions = a.actions + (size_t)p * B * A;
    const float* logp = a.logp + (size_t)p * B;
    const float* values = a.values + (size_t)p * (T + 1) * N * K;
    const float* returns = a.returns + (size_t)p * (T + 1) * N * K;
    const float* advs = a.adv + (size_t)p * B;

    // ---- parameter working copy
    for_each_tensor(S, [&](int tsr, int n, auto slot) {
        const int off = L.off[tsr];
#pragma unroll 4
        for (int j = t; j < n; j += MT) *slot(j) = P[off + j];
    });
    for (int i = t; i < 2 * Q * H; i += MT) {  // head rows beyond K (critic) stay zero
        const int mm = i / (Q * H), q = (i / H) % Q;
        if (q >= (mm == 0 ? K : A)) S.Wh[mm][q][i % H] = 0.f;
    }
    for (int i = t; i < 2 * Q; i += MT)
        if (i % Q >= (i / Q == 0 ? K : A)) S.bh[i / Q][i % Q] = 0.f;
    __syncthreads();

    const int step0 = a.step[p];
    const double lr = a.lr[p];
    const float b1c = a.hp.beta1, b2c = a.hp.beta2, eps = a.hp.adam_eps;
    const float vscale = a.hp.value_loss_coef * 0.5f / (float)(mb * K);
    const float ascale = -1.f / (float)mb;
    float st_v = 0.f, st_a = 0.f, st_e = 0.f;
    int nstep = 0;
    float* scr = &S.big.s.scr[w][0][0];
    PGM_STAMP_DECL

    for (int e = 0; e < E; ++e) {
        const int32_t* perm = a.perms + (size_t)e * B;
        for (int bb = 0; bb < nb; ++bb) {
            f32x16 gW2[2][2], gW1[2];  // [in tile][out tile], [out tile] (O <= 32: one in tile)
            float gWh[2][Q], gB1[2], gB2[2], gBh[Q], gLs[A];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j) gW2[i][j] = f32x16{0};
                gW1[i] = f32x16{0};
                gB1[i] = gB2[i] = 0.f;
#pragma unroll
                for (int q = 0; q < Q; ++q) gWh[i][q] = 0.f;
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) gBh[q] = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) gLs[q] = 0.f;
            float lsum = 0.f;

            for (int s0 = 0; s0 < mb; s0 += SB) {
                const int ns = min(SB, mb - s0);
                // ---- stage rows perm[bb*mb + s0 + i]: X image and per-sample data
                for (int i = t; i < SB; i += MT) {
                    const bool ok = i < ns;
                    const int idx = ok ? perm[bb * mb + s0 + i] : 0;
#pragma unroll
                    for (int k = 0; k < OX; ++k) S.big.s.X[i][k] = (ok && k < O) ? obs[(size_t)idx * O + k] : 0.f;
                    S.oldlp[i] = ok ? logp[idx] : 0.f;
                    S.adv[i] = ok ? advs[idx] : 0.f;
#pragma unroll
                    for (int q = 0; q < A; ++q) S.act[i][q] = ok ? actions[(size_t)idx * A + q] : 0.f;
#pragma unroll
                    for (int q = 0; q < K; ++q) {
                        S.vold[i][q] = ok ? values[(size_t)idx * K + q] : 0.f;
                        S.ret[i][q] = ok ? returns[(size_t)idx * K + q] : 0.f;
                    }
                }
                lds_sync_m();
                PGM_STAMP(0);

                for (int tile = sh; tile * TS < ns; tile += NWT) {
                    const int ts0 = tile * TS;
                    // ---- layer 1: Z1[s][h] = X[s][:] . W1t[:][h]
                    f32x16 z[2] = {f32x16{0}, f32x16{0}};
#pragma unroll
                    for (int ks = 0; ks < KS1; ++ks) {
                        const int k = 2 * ks + h;
                        const float av = k < O ? S.big.s.X[ts0 + c][k] : 0.f;
#pragma unroll
                        for (int hb = 0; hb < 2; ++hb) {
                            const float bv = k < O ? S.W1t[m][k][hb * TS + c] : 0.f;
                            z[hb] = mfma(av, bv, z[hb]);
                        }
                    }
                    f32x16 H1[2];
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb) {
                        const float bias = S.b1[m][hb * TS + c];
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            H1[hb][r] = tanh_f(z[hb][r] + bias);
                            scr[rowof(r, h) * SCR + hb * TS + c] = H1[hb][r];
                        }
                    }
                    wave_lds_fence();
                    // ---- layer 2: Z2[s][o] = H1[s][:] . W2t[:][o]   (A from the transpose tile)
                    z[0] = z[1] = f32x16{0};
#pragma unroll 8
                    for (int ks = 0; ks < H / 2; ++ks) {
                        const int k = 2 * ks + h;
                        const float av = scr[c * SCR + k];
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob) z[ob] = mfma(av, S.W2t[m][k][ob * TS + c], z[ob]);
                    }
                    f32x16 H2[2];
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob) {
                        const float bias = S.b2[m][ob * TS + c];
#pragma unroll
                        for (int r = 0; r < 16; ++r) H2[ob][r] = tanh_f(z[ob][r] + bias);
                    }
                    wave_lds_fence();  // every lane finished reading the H1 tile
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ob * TS + c] = H2[ob][r];
                    wave_lds_fence();
                    // ---- heads on the VALU: lane = sample c, half h sums units [32h, 32h+32)
                    float outv[Q];
#pragma unroll
                    for (int q = 0; q < Q; ++q) outv[q] = 0.f;
#pragma unroll 4
                    for (int u = 0; u < TS; ++u) {
                        const float hv = scr[c * SCR + h * TS + u];
#pragma unroll
                        for (int q = 0; q < Q; ++q) outv[q] = fmaf(hv, S.Wh[m][q][h * TS + u], outv[q]);
                    }
#pragma unroll
                    for (int q = 0; q < Q; ++q) outv[q] += xhalf(outv[q]) + S.bh[m][q];
                    // ---- per-sample loss gradients (ppo.py:80-96); both halves compute the same sample
                    const int si = ts0 + c;
                    const bool ok = si < ns;
                    float dO[Q];
#pragma unroll
                    for (int q = 0; q < Q; ++q) dO[q] = 0.f;
                    if (m == 0) {  // value loss
                        float ls = 0.f;
#pragma unroll
                        for (int q = 0; q < K; ++q) {
                            const float V = outv[q], Vo = S.vold[si][q], R = S.ret[si][q];
                            float gv;
                            if (a.hp.use_clipped_value_loss) {
                                const float dv = V - Vo;
                                const float vc = Vo + fminf(fmaxf(dv, -clip), clip);
                                const float l1 = (V - R) * (V - R), l2 = (vc - R) * (vc - R);
                                const float inr = (dv >= -clip && dv <= clip) ? 1.f : 0.f;
                                gv = wmax2(l1, l2) * 2.f * (V - R) + wmax2(l2, l1) * 2.f * (vc - R) * inr;
                                ls += fmaxf(l1, l2);
                            } else {
                                gv = 2.f * (V - R);
                                ls += (R - V) * (R - V);
                            }
                            dO[q] = ok ? vscale * gv : 0.f;
                        }
                        if (ok && h == 0) lsum += ls;
                    } else {  // clipped surrogate
                        float lp = 0.f;
#pragma unroll
                        for (int q = 0; q < A; ++q) {
                            const float sd = expf(S.logstd[q]);
                            const float dz = (S.act[si][q] - outv[q]) / sd;
                            lp += -0.5f * dz * dz - S.logstd[q] - LOG_SQRT_2PI;
                        }
                        const float ratio = expf(lp - S.oldlp[si]);
                        const float ad = S.adv[si];
                        const float s1 = ratio * ad;
                        const float s2 = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip) * ad;
                        const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
                        const float gr = ad * (wmin2(s1, s2) + wmin2(s2, s1) * inr);
                        const float dlp = ok ? ascale * gr * ratio : 0.f;
                        if (ok && h == 0) lsum += -fminf(s1, s2);
#pragma unroll
                        for (int q = 0; q < A; ++q) {
                            const float sd = expf(S.logstd[q]);
                            const float diff = S.act[si][q] - outv[q];
                            const float iv = 1.f / (sd * sd);
                            dO[q] = dlp * diff * iv;
                            if (h == 0) gLs[q] += dlp * (diff * diff * iv - 1.f);
                        }
                    }
                    if (h == 0) {
#pragma unroll
                        for (int q = 0; q < Q; ++q) {
                            gBh[q] += dO[q];
                            S.dout[w][c][q] = dO[q];
                        }
                    }
                    wave_lds_fence();
                    // ---- head-weight grads (VALU, C layout): gWh[ob][q] += sum_r H2[s][u] dO[s][q]
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int s = rowof(r, h);
#pragma unroll
                            for (int q = 0; q < Q; ++q) gWh[ob][q] = fmaf(H2[ob][r], S.dout[w][s][q], gWh[ob][q]);
                        }
                    // ---- dH2 = dO . Wh  (MFMA; A = this lane's sample, k = head output) -> dZ2
                    z[0] = z[1] = f32x16{0};
#pragma unroll
                    for (int ks = 0; ks < (Q + 1) / 2; ++ks) {
                        const int q = 2 * ks + h;
                        const float av = h ? (2 * ks + 1 < Q ? dO[2 * ks + 1] : 0.f) : dO[2 * ks];
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob) z[ob] = mfma(av, q < Q ? S.Wh[m][q][ob * TS + c] : 0.f, z[ob]);
                    }
                    f32x16 dZ2[2];
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            dZ2[ob][r] = z[ob][r] * (1.f - H2[ob][r] * H2[ob][r]);
                            gB2[ob] += dZ2[ob][r];
                        }
                    // ---- dW2^T[in][o] += H1^T dZ2: straight from the C-layout registers
#pragma unroll
                    for (int r = 0; r < 16; ++r)
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                            for (int ob = 0; ob < 2; ++ob) gW2[ib][ob] = mfma(H1[ib][r], dZ2[ob][r], gW2[ib][ob]);
                    // ---- dH1 = dZ2 W2  (A = dZ2 through the transpose tile, B = W2t[in][o] column)
                    wave_lds_fence();  // heads finished reading the H2 tile
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ob * TS + c] = dZ2[ob][r];
                    wave_lds_fence();
                    z[0] = z[1] = f32x16{0};
#pragma unroll 8
                    for (int ks = 0; ks < H / 2; ++ks) {
                        const int k = 2 * ks + h;  // output unit o
                        const float av = scr[c * SCR + k];
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib) z[ib] = mfma(av, S.W2t[m][ib * TS + c][k], z[ib]);
                    }
                    f32x16 dZ1[2];
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            dZ1[ib][r] = z[ib][r] * (1.f - H1[ib][r] * H1[ib][r]);
                            gB1[ib] += dZ1[ib][r];
                        }
                    // ---- dW1^T[k][h] += X^T dZ1  (A = X[s(r)][k = lane], B = dZ1 reg r)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float av = S.big.s.X[ts0 + rowof(r, h)][c < OX ? c : 0];
#pragma unroll
                        for (int hb = 0; hb < 2; ++hb) gW1[hb] = mfma(c < O ? av : 0.f, dZ1[hb][r], gW1[hb]);
                    }
                    wave_lds_fence();  // dH1 finished reading the dZ2 tile before the next tile's writes
                }  // tiles
                lds_sync_m();  // X / per-sample rows are re-staged by the next pass
                PGM_STAMP(1);
            }  // passes

            // ---- combine the lane halves of the per-column partial sums
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                gB1[i] += xhalf(gB1[i]);
                gB2[i] += xhalf(gB2[i]);
#pragma unroll
                for (int q = 0; q < Q; ++q) gWh[i][q] += xhalf(gWh[i][q]);
            }
            // per-sample partials (held by half 0 lanes): 64-lane sums (half 1 holds zeros)
#pragma unroll
            for (int q = 0; q < Q; ++q) gBh[q] = wave_sum64(gBh[q]);
#pragma unroll
            for (int q = 0; q < A; ++q) gLs[q] = wave_sum64(gLs[q]);
            lsum = wave_sum64(lsum);
            // entropy with the logstd of this step (before Adam)
            float ent = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) ent += 0.5f + LOG_SQRT_2PI + S.logstd[q];

            // ---- gradient image in parameter layout: zero, sample-half 0 stores, sample-half 1 adds
            float* G = S.big.G;
            for (int i = t; i < L.total; i += MT) G[i] = 0.f;
            lds_sync_m();
            const int offW1 = m == 0 ? L.off[PGM_P_CRITIC_W1] : L.off[PGM_P_ACTOR_W1];
            const int offB1 = m == 0 ? L.off[PGM_P_CRITIC_B1] : L.off[PGM_P_ACTOR_B1];
            const int offW2 = m == 0 ? L.off[PGM_P_CRITIC_W2] : L.off[PGM_P_ACTOR_W2];
            const int offB2 = m == 0 ? L.off[PGM_P_CRITIC_B2] : L.off[PGM_P_ACTOR_B2];
            const int offWh = m == 0 ? L.off[PGM_P_VALUE_W] : L.off[PGM_P_MEAN_W];
            const int offBh = m == 0 ? L.off[PGM_P_VALUE_B] : L.off[PGM_P_MEAN_B];
            for (int round = 0; round < NWT; ++round) {
                if (sh == round) {
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                            for (int r = 0; r < 16; ++r) {
                                const int gi = offW2 + (ib * TS + rowof(r, h)) * H + ob * TS + c;
                                G[gi] += gW2[ib][ob][r];
                            }
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int k = rowof(r, h);
                            if (k < O) G[offW1 + k * H + hb * TS + c] += gW1[hb][r];
                        }
                    if (h == 0) {
#pragma unroll
                        for (int i = 0; i < 2; ++i) {
                            G[offB1 + i * TS + c] += gB1[i];
                            G[offB2 + i * TS + c] += gB2[i];
#pragma unroll
                            for (int q = 0; q < Q; ++q)
                                if (q < NQ) G[offWh + (i * TS + c) * NQ + q] += gWh[i][q];
                        }
                    }
                    if (l == 0) {
#pragma unroll
                        for (int q = 0; q < Q; ++q)
                            if (q < NQ) G[offBh + q] += gBh[q];
                        if (m == 1) {
#pragma unroll
                            for (int q = 0; q < A; ++q)
                                G[L.off[PGM_P_LOGSTD] + q] += gLs[q] - (round == 0 ? a.hp.entropy_coef : 0.f);
                        }
                        S.red[8 + w] = lsum;
                    }
                }
                lds_sync_m();
            }
            PGM_STAMP(2);
            // ---- clip_grad_norm_ over every parameter (G holds zeros outside this workgroup's tensors)
            float sq = 0.f;
            for (int i = t; i < L.total; i += MT) sq = fmaf(G[i], G[i], sq);
            sq = wave_sum64(sq);
            if (l == 0) S.red[w] = sq;
            lds_sync_m();
            float total = (S.red[0] + S.red[1]) + (S.red[2] + S.red[3]);
            if constexpr (SPLIT) {  // tagged 8-byte granule hand-off with the other tower's workgroup
                if (t == 0) {
                    const unsigned tag = (unsigned)(nstep + 1);
                    unsigned long long* ws = a.ws + 2 * p;
                    __hip_atomic_store(ws + m, ((unsigned long long)tag << 32) | __float_as_uint(total),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    unsigned long long x = 0;
                    const bool failed = __hip_atomic_load(a.ws + 2 * a.P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    for (unsigned spins = 0; !failed; ++spins) {
                        x = __hip_atomic_load(ws + (1 - m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned)(x >> 32) == tag) break;
                        if (spins > (1u << 26)) {  // partner never arrived: flag it, continue unclipped-safe
                            __hip_atomic_store(a.ws + 2 * a.P, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            x = 0;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    const float other = __uint_as_float((unsigned)x);
                    S.red[4] = m == 0 ? total + other : other + total;  // critic + actor in both workgroups
                }
                lds_sync_m();
                total = S.red[4];
            }
            const float coef = fminf(a.hp.max_grad_norm / (sqrtf(total) + 1e-6f), 1.f);
            if (t == 0) {
                if constexpr (SPLIT) {
                    const float ls = (S.red[8] + S.red[9]) + (S.red[10] + S.red[11]);
                    if (m == 0) st_v += 0.5f * ls / (float)(mb * K);
                    else st_a += ls / (float)mb;
                } else {
                    st_v += 0.5f * (S.red[8] + S.red[10]) / (float)(mb * K);
                    st_a += (S.red[9] + S.red[11]) / (float)mb;
                }
                st_e += ent;
            }
            // ---- Adam (coalesced over the flat parameter vector; padding slots stay 0)
            ++nstep;
            const int stepi = step0 + nstep;
            const double bc1 = 1.0 - pow((double)b1c, (double)stepi);
            const double bc2 = 1.0 - pow((double)b2c, (double)stepi);
            const float step_size = (float)(lr / bc1);
            const float bc2s = (float)sqrt(bc2);
            // flat coalesced pass over this workgroup's parameter ranges (padding slots: g = m = v = 0
            // keeps p = 0); new values land in G.  Critic tensors are [off(critic_w1), off(mean_w)),
            // the actor owns the rest (layout order: actor tower, critic tower, value head, mean head, logstd).
            const int cb = L.off[PGM_P_CRITIC_W1], ce = L.off[PGM_P_MEAN_W];
            for (int rg = 0; rg < 2; ++rg) {
                int lo = 0, hi = L.total;
                if constexpr (SPLIT) {
                    if (m == 0) { lo = rg == 0 ? cb : 0; hi = rg == 0 ? ce : 0; }
                    else { lo = rg == 0 ? 0 : ce; hi = rg == 0 ? cb : L.total; }
                } else if (rg == 1) {
                    hi = 0;
                }
#pragma unroll 4
                for (int i = lo + t; i < hi; i += MT) {
                    const float g = G[i] * coef;
                    float mm = Mo[i], vv = Vo[i];
                    mm = mm + (1.f - b1c) * (g - mm);
                    vv = vv * b2c + (1.f - b2c) * (g * g);
                    const float pn = P[i] - step_size * (mm / (sqrtf(vv) / bc2s + eps));
                    Mo[i] = mm;
                    Vo[i] = vv;
                    P[i] = pn;
                    G[i] = pn;
                }
            }
            lds_sync_m();
            for_each_tensor(S, [&](int tsr, int n, auto slot) {  // refresh the LDS working copy from G
                const bool mine = !SPLIT || ((tsr >= PGM_P_CRITIC_W1 && tsr < PGM_P_MEAN_W) == (m == 0));
                if (!mine) return;
                const int off = L.off[tsr];
                for (int j = t; j < n; j += MT) *slot(j) = G[off + j];
            });
            lds_sync_m();
            PGM_STAMP(3);
        }  // minibatches
    }      // epochs
    if (t == 0) {
        const float n = (float)(E * M);
        if (!SPLIT || m == 0) a.stats[p * 3 + 0] = st_v / n;
        if (!SPLIT || m == 1) {
            a.step[p] = step0 + nstep;
            a.stats[p * 3 + 1] = st_a / n;
            a.stats[p * 3 + 2] = st_e / n;
        }
    }
}

static int device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 1;
    }
    return cus;
}

template <int O, int A, int K>
int launch_ppo_update_mfma(const pgm_dims* d, const MArgs& a, hipStream_t stream) {
    const size_t smem = sizeof(MSmem<O, A, K>);
    if (smem > 160 * 1024) {
        set_error("pgm_ppo_update: LDS image %zu bytes exceeds 160 KiB", smem);
        return PGM_E_UNSUPPORTED;
    }
    if ((size_t)a.L.total > big_floats<O, A, K>()) {
        set_error("pgm_ppo_update: %d parameters exceed the LDS gradient image", a.L.total);
        return PGM_E_UNSUPPORTED;
    }
    // the split needs both workgroups of a task resident at once: one workgroup per CU (LDS + 512
    // registers per lane), so 2P must not exceed the CU count; otherwise run one workgroup per task
    const char* sel = getenv("PGM_UPDATE_SPLIT");
    const bool split = a.ws && 2 * d->P <= device_cus() && !(sel && sel[0] == '0');
    auto kern = split ? ppo_update_mfma_kernel<O, A, K, true> : ppo_update_mfma_kernel<O, A, K, false>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update");
    if (split) {
        e = hipMemsetAsync(a.ws, 0, ppo_workspace_bytes(d->P), stream);
        if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update (workspace reset)");
    }
    hipLaunchKernelGGL(kern, dim3(split ? 2 * d->P : d->P), dim3(MT), smem, stream, a);
    return launch_status("pgm_ppo_update");
}

int ppo_update_mfma(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m, float* adam_v,
                    int32_t* adam_step, const float* lr, const int32_t* perms, const pgm_rollout_buf* rb, float* stats,
                    void* workspace, hipStream_t stream) {
    MArgs a{d->N, d->T, make_layout(d->O, d->A, d->K, d->H), *hp, params, adam_m, adam_v, adam_step, lr, perms,
            rb->obs, rb->actions, rb->logp, rb->values, rb->returns, rb->adv, stats,
            (unsigned long long*)workspace, d->P};
    return dispatch_dims(d->O, d->A, d->K, "pgm_ppo_update", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (O > 32) {
            set_error("pgm_ppo_update: obs_dim %d > 32 not supported by the MFMA update kernel", O);
            return PGM_E_UNSUPPORTED;
        } else {
            return launch_ppo_update_mfma<O, A, K>(d, a, stream);
        }
    });
}

}  // namespace pgm
