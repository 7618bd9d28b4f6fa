// Scalarised clipped-PPO update for WIDE observations (obs_dim > 32: Humanoid's 376) on the f32 matrix
// cores.  Same semantics as pgm_ppo_mfma.hip (a2c_ppo_acktr/algo/ppo.py:58-115, storage.py:118-154,
// model.py:75-82, distributions.py:29-40; torch min/max/clamp tie rules), different data placement:
//
//   * one 256-thread workgroup per tower (critic / actor), the two exchanging the squared gradient norm
//     through one tagged granule per Adam step, as in the narrow kernel's MODE 1;
//   * layer 1 (O x 64 = 96 KB for Humanoid) does not fit LDS next to the rest, so it stays in HBM / L2:
//     the forward reads W1 with sc1 (L1-bypassing) buffer loads, double-buffered in registers 4 k-steps
//     ahead; the minibatch rows are read straight from the rollout buffers (no packed table);
//   * dW1 never goes through LDS: wave w owns the 32-feature tiles kt = w, w + 4, w + 8 of dW1 and keeps
//     their running sums in a per-tower workspace slice that only the owning lane reads and writes; every
//     wave's dZ1 tile is shared through its LDS transpose tile, so each wave contracts its feature tiles
//     over ALL samples of the pass.  Clip and Adam read those sums back (moments in HBM); W1's sum of
//     squares is a register reduction over them;
//   * everything but layer 1 (W2, heads, biases, logstd) is an LDS "small image" with LDS-resident Adam
//     moments, reduced / clipped / updated exactly like the narrow kernel's tower images.
// Layer-1 k-steps pair features (h*KH + ks) of the two lane halves: any bijection between the MFMA's two
// k-slots and the features works as long as the A (X) and B (W1) operands use the same one.
#include <stdlib.h>

#include "pgm_dispatch.hpp"
#include "pgm_mfma.hpp"

namespace pgm {

template <int A, int K>
struct SmallImg {
    static constexpr int Q = qmax<A, K>();
    float W2t[H][SCR];
    float Wh[Q][H];
    float b1[H], b2[H], bh[Q], logstd[A];
};
template <int A, int K>
constexpr int simg_floats() { return (int)(sizeof(SmallImg<A, K>) / sizeof(float)); }

// small-image slot -> flat parameter index (pgm_param_layout order), -1 for padding / unused slots
template <int A, int K>
__device__ __forceinline__ int simg_to_flat(int i, int m, const Layout& L) {
    constexpr int Q = qmax<A, K>();
    constexpr int s2 = H * SCR, s3 = s2 + Q * H, s4 = s3 + H, s5 = s4 + H, s6 = s5 + Q, s7 = s6 + A;
    const int NQ = m == 0 ? K : A;
    if (i < s2) {
        const int in = i / SCR, o = i - in * SCR;
        return o < H ? L.off[m ? PGM_P_ACTOR_W2 : PGM_P_CRITIC_W2] + in * H + o : -1;
    }
    if (i < s3) {  // reference head weight [NQ][H] stored transposed [H][NQ]
        const int j = i - s2, q = j / H, u = j - q * H;
        return q < NQ ? L.off[m ? PGM_P_MEAN_W : PGM_P_VALUE_W] + u * NQ + q : -1;
    }
    if (i < s4) return L.off[m ? PGM_P_ACTOR_B1 : PGM_P_CRITIC_B1] + (i - s3);
    if (i < s5) return L.off[m ? PGM_P_ACTOR_B2 : PGM_P_CRITIC_B2] + (i - s4);
    if (i < s6) return (i - s5) < NQ ? L.off[m ? PGM_P_MEAN_B : PGM_P_VALUE_B] + (i - s5) : -1;
    if (i < s7) return m ? L.off[PGM_P_LOGSTD] + (i - s6) : -1;
    return -1;
}

template <int A, int K>
struct WSmem {
    static constexpr int Q = qmax<A, K>();
    static constexpr int IMG = simg_floats<A, K>();
    SmallImg<A, K> Pm;     // parameters but layer 1
    float MV[2 * IMG];     // Adam exp_avg | exp_avg_sq of the small image
    float dout[4][TS][Q];  // per-wave dL/d(head output) of the current tile
    float aiv[A];          // actor 1 / std^2
    float red[16];
    int32_t rowid[4][TS];  // rollout rows of every wave's tile of the current pass
    union Big {            // per-wave transpose tiles (dZ1 shared at the pass end), gradient images after
        float scr[4][TS][SCR];
        float GA[2][IMG];
    } big;
};

struct WArgs {
    int N, T, P;
    Layout L;
    pgm_ppo_hparams hp;
    float *params, *m, *v;
    int32_t* step;
    const float* lr;
    const int32_t* perms;
    const float *obs, *actions, *logp, *adv, *values, *returns;
    float* stats;
    unsigned long long* ws;  // [2P] tagged norm granules + timeout flag (word 2P), zeroed before the launch
    float* dw1;              // [P][2][ceil(O/32)*32][H] layer-1 gradient running sums (workspace)
};

template <int O, int A, int K>
__global__ __launch_bounds__(MT) void ppo_update_wide_kernel(WArgs a) {
    static_assert(O > 32 && O % 8 == 0, "wide kernel: obs_dim > 32, multiple of 8 (float4 halves)");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    using Sm = WSmem<A, K>;
    auto& S = *reinterpret_cast<Sm*>(smem_raw);
    constexpr int Q = qmax<A, K>();
    constexpr int IMG = Sm::IMG;
    constexpr int KH = O / 2;                  // layer-1 k-steps: lane half h covers features [h*KH, h*KH + KH)
    constexpr int KG = 4;                      // k-steps per register group (one float4 of X per lane)
    constexpr int NG = KH / KG;
    static_assert(NG * KG == KH, "KH multiple of 4");
    constexpr int NKT = (O + TS - 1) / TS;     // 32-feature tiles of dW1
    constexpr int NKW = (NKT + 3) / 4;         // tiles owned per wave: kt = w + 4j
    constexpr int oWh = H * SCR, oB1 = oWh + Q * H, oB2 = oB1 + H, oBh = oB2 + H, oLs = oBh + Q;
    const int t = threadIdx.x, w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const int p = (int)(blockIdx.x >> 1), m = (int)(blockIdx.x & 1);
    const int NQ = m == 0 ? K : A;
    const int N = a.N, T = a.T, B = T * N;
    const int E = a.hp.ppo_epoch, M = a.hp.num_mini_batch;
    const int mb = B / M, nb = B / mb;
    const int npass = (mb + 4 * TS - 1) / (4 * TS);
    const float clip = a.hp.clip_param;
    const Layout& L = a.L;
    float* __restrict__ P = a.params + (size_t)p * L.total;
    float* __restrict__ Mo = a.m + (size_t)p * L.total;
    float* __restrict__ Vo = a.v + (size_t)p * L.total;
    const int offW1 = L.off[m ? PGM_P_ACTOR_W1 : PGM_P_CRITIC_W1];
    float* __restrict__ dw1 = a.dw1 + (size_t)(p * 2 + m) * NKT * TS * H;  // this tower's dW1 running sums
    const float* obs = a.obs + (size_t)p * (T + 1) * N * O;
    const float* acts = a.actions + (size_t)p * B * A;
    const float* oldlp = a.logp + (size_t)p * B;
    const float* advs = a.adv + (size_t)p * B;
    const float* vals = a.values + (size_t)p * (T + 1) * N * K;
    const float* rets = a.returns + (size_t)p * (T + 1) * N * K;
    // this task's parameters as a buffer: layer-1 weights are re-read every tile with sc1 (L2) loads
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(P, 0, L.total * 4, 0x00020000);
    constexpr int SC1 = 16;
    auto w1 = [&](int k, int col) {  // W1^T[k][col] from L2
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(prs, (offW1 + k * H + col) * 4, 0, SC1));
    };

    // ---- small image + its Adam moments
    float* Pf = &S.Pm.W2t[0][0];
    if (t < A) S.aiv[t] = expf(-2.f * P[L.off[PGM_P_LOGSTD] + t]);
    for (int i = t; i < IMG; i += MT) {
        const int f = simg_to_flat<A, K>(i, m, L);
        Pf[i] = f >= 0 ? P[f] : 0.f;
        S.MV[i] = f >= 0 ? Mo[f] : 0.f;
        S.MV[IMG + i] = f >= 0 ? Vo[f] : 0.f;
    }
    __syncthreads();
    auto& W = S.Pm;
    const float* lstd = S.Pm.logstd;  // actor logstd (critic: zeros, unused)

    const int step0 = a.step[p];
    const double lr = a.lr[p];
    const float b1c = a.hp.beta1, b2c = a.hp.beta2, eps = a.hp.adam_eps;
    const float vscale = a.hp.value_loss_coef * 0.5f / (float)(mb * K);
    const float ascale = -1.f / (float)mb;
    float st_v = 0.f, st_a = 0.f, st_e = 0.f;
    int nstep = 0;
    double b1p = pow((double)b1c, (double)step0), b2p = pow((double)b2c, (double)step0);
    float* scr = &S.big.scr[w][0][0];

    for (int e = 0; e < E; ++e) {
        for (int bb = 0; bb < nb; ++bb) {
            const int32_t* perm = a.perms + (size_t)e * B + bb * mb;
            f32x16 gW2[2][2];
            float gWh[2][Q], gB1[2], gB2[2], gBh[Q], gLs[A];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j) gW2[i][j] = f32x16{0};
                gB1[i] = gB2[i] = 0.f;
#pragma unroll
                for (int q = 0; q < Q; ++q) gWh[i][q] = 0.f;
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) gBh[q] = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) gLs[q] = 0.f;
            float lsum = 0.f;

            for (int ps = 0; ps < npass; ++ps) {
                const int i0 = (ps * 4 + w) * TS;  // this wave's tile of the pass
                const int si = i0 + c;
                const bool ok = si < mb;
                const int row = perm[min(si, mb - 1)];
                if (h == 0) S.rowid[w][c] = row;
                if (i0 < mb) {  // wave-uniform
                    // ---- layer 1 from L2: Z1[s][u] = sum_k X[s][k] W1t[k][u], X row of sample c, features
                    // h*KH + ks; register groups of KG k-steps loaded one group ahead
                    const float4* xr = reinterpret_cast<const float4*>(obs + (size_t)row * O + h * KH);
                    f32x16 z[2] = {f32x16{0}, f32x16{0}};
                    float4 xa = xr[0];
                    float wa[KG][2];
#pragma unroll
                    for (int q = 0; q < KG; ++q) {
                        wa[q][0] = w1(h * KH + q, c);
                        wa[q][1] = w1(h * KH + q, TS + c);
                    }
#pragma unroll 1
                    for (int g = 0; g < NG; ++g) {
                        float4 xn = xa;
                        float wn[KG][2];
                        if (g + 1 < NG) {
                            xn = xr[g + 1];
#pragma unroll
                            for (int q = 0; q < KG; ++q) {
                                wn[q][0] = w1(h * KH + (g + 1) * KG + q, c);
                                wn[q][1] = w1(h * KH + (g + 1) * KG + q, TS + c);
                            }
                        }
                        const float xv[4] = {xa.x, xa.y, xa.z, xa.w};
#pragma unroll
                        for (int q = 0; q < KG; ++q) {
                            z[0] = mfma(xv[q], wa[q][0], z[0]);
                            z[1] = mfma(xv[q], wa[q][1], z[1]);
                        }
                        xa = xn;
#pragma unroll
                        for (int q = 0; q < KG; ++q) {
                            wa[q][0] = wn[q][0];
                            wa[q][1] = wn[q][1];
                        }
                    }
                    f32x16 H1[2];
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb) {
                        const float bias = W.b1[hb * TS + c];
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            H1[hb][r] = tanh_fast(z[hb][r] + bias);
                            scr[rowof(r, h) * SCR + hb * TS + c] = H1[hb][r];
                        }
                    }
                    wave_lds_fence();
                    // ---- layer 2 (A from the transpose tile)
                    z[0] = z[1] = f32x16{0};
#pragma unroll 8
                    for (int ks = 0; ks < H / 2; ++ks) {
                        const int k = 2 * ks + h;
                        const float av = scr[c * SCR + k];
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob) z[ob] = mfma(av, W.W2t[k][ob * TS + c], z[ob]);
                    }
                    f32x16 H2[2];
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob) {
                        const float bias = W.b2[ob * TS + c];
#pragma unroll
                        for (int r = 0; r < 16; ++r) H2[ob][r] = tanh_fast(z[ob][r] + bias);
                    }
                    wave_lds_fence();
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ob * TS + c] = H2[ob][r];
                    wave_lds_fence();
                    // ---- heads (VALU): lane = sample c, half h sums units [32h, 32h+32)
                    float outv[Q];
#pragma unroll
                    for (int q = 0; q < Q; ++q) outv[q] = 0.f;
#pragma unroll 4
                    for (int u = 0; u < TS; ++u) {
                        const float hv = scr[c * SCR + h * TS + u];
#pragma unroll
                        for (int q = 0; q < Q; ++q) outv[q] = fmaf(hv, W.Wh[q][h * TS + u], outv[q]);
                    }
#pragma unroll
                    for (int q = 0; q < Q; ++q) outv[q] = half_sum(outv[q]) + W.bh[q];
                    // ---- per-sample loss gradients (ppo.py:80-96)
                    float dO[Q];
#pragma unroll
                    for (int q = 0; q < Q; ++q) dO[q] = 0.f;
                    if (m == 0) {  // value loss
                        float ls = 0.f;
#pragma unroll
                        for (int q = 0; q < K; ++q) {
                            const float V = outv[q], Vp = vals[(size_t)row * K + q], R = rets[(size_t)row * K + q];
                            float gv;
                            if (a.hp.use_clipped_value_loss) {
                                const float dv = V - Vp;
                                const float vc = Vp + fminf(fmaxf(dv, -clip), clip);
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
                        float act[A];
#pragma unroll
                        for (int q = 0; q < A; ++q) act[q] = acts[(size_t)row * A + q];
                        const float lpo = oldlp[row], ad = advs[row];
                        float lp = 0.f;
#pragma unroll
                        for (int q = 0; q < A; ++q) {
                            const float diff = act[q] - outv[q];
                            lp += -0.5f * diff * diff * S.aiv[q] - lstd[q] - LOG_SQRT_2PI;
                        }
                        const float ratio = expf(lp - lpo);
                        const float s1 = ratio * ad;
                        const float s2 = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip) * ad;
                        const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
                        const float gr = ad * (wmin2(s1, s2) + wmin2(s2, s1) * inr);
                        const float dlp = ok ? ascale * gr * ratio : 0.f;
                        if (ok && h == 0) lsum += -fminf(s1, s2);
#pragma unroll
                        for (int q = 0; q < A; ++q) {
                            const float diff = act[q] - outv[q];
                            const float iv = S.aiv[q];
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
                    // ---- head-weight grads (VALU, C layout); one dO row per register, scheduling fences keep the
                    // Q-wide row loads from being hoisted (Q = 17 would not fit the register file)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int s = rowof(r, h);
                        float dv[Q];
#pragma unroll
                        for (int q = 0; q < Q; ++q) dv[q] = S.dout[w][s][q];
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                            for (int q = 0; q < Q; ++q) gWh[ob][q] = fmaf(H2[ob][r], dv[q], gWh[ob][q]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    // ---- dH2 = dO . Wh (MFMA) -> dZ2; dW2^T += H1^T dZ2
                    z[0] = z[1] = f32x16{0};
#pragma unroll
                    for (int ks = 0; ks < (Q + 1) / 2; ++ks) {
                        const int q = 2 * ks + h;
                        const float av = h ? (2 * ks + 1 < Q ? dO[2 * ks + 1] : 0.f) : dO[2 * ks];
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob) z[ob] = mfma(av, q < Q ? W.Wh[q][ob * TS + c] : 0.f, z[ob]);
                    }
                    f32x16 dZ2[2];
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            dZ2[ob][r] = z[ob][r] * (1.f - H2[ob][r] * H2[ob][r]);
                            gB2[ob] += dZ2[ob][r];
                        }
#pragma unroll
                    for (int r = 0; r < 16; ++r)
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                            for (int ob = 0; ob < 2; ++ob) gW2[ib][ob] = mfma(H1[ib][r], dZ2[ob][r], gW2[ib][ob]);
                    // ---- dH1 = dZ2 W2 -> dZ1
                    wave_lds_fence();
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ob * TS + c] = dZ2[ob][r];
                    wave_lds_fence();
                    z[0] = z[1] = f32x16{0};
#pragma unroll 8
                    for (int ks = 0; ks < H / 2; ++ks) {
                        const int k = 2 * ks + h;
                        const float av = scr[c * SCR + k];
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib) z[ib] = mfma(av, W.W2t[ib * TS + c][k], z[ib]);
                    }
                    f32x16 dZ1[2];
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            dZ1[ib][r] = z[ib][r] * (1.f - H1[ib][r] * H1[ib][r]);
                            gB1[ib] += dZ1[ib][r];
                        }
                    // ---- dZ1 to this wave's transpose tile: every wave contracts it with its dW1 tiles
                    wave_lds_fence();
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ib * TS + c] = dZ1[ib][r];
                }
                lds_sync_m();  // every tile's dZ1 and rows visible
                // ---- dW1^T[k][u] += X^T dZ1 over the pass's tiles, for this wave's feature tiles.  The running
                // sums live in the workspace (each element read and written only by its owning lane), one
                // 32-feature tile in registers at a time
                {
                    int rw[4][16];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int r = 0; r < 16; ++r) rw[u][r] = S.rowid[u][rowof(r, h)];
                    const int nu = min(4, (mb - ps * 4 * TS + TS - 1) / TS);  // tiles of this pass
#pragma unroll 1
                    for (int j = 0; j < NKW; ++j) {
                        const int kt = w + 4 * j;
                        if (kt >= NKT) break;
                        const int kf = kt * TS + c;
                        float* gp = dw1 + (size_t)(kt * TS) * H + c;
                        f32x16 acc[2];
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                            for (int r = 0; r < 16; ++r) acc[ib][r] = ps == 0 ? 0.f : gp[rowof(r, h) * H + ib * TS];
#pragma unroll 1
                        for (int u = 0; u < nu; ++u) {
                            const float* dz = &S.big.scr[u][0][0];
                            float xv[16];
#pragma unroll
                            for (int r = 0; r < 16; ++r) xv[r] = kf < O ? obs[(size_t)rw[u][r] * O + kf] : 0.f;
#pragma unroll
                            for (int r = 0; r < 16; ++r) {
                                const int s = rowof(r, h);
#pragma unroll
                                for (int ib = 0; ib < 2; ++ib) acc[ib] = mfma(xv[r], dz[s * SCR + ib * TS + c], acc[ib]);
                            }
                        }
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                            for (int r = 0; r < 16; ++r) gp[rowof(r, h) * H + ib * TS] = acc[ib][r];
                    }
                }
                lds_sync_m();  // transpose tiles / row ids reused by the next pass
            }  // passes

            // ---- lane halves of the per-column partial sums; 64-lane sums of the per-sample ones
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                gB1[i] = half_sum(gB1[i]);
                gB2[i] = half_sum(gB2[i]);
#pragma unroll
                for (int q = 0; q < Q; ++q) gWh[i][q] = half_sum(gWh[i][q]);
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) gBh[q] = wave_sum64(gBh[q]);
#pragma unroll
            for (int q = 0; q < A; ++q) gLs[q] = wave_sum64(gLs[q]);
            lsum = wave_sum64(lsum);
            float ent = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) ent += 0.5f + LOG_SQRT_2PI + lstd[q];

            // ---- small-image gradients: waves 1 / 3 store into GA[0] / GA[1], then waves 0 / 2 add theirs
            for (int stage = 0; stage < 2; ++stage) {
                if ((w & 1) != stage) {
                    float* Gt = S.big.GA[w >> 1];
                    const bool add = stage == 1;
                    auto acc = [&](int idx, float val) { Gt[idx] = add ? Gt[idx] + val : val; };
                    auto acc16 = [&](auto idx, const f32x16& val) {
                        if (add) {
                            float tmp[16];
#pragma unroll
                            for (int r = 0; r < 16; ++r) tmp[r] = Gt[idx(r)];
#pragma unroll
                            for (int r = 0; r < 16; ++r) Gt[idx(r)] = tmp[r] + val[r];
                        } else {
#pragma unroll
                            for (int r = 0; r < 16; ++r) Gt[idx(r)] = val[r];
                        }
                    };
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob)
                            acc16([&](int r) { return (ib * TS + rowof(r, h)) * SCR + ob * TS + c; }, gW2[ib][ob]);
                    if (h == 0) {
#pragma unroll
                        for (int i = 0; i < 2; ++i) {
                            acc(oB1 + i * TS + c, gB1[i]);
                            acc(oB2 + i * TS + c, gB2[i]);
#pragma unroll
                            for (int q = 0; q < Q; ++q) acc(oWh + q * H + i * TS + c, q < NQ ? gWh[i][q] : 0.f);
                        }
                    }
                    if (l == 0) {
#pragma unroll
                        for (int q = 0; q < Q; ++q)
                            if (q < NQ) acc(oBh + q, gBh[q]);
                        if (m == 1) {  // -entropy_coef * d(mean entropy)/d logstd enters once (ppo.py:98)
                            const float ec = add ? 0.f : a.hp.entropy_coef;
#pragma unroll
                            for (int q = 0; q < A; ++q) acc(oLs + q, gLs[q] - ec);
                        }
                        S.red[8 + w] = lsum;
                    }
                    if (!add) {  // padding slots of a freshly written image
                        Gt[l * SCR + H] = 0.f;
                        if (l >= NQ && l < Q) Gt[oBh + l] = 0.f;
                        if (m == 0 && l < A) Gt[oLs + l] = 0.f;
                    }
                }
                lds_sync_m();
            }
            // ---- clip_grad_norm_: small image + this wave's dW1 registers
            const float* GA0 = S.big.GA[0];
            const float* GA1 = S.big.GA[1];
            float sq = 0.f;
            for (int i = t; i < IMG; i += MT) {
                const float g = GA0[i] + GA1[i];
                sq = fmaf(g, g, sq);
            }
            for (int j = 0; j < NKW; ++j) {  // this wave's dW1 tiles (rows k >= O hold zeros)
                const int kt = w + 4 * j;
                if (kt >= NKT) break;
                const float* gp = dw1 + (size_t)(kt * TS) * H + c;
#pragma unroll
                for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float g = gp[rowof(r, h) * H + ib * TS];
                        sq = fmaf(g, g, sq);
                    }
            }
            sq = wave_sum64(sq);
            if (l == 0) S.red[w] = sq;
            lds_sync_m();
            float total = (S.red[0] + S.red[1]) + (S.red[2] + S.red[3]);
            if (t == 0) {  // tagged 8-byte granule hand-off with the other tower's workgroup
                const unsigned tag = (unsigned)(nstep + 1);
                unsigned long long* ws = a.ws + 2 * p;
                __hip_atomic_store(ws + m, ((unsigned long long)tag << 32) | __float_as_uint(total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                unsigned long long x = 0;
                const bool failed = __hip_atomic_load(a.ws + 2 * a.P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (unsigned spins = 0; !failed; ++spins) {
                    x = __hip_atomic_load(ws + (1 - m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((unsigned)(x >> 32) == tag) break;
                    if (spins > (1u << 26)) {
                        __hip_atomic_store(a.ws + 2 * a.P, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        x = 0;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                const float other = __uint_as_float((unsigned)x);
                S.red[4] = m == 0 ? total + other : other + total;
            }
            lds_sync_m();
            total = S.red[4];
            const float coef = fminf(a.hp.max_grad_norm / (sqrtf(total) + 1e-6f), 1.f);
            if (t == 0) {
                const float ls = (S.red[8] + S.red[9]) + (S.red[10] + S.red[11]);
                if (m == 0) st_v += 0.5f * ls / (float)(mb * K);
                else st_a += ls / (float)mb;
                st_e += ent;
            }
            // ---- Adam: the small image in LDS, layer 1 from the owning wave's registers (moments in HBM)
            ++nstep;
            b1p *= (double)b1c;
            b2p *= (double)b2c;
            const float step_size = (float)(lr / (1.0 - b1p));
            const float inv_bc2s = 1.f / (float)sqrt(1.0 - b2p);
            auto adam = [&](float g, float& mm, float& vv, float& pp) {
                const float gc = g * coef;
                mm = mm + (1.f - b1c) * (gc - mm);
                vv = vv * b2c + (1.f - b2c) * (gc * gc);
                const float den = __builtin_amdgcn_sqrtf(vv) * inv_bc2s + eps;
                pp -= step_size * mm * __builtin_amdgcn_rcpf(den);
            };
            for (int i = t; i < IMG; i += MT) {
                float mm = S.MV[i], vv = S.MV[IMG + i], pp = Pf[i];
                adam(GA0[i] + GA1[i], mm, vv, pp);
                S.MV[i] = mm;
                S.MV[IMG + i] = vv;
                Pf[i] = pp;
                if (m == 1 && i >= oLs && i < oLs + A) S.aiv[i - oLs] = expf(-2.f * pp);
            }
#pragma unroll
            for (int j = 0; j < NKW; ++j) {
                const int kt = w + 4 * j;
                if (kt >= NKT) break;
                const float* gp = dw1 + (size_t)(kt * TS) * H + c;
#pragma unroll
                for (int ib = 0; ib < 2; ++ib) {
                    float mm[16], vv[16], pp[16], gg[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int k = min(kt * TS + rowof(r, h), O - 1);
                        const int f = offW1 + k * H + ib * TS + c;
                        mm[r] = Mo[f];
                        vv[r] = Vo[f];
                        pp[r] = P[f];
                        gg[r] = gp[rowof(r, h) * H + ib * TS];
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int k = kt * TS + rowof(r, h);
                        if (k >= O) continue;
                        const int f = offW1 + k * H + ib * TS + c;
                        adam(gg[r], mm[r], vv[r], pp[r]);
                        Mo[f] = mm[r];
                        Vo[f] = vv[r];
                        P[f] = pp[r];
                    }
                    __builtin_amdgcn_sched_barrier(0);  // one 16-element block of loads in flight at a time
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // layer-1 stores land in L2 before any re-read
            lds_sync_m();
        }  // minibatches
    }      // epochs
    // ---- write back the small image (layer 1 was updated in place)
    for (int i = t; i < IMG; i += MT) {
        const int f = simg_to_flat<A, K>(i, m, L);
        if (f < 0) continue;
        P[f] = Pf[i];
        Mo[f] = S.MV[i];
        Vo[f] = S.MV[IMG + i];
    }
    if (t == 0) {
        const float n = (float)(E * M);
        if (m == 0) a.stats[p * 3 + 0] = st_v / n;
        if (m == 1) {
            a.step[p] = step0 + nstep;
            a.stats[p * 3 + 1] = st_a / n;
            a.stats[p * 3 + 2] = st_e / n;
        }
    }
}

int ppo_update_wide(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m, float* adam_v,
                    int32_t* adam_step, const float* lr, const int32_t* perms, const pgm_rollout_buf* rb, float* stats,
                    void* workspace, hipStream_t stream) {
    if (!workspace) {
        set_error("pgm_ppo_update: the wide update needs the workspace (pgm_ppo_update_workspace_bytes)");
        return PGM_E_INVALID_ARG;
    }
    if (2 * d->P > device_cu_count()) {
        set_error("pgm_ppo_update: the wide update needs 2P <= CUs (P=%d); shard the tasks over more GPUs", d->P);
        return PGM_E_UNSUPPORTED;
    }
    WArgs a{d->N, d->T, d->P, make_layout(d->O, d->A, d->K, d->H), *hp, params, adam_m, adam_v, adam_step, lr, perms,
            rb->obs, rb->actions, rb->logp, rb->adv, rb->values, rb->returns, stats, (unsigned long long*)workspace,
            (float*)((char*)workspace + ppo_flag_bytes(d->P))};
    return dispatch_dims(d->O, d->A, d->K, "pgm_ppo_update", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (O <= 32 || O % 8 != 0) {
            set_error("pgm_ppo_update: obs_dim %d outside the wide kernel", O);
            return PGM_E_UNSUPPORTED;
        } else {
            const size_t smem = sizeof(WSmem<A, K>);
            static_assert(sizeof(WSmem<A, K>) > 80 * 1024 || O <= 32, "residency argument needs > 80 KiB LDS");
            if (smem > 160 * 1024) {
                set_error("pgm_ppo_update: LDS image %zu bytes exceeds 160 KiB", smem);
                return PGM_E_UNSUPPORTED;
            }
            auto kern = ppo_update_wide_kernel<O, A, K>;
            hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update");
            e = hipMemsetAsync(workspace, 0, ppo_flag_bytes(d->P), stream);
            if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update (workspace reset)");
            hipLaunchKernelGGL(kern, dim3(2 * d->P), dim3(MT), smem, stream, a);
            return launch_status("pgm_ppo_update");
        }
    });
}

}  // namespace pgm
