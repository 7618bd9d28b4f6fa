// Scalarised clipped-PPO update for WIDE observations (obs_dim > 32: Humanoid's 376) on the f32 matrix
// cores.  Same semantics as pgm_ppo_mfma.hip (a2c_ppo_acktr/algo/ppo.py:58-115, storage.py:118-154,
// model.py:75-82, distributions.py:29-40; torch min/max/clamp tie rules), different data placement:
//
//   * each tower (critic / actor) on NS workgroups (NS = 4 while 32 ceil(P/4) <= CUs, else 2 while
//     16 ceil(P/4) <= CUs, else 1): each takes 1/NS of every minibatch's rows, in passes of 128 rows (one
//     32-row MFMA tile per wave); the NS gradient images (small image + dW1) are added through a 16-B sc1
//     publish + tagged flag hand-off (cdna_hip_programming.md G16 R1), every part sums them in part order
//     0..NS-1, so the NS Adam steps stay bitwise identical; the two towers exchange the squared gradient
//     norm through one tagged granule per (step, row part) (the narrow kernel's protocol);
//   * layer 1 (O x 64 = 96 KB) does not fit LDS next to the rest: the forward streams W1 through L1 (the
//     four waves read the same rows) and the observation rows straight from the rollout buffer (float4 per
//     lane), both three 4-k-step groups ahead of the MFMAs; the rows were touched into L2 one Adam step
//     earlier, under the previous step's exchange.  Layer-1 k-steps pair features (h*KH + ks) of the two
//     lane halves: any bijection between the MFMA's two k-slots and the features works as long as the A (X)
//     and B (W1) operands use the same one;
//   * dW1 stays in REGISTERS: wave w owns the 32-feature tiles kt = w, w + 4, w + 8 of dW1 (96 accumulator
//     registers) for the whole minibatch; every wave's dZ1 tile is shared through its LDS transpose tile, so
//     each wave contracts its feature tiles over ALL samples of a pass, the observation values gathered from
//     HBM one (tile, feature-tile) ahead.  Clip and Adam read those registers directly (moments in HBM);
//   * everything but layer 1 (W2, heads, biases, logstd) is an LDS "small image" with LDS-resident Adam
//     moments, reduced / clipped / updated like the narrow kernel's tower images; the head-weight gradient
//     is an MFMA with the per-sample head gradients transposed through LDS.
// Layer 1 (the bulk of the parameters) is sharded over the NS parts for the clip / Adam step: every part
// sums, clips and updates only its slice of dW1 and hands the new weights to the others, which write them
// into their own layer-1 copy.  Every workgroup streams W1 from a private copy in the workspace in k-quad
// layout ([O/4][H][4]: a lane's four consecutive k-rows of one column are one 16-B load, a quarter of the
// 4-B loads of the caller's row layout; the Adam slice and the partners' slices are 16-B accesses too), so no
// part reads weights another is rewriting; part 0 writes layer 1 back to the caller's row at the end.
#include <stdio.h>
#include <stdlib.h>

#include "pgm_dispatch.hpp"
#include "pgm_mfma.hpp"

PGM_STAMP_UNIT(wupd)

// unroll depth of the layer-2 / dH1 loops (deeper unrolls: spills unchanged or higher)
#define PGM_PRAGMA_W(x) _Pragma(#x)
#define PGM_UNROLL_W(n) PGM_PRAGMA_W(unroll n)
#define PGM_UW_L2 8
// block map: the two towers of a row part on one XCD (they read the same observation rows in the same phase, so the
// second read hits that XCD's L2): Humanoid P = 20 update 31.1 -> 30.4 ms, 56.2 -> 47.8 GB per launch against the
// round-2 map, the NS parts of one tower on one XCD (profiles/r03o_*)
// (the VALU heads and elementwise tanh on register pairs through the packed fp32 ALU, as in the narrow kernels, made
// this kernel slower: 30.4 -> 33.3 ms at Humanoid P = 20, it already runs at the 512-register limit)
// (all 2 NS workgroups of a task on one XCD, groups of 8 tasks: 30.4 -> 30.6-30.7 ms, kept out)
namespace pgm {
inline int wide_grid(int P, int NS) { return NS == 1 ? 2 * P : 8 * NS * ((P + 3) / 4); }
}  // namespace pgm

namespace pgm {

namespace {

constexpr int WHS = H + 4;  // head-weight row stride: 16-B rows (the VALU heads read them as b128) whose starts
                            // fall on 8 bank quads (the reduction's column writes, lane = output q: 3-way, not 17-way)
template <int A, int K>
struct SmallImg {
    static constexpr int Q = qmax<A, K>();
    float W2t[H][SCR];
    float Wh[Q][WHS];
    float b1[H], b2[H], bh[Q], logstd[A];
};
template <int A, int K>
constexpr int simg_floats() { return (int)(sizeof(SmallImg<A, K>) / sizeof(float)); }

// small-image slot -> flat parameter index (pgm_param_layout order), -1 for padding / unused slots
template <int A, int K>
__device__ __forceinline__ int simg_to_flat(int i, int m, const Layout& L) {
    constexpr int Q = qmax<A, K>();
    constexpr int s2 = H * SCR, s3 = s2 + Q * WHS, s4 = s3 + H, s5 = s4 + H, s6 = s5 + Q, s7 = s6 + A;
    const int NQ = m == 0 ? K : A;
    if (i < s2) {
        const int in = i / SCR, o = i - in * SCR;
        return o < H ? L.off[m ? PGM_P_ACTOR_W2 : PGM_P_CRITIC_W2] + in * H + o : -1;
    }
    if (i < s3) {  // reference head weight [NQ][H] stored transposed [H][NQ] (rows padded to WHS)
        const int j = i - s2, q = j / WHS, u = j - q * WHS;
        return q < NQ && u < H ? L.off[m ? PGM_P_MEAN_W : PGM_P_VALUE_W] + u * NQ + q : -1;
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
    float dls[4][TS][Q];   // per-wave per-sample dL/d(logstd) of the current tile (actor)
    float aiv[A];          // actor 1 / std^2
    float red[32];  // [0,4) wave sums of squares, 4 norm total, [8,12) wave loss sums, 12 loss total,
                    // [16, 16 + 2 NS) norm parts, [24, 24 + NS) loss parts (one polling lane each)
    int32_t rowid[4][TS];  // rollout rows of every wave's tile of the current pass
    int32_t nrowid[4][TS];  // ... of the next minibatch's first pass (prefetched into L2 under the exchange)
    float act2[4][TS][SCR];  // per-wave tile B: H2, then dZ2
    union Big {            // per-wave transpose tiles (dZ1 shared at the pass end), gradient images after
        float scr[4][TS][SCR];
        float GA[2][IMG];
    } big;
};

constexpr int WSPLIT = 16;  // cache-policy aux bit of the buffer builtins: sc1

// A per-lane base value the optimiser cannot see through: addresses derived from it stay base + constant
// (one VGPR) instead of being hoisted out of the step loop as one precomputed VGPR per element.
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

struct WArgs {
    int N, T, P;
    Layout L;
    pgm_ppo_hparams hp;
    float *params, *m, *v;  // caller's arrays (half 0)
    float* copies;          // every workgroup's layer-1 copy, k-quad layout [P][2 towers][NS parts][O H]
    int32_t* step;
    const float* lr;
    const int32_t* perms;
    const float *obs, *actions, *logp, *adv, *values, *returns;
    float* stats;
    unsigned long long* ws;  // tagged norm granules + timeout flag (word 2P), zeroed before the launch
    unsigned long long* xb;  // NS > 1: gradient exchange slots [P][2 towers][NS parts][2 parities][xslot]
    int xslot;               // 8-byte words per exchange slot (image | dW1 | flag granule)
    int xbytes;
};

}  // namespace

// exchange-slot geometry shared with the host-side workspace size (pgm_common.hpp declares it)
int wide_xslot_words(int O, int A, int K) {
    const int Q = A > K ? A : K;
    const int img = H * (H + 1) + Q * WHS + 2 * H + Q + A;
    const int nkt = (O + 31) / 32;
    const int nkw = (nkt + 3) / 4;
    // small image (+ padding to 16 B) | dW1 block | new-W1 slices [2 nkw][16/NS][256 threads] (NS >= 2) | 2 flag granules
    return ((img + 4 + nkt * 32 * H + nkw * 16 * 256 + 1) / 2 + 2 + 31) / 32 * 32;  // 8-byte words, 256-B aligned
}

namespace {

// ONE: mb = NS * 4 * 32 (each wave owns exactly one 32-row tile of one pass per minibatch; Humanoid N = 8, NS = 4):
// the pass loop is straight-line, so the gradient accumulators are not loop-carried
template <int O, int A, int K, int NS, bool ONE>
__global__ __launch_bounds__(MT) void ppo_update_wide_kernel(WArgs a) {
    static_assert(O > 32 && O % 8 == 0, "wide kernel: obs_dim > 32, multiple of 8 (float4 halves)");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    using Sm = WSmem<A, K>;
    auto& S = *reinterpret_cast<Sm*>(smem_raw);
    constexpr int Q = qmax<A, K>();
    constexpr int IMG = Sm::IMG;
    constexpr int KH = O / 2;              // layer-1 k-steps: lane half h covers features [h*KH, h*KH + KH)
    constexpr int KG = 4;                  // k-steps per group (one float4 of X per lane)
    constexpr int NG = KH / KG;
    static_assert(NG * KG == KH, "KH multiple of 4");
    constexpr int NKT = (O + TS - 1) / TS;  // 32-feature tiles of dW1
    constexpr int NKW = (NKT + 3) / 4;      // tiles owned per wave: kt = w + 4j
    constexpr int oWh = H * SCR, oB1 = oWh + Q * WHS, oB2 = oB1 + H, oBh = oB2 + H, oLs = oBh + Q;
    const int t = threadIdx.x, w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    // block map (NS > 1), groups of 8 NS blocks for 4 tasks; blocks b, b + 8, ... share an XCD under round-robin
    // dispatch (speed only: every hand-off is correct under any placement)
    const int bx = (int)blockIdx.x;
    const int r8 = bx % (8 * NS);
    // co-located map (NS > 1): XCD slot x = r8 & 7 holds task 4g + (x >> 1) and BOTH towers of its parts
    // (NS = 4: parts 2 (x & 1), 2 (x & 1) + 1; NS = 2: part x & 1), so the critic and actor workgroups of a row part --
    // which read the same observation rows in the same phase, kept in step by the per-step norm hand-off -- share one L2
    const int x8 = r8 & 7, j8 = r8 >> 3;
    const int p = NS > 1 ? 4 * (bx / (8 * NS)) + (x8 >> 1) : (bx >> 1);
    const int hs = NS == 4 ? 2 * (x8 & 1) + (j8 >> 1) : NS == 2 ? (x8 & 1) : 0;
    if (p >= a.P) return;
    const int m = NS > 1 ? (j8 & 1) : (bx & 1);
    const int NQ = m == 0 ? K : A;
    const int N = a.N, T = a.T, B = T * N;
    const int E = a.hp.ppo_epoch, M = a.hp.num_mini_batch;
    const int mb = B / M, nb = B / mb;
    const int r0 = hs * mb / NS, mbs = (hs + 1) * mb / NS - r0;  // this workgroup's rows of each minibatch
    const int npass = (mbs + 4 * TS - 1) / (4 * TS);
    const float clip = a.hp.clip_param;
    const Layout& L = a.L;
    // parameters: part 0 the caller's row, parts 1..NS-1 private copies; Adam moments: the caller's rows for
    // every part (layer-1 elements are owned by one part each; the small image is written back by part 0 only)
    // parameters: the caller's row (the small image is read from it by every part, written back by part 0); layer 1
    // lives in a private copy per workgroup in k-quad layout [O / 4][H][4] (W1^T[k][u] at (k / 4 H + u) 4 + k % 4),
    // so a lane's four consecutive k-rows of one column are one 16-B load; part 0 writes it back at the end
    float* __restrict__ P = a.params + (size_t)p * L.total;
    float* __restrict__ Wq = a.copies + (((size_t)p * 2 + m) * NS + hs) * (size_t)(O * H);
    auto qidx = [](int k, int u) { return ((k >> 2) * H + u) * 4 + (k & 3); };
    float* __restrict__ Mo = a.m + (size_t)p * L.total;
    float* __restrict__ Vo = a.v + (size_t)p * L.total;
    const int offW1 = L.off[m ? PGM_P_ACTOR_W1 : PGM_P_CRITIC_W1];
    const float* obs = a.obs + (size_t)p * (T + 1) * N * O;
    const float* acts = a.actions + (size_t)p * B * A;
    const float* oldlp = a.logp + (size_t)p * B;
    const float* advs = a.adv + (size_t)p * B;
    const float* vals = a.values + (size_t)p * (T + 1) * N * K;
    const float* rets = a.returns + (size_t)p * (T + 1) * N * K;
    // this workgroup's parameters as a buffer: layer-1 weights are re-read every tile with sc1 (L2) loads
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(Wq, 0, O * H * 4, 0x00020000);
    auto w1q = [&](int kq, int col) {  // W1^T[4 kq .. 4 kq + 3][col]: through L1 (the 4 waves stream the same rows)
        return __builtin_amdgcn_raw_buffer_load_b128(wrs, (kq * H + col) * 16, 0, 0);
    };
    // the task's observation rows as a buffer: a padding or dead element is a load at byte offset XOOB, past the
    // range, which the hardware returns as 0.  (A select `ok ? load : 0` on the loaded value -- or a load under an
    // exec mask -- made the compiler wait for the load right after issuing it: the layer-1 stream's X loads and the
    // dW1 gather each lost their lookahead.)
    constexpr int XOOB = (int)0x80000000u;
    const __amdgpu_buffer_rsrc_t ors =
        __builtin_amdgcn_make_buffer_rsrc((void*)obs, 0, (T + 1) * N * O * (int)sizeof(float), 0x00020000);

    // ---- this workgroup's layer-1 copy (k-quad layout) from the caller's W1; visible to every wave after the barrier
    for (int i = t; i < O * H; i += MT) {
        const int kq = i / (4 * H), rem = i - kq * 4 * H, u = rem >> 2, k = 4 * kq + (rem & 3);
        Wq[i] = P[offW1 + k * H + u];
    }
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
    float* scr = &S.big.scr[w][0][0];  // tile A: H1, then dZ1
    float* scr2 = &S.act2[w][0][0];     // tile B: H2, then dZ2

    PGM_STAMP_DECL
    for (int e = 0; e < E; ++e) {
        for (int bb = 0; bb < nb; ++bb) {
            const int32_t* perm = a.perms + (size_t)e * B + bb * mb + r0;
            // the next minibatch (the last step re-touches its own rows)
            const bool has_next = bb + 1 < nb || e + 1 < E;
            const int32_t* nperm = !has_next ? perm : bb + 1 < nb ? perm + mb : a.perms + (size_t)(e + 1) * B + r0;
            f32x16 gW2[2][2], gWh[2], dW1[NKW][2];
            float gB1[2], gB2[2];
            float gsm = 0.f;  // lanes q < Q: head-bias gradient q; lanes 32 + q (actor): logstd gradient q
#pragma unroll
            for (int i = 0; i < 2; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j) gW2[i][j] = f32x16{0};
                gWh[i] = f32x16{0};
                gB1[i] = gB2[i] = 0.f;
            }
#pragma unroll
            for (int j = 0; j < NKW; ++j) dW1[j][0] = dW1[j][1] = f32x16{0};
            float lsum = 0.f;

            for (int ps = 0; ONE ? ps < 1 : ps < npass; ++ps) {
                const int i0 = (ps * 4 + w) * TS;  // this wave's tile of the pass
                const int si = i0 + c;
                const bool ok = si < mbs;
                const int row = perm[min(si, mbs - 1)];
                if (h == 0) S.rowid[w][c] = row;
                if (ps == 0) {
                    const int nrow = nperm[min(si, mbs - 1)];
                    if (h == 0) S.nrowid[w][c] = nrow;
                }
                if (ONE || i0 < mbs) {  // wave-uniform
                    // per-sample loss operands of this lane's sample, gathered now (random rows: an HBM round trip
                    // that the layer-1 stream hides) -- critic: old values, returns; actor: action, old logp, adv
                    float pa[A], pv[K], pr[K], plp = 0.f, pad = 0.f;
                    if (m == 0) {
#pragma unroll
                        for (int q = 0; q < K; ++q) {
                            pv[q] = vals[(size_t)row * K + q];
                            pr[q] = rets[(size_t)row * K + q];
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < A; ++q) pa[q] = acts[(size_t)row * A + q];
                        plp = oldlp[row];
                        pad = advs[row];
                    }
                    // ---- layer 1: Z1[s][u] = sum_k X[s][k] W1t[k][u]; X row of sample c, features h*KH + ks;
                    // groups of KG k-steps, three groups in flight ahead of the MFMAs
#ifdef PGM_DIAG_XFIXED  // timing-only A/B (wrong results): every lane of a half streams ONE row (one line per load)
                    const int xo = (S.rowid[w][0] * O + h * KH) * (int)sizeof(float);
#else
                    const int xo = (row * O + h * KH) * (int)sizeof(float);  // byte offset of the lane's half row
#endif
                    f32x16 z[2] = {f32x16{0}, f32x16{0}};
                    // four register groups in rotation, each loaded three groups (24 MFMAs) ahead of its MFMAs;
                    // branch-free trips (the group count padded to a multiple of 4, padding groups read X = 0 past the
                    // buffer's range and W1 at clamped addresses) keep the loads outstanding across trips
                    constexpr int RING = 4;  // (6 or 7 groups in rotation: layer 1 slower, 54.6 -> 60.5 / 61.7 K cycles)
                    float4 xq[RING];
                    float wq[RING][KG][2];
                    constexpr int NGP = (NG + RING - 1) / RING * RING;
                    auto load_group = [&](int g, float4& x, float (&wv)[KG][2]) {
                        const int gg = min(g, NG - 1);
                        const u32x4 xv = __builtin_amdgcn_raw_buffer_load_b128(ors, g < NG ? xo + 16 * g : XOOB, 0, 0);
                        x = make_float4(__uint_as_float(xv[0]), __uint_as_float(xv[1]), __uint_as_float(xv[2]),
                                        __uint_as_float(xv[3]));
                        static_assert(KG == 4 && KH % 4 == 0, "a group's k-rows are one k-quad");
                        const u32x4 wa = w1q(h * (KH / 4) + gg, c), wb = w1q(h * (KH / 4) + gg, TS + c);
#pragma unroll
                        for (int q = 0; q < KG; ++q) {
                            wv[q][0] = __uint_as_float(wa[q]);
                            wv[q][1] = __uint_as_float(wb[q]);
                        }
                    };
                    auto mfma_group = [&](const float4& x, const float (&wv)[KG][2]) {
                        const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                        for (int q = 0; q < KG; ++q) {
                            z[0] = mfma(xv[q], wv[q][0], z[0]);
                            z[1] = mfma(xv[q], wv[q][1], z[1]);
                        }
                    };
#pragma unroll
                    for (int b = 0; b < RING; ++b) load_group(b, xq[b], wq[b]);
#pragma unroll 1
                    for (int g = 0; g < NGP; g += RING) {
#pragma unroll
                        for (int b = 0; b < RING; ++b) {
                            mfma_group(xq[b], wq[b]);
                            load_group(min(g + b + RING, NGP - 1), xq[b], wq[b]);
                        }
                    }
                    // activations live in two per-wave LDS tiles, not registers (the 230 accumulator registers
                    // leave no room): tile A = H1 (later dZ1), tile B = H2 (later dZ2)
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb) {
                        const float bias = W.b1[hb * TS + c];
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + hb * TS + c] = tanh_fast(z[hb][r] + bias);
                    }
                    wave_lds_fence();
                    PGM_STAMP(0);
                    // ---- layer 2 (A from tile A, transposed)
                    z[0] = z[1] = f32x16{0};
PGM_UNROLL_W(PGM_UW_L2)
                    for (int ks = 0; ks < H / 2; ++ks) {
                        const int k = 2 * ks + h;
                        const float av = scr[c * SCR + k];
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob) z[ob] = mfma(av, W.W2t[k][ob * TS + c], z[ob]);
                    }
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob) {
                        const float bias = W.b2[ob * TS + c];
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr2[rowof(r, h) * SCR + ob * TS + c] = tanh_fast(z[ob][r] + bias);
                    }
                    wave_lds_fence();
                    PGM_STAMP(1);
                    // ---- heads on the MFMA: out[s][q] = H2[s][:] . Wh[q][:] (A = H2 from tile B as in layer 2, B =
                    // Wh^T with the output q on the lane column, q >= Q zero), through the dO tile to lane = sample
                    float outv[Q];
                    {
                        f32x16 ho = f32x16{0};
#pragma unroll 1
                        for (int k0 = 0; k0 < H / 2; k0 += 8) {
                            float av[8], bq[8];
#pragma unroll
                            for (int i = 0; i < 8; ++i) {
                                const int k = 2 * (k0 + i) + h;
                                av[i] = scr2[c * SCR + k];
                                bq[i] = c < Q ? W.Wh[c < Q ? c : 0][k] : 0.f;
                            }
                            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                            for (int i = 0; i < 8; ++i) ho = mfma(av[i], bq[i], ho);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                        if (c < Q) {
                            const float bias = W.bh[c];
#pragma unroll
                            for (int r = 0; r < 16; ++r) S.dout[w][rowof(r, h)][c] = ho[r] + bias;
                        }
                        wave_lds_fence();
#pragma unroll
                        for (int q = 0; q < Q; ++q) outv[q] = S.dout[w][c][q];
                    }
                    // ---- per-sample loss gradients (ppo.py:80-96)
                    float dO[Q];
#pragma unroll
                    for (int q = 0; q < Q; ++q) dO[q] = 0.f;
                    if (m == 0) {  // value loss
                        float ls = 0.f;
#pragma unroll
                        for (int q = 0; q < K; ++q) {
                            const float V = outv[q], Vp = pv[q], R = pr[q];
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
                        const float lpo = plp, ad = pad;
                        float lp = 0.f;
#pragma unroll
                        for (int q = 0; q < A; ++q) {
                            const float diff = pa[q] - outv[q];
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
                            const float diff = pa[q] - outv[q];
                            const float iv = S.aiv[q];
                            dO[q] = dlp * diff * iv;
                            if (h == 0) S.dls[w][c][q] = dlp * (diff * diff * iv - 1.f);
                        }
                    }
                    if (h == 0) {
#pragma unroll
                        for (int q = 0; q < Q; ++q) S.dout[w][c][q] = dO[q];
                    }
                    wave_lds_fence();
                    // per-column sums of the tile: lane q sums dO[.][q], lane 32 + q the logstd terms
                    if (c < (h == 0 ? Q : (m == 1 ? A : 0))) {
                        const float* src = (h == 0 ? &S.dout[w][0][0] : &S.dls[w][0][0]) + c;
#pragma unroll 8
                        for (int cc = 0; cc < TS; ++cc) gsm += src[cc * Q];
                    }
                    PGM_STAMP(2);
                    // ---- head-weight grads on the MFMA: gWh^T[u][q] += sum_s H2[s][u] dO[s][q]
                    // (A = H2 in the C layout from tile B: lane u, samples rowof(r, 0/1); B = dO, lane q)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float bq = c < Q ? S.dout[w][rowof(r, h)][c < Q ? c : 0] : 0.f;
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob) gWh[ob] = mfma(scr2[rowof(r, h) * SCR + ob * TS + c], bq, gWh[ob]);
                    }
                    // ---- dH2 = dO . Wh (MFMA) -> dZ2 (H2 from tile B); dW2^T += H1^T dZ2 (H1 from tile A)
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
                            const float h2 = scr2[rowof(r, h) * SCR + ob * TS + c];
                            dZ2[ob][r] = z[ob][r] * (1.f - h2 * h2);
                            gB2[ob] += dZ2[ob][r];
                        }
#pragma unroll
                    for (int r = 0; r < 16; ++r)
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib) {
                            const float h1 = scr[rowof(r, h) * SCR + ib * TS + c];
#pragma unroll
                            for (int ob = 0; ob < 2; ++ob) gW2[ib][ob] = mfma(h1, dZ2[ob][r], gW2[ib][ob]);
                        }
                    // ---- dH1 = dZ2 W2 -> dZ1 (dZ2 through tile B, transposed)
                    wave_lds_fence();  // every H2 read of tile B returned before the overwrite
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr2[rowof(r, h) * SCR + ob * TS + c] = dZ2[ob][r];
                    wave_lds_fence();
                    z[0] = z[1] = f32x16{0};
PGM_UNROLL_W(PGM_UW_L2)
                    for (int ks = 0; ks < H / 2; ++ks) {
                        const int k = 2 * ks + h;
                        const float av = scr2[c * SCR + k];
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib) z[ib] = mfma(av, W.W2t[ib * TS + c][k], z[ib]);
                    }
                    f32x16 dZ1[2];
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float h1 = scr[rowof(r, h) * SCR + ib * TS + c];
                            dZ1[ib][r] = z[ib][r] * (1.f - h1 * h1);
                            gB1[ib] += dZ1[ib][r];
                        }
                    // ---- dZ1 to tile A: every wave contracts it with its dW1 tiles
                    wave_lds_fence();
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ib * TS + c] = dZ1[ib][r];
                }
                PGM_STAMP(3);
                lds_sync_m();  // every tile's dZ1 and rows visible
                PGM_STAMP(4);
                // ---- dW1^T[k][u] += X^T dZ1 over the pass's tiles for this wave's feature tiles; the X values
                // of (tile u, feature tile kt) are gathered from HBM one round ahead (rows of the tile)
                {
                    const int nu = min(4, (mbs - ps * 4 * TS + TS - 1) / TS);  // tiles of this pass
                    constexpr int NR = NKW * 4;                                // rounds (j, u)
                    auto gather = [&](int rd, float (&xv)[16]) {
                        const int j = rd >> 2, u = rd & 3, kf = (w + 4 * j) * TS + c;
                        // dead elements (features past O, tiles past the pass) at + XOOB: an integer add, not a select
                        const int dead = u < nu && kf < O ? 0 : XOOB;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
#ifdef PGM_DIAG_DXFIXED  // timing-only A/B (wrong results): the dW1 gather reads one row per tile
                            const int rr = S.rowid[u][0];
#else
                            const int rr = S.rowid[u][rowof(r, h)];
#endif
                            xv[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                ors, (rr * O + kf) * (int)sizeof(float) + dead, 0, 0));
                        }
                    };
                    float xa[16], xb[16];
                    gather(0, xa);
#pragma unroll
                    for (int rd = 0; rd < NR; ++rd) {
                        float(&cur)[16] = (rd & 1) ? xb : xa;
                        float(&nxt)[16] = (rd & 1) ? xa : xb;
                        if (rd + 1 < NR) gather(rd + 1, nxt);
                        // the next round's loads stay ahead of this round's MFMAs (no sinking / interleaving), and at
                        // ONE with whole 4-tile groups the round is unconditional (a branch here let the compiler sink
                        // the first gather into the round and wait for each load before its MFMA)
                        __builtin_amdgcn_sched_barrier(0);
                        const int j = rd >> 2, u = rd & 3;
                        if ((ONE || u < nu) && (NKT % 4 == 0 || w + 4 * j < NKT)) {
                            const float* dz = &S.big.scr[u][0][0];
                            // the round's B operands (dZ1 of tile u) read up front: one read per MFMA pair into the
                            // same two registers had put an LDS round trip in front of every pair
                            float bz[16][2];
#pragma unroll
                            for (int r = 0; r < 16; ++r)
#pragma unroll
                                for (int ib = 0; ib < 2; ++ib) bz[r][ib] = dz[rowof(r, h) * SCR + ib * TS + c];
                            __builtin_amdgcn_sched_barrier(0);  // (left alone, the scheduler sinks each read to its MFMA)
#pragma unroll
                            for (int r = 0; r < 16; ++r)
#pragma unroll
                                for (int ib = 0; ib < 2; ++ib) dW1[j][ib] = mfma(cur[r], bz[r][ib], dW1[j][ib]);
                        }
                    }
                }
                PGM_STAMP(5);
                lds_sync_m();  // transpose tiles / row ids reused by the next pass
                PGM_STAMP(6);
            }  // passes

            // ---- the next minibatch's observation rows (this wave's tile of its first pass) into L2 while this step
            // reduces, exchanges and updates: one 4-B touch per 128-B line of the lane's half row (and its last float),
            // held in registers until the step's final vmcnt(0).  The layer-1 stream then meets L2 hits instead of
            // HBM misses: layer 1 54.6 -> 39.6 K cycles per Adam step (the touches' issue costs the reduction ~2.7 K).
            // (An LDS-DMA discard would hold no registers but puts a vmcnt(0) before the reduction's first LDS write:
            // the compiler cannot tell the DMA's LDS target from the reduction's.  64-B touches, the two towers of a
            // row part taking alternate lines, or the touches after the publish drain: no faster, or slower.)
            constexpr int PF_NSEG = (KH * 4 + 127) / 128;
            constexpr int NTOUCH = PF_NSEG + 1;
            float pft[NTOUCH];
            {
                const int xo = (S.nrowid[w][c] * O + h * KH) * (int)sizeof(float);
#pragma unroll
                for (int i = 0; i < NTOUCH; ++i)
                    pft[i] = __uint_as_float(
                        __builtin_amdgcn_raw_buffer_load_b32(ors, xo + (i < PF_NSEG ? 128 * i : 4 * (KH - 1)), 0, 0));
            }

            // ---- lane halves of the per-column partial sums; 64-lane sums of the per-sample ones
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                gB1[i] = half_sum(gB1[i]);
                gB2[i] = half_sum(gB2[i]);
            }
            lsum = wave_sum64(lsum);
            float ent = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) ent += 0.5f + LOG_SQRT_2PI + lstd[q];

            // ---- small-image gradients: waves 0/1 -> GA[0], 2/3 -> GA[1]; the two waves of a pair split the
            // image in two halves: in stage 0 each stores its partial of one half, in stage 1 it adds its partial
            // of the other half (every element = one wave's partial + the other's: deterministic)
            if (l == 0) S.red[8 + w] = lsum;
            {
                float* Gt = S.big.GA[w >> 1];
                for (int stage = 0; stage < 2; ++stage) {
                    const bool add = stage == 1;
                    const int half = (stage == 0) == ((w & 1) == 1) ? 0 : 1;
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
                    for (int ib = 0; ib < 2; ++ib) {
                        if (ib != half) continue;
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob)
                            acc16([&](int r) { return (ib * TS + rowof(r, h)) * SCR + ob * TS + c; }, gW2[ib][ob]);
                        // head weights: gWh[ob] row rowof(r,h) = unit ob*32 + rowof, column c = output q (c < Q)
                        if (c < Q) acc16([&](int r) { return oWh + c * WHS + ib * TS + rowof(r, h); }, gWh[ib]);
                        if (h == 0) {
                            acc(oB1 + ib * TS + c, gB1[ib]);
                            acc(oB2 + ib * TS + c, gB2[ib]);
                        }
                    }
                    if (half == 1) {
                        if (h == 0 && c < NQ) acc(oBh + c, gsm);
                        if (m == 1 && h == 1 && c < A) {  // -entropy_coef * d(mean entropy)/d logstd enters once (ppo.py:98)
                            const float ec = add || hs != 0 || (w >> 1) != 0 ? 0.f : a.hp.entropy_coef;  // once per tower: part 0, image 0
                            acc(oLs + c, gsm - ec);
                        }
                        if (!add) {  // padding slots of a freshly written image
                            Gt[l * SCR + H] = 0.f;
                            for (int i = l; i < Q * (WHS - H); i += 64) Gt[oWh + (i / (WHS - H)) * WHS + H + i % (WHS - H)] = 0.f;
                            if (l >= NQ && l < Q) Gt[oBh + l] = 0.f;
                            if (m == 0 && l < A) Gt[oLs + l] = 0.f;
                        }
                    }
                    lds_sync_m();
                }
            }
            // head rows q >= NQ (critic: 2..16) are exactly zero: dO[q] = 0 for them
            PGM_STAMP(7);
            float* G0 = S.big.GA[0];
            const float* G1 = S.big.GA[1];
            const float lsum_wg = (S.red[8] + S.red[9]) + (S.red[10] + S.red[11]);
            float lsum_task = lsum_wg;
            // Layer 1 is SHARDED over the NS row parts: part hs owns values r in [RS hs, RS hs + RS) of every
            // 16-value dW1 register block of every lane (rows 8 (r >> 2) + (r & 3) + 4 h of the block's feature
            // tile), sums only those over the parts, clips / Adam-updates only them (moments straight in the
            // caller's arrays: the parts' elements are disjoint) and hands the new weights to the other parts.
            constexpr int RS = 16 / NS;  // values per block this part owns
            constexpr int NB = NKW * 2;  // dW1 register blocks per lane
            const int rbase = RS * hs;
            float gs[NB][RS];  // this part's slice of the task's summed dW1
            const int kb = opaque(w * TS + 4 * h);           // lane's first layer-1 row (feature)
            const int fb = opaque(offW1 + kb * H + c);       // ... its flat parameter index
            auto krow = [&](int j, int r) { return 4 * j * TS + (r & 3) + 8 * (r >> 2); };  // row - kb of value r
            auto live = [&](int j, int r) { return w + 4 * j < NKT && kb + krow(j, r) < O; };
            const unsigned tag = (unsigned)(nstep + 1);
            const int par = nstep & 1;
            auto slot_of = [&](int hh) { return ((p * 2 + m) * NS + hh) * 2 + par; };
            const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(a.xb, 0, a.xbytes, 0x00020000);
            // slot = small image | dW1 block [block b][quad q][thread][4] (lane t's values r = 4q .. 4q + 3 of register
            // block b as one 16-B piece, so publish and gather are 16-B accesses, one contiguous KiB per wave and
            // instruction) | new-W1 slices [b][quad][thread][4] | 2 flag granules
            constexpr int DW = (IMG * 4 + 15) / 16 * 16;       // byte offset of the dW1 block inside a slot
            constexpr int DS = DW + NKT * TS * H * 4;          // byte offset of the new-W1-slice block
            static_assert(NB * 16 * MT == NKT * TS * H, "dW1 exchange block: 16 values per lane and register block");
            static_assert(RS % 4 == 0, "a part's slice is whole 16-B quads");
            auto spin = [&](const unsigned long long* fl, unsigned want) {  // one lane; bounded
                unsigned long long x = 0;
                for (unsigned spins = 0;; ++spins) {
                    x = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((unsigned)(x >> 32) == want) break;
                    if (spins > (1u << 26)) {  // a partner never arrived: flag the launch as failed
                        __hip_atomic_store(a.ws + 2 * a.P, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        return 0ull;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                return x;
            };
            // this part's own partial of its slice (a select among NS candidates per value)
#pragma unroll
            for (int j = 0; j < NKW; ++j)
#pragma unroll
                for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                    for (int ri = 0; ri < RS; ++ri) {
                        float v = dW1[j][ib][ri];
#pragma unroll
                        for (int hh = 1; hh < NS; ++hh)
                            if (hs == hh) v = dW1[j][ib][RS * hh + ri];
                        gs[j * 2 + ib][ri] = v;
                    }
            if constexpr (NS > 1) {
                // ---- the parts' gradients: 16-B sc1 stores of the small image G0 + G1 and of the dW1 registers
                // (all but this part's own slice, which no partner reads), every wave drains, barrier, one lane stores the tagged flag granule {step, loss
                // sum} and polls the other parts' flags, barrier, sc1 loads of the other parts' small images and
                // of THIS part's dW1 slice.  Sums in part order 0..NS-1 (the small-image Adam steps of the parts
                // stay bitwise identical).  Slots are double-buffered by step parity.
                const int off_mine = slot_of(hs) * a.xslot * 8;
                constexpr int NV4 = IMG / 4, TAIL = IMG - 4 * NV4;
                for (int i = t; i < NV4; i += MT) {
                    u32x4 v;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float g = G0[4 * i + q] + G1[4 * i + q];
                        G0[4 * i + q] = g;
                        v[q] = __float_as_uint(g);
                    }
                    __builtin_amdgcn_raw_buffer_store_b128(v, xr, off_mine + 16 * i, 0, WSPLIT);
                }
                if (t < TAIL) {
                    const float g = G0[4 * NV4 + t] + G1[4 * NV4 + t];
                    G0[4 * NV4 + t] = g;
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g), xr, off_mine + 16 * NV4 + 4 * t, 0, WSPLIT);
                }
                const int dwq = opaque(16 * t);  // this lane's 16-B piece of every (block, quad) row
#pragma unroll
                for (int j = 0; j < NKW; ++j)
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if (4 * q / RS == hs) continue;  // own slice: kept in registers, never read by a partner
                            const u32x4 v = {__float_as_uint(dW1[j][ib][4 * q]), __float_as_uint(dW1[j][ib][4 * q + 1]),
                                             __float_as_uint(dW1[j][ib][4 * q + 2]), __float_as_uint(dW1[j][ib][4 * q + 3])};
                            __builtin_amdgcn_raw_buffer_store_b128(v, xr, dwq,
                                                                   off_mine + DW + ((j * 2 + ib) * 4 + q) * MT * 16, WSPLIT);
                        }
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                lds_sync_m();
                if (t == 0) {
                    unsigned long long* flag_mine = a.xb + (size_t)slot_of(hs) * a.xslot + a.xslot - 1;
                    __hip_atomic_store(flag_mine, ((unsigned long long)tag << 32) | __float_as_uint(lsum_wg),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (t < NS)  // lane h polls part h's flag: the NS - 1 polls run concurrently
                    S.red[24 + t] = t == hs ? lsum_wg
                                            : __uint_as_float((unsigned)spin(a.xb + (size_t)slot_of(t) * a.xslot + a.xslot - 1, tag));
                PGM_STAMP(8);
                lds_sync_m();  // every polling lane matched: every wave may load the other parts' gradients
                if (t == 0) {
                    float ls = 0.f;
                    for (int hh = 0; hh < NS; ++hh) ls = hh == 0 ? S.red[24] : ls + S.red[24 + hh];  // part order
                    S.red[12] = ls;
                }
                {  // this part's dW1 slice: its own partial plus the other parts' in the fixed order hs + 1, hs + 2, ...
                   // (each element has one owner, so any fixed order is deterministic), the next partner's loads in
                   // flight while one is added.  (All three partners loaded at once beside the own partials -- 96 live
                   // values -- went through scratch, each group of four loads behind a vmcnt(0).)
                    float pb[2][NB][RS];
                    auto ldp = [&](int q, float (&v)[NB][RS]) {
                        int hh = hs + 1 + q;
                        hh = hh >= NS ? hh - NS : hh;
#pragma unroll
                        for (int b = 0; b < NB; ++b)
#pragma unroll
                            for (int qq = 0; qq < RS / 4; ++qq) {
                                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(
                                    xr, dwq, slot_of(hh) * a.xslot * 8 + DW + (b * 4 + (rbase >> 2) + qq) * MT * 16, WSPLIT);
#pragma unroll
                                for (int e = 0; e < 4; ++e) v[b][4 * qq + e] = __uint_as_float(x[e]);
                            }
                    };
                    ldp(0, pb[0]);
#pragma unroll
                    for (int q = 0; q < NS - 1; ++q) {
                        if (q + 1 < NS - 1) ldp(q + 1, pb[(q + 1) & 1]);
#pragma unroll
                        for (int b = 0; b < NB; ++b)
#pragma unroll
                            for (int ri = 0; ri < RS; ++ri) gs[b][ri] += pb[q & 1][b][ri];
                    }
                }
                {  // the small images: every part's slot (this part's own too: the same bits it published), all
                   // NS loads of the next trip in flight while this trip sums -- straight-line and branch-free (a
                   // per-partner `hh != hs` test had made every trip a chain of branches, each value behind its
                   // own vmcnt(0): ~6 serial round trips, 29 K cycles per Adam step with the dW1 slice loads)
                    constexpr int NIT = (NV4 + MT - 1) / MT;
                    u32x4 pa_[NS], pb_[NS];
                    auto ld = [&](int it, u32x4 (&v)[NS]) {
                        const int i = min(t + it * MT, NV4 - 1);  // (the tail trip re-reads a valid entry, unused)
#pragma unroll
                        for (int hh = 0; hh < NS; ++hh)
                            v[hh] = __builtin_amdgcn_raw_buffer_load_b128(xr, slot_of(hh) * a.xslot * 8 + 16 * i, 0, WSPLIT);
                    };
                    ld(0, pa_);
#pragma unroll
                    for (int it = 0; it < NIT; ++it) {
                        u32x4(&cur)[NS] = (it & 1) ? pb_ : pa_;
                        u32x4(&nxt)[NS] = (it & 1) ? pa_ : pb_;
                        if (it + 1 < NIT) ld(it + 1, nxt);
                        const int i = t + it * MT;
                        if (i < NV4) {
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                float acc = 0.f;
#pragma unroll
                                for (int hh = 0; hh < NS; ++hh) {
                                    const float v = __uint_as_float(cur[hh][q]);
                                    acc = hh == 0 ? v : acc + v;
                                }
                                G0[4 * i + q] = acc;
                            }
                        }
                    }
                }
                if (t < TAIL) {
                    float acc = 0.f;
#pragma unroll
                    for (int hh = 0; hh < NS; ++hh) {
                        const float v = hh == hs ? G0[4 * NV4 + t]
                                                 : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                                       xr, slot_of(hh) * a.xslot * 8 + 16 * NV4 + 4 * t, 0, WSPLIT));
                        acc = hh == 0 ? v : acc + v;
                    }
                    G0[4 * NV4 + t] = acc;
                }
                lds_sync_m();
                lsum_task = S.red[12];
            } else {
                for (int i = t; i < IMG; i += MT) G0[i] = G0[i] + G1[i];
                lds_sync_m();
            }
            PGM_STAMP(9);
            // ---- clip_grad_norm_: part 0 counts the small image, every part its dW1 slice (rows k >= O hold
            // zeros); the 2 NS partial sums of the task meet through tagged granules, summed in (tower, part)
            // order in every workgroup
            float sq = 0.f;
            if (hs == 0)
                for (int i = t; i < IMG; i += MT) sq = fmaf(G0[i], G0[i], sq);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int ri = 0; ri < RS; ++ri) sq = fmaf(gs[b][ri], gs[b][ri], sq);
            sq = wave_sum64(sq);
            if (l == 0) S.red[w] = sq;
            lds_sync_m();
            float total = (S.red[0] + S.red[1]) + (S.red[2] + S.red[3]);
            if (t == 0)
                __hip_atomic_store(a.ws + ppo_norm_granule(a.P, p, m, hs, par), ((unsigned long long)tag << 32) | __float_as_uint(total),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t < 2 * NS) {  // lane (mm, hh) = (t / NS, t % NS) polls that workgroup's granule, all concurrently
                const int mm = t / NS, hh = t - mm * NS;
                float v = total;
                if (mm != m || hh != hs) {
                    const bool failed = __hip_atomic_load(a.ws + 2 * a.P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    v = failed ? 0.f : __uint_as_float((unsigned)spin(a.ws + ppo_norm_granule(a.P, p, mm, hh, par), tag));
                }
                S.red[16 + t] = v;
            }
            lds_sync_m();
            {  // (tower, part) order, identical in every workgroup of the task
                float tot = S.red[16];
                for (int i = 1; i < 2 * NS; ++i) tot += S.red[16 + i];
                total = tot;
            }
            const float coef = fminf(a.hp.max_grad_norm / (sqrtf(total) + 1e-6f), 1.f);
            if (t == 0) {
                if (m == 0) st_v += 0.5f * lsum_task / (float)(mb * K);
                else st_a += lsum_task / (float)mb;
                st_e += ent;
            }
            PGM_STAMP(10);
            // ---- Adam: layer 1 first (this part's slice; moments in HBM), its new weights handed to the other
            // parts while the small image (LDS) updates, then the other parts' slices into this part's copy
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
            {
                // loads of CB blocks in flight at a time (all of them at NS = 4)
                constexpr int CB = RS >= 16 ? 1 : RS >= 8 ? 3 : NB;
#pragma unroll
                for (int b0 = 0; b0 < NB; b0 += CB) {
                    float bm[CB][RS], bv[CB][RS], bp[CB][RS];
#pragma unroll
                    for (int bb = 0; bb < CB; ++bb)
#pragma unroll
                        for (int ri = 0; ri < RS; ++ri) {
                            const int b = b0 + bb, j = b >> 1, ib = b & 1, r = rbase + ri;
                            const bool lv = b < NB && live(j, r);
                            const int f = lv ? fb + krow(j, r) * H + ib * TS : offW1;
                            bm[bb][ri] = Mo[f];
                            bv[bb][ri] = Vo[f];
                            if ((ri & 3) == 0) {  // the quad's four k-rows of one column: 16 B of the copy (0 past its range)
                                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                                    wrs, lv ? qidx(kb + krow(j, r), ib * TS + c) * 4 : XOOB, 0, 0);
#pragma unroll
                                for (int e = 0; e < 4; ++e) bp[bb][ri + e] = __uint_as_float(v[e]);
                            }
                        }
#pragma unroll
                    for (int bb = 0; bb < CB; ++bb)
#pragma unroll
                        for (int ri = 0; ri < RS; ++ri) {
                            const int b = b0 + bb, j = b >> 1, ib = b & 1, r = rbase + ri;
                            if (b >= NB) continue;
                            adam(gs[b][ri], bm[bb][ri], bv[bb][ri], bp[bb][ri]);
                            gs[b][ri] = bp[bb][ri];
                            if ((ri & 3) == 3) {  // the quad's new parameters as one 16-B store (dropped past the range)
                                const int r0 = r - 3;
                                const u32x4 v = {__float_as_uint(bp[bb][ri - 3]), __float_as_uint(bp[bb][ri - 2]),
                                                 __float_as_uint(bp[bb][ri - 1]), __float_as_uint(bp[bb][ri])};
                                __builtin_amdgcn_raw_buffer_store_b128(
                                    v, wrs, live(j, r0) ? qidx(kb + krow(j, r0), ib * TS + c) * 4 : XOOB, 0, 0);
                            }
                            if (!live(j, r)) continue;
                            const int f = fb + krow(j, r) * H + ib * TS;
                            Mo[f] = bm[bb][ri];
                            Vo[f] = bv[bb][ri];
                        }
                }
            }
            PGM_STAMP(12);
            if constexpr (NS > 1) {  // publish the new slice (16-B sc1 stores, [block][quad][thread][4]), drain, flag
#pragma unroll
                for (int b = 0; b < NB; ++b)
#pragma unroll
                    for (int qq = 0; qq < RS / 4; ++qq) {
                        const u32x4 v = {__float_as_uint(gs[b][4 * qq]), __float_as_uint(gs[b][4 * qq + 1]),
                                         __float_as_uint(gs[b][4 * qq + 2]), __float_as_uint(gs[b][4 * qq + 3])};
                        __builtin_amdgcn_raw_buffer_store_b128(v, xr, 16 * t,
                                                               slot_of(hs) * a.xslot * 8 + DS + (b * (RS / 4) + qq) * MT * 16,
                                                               WSPLIT);
                    }
            }
            // (the slice stores drain under the small image's Adam, an LDS-only loop: the wave's vmcnt(0) is taken
            // after it, before the barrier that releases the flag store -- R1 order unchanged)
            for (int i = t; i < IMG; i += MT) {
                float mm = S.MV[i], vv = S.MV[IMG + i], pp = Pf[i];
                adam(G0[i], mm, vv, pp);
                S.MV[i] = mm;
                S.MV[IMG + i] = vv;
                Pf[i] = pp;
                if (m == 1 && i >= oLs && i < oLs + A) S.aiv[i - oLs] = expf(-2.f * pp);
            }
            PGM_STAMP(13);
            if constexpr (NS > 1) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                lds_sync_m();  // every wave's slice stores drained
                PGM_STAMP(14);
                if (t == 0)
                    __hip_atomic_store(a.xb + (size_t)slot_of(hs) * a.xslot + a.xslot - 2, (unsigned long long)tag << 32,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (t < NS && t != hs) spin(a.xb + (size_t)slot_of(t) * a.xslot + a.xslot - 2, tag);  // concurrent polls
                lds_sync_m();
                PGM_STAMP(15);
                // the other parts' new slices -> this part's layer-1 copy, the next part's loads in flight while one
                // part's values are stored
                float nvb[2][NB][RS];
                auto ldn = [&](int q, float (&nv)[NB][RS]) {
                    const int hh = q < hs ? q : q + 1;
#pragma unroll
                    for (int b = 0; b < NB; ++b)
#pragma unroll
                        for (int qq = 0; qq < RS / 4; ++qq) {
                            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(
                                xr, 16 * t, slot_of(hh) * a.xslot * 8 + DS + (b * (RS / 4) + qq) * MT * 16, WSPLIT);
#pragma unroll
                            for (int e = 0; e < 4; ++e) nv[b][4 * qq + e] = __uint_as_float(x[e]);
                        }
                };
                ldn(0, nvb[0]);
#pragma unroll
                for (int q = 0; q < NS - 1; ++q) {
                    const int hh = q < hs ? q : q + 1;
                    if (q + 1 < NS - 1) ldn(q + 1, nvb[(q + 1) & 1]);
#pragma unroll
                    for (int b = 0; b < NB; ++b)
#pragma unroll
                        for (int ri = 0; ri < RS; ++ri) {
                            const int j = b >> 1, ib = b & 1, r = RS * hh + ri;
                            if ((ri & 3) == 0) {  // 16 B: the quad's four k-rows of one column
                                const u32x4 v = {__float_as_uint(nvb[q & 1][b][ri]), __float_as_uint(nvb[q & 1][b][ri + 1]),
                                                 __float_as_uint(nvb[q & 1][b][ri + 2]), __float_as_uint(nvb[q & 1][b][ri + 3])};
                                __builtin_amdgcn_raw_buffer_store_b128(
                                    v, wrs, live(j, r) ? qidx(kb + krow(j, r), ib * TS + c) * 4 : XOOB, 0, 0);
                            }
                        }
                }
            }
            // every layer-1 store of the step drained before any wave's next W1 stream.  No L1 invalidate: every
            // byte of this workgroup's layer-1 copy is written by this workgroup (its own slice by the Adam above,
            // the partners' slices from their sc1-loaded values), and one CU's own stores keep its L1 coherent
            // (workgroup scope); the partners' bytes themselves only ever arrive through sc1 loads
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < NTOUCH; ++i) asm volatile("" ::"v"(pft[i]));  // the prefetch's values retire here
            lds_sync_m();
            PGM_STAMP(11);
        }  // minibatches
    }      // epochs
    PGM_STAMP_FLUSH;
    if (hs != 0) return;  // parts 1..NS-1: copies only
    // ---- write back layer 1 (part 0's copy holds every part's slice after the last step) and the small image
    for (int i = t; i < O * H; i += MT) P[offW1 + i] = Wq[qidx(i / H, i - (i / H) * H)];
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

}  // namespace

static int wide_choose_ns(const pgm_dims* d, const pgm_launch_opts& o) {
    const int cap = split_cap(o);
    const int cus = device_cu_count();
    return cap >= 4 && wide_grid(d->P, 4) <= cus ? 4 : cap >= 2 && wide_grid(d->P, 2) <= cus ? 2 : 1;
}

int describe_update_wide(const pgm_dims* d, const pgm_launch_opts& o, char* buf, int n) {
    return snprintf(buf, n, "ppo_update_wide_kernel (NS=%d)", wide_choose_ns(d, o));
}

int ppo_update_wide(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m, float* adam_v,
                    int32_t* adam_step, const float* lr, const int32_t* perms, const pgm_rollout_buf* rb, float* stats,
                    void* workspace, const pgm_launch_opts& o, hipStream_t stream) {
    if (!workspace) {
        set_error("pgm_ppo_update: the wide update needs the workspace (pgm_ppo_update_workspace_bytes)");
        return PGM_E_INVALID_ARG;
    }
    // NS = 4 (each tower on four CUs) while the 32-block groups fit the CU count, else NS = 2 while the
    // 16-block groups do, else 1; opts.update_split caps it (TASK / TOWER: one workgroup per tower, HALVES: two)
    const int cus = device_cu_count();
    const int ns = wide_choose_ns(d, o);
    if (ns == 1 && 2 * d->P > cus) {
        set_error("pgm_ppo_update: the wide update needs 2P <= CUs (P=%d); shard the tasks over more GPUs", d->P);
        return PGM_E_UNSUPPORTED;
    }
    if ((long long)(d->T + 1) * d->N * d->O * (long long)sizeof(float) >= (1ll << 31)) {
        set_error("pgm_ppo_update: the wide update addresses a task's observations with 31-bit byte offsets "
                  "((T+1) N O = %lld floats)", (long long)(d->T + 1) * d->N * d->O);
        return PGM_E_UNSUPPORTED;
    }
    const Layout L = make_layout(d->O, d->A, d->K, d->H);
    char* ws = (char*)workspace;
    const size_t flags = ppo_flag_bytes(d->P);
    const int xslot = wide_xslot_words(d->O, d->A, d->K);
    const size_t xcap = wide_xbuf_bytes(d);  // sized for PGM_NS_MAX parts
    const size_t xbytes = (size_t)d->P * 2 * ns * 2 * xslot * 8;
    float* copies = (float*)(ws + flags + xcap);
    WArgs a{d->N, d->T, d->P, L, *hp, params, adam_m, adam_v, copies, adam_step, lr, perms,
            rb->obs, rb->actions, rb->logp, rb->adv, rb->values, rb->returns, stats, (unsigned long long*)ws,
            (unsigned long long*)(ws + flags), xslot, (int)xbytes};
    hipError_t e = hipSuccess;
    if (!ws_take_zeroed(workspace, flags + (ns > 1 ? xbytes : 0))) {
        e = hipMemsetAsync(workspace, 0, flags + (ns > 1 ? xbytes : 0), stream);
        if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update (workspace reset)");
    }
    // every workgroup's layer-1 copy [P][2 towers][ns parts][O H] (filled by the kernel) in the workspace's copy region,
    // sized for PGM_NS_MAX parts (ppo_workspace_bytes)
    if (ns > PGM_NS_MAX) {
        set_error("pgm_ppo_update: wide layer-1 copies exceed the workspace (ns=%d)", ns);
        return PGM_E_INVALID_ARG;
    }
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
            auto launch = [&](auto kern, int grid) -> int {
                hipError_t e2 = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    (int)smem);
                if (e2 != hipSuccess) return hip_fail(e2, "pgm_ppo_update");
                if (int rc = check_coresident((const void*)kern, MT, smem, grid, "pgm_ppo_update")) return rc;
                hipLaunchKernelGGL(kern, dim3(grid), dim3(MT), smem, stream, a);
                return launch_status("pgm_ppo_update");
            };
            const int mb = d->T * d->N / hp->num_mini_batch;
            if (ns == 4 && mb == 4 * 4 * TS) return launch(ppo_update_wide_kernel<O, A, K, 4, true>, wide_grid(d->P, 4));
            if (ns == 4) return launch(ppo_update_wide_kernel<O, A, K, 4, false>, wide_grid(d->P, 4));
            if (ns == 2) return launch(ppo_update_wide_kernel<O, A, K, 2, false>, wide_grid(d->P, 2));
            return launch(ppo_update_wide_kernel<O, A, K, 1, false>, 2 * d->P);
        }
    });
}

}  // namespace pgm
