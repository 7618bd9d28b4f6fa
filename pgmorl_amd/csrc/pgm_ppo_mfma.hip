// Scalarised clipped-PPO update on the f32 matrix cores (v_mfma_f32_32x32x2_f32, exact fp32).
//
// Work split.  SPLIT mode (default while 2P <= CUs): two 256-thread workgroups per task, one per tower
// (critic / actor), each on its own CU; the only coupling inside a minibatch step is the global grad
// norm, exchanged as one tagged 8-byte granule per step.  Parameters AND Adam moments of the tower stay
// in LDS for the whole launch (one HBM read at the start, one write at the end).  Joint mode: one
// workgroup per task, waves 0/2 critic and 1/3 actor, Adam moments in HBM.
//
// Staging.  pack_rows_kernel first writes a packed sample table, one RS-float row per sample
// (obs | action | old logp | adv | old value | return; 128 B for Walker).  The update consumes the
// permuted rows of each minibatch in passes of SBk samples, staged HBM -> LDS by global_load_lds
// (16 B per lane, no VGPRs) one pass AHEAD into a second buffer, with the permutation indices of the
// pass after that staged the same way (4-B LDS-DMA) one pass earlier still.
//
// Tiles.  32 samples per MFMA tile; samples are the accumulator ROWS (registers), features the
// COLUMNS (lanes), i.e. every activation H1, H2, dZ2, dZ1 lives in the standard C layout
//     lane l, register r  <->  (sample rowof(r, l>>5), feature l & 31),  rowof(r,h) = (r&3)+8(r>>2)+4h.
//   * weight gradients (dW2^T = H1^T dZ2, dW1^T = X^T dZ1) sum over samples = over registers:
//     MFMA(A = H1 reg r, B = dZ2 reg r), no data movement;
//   * the products summing over a FEATURE (Z2 = H1 W2^T, dH1 = dZ2 W2) take A from a per-wave [32][65]
//     LDS transpose tile; the value / mean heads and the per-sample losses run on the VALU.
// Gradients accumulate in registers over the minibatch and are reduced across the tower's waves into
// two LDS images in a fixed order (deterministic); clip_grad_norm_ and Adam are flat passes.
//
// Reference semantics: a2c_ppo_acktr/algo/ppo.py:58-115 (losses, clip_grad_norm_, Adam),
// a2c_ppo_acktr/storage.py:118-154 (minibatch rows), a2c_ppo_acktr/model.py:75-82,
// a2c_ppo_acktr/distributions.py:29-40 (log_probs / entropy).  torch.min/max/clamp backward
// (ties split the gradient in half) are reproduced exactly.
#include <stdio.h>
#include <stdlib.h>

#include "pgm_dispatch.hpp"
#include "pgm_ppo_shared.hpp"

PGM_STAMP_UNIT(mfma)

#define PGM_PRAGMA(x) _Pragma(#x)
#define PGM_UNROLL(n) PGM_PRAGMA(unroll n)
// unroll depths of the feature-contracting MFMA loops (measured, Walker: MODE 2 layer-2 / dH1 loops 8 -> 32: 6.54 ->
// 6.46 ms; VALU heads 4 -> 32: -> 6.48 ms; t16 loops 4 -> 16: 5.40 -> 5.12 ms)
#define PGM_U_L2 32
#define PGM_U16 16
// Measured and dropped (rounds 2-3): heads of the 32-row kernel on the 16x16x4 MFMA with the head outputs on the
// accumulator rows (6.33 vs the VALU heads' 6.25 ms at Walker P = 40; samples on the accumulator rows: 6.72 ms); the
// MODE 2 tower norms exchanged as a separate granule hand-off instead of gathered (below: 6.17 vs 6.10 ms); the
// round-2 block maps (a tower's parts on one XCD, the towers on two: 5.90 vs 5.85 ms, 2.72 vs 2.44 GB per t16 launch);
// ds_add_f32 image rounds (~20x slower on gfx950); elementwise tanh / tanh' one element per instruction (5.80 vs 5.77
// ms); the next pass's rows staged at the top of a step or behind the layer-1 MFMAs; dW2 issued before dH1.
//
// MODE 2 global grad norm: every workgroup of a task gathers all three other half images (its partner half's and both
// halves of the other tower) and forms the other tower's sum of squares itself, in exactly the owner's element order
// and reduction tree, so the totals stay bitwise equal in the four workgroups and the separate norm-granule hand-off
// (one more cross-CU round trip per Adam step) disappears.
//
// Block maps of the split launches: every workgroup of a task on ONE XCD (groups of 8 tasks; blocks b, b + 8, ... share
// an XCD under round-robin dispatch), so the per-step image hand-offs stay inside one L2: MODE 2 Walker P = 40 5.90 ->
// 5.85-5.89 ms, t16 HalfCheetah P = 20 4.95 -> 4.88-4.90 ms, Walker P = 5 4.90 -> 4.85-4.87 ms (profiles/r03p_*).
namespace pgm {
// grids of the split launches (padding blocks of a partial group of tasks exit at once)
inline int mode2_grid(int P) { return 32 * ((P + 7) / 8); }
inline int t16_grid(int P, int NS) { return 16 * NS * ((P + 7) / 8); }
}  // namespace pgm

namespace pgm {

// the tiles' elementwisenamespace pgm {

// the tiles' elementwise tanh(z + b) and tanh' products on register PAIRS through the packed fp32 ALU (v_pk_add /
// v_pk_mul / v_pk_fma_f32; per element the same operations as tanh_fast): MODE 2 Walker P = 40 5.80 -> 5.76-5.77 ms,
// t16 unchanged.  (MODE 2's Adam on element pairs: no change, 5.76.)

// The image reductions add exactly ONE partial onto a stored one per element per round (store and add ordered by a
// barrier): a read + add + write in the wave (ds_add_f32 instead measured ~20x slower on gfx950: MODE 2 stage 1 2.1 K ->
// 40.5 K cycles per Adam step)
__device__ __forceinline__ void lds_add(float* p, float v) { *p += v; }


// ---------------------------------------------------------------- packed sample table
struct PackArgs {
    int P, N, T;
    const float *obs, *actions, *logp, *adv, *values, *returns;
    float* rows;  // [P][T*N][RS]
};

template <int O, int A, int K>
__global__ __launch_bounds__(256) void pack_rows_kernel(PackArgs a) {
    constexpr int RS = row_stride<O, A, K>();
    const int B = a.T * a.N, BV = (a.T + 1) * a.N;  // rows per task; obs / value slots per task
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;  // one float4 of one row
    if (i >= (long long)a.P * B * (RS / 4)) return;
    const long long row = i / (RS / 4);
    const int k0 = (int)(i - row * (RS / 4)) * 4;
    const int p = (int)(row / B), b = (int)(row - (long long)p * B);
    float4 v;
    float* vp = &v.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = k0 + j;
        float x = 0.f;
        if (k < O) x = a.obs[((size_t)p * BV + b) * O + k];
        else if (k < O + A) x = a.actions[((size_t)p * B + b) * A + (k - O)];
        else if (k == O + A) x = a.logp[(size_t)p * B + b];
        else if (k == O + A + 1) x = a.adv[(size_t)p * B + b];
        else if (k < O + A + 2 + K) x = a.values[((size_t)p * BV + b) * K + (k - O - A - 2)];
        else if (k < O + A + 2 + 2 * K) x = a.returns[((size_t)p * BV + b) * K + (k - O - A - 2 - K)];
        vp[j] = x;
    }
    *reinterpret_cast<float4*>(a.rows + (size_t)row * RS + k0) = v;
}


template <int O, int A, int K, bool SPLIT, int NBUF>
struct MSmemT {
    static constexpr int Q = qmax<A, K>();
    static constexpr int NT = SPLIT ? 1 : 2;  // tower images held by the workgroup
    static constexpr int IMG = img_floats<O, A, K>();
    static constexpr int RS = row_stride<O, A, K>();
    static constexpr int SBk = RS <= 32 ? 128 : 64;  // samples staged per pass
    TowerImg<O, A, K> Pm[NT];              // parameters
    float MV[SPLIT ? 2 * IMG : 1];         // SPLIT: Adam exp_avg | exp_avg_sq images (else in HBM)
    static constexpr int RSL = RS + 4;     // LDS row stride: 2-way bank conflicts on per-sample column reads
    alignas(16) float RB[NBUF][SBk * RSL]; // packed rows of the current / next pass
    int32_t IB[2][SBk];                    // sample indices of the next two passes
    float dout[4][TS][Q];                  // per-wave dL/d(head output) of the current tile
    float dls[4][TS][Q];                   // per-wave per-sample dL/d(logstd) of the current tile (actor)
    float aiv[A];                          // actor 1 / std^2 = exp(-2 logstd), refreshed by Adam
    float red[16];
    union Big {                            // transpose tiles during the passes, gradient images after
        float scr[4][TS][SCR];
        float GA[2][IMG];
    } big;
};

template <int O, int A, int K, bool SPLIT>
constexpr int nbuf() { return sizeof(MSmemT<O, A, K, SPLIT, 2>) <= 160 * 1024 ? 2 : 1; }
template <int O, int A, int K, bool SPLIT>
using MSmem = MSmemT<O, A, K, SPLIT, nbuf<O, A, K, SPLIT>()>;



// MODE 0: one workgroup per task (joint towers).  MODE 1 (SPLIT): one workgroup per tower.  MODE 2: each tower
// on TWO workgroups that take one half of every minibatch's rows each and add their gradient images through
// tagged granules (both compute half0 + half1 in that order, so their Adam steps stay bitwise identical).
// ONE (MODE 2, mb = 256): every wave owns exactly one 32-row tile of one pass per minibatch; the pass and tile
// loops are straight-line so the gradient accumulators are not loop-carried
template <int O, int A, int K, int MODE, bool ONE>
__global__ __launch_bounds__(MT) void ppo_update_mfma_kernel(MArgs a) {
    constexpr bool SPLIT = MODE >= 1;
    constexpr int NS = MODE == 2 ? 2 : 1;  // workgroups per tower
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    using Sm = MSmem<O, A, K, SPLIT>;
    auto& S = *reinterpret_cast<Sm*>(smem_raw);
    constexpr int Q = qmax<A, K>();
    constexpr int KS1 = (O + 1) / 2;  // k-steps of layer 1
    constexpr int IMG = Sm::IMG, NT = Sm::NT, SBk = Sm::SBk, RS = Sm::RS;
    constexpr int NBUF = nbuf<O, A, K, SPLIT>();
    constexpr int RSL = Sm::RSL;
    // single-tile MODE 2: the next pass's row DMA is issued by waves 1-3 while wave 0 polls the image flags (they
    // wait at that barrier anyway) and retired by the step's last barrier, instead of at the top of the step; wave 0
    // keeps no DMA in its queue so its polls' vmcnt waits do not include it (6.17 -> 6.10 ms against issuing it after
    // the sum of squares)
    constexpr bool EARLY_STAGE = ONE && MODE == 2 && NBUF == 2;
    constexpr int CR = RS / 4;                         // 16-B chunks per packed row
    constexpr int NDT = (SBk * RSL) / 256;             // LDS-DMA wave instructions per pass (1 KiB each)
    static_assert(NDT * 256 == SBk * RSL, "staging split");
    constexpr int oW2 = O * H, oWh = oW2 + H * SCR, oB1 = oWh + Q * H, oB2 = oB1 + H, oBh = oB2 + H, oLs = oBh + Q;
    constexpr int NWT = SPLIT ? 4 : 2;  // waves per tower
    const int t = threadIdx.x, w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    // MODE 2 block map (speed only: the hand-off is correct under any placement; blocks b, b + 8, ... share an XCD
    // under round-robin dispatch)
    const int bx = (int)blockIdx.x;
    // groups of 32 blocks for 8 tasks: block r holds half (r >> 4) & 1 of tower (r >> 3) & 1 of task 8g + (r & 7)
    const int p = MODE == 2 ? 8 * (bx >> 5) + (bx & 7) : SPLIT ? (bx >> 1) : bx;
    const int hs = MODE == 2 ? (bx >> 4) & 1 : 0;  // half of the minibatch rows
    if (p >= a.P) return;
    const int m = MODE == 2 ? (bx >> 3) & 1 : SPLIT ? (bx & 1) : (w & 1);  // tower of this wave
    const int sh = SPLIT ? w : (w >> 1);                      // wave index within the tower
    const int NQ = m == 0 ? K : A;
    const int N = a.N, T = a.T, B = T * N;
    const int E = a.hp.ppo_epoch, M = a.hp.num_mini_batch;
    const int mb = B / M, nb = B / mb;
    const int r0 = hs * mb / NS, mbs = (hs + 1) * mb / NS - r0;  // this workgroup's rows of each minibatch
    const int npm = (mbs + SBk - 1) / SBk;  // passes per minibatch
    const int npass = E * nb * npm;
    const float clip = a.hp.clip_param;
    const Layout& L = a.L;
    float* __restrict__ P = a.params + (size_t)p * L.total;
    float* __restrict__ Mo = a.m + (size_t)p * L.total;
    float* __restrict__ Vo = a.v + (size_t)p * L.total;
    const float* rows = a.rows + (size_t)p * B * RS;
    auto img_tower = [&](int mi) { return SPLIT ? m : mi; };  // tower of image mi

    // ---- staging: pass gp = ((e * nb) + bb) * npm + j covers minibatch rows [j*SBk, j*SBk + ns).
    // The pass's permutation indices go first into IB (4-B LDS-DMA, one pass earlier than the rows).
    // Row DMA: instruction d (waves take d = w, w+4, ...) fills LDS floats [256 d, 256 d + 256); lane l's
    // 16 B land at float 256 d + 4 l = row * RSL + 4 chunk.  The pad chunk of a row (chunk == CR)
    // re-reads the row's first chunk.
    // (wi, nwv): this wave's index among the nwv waves that share the issue (default: all four)
    auto issue_idx = [&](int g, int buf, int wi = -1, int nwv = 4) {
        if (wi < 0) wi = w;
        const int e = g / (nb * npm), rem = g - e * nb * npm, bb = rem / npm, j = rem - bb * npm;
        const int ns = min(SBk, mbs - j * SBk);
        const int32_t* src = a.perms + (size_t)e * B + bb * mb + r0 + j * SBk;
        for (int r0 = wi * 64; r0 < SBk; r0 += 64 * nwv)  // rows beyond ns re-read the last valid index
            __builtin_amdgcn_global_load_lds((const void*)(src + min(r0 + l, ns - 1)),
                                             (lds_void_t*)&S.IB[buf][r0], 4, 0, 0);
    };
    auto issue_rows_n = [&](int buf, int ibuf, int wi, auto nwc) {
        constexpr int NWV = decltype(nwc)::value;
        float* base = &S.RB[buf][0];
        constexpr int NI = (NDT + NWV - 1) / NWV;  // instructions per wave (the last round is partial)
        int idx[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {  // all index reads first: one LDS latency for the batch
            const int d = wi + NWV * i, pos = d * 256 + 4 * l, row = min(pos / RSL, SBk - 1);
            idx[i] = S.IB[ibuf][row];
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int d = wi + NWV * i;
            if (d < NDT) {
                const int pos = d * 256 + 4 * l, row = pos / RSL, chunk = (pos - row * RSL) >> 2;
                const float* src = rows + (size_t)idx[i] * RS + (chunk < CR ? chunk : 0) * 4;
                __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(base + d * 256), 16, 0, 0);
            }
        }
    };
    auto issue_rows = [&](int buf, int ibuf) { issue_rows_n(buf, ibuf, w, ic<4>{}); };
    // element k of row cs of a tile starting at rt
    auto rowf = [&](const float* rt, int cs, int k) { return rt[cs * RSL + k]; };

    // ---- parameter (and SPLIT: Adam moment) images from the flat HBM vectors
    float* Pf = &S.Pm[0].W1t[0][0];
    if (t < A) S.aiv[t] = expf(-2.f * P[L.off[PGM_P_LOGSTD] + t]);
    for (int i = t; i < NT * IMG; i += MT) {
        const int mi = i / IMG, f = img_to_flat<O, A, K>(i - mi * IMG, img_tower(mi), L);
        Pf[i] = f >= 0 ? P[f] : 0.f;
        if constexpr (SPLIT) {
            S.MV[i] = f >= 0 ? Mo[f] : 0.f;
            S.MV[IMG + i] = f >= 0 ? Vo[f] : 0.f;
        }
    }
    issue_idx(0, 0);
    if (npass > 1) issue_idx(1, 1);
    dma_sync_m();
    issue_rows(0, 0);
    dma_sync_m();
    auto& W = S.Pm[SPLIT ? 0 : m];                   // this wave's tower
    const float* lstd = S.Pm[SPLIT ? 0 : 1].logstd;  // actor logstd (SPLIT critic: zeros, unused)

    const int step0 = a.step[p];
    const double lr = a.lr[p];
    const float b1c = a.hp.beta1, b2c = a.hp.beta2, eps = a.hp.adam_eps;
    const float vscale = a.hp.value_loss_coef * 0.5f / (float)(mb * K);
    const float ascale = -1.f / (float)mb;
    const float vstat = 0.5f / (float)(mb * K), astat = 1.f / (float)mb;  // loss statistics scales
    float st_v = 0.f, st_a = 0.f, st_e = 0.f;
    int nstep = 0, gp = 0;
    double b1p = pow((double)b1c, (double)step0), b2p = pow((double)b2c, (double)step0);
    float* scr = &S.big.scr[w][0][0];
    PGM_STAMP_DECL

    for (int e = 0; e < E; ++e) {
        for (int bb = 0; bb < nb; ++bb) {
            // this step's Adam scalars: beta^step carried in fp64 (torch: 1 - beta ** step), lr / bias correction 1,
            // 1 / sqrt(bias correction 2); MODE 2 forms them while its image stores drain
            double b1n = 0.0, b2n = 0.0;
            float step_size = 0.f, inv_bc2s = 0.f;
            auto adam_scalars = [&]() {
                b1n = b1p * (double)b1c;
                b2n = b2p * (double)b2c;
                step_size = (float)(lr / (1.0 - b1n));
                inv_bc2s = 1.f / (float)sqrt(1.0 - b2n);
                asm volatile("" : "+v"(step_size), "+v"(inv_bc2s));  // formed HERE (the compiler would sink them)
            };
            f32x16 gW2[2][2], gW1[2];  // [in tile][out tile], [out tile] (O <= 32: one in tile)
            float gWh[2][Q], gB1[2], gB2[2];
            float gsm = 0.f;  // lanes q < Q: head-bias gradient q; lanes 32 + q (actor): logstd gradient q
#pragma unroll
            for (int i = 0; i < 2; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j) gW2[i][j] = f32x16{0};
                gW1[i] = f32x16{0};
                gB1[i] = gB2[i] = 0.f;
#pragma unroll
                for (int q = 0; q < Q; ++q) gWh[i][q] = 0.f;
            }
            float lsum = 0.f;

            for (int s0 = 0; ONE ? s0 < 1 : s0 < mbs; s0 += (ONE ? 1 : SBk), ++gp) {
                const int ns = ONE ? SBk : min(SBk, mbs - s0);
                const int cur = NBUF == 2 ? (gp & 1) : 0;
                // stage the next pass while this one computes
                if constexpr (NBUF == 2 && !EARLY_STAGE) {
                    if (gp + 1 < npass) issue_rows(cur ^ 1, (gp + 1) & 1);
                    if (gp + 2 < npass) issue_idx(gp + 2, gp & 1);
                }
                const float* rb = &S.RB[cur][0];
                PGM_STAMP(0);

                for (int tile = sh; ONE ? tile < sh + 1 : tile * TS < ns; tile += (ONE ? 1 : NWT)) {
                    const int ts0 = tile * TS;
                    const float* rt = rb + ts0 * RSL;  // this tile's staged rows
                    // ---- layer 1: Z1[s][h] = X[s][:] . W1t[:][h]  (two independent accumulator chains
                    // interleaved: the 32x32x2 f32 MFMA has a 64-cycle dependent-accumulator latency)
                    f32x16 z[2] = {f32x16{0}, f32x16{0}};
                    f32x16 H1[2];
#pragma unroll
                    for (int ks = 0; ks < KS1; ++ks) {
                        const int k = 2 * ks + h;
                        const float av = k < O ? rowf(rt, c, k) : 0.f;
#pragma unroll
                        for (int hb = 0; hb < 2; ++hb) z[hb] = mfma(av, k < O ? W.W1t[k][hb * TS + c] : 0.f, z[hb]);
                    }
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb) {
                        const float bias = W.b1[hb * TS + c];
                        tanh_bias_pk<16>(z[hb], bias, H1[hb]);
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + hb * TS + c] = H1[hb][r];
                    }
                    wave_lds_fence();
                    // ---- layer 2: Z2[s][o] = H1[s][:] . W2t[:][o]   (A from the transpose tile)
                    z[0] = z[1] = f32x16{0};
PGM_UNROLL(ONE ? PGM_U_L2 : 8)
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
                        tanh_bias_pk<16>(z[ob], bias, H2[ob]);
                    }
                    PGM_STAMP(4);
                    wave_lds_fence();  // every lane finished reading the H1 tile
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ob * TS + c] = H2[ob][r];
                    wave_lds_fence();
                    // ---- heads on the VALU: lane = sample c, half h sums units [32h, 32h+32)
                    float outv[Q];
                    // packed: v_pk_fma_f32 over unit pairs (even / odd partial sums, added at the end; Walker P = 40
                    // 5.845 -> 5.79-5.83 ms against one scalar FMA chain per output)
                    f2v acc2[Q];
#pragma unroll
                    for (int q = 0; q < Q; ++q) acc2[q] = f2v{0.f, 0.f};
PGM_UNROLL(16)
                    for (int u2 = 0; u2 < TS / 2; ++u2) {
                        const f2v hv = f2v{scr[c * SCR + h * TS + 2 * u2], scr[c * SCR + h * TS + 2 * u2 + 1]};
#pragma unroll
                        for (int q = 0; q < Q; ++q)
                            acc2[q] = __builtin_elementwise_fma(hv, *reinterpret_cast<const f2v*>(&W.Wh[q][h * TS + 2 * u2]),
                                                                acc2[q]);
                    }
#pragma unroll
                    for (int q = 0; q < Q; ++q) outv[q] = acc2[q].x + acc2[q].y;
#pragma unroll
                    for (int q = 0; q < Q; ++q) outv[q] = half_sum(outv[q]) + W.bh[q];
                    PGM_STAMP(16);
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
                            const float V = outv[q], Vo = rowf(rt, c, O + A + 2 + q);
                            const float R = rowf(rt, c, O + A + 2 + K + q);
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
                            const float diff = rowf(rt, c, O + q) - outv[q];
                            lp += -0.5f * diff * diff * S.aiv[q] - lstd[q] - LOG_SQRT_2PI;
                        }
                        const float ratio = expf(lp - rowf(rt, c, O + A));
                        const float ad = rowf(rt, c, O + A + 1);
                        const float s1 = ratio * ad;
                        const float s2 = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip) * ad;
                        const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
                        const float gr = ad * (wmin2(s1, s2) + wmin2(s2, s1) * inr);
                        const float dlp = ok ? ascale * gr * ratio : 0.f;
                        if (ok && h == 0) lsum += -fminf(s1, s2);
#pragma unroll
                        for (int q = 0; q < A; ++q) {
                            const float diff = rowf(rt, c, O + q) - outv[q];
                            const float iv = S.aiv[q];
                            dO[q] = dlp * diff * iv;
                            if (h == 0) S.dls[w][c][q] = dlp * (diff * diff * iv - 1.f);
                        }
                    }
                    if (h == 0) {
#pragma unroll
                        for (int q = 0; q < Q; ++q) S.dout[w][c][q] = dO[q];
                    }
                    PGM_STAMP(17);
                    wave_lds_fence();
                    PGM_STAMP(18);
                    // per-column sums of the tile (registers: one accumulator per lane instead of Q + A):
                    // lane q sums dO[.][q], lane 32 + q the logstd terms
                    if (c < (h == 0 ? Q : (m == 1 ? A : 0))) {
                        const float* src = (h == 0 ? &S.dout[w][0][0] : &S.dls[w][0][0]) + c;
#pragma unroll 8
                        for (int cc = 0; cc < TS; ++cc) gsm += src[cc * Q];
                    }
                    PGM_STAMP(5);
                    // ---- head-weight grads (VALU, C layout): gWh[ob][q] += sum_r H2[s][u] dO[s][q]; output pairs on the
                    // packed ALU (each output still sums over r in order: the same values)
                    constexpr bool GWH_PK = Q % 2 == 0;
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int s = rowof(r, h);
                            if constexpr (GWH_PK) {
                                const f2v hv = f2v{H2[ob][r], H2[ob][r]};
#pragma unroll
                                for (int q = 0; q < Q; q += 2) {
                                    const f2v a2 = __builtin_elementwise_fma(
                                        hv, *reinterpret_cast<const f2v*>(&S.dout[w][s][q]), f2v{gWh[ob][q], gWh[ob][q + 1]});
                                    gWh[ob][q] = a2.x;
                                    gWh[ob][q + 1] = a2.y;
                                }
                            } else {
#pragma unroll
                                for (int q = 0; q < Q; ++q) gWh[ob][q] = fmaf(H2[ob][r], S.dout[w][s][q], gWh[ob][q]);
                            }
                        }
                    // ---- dH2 = dO . Wh  (MFMA; A = this lane's sample, k = head output) -> dZ2
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
                    for (int ob = 0; ob < 2; ++ob) {
                        dtanh_pk<16>(z[ob], H2[ob], dZ2[ob]);
#pragma unroll
                        for (int r = 0; r < 16; ++r) gB2[ob] += dZ2[ob][r];
                    }
                    PGM_STAMP(6);
                    // ---- dH1 = dZ2 W2  (A = dZ2 through the transpose tile, B = W2t[in][o] column); the critical
                    // path, so its MFMAs go into the pipe first and dW2 queues behind them
                    wave_lds_fence();  // heads finished reading the H2 tile
#pragma unroll
                    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
                        for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ob * TS + c] = dZ2[ob][r];
                    wave_lds_fence();
                    z[0] = z[1] = f32x16{0};
PGM_UNROLL(ONE ? PGM_U_L2 : 8)
                    for (int ks = 0; ks < H / 2; ++ks) {
                        const int k = 2 * ks + h;  // output unit o
                        const float av = scr[c * SCR + k];
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib) z[ib] = mfma(av, W.W2t[ib * TS + c][k], z[ib]);
                    }
                    // ---- dW2^T[in][o] += H1^T dZ2: straight from the C-layout registers, behind dH1 in the MFMA pipe
                    // while the VALU forms dZ1 from the dH1 results
#pragma unroll
                    for (int r = 0; r < 16; ++r)
#pragma unroll
                        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
                            for (int ob = 0; ob < 2; ++ob) gW2[ib][ob] = mfma(H1[ib][r], dZ2[ob][r], gW2[ib][ob]);
                    f32x16 dZ1[2];
#pragma unroll
                    for (int ib = 0; ib < 2; ++ib) {
                        dtanh_pk<16>(z[ib], H1[ib], dZ1[ib]);
#pragma unroll
                        for (int r = 0; r < 16; ++r) gB1[ib] += dZ1[ib][r];
                    }
                    // ---- dW1^T[k][h] += X^T dZ1  (A = X[s(r)][k = lane], B = dZ1 reg r)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float av = c < O ? rowf(rt, rowof(r, h), c) : 0.f;
#pragma unroll
                        for (int hb = 0; hb < 2; ++hb) gW1[hb] = mfma(av, dZ1[hb][r], gW1[hb]);
                    }
                    wave_lds_fence();  // dH1 finished reading the dZ2 tile before the next tile's writes
                    PGM_STAMP(7);
                }  // tiles
                if constexpr (EARLY_STAGE) {
                    lds_sync_m();  // every wave's tiles done: the image rounds below overwrite the transpose tiles
                } else if constexpr (NBUF == 2) {
                    dma_sync_m();  // next pass landed (issued a pass ago); this buffer free for reuse
                } else {
                    lds_sync_m();
                    if (gp + 1 < npass) {
                        issue_rows(0, (gp + 1) & 1);
                        if (gp + 2 < npass) issue_idx(gp + 2, gp & 1);
                        dma_sync_m();
                    }
                }
                PGM_STAMP(1);
            }  // passes
            // (gp is now the next pass)

            // ---- combine the lane halves of the per-column partial sums
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                gB1[i] = half_sum(gB1[i]);
                gB2[i] = half_sum(gB2[i]);
#pragma unroll
                for (int q = 0; q < Q; ++q) gWh[i][q] = half_sum(gWh[i][q]);
            }
            lsum = wave_sum64(lsum);
            // entropy with the logstd of this step (before Adam)
            float ent = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) ent += 0.5f + LOG_SQRT_2PI + lstd[q];
            PGM_STAMP(12);

            // ---- gradient images.  The two waves of a pair (SPLIT: waves 0/1 -> GA[0], 2/3 -> GA[1]; joint: the
            // two waves of tower m -> GA[m]) split the image in two halves: in stage 0 each stores its partial of
            // one half, in stage 1 it adds its partial of the other half; g = GA[0] + GA[1] (joint: GA[m]).
            // Every element is (partial of one wave) + (partial of the other): deterministic.
            if (l == 0) S.red[8 + w] = lsum;
            {
                const int pr = SPLIT ? (w & 1) : sh;  // position in the pair
                float* Gt = S.big.GA[SPLIT ? (w >> 1) : m];
                for (int stage = 0; stage < 2; ++stage) {
                    const bool add = stage == 1;
                    const int half = (stage == 0) == (pr == 1) ? 0 : 1;  // image half handled in this stage
                    auto acc = [&](int idx, float val) {
                        if (add) lds_add(&Gt[idx], val);
                        else Gt[idx] = val;
                    };
                    // 16-register blocks; stage 1 adds in the LDS (ds_add_f32: no read latency in the wave)
                    auto acc16 = [&](auto idx, const f32x16& val) {
                        if (add) {
#pragma unroll
                            for (int r = 0; r < 16; ++r) lds_add(&Gt[idx(r)], val[r]);
                        } else {
#pragma unroll
                            for (int r = 0; r < 16; ++r) Gt[idx(r)] = val[r];
                        }
                    };
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (i != half) continue;
#pragma unroll
                        for (int ob = 0; ob < 2; ++ob)
                            acc16([&](int r) { return oW2 + (i * TS + rowof(r, h)) * SCR + ob * TS + c; }, gW2[i][ob]);
                        // rows k >= O of dW1 are exactly zero (A operand 0); they go to distinct W2 padding
                        // slots (column H of row k), which hold zeros
                        acc16([&](int r) {
                            const int k = rowof(r, h);
                            return k < O ? k * H + i * TS + c : oW2 + k * SCR + H;
                        }, gW1[i]);
                        if (h == 0) {  // per-unit sums of unit block i: b1, b2 and the head weights
                            constexpr int NU = 2 + Q;
                            float val[NU], tmp[NU];
                            int idx[NU];
                            idx[0] = oB1 + i * TS + c;
                            val[0] = gB1[i];
                            idx[1] = oB2 + i * TS + c;
                            val[1] = gB2[i];
#pragma unroll
                            for (int q = 0; q < Q; ++q) {  // rows q >= NQ are padding (zeroed below)
                                idx[2 + q] = oWh + q * H + i * TS + c;
                                val[2 + q] = q < NQ ? gWh[i][q] : 0.f;
                            }
                            if (add) {
#pragma unroll
                                for (int j = 0; j < NU; ++j) lds_add(&Gt[idx[j]], val[j]);
                            } else {
#pragma unroll
                                for (int j = 0; j < NU; ++j) Gt[idx[j]] = val[j];
                            }
                        }
                    }
                    if (half == 1) {
                        if (h == 0 && c < NQ) acc(oBh + c, gsm);
                        if (m == 1 && h == 1 && c < A) {  // -entropy_coef * d(mean entropy)/d logstd enters once (ppo.py:98)
                            const float ec = add || hs != 0 || (w >> 1) != 0 ? 0.f : a.hp.entropy_coef;  // once per tower: part 0, image 0
                            acc(oLs + c, gsm - ec);
                        }
                        if (!add) {  // padding slots of a freshly written image
                            Gt[oW2 + l * SCR + H] = 0.f;
                            for (int q = NQ; q < Q; ++q) Gt[oWh + q * H + l] = 0.f;
                            if (l >= NQ && l < Q) Gt[oBh + l] = 0.f;
                            if (m == 0 && l < A) Gt[oLs + l] = 0.f;
                        }
                    }
                    PGM_STAMP(13 + stage);
                    lds_sync_m();
                    if (stage == 0) PGM_STAMP(15);
                }
            }
            PGM_STAMP(2);
            constexpr int NV4 = IMG / 4, TAIL = IMG - 4 * NV4;
            constexpr int NG4 = (NV4 + MT - 1) / MT;  // MODE 2: float4 groups per thread
            float4 ag[NS == 2 ? NG4 : 1], am[NS == 2 ? NG4 : 1], av[NS == 2 ? NG4 : 1], ap[NS == 2 ? NG4 : 1];
            float agt = 0.f, sq2 = 0.f;
            if constexpr (NS == 2) {
                // ---- add the other half's gradient image.  Publish: 16-B sc1 (write-through) buffer stores,
                // every wave drains them, barrier, ONE lane stores the tagged flag granule {step, loss sum}.
                // Consume: ONE lane polls the partner's flag, barrier, 16-B sc1 loads of its image (no acquire
                // fence needed: every load of the handed-off bytes is sc1; cdna_hip_programming.md G16 R1).
                // Slots are double-buffered by step parity: a half can only rewrite a slot after the partner
                // has published the next step, i.e. after it finished reading this one.
                const unsigned tag = (unsigned)(nstep + 1);
                const int par = nstep & 1;
                const int slot_mine = ((p * 2 + m) * 2 + hs) * 2 + par;
                const int slot_other = ((p * 2 + m) * 2 + (1 - hs)) * 2 + par;
                const int off_mine = slot_mine * a.xslot * 8, off_other = slot_other * a.xslot * 8;
                const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(a.xb, 0, a.xbytes, 0x00020000);
                constexpr int SC1 = 16;  // cache-policy aux bit of the buffer builtins: sc1
                float* G0 = S.big.GA[0];
                const float* G1 = S.big.GA[1];
                const float lsum_wg = (S.red[8] + S.red[9]) + (S.red[10] + S.red[11]);
                dbg_delay(a.dbg, nstep, 0);
                for (int i = t; i < NV4; i += MT) {
                    u32x4 v;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float g = G0[4 * i + q] + G1[4 * i + q];
                        G0[4 * i + q] = g;
                        v[q] = __float_as_uint(g);
                    }
                    __builtin_amdgcn_raw_buffer_store_b128(v, xr, off_mine + 16 * i, 0, SC1);
                }
                if (t < TAIL) {
                    const float g = G0[4 * NV4 + t] + G1[4 * NV4 + t];
                    G0[4 * NV4 + t] = g;
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g), xr, off_mine + 16 * NV4 + 4 * t, 0, SC1);
                }
                adam_scalars();  // fp64 bias corrections while the stores drain
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
                lds_sync_m();
                PGM_STAMP(10);
                if constexpr (EARLY_STAGE) {  // next pass: rows by waves 1-3 while wave 0 polls
                    if (w != 0) {
                        if (gp < npass) issue_rows_n(gp & 1, gp & 1, w - 1, ic<3>{});
                        if (gp + 1 < npass) issue_idx(gp + 1, (gp + 1) & 1, w - 1, 3);
                    }
                }
                // the other tower's half slots (their images are gathered too)
                const int slot_t0 = ((p * 2 + (1 - m)) * 2 + 0) * 2 + par;
                const int off_t0 = slot_t0 * a.xslot * 8, off_t1 = (slot_t0 + 2) * a.xslot * 8;
                if (t < 3) {  // lane 0: the partner half; lanes 1, 2: the other tower's halves
                    if (t == 0) {
                        unsigned long long* flag_mine = a.xb + (size_t)slot_mine * a.xslot + a.xslot - 1;
                        __hip_atomic_store(flag_mine, ((unsigned long long)tag << 32) | __float_as_uint(lsum_wg),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    dbg_delay(a.dbg, nstep, t == 0 ? 1 : 2);
                    const int pslot = t == 0 ? slot_other : slot_t0 + 2 * (t - 1);
                    const unsigned long long* flag_p = a.xb + (size_t)pslot * a.xslot + a.xslot - 1;
                    unsigned long long x = 0;
                    for (unsigned spins = 0;; ++spins) {
                        x = __hip_atomic_load(flag_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned)(x >> 32) == tag) break;
                        if (spins > (1u << 26)) {  // partner never arrived: flag the launch as failed
                            __hip_atomic_store(a.ws + 2 * a.P, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            x = 0;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    if (t == 0) {
                        const float lo = __uint_as_float((unsigned)x);
                        S.red[12] = hs == 0 ? lsum_wg + lo : lo + lsum_wg;
                    }
                }
                lds_sync_m();  // the polling lanes matched: every wave may load the partners' images
                // every image load of this thread first (the partner half's and both halves of the other tower).  (Issuing the next pass's row DMA right behind them, all four waves: 6.16 -> 6.25 ms.)
                u32x4 vo[NG4];
#pragma unroll
                for (int k = 0; k < NG4; ++k)
                    vo[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, off_other + 16 * min(t + k * MT, NV4 - 1), 0, SC1);
                float ovt = 0.f;
                if (t < TAIL)
                    ovt = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off_other + 16 * NV4 + 4 * t, 0, SC1));
                u32x4 o0[NG4], o1[NG4];
#pragma unroll
                for (int k = 0; k < NG4; ++k) {
                    const int i = min(t + k * MT, NV4 - 1);
                    o0[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, off_t0 + 16 * i, 0, SC1);
                    o1[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, off_t1 + 16 * i, 0, SC1);
                }
                float ot0 = 0.f, ot1 = 0.f;
                if (t < TAIL) {
                    ot0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off_t0 + 16 * NV4 + 4 * t, 0, SC1));
                    ot1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, off_t1 + 16 * NV4 + 4 * t, 0, SC1));
                }
                // g = half0 + half1 of this thread's float4 groups i = t + k*MT stays in registers (no LDS
                // round trip); the sum of squares is fused in
#pragma unroll
                for (int k = 0; k < NG4; ++k) {
                    const int i = min(t + k * MT, NV4 - 1);
                    const float4 mine = *reinterpret_cast<const float4*>(&G0[4 * i]);
                    const float mv[4] = {mine.x, mine.y, mine.z, mine.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float ov = __uint_as_float(vo[k][q]);
                        ag[k][q] = hs == 0 ? mv[q] + ov : ov + mv[q];
                        if (t + k * MT < NV4) sq2 = fmaf(ag[k][q], ag[k][q], sq2);
                    }
                }
                if (t < TAIL) {
                    const float mine = G0[4 * NV4 + t];
                    agt = hs == 0 ? mine + ovt : ovt + mine;
                    sq2 = fmaf(agt, agt, sq2);
                }
                // the other tower's g = half0 + half1 and its sum of squares, element by element in the owner's order
                // (the owner forms the same sums from its own half and this very slot pair)
                {
                    float sqo = 0.f;
#pragma unroll
                    for (int k = 0; k < NG4; ++k)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float g = __uint_as_float(o0[k][q]) + __uint_as_float(o1[k][q]);
                            if (t + k * MT < NV4) sqo = fmaf(g, g, sqo);
                        }
                    if (t < TAIL) {
                        const float g = ot0 + ot1;
                        sqo = fmaf(g, g, sqo);
                    }
                    sqo = wave_sum64(sqo);
                    if (l == 0) S.red[4 + w] = sqo;
                }
                // the Adam operands of the same groups
#pragma unroll
                for (int k = 0; k < NG4; ++k) {
                    const int i = min(t + k * MT, NV4 - 1);
                    am[k] = *reinterpret_cast<const float4*>(&S.MV[4 * i]);
                    av[k] = *reinterpret_cast<const float4*>(&S.MV[IMG + 4 * i]);
                    ap[k] = *reinterpret_cast<const float4*>(&Pf[4 * i]);
                }
                PGM_STAMP(11);
            }
            // ---- clip_grad_norm_ over every parameter (padding slots hold zeros)
            constexpr int NG = SPLIT ? IMG : 2 * IMG;
            const float* GA0 = S.big.GA[0];
            const float* GA1 = S.big.GA[1];
            // SPLIT: g = GA[0] + GA[1] (MODE 2: already summed into GA[0]); joint: GA[0..1] contiguous
            auto gval = [&](int i) { return SPLIT && NS == 1 ? GA0[i] + GA1[i] : GA0[i]; };
            float sq = sq2;
            if constexpr (NS != 2) {
                for (int i = t; i < NG; i += MT) {
                    const float g = gval(i);
                    sq = fmaf(g, g, sq);
                }
            }
            sq = wave_sum64(sq);
            if (l == 0) S.red[w] = sq;
            lds_sync_m();
            PGM_STAMP(8);
            float total = (S.red[0] + S.red[1]) + (S.red[2] + S.red[3]);
            if constexpr (SPLIT && NS == 2) {  // the other tower's total, formed here
                const float other = (S.red[4] + S.red[5]) + (S.red[6] + S.red[7]);
                total = m == 0 ? total + other : other + total;  // critic + actor in all four workgroups
            } else if constexpr (SPLIT) {  // tagged 8-byte granule hand-off with the other tower's workgroup
                if (t == 0) {
                    const unsigned tag = (unsigned)(nstep + 1);
                    unsigned long long* ws = a.ws + ppo_norm_granule(a.P, p, 0, hs, nstep & 1);
                    __hip_atomic_store(ws + m, ((unsigned long long)tag << 32) | __float_as_uint(total),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    dbg_delay(a.dbg, nstep, 2);
                    unsigned long long x = 0;
                    const bool failed = __hip_atomic_load(a.ws + 2 * a.P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    for (unsigned spins = 0; !failed; ++spins) {
                        x = __hip_atomic_load(ws + (1 - m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned)(x >> 32) == tag) break;
                        if (spins > (1u << 26)) {  // partner never arrived: flag the launch as failed
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
            PGM_STAMP(9);
            const float coef = clip_coef(a.hp.max_grad_norm, total);
            if (t == 0) {
                if constexpr (SPLIT) {
                    const float ls = NS == 2 ? S.red[12] : (S.red[8] + S.red[9]) + (S.red[10] + S.red[11]);
                    if (m == 0) st_v += ls * vstat;
                    else st_a += ls * astat;
                } else {
                    st_v += (S.red[8] + S.red[10]) * vstat;
                    st_a += (S.red[9] + S.red[11]) * astat;
                }
                st_e += ent;
            }
            // ---- Adam, one flat pass over the images (padding: g = m = v = 0 keeps p = 0)
            ++nstep;
            if constexpr (NS != 2) adam_scalars();
            b1p = b1n;
            b2p = b2n;
            auto adam1 = [&](float g, float& mm, float& vv, float& pp) {
                const float gc = g * coef;
                mm = mm + (1.f - b1c) * (gc - mm);
                vv = vv * b2c + (1.f - b2c) * (gc * gc);
                // torch: p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps); hardware sqrt / rcp
                const float den = __builtin_amdgcn_sqrtf(vv) * inv_bc2s + eps;
                pp -= step_size * mm * __builtin_amdgcn_rcpf(den);
            };
            if constexpr (NS == 2) {  // operands already in registers (float4 groups of the gather)
#pragma unroll
                for (int k = 0; k < NG4; ++k) {
                    const int i = t + k * MT;
                    if (i >= NV4) break;
                    float* g4 = &ag[k].x;
                    float* m4 = &am[k].x;
                    float* v4 = &av[k].x;
                    float* p4 = &ap[k].x;
#pragma unroll
                    for (int q = 0; q < 4; ++q) adam1(g4[q], m4[q], v4[q], p4[q]);
                    *reinterpret_cast<float4*>(&S.MV[4 * i]) = am[k];
                    *reinterpret_cast<float4*>(&S.MV[IMG + 4 * i]) = av[k];
                    *reinterpret_cast<float4*>(&Pf[4 * i]) = ap[k];
                }
                if (t < TAIL) {
                    const int i = 4 * NV4 + t;
                    float mm = S.MV[i], vv = S.MV[IMG + i], pp = Pf[i];
                    adam1(agt, mm, vv, pp);
                    S.MV[i] = mm;
                    S.MV[IMG + i] = vv;
                    Pf[i] = pp;
                }
                PGM_STAMP(19);
                // exp(-2 logstd) of the new actor logstd, by the compile-time owners of elements oLs .. oLs + A - 1
                // (inside the element loop it put a branch + exp on every element of those groups)
                if (m == 1) {
#pragma unroll
                    for (int j = 0; j < A; ++j) {
                        constexpr int e0 = oLs;
                        const int e = e0 + j;
                        if (e < 4 * NV4) {
                            const int i4 = e >> 2, k = i4 / MT;
                            if (t == i4 - k * MT) S.aiv[j] = expf(-2.f * (&ap[k].x)[e & 3]);
                        } else if (t == e - 4 * NV4) {
                            S.aiv[j] = expf(-2.f * Pf[e]);
                        }
                    }
                }
            } else if constexpr (SPLIT) {
                // batches of 4 elements per thread: every LDS read of a batch before any write
                for (int i0 = t; i0 < IMG; i0 += 4 * MT) {
                    float g[4], mm[4], vv[4], pp[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = min(i0 + j * MT, IMG - 1);
                        g[j] = gval(i);
                        mm[j] = S.MV[i];
                        vv[j] = S.MV[IMG + i];
                        pp[j] = Pf[i];
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float gc = g[j] * coef;
                        mm[j] = mm[j] + (1.f - b1c) * (gc - mm[j]);
                        vv[j] = vv[j] * b2c + (1.f - b2c) * (gc * gc);
                        // torch: p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps); hardware sqrt / rcp
                        // (<= 2 ulp on the step, against an fp64 reference anyway)
                        const float den = __builtin_amdgcn_sqrtf(vv[j]) * inv_bc2s + eps;
                        pp[j] -= step_size * mm[j] * __builtin_amdgcn_rcpf(den);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = i0 + j * MT;
                        if (i < IMG) {
                            S.MV[i] = mm[j];
                            S.MV[IMG + i] = vv[j];
                            Pf[i] = pp[j];
                            if (m == 1 && i >= oLs && i < oLs + A) S.aiv[i - oLs] = expf(-2.f * pp[j]);
                        }
                    }
                }
            } else {  // moments in HBM (flat layout)
                for (int i = t; i < NG; i += MT) {
                    const int mi = i / IMG, f = img_to_flat<O, A, K>(i - mi * IMG, mi, L);
                    if (f < 0) continue;
                    const float g = gval(i) * coef;
                    float mm = Mo[f], vv = Vo[f];
                    mm = mm + (1.f - b1c) * (g - mm);
                    vv = vv * b2c + (1.f - b2c) * (g * g);
                    Mo[f] = mm;
                    Vo[f] = vv;
                    const float pn = Pf[i] - step_size * (mm / (sqrtf(vv) * inv_bc2s + eps));
                    Pf[i] = pn;
                    if (i >= IMG + oLs && i < IMG + oLs + A) S.aiv[i - IMG - oLs] = expf(-2.f * pn);
                }
            }
            if constexpr (EARLY_STAGE) dma_sync_m();  // + the next pass's rows landed
            else lds_sync_m();  // parameters updated before the next minibatch; GA region reused as scr
            PGM_STAMP(3);
        }  // minibatches
    }      // epochs
    // ---- write back (parameters; SPLIT also the moments); MODE 2: the halves hold identical copies
    if (hs != 0) {
        PGM_STAMP_FLUSH;
        return;
    }
    for (int i = t; i < NT * IMG; i += MT) {
        const int mi = i / IMG, f = img_to_flat<O, A, K>(i - mi * IMG, img_tower(mi), L);
        if (f < 0) continue;
        P[f] = Pf[i];
        if constexpr (SPLIT) {
            Mo[f] = S.MV[i];
            Vo[f] = S.MV[IMG + i];
        }
    }
    if (t == 0) {
        const float n = (float)(E * M);
        if (!SPLIT || m == 0) a.stats[p * 3 + 0] = st_v / n;
        if (!SPLIT || m == 1) {
            a.step[p] = step0 + nstep;
            a.stats[p * 3 + 1] = st_a / n;
            a.stats[p * 3 + 2] = st_e / n;
        }
    }
    PGM_STAMP_FLUSH;
}

// ================================================================ 16-row tiles, NS workgroups per tower
// ppo_update_t16_kernel<O, A, K, NS, W>: each tower of a task runs on NS workgroups of W waves; workgroup hs
// takes rows [hs mb / NS, (hs + 1) mb / NS) of every minibatch, one 16-sample tile per wave on the
// v_mfma_f32_16x16x4_f32 (half the rows of the 32x32x2 tile, so a tile's dependent chain is about half as
// long, and with W = 8 two waves share each SIMD's matrix pipe).  Layout of the 16x16x4 form:
//     C/D:  lane l, register r  <->  (sample 4(l >> 4) + r, feature l & 15)
//     A:    lane l holds A[i = l & 15][k = l >> 4];   B: lane l holds B[k = l >> 4][j = l & 15]
// so, as in the 32-row kernel, weight gradients (sums over samples) take both operands straight from the C
// registers (register r = k-step r), and only the feature-contracting products (Z2 = H1 W2^T,
// dH1 = dZ2 W2, the heads) transpose through a per-wave LDS tile.  The heads run on the MFMA too, which
// leaves every per-(sample, output) loss term in C layout: the actor's log-prob sums over the outputs of a
// sample are 16-lane DPP row sums.
//
// Per minibatch step: the W waves' register partials are summed into ONE LDS image in W rounds (round j:
// wave w adds its blocks of slice (w + j) mod W; every slice is summed in a fixed wave order), the NS
// images of a tower are exchanged through 16-B sc1 publishes + tagged flags (every workgroup sums them in
// row-part order h = 0..NS-1, so all NS copies of the Adam step are bitwise identical), the two towers
// exchange their squared norms as tagged 8-byte granules, and Adam runs from registers.


template <int O, int A, int K, int W, int NBUF, int NIMG_>
struct T16SmemT {
    static constexpr int Q = qmax<A, K>();
    static constexpr int IMG = img_floats<O, A, K>();
    static constexpr int RS = row_stride<O, A, K>();
    static constexpr int SBk = W * T16;     // samples staged per pass (one tile per wave)
    static constexpr int RSL = RS + 4;
    TowerImg<O, A, K> Pm;                   // parameters of this workgroup's tower
    float MV[2 * IMG];                      // Adam exp_avg | exp_avg_sq images
    alignas(16) float RB[NBUF][SBk * RSL];  // packed rows of the current / next pass
    int32_t IB[2][SBk];                     // sample indices of the next two passes
    float dout[W][T16][DQS];                // per-wave dL/d(head output), transposed for dH2
    float aiv[A];                           // actor 1 / std^2
    float red[32];
    static constexpr int NIMG = NIMG_;  // 2: waves [0, W/2) and [W/2, W) fill one image each
    static constexpr int IMGP = (IMG + 3) & ~3;  // image stride: every image 16-B aligned (float4 / LDS-DMA)
    union alignas(16) Big {
        float scr[W][T16][S16];             // transpose tiles during the passes
        float GA[NIMG][IMGP];               // the workgroup's gradient image(s) after them
    } big;
};
// LDS plan: double-buffered staging first, then two gradient images (W >= 4), within the 160 KiB of a CU
template <int O, int A, int K, int W>
constexpr int t16_nbuf() { return sizeof(T16SmemT<O, A, K, W, 2, 1>) <= 160 * 1024 ? 2 : 1; }
template <int O, int A, int K, int W>
constexpr int t16_nimg() {
    return W >= 4 && sizeof(T16SmemT<O, A, K, W, t16_nbuf<O, A, K, W>(), 2>) <= 160 * 1024 ? 2 : 1;
}
template <int O, int A, int K, int W>
using T16Smem = T16SmemT<O, A, K, W, t16_nbuf<O, A, K, W>(), t16_nimg<O, A, K, W>()>;

// ONE: the launcher checked mb == NS * W * 16 (every wave owns exactly one tile of one pass per minibatch), so
// the pass and tile loops are straight-line and the gradient accumulators are no longer loop-carried: they go
// live at their first MFMA instead of spanning the whole tile (W = 8: no spills)
template <int O, int A, int K, int NS, int W, bool ONE>
__global__ __launch_bounds__(64 * W) void ppo_update_t16_kernel(MArgs a) {
    static_assert(O <= 32, "two 16-feature blocks of layer-1 inputs");
    using Sm = T16Smem<O, A, K, W>;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<Sm*>(smem_raw);
    constexpr int NT = 64 * W;
    constexpr int Q = qmax<A, K>();
    static_assert(Q <= DQ, "head outputs beyond the dO tile");
    constexpr int KS1 = (O + 3) / 4;   // k-steps of layer 1
    constexpr int K1B = (O + 15) / 16; // 16-feature blocks of the layer-1 inputs
    constexpr int IMG = Sm::IMG, SBk = Sm::SBk, RS = Sm::RS, RSL = Sm::RSL;
    constexpr int NBUF = t16_nbuf<O, A, K, W>();
    constexpr int CR = RS / 4;
    // single-tile: the next pass's row DMA by waves 1..W-1 while wave 0 polls the tower-norm granule, retired by the
    // step's last barrier (as in the 32-row kernel)
    constexpr bool EARLY_STAGE = ONE && NBUF == 2 && W > 1;
    constexpr int NDT = (SBk * RSL) / 256;
    static_assert(NDT * 256 == SBk * RSL, "staging split");
    constexpr int oW2 = O * H, oWh = oW2 + H * SCR, oB1 = oWh + Q * H, oB2 = oB1 + H, oBh = oB2 + H, oLs = oBh + Q;
    const int t = threadIdx.x, l = t & 63, g = l >> 4, c = l & 15;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    // block map (speed only: the hand-offs are correct under any placement; blocks b, b + 8, ... share an XCD under
    // round-robin dispatch)
    const int bx = (int)blockIdx.x;
    // groups of 16 NS blocks for 8 tasks: block r holds part (r >> 4) % NS of tower (r >> 3) & 1 of task 8 G + (r & 7)
    const int j16 = (bx >> 3) % (2 * NS);
    const int p = 8 * (bx / (16 * NS)) + (bx & 7);
    const int hs = j16 >> 1, m = j16 & 1;
    if (p >= a.P) return;
    const int NQ = m == 0 ? K : A;
    const int N = a.N, T = a.T, B = T * N;
    const int E = a.hp.ppo_epoch, M = a.hp.num_mini_batch;
    const int mb = B / M, nb = B / mb;
    const int r0 = hs * mb / NS, mbs = (hs + 1) * mb / NS - r0;
    const int npm = (mbs + SBk - 1) / SBk;
    const int npass = E * nb * npm;
    const float clip = a.hp.clip_param;
    const Layout& L = a.L;
    float* __restrict__ P = a.params + (size_t)p * L.total;
    float* __restrict__ Mo = a.m + (size_t)p * L.total;
    float* __restrict__ Vo = a.v + (size_t)p * L.total;
    const float* rows = a.rows + (size_t)p * B * RS;

    // (wi, nwv): this wave's index among the nwv waves sharing the issue
    auto issue_idx = [&](int gi, int buf, int wi = -1, int nwv = W) {
        if (wi < 0) wi = w;
        const int e = gi / (nb * npm), rem = gi - e * nb * npm, bb = rem / npm, j = rem - bb * npm;
        const int ns = min(SBk, mbs - j * SBk);
        const int32_t* src = a.perms + (size_t)e * B + bb * mb + r0 + j * SBk;
        for (int q0 = wi * 64; q0 < SBk; q0 += 64 * nwv)  // rows beyond ns re-read the last valid index
            __builtin_amdgcn_global_load_lds((const void*)(src + min(q0 + l, ns - 1)),
                                             (lds_void_t*)&S.IB[buf][q0], 4, 0, 0);
    };
    auto issue_rows_n = [&](int buf, int ibuf, int wi, auto nwc) {
        constexpr int NWV = decltype(nwc)::value;
        float* base = &S.RB[buf][0];
        constexpr int NI = (NDT + NWV - 1) / NWV;
        int idx[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int d = wi + NWV * i, pos = d * 256 + 4 * l, row = min(pos / RSL, SBk - 1);
            idx[i] = S.IB[ibuf][row];
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int d = wi + NWV * i;
            if (d < NDT) {
                const int pos = d * 256 + 4 * l, row = pos / RSL, chunk = (pos - row * RSL) >> 2;
                const float* src = rows + (size_t)idx[i] * RS + (chunk < CR ? chunk : 0) * 4;
                __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(base + d * 256), 16, 0, 0);
            }
        }
    };
    auto issue_rows = [&](int buf, int ibuf) { issue_rows_n(buf, ibuf, w, ic<W>{}); };

    // ---- parameter and Adam moment images from the flat HBM vectors
    float* Pf = &S.Pm.W1t[0][0];
    if (t < A) S.aiv[t] = expf(-2.f * P[L.off[PGM_P_LOGSTD] + t]);
    for (int i = t; i < IMG; i += NT) {
        const int f = img_to_flat<O, A, K>(i, m, L);
        Pf[i] = f >= 0 ? P[f] : 0.f;
        S.MV[i] = f >= 0 ? Mo[f] : 0.f;
        S.MV[IMG + i] = f >= 0 ? Vo[f] : 0.f;
    }
    issue_idx(0, 0);
    if (npass > 1) issue_idx(1, 1);
    dma_sync_m();
    issue_rows(0, 0);
    dma_sync_m();
    auto& Wt = S.Pm;
    const float* lstd = S.Pm.logstd;  // actor logstd (critic: zeros, unused)

    const int step0 = a.step[p];
    const double lr = a.lr[p];
    const float b1c = a.hp.beta1, b2c = a.hp.beta2, eps = a.hp.adam_eps;
    const float vscale = a.hp.value_loss_coef * 0.5f / (float)(mb * K);
    const float ascale = -1.f / (float)mb;
    const float vstat = 0.5f / (float)(mb * K), astat = 1.f / (float)mb;  // loss statistics scales
    float st_v = 0.f, st_a = 0.f, st_e = 0.f;
    int nstep = 0, gp = 0;
    double b1p = pow((double)b1c, (double)step0), b2p = pow((double)b2c, (double)step0);
    float* scr = &S.big.scr[w][0][0];
    float* dtile = &S.dout[w][0][0];
    PGM_STAMP_DECL

    for (int e = 0; e < E; ++e) {
        for (int bb = 0; bb < nb; ++bb) {
            f32x4 gW2[4][4], gW1[K1B][4], gWh[4];
            float gB1[4], gB2[4], gbh = 0.f, gls = 0.f, lsum = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int j = 0; j < 4; ++j) gW2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kb = 0; kb < K1B; ++kb) gW1[kb][i] = f32x4{0.f, 0.f, 0.f, 0.f};
                gWh[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                gB1[i] = gB2[i] = 0.f;
            }

            for (int s0 = 0; ONE ? s0 < 1 : s0 < mbs; s0 += (ONE ? 1 : SBk), ++gp) {
                const int ns = ONE ? SBk : min(SBk, mbs - s0);
                const int cur = NBUF == 2 ? (gp & 1) : 0;
                if constexpr (NBUF == 2 && !EARLY_STAGE) {
                    if (gp + 1 < npass) issue_rows(cur ^ 1, (gp + 1) & 1);
                    if (gp + 2 < npass) issue_idx(gp + 2, gp & 1);
                }
                const float* rb = &S.RB[cur][0];
                PGM_STAMP(0);

                for (int tile = w; ONE ? tile < w + 1 : tile * T16 < ns; tile += (ONE ? 1 : W)) {
                    const int ts0 = tile * T16;
                    const float* rt = rb + ts0 * RSL;
                    // ---- layer 1: Z1[s][h] = X[s][:] . W1t[:][h]
                    f32x4 z[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                                  f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                    for (int ks = 0; ks < KS1; ++ks) {
                        const int k = 4 * ks + g;
                        const bool kv = k < O;
                        const float av = kv ? rt[c * RSL + k] : 0.f;
#pragma unroll
                        for (int hb = 0; hb < 4; ++hb) z[hb] = mfma16(av, kv ? Wt.W1t[kv ? k : 0][hb * T16 + c] : 0.f, z[hb]);
                    }
                    f32x4 H1[4];
#pragma unroll
                    for (int hb = 0; hb < 4; ++hb) {
                        const float bias = Wt.b1[hb * T16 + c];
                        tanh_bias_pk<4>(z[hb], bias, H1[hb]);
#pragma unroll
                        for (int r = 0; r < 4; ++r) scr[(4 * g + r) * S16 + hb * T16 + c] = H1[hb][r];
                    }
                    wave_lds_fence();
                    // ---- layer 2: Z2[s][o] = H1[s][:] . W2t[:][o]  (A from the transpose tile)
#pragma unroll
                    for (int ob = 0; ob < 4; ++ob) z[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
PGM_UNROLL(ONE ? PGM_U16 : 4)
                    for (int ks = 0; ks < H / 4; ++ks) {
                        const int k = 4 * ks + g;
                        const float av = scr[c * S16 + k];
#pragma unroll
                        for (int ob = 0; ob < 4; ++ob) z[ob] = mfma16(av, Wt.W2t[k][ob * T16 + c], z[ob]);
                    }
                    f32x4 H2[4];
#pragma unroll
                    for (int ob = 0; ob < 4; ++ob) {
                        const float bias = Wt.b2[ob * T16 + c];
                        tanh_bias_pk<4>(z[ob], bias, H2[ob]);
                    }
                    PGM_STAMP(4);
                    wave_lds_fence();  // every lane finished reading the H1 tile
#pragma unroll
                    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
                        for (int r = 0; r < 4; ++r) scr[(4 * g + r) * S16 + ob * T16 + c] = H2[ob][r];
                    wave_lds_fence();
                    // ---- heads on the MFMA: out[s][q] = H2[s][:] . Wh[q][:]  (q = lane column, < Q)
                    f32x4 ho = f32x4{0.f, 0.f, 0.f, 0.f};
                    const bool qv = c < Q;
PGM_UNROLL(ONE ? PGM_U16 : 4)
                    for (int ks = 0; ks < H / 4; ++ks) {
                        const int k = 4 * ks + g;
                        ho = mfma16(scr[c * S16 + k], qv ? Wt.Wh[qv ? c : 0][k] : 0.f, ho);
                    }
                    // ---- per-(sample, output) loss gradients in C layout (ppo.py:80-96): register r is sample
                    // 4g + r of the tile, lane column c is head output q
                    const float bh = qv ? Wt.bh[c] : 0.f;
                    f32x4 dO;
                    if (m == 0) {  // value loss over the K objectives
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int s = 4 * g + r;
                            const bool ok = ts0 + s < ns && c < K;
                            const float V = ho[r] + bh;
                            const float Vold = rt[s * RSL + O + A + 2 + (c < K ? c : 0)];
                            const float R = rt[s * RSL + O + A + 2 + K + (c < K ? c : 0)];
                            float gv, ls;
                            if (a.hp.use_clipped_value_loss) {
                                const float dv = V - Vold;
                                const float vc = Vold + fminf(fmaxf(dv, -clip), clip);
                                const float l1 = (V - R) * (V - R), l2 = (vc - R) * (vc - R);
                                const float inr = (dv >= -clip && dv <= clip) ? 1.f : 0.f;
                                gv = wmax2(l1, l2) * 2.f * (V - R) + wmax2(l2, l1) * 2.f * (vc - R) * inr;
                                ls = fmaxf(l1, l2);
                            } else {
                                gv = 2.f * (V - R);
                                ls = (R - V) * (R - V);
                            }
                            dO[r] = ok ? vscale * gv : 0.f;
                            lsum += ok ? ls : 0.f;
                        }
                    } else {  // clipped surrogate; the log-prob of a sample is a row sum over its outputs
                        const bool av_ = c < A;
                        const float aiv = S.aiv[av_ ? c : 0], ls_c = av_ ? lstd[c] : 0.f;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int s = 4 * g + r;
                            const bool ok = ts0 + s < ns;
                            const float diff = av_ ? rt[s * RSL + O + c] - (ho[r] + bh) : 0.f;
                            const float lpe = av_ ? -0.5f * diff * diff * aiv - ls_c - LOG_SQRT_2PI : 0.f;
                            const float lp = row_sum16(lpe);
                            const float ratio = expf(lp - rt[s * RSL + O + A]);
                            const float ad = rt[s * RSL + O + A + 1];
                            const float s1 = ratio * ad;
                            const float s2 = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip) * ad;
                            const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
                            const float gr = ad * (wmin2(s1, s2) + wmin2(s2, s1) * inr);
                            const float dlp = ok ? ascale * gr * ratio : 0.f;
                            lsum += (ok && c == 0) ? -fminf(s1, s2) : 0.f;
                            dO[r] = av_ ? dlp * diff * aiv : 0.f;
                            gls += av_ ? dlp * (diff * diff * aiv - 1.f) : 0.f;
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        gbh += dO[r];
                        if (c < DQ) dtile[(4 * g + r) * DQS + c] = dO[r];
                    }
                    PGM_STAMP(5);
                    // ---- head-weight gradient gWh^T[u][q] += H2^T dO  (both operands in C registers)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int ub = 0; ub < 4; ++ub) gWh[ub] = mfma16(H2[ub][r], dO[r], gWh[ub]);
                    wave_lds_fence();  // dO tile written; H2 tile reads (heads) done
                    // ---- dH2 = dO . Wh  (A = dO through its transpose tile) -> dZ2
#pragma unroll
                    for (int ob = 0; ob < 4; ++ob) z[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int ks = 0; ks < (Q + 3) / 4; ++ks) {
                        const int q = 4 * ks + g;
                        const float av = q < Q ? dtile[c * DQS + q] : 0.f;
#pragma unroll
                        for (int ob = 0; ob < 4; ++ob) z[ob] = mfma16(av, q < Q ? Wt.Wh[q < Q ? q : 0][ob * T16 + c] : 0.f, z[ob]);
                    }
                    f32x4 dZ2[4];
#pragma unroll
                    for (int ob = 0; ob < 4; ++ob) {
                        dtanh_pk<4>(z[ob], H2[ob], dZ2[ob]);
#pragma unroll
                        for (int r = 0; r < 4; ++r) gB2[ob] += dZ2[ob][r];
                    }
                    PGM_STAMP(6);
#pragma unroll
                    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
                        for (int r = 0; r < 4; ++r) scr[(4 * g + r) * S16 + ob * T16 + c] = dZ2[ob][r];
                    wave_lds_fence();
                    // ---- dH1 = dZ2 W2 (A = dZ2 through the transpose tile, B = W2t[in][o] column)
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib) z[ib] = f32x4{0.f, 0.f, 0.f, 0.f};
PGM_UNROLL(ONE ? PGM_U16 : 4)
                    for (int ks = 0; ks < H / 4; ++ks) {
                        const int k = 4 * ks + g;  // output unit o
                        const float av = scr[c * S16 + k];
#pragma unroll
                        for (int ib = 0; ib < 4; ++ib) z[ib] = mfma16(av, Wt.W2t[ib * T16 + c][k], z[ib]);
                    }
                    // ---- dW2^T[in][o] += H1^T dZ2 straight from the C registers, behind dH1 (whose MFMAs go first)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                            for (int ob = 0; ob < 4; ++ob) gW2[ib][ob] = mfma16(H1[ib][r], dZ2[ob][r], gW2[ib][ob]);
                    f32x4 dZ1[4];
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib) {
                        dtanh_pk<4>(z[ib], H1[ib], dZ1[ib]);
#pragma unroll
                        for (int r = 0; r < 4; ++r) gB1[ib] += dZ1[ib][r];
                    }
                    // ---- dW1^T[k][h] += X^T dZ1  (A = X[sample 4g + r][feature 16 kb + c], B = dZ1 register r)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
#pragma unroll
                        for (int kb = 0; kb < K1B; ++kb) {
                            const int k = kb * T16 + c;
                            const float ax = k < O ? rt[(4 * g + r) * RSL + (k < O ? k : 0)] : 0.f;
#pragma unroll
                            for (int hb = 0; hb < 4; ++hb) gW1[kb][hb] = mfma16(ax, dZ1[hb][r], gW1[kb][hb]);
                        }
                    }
                    wave_lds_fence();  // dH1 finished reading the dZ2 tile before the next tile's writes
                    PGM_STAMP(7);
                }  // tiles
                if constexpr (EARLY_STAGE) {
                    lds_sync_m();  // every wave's tiles done: the image rounds overwrite the transpose tiles
                } else if constexpr (NBUF == 2) {
                    dma_sync_m();
                } else {
                    lds_sync_m();
                    if (gp + 1 < npass) {
                        issue_rows(0, (gp + 1) & 1);
                        if (gp + 2 < npass) issue_idx(gp + 2, gp & 1);
                        dma_sync_m();
                    }
                }
                PGM_STAMP(1);
            }  // passes

            // ---- per-column sums over the four lane groups (column c of block i)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                gB1[i] = group4_sum(gB1[i]);
                gB2[i] = group4_sum(gB2[i]);
            }
            gbh = group4_sum(gbh);
            gls = group4_sum(gls);
            lsum = wave_sum64(lsum);
            float ent = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) ent += 0.5f + LOG_SQRT_2PI + lstd[q];
            if (l == 0) S.red[8 + w] = lsum;
            PGM_STAMP(12);

            // ---- the W waves' register partials -> the workgroup's image.  The two wave halves fill images A, B in
            // W/2 rounds each (round j: wave w owns slice (w mod W/2 + j) mod W/2 of its image, the first round
            // stores, later rounds add: a fixed wave order per element), and the publish sums A + B.  W = 4: every
            // element is (w0 + w1) + (w2 + w3).
            // Blocks: 0-15 dW2, 16-16+4 K1B dW1, then dWh, then the vectors (b1, b2, head bias, logstd).  The slice
            // is a compile-time parameter of the round body (a uniform branch picks it), so every (index, value)
            // pair is a register and a round's reads all issue before its writes.
            {
                constexpr int BW1 = 16, BWH = 16 + 4 * K1B, BV = BWH + 4;
                constexpr int WPI = W / Sm::NIMG;  // waves per image
                constexpr int NSL = WPI;            // slices = rounds
                float* Gt = S.big.GA[w / WPI];
                auto round = [&](auto slc, auto addc) {
                    constexpr int SL = decltype(slc)::value;
                    constexpr bool add = decltype(addc)::value != 0;
                    // one 4-register block at a time; the later rounds add in the LDS (ds_add_f32, one add per
                    // element per round: the wave order of every element stays fixed)
                    auto put4 = [&](auto idx, const f32x4& v) {
                        if constexpr (add) {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (idx(r) >= 0) lds_add(&Gt[idx(r)], v[r]);
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (idx(r) >= 0) Gt[idx(r)] = v[r];
                        }
                    };
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                        for (int ob = 0; ob < 4; ++ob)
                            if ((ib * 4 + ob) % NSL == SL)
                                put4([&](int r) { return oW2 + (ib * T16 + 4 * g + r) * SCR + ob * T16 + c; }, gW2[ib][ob]);
#pragma unroll
                    for (int kb = 0; kb < K1B; ++kb)
#pragma unroll
                        for (int hb = 0; hb < 4; ++hb)
                            if ((BW1 + kb * 4 + hb) % NSL == SL)  // rows k >= O are exactly zero and not in the image
                                put4([&](int r) { const int k = kb * T16 + 4 * g + r; return k < O ? k * H + hb * T16 + c : -1; },
                                     gW1[kb][hb]);
#pragma unroll
                    for (int ub = 0; ub < 4; ++ub)
                        if ((BWH + ub) % NSL == SL)
                            put4([&](int r) { return c < Q ? oWh + c * H + ub * T16 + 4 * g + r : -1; }, gWh[ub]);
                    if constexpr (BV % NSL == SL) {  // vectors: lanes of group 0 (every group holds the sums)
                        // -entropy_coef * d(mean entropy)/d logstd enters once (ppo.py:98)
                        const float lsv = m == 1 ? gls - (add || hs != 0 || w >= WPI ? 0.f : a.hp.entropy_coef) : 0.f;  // once per tower: part 0, image A
                        put4([&](int r) { return g == 0 ? oB1 + r * T16 + c : -1; }, f32x4{gB1[0], gB1[1], gB1[2], gB1[3]});
                        put4([&](int r) { return g == 0 ? oB2 + r * T16 + c : -1; }, f32x4{gB2[0], gB2[1], gB2[2], gB2[3]});
                        put4([&](int r) { return g == 0 && r == 0 && c < Q ? oBh + c : g == 0 && r == 1 && c < A ? oLs + c : -1; },
                             f32x4{c < NQ ? gbh : 0.f, lsv, 0.f, 0.f});
                        if (!add) Gt[oW2 + (g * T16 + c) * SCR + H] = 0.f;  // W2 padding column, rows 0..63
                    }
                };
                auto rounds = [&](int j, auto addc) {
                    const int sl = (w % WPI + j) % WPI;
                    if constexpr (NSL == 2) {
                        if (sl == 0) round(ic<0>{}, addc);
                        else round(ic<1>{}, addc);
                    } else {
                        switch (sl) {
                            case 0: round(ic<0>{}, addc); break;
                            case 1: round(ic<1 % NSL>{}, addc); break;
                            case 2: round(ic<2 % NSL>{}, addc); break;
                            case 3: round(ic<3 % NSL>{}, addc); break;
                            case 4: round(ic<4 % NSL>{}, addc); break;
                            case 5: round(ic<5 % NSL>{}, addc); break;
                            case 6: round(ic<6 % NSL>{}, addc); break;
                            default: round(ic<7 % NSL>{}, addc); break;
                        }
                    }
                };
                for (int j = 0; j < NSL; ++j) {
                    if (j == 0) rounds(j, ic<0>{});
                    else rounds(j, ic<1>{});
                    lds_sync_m();
                }
            }
            PGM_STAMP(13);

            // ---- the NS row parts' images: publish this one (16-B sc1 stores, every wave drains, barrier,
            // one lane stores the tagged flag {step, loss sum}); wait for the other parts' flags; sum the NS
            // images in part order (identical in every part) into registers, squared norm fused in
            constexpr int NV4 = IMG / 4, TAIL = IMG - 4 * NV4;
            constexpr int NG4 = (NV4 + NT - 1) / NT;
            f32x4 ag[NG4], am[NG4], av[NG4], ap[NG4];
            float agt = 0.f, sq2 = 0.f;
            float lsum_all = 0.f;
            {
                const unsigned tag = (unsigned)(nstep + 1);
                const int par = nstep & 1;
                auto slot_of = [&](int h) { return (((p * 2 + m) * NS + h) * 2 + par); };
                const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(a.xb, 0, a.xbytes, 0x00020000);
                constexpr int SC1 = 16;
                float* G0 = S.big.GA[0];
                float lsum_wg = 0.f;
#pragma unroll
                for (int i = 0; i < W; ++i) lsum_wg += S.red[8 + i];
                // this part's image (A + B summed in fixed order) in registers: published from them and
                // reused as the own term of the gather (no LDS write-back)
                f32x4 own4[NG4];
#pragma unroll
                for (int k = 0; k < NG4; ++k) {
                    const int i = min(t + k * NT, NV4 - 1);
                    const float4 v4 = *reinterpret_cast<const float4*>(&G0[4 * i]);
                    own4[k] = f32x4{v4.x, v4.y, v4.z, v4.w};
                }
                if constexpr (Sm::NIMG == 2) {
#pragma unroll
                    for (int k = 0; k < NG4; ++k) {
                        const int i = min(t + k * NT, NV4 - 1);
                        const float4 b4 = *reinterpret_cast<const float4*>(&S.big.GA[1][4 * i]);
                        own4[k] += f32x4{b4.x, b4.y, b4.z, b4.w};
                    }
                }
                if constexpr (NS > 1) {
                    dbg_delay(a.dbg, nstep, 0);
                    const int off_mine = slot_of(hs) * a.xslot * 8;
#pragma unroll
                    for (int k = 0; k < NG4; ++k) {
                        const int i = t + k * NT;
                        if (i < NV4) {
                            const u32x4 v = {__float_as_uint(own4[k][0]), __float_as_uint(own4[k][1]),
                                             __float_as_uint(own4[k][2]), __float_as_uint(own4[k][3])};
                            __builtin_amdgcn_raw_buffer_store_b128(v, xr, off_mine + 16 * i, 0, SC1);
                        }
                    }
                    if (t < TAIL) {
                        float v = G0[4 * NV4 + t];
                        if constexpr (Sm::NIMG == 2) {
                            v += S.big.GA[1][4 * NV4 + t];
                            G0[4 * NV4 + t] = v;
                        }
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), xr, off_mine + 16 * NV4 + 4 * t, 0, SC1);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
                    lds_sync_m();
                    PGM_STAMP(10);
                    if (t == 0) {
                        unsigned long long* flag_mine = a.xb + (size_t)slot_of(hs) * a.xslot + a.xslot - 1;
                        __hip_atomic_store(flag_mine, ((unsigned long long)tag << 32) | __float_as_uint(lsum_wg),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (t < NS) {  // lane h polls part h's flag: the NS - 1 polls run concurrently
                        dbg_delay(a.dbg, nstep, 1);
                        float lp = lsum_wg;
                        if (t != hs) {
                            const unsigned long long* flag_h = a.xb + (size_t)slot_of(t) * a.xslot + a.xslot - 1;
                            unsigned long long x = 0;
                            for (unsigned spins = 0;; ++spins) {
                                x = __hip_atomic_load(flag_h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                if ((unsigned)(x >> 32) == tag) break;
                                if (spins > (1u << 26)) {  // a part never arrived: flag the launch as failed
                                    __hip_atomic_store(a.ws + 2 * a.P, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    x = 0;
                                    break;
                                }
                                __builtin_amdgcn_s_sleep(1);
                            }
                            lp = __uint_as_float((unsigned)x);
                        }
                        S.red[16 + t] = lp;
                    }
                    lds_sync_m();
                    if (t == 0) {
                        float ls = 0.f;
                        for (int h = 0; h < NS; ++h) ls += S.red[16 + h];  // part order
                        S.red[4] = ls;
                    }
                    lds_sync_m();
                } else {
                    if (t == 0) S.red[4] = lsum_wg;
                    lds_sync_m();
                }
                lsum_all = S.red[4];
                if constexpr (NS == 4 && Sm::NIMG == 2) {
                    // every partner byte in flight at once: the first two partners (part order) by LDS-DMA into
                    // the two image buffers (free since own4 was formed: the barriers above), the third into
                    // registers; one retire + barrier, then the sums in part order
                    const int hA = hs == 0 ? 1 : 0, hB = hs <= 1 ? 2 : 1, hC = hs <= 2 ? 3 : 2;
                    const char* xbase = reinterpret_cast<const char*>(a.xb);
                    constexpr int NDI = (NV4 * 16 + 1023) / 1024;  // 1-KiB LDS-DMA pieces per image
                    for (int d = w; d < NDI; d += W) {
                        const int byte = d * 1024 + 16 * l;
                        if (byte < NV4 * 16) {  // the image tail (TAIL floats) stays untouched in GA[0]
                            __builtin_amdgcn_global_load_lds((const void*)(xbase + (size_t)slot_of(hA) * a.xslot * 8 + byte),
                                                             (lds_void_t*)&S.big.GA[0][d * 256], 16, 0, SC1);
                            __builtin_amdgcn_global_load_lds((const void*)(xbase + (size_t)slot_of(hB) * a.xslot * 8 + byte),
                                                             (lds_void_t*)&S.big.GA[1][d * 256], 16, 0, SC1);
                        }
                    }
                    u32x4 pc[NG4];
#pragma unroll
                    for (int k = 0; k < NG4; ++k) {
                        const int i = min(t + k * NT, NV4 - 1);
                        pc[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, slot_of(hC) * a.xslot * 8 + 16 * i, 0, SC1);
                    }
                    dma_sync_m();
#pragma unroll
                    for (int k = 0; k < NG4; ++k) {
                        const int i = min(t + k * NT, NV4 - 1);
                        const float4 va = *reinterpret_cast<const float4*>(&S.big.GA[0][4 * i]);
                        const float4 vb = *reinterpret_cast<const float4*>(&S.big.GA[1][4 * i]);
                        const f32x4 fa = f32x4{va.x, va.y, va.z, va.w}, fb = f32x4{vb.x, vb.y, vb.z, vb.w};
                        const f32x4 fc = f32x4{__uint_as_float(pc[k][0]), __uint_as_float(pc[k][1]),
                                               __uint_as_float(pc[k][2]), __uint_as_float(pc[k][3])};
                        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int h = 0; h < NS; ++h) {
                            const f32x4 v = h == hs ? own4[k] : h == hA ? fa : h == hB ? fb : fc;
                            acc = h == 0 ? v : acc + v;
                        }
                        ag[k] = acc;
                        if (t + k * NT < NV4)
#pragma unroll
                            for (int q = 0; q < 4; ++q) sq2 = fmaf(acc[q], acc[q], sq2);
                    }
                } else {
                // partner loads in flight KC groups at a time (registers), then the sums in part order
                constexpr int KC = 2;  // 3 measured slower
#pragma unroll
                for (int k0 = 0; k0 < NG4; k0 += KC) {
                    u32x4 pl[KC][NS];
#pragma unroll
                    for (int kk = 0; kk < KC; ++kk) {
                        const int i = min(t + (k0 + kk) * NT, NV4 - 1);
#pragma unroll
                        for (int h = 0; h < NS; ++h)
                            if (k0 + kk < NG4 && h != hs)
                                pl[kk][h] = __builtin_amdgcn_raw_buffer_load_b128(xr, slot_of(h) * a.xslot * 8 + 16 * i, 0, SC1);
                    }
#pragma unroll
                    for (int kk = 0; kk < KC; ++kk) {
                        const int k = k0 + kk;
                        if (k >= NG4) break;
                        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int h = 0; h < NS; ++h) {
                            const f32x4 v = h == hs ? own4[k]
                                                    : f32x4{__uint_as_float(pl[kk][h][0]), __uint_as_float(pl[kk][h][1]),
                                                            __uint_as_float(pl[kk][h][2]), __uint_as_float(pl[kk][h][3])};
                            acc = h == 0 ? v : acc + v;
                        }
                        ag[k] = acc;
                        if (t + k * NT < NV4)
#pragma unroll
                            for (int q = 0; q < 4; ++q) sq2 = fmaf(acc[q], acc[q], sq2);
                    }
                }
                }
                if (t < TAIL) {
                    float acc = 0.f;
#pragma unroll
                    for (int h = 0; h < NS; ++h) {
                        const float v = h == hs ? G0[4 * NV4 + t]
                                                : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                                      xr, slot_of(h) * a.xslot * 8 + 16 * NV4 + 4 * t, 0, SC1));
                        acc = h == 0 ? v : acc + v;
                    }
                    agt = acc;
                    sq2 = fmaf(agt, agt, sq2);
                }
#pragma unroll
                for (int k = 0; k < NG4; ++k) {
                    const int i = min(t + k * NT, NV4 - 1);
                    const float4 m4 = *reinterpret_cast<const float4*>(&S.MV[4 * i]);
                    const float4 v4 = *reinterpret_cast<const float4*>(&S.MV[IMG + 4 * i]);
                    const float4 p4 = *reinterpret_cast<const float4*>(&Pf[4 * i]);
                    am[k] = f32x4{m4.x, m4.y, m4.z, m4.w};
                    av[k] = f32x4{v4.x, v4.y, v4.z, v4.w};
                    ap[k] = f32x4{p4.x, p4.y, p4.z, p4.w};
                }
            }
            PGM_STAMP(11);
            // ---- clip_grad_norm_: this tower's squared norm (waves summed in order), exchanged with the other
            // tower's workgroup of the same row part as one tagged 8-byte granule
            float sq = wave_sum64(sq2);
            if (l == 0) S.red[w] = sq;
            lds_sync_m();
            float total = 0.f;
#pragma unroll
            for (int i = 0; i < W; ++i) total += S.red[i];
            PGM_STAMP(8);
            // this step's Adam scalars (fp64 bias corrections) while the norm granule travels
            const double b1n = b1p * (double)b1c, b2n = b2p * (double)b2c;
            float step_size = (float)(lr / (1.0 - b1n));
            float inv_bc2s = 1.f / (float)sqrt(1.0 - b2n);
            asm volatile("" : "+v"(step_size), "+v"(inv_bc2s));  // formed HERE (the compiler would sink them)
            if constexpr (EARLY_STAGE) {  // next pass (gp after the pass loop): rows by waves 1..W-1
                if (w != 0) {
                    if (gp < npass) issue_rows_n(gp & 1, gp & 1, w - 1, ic<W - 1>{});
                    if (gp + 1 < npass) issue_idx(gp + 1, (gp + 1) & 1, w - 1, W - 1);
                }
            }
            if (t == 0) {
                const unsigned tag = (unsigned)(nstep + 1);
                unsigned long long* gr = a.ws + ppo_norm_granule(a.P, p, 0, hs, nstep & 1);
                __hip_atomic_store(gr + m, ((unsigned long long)tag << 32) | __float_as_uint(total), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                dbg_delay(a.dbg, nstep, 2);
                unsigned long long x = 0;
                const bool failed = __hip_atomic_load(a.ws + 2 * a.P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (unsigned spins = 0; !failed; ++spins) {
                    x = __hip_atomic_load(gr + (1 - m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((unsigned)(x >> 32) == tag) break;
                    if (spins > (1u << 26)) {
                        __hip_atomic_store(a.ws + 2 * a.P, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        x = 0;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                const float other = __uint_as_float((unsigned)x);
                S.red[5] = m == 0 ? total + other : other + total;  // critic + actor in every workgroup
            }
            lds_sync_m();
            total = S.red[5];
            PGM_STAMP(9);
            const float coef = clip_coef(a.hp.max_grad_norm, total);
            if (t == 0) {
                if (m == 0) st_v += lsum_all * vstat;
                else st_a += lsum_all * astat;
                st_e += ent;
            }
            // ---- Adam from registers (padding: g = m = v = 0 keeps p = 0)
            ++nstep;
            b1p = b1n;
            b2p = b2n;
            auto adam1 = [&](float gg, float& mm, float& vv, float& pp) {
                const float gc = gg * coef;
                mm = mm + (1.f - b1c) * (gc - mm);
                vv = vv * b2c + (1.f - b2c) * (gc * gc);
                const float den = __builtin_amdgcn_sqrtf(vv) * inv_bc2s + eps;
                pp -= step_size * mm * __builtin_amdgcn_rcpf(den);
            };
#pragma unroll
            for (int k = 0; k < NG4; ++k) {
                const int i = t + k * NT;
                if (i >= NV4) break;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    float mm = am[k][q], vv = av[k][q], pp = ap[k][q];
                    adam1(ag[k][q], mm, vv, pp);
                    am[k][q] = mm;
                    av[k][q] = vv;
                    ap[k][q] = pp;
                }
                *reinterpret_cast<float4*>(&S.MV[4 * i]) = make_float4(am[k][0], am[k][1], am[k][2], am[k][3]);
                *reinterpret_cast<float4*>(&S.MV[IMG + 4 * i]) = make_float4(av[k][0], av[k][1], av[k][2], av[k][3]);
                *reinterpret_cast<float4*>(&Pf[4 * i]) = make_float4(ap[k][0], ap[k][1], ap[k][2], ap[k][3]);
            }
            if (t < TAIL) {
                const int i = 4 * NV4 + t;
                float mm = S.MV[i], vv = S.MV[IMG + i], pp = Pf[i];
                adam1(agt, mm, vv, pp);
                S.MV[i] = mm;
                S.MV[IMG + i] = vv;
                Pf[i] = pp;
            }
            if (m == 1) {  // exp(-2 logstd) of the new actor logstd by the compile-time owners of its elements
#pragma unroll
                for (int j = 0; j < A; ++j) {
                    const int e = oLs + j;
                    if (e < 4 * NV4) {
                        const int i4 = e >> 2, k = i4 / NT;
                        if (t == i4 - k * NT) S.aiv[j] = expf(-2.f * ap[k][e & 3]);
                    } else if (t == e - 4 * NV4) {
                        S.aiv[j] = expf(-2.f * Pf[e]);
                    }
                }
            }
            if constexpr (EARLY_STAGE) dma_sync_m();  // + the next pass's rows landed
            else lds_sync_m();  // parameters updated before the next minibatch; GA region reused as scr
            PGM_STAMP(3);
        }  // minibatches
    }      // epochs
    PGM_STAMP_FLUSH;
    if (hs != 0) return;  // the NS parts hold identical copies
    for (int i = t; i < IMG; i += NT) {
        const int f = img_to_flat<O, A, K>(i, m, L);
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

template <int O, int A, int K, int NS, int W, bool ONE>
static int launch_t16_k(const pgm_dims* d, const MArgs& a, hipStream_t stream) {
    using Sm = T16Smem<O, A, K, W>;
    const size_t smem = sizeof(Sm);
    if (smem > 160 * 1024) {
        set_error("pgm_ppo_update: LDS image %zu bytes exceeds 160 KiB", smem);
        return PGM_E_UNSUPPORTED;
    }
    static_assert(sizeof(Sm) > 80 * 1024, "residency argument (one workgroup per CU) needs > 80 KiB LDS");
    auto kern = ppo_update_t16_kernel<O, A, K, NS, W, ONE>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update");
    const int grid = t16_grid(d->P, NS);
    if (int rc = check_coresident((const void*)kern, 64 * W, smem, grid, "pgm_ppo_update")) return rc;
    const size_t zb = ppo_flag_bytes(d->P) + ppo_xbuf_bytes(d, NS);
    if (!ws_take_zeroed(a.ws, zb)) {
        e = hipMemsetAsync(a.ws, 0, zb, stream);
        if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update (workspace reset)");
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * W), smem, stream, a);
    return launch_status("pgm_ppo_update");
}

template <int O, int A, int K, int NS, int W>
int launch_t16(const pgm_dims* d, const MArgs& a, hipStream_t stream) {
    const int mb = d->T * d->N / a.hp.num_mini_batch;
    if (mb == NS * W * T16) return launch_t16_k<O, A, K, NS, W, true>(d, a, stream);
    return launch_t16_k<O, A, K, NS, W, false>(d, a, stream);
}

static int device_cus() { return device_cu_count(); }

template <int O, int A, int K, int MODE, bool ONE>
int launch_mode_k(const pgm_dims* d, const MArgs& a, hipStream_t stream) {
    constexpr bool SPLIT = MODE >= 1;
    const size_t smem = sizeof(MSmem<O, A, K, SPLIT>);
    if (smem > 160 * 1024) {
        set_error("pgm_ppo_update: LDS image %zu bytes exceeds 160 KiB", smem);
        return PGM_E_UNSUPPORTED;
    }
    auto kern = ppo_update_mfma_kernel<O, A, K, MODE, ONE>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update");
    // norm granules, timeout flag (and MODE 2: the exchange slots) start at tag 0; MODE 0 resets the flag
    // word too, so word 2P always reports THIS call
    const int grid = MODE == 2 ? mode2_grid(d->P) : SPLIT ? 2 * d->P : d->P;
    if constexpr (SPLIT) {  // workgroups exchange through spin-waits: all of them must be resident together
        if (int rc = check_coresident((const void*)kern, MT, smem, grid, "pgm_ppo_update")) return rc;
    }
    const size_t zb = ppo_flag_bytes(d->P) + (MODE == 2 ? ppo_xbuf_bytes(d) : 0);
    if (!ws_take_zeroed(a.ws, zb)) {
        e = hipMemsetAsync(a.ws, 0, zb, stream);
        if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update (workspace reset)");
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(MT), smem, stream, a);
    return launch_status("pgm_ppo_update");
}

template <int O, int A, int K, int MODE>
int launch_mode(const pgm_dims* d, const MArgs& a, hipStream_t stream) {
    using Sm = MSmem<O, A, K, true>;
    if constexpr (MODE == 2) {  // 2 workgroups x 4 waves x one 32-row tile = the minibatch, in one pass
        if (d->T * d->N / a.hp.num_mini_batch == 2 * 4 * TS && Sm::SBk >= 4 * TS)
            return launch_mode_k<O, A, K, MODE, true>(d, a, stream);
    }
    return launch_mode_k<O, A, K, MODE, false>(d, a, stream);
}

int fs_choose_ns(const pgm_dims* d, int mb, bool dual_ok, int* dual);
int ppo_update_fs(const pgm_dims* d, const MArgs& a, int ns, bool dual, hipStream_t stream);

// Which obs_dim <= 32 update runs (one rule for the launcher and pgm_ppo_update_variant):
//   * feature-split with the reduce-scattered Adam (pgm_ppo_fs.hip) while it gets >= FS_AUTO_NS parts per tower
//     (small per-GPU populations: the latency form), or always with opts.update_kernel = PGM_UPDATE_FS;
//   * else the row-split kernels, opts.update_split capping them: four workgroups per tower (default) = 16-row tiles
//     (8 CUs per task, while t16_grid(P, 4) <= CUs), two = 32-row tiles (MODE 2, while mode2_grid(P) <= CUs), one per
//     tower (2P <= CUs), one per task; each falls back to the next one down.  (16-row tiles on 2 workgroups of 8
//     waves measured slower than MODE 2 everywhere: 7.37 vs 6.55 ms.)
// opts.update_kernel = PGM_UPDATE_ROWSPLIT (the tests' row-split A/B) or any update_split keeps the row-split kernels.
constexpr int FS_AUTO_NS = 4;
struct UpdateChoice {
    int kind;  // 0 = MODE (mode), 1 = t16 (ns, w), 2 = feature-split (ns, dual: two workgroups per CU)
    int ns, w, mode, dual;
};
static UpdateChoice choose_update(const pgm_dims* d, int mb, const pgm_launch_opts& o) {
    const bool force_fs = o.update_kernel == PGM_UPDATE_FS;
    const bool auto_k = o.update_split == PGM_SPLIT_AUTO && o.update_kernel == PGM_UPDATE_AUTO;
    int fs_dual = 0;
    const int fs_ns = fs_choose_ns(d, mb, o.fs_one_per_cu == 0, &fs_dual);
    if (fs_ns > 0 && (force_fs || (auto_k && fs_ns >= FS_AUTO_NS))) return {2, fs_ns, 4, 0, fs_dual};
    const int cap = split_cap(o);
    const int cus = device_cu_count();
    if (cap >= 4 && t16_grid(d->P, 4) <= cus) return {1, 4, 4, 0, 0};
    if (cap >= 2 && mode2_grid(d->P) <= cus) return {0, 2, 4, 2, 0};
    if (cap >= 1 && 2 * d->P <= cus) return {0, 1, 4, 1, 0};
    return {0, 1, 4, 0, 0};
}

int describe_update_mfma(const pgm_dims* d, const pgm_ppo_hparams* hp, const pgm_launch_opts& o, char* buf, int n) {
    const int mb = d->T * d->N / hp->num_mini_batch;
    const UpdateChoice c = choose_update(d, mb, o);
    if (c.kind == 2)
        return snprintf(buf, n, "ppo_update_fs_kernel (NS=%d, R=%d%s)", c.ns, (mb / 16 + c.ns - 1) / c.ns,
                        c.dual ? ", 2 per CU" : "");
    if (c.kind == 1) return snprintf(buf, n, "ppo_update_t16_kernel (NS=%d, W=%d)", c.ns, c.w);
    return snprintf(buf, n, "ppo_update_mfma_kernel (MODE %d)", c.mode);
}

template <int O, int A, int K>
int launch_ppo_update_mfma(const pgm_dims* d, const MArgs& a, const pgm_rollout_buf* rb, const pgm_launch_opts& o,
                           hipStream_t stream) {
    // packed sample table, then the update
    constexpr int RS = row_stride<O, A, K>();
    static_assert(img_floats<O, A, K>() == ppo_img_floats(O, A, K), "host exchange-slot size out of sync");
    PackArgs pa{d->P, d->N, d->T, rb->obs, rb->actions, rb->logp, rb->adv, rb->values, rb->returns,
                const_cast<float*>(a.rows)};
    const long long n4 = (long long)d->P * d->T * d->N * (RS / 4);
    auto pack = pack_rows_kernel<O, A, K>;
    hipLaunchKernelGGL(pack, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream, pa);
    if (int rc = launch_status("pgm_ppo_update (pack rows)")) return rc;
    // every workgroup of a split launch must be resident at once: one per CU (LDS > 80 KiB, 512 registers
    // per lane), so the grid must fit the CU count (choose_update)
    static_assert(sizeof(MSmem<O, A, K, true>) > 80 * 1024, "split residency argument needs > 80 KiB LDS");
    const UpdateChoice c = choose_update(d, d->T * d->N / a.hp.num_mini_batch, o);
    if (c.kind == 2) return ppo_update_fs(d, a, c.ns, c.dual != 0, stream);
    if (c.kind == 1) return launch_t16<O, A, K, 4, 4>(d, a, stream);
    if (c.mode == 2) return launch_mode<O, A, K, 2>(d, a, stream);
    if (c.mode == 1) return launch_mode<O, A, K, 1>(d, a, stream);
    return launch_mode<O, A, K, 0>(d, a, stream);
}

int ppo_update_mfma(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m, float* adam_v,
                    int32_t* adam_step, const float* lr, const int32_t* perms, const pgm_rollout_buf* rb, float* stats,
                    void* workspace, const pgm_launch_opts& opts, hipStream_t stream) {
    if (!workspace) {
        set_error("pgm_ppo_update: the MFMA update needs the workspace (pgm_ppo_update_workspace_bytes)");
        return PGM_E_INVALID_ARG;
    }
    char* ws = (char*)workspace;
    MArgs a{d->N, d->T, make_layout(d->O, d->A, d->K, d->H), *hp, params, adam_m, adam_v, adam_step, lr, perms,
            (const float*)(ws + ppo_flag_bytes(d->P) + ppo_xbuf_bytes(d)), stats, (unsigned long long*)ws,
            (unsigned long long*)(ws + ppo_flag_bytes(d->P)), ppo_xslot(d->O, d->A, d->K), (int)ppo_xbuf_bytes(d),
            d->P, dbg_delay_hook(),
            ws + ppo_flag_bytes(d->P) + ppo_xbuf_bytes(d) + (size_t)d->P * d->T * d->N * ppo_row_stride(d->O, d->A, d->K) * sizeof(float)};
    return dispatch_dims(d->O, d->A, d->K, "pgm_ppo_update", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (O > 32) {
            set_error("pgm_ppo_update: obs_dim %d > 32 not supported by the MFMA update kernel", O);
            return PGM_E_UNSUPPORTED;
        } else {
            return launch_ppo_update_mfma<O, A, K>(d, a, rb, opts, stream);
        }
    });
}

}  // namespace pgm
