// Feature-split PPO update with a reduce-scattered Adam (obs_dim <= 32): the latency form of the update for small
// per-GPU populations (strong scaling: pop 40 over 8 GPUs = 5 tasks per GPU) and the alternative at every P.
//
// Work split.  Each tower of a task runs on NS workgroups (2 NS per task, all on one XCD under round-robin dispatch);
// workgroup hs takes its share of every minibatch's 16-row tiles: R = ceil(mb / (16 NS)) (NS = 6: 3 / 3 / 3 / 3 / 2 / 2
// on a 256-row minibatch, a missing tile a zero-gradient dummy).  Inside
// a workgroup the FOUR WAVES SPLIT THE 64 HIDDEN FEATURES (wave w: features 16w .. 16w + 15) instead of the rows, on
// the v_mfma_f32_16x16x4_f32 layout
//     C/D: lane l, register r <-> (row 4(l >> 4) + r, column l & 15); A: lane l holds A[l & 15][l >> 4];
//     B: lane l holds B[l >> 4][l & 15]
// so a wave's gradient partials are DISJOINT blocks of the tower's gradient (no intra-workgroup image reduction):
// dW1^T / dW2^T rows x the wave's 16 output columns, the head weights of its 16 units, its b1 / b2 entries.  The
// feature-contracting products (Z2 = H1 W2^T, the heads, dH1 = dZ2 W2) read the other waves' activations from
// shared LDS tiles, three workgroup barriers per minibatch step.
//
// Exchange (per Adam step, tags = step + 1, slots double-buffered by step parity):
//   1. every wave publishes its gradient blocks (1 KiB "fragments" = the f32x4 C registers of 64 lanes; obs_dim <= 20:
//      6 per wave, the head block's free columns carrying b1 / b2 / head bias / logstd and dW1 inputs 16..19) with
//      16-B sc1 stores, the workgroup drains and one lane stores the tagged image flag {step, loss sum};
//   2. REDUCE-SCATTER: block b belongs to part b mod NS, which sums it over the NS parts in part order (sc1 loads) --
//      a sum only its owner forms, so it is deterministic without being replicated;
//   3. the owners' squared norms meet through one tagged 8-B granule per (tower, part): every workgroup sums the
//      2 NS granules in one fixed order (clip_grad_norm_ over both towers);
//   4. each owner runs Adam on ITS blocks (parameters and moments of the owned blocks live in registers for the whole
//      launch), publishes the new parameter blocks (sc1) + a tagged flag, and every workgroup gathers the other
//      parts' blocks into its LDS parameter image.
// Three cross-CU hops per Adam step, each moving ~1/NS of the image per reader instead of every partner's whole
// image (pgm_ppo_mfma.hip's t16 / MODE 2), and Adam on 1/NS of the parameters per workgroup.  The parameter gather of
// step s is issued at its end and written into the image during step s + 1, each block just before its first reader
// (every wave gathers its own feature block).  Measured and dropped: a two-hop form (owners publish the reduced
// gradient, every workgroup gathers all of it and runs Adam on the whole tower) -- one hop fewer, but Adam on ~32
// elements per thread plus the wider gather cost more than the hop (P = 5: 28.1 K vs 24.7 K cycles per Adam step,
// profiles/r04c_fs2_stamps_p5.txt, r04c_fs3_stamps_p5.txt; again with compact fragments and feature-block Adam:
// HalfCheetah P = 20 +5 %, Walker P = 40 equal, profiles/r05m_fs_twohop_ab.txt).
//
// Padding kept off the critical path: obs inputs 16..19 (one valid row of a 16-input MFMA block at obs_dim 17) are
// VALU FMAs in layer 1 and dW1, and the actor's per-sample loss runs two tiles per pass (R = 2 / 3).
//
// Reference semantics (a2c_ppo_acktr/algo/ppo.py:58-115, storage.py:118-154, model.py:75-82, distributions.py:29-40)
// as in pgm_ppo_mfma.hip, including torch.min/max/clamp tie gradients; entropy_coef enters once per tower.
#include <stdlib.h>

#include "pgm_dispatch.hpp"
#include "pgm_ppo_shared.hpp"

PGM_STAMP_UNIT(fs)

namespace pgm {

// ---------------------------------------------------------------- geometry shared by host and device
// gradient / parameter fragments of one tower: per wave w (feature block w) K1M dW1 blocks, 4 dW2 blocks, 1 head
// block, 1 vector block (b1, b2 and, wave 0, head bias / logstd). Compact form (obs_dim <= 20, <= 8 head columns):
// the head block's free lanes (columns 8..15) carry the vector block and dW1 input rows 16..19, so a wave exchanges
// 6 blocks instead of 7 / 8 (a quarter fewer bytes per hand-off at obs_dim 17)
constexpr bool fs_compact(int O) { return O <= 20; }
constexpr int fs_k1m(int O) { return fs_compact(O) ? 1 : (O + 15) / 16; }
constexpr int fs_bpw(int O) { return fs_k1m(O) + (fs_compact(O) ? 5 : 6); }
constexpr int fs_nb(int O) { return 4 * fs_bpw(O); }
constexpr int fs_nown(int O, int NS) { return (fs_nb(O) + NS - 1) / NS; }  // blocks per owner (max)
// parameter-slot positions a part writes: every wave publishes the same number of blocks (ceil(NOWN / 4)), past NOWN
// unused values, so a slot holds 4 ceil(NOWN / 4) block positions
constexpr int fs_pslots(int O, int NS) { return 4 * ((fs_nown(O, NS) + 3) / 4); }
// payload: image slots [P][2][NS][2 parities][NB KiB], then parameter slots [P][2][NS][2][fs_pslots KiB]
inline size_t fs_payload_bytes(int P, int O, int NS) {
    return (size_t)P * 2 * NS * 2 * (size_t)(fs_nb(O) + fs_pslots(O, NS)) * 1024;
}
// parts per tower the update is built for, largest first (6: 96 blocks per group of 8 tasks, so that five groups --
// 33..40 tasks -- fit a 256-CU MI355X twice over with two workgroups per CU)
constexpr int FS_NS_LIST[] = {16, 8, 6, 4, 2};
// (parts, 16-row tiles per part) pairs the library is built for: minibatches of 64 / 128 / 256 / 512 rows on power-of-two
// parts and tiles, and 6 parts of 3 tiles
constexpr bool fs_built(int ns, int R) {
    const int mb = 16 * ns * R;
    return (ns == 6 && R == 3) ||
           (ns != 6 && (R == 1 || R == 2 || R == 4 || R == 8) && (mb == 64 || mb == 128 || mb == 256 || mb == 512));
}
// 16-row tiles of the part with the most (parts 0 .. (mb / 16) % NS - 1 take one more than the others)
inline int fs_tiles(int mb, int ns) { return (mb / 16 + ns - 1) / ns; }
inline int fs_grid(int P, int NS) { return 16 * NS * ((P + 7) / 8); }
// tagged granules of the exchange, in the zeroed flag region after the norm granules of the other updates:
// kind 0 = image flag, 1 = squared-norm granule, 2 = parameter flag
__host__ __device__ inline int fs_gran(int P, int NS, int kind, int p, int m, int hs, int par) {
    return 16 * P + 8 + ((((kind * P + p) * 2 + m) * NS + hs) * 2 + par);
}

// Sized for the largest NS (16), not the NS a launch with P tasks picks: a caller may allocate the workspace for a capacity P and launch
// with fewer active tasks (TaskBatch.set_active), whose cap can be LARGER (8 parts at P = 32, 4 at P = 33), and
// NS (NB + pslots(NS)) grows with NS, so this bounds the payload of every launch with P' <= P tasks.
size_t fs_workspace_extra(const pgm_dims* d) {
    if (d->O > 32) return 0;
    return fs_payload_bytes(d->P, d->O, 16);
}

// compact head block, column c of feature block wb: entry v (= 4 g + r) at image index base + v for v < lim -- head
// column c (c < 8), b1, b2, head bias, logstd (8..11), dW1 input 16 + (c - 12) (12..15)
template <int O, int A, int K>
__host__ __device__ __forceinline__ void cpt_column(int c, int wb, int m, int& base, int& lim) {
    constexpr int Q = qmax<A, K>();
    constexpr int oW2 = O * H, oWh = oW2 + H * SCR, oB1 = oWh + Q * H, oB2 = oB1 + H, oBh = oB2 + H, oLs = oBh + Q;
    const int NQ = m == 0 ? K : A, in = 16 + c - 12;
    base = c < 8 ? oWh + c * H + 16 * wb
         : c == 8 ? oB1 + 16 * wb
         : c == 9 ? oB2 + 16 * wb
         : c == 10 ? oBh
         : c == 11 ? oLs
                   : in * H + 16 * wb;
    lim = c < 8 ? (c < NQ ? 16 : 0)
        : c < 10 ? 16
        : c == 10 ? (wb == 0 ? NQ : 0)
        : c == 11 ? (wb == 0 && m == 1 ? A : 0)
                  : (in < O ? 16 : 0);
}

// fragment slot (block b, lane l, register r) -> tower image index (TowerImg), -1 for padding
template <int O, int A, int K>
__host__ __device__ __forceinline__ int frag_img(int b, int l, int r, int m) {
    constexpr int Q = qmax<A, K>(), K1M = fs_k1m(O), BPW = fs_bpw(O);
    constexpr int oW2 = O * H, oWh = oW2 + H * SCR, oB1 = oWh + Q * H, oB2 = oB1 + H, oBh = oB2 + H, oLs = oBh + Q;
    static_assert(!fs_compact(O) || Q <= 8, "compact fragments: head columns 0..7 only");
    const int wb = b / BPW, k = b - wb * BPW, g = l >> 4, c = l & 15;
    const int NQ = m == 0 ? K : A;
    if (k < K1M) {
        const int in = 16 * k + 4 * g + r;
        return in < O ? in * H + 16 * wb + c : -1;
    }
    if (k < K1M + 4) return oW2 + (16 * (k - K1M) + 4 * g + r) * SCR + 16 * wb + c;
    if (k == K1M + 4) {
        if (!fs_compact(O)) return c < NQ ? oWh + c * H + 16 * wb + 4 * g + r : -1;
        int base, lim;
        cpt_column<O, A, K>(c, wb, m, base, lim);
        return 4 * g + r < lim ? base + 4 * g + r : -1;
    }
    if (g != 0) return -1;
    if (r == 0) return oB1 + 16 * wb + c;
    if (r == 1) return oB2 + 16 * wb + c;
    if (r == 2) return wb == 0 && c < NQ ? oBh + c : -1;
    return wb == 0 && m == 1 && c < A ? oLs + c : -1;
}

constexpr int SF = 72;  // fs activation-tile row stride (floats)

template <int O, int A, int K, int R>
struct FsSmem {
    static constexpr int Q = qmax<A, K>();
    static constexpr int RS = row_stride<O, A, K>();
    static constexpr int RSL = RS + 4;
    static constexpr int SB = 16 * R;                          // rows of this part per minibatch
    static constexpr int NDT = (SB * RSL + 255) / 256;         // 1-KiB LDS-DMA pieces per staged pass
    static constexpr int SBI = 64 * ((SB + 63) / 64);          // index slots (one 64-lane DMA per wave)
    // dZ2 tile aliases the H2 tile (LDS budget: R = 8 for 160 KiB; R = 2 to stay under 80 KiB, two workgroups per CU)
    static constexpr bool ZA = R >= 8 || R == 2 || R == 3;
    static constexpr int NHP = R >= 4 ? 1 : 4;                 // partial head outputs (R < 4: one tile per wave)
    TowerImg<O, A, K> Pm;                                      // parameters (working copy of every part)
    alignas(16) float RB[2][NDT * 256];                        // packed rows of this / the next minibatch
    int32_t IB[2][SBI];                                        // sample indices of the next two minibatches
    // activation tiles [sample][feature], row stride SF = 72 floats (= 8 mod 64): the feature-contracting products read
    // 4 consecutive features per lane with ds_read_b128 (16-B aligned, conflict-free for the 16-row tiles)
    static constexpr bool HT = R <= 4 && R != 3;               // H1 also [feature][sample] (the dW2 A operand;
                                                               // R = 3: not, to fit two workgroups per CU)
    static constexpr int STT = HT ? 72 : 4;                    // its row stride (16 R <= 64 samples, = 8 mod 64)
    alignas(16) float H1s[SB][SF];                             // H1 of all tiles, all 64 features
    alignas(16) float H2s[SB][SF];                             // H2 (R >= 8: then dZ2)
    alignas(16) float Zs[ZA ? 1 : SB][SF];                     // dZ2
    alignas(16) float H1T[HT ? H : 1][STT];                    // H1 transposed (R <= 4)
    float dOs[SB][DQS];                                        // dL/d(head output), transposed for dH2
    alignas(16) float HP[NHP][SB][DQS];                        // R < 4: the waves' partial head outputs (after B3:
                                                               // the waves' compact head-block staging, 128 floats each)
    float aiv[A];                                              // actor 1 / std^2
    float red[192];  // [0, 64) head-bias partials / poll results, [64, 128) logstd partials / norms, 128+ loss sums
};
// one workgroup per CU: padded past 80 KiB (the placement the launcher's grid assumes); dual (two per CU, 16 NS ceil(P/8)
// > CUs): the struct itself, which must then fit 80 KiB
template <int O, int A, int K, int R>
constexpr size_t fs_smem_bytes(bool dual) {
    return dual || sizeof(FsSmem<O, A, K, R>) > 81 * 1024 ? sizeof(FsSmem<O, A, K, R>) : 81 * 1024;
}

// (Measured and dropped: the parameter hop without a flag -- owners storing every new value as an 8-B {value, tag}
// granule, readers re-loading a block until all its tags are this step's: P = 5 3.45 vs 2.93 ms, P = 20 5.06 vs 4.38 ms.)
template <int O, int A, int K, int NS, int R>
// R = 3: held to 256 registers, so that two workgroups share a CU (fs_choose_ns dual; R = 2 fits by itself)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R == 3 ? 2 : 1))) void ppo_update_fs_kernel(MArgs a) {
    static_assert(O <= 32 && (R == 1 || R == 2 || R == 3 || R == 4 || R == 8), "fs tiles");
    using Sm = FsSmem<O, A, K, R>;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<Sm*>(smem_raw);
    constexpr int Q = qmax<A, K>();
    static_assert(Q <= DQ, "head outputs beyond the dO tile");
    constexpr int KS1 = (O + 3) / 4, K1B = (O + 15) / 16;
    constexpr int IMG = img_floats<O, A, K>(), RS = Sm::RS, RSL = Sm::RSL, SB = Sm::SB, NDT = Sm::NDT;
    constexpr int CR = RS / 4;
    constexpr int BPW = fs_bpw(O), NB = fs_nb(O), NOWN = fs_nown(O, NS), K1M = fs_k1m(O);
    constexpr bool CPT = fs_compact(O);
    constexpr int KV = K1M + (CPT ? 4 : 5);  // the block b1 lives in (compact: the head block)
    static_assert(!CPT || Sm::NHP * Sm::SB * DQS >= 512, "compact head-block staging: 128 floats per wave");
    constexpr int OWV = (NOWN + 3) / 4;  // owned blocks per wave (block j of the part: wave j mod 4)
    constexpr int ISB = NB * 1024, PSB = fs_pslots(O, NS) * 1024;
    constexpr bool HSPLIT = R >= 4;      // heads: row tiles split over the waves (else units + samples split)
    constexpr int NHT = HSPLIT ? R / 4 : R;
    constexpr int NC = R == 1 ? 2 : 1;   // accumulator chains per tile of the 16-deep contractions
    constexpr int oW2 = O * H, oWh = oW2 + H * SCR, oB1 = oWh + Q * H, oB2 = oB1 + H, oBh = oB2 + H, oLs = oBh + Q;
    const int t = threadIdx.x, l = t & 63, g = l >> 4, c = l & 15;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    // block map: groups of 16 NS blocks for 8 tasks; block r holds part (r >> 4) % NS of tower (r >> 3) & 1 of task
    // 8 G + (r & 7), so every workgroup of a task shares blocks b, b + 8, ... (one XCD: speed only)
    const int bx = (int)blockIdx.x;
    const int j16 = (bx >> 3) % (2 * NS);
    const int p = 8 * (bx / (16 * NS)) + (bx & 7);
    const int hs = j16 >> 1, m = j16 & 1;
    if (p >= a.P) return;
    const int NQ = m == 0 ? K : A;
    const int N = a.N, T = a.T, B = T * N;
    const int E = a.hp.ppo_epoch, M = a.hp.num_mini_batch;
    const int mb = B / M, nb = B / mb;
    // this part's rows of every minibatch: the mb / 16 row tiles dealt over the NS parts, the first (mb / 16) % NS parts
    // one more (NS = 6 on a 256-row minibatch: 3 / 3 / 3 / 3 / 2 / 2); tiles past the part's own count are dummies
    // (their rows repeat its last one) whose loss gradients and loss terms are zeroed, so they add exact zeros
    const int ntl = mb >> 4, tb0 = ntl / NS, tex = ntl - tb0 * NS;
    const int rown = 16 * (tb0 + (hs < tex ? 1 : 0));
    const int r0 = 16 * (hs * tb0 + min(hs, tex));
    const int npass = E * nb;
    const float clip = a.hp.clip_param;
    const Layout& L = a.L;
    float* __restrict__ P = a.params + (size_t)p * L.total;
    float* __restrict__ Mo = a.m + (size_t)p * L.total;
    float* __restrict__ Vo = a.v + (size_t)p * L.total;
    const float* rows = a.rows + (size_t)p * B * RS;
    const int fsbytes = (int)((size_t)a.P * 2 * NS * 2 * (ISB + PSB));
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(a.fsp, 0, fsbytes, 0x00020000);
    constexpr int SC1 = 16;
    auto islot = [&](int h, int par) { return ((((p * 2 + m) * NS + h) * 2 + par)) * ISB; };
    auto pslot = [&](int h, int par) { return a.P * 2 * NS * 2 * ISB + ((((p * 2 + m) * NS + h) * 2 + par)) * PSB; };
    auto gran = [&](int kind, int mm, int h, int par) { return a.ws + fs_gran(a.P, NS, kind, p, mm, h, par); };
    unsigned long long* const fail_word = a.ws + 2 * a.P;
    // the timed-out wait, for the host's error message: bit 0, bit 1 + site (0 image flags, 1 norm granules, 2 parameter
    // flags), the awaited tag in bits 8..23, the workgroup (task, tower, part) from bit 24
    auto fail_code = [&](int site, unsigned tg) -> unsigned long long {
        return 1ull | (2ull << site) | ((unsigned long long)(tg & 0xffff) << 8) |
               ((unsigned long long)((p * 2 + m) * NS + hs) << 24);
    };

    // ---- staging (as the 16-row kernel): the minibatch's permutation indices by 4-B LDS-DMA one minibatch
    // earlier than its rows; rows by 16-B LDS-DMA (pieces past SB * RSL re-read the last row into padding)
    auto issue_idx = [&](int gi, int buf, int wi, int nwv) {
        const int e = gi / nb, bb = gi - e * nb;
        const int32_t* src = a.perms + (size_t)e * B + bb * mb + r0;
        for (int q0 = wi * 64; q0 < SB; q0 += 64 * nwv)
            __builtin_amdgcn_global_load_lds((const void*)(src + min(q0 + l, rown - 1)), (lds_void_t*)&S.IB[buf][q0], 4,
                                             0, 0);
    };
    auto issue_rows = [&](int buf, int ibuf, int wi, int nwv) {
        float* base = &S.RB[buf][0];
        for (int d = wi; d < NDT; d += nwv) {
            const int pos = d * 256 + 4 * l, row = min(pos / RSL, SB - 1), chunk = (pos - (pos / RSL) * RSL) >> 2;
            const int idx = S.IB[ibuf][row];
            const float* src = rows + (size_t)idx * RS + (chunk < CR ? chunk : 0) * 4;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(base + d * 256), 16, 0, 0);
        }
    };

    // ---- parameter image, owned blocks' parameters and moments (registers for the whole launch)
    float* Pf = &S.Pm.W1t[0][0];
    for (int i = t; i < IMG; i += 256) {
        const int f = img_to_flat<O, A, K>(i, m, L);
        Pf[i] = f >= 0 ? P[f] : 0.f;
    }
    if (t < A) S.aiv[t] = expf(-2.f * P[L.off[PGM_P_LOGSTD] + t]);
    // parameters + moments of this part's own blocks b = hs + NS j (block j of the part: wave j mod 4)
    // (their image indices, fixed for the launch, stay in registers: the Adam writes and the write-back reuse them)
    f32x4 op[OWV], om[OWV], ov[OWV];
    int oix[OWV][4];
#pragma unroll
    for (int i = 0; i < OWV; ++i) {
        const int b = hs + NS * (w + 4 * i);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int ii = b < NB ? frag_img<O, A, K>(b, l, r, m) : -1;
            asm volatile("" : "+v"(ii));
            oix[i][r] = ii;
            const int f = ii >= 0 ? img_to_flat<O, A, K>(ii, m, L) : -1;
            op[i][r] = f >= 0 ? P[f] : 0.f;
            om[i][r] = f >= 0 ? Mo[f] : 0.f;
            ov[i][r] = f >= 0 ? Vo[f] : 0.f;
        }
    }
    issue_idx(0, 0, w, 4);
    if (npass > 1) issue_idx(1, 1, w, 4);
    dma_sync_m();
    issue_rows(0, 0, w, 4);
    dma_sync_m();

    const int step0 = a.step[p];
    const double lr = a.lr[p];
    const float b1c = a.hp.beta1, b2c = a.hp.beta2, eps = a.hp.adam_eps;
    const float vscale = a.hp.value_loss_coef * 0.5f / (float)(mb * K);
    const float ascale = -1.f / (float)mb;
    const float vstat = 0.5f / (float)(mb * K), astat = 1.f / (float)mb;
    float st_v = 0.f, st_a = 0.f, st_e = 0.f;
    double b1p = pow((double)b1c, (double)step0), b2p = pow((double)b2c, (double)step0);
    auto& Wt = S.Pm;
    const int fb = 16 * w;  // this wave's feature block
    PGM_STAMP_DECL

    // the other parts' new parameter blocks of THIS wave's feature block (b = BPW w + k), loaded at the end of a step
    // and written into the image during the next one, each just before its first reader: W1 + vector block before
    // layer 1, W2 before layer 2, the head block before B2 (heads read every wave's); the own part's blocks are
    // written by their owners before the parameter hand-off
    u32x4 pv[BPW];
    // compact head block of this wave: entry v = 4 g + r of the lane's column at kvb + v for v < kvl (frag_img)
    int kvb = 0, kvl = 0;
    if constexpr (CPT) {
        cpt_column<O, A, K>(c, w, m, kvb, kvl);
        asm volatile("" : "+v"(kvb), "+v"(kvl));
    }
    auto put_block = [&](int k) {  // (the own part's blocks rewrite the values their owners already wrote)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float v = __uint_as_float(pv[k][r]);
            if (k < K1M) {  // dW1 rows 16 k + 4 g + r, this wave's features
                const int in = 16 * k + 4 * g + r;
                if (in < O) Pf[in * H + fb + c] = v;
            } else if (k < K1M + 4) {  // dW2 rows 16 (k - K1M) + 4 g + r
                Pf[oW2 + (16 * (k - K1M) + 4 * g + r) * SCR + fb + c] = v;
            } else if (CPT) {  // the compact head block: launch-fixed column base / limit
                if (4 * g + r < kvl) Pf[kvb + 4 * g + r] = v;
            } else {
                const int ii = frag_img<O, A, K>(BPW * w + k, l, r, m);
                if (ii >= 0) Pf[ii] = v;
            }
        }
    };
    auto pload = [&](int k, int par_) {
        const int b = BPW * w + k, h = b % NS, jj = b / NS;  // (own part's blocks too: straight-line loads)
        pv[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, pslot(h, par_) + (jj * 64 + l) * 16, 0, SC1);
    };
    for (int gp = 0; gp < npass; ++gp) {
        const int cur = gp & 1, par = gp & 1;
        const unsigned tag = (unsigned)(gp + 1);
        const float* rb = &S.RB[cur][0];
        auto rt = [&](int ti) { return rb + ti * 16 * RSL; };
        // ================================================================ tiles
        if (gp > 0) {
#pragma unroll
            for (int k = 0; k < K1M; ++k) put_block(k);
            put_block(KV);
            if (m == 1 && w == 0 && l < A) S.aiv[l] = expf(-2.f * Wt.logstd[l]);  // read in the heads, after B2
        }
        // ---- layer 1: Z1[s][fb + c] over the inputs (A = X rows, B = W1t, shared by the tiles)
        f32x4 z[R][NC], H1[R];
#pragma unroll
        for (int ti = 0; ti < R; ++ti)
#pragma unroll
            for (int q = 0; q < NC; ++q) z[ti][q] = f32x4{0.f, 0.f, 0.f, 0.f};
        // (compact: inputs 16.. -- at most 4, one mostly-padding k-step -- on the VALU, added below)
        constexpr int KS1M = fs_compact(O) && O > 16 ? 4 : KS1, NT1 = KS1M < KS1 ? O - 16 : 0;
#pragma unroll
        for (int ks = 0; ks < KS1M; ++ks) {
            const int k = 4 * ks + g;
            const bool kv = k < O;
            const float bw = kv ? Wt.W1t[kv ? k : 0][fb + c] : 0.f;
#pragma unroll
            for (int ti = 0; ti < R; ++ti) {
                const float av = kv ? rt(ti)[c * RSL + (kv ? k : 0)] : 0.f;
                z[ti][ks % NC] = mfma16(av, bw, z[ti][ks % NC]);
            }
        }
        if constexpr (NT1 > 0) {  // z[sample 4 g + r][feature c] += X[sample][16 + j] W1t[16 + j][fb + c]
            float w16[NT1 > 0 ? NT1 : 1];
#pragma unroll
            for (int j = 0; j < NT1; ++j) w16[j] = Wt.W1t[16 + j][fb + c];
#pragma unroll
            for (int ti = 0; ti < R; ++ti)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float* xr16 = rt(ti) + (4 * g + r) * RSL + 16;
#pragma unroll
                    for (int j = 0; j < NT1; ++j) z[ti][0][r] = fmaf(xr16[j], w16[j], z[ti][0][r]);
                }
        }
        {
            const float bias = Wt.b1[fb + c];
#pragma unroll
            for (int ti = 0; ti < R; ++ti) {
                f32x4 zz = z[ti][0];
                if constexpr (NC == 2) zz += z[ti][1];
                tanh_bias_pk<4>(zz, bias, H1[ti]);
#pragma unroll
                for (int r = 0; r < 4; ++r) S.H1s[16 * ti + 4 * g + r][fb + c] = H1[ti][r];
                if constexpr (Sm::HT)
                    *reinterpret_cast<float4*>(&S.H1T[fb + c][16 * ti + 4 * g]) =
                        make_float4(H1[ti][0], H1[ti][1], H1[ti][2], H1[ti][3]);
            }
        }
        PGM_STAMP(0);
        if (gp > 0) {
#pragma unroll
            for (int k = K1M; k < K1M + (CPT ? 4 : 5); ++k) put_block(k);
        }
        PGM_STAMP(11);
        lds_sync_m();  // B1: H1 of every feature block (and every wave's head block)
        PGM_STAMP(12);
        // ---- layer 2: Z2[s][fb + c] = H1[s][:] . W2t[:][fb + c]
        f32x4 H2[R];
#pragma unroll
        for (int ti = 0; ti < R; ++ti)
#pragma unroll
            for (int q = 0; q < NC; ++q) z[ti][q] = f32x4{0.f, 0.f, 0.f, 0.f};
        // k-step (j, i) contracts input k = 16 j + 4 g + i in lane group g: four consecutive inputs per lane and j, so
        // the A operands of four k-steps are one ds_read_b128 (the B rows follow the same order)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float bw[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) bw[i] = Wt.W2t[16 * j + 4 * g + i][fb + c];
#pragma unroll
            for (int ti = 0; ti < R; ++ti) {
                const float4 a4 = *reinterpret_cast<const float4*>(&S.H1s[16 * ti + c][16 * j + 4 * g]);
                const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) z[ti][(4 * j + i) % NC] = mfma16(av[i], bw[i], z[ti][(4 * j + i) % NC]);
            }
        }
        {
            const float bias = Wt.b2[fb + c];
#pragma unroll
            for (int ti = 0; ti < R; ++ti) {
                f32x4 zz = z[ti][0];
                if constexpr (NC == 2) zz += z[ti][1];
                tanh_bias_pk<4>(zz, bias, H2[ti]);
#pragma unroll
                for (int r = 0; r < 4; ++r) S.H2s[16 * ti + 4 * g + r][fb + c] = H2[ti][r];
            }
        }
        PGM_STAMP(1);
        lds_sync_m();  // B2: H2 of every feature block
        PGM_STAMP(13);
        // ---- heads on the MFMA: out[s][q] = H2[s][:] . Wh[q][:] (q = lane column < Q), then the per-(sample,
        // output) loss gradients dO (ppo.py:80-96) into the shared dO tile.  R >= 4: wave w takes row tiles w, w + 4, ...
        // whole; R < 4: wave w contracts its own 16 units for every tile (partial outputs added through LDS) and
        // finishes samples 4g + w of every tile (C register w).  Either way a quarter of the loss work per wave.
        const bool qv = c < Q;
        const float bhb = qv ? Wt.bh[c] : 0.f;
        float gbh = 0.f, gls = 0.f, lsum = 0.f;
        // dL/d(head output) of sample s, output c (this lane), from the head output `out` (bias included); tv = the
        // tile is one of this part's own (a dummy tile's gradients and loss terms are zero)
        auto loss1 = [&](const float* rr, int s, float out, bool tv) -> float {
            if (m == 0) {  // value loss over the K objectives
                const bool ok = c < K && tv;
                const float Vold = rr[s * RSL + O + A + 2 + (c < K ? c : 0)];
                const float Rt = rr[s * RSL + O + A + 2 + K + (c < K ? c : 0)];
                float gv, ls;
                if (a.hp.use_clipped_value_loss) {
                    const float dv = out - Vold;
                    const float vc = Vold + fminf(fmaxf(dv, -clip), clip);
                    const float l1 = (out - Rt) * (out - Rt), l2 = (vc - Rt) * (vc - Rt);
                    const float inr = (dv >= -clip && dv <= clip) ? 1.f : 0.f;
                    gv = wmax2(l1, l2) * 2.f * (out - Rt) + wmax2(l2, l1) * 2.f * (vc - Rt) * inr;
                    ls = fmaxf(l1, l2);
                } else {
                    gv = 2.f * (out - Rt);
                    ls = (Rt - out) * (Rt - out);
                }
                lsum += ok ? ls : 0.f;
                return ok ? vscale * gv : 0.f;
            }
            // clipped surrogate; a sample's log-prob is a 16-lane row sum over its outputs
            const bool av_ = c < A;
            const float aiv = S.aiv[av_ ? c : 0], ls_c = av_ ? Wt.logstd[av_ ? c : 0] : 0.f;
            const float diff = av_ ? rr[s * RSL + O + (av_ ? c : 0)] - out : 0.f;
            const float lpe = av_ ? -0.5f * diff * diff * aiv - ls_c - LOG_SQRT_2PI : 0.f;
            const float lp = row_sum16(lpe);
            const float ratio = expf(lp - rr[s * RSL + O + A]);
            const float ad = rr[s * RSL + O + A + 1];
            const float s1 = ratio * ad;
            const float s2 = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip) * ad;
            const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
            const float gr = ad * (wmin2(s1, s2) + wmin2(s2, s1) * inr);
            const float dlp = tv ? ascale * gr * ratio : 0.f;
            lsum += c == 0 && tv ? -fminf(s1, s2) : 0.f;
            gls += av_ ? dlp * (diff * diff * aiv - 1.f) : 0.f;
            return av_ ? dlp * diff * aiv : 0.f;
        };
        float* dt = &S.dOs[0][0];
        if constexpr (HSPLIT) {
            float4 bh4[4];  // head rows in the permuted k order (16 j + 4 g + i), one ds_read_b128 per j
#pragma unroll
            for (int j = 0; j < 4; ++j)
                bh4[j] = qv ? *reinterpret_cast<const float4*>(&Wt.Wh[qv ? c : 0][16 * j + 4 * g]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int hi = 0; hi < NHT; ++hi) {
                const int ti = w + 4 * hi;
                f32x4 ho[NC];
#pragma unroll
                for (int q = 0; q < NC; ++q) ho[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float4 a4 = *reinterpret_cast<const float4*>(&S.H2s[16 * ti + c][16 * j + 4 * g]);
                    const float av[4] = {a4.x, a4.y, a4.z, a4.w}, bv[4] = {bh4[j].x, bh4[j].y, bh4[j].z, bh4[j].w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) ho[(4 * j + i) % NC] = mfma16(av[i], bv[i], ho[(4 * j + i) % NC]);
                }
                if constexpr (NC == 2) ho[0] += ho[1];
                PGM_STAMP(14);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float d = loss1(rt(ti), 4 * g + r, ho[0][r] + bhb, 16 * ti < rown);
                    gbh += d;
                    if (c < DQ) dt[(16 * ti + 4 * g + r) * DQS + c] = d;
                }
            }
        } else {
            // this wave's units k = fb + 4 g + i (one ds_read_b128 of the head row and of the H2 row)
            const float4 b4 = qv ? *reinterpret_cast<const float4*>(&Wt.Wh[qv ? c : 0][fb + 4 * g]) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
            for (int ti = 0; ti < R; ++ti) {
                f32x4 ho = f32x4{0.f, 0.f, 0.f, 0.f};
                const float4 a4 = *reinterpret_cast<const float4*>(&S.H2s[16 * ti + c][fb + 4 * g]);
                const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) ho = mfma16(av[i], bv[i], ho);
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (c < DQ) S.HP[w][16 * ti + 4 * g + r][c] = ho[r];
            }
            PGM_STAMP(14);
            lds_sync_m();  // B2h: every wave's partial head outputs
            if (R >= 2 && m == 1) {
                // the actor (whose loss sits on the step's critical path: the critic waits for it at the norm
                // granules): two tiles per pass, lanes c < 8 tile p2 and c >= 8 tile p2 + 1 (output c & 7; A <= 8),
                // log-probs as 8-lane row sums -- a third (R = 3) / half (R = 2) fewer passes of the surrogate
                // arithmetic.  (The critic packed the same way measured no faster: r05z.)
                const int hf = c >> 3, cc = c & 7;
                const bool avp = cc < NQ;
                const float aivp = S.aiv[avp ? cc : 0], lsp = avp ? Wt.logstd[avp ? cc : 0] : 0.f;
                const float bhp = avp ? Wt.bh[avp ? cc : 0] : 0.f;
#pragma unroll
                for (int p2 = 0; p2 < R; p2 += 2) {
                    const bool tin = p2 + hf < R;  // (R odd: the last pass's upper half recomputes tile p2, zeroed)
                    const int ti = tin ? p2 + hf : p2, row = 16 * ti + 4 * g + w;
                    const bool tv = tin && 16 * ti < rown;
                    const float out = ((S.HP[0][row][cc] + S.HP[1][row][cc]) + S.HP[2][row][cc]) + S.HP[3][row][cc] + bhp;
                    const float* q = rt(ti) + (4 * g + w) * RSL + O;
                    // the clipped surrogate as loss1's, output cc
                    const float diff = avp ? q[avp ? cc : 0] - out : 0.f;
                    const float lpe = avp ? -0.5f * diff * diff * aivp - lsp - LOG_SQRT_2PI : 0.f;
                    const float lp = row_sum8(lpe);
                    const float ratio = expf(lp - q[A]);
                    const float ad = q[A + 1];
                    const float s1 = ratio * ad;
                    const float s2 = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip) * ad;
                    const float inr = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
                    const float gr = ad * (wmin2(s1, s2) + wmin2(s2, s1) * inr);
                    const float dlp = tv ? ascale * gr * ratio : 0.f;
                    lsum += cc == 0 && tv ? -fminf(s1, s2) : 0.f;
                    gls += avp ? dlp * (diff * diff * aivp - 1.f) : 0.f;
                    const float d = avp ? dlp * diff * aivp : 0.f;
                    gbh += d;
                    if (tin) dt[row * DQS + cc] = d;
                }
                // the upper half's partial sums into lanes c < 8 (row_ror:8: both halves then hold the total)
                gbh += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(gbh), 0x128, 0xf, 0xf, true));
                gls += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(gls), 0x128, 0xf, 0xf, true));
            } else {
#pragma unroll
                for (int ti = 0; ti < R; ++ti) {
                    const int s = 4 * g + w, row = 16 * ti + s;
                    const int cq = c < DQ ? c : 0;
                    const float out = c < DQ ? ((S.HP[0][row][cq] + S.HP[1][row][cq]) + S.HP[2][row][cq]) + S.HP[3][row][cq] : 0.f;
                    const float d = loss1(rt(ti), s, out + bhb, 16 * ti < rown);
                    gbh += d;
                    if (c < DQ) dt[row * DQS + c] = d;
                }
            }
        }
        PGM_STAMP(15);
        gbh = group4_sum(gbh);
        gls = group4_sum(gls);
        lsum = wave_sum64(lsum);
        if (g == 0) {  // this wave's partial head sums (its row tiles / its samples): summed in wave order later
            S.red[16 * w + c] = gbh;
            S.red[64 + 16 * w + c] = gls;
        }
        if (t == 64 * w) S.red[128 + w] = lsum;
        PGM_STAMP(2);
        lds_sync_m();  // B2b: the dO tile of every wave's rows / samples (and, R = 8, H2 reads done before dZ2)
        // ---- head-weight gradient gWh^T[u][q] += H2^T dO, dH2 = dO . Wh -> dZ2 (this wave's units)
        // (compact: dW1 inputs 16.. (at most 4, mostly padding in a 16-row MFMA block) on the VALU: gT[j] = input 16 + j)
        constexpr int K1G = CPT ? K1M : K1B, NT = CPT && O > 16 ? O - 16 : 0;
        f32x4 gWh = f32x4{0.f, 0.f, 0.f, 0.f}, gW2[4], gW1[K1G];
        float gT[NT > 0 ? NT : 1] = {};
        float gB1 = 0.f, gB2 = 0.f;
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) gW2[ib] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < K1G; ++kb) gW1[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* dtl = &S.dOs[0][0];
        float (*Zt)[SF] = Sm::ZA ? S.H2s : S.Zs;
        f32x4 dZ2[R];
#pragma unroll
        for (int ti = 0; ti < R; ++ti) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float bo = qv ? dtl[(16 * ti + 4 * g + r) * DQS + (qv ? c : 0)] : 0.f;
                gWh = mfma16(H2[ti][r], bo, gWh);
            }
            f32x4 zz = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < (Q + 3) / 4; ++ks) {
                const int q = 4 * ks + g;
                const bool qq = q < Q;
                const float av = qq ? dtl[(16 * ti + c) * DQS + (qq ? q : 0)] : 0.f;
                zz = mfma16(av, qq ? Wt.Wh[qq ? q : 0][fb + c] : 0.f, zz);
            }
            dtanh_pk<4>(zz, H2[ti], dZ2[ti]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                gB2 += dZ2[ti][r];
                Zt[16 * ti + 4 * g + r][fb + c] = dZ2[ti][r];
            }
            // dW2^T[in][fb + c] += H1^T dZ2 (A = H1 of every feature block in C layout from its tile)
            if constexpr (Sm::HT) {  // A = H1[sample 16 ti + 4 g + r][16 ib + c]: one ds_read_b128 of the transposed tile
#pragma unroll
                for (int ib = 0; ib < 4; ++ib) {
                    const float4 a4 = *reinterpret_cast<const float4*>(&S.H1T[16 * ib + c][16 * ti + 4 * g]);
                    const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r) gW2[ib] = mfma16(av[r], dZ2[ti][r], gW2[ib]);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib)
                        gW2[ib] = mfma16(S.H1s[16 * ti + 4 * g + r][16 * ib + c], dZ2[ti][r], gW2[ib]);
            }
        }
        // this wave's dW2 / head-weight blocks are final: out now (write-through under the dH1 / dW1 pass)
        auto pub = [&](int k, const f32x4& v) {
            const u32x4 u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
            __builtin_amdgcn_raw_buffer_store_b128(u, xr, islot(hs, par) + ((w * BPW + k) * 64 + l) * 16, 0, SC1);
        };
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) pub(K1M + ib, gW2[ib]);
        if (!CPT || c < 8) pub(K1M + 4, gWh);  // (compact: the head columns now, the rest of the block at the end)
        PGM_STAMP(3);
        lds_sync_m();  // B3: dZ2 of every feature block
        // ---- dH1 = dZ2 W2 for this wave's input block, dZ1, dW1^T[k][fb + c] += X^T dZ1
#pragma unroll
        for (int ti = 0; ti < R; ++ti)
#pragma unroll
            for (int q = 0; q < NC; ++q) z[ti][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // output o = 16 j + 4 g + i of k-step (j, i), as in layer 2
            float bw[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) bw[i] = Wt.W2t[fb + c][16 * j + 4 * g + i];
#pragma unroll
            for (int ti = 0; ti < R; ++ti) {
                const float4 a4 = *reinterpret_cast<const float4*>(&Zt[16 * ti + c][16 * j + 4 * g]);
                const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) z[ti][(4 * j + i) % NC] = mfma16(av[i], bw[i], z[ti][(4 * j + i) % NC]);
            }
        }
#pragma unroll
        for (int ti = 0; ti < R; ++ti) {
            f32x4 zz = z[ti][0], dZ1;
            if constexpr (NC == 2) zz += z[ti][1];
            dtanh_pk<4>(zz, H1[ti], dZ1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                gB1 += dZ1[r];
#pragma unroll
                for (int kb = 0; kb < K1G; ++kb) {
                    const int k = 16 * kb + c;
                    const float ax = k < O ? rt(ti)[(4 * g + r) * RSL + (k < O ? k : 0)] : 0.f;
                    gW1[kb] = mfma16(ax, dZ1[r], gW1[kb]);
                }
                if constexpr (NT > 0) {  // this lane group's 4 samples; the groups are summed after the tiles
                    const float* xr16 = rt(ti) + (4 * g + r) * RSL + 16;
#pragma unroll
                    for (int j = 0; j < NT; ++j) gT[j] = fmaf(xr16[j], dZ1[r], gT[j]);
                }
            }
        }
        gB1 = group4_sum(gB1);
#pragma unroll
        for (int j = 0; j < NT; ++j) gT[j] = group4_sum(gT[j]);
        gB2 = group4_sum(gB2);
        PGM_STAMP(4);

        // ================================================================ exchange
        // ---- 1. publish this wave's gradient blocks (its feature block of every tensor; the dW2 / head blocks
        // went out before B3, so their write-through overlapped the dH1 / dW1 pass)
        dbg_delay(a.dbg, gp, 0);
        {
            float vb2 = 0.f, vls = 0.f;
            if (w == 0) {  // the waves' head partial sums (written before B2b), in wave order
                vb2 = ((S.red[c] + S.red[16 + c]) + S.red[32 + c]) + S.red[48 + c];
                vls = ((S.red[64 + c] + S.red[80 + c]) + S.red[96 + c]) + S.red[112 + c];
                // -entropy_coef * d(mean entropy)/d logstd enters once per tower (ppo.py:98): part 0
                if (hs == 0) vls -= a.hp.entropy_coef;
            }
            if constexpr (CPT) {
                pub(0, gW1[0]);
                // the head block's columns 8..15 through LDS (the head partials are dead after B3): lane v writes entry
                // v of b1 / b2 / head bias / logstd and dW1 inputs 16..19 of feature v (gT) to
                // column 8 + kind, row v; lane (g, c >= 8) reads rows 4 g .. 4 g + 3 of column c
                float* hs_ = &S.HP[0][0][0] + 128 * w;
                if (l < 16) {
                    hs_[l] = gB1;
                    hs_[16 + l] = gB2;
                    hs_[32 + l] = c < NQ ? vb2 : 0.f;
                    hs_[48 + l] = m == 1 && c < A ? vls : 0.f;
#pragma unroll
                    for (int j = 0; j < 4; ++j) hs_[64 + 16 * j + l] = j < NT ? gT[j < NT ? j : 0] : 0.f;
                }
                const float4 h4 = *reinterpret_cast<const float4*>(&hs_[16 * (c - 8 < 0 ? 0 : c - 8) + 4 * g]);
                const f32x4 hv = f32x4{h4.x, h4.y, h4.z, h4.w};
                if (c >= 8) pub(K1M + 4, hv);
            } else {
                const f32x4 vec = g == 0 ? f32x4{gB1, gB2, c < NQ ? vb2 : 0.f, m == 1 && c < A ? vls : 0.f}
                                         : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kb = 0; kb < K1B; ++kb) pub(kb, gW1[kb]);
                pub(K1M + 5, vec);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
        lds_sync_m();
        PGM_STAMP(5);
        const float lsum_wg = ((S.red[128] + S.red[129]) + S.red[130]) + S.red[131];
        if (t == 0)
            __hip_atomic_store(gran(0, m, hs, par), ((unsigned long long)tag << 32) | __float_as_uint(lsum_wg),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // spin on a tagged granule (bounded; a timeout marks the launch failed and every later poll skips)
        auto spin = [&](const unsigned long long* gr, int site) -> unsigned long long {
            if (__hip_atomic_load(fail_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return 0ull;
            for (unsigned spins = 0;; ++spins) {
                const unsigned long long x = __hip_atomic_load(gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((unsigned)(x >> 32) == tag) return x;
                if (spins > (1u << 26)) {
                    __hip_atomic_store(fail_word, fail_code(site, tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return 0ull;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        };
        if (w == 0) {
            if (l < NS) {  // lane h polls part h's image flag (the NS - 1 polls run concurrently)
                dbg_delay(a.dbg, gp, 1);
                S.red[l] = l == hs ? lsum_wg : __uint_as_float((unsigned)spin(gran(0, m, l, par), 0));
            }
        } else {  // the next minibatch's rows (and the one after's indices) while wave 0 polls
            if (gp + 1 < npass) issue_rows((gp + 1) & 1, (gp + 1) & 1, w - 1, 3);
            if (gp + 2 < npass) issue_idx(gp + 2, gp & 1, w - 1, 3);
        }
        lds_sync_m();
        float lsum_all = 0.f;
#pragma unroll
        for (int h = 0; h < NS; ++h) lsum_all += S.red[h];  // part order
        PGM_STAMP(6);
        // ---- 2. reduce-scatter: this part's blocks summed over the NS parts in part order, squared norm
        // (every fragment load of the wave in flight at once: a block past NB loads from beyond the buffer's range,
        // which returns zeros, so there is no branch between the batches)
        f32x4 gr_[OWV];
        float sq = 0.f;
        {
            u32x4 pl[OWV][NS];
#pragma unroll
            for (int i = 0; i < OWV; ++i) {
                const int b = hs + NS * (w + 4 * i);
#pragma unroll
                for (int h = 0; h < NS; ++h)
                    pl[i][h] = __builtin_amdgcn_raw_buffer_load_b128(
                        xr, b < NB ? islot(h, par) + (b * 64 + l) * 16 : 0x7ffffff0, 0, SC1);
            }
#pragma unroll
            for (int i = 0; i < OWV; ++i) {
#pragma unroll
                for (int h = 0; h < NS; ++h) {
                    const f32x4 v = f32x4{__uint_as_float(pl[i][h][0]), __uint_as_float(pl[i][h][1]),
                                          __uint_as_float(pl[i][h][2]), __uint_as_float(pl[i][h][3])};
                    gr_[i] = h == 0 ? v : gr_[i] + v;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) sq = fmaf(gr_[i][r], gr_[i][r], sq);
            }
        }
        sq = wave_sum64(sq);
        if (l == 0) S.red[32 + w] = sq;
        lds_sync_m();
        const float sq_wg = ((S.red[32] + S.red[33]) + S.red[34]) + S.red[35];
        PGM_STAMP(7);
        // ---- 3. squared norms of both towers' parts: one granule each, summed in (tower, part) order
        if (t == 0)
            __hip_atomic_store(gran(1, m, hs, par), ((unsigned long long)tag << 32) | __float_as_uint(sq_wg),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // this step's Adam scalars (fp64 bias corrections) while the granules travel
        const double b1n = b1p * (double)b1c, b2n = b2p * (double)b2c;
        float step_size = (float)(lr / (1.0 - b1n));
        float inv_bc2s = 1.f / (float)sqrt(1.0 - b2n);
        asm volatile("" : "+v"(step_size), "+v"(inv_bc2s));
        if (w == 0 && l < 2 * NS) {
            dbg_delay(a.dbg, gp, 2);
            const int mm = l / NS, hh = l - mm * NS;
            S.red[64 + l] = mm == m && hh == hs ? sq_wg : __uint_as_float((unsigned)spin(gran(1, mm, hh, par), 1));
        }
        lds_sync_m();
        float total = 0.f;
#pragma unroll
        for (int i = 0; i < 2 * NS; ++i) total += S.red[64 + i];
        const float coef = clip_coef(a.hp.max_grad_norm, total);
        if (t == 0) {
            if (m == 0) st_v += lsum_all * vstat;
            else st_a += lsum_all * astat;
            float ent = 0.f;
#pragma unroll
            for (int q = 0; q < A; ++q) ent += 0.5f + LOG_SQRT_2PI + Wt.logstd[q];
            st_e += ent;
        }
        b1p = b1n;
        b2p = b2n;
        PGM_STAMP(8);
        dbg_delay(a.dbg, gp, 3);
        auto adam = [&](float gg, float& mm_, float& vv_, float& pp_) {
            const float gc = gg * coef;
            mm_ = mm_ + (1.f - b1c) * (gc - mm_);
            vv_ = vv_ * b2c + (1.f - b2c) * (gc * gc);
            const float den = __builtin_amdgcn_sqrtf(vv_) * inv_bc2s + eps;
            pp_ -= step_size * mm_ * __builtin_amdgcn_rcpf(den);
        };
        // ---- 4. Adam on the owned blocks (registers), publish them, write them into this part's image
#pragma unroll
        for (int i = 0; i < OWV; ++i) {
            const int b = hs + NS * (w + 4 * i);
            if (b < NB) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float mm = om[i][r], vv = ov[i][r], pp = op[i][r];
                    adam(gr_[i][r], mm, vv, pp);
                    om[i][r] = mm;
                    ov[i][r] = vv;
                    op[i][r] = pp;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (oix[i][r] >= 0) Pf[oix[i][r]] = op[i][r];
            }
            // the part's owned block w + 4 i (slot position always valid: blocks past NB publish unused values, so every
            // wave issues the same number of stores)
            const int jj = w + 4 * i;
            const u32x4 u = {__float_as_uint(op[i][0]), __float_as_uint(op[i][1]), __float_as_uint(op[i][2]),
                             __float_as_uint(op[i][3])};
            __builtin_amdgcn_raw_buffer_store_b128(u, xr, pslot(hs, par) + (jj * 64 + l) * 16, 0, SC1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // + the row DMA issued during the image poll
        lds_sync_m();
        if (t == 0)
            __hip_atomic_store(gran(2, m, hs, par), (unsigned long long)tag << 32, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (w == 0 && l < NS && l != hs) spin(gran(2, m, l, par), 2);
        lds_sync_m();  // every part's blocks published; the next minibatch's rows landed
        PGM_STAMP(9);
        // ---- the other parts' new blocks of this wave's feature block: loads in flight into the next step
        if (gp + 1 < npass) {
#pragma unroll
            for (int k = 0; k < BPW; ++k) pload(k, par);
        }
        PGM_STAMP(10);
    }
    PGM_STAMP_FLUSH;
    // ---- owners write their blocks' parameters and moments back; statistics and the step by part 0
#pragma unroll
    for (int i = 0; i < OWV; ++i) {
        const int b = hs + NS * (w + 4 * i);
        if (b < NB) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ii = oix[i][r];
                const int f = ii >= 0 ? img_to_flat<O, A, K>(ii, m, L) : -1;
                if (f >= 0) {
                    P[f] = op[i][r];
                    Mo[f] = om[i][r];
                    Vo[f] = ov[i][r];
                }
            }
        }
    }
    if (hs == 0 && t == 0) {
        const float n = (float)(E * M);
        if (m == 0) a.stats[p * 3 + 0] = st_v / n;
        if (m == 1) {
            a.step[p] = step0 + npass;
            a.stats[p * 3 + 1] = st_a / n;
            a.stats[p * 3 + 2] = st_e / n;
        }
    }
}

// op 0: launch (dual: two workgroups per CU); op 1: 1 if two workgroups of this kernel fit one CU (LDS and registers),
// else 0; op 2: 1 if one workgroup's LDS fits a CU (160 KiB), else 0
template <int O, int A, int K, int NS, int R>
static int launch_fs_k(const pgm_dims* d, const MArgs& a, bool dual, int op, hipStream_t stream) {
    const size_t smem = fs_smem_bytes<O, A, K, R>(dual || op == 1);
    if (op == 2) return smem <= 160 * 1024 ? 1 : 0;
    if (smem > 160 * 1024) {
        set_error("pgm_ppo_update (fs): LDS %zu bytes exceeds 160 KiB", smem);
        return op == 1 ? 0 : PGM_E_UNSUPPORTED;
    }
    auto kern = ppo_update_fs_kernel<O, A, K, NS, R>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return op == 1 ? 0 : hip_fail(e, "pgm_ppo_update (fs)");
    if (op == 1) {
        int per_cu = 0;
        if (smem > 80 * 1024 || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 256, smem) != hipSuccess)
            return 0;
        return per_cu >= 2 ? 1 : 0;
    }
    const int grid = fs_grid(d->P, NS);
    if (int rc = check_coresident((const void*)kern, 256, smem, grid, "pgm_ppo_update (fs)")) return rc;
    const size_t zb = ppo_flag_bytes(d->P);  // norm / flag granules (the payload needs no reset: tags order it)
    if (!ws_take_zeroed(a.ws, zb)) {
        e = hipMemsetAsync(a.ws, 0, zb, stream);
        if (e != hipSuccess) return hip_fail(e, "pgm_ppo_update (workspace reset)");
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), smem, stream, a);
    return launch_status("pgm_ppo_update (fs)");
}

int ppo_update_fs_op(const pgm_dims* d, const MArgs& a, int ns, bool dual, int op, hipStream_t stream);

// NS parts per tower for this launch: the workspace cap, the device's CUs, mb divisible into 16-row tiles of at most
// 8 per part; 0 = the feature-split update does not apply.  *dual = 1: the grid (16 NS ceil(P/8) workgroups) exceeds
// the CU count and runs two workgroups per CU, taken for R = 2 where both fit one CU (<= 80 KiB LDS, <= 256
// registers): a step's three hand-offs then overlap the other workgroup's tiles (HalfCheetah P = 20: NS 4, R 4
// 4.45 ms -> NS 8, R 2 4.01 ms; profiles/r04r_fs_dual_ab.json).  dual_ok = false (pgm_launch_opts.fs_one_per_cu): one
// per CU only.  The occupancy of the exact kernel is queried at every call (no cached answer: the library keeps no
// mutable state, pgm_abi.h).
int fs_choose_ns(const pgm_dims* d, int mb, bool dual_ok, int* dual) {
    *dual = 0;
    if (d->O > 32) return 0;
    const int cus = device_cu_count();
    if (mb % 16 != 0) return 0;
    for (const int ns : FS_NS_LIST) {
        // (6 parts: the row tiles dealt raggedly, at most 3 per part; other counts: an exact split)
        if (ns != 6 && mb % (16 * ns) != 0) continue;
        const int R = fs_tiles(mb, ns);
        if (!fs_built(ns, R)) continue;
        const int grid = fs_grid(d->P, ns);
        if (grid > 2 * cus) continue;
        MArgs q{};
        q.hp.num_mini_batch = d->T * d->N / mb;
        // (O = 27: 8 tiles per part overflow the LDS; the next NS down is taken instead)
        if (grid <= cus && ppo_update_fs_op(d, q, ns, false, 2, nullptr) == 1) return ns;
        // two workgroups per CU for R = 2 / 3 (R 4 -> 2 pays; R 2 -> 1 does not: Walker P = 10 3.18 -> 3.70 ms)
        if (grid > cus && dual_ok && (R == 2 || R == 3)) {
            if (ppo_update_fs_op(d, q, ns, true, 1, nullptr) == 1) {
                *dual = 1;
                return ns;
            }
        }
    }
    return 0;
}

template <int O, int A, int K, int NS>
static int launch_fs_ns(const pgm_dims* d, const MArgs& a, int R, bool dual, int op, hipStream_t stream) {
    // minibatches of 64 / 128 / 256 / 512 rows (N = 1 / 2 / 4 / 8 at T = 2048, M = 32): 16 NS R = mb
    auto one = [&](auto rc) -> int {
        constexpr int RR = decltype(rc)::value, MB = 16 * NS * RR;
        if constexpr (fs_built(NS, RR)) return launch_fs_k<O, A, K, NS, RR>(d, a, dual, op, stream);
        set_error("pgm_ppo_update (fs): minibatch of %d rows unsupported", MB);
        return PGM_E_UNSUPPORTED;
    };
    switch (R) {
        case 1: return one(ic<1>{});
        case 2: return one(ic<2>{});
        case 3: return one(ic<3>{});
        case 4: return one(ic<4>{});
        case 8: return one(ic<8>{});
    }
    set_error("pgm_ppo_update (fs): %d row tiles per part unsupported", R);
    return PGM_E_UNSUPPORTED;
}

// called by pgm_ppo_mfma.hip's launcher after the sample table is packed
int ppo_update_fs(const pgm_dims* d, const MArgs& a, int ns, bool dual, hipStream_t stream) {
    return ppo_update_fs_op(d, a, ns, dual, 0, stream);
}
int ppo_update_fs_op(const pgm_dims* d, const MArgs& a, int ns, bool dual, int op, hipStream_t stream) {
    const int mb = d->T * d->N / a.hp.num_mini_batch;
    const int R = fs_tiles(mb, ns);
    return dispatch_dims(d->O, d->A, d->K, "pgm_ppo_update (fs)", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
#ifdef PGM_STAMPS
        constexpr bool skip = O != 17;  // diagnostic builds: the Walker / HalfCheetah dims only (compile time)
#else
        constexpr bool skip = false;
#endif
        if constexpr (O > 32 || skip) {
            return op != 0 ? 0 : PGM_E_UNSUPPORTED;
        } else {
            switch (ns) {
                case 2: return launch_fs_ns<O, A, K, 2>(d, a, R, dual, op, stream);
                case 4: return launch_fs_ns<O, A, K, 4>(d, a, R, dual, op, stream);
                case 6: return launch_fs_ns<O, A, K, 6>(d, a, R, dual, op, stream);
                case 8: return launch_fs_ns<O, A, K, 8>(d, a, R, dual, op, stream);
                case 16: return launch_fs_ns<O, A, K, 16>(d, a, R, dual, op, stream);
            }
            set_error("pgm_ppo_update (fs): NS=%d unsupported", ns);
            return PGM_E_UNSUPPORTED;
        }
    });
}

}  // namespace pgm

// the fragment map as the kernels use it (frag_img on the host): what the CPU tests check for a bijection onto the
// tower's parameters
extern "C" int pgm_ppo_fs_fragment_map(int32_t O, int32_t A, int32_t K, int32_t m, int32_t* out, int32_t cap) {
    using namespace pgm;
    return dispatch_dims(O, A, K, "pgm_ppo_fs_fragment_map", [&](auto o, auto aa, auto k) -> int {
        constexpr int O_ = decltype(o)::value, A_ = decltype(aa)::value, K_ = decltype(k)::value;
        if constexpr (O_ > 32) {
            set_error("pgm_ppo_fs_fragment_map: obs_dim %d > 32 has no feature-split update", O_);
            return PGM_E_UNSUPPORTED;
        } else {
            constexpr int NB = fs_nb(O_);
            if (!out || cap < NB * 256 || (m != 0 && m != 1)) {
                set_error("pgm_ppo_fs_fragment_map: tower %d, buffer %d < %d entries", m, cap, NB * 256);
                return PGM_E_INVALID_ARG;
            }
            for (int b = 0; b < NB; ++b)
                for (int l = 0; l < 64; ++l)
                    for (int r = 0; r < 4; ++r) out[(b * 64 + l) * 4 + r] = frag_img<O_, A_, K_>(b, l, r, m);
            return NB;
        }
    });
}
