// Shared pieces of the obs_dim <= 32 PPO update kernels (pgm_ppo_mfma.hip: MODE 0/1/2 and 16-row tiles;
// pgm_ppo_fs.hip: feature-split tiles with a reduce-scattered Adam): the LDS tower image, its map to the flat
// parameter layout, the launch arguments and the clip coefficient.
#pragma once
#include "pgm_mfma.hpp"

namespace pgm {

// clip_grad_norm_'s coefficient min(max_norm / (sqrt(sum of squares) + 1e-6), 1) (torch nn/utils/clip_grad.py):
// hardware sqrt and a Newton-refined reciprocal (<= 1 ulp) instead of the IEEE expansions, off the critical path's
// division sequences
__device__ __forceinline__ float clip_coef(float max_norm, float sumsq) {
    const float d = __builtin_amdgcn_sqrtf(sumsq) + 1e-6f;
    float r = __builtin_amdgcn_rcpf(d);
    r = fmaf(fmaf(-d, r, 1.f), r, r);
    return fminf(max_norm * r, 1.f);
}

// ---------------------------------------------------------------- tower images
// One tower's parameters as an LDS image: W1^T [in][out], W2^T [in][out] with a padded row stride,
// head weights [output][unit], biases, logstd (actor only).  Padding slots and head rows beyond the
// tower's output count hold zeros for the whole launch (their gradient, Adam moments and update are 0).
// The same image type holds gradients and (SPLIT) the Adam moments, so clip_grad_norm_ and Adam are
// flat passes over images, and the working copy IS the master copy until the launch writes it back.
template <int O, int A, int K>
struct TowerImg {
    static constexpr int Q = qmax<A, K>();
    float W1t[O][H];
    float W2t[H][SCR];
    float Wh[Q][H];
    float b1[H], b2[H], bh[Q], logstd[A];
};
template <int O, int A, int K>
constexpr int img_floats() { return (int)(sizeof(TowerImg<O, A, K>) / sizeof(float)); }

// image slot -> flat parameter index (pgm_param_layout order), -1 for padding / unused slots
template <int O, int A, int K>
__device__ __forceinline__ int img_to_flat(int i, int m, const Layout& L) {
    constexpr int Q = qmax<A, K>();
    constexpr int s1 = O * H, s2 = s1 + H * SCR, s3 = s2 + Q * H, s4 = s3 + H, s5 = s4 + H, s6 = s5 + Q, s7 = s6 + A;
    const int NQ = m == 0 ? K : A;
    if (i < s1) return L.off[m ? PGM_P_ACTOR_W1 : PGM_P_CRITIC_W1] + i;
    if (i < s2) {
        const int j = i - s1, in = j / SCR, o = j - in * SCR;
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

struct MArgs {
    int N, T;
    Layout L;
    pgm_ppo_hparams hp;
    float *params, *m, *v;
    int32_t* step;
    const float* lr;
    const int32_t* perms;
    const float* rows;       // packed sample table [P][T*N][RS]
    float* stats;
    unsigned long long* ws;  // SPLIT: tagged norm granules + timeout flag (word 2P), zeroed before the launch
    unsigned long long* xb;  // MODE 2: gradient-image exchange slots, zeroed before the launch
    int xslot;               // 8-byte words per exchange slot (image payload, flag granule in the last word)
    int xbytes;              // bytes of the exchange buffer
    int P;
    DbgDelay dbg;            // test-only exchange delay (PGM_TEST_DELAY; cycles 0 = off)
    char* fsp;               // feature-split update: exchange payload (pgm_ppo_fs.hip), after the sample table
};

constexpr int T16 = 16;       // samples per tile
constexpr int S16 = H + 2;    // transpose-tile row stride: conflict-free A-operand reads, 2-way (free) writes
constexpr int DQ = 8;         // head-output columns of the dO transpose tile (Q <= 8)
constexpr int DQS = DQ + 1;

}  // namespace pgm
