// Lane-parallel rollout, critic-value and evaluation kernels (obs_dim <= 48, the default path for every
// SynthMO env but Humanoid; Humanoid uses the block-per-task kernels of pgm_policy_env.hip).
//
// rollout_lane_kernel: one workgroup per task, env n on wave n % 4.  A wave's lanes hold unit l of the
// ACTOR tower (the env step only needs the action) and feature l of its env's state.  The critic is not on
// the T-step dependency chain at all: value_kernel evaluates it afterwards for all (T+1) x N stored
// observations at once.  The one cross-env step of an iteration, the VecNormalize running statistics, is
// computed REDUNDANTLY by every wave from a double-buffered LDS row per env (lane l < O: feature l of
// ob_rms; lanes O..O+K-1: obj_rms; lane O+K: ret_rms), so a step costs one workgroup barrier and the
// normalised observation never leaves the wave that needs it.  The action mean is wave-uniform (DPP sums
// end in readlanes), so the Gaussian draw, the clipped action and the log-prob are computed uniformly in
// every lane: no cross-lane traffic between the policy head and the dynamics.
//
// eval_wave_kernel: one wave per evaluation episode (morl/mopg.py:25-46), no workgroup barriers.
//
// Reference semantics (paths relative to the reference tree):
//   Policy.act / get_value                 a2c_ppo_acktr/model.py:57-73, 237-246
//   DiagGaussian sample + log_prob         a2c_ppo_acktr/distributions.py:29-40,71-90
//   DummyVecEnv auto-reset                 baselines/common/vec_env/dummy_vec_env.py:45-56
//   TimeLimitMask bad_transition           a2c_ppo_acktr/envs.py:122-131
//   VecNormalize.step_wait                 baselines/common/vec_env/vec_normalize.py:29-61
//   RunningMeanStd Chan merge              baselines/common/running_mean_std.py:3-31
//   masks / bad_masks / obj_tensor         morl/mopg.py:110-130
//   RolloutStorage.insert / after_update   a2c_ppo_acktr/storage.py:50-75
//   bootstrap value (get_value on obs[T])  morl/mopg.py:132-135, storage.py:85
//   evaluation()                           morl/mopg.py:25-46
#include "pgm_dispatch.hpp"
#include "pgm_rollout.hpp"
#include "pgm_mfma.hpp"
#include <utility>

PGM_STAMP_UNIT(lanes)

namespace pgm {

typedef float f2 __attribute__((ext_vector_type(2)));

template <int O, int K>
constexpr bool lanes_fit() { return O <= 48 && O + K + 1 <= 64; }


template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// NR row-broadcast copies of v: copy j holds, in EVERY 16-lane row, row j of v (lane 16 r + i <- lane 16 j + i).
// One v_permlane32_swap (rows [0 1 0 1] / [2 3 2 3]) and one v_permlane16_swap per pair of copies.
template <int NR>
__device__ __forceinline__ void row_copies(float v, float (&V)[NR]) {
    static_assert(NR >= 1 && NR <= 4, "1..4 rows");
    const unsigned u = __float_as_uint(v);
    const auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    const auto q0 = __builtin_amdgcn_permlane16_swap(p[0], p[0], false, false);
    V[0] = __uint_as_float(q0[0]);
    if constexpr (NR > 1) V[1] = __uint_as_float(q0[1]);
    if constexpr (NR > 2) {
        const auto q1 = __builtin_amdgcn_permlane16_swap(p[1], p[1], false, false);
        V[2] = __uint_as_float(q1[0]);
        if constexpr (NR > 3) V[3] = __uint_as_float(q1[1]);
    }
}
// acc[i % 4] += (lane i of this lane's 16-lane row of v) * w[i], i = 0..NK-1: v_fmac_f32 with a DPP row_newbcast:i
// source operand (gfx90a+; the compiler's DPP combiner does not fold a row_newbcast mov into fmac), ONE asm block per
// row, whose leading s_nop covers the VALU-write -> DPP-read hazard on v (the asm hides the DPP read from the hazard
// recognizer; inside one block nothing can write v).  Four accumulator chains.
#define PGM_FL0 "v_fmac_f32_dpp %0, %4, %5 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL1 "v_fmac_f32_dpp %1, %4, %6 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL2 "v_fmac_f32_dpp %2, %4, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL3 "v_fmac_f32_dpp %3, %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL4 "v_fmac_f32_dpp %0, %4, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL5 "v_fmac_f32_dpp %1, %4, %10 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL6 "v_fmac_f32_dpp %2, %4, %11 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL7 "v_fmac_f32_dpp %3, %4, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL8 "v_fmac_f32_dpp %0, %4, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL9 "v_fmac_f32_dpp %1, %4, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL10 "v_fmac_f32_dpp %2, %4, %15 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL11 "v_fmac_f32_dpp %3, %4, %16 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL12 "v_fmac_f32_dpp %0, %4, %17 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL13 "v_fmac_f32_dpp %1, %4, %18 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL14 "v_fmac_f32_dpp %2, %4, %19 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FL15 "v_fmac_f32_dpp %3, %4, %20 row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FU1 PGM_FL0
#define PGM_FU2 PGM_FU1 PGM_FL1
#define PGM_FU3 PGM_FU2 PGM_FL2
#define PGM_FU4 PGM_FU3 PGM_FL3
#define PGM_FU5 PGM_FU4 PGM_FL4
#define PGM_FU6 PGM_FU5 PGM_FL5
#define PGM_FU7 PGM_FU6 PGM_FL6
#define PGM_FU8 PGM_FU7 PGM_FL7
#define PGM_FU9 PGM_FU8 PGM_FL8
#define PGM_FU10 PGM_FU9 PGM_FL9
#define PGM_FU11 PGM_FU10 PGM_FL10
#define PGM_FU12 PGM_FU11 PGM_FL11
#define PGM_FU13 PGM_FU12 PGM_FL12
#define PGM_FU14 PGM_FU13 PGM_FL13
#define PGM_FU15 PGM_FU14 PGM_FL14
#define PGM_FU16 PGM_FU15 PGM_FL15
// (volatile in the stamps build only: a plain asm block may move across the s_memtime stamps)
#ifdef PGM_STAMPS
#define PGM_ASM_Q volatile
#else
#define PGM_ASM_Q
#endif
#define PGM_FMAC_ASM(body)                                                                                       \
    asm PGM_ASM_Q("s_nop 1\n\t" body                                                                          \
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])                                                \
        : "v"(v), "v"(wv[0]), "v"(wv[1]), "v"(wv[2]), "v"(wv[3]), "v"(wv[4]), "v"(wv[5]), "v"(wv[6]), "v"(wv[7]), \
          "v"(wv[8]), "v"(wv[9]), "v"(wv[10]), "v"(wv[11]), "v"(wv[12]), "v"(wv[13]), "v"(wv[14]), "v"(wv[15]))
// FIRST: the layer's first row -- accumulators 1..3 start with a v_mul_f32_dpp instead of a zeroing v_mov + v_fmac
#define PGM_FM1 "v_mul_f32_dpp %1, %4, %6 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FM2 "v_mul_f32_dpp %2, %4, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FM3 "v_mul_f32_dpp %3, %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
#define PGM_FMAC_ASM_FIRST(body)                                                                                 \
    asm PGM_ASM_Q("s_nop 1\n\t" body                                                                          \
        : "+v"(acc[0]), "=&v"(acc[1]), "=&v"(acc[2]), "=&v"(acc[3])                                             \
        : "v"(v), "v"(wv[0]), "v"(wv[1]), "v"(wv[2]), "v"(wv[3]), "v"(wv[4]), "v"(wv[5]), "v"(wv[6]), "v"(wv[7]), \
          "v"(wv[8]), "v"(wv[9]), "v"(wv[10]), "v"(wv[11]), "v"(wv[12]), "v"(wv[13]), "v"(wv[14]), "v"(wv[15]))
#define PGM_FF4 PGM_FL0 PGM_FM1 PGM_FM2 PGM_FM3
#define PGM_FF5 PGM_FF4 PGM_FL4
#define PGM_FF6 PGM_FF5 PGM_FL5
#define PGM_FF7 PGM_FF6 PGM_FL6
#define PGM_FF8 PGM_FF7 PGM_FL7
#define PGM_FF9 PGM_FF8 PGM_FL8
#define PGM_FF10 PGM_FF9 PGM_FL9
#define PGM_FF11 PGM_FF10 PGM_FL10
#define PGM_FF12 PGM_FF11 PGM_FL11
#define PGM_FF13 PGM_FF12 PGM_FL12
#define PGM_FF14 PGM_FF13 PGM_FL13
#define PGM_FF15 PGM_FF14 PGM_FL14
#define PGM_FF16 PGM_FF15 PGM_FL15
template <int NK, bool FIRST = false>
__device__ __forceinline__ void fmac_row_bcast(float (&acc)[4], float v, const float* w) {
    static_assert(NK >= 1 && NK <= 16, "1..16 lanes");
    float wv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) wv[i] = i < NK ? w[i] : 0.f;
    if constexpr (FIRST && NK >= 4) {
        if constexpr (NK == 4) PGM_FMAC_ASM_FIRST(PGM_FF4);
        else if constexpr (NK == 5) PGM_FMAC_ASM_FIRST(PGM_FF5);
        else if constexpr (NK == 6) PGM_FMAC_ASM_FIRST(PGM_FF6);
        else if constexpr (NK == 7) PGM_FMAC_ASM_FIRST(PGM_FF7);
        else if constexpr (NK == 8) PGM_FMAC_ASM_FIRST(PGM_FF8);
        else if constexpr (NK == 9) PGM_FMAC_ASM_FIRST(PGM_FF9);
        else if constexpr (NK == 10) PGM_FMAC_ASM_FIRST(PGM_FF10);
        else if constexpr (NK == 11) PGM_FMAC_ASM_FIRST(PGM_FF11);
        else if constexpr (NK == 12) PGM_FMAC_ASM_FIRST(PGM_FF12);
        else if constexpr (NK == 13) PGM_FMAC_ASM_FIRST(PGM_FF13);
        else if constexpr (NK == 14) PGM_FMAC_ASM_FIRST(PGM_FF14);
        else if constexpr (NK == 15) PGM_FMAC_ASM_FIRST(PGM_FF15);
        else PGM_FMAC_ASM_FIRST(PGM_FF16);
    } else if constexpr (FIRST) {
        acc[1] = acc[2] = acc[3] = 0.f;  // (NK < 4: zeroed, then accumulated)
        fmac_row_bcast<NK, false>(acc, v, w);
    } else {
        if constexpr (NK == 1) PGM_FMAC_ASM(PGM_FU1);
        else if constexpr (NK == 2) PGM_FMAC_ASM(PGM_FU2);
        else if constexpr (NK == 3) PGM_FMAC_ASM(PGM_FU3);
        else if constexpr (NK == 4) PGM_FMAC_ASM(PGM_FU4);
        else if constexpr (NK == 5) PGM_FMAC_ASM(PGM_FU5);
        else if constexpr (NK == 6) PGM_FMAC_ASM(PGM_FU6);
        else if constexpr (NK == 7) PGM_FMAC_ASM(PGM_FU7);
        else if constexpr (NK == 8) PGM_FMAC_ASM(PGM_FU8);
        else if constexpr (NK == 9) PGM_FMAC_ASM(PGM_FU9);
        else if constexpr (NK == 10) PGM_FMAC_ASM(PGM_FU10);
        else if constexpr (NK == 11) PGM_FMAC_ASM(PGM_FU11);
        else if constexpr (NK == 12) PGM_FMAC_ASM(PGM_FU12);
        else if constexpr (NK == 13) PGM_FMAC_ASM(PGM_FU13);
        else if constexpr (NK == 14) PGM_FMAC_ASM(PGM_FU14);
        else if constexpr (NK == 15) PGM_FMAC_ASM(PGM_FU15);
        else PGM_FMAC_ASM(PGM_FU16);
    }
}

// per-lane actor tower: unit l of both layers, every head row of unit l (weights constant in a launch)
template <int O, int A>
struct ActorLane {
    float w1[O], w2[H], wm[A], bm[A], ls[A], sd[A], rsd[A];
    float b1, b2;
    __device__ void load(const float* __restrict__ prm, const Layout& L, int l) {
#pragma unroll
        for (int k = 0; k < O; ++k) w1[k] = prm[L.off[PGM_P_ACTOR_W1] + k * H + l];
#pragma unroll
        for (int k = 0; k < H; ++k) w2[k] = prm[L.off[PGM_P_ACTOR_W2] + k * H + l];
#pragma unroll
        for (int j = 0; j < A; ++j) {
            wm[j] = prm[L.off[PGM_P_MEAN_W] + l * A + j];
            bm[j] = prm[L.off[PGM_P_MEAN_B] + j];
            ls[j] = prm[L.off[PGM_P_LOGSTD] + j];
            sd[j] = expf(ls[j]);
            rsd[j] = 1.0f / sd[j];
        }
        b1 = prm[L.off[PGM_P_ACTOR_B1] + l];
        b2 = prm[L.off[PGM_P_ACTOR_B2] + l];
        // the per-action constants are wave-uniform; kept in VGPRs (the SGPR file is the step loop's scarce
        // resource: spilled SGPRs come back through v_readlane + s_nop every step)
#pragma unroll
        for (int j = 0; j < A; ++j) {
            asm volatile("" : "+v"(bm[j]));
            asm volatile("" : "+v"(ls[j]));
            asm volatile("" : "+v"(sd[j]));
            asm volatile("" : "+v"(rsd[j]));
        }
    }
    // action mean of this lane's input: lane k < O holds input feature k (other lanes: anything), -> mu[A],
    // wave-uniform.  Every input reaches every lane by a row copy + row_newbcast
    // DPP operand of the FMA (no LDS round trip, no v_readlane); four accumulator chains per layer.  (Measured and
    // dropped: the LDS input row with 64 v_readlane for layer 2, and layer-2 inputs by an LDS row into packed FMAs.)
    // murow (optional): the head sums' two reduced rows for another wave (wave_sum64_multi rows)
    __device__ void forward_reg(float xv, float (&mu)[A], float* murow = nullptr) const {
        constexpr int R1 = (O + 15) / 16;
        float X[R1];
        row_copies<R1>(xv, X);
        float z[4];
        z[0] = b1;
        static_for<R1>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            fmac_row_bcast<(O - 16 * j < 16 ? O - 16 * j : 16), j == 0>(z, X[j], &w1[16 * j]);
        });
        const float hl = tanh_fast((z[0] + z[1]) + (z[2] + z[3]));
        float Hc[4];
        row_copies<4>(hl, Hc);
        float y[4];
        y[0] = b2;
        fmac_row_bcast<16, true>(y, Hc[0], &w2[0]);
#pragma unroll
        for (int j = 1; j < 4; ++j) fmac_row_bcast<16>(y, Hc[j], &w2[16 * j]);
        const float h2 = tanh_fast((y[0] + y[1]) + (y[2] + y[3]));
        float pr[A];
#pragma unroll
        for (int j = 0; j < A; ++j) pr[j] = h2 * wm[j];
        wave_sum64_multi<A>(pr, mu, murow);
#pragma unroll
        for (int j = 0; j < A; ++j) mu[j] += bm[j];
    }
};

// per-lane SynthMO constants of feature o = l (zeros beyond O) and the wave-uniform ones
template <int O, int A, int K>
struct EnvLane {
    double U[A], V[K], d, c;
    double lo[A], hi[A], ebase[K], ecoef[K];
    __device__ void load(const pgm_env_spec& g, int l) {
        const bool fl = l < O;
        const int o = fl ? l : 0;
#pragma unroll
        for (int j = 0; j < A; ++j) {
            U[j] = fl ? g.U[o * A + j] : 0.0;
            lo[j] = g.act_lo[j];
            hi[j] = g.act_hi[j];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            V[k] = fl ? g.V[k * O + o] : 0.0;
            ebase[k] = g.ebase[k];
            ecoef[k] = g.ecoef[k];
        }
        d = fl ? g.d[o] : 0.0;
        c = fl ? g.c[o] : 0.0;
#pragma unroll
        for (int j = 0; j < A; ++j) {  // wave-uniform constants in VGPRs (see ActorLane::load)
            asm volatile("" : "+v"(lo[j]));
            asm volatile("" : "+v"(hi[j]));
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            asm volatile("" : "+v"(ebase[k]));
            asm volatile("" : "+v"(ecoef[k]));
        }
    }
    // s' = tanh(d*s + U clip(a) + c) for this lane's feature; raw objectives (wave-uniform):
    // obj_k = V_k . s' + ebase_k - ecoef_k * |clip(a)|^2   (the Walker form, environments/walker2d.py:23-25)
    // s' of this lane's feature (rcp-based fp64 tanh: no IEEE division on the step chain)
    __device__ double next_state(double s, const double (&ac)[A]) const {
        double pu[A];
#pragma unroll
        for (int j = 0; j < A; ++j) pu[j] = U[j] * ac[j];
        return tanh_d2(d * s + tree_sum(pu) + c);
    }
    // raw objectives of next state sn (wave-uniform)
    __device__ void objectives(double sn, double e2, double (&objraw)[K]) const {
#pragma unroll
        for (int k = 0; k < K; ++k) objraw[k] = V[k] * sn;
        wave_sum64_d_multi<K>(objraw, objraw);
#pragma unroll
        for (int k = 0; k < K; ++k) objraw[k] += ebase[k] - ecoef[k] * e2;
    }
    __device__ double step(double s, const double (&ac)[A], double e2, double (&objraw)[K]) const {
        double pu[A];
#pragma unroll
        for (int j = 0; j < A; ++j) pu[j] = U[j] * ac[j];
        const double sn = tanh_d(d * s + tree_sum(pu) + c);
#pragma unroll
        for (int k = 0; k < K; ++k) objraw[k] = V[k] * sn;
        wave_sum64_d_multi<K>(objraw, objraw);
#pragma unroll
        for (int k = 0; k < K; ++k) objraw[k] += ebase[k] - ecoef[k] * e2;
        return sn;
    }
};

// ------------------------------------------------------------------------------------------ rollout
constexpr int NCH = 32;  // rollout steps per staged noise chunk
// The step's action side is off the chain: the chain waves draw the action and step the dynamics only; the objective
// waves redo the draw from the head sums' rows (same fp32 operations, so the same action), and own the log-prob,
// |clip(a)|^2, the action / log-prob / mask stores.  A single wave issues at most one VALU instruction per ~4 cycles,
// and the chain wave is the one whose instruction count sets the step time (two waves per SIMD).

template <int O, int A, int NN>
struct LaneSmem {
    double sr[2][NN][64];                // statistics rows, double-buffered by step parity
    double sn[2][NN][64];                // pre-reset next state of env n (feature lanes), by step parity
    int dn[2][NN];                       // done of env n, by step parity
    double t2[32];                       // 2^(j/32): tanh_d3's exp table
    double rinv[2][64];                  // the chain's merged 1 / sqrt(var + eps) per statistic lane, by step parity
    float mur[2][NN][128];               // env n's action-mean rows (wave_sum64_multi rows), by step parity
    alignas(16) float eps[2][NN][NCH * A];  // action noise of env n for NCH steps, double-buffered
};

// raw buffer store of one dword per lane; a lane whose offset is OOB_OFF stores nothing (the buffer's range
// check drops it), so the per-role output stores need no exec-mask branches inside the step loop
constexpr uint32_t OOB_OFF = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void* base, size_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void store_lane(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, 0, 0);
}
// clip as two bare v_max_f64 / v_min_f64 that the scheduler may move (clipd_hw is a volatile asm barrier)
__device__ __forceinline__ double clipd_s(double x, double lo, double hi) {
    double r;
    asm("v_max_f64 %0, %1, %2\n\tv_min_f64 %0, %0, %3" : "=&v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

// Two wave roles per env slot (2 NW waves, NW = min(N, 4); two waves per SIMD):
//  * CHAIN waves (w < NW) run the observation chain: policy -> Gaussian draw -> fp64 dynamics -> time
//    limit / auto-reset -> ob_rms merge -> next normalised input, and store obs / actions / log-probs / masks;
//  * OBJECTIVE waves (w >= NW, env slots of wave w - NW) run everything the chain does not need: the raw
//    objectives (fp64 wave sums of V . s'), the discounted objective / ret accumulators and the rewards,
//    reading s', |a|^2 and done from parity-buffered LDS rows after each step's barrier.  They run one step
//    behind (step t's objective side after barrier t), so they only fill the chain waves' stall slots on the
//    shared SIMDs.  The obj_rms / ret_rms merges of their accumulators (after barrier t + 1) run in the CHAIN
//    waves' ob_rms merge, which executes all 64 statistic lanes of the row anyway: the two roles share each
//    SIMD's issue slots, so the objective waves' own copy of that fp64 merge was pure extra issue.  The merged
//    reciprocal std goes to LDS, and step t's reward leaves after barrier t + 2.
// Both roles execute the same barriers (one per step plus two drain barriers).
//
// (Measured and dropped: the two roles in two workgroups per task, the chain streaming its states, action-mean rows and
// done flags to a scratch with sc1 stores and publishing every 16 steps -- 2.31 vs 1.91 ms per Walker P = 40 rollout:
// every publish drains the chain's sc1 stores and each chunk's loads pay a memory round trip.)
template <int O, int A, int K, int NN>
__global__ __launch_bounds__(512) void rollout_lane_kernel(RolloutArgs a) {
    static_assert(lanes_fit<O, K>(), "lane roles need O + K + 1 <= 64");
    constexpr int NW = NN < 4 ? NN : 4;  // waves per role
    constexpr int NE = (NN + 3) / 4;     // env slots per wave
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<LaneSmem<O, A, NN>*>(smem_raw);
    const int p = (int)blockIdx.x, l = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool chain = wv < NW;
    const int w = chain ? wv : wv - NW;  // env slot base of this wave
    const int T = a.T;
    const NormCfg nc = norm_cfg(a.ns);
    const Layout& L = a.L;
    float* obs = a.rb.obs + (size_t)p * (T + 1) * NN * O;
    float* masks = a.rb.masks + (size_t)p * (T + 1) * NN;
    float* bad = a.rb.bad_masks + (size_t)p * (T + 1) * NN;
    const bool fl = l < O;
    const int lo = fl ? l : 0;

    // ---- running statistics, one lane per statistic (role 0: ob feature l, 1: objective l - O, 2: ret),
    // replicated in every wave (the chain waves use role 0, the objective waves roles 1 and 2)
    const int role = l < O ? 0 : l < O + K ? 1 : l == O + K ? 2 : 3;
    const int ko = role == 1 ? l - O : 0;
    double mean = 0.0, var = 1.0, cnt = 1.0;
    if (role == 0) {
        mean = a.ns.ob_mean[(size_t)p * O + l];
        var = a.ns.ob_var[(size_t)p * O + l];
        cnt = a.ns.ob_count[p];
    } else if (role == 1) {
        mean = a.ns.obj_mean[p * K + ko];
        var = a.ns.obj_var[p * K + ko];
        cnt = a.ns.obj_count[p];
    } else if (role == 2) {
        mean = a.ns.ret_mean[p];
        var = a.ns.ret_var[p];
        cnt = a.ns.ret_count[p];
    }
    const bool upd = role == 0 ? nc.use_ob != 0 : role == 1 ? nc.use_obj != 0 : role == 2;
    double inv = 1.0;
    // 1 / (count + N) for the next merge: hardware reciprocal + two Newton steps, formed before the barrier.
    // (Measured and dropped: the merge's old-statistics factors var cnt / tot, cnt N / tot^2, N / tot formed here too,
    // so that var' = fma(delta^2, ., fma(sq, 1 / tot, .)) after the barrier: 1.90 -> 1.99 ms per Walker P = 40 rollout.)
    double itot = 0.0;
    auto prep_merge = [&]() {
        const double tot = cnt + (double)NN;
        double r = __builtin_amdgcn_rcp(tot);
        r = fma(r, fma(-tot, r, 1.0), r);
        itot = fma(r, fma(-tot, r, 1.0), r);
    };
    // 1 / sqrt(x) to ~4e-15 relative (one Newton step): the normalised observations and the rewards leave as fp32
    auto rsqrt_1 = [](double x) {
        const double r = __builtin_amdgcn_rsq(x);
        return fma(r * fma(-x * r, r, 1.0), 0.5, r);
    };
    // statistics merge of this lane's role (counts from before the merge; numpy's mean / var divide by N,
    // exact for N a power of two); prep_merge() ran since the last merge
    auto merge = [&](int buf, bool active) {
        double v[NN];
#pragma unroll
        for (int n = 0; n < NN; ++n) v[n] = S.sr[buf][n][l];
        double sum = v[0];  // numpy's add.reduce order over the env axis
#pragma unroll
        for (int n = 1; n < NN; ++n) sum += v[n];
        constexpr double rn = 1.0 / NN;
        const double bm = sum * rn;
        double d2[NN];
#pragma unroll
        for (int n = 0; n < NN; ++n) d2[n] = (v[n] - bm) * (v[n] - bm);
        double sq = d2[0];  // numpy's var(axis=0): the squared deviations also summed in env order
#pragma unroll
        for (int n = 1; n < NN; ++n) sq += d2[n];
        if (upd && active) {
            const double delta = bm - mean;
            mean = mean + delta * (double)NN * itot;
            var = (var * cnt + (sq * rn) * (double)NN + delta * delta * cnt * (double)NN * itot) * itot;
            cnt += (double)NN;
            inv = rsqrt_1(var + nc.eps);  // (two Newton steps measured 2.02 vs 1.90 ms per Walker P = 40 rollout)
        }
    };
    if (threadIdx.x < 32) S.t2[threadIdx.x] = exp2((double)threadIdx.x / 32.0);
    lds_sync();  // (every wave: the two roles execute the same barriers)
    PGM_STAMP_DECL

    if (chain) {
        // =========================================================== chain waves
        // issue priority over the objective waves that share their SIMDs (those only fill the chain's stalls)
        __builtin_amdgcn_s_setprio(3);
        const float* prm = a.params + (size_t)p * L.total;
        const int maxs = a.spec.max_episode_steps;
        const auto r_obs = out_rsrc(obs, (size_t)(T + 1) * NN * O * 4);
        ActorLane<O, A> pol;
        pol.load(prm, L, l);
        // per-lane SynthMO constants of feature l (the dynamics; the objective constants live in the
        // objective waves)
        double U[A], dd, cc, alo[A], ahi[A];
        {
            const pgm_env_spec& g = a.spec;
#pragma unroll
            for (int j = 0; j < A; ++j) {
                U[j] = fl ? g.U[lo * A + j] : 0.0;
                alo[j] = g.act_lo[j];
                ahi[j] = g.act_hi[j];
                asm volatile("" : "+v"(alo[j]));  // wave-uniform constants in VGPRs (see ActorLane::load)
                asm volatile("" : "+v"(ahi[j]));
            }
            dd = fl ? g.d[lo] : 0.0;
            cc = fl ? g.c[lo] : 0.0;
        }
        double s_o[NE], s0_o[NE];
        int elapsed[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int n = min(w + 4 * e, NN - 1);
            s_o[e] = a.st.s[((size_t)p * NN + n) * O + lo];
            s0_o[e] = a.st.s0[(size_t)n * O + lo];
            elapsed[e] = a.st.elapsed[p * NN + n];
        }

        // ---- slot 0: after_update() carry (storage.py:71-75) and the first policy input
        float xr[NE];  // normalised input feature l of env slot e (lanes < O)
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            xr[e] = 0.f;
            const int n = w + 4 * e;
            if (n >= NN) break;
            if (fl) {
                float v = obs[(size_t)(a.carry ? T : 0) * NN * O + n * O + l];
                if (a.carry) obs[n * O + l] = v;
                xr[e] = v;
            }
            if (a.carry && l == 0) {
                masks[n] = masks[(size_t)T * NN + n];
                bad[n] = bad[(size_t)T * NN + n];
            }
        }
        // action noise, staged per wave in LDS chunks of NCH steps: the next chunk is loaded into registers a
        // whole chunk ahead and written to LDS at the chunk boundary, so its vmcnt wait (which also drains the
        // wave's rollout-storage stores) is paid once per NCH steps.  NULL noise: the perf-mode counter stream.
        constexpr int CA = NCH * A, CR = (CA + 63) / 64;
        float nreg[NE][CR];
        auto load_eps = [&](int c) {
            size_t idx[NE][CR];
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int n = min(w + 4 * e, NN - 1);
#pragma unroll
                for (int r = 0; r < CR; ++r) {
                    const int i = min(64 * r + l, CA - 1);
                    const int st = min(c * NCH + i / A, T - 1), j = i % A;
                    idx[e][r] = ((size_t)st * NN + n) * A + j;
                }
            }
            if (a.noise) {  // uniform branch: plain loads, consumed a chunk later
#pragma unroll
                for (int e = 0; e < NE; ++e)
#pragma unroll
                    for (int r = 0; r < CR; ++r) nreg[e][r] = a.noise[idx[e][r]];
            } else {
#pragma unroll
                for (int e = 0; e < NE; ++e)
#pragma unroll
                    for (int r = 0; r < CR; ++r) nreg[e][r] = counter_normal(a.seed, idx[e][r]);
            }
        };
        auto store_eps = [&](int cb) {
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int n = w + 4 * e;
                if (n >= NN) break;
#pragma unroll
                for (int r = 0; r < CR; ++r)
                    if (64 * r + l < CA) S.eps[cb][n][64 * r + l] = nreg[e][r];
            }
        };
        load_eps(0);
        store_eps(0);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): preamble loads retired where the compiler sees it
        if (NCH < T) load_eps(1);
        wave_lds_fence_r();
        // this step's noise comes from registers loaded one step ahead (ejn), so no LDS latency sits between the
        // forward and the Gaussian draw; chunk c + 1 is staged at the last step of chunk c for that read.  (Not
        // where the extra registers would spill: two env slots per wave or A > 6 read it in the step.)
        constexpr bool PREF = NE == 1 && A <= 6;
        float ejn[1][A];
#pragma unroll
        for (int j = 0; j < A; ++j) ejn[0][j] = PREF ? S.eps[0][min(w, NN - 1)][j] : 0.f;

        for (int step = 0; step < T; ++step) {
            const int buf = step & 1;
            const int cs = step % NCH;
            if (cs == NCH - 1 && step + 1 < T) {  // chunk (step+1) / NCH (loaded a chunk ago) into LDS; load the next
                store_eps(((step + 1) / NCH) & 1);
                if (step + 1 + NCH < T) load_eps((step + 1) / NCH + 1);
                wave_lds_fence_r();
            }
            // 1 / (count + N) of this step's merge: the counts are known since the last merge, and formed here its
            // fp64 reciprocal and Newton steps interleave with the forward instead of stalling before the barrier
            prep_merge();
            float ejc[A];  // PREF: this step's noise of env slot 0 (from ejn); the next step's goes into ejn
            if constexpr (PREF) {
                const int n = min(w, NN - 1), s1 = step + 1 < T ? step + 1 : step;
#pragma unroll
                for (int j = 0; j < A; ++j) {
                    ejc[j] = ejn[0][j];
                    ejn[0][j] = S.eps[(s1 / NCH) & 1][n][(s1 % NCH) * A + j];
                }
            }
            PGM_STAMP(0);
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int n = w + 4 * e;
                if (n >= NN) break;
                float ej[A];
#pragma unroll
                for (int j = 0; j < A; ++j) ej[j] = PREF ? ejc[j] : S.eps[(step / NCH) & 1][n][cs * A + j];
                float mu[A];
                pol.forward_reg(xr[e], mu, &S.mur[buf][n][0]);
                PGM_STAMP(1);
                // Gaussian draw (torch.normal(mean, std) = eps * std + mean) and clipped action, wave-uniform
                double ac[A], pu[A];
#pragma unroll
                for (int j = 0; j < A; ++j) {
                    const float av = fmaf(ej[j], pol.sd[j], mu[j]);
                    ac[j] = clipd_s((double)av, alo[j], ahi[j]);
                    pu[j] = U[j] * ac[j];
                }
                // dynamics (fp64, lane = feature): s' = tanh(d s + U clip(a) + c)
                const double sn = tanh_d3(dd * s_o[e] + tree_sum(pu) + cc, S.t2);
                PGM_STAMP(6);
                // time limit, auto-reset; the objective side's inputs (s', |a|^2, done) to the parity rows
                const int el = elapsed[e] + 1;
                const int dn = el >= maxs;
                const int bf = dn && el == maxs;
                elapsed[e] = dn ? 0 : el;
                s_o[e] = dn ? s0_o[e] : sn;
                if (role == 0) S.sr[buf][n][l] = s_o[e];  // lanes O.. of the row belong to the objective waves
                S.sn[buf][n][l] = sn;
                if (l == 0) S.dn[buf][n] = dn | bf << 1;
                if (e == 0) PGM_STAMP(2);
            }
            lds_sync();
            PGM_STAMP(3);
            // every statistic of the row: ob_rms (lanes < O, this step's states) and, for the objective waves, obj_rms /
            // ret_rms (their accumulators of the previous step; nothing in step 0's row).  The chain waves execute all
            // 64 lanes of the merge anyway; the objective waves read the reciprocal std from S.rinv a barrier later.
            merge(buf, role == 0 || step > 0);
            PGM_STAMP(4);
            // ---- normalised fp32 obs: the next input and the rollout buffer
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int n = w + 4 * e;
                if (n >= NN) break;
                double v = s_o[e];
                if (nc.use_ob) v = clipd_s((v - mean) * inv, -nc.clipob, nc.clipob);
                const float f = (float)v;  // VecPyTorch .float() (envs.py:192)
                xr[e] = f;
                store_lane(r_obs, role == 0 ? (uint32_t)(((size_t)(step + 1) * NN + n) * O + l) * 4 : OOB_OFF, f);
            }
            if (w == 0) S.rinv[buf][l] = inv;  // read after the next barrier (off this wave's chain)
            PGM_STAMP(5);
        }
        // drain: the last step's objective / ret accumulators (row T & 1), then one more barrier for their reward
        prep_merge();  // (the counts after step T - 1's merge)
        lds_sync();
        merge(T & 1, role == 1 || role == 2);
        if (w == 0) S.rinv[T & 1][l] = inv;
        lds_sync();
        // ---- env state and observation statistics back to HBM
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int n = w + 4 * e;
            if (n >= NN) break;
            if (fl) a.st.s[((size_t)p * NN + n) * O + l] = s_o[e];
            if (l == 0) a.st.elapsed[p * NN + n] = elapsed[e];
        }
        if (w == 0) {
            if (role == 0) {
                a.ns.ob_mean[(size_t)p * O + l] = mean;
                a.ns.ob_var[(size_t)p * O + l] = var;
                if (l == 0) a.ns.ob_count[p] = cnt;
            } else if (role == 1) {
                a.ns.obj_mean[p * K + ko] = mean;
                a.ns.obj_var[p * K + ko] = var;
                if (ko == 0) a.ns.obj_count[p] = cnt;
            } else if (role == 2) {
                a.ns.ret_mean[p] = mean;
                a.ns.ret_var[p] = var;
                a.ns.ret_count[p] = cnt;
            }
        }
    } else {
        // =========================================================== objective waves
        float* rew = a.rb.rewards + (size_t)p * T * NN * K;
        const auto r_rew = out_rsrc(rew, (size_t)T * NN * K * 4);
        const auto r_act = out_rsrc(a.rb.actions + (size_t)p * T * NN * A, (size_t)T * NN * A * 4);
        const auto r_logp = out_rsrc(a.rb.logp + (size_t)p * T * NN, (size_t)T * NN * 4);
        const auto r_msk = out_rsrc(masks, (size_t)(T + 1) * NN * 4);
        const auto r_bad = out_rsrc(bad, (size_t)(T + 1) * NN * 4);
        // the action side: the policy's per-action constants as the chain's ActorLane holds them
        float bm[A], ls[A], sd[A], rsd[A];
        double alo[A], ahi[A];
        {
            const float* prm = a.params + (size_t)p * L.total;
#pragma unroll
            for (int j = 0; j < A; ++j) {
                bm[j] = prm[L.off[PGM_P_MEAN_B] + j];
                ls[j] = prm[L.off[PGM_P_LOGSTD] + j];
                sd[j] = expf(ls[j]);
                rsd[j] = 1.0f / sd[j];
                alo[j] = a.spec.act_lo[j];
                ahi[j] = a.spec.act_hi[j];
                asm volatile("" : "+v"(bm[j]), "+v"(ls[j]), "+v"(sd[j]), "+v"(rsd[j]));
                asm volatile("" : "+v"(alo[j]), "+v"(ahi[j]));
            }
        }
        double V[K], ebase[K], ecoef[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            V[k] = fl ? a.spec.V[k * O + lo] : 0.0;
            ebase[k] = a.spec.ebase[k];
            ecoef[k] = a.spec.ecoef[k];
            asm volatile("" : "+v"(ebase[k]));
            asm volatile("" : "+v"(ecoef[k]));
        }
        double objacc[NE][K], ret[NE], objraw[NE][K], objprev[NE][K];
        int dprev[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int n = min(w + 4 * e, NN - 1);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                objacc[e][k] = a.st.obj_acc[((size_t)p * NN + n) * K + k];
                objraw[e][k] = 0.0;
                objprev[e][k] = 0.0;
            }
            ret[e] = a.st.ret[p * NN + n];
            dprev[e] = 0;
        }
        int obj_valid = a.st.obj_acc_valid[p];
        // wave-uniform constants of the step loop in VGPRs: as SGPRs they are spilled (the NormCfg tuple) and reloaded by
        // v_readlane every step
        double clip_lo = -nc.cliprew, clip_hi = nc.cliprew, gam = nc.gamma;
        asm volatile("" : "+v"(clip_lo), "+v"(clip_hi), "+v"(gam));
        const bool scale_out = nc.use_obj != 0;
        // reward of step ts (role-1 lanes) from its raw objectives and the reciprocal std after the merge of its
        // accumulators: clip(obj / sqrt(var + eps))
        auto emit_reward = [&](int n, int ts, const double (&raw)[K], double rinv) {
            double r = sel_lane_d(raw, ko);
            if (scale_out) r = clipd_s(r * rinv, clip_lo, clip_hi);
            store_lane(r_rew, role == 1 ? (uint32_t)((((size_t)ts * NN + n) * K + ko) * 4) : OOB_OFF, (float)r);
        };
        // the statistics row lanes of roles 1 / 2 for the chain's merge after barrier t + 1 (step t's
        // accumulators); the first row (step 0's barrier) carries nothing for them.  That merge's reciprocal std
        // reaches S.rinv before barrier t + 2, so step t's reward leaves two steps behind.
        for (int step = 0; step < T; ++step) {
            const int buf = step & 1;
            lds_sync();
            const double rinv = S.rinv[buf ^ 1][l];  // the chain's merge after barrier step - 1
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const int n = w + 4 * e;
                if (n >= NN) break;
                if (step > 1) emit_reward(n, step - 2, objprev[e], rinv);
#pragma unroll
                for (int k = 0; k < K; ++k) objprev[e][k] = objraw[e][k];
                // objective side of step t: reset by done_{t-1}, raw objectives (wave sums), discounted
                // accumulators (vec_normalize.py:32-45), the row of step t + 1
                if (dprev[e]) {
#pragma unroll
                    for (int k = 0; k < K; ++k) objacc[e][k] = 0.0;
                    ret[e] = 0.0;
                }
                const double sn = S.sn[buf][n][l];
                const int dnb = S.dn[buf][n];
                double e2;
                {
                    // the chain's Gaussian draw again (same fp32 operations on the same mean and noise), the log-prob,
                    // |clip(a)|^2 and the action / log-prob / mask stores of step `step`
                    constexpr int lane_of[4] = {0, 32, 16, 48};
                    float lpt[A], avs[A];
                    double sq[A];
#pragma unroll
                    for (int j = 0; j < A; ++j) {
                        const float muj = S.mur[buf][n][(j >> 2) * 64 + lane_of[j & 3]] + bm[j];
                        const float ej = S.eps[(step / NCH) & 1][n][(step % NCH) * A + j];
                        const float av = fmaf(ej, sd[j], muj);
                        const float dz = (av - muj) * rsd[j];
                        lpt[j] = -0.5f * dz * dz - ls[j] - LOG_SQRT_2PI;
                        avs[j] = av;
                        const double ac = clipd_s((double)av, alo[j], ahi[j]);
                        sq[j] = ac * ac;
                    }
                    e2 = tree_sum(sq);
                    const float lp = tree_sum(lpt);
                    store_lane(r_act, l < A ? (uint32_t)(((size_t)step * NN + n) * A + l) * 4 : OOB_OFF, sel_lane(avs, l));
                    store_lane(r_logp, l == 0 ? (uint32_t)((size_t)step * NN + n) * 4 : OOB_OFF, lp);
                    const uint32_t moff = (uint32_t)((size_t)(step + 1) * NN + n) * 4;
                    store_lane(r_msk, l == 0 ? moff : OOB_OFF, (dnb & 1) ? 0.f : 1.f);
                    store_lane(r_bad, l == 0 ? moff : OOB_OFF, (dnb & 2) ? 0.f : 1.f);
                }
                dprev[e] = dnb & 1;
                double ob[K];
#pragma unroll
                for (int k = 0; k < K; ++k) ob[k] = V[k] * sn;
                wave_sum64_d_multi<K>(ob, ob);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    ob[k] += ebase[k] - ecoef[k] * e2;
                    objraw[e][k] = ob[k];
                    objacc[e][k] = obj_valid ? objacc[e][k] * gam + ob[k] : ob[k];
                }
                ret[e] = ret[e] * gam + 0.0;  // SynthMO's scalar reward is 0 (vec_normalize.py:32)
                const double rv = role == 1 ? sel_lane_d(objacc[e], ko) : role == 2 ? ret[e] : 0.0;
                if (role == 1 || role == 2) S.sr[buf ^ 1][n][l] = rv;
            }
            obj_valid = 1;
        }
        // ---- drain: the reward of step T - 2 (barrier T, the chain then merges step T - 1's accumulators), the done
        // reset, the reward of step T - 1 (barrier T + 1)
        lds_sync();
        const double rinv_a = S.rinv[(T - 1) & 1][l];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int n = w + 4 * e;
            if (n >= NN) break;
            if (T > 1) emit_reward(n, T - 2, objprev[e], rinv_a);
        }
        lds_sync();
        const double rinv_b = S.rinv[T & 1][l];
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int n = w + 4 * e;
            if (n >= NN) break;
            emit_reward(n, T - 1, objraw[e], rinv_b);
            if (dprev[e]) {
#pragma unroll
                for (int k = 0; k < K; ++k) objacc[e][k] = 0.0;
                ret[e] = 0.0;
            }
            if (l < K) a.st.obj_acc[((size_t)p * NN + n) * K + l] = sel_lane_d(objacc[e], l);
            if (l == 0) a.st.ret[p * NN + n] = ret[e];
        }
        if (w == 0 && l == 0) a.st.obj_acc_valid[p] = obj_valid;
    }
    PGM_STAMP_FLUSH;
}
// ------------------------------------------------------------------------------------------ critic values
// values[p][i][:] = critic(obs[p][i]) for all (T+1) x N stored rows of a task (get_value on every step's
// obs, model.py:71-73, and the bootstrap value on obs[T]).  One thread per row, critic tower in LDS
// (read as wave-wide broadcasts), activations in registers.
struct ValueArgs {
    int R;  // rows per task
    Layout L;
    const float* params;
    const float* obs;  // [P][R][O]
    float* values;     // [P][R][K]
};

template <int O, int K>
struct CriticSmem {
    alignas(16) float W1t[O][H];
    alignas(16) float W2t[H][H];
    alignas(16) float Wv[K][H];
    alignas(16) float b1[H];
    alignas(16) float b2[H];
    float bv[K];
};

template <int O, int K>
__global__ __launch_bounds__(256) void value_kernel(ValueArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<CriticSmem<O, K>*>(smem_raw);
    const int p = blockIdx.y, t = threadIdx.x;
    const Layout& L = a.L;
    const float* prm = a.params + (size_t)p * L.total;
    for (int i = t; i < O * H; i += 256) (&S.W1t[0][0])[i] = prm[L.off[PGM_P_CRITIC_W1] + i];
    for (int i = t; i < H * H; i += 256) (&S.W2t[0][0])[i] = prm[L.off[PGM_P_CRITIC_W2] + i];
    for (int i = t; i < K * H; i += 256) S.Wv[i / H][i % H] = prm[L.off[PGM_P_VALUE_W] + (i % H) * K + i / H];
    if (t < H) {
        S.b1[t] = prm[L.off[PGM_P_CRITIC_B1] + t];
        S.b2[t] = prm[L.off[PGM_P_CRITIC_B2] + t];
    }
    if (t < K) S.bv[t] = prm[L.off[PGM_P_VALUE_B] + t];
    __syncthreads();
    const int r = blockIdx.x * 256 + t;
    if (r >= a.R) return;
    const float* x = a.obs + ((size_t)p * a.R + r) * O;
    float h1[H];
#pragma unroll
    for (int j = 0; j < H; ++j) h1[j] = S.b1[j];
    for (int k = 0; k < O; ++k) {  // z1 = b1 + sum_k x_k W1t[k][:]
        const float xk = x[k];
#pragma unroll
        for (int j = 0; j < H; j += 4) {
            const float4 wv = *reinterpret_cast<const float4*>(&S.W1t[k][j]);
            h1[j] = fmaf(xk, wv.x, h1[j]);
            h1[j + 1] = fmaf(xk, wv.y, h1[j + 1]);
            h1[j + 2] = fmaf(xk, wv.z, h1[j + 2]);
            h1[j + 3] = fmaf(xk, wv.w, h1[j + 3]);
        }
    }
#pragma unroll
    for (int j = 0; j < H; ++j) h1[j] = tanh_fast(h1[j]);
    float v[K];
#pragma unroll
    for (int q = 0; q < K; ++q) v[q] = S.bv[q];
    for (int j = 0; j < H; j += 4) {  // four output units per pass over h1
        float4 z = *reinterpret_cast<const float4*>(&S.b2[j]);
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const float4 wv = *reinterpret_cast<const float4*>(&S.W2t[i][j]);
            z.x = fmaf(h1[i], wv.x, z.x);
            z.y = fmaf(h1[i], wv.y, z.y);
            z.z = fmaf(h1[i], wv.z, z.z);
            z.w = fmaf(h1[i], wv.w, z.w);
        }
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const float4 wq = *reinterpret_cast<const float4*>(&S.Wv[q][j]);
            v[q] = fmaf(tanh_fast(z.x), wq.x, v[q]);
            v[q] = fmaf(tanh_fast(z.y), wq.y, v[q]);
            v[q] = fmaf(tanh_fast(z.z), wq.z, v[q]);
            v[q] = fmaf(tanh_fast(z.w), wq.w, v[q]);
        }
    }
#pragma unroll
    for (int q = 0; q < K; ++q) a.values[((size_t)p * a.R + r) * K + q] = v[q];
}

// The same values on the f32 matrix cores (O <= 32), persistent: grid (CUs / P, P), each workgroup stages its
// task's critic tower in LDS ONCE and its 4 waves loop over 32-row tiles (samples on the MFMA accumulator rows, as
// in the update kernel's forward), the next tile's observation rows prefetched into registers during the current
// one.  Layer 1 from a per-wave LDS copy of the tile's rows, layer 2 through a [32][65] transpose tile, the K value
// outputs on the VALU (lane = sample, half h = units 32h..32h+31).  fp32 and tanh_fast as value_kernel, a different
// summation order (81 vs 84 us per Walker P = 40 launch against value_kernel, which Humanoid keeps).
template <int O, int K>
struct CriticMSmem {
    static constexpr int XS = O | 1;  // odd row stride: the tile's column reads are conflict-free
    float W1t[O][H];
    float W2t[H][H];
    float Wv[K][H];
    float b1[H], b2[H], bv[K];
    float x[4][32 * XS];
    float scr[4][32 * SCR];
};

template <int O, int K>
__global__ __launch_bounds__(256) void value_mfma_kernel(ValueArgs a) {
    static_assert(O <= 32, "one 32-input block");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    using Sm = CriticMSmem<O, K>;
    constexpr int XS = Sm::XS, KS1 = (O + 1) / 2, XL = (32 * O + 63) / 64;  // floats per lane of a tile's rows
    auto& S = *reinterpret_cast<Sm*>(smem_raw);
    const int p = blockIdx.y, t = threadIdx.x, w = t >> 6, l = t & 63, h = l >> 5, c = l & 31;
    const Layout& L = a.L;
    const float* prm = a.params + (size_t)p * L.total;
    for (int i = t; i < O * H; i += 256) (&S.W1t[0][0])[i] = prm[L.off[PGM_P_CRITIC_W1] + i];
    for (int i = t; i < H * H; i += 256) (&S.W2t[0][0])[i] = prm[L.off[PGM_P_CRITIC_W2] + i];
    for (int i = t; i < K * H; i += 256) S.Wv[i / H][i % H] = prm[L.off[PGM_P_VALUE_W] + (i % H) * K + i / H];
    if (t < H) {
        S.b1[t] = prm[L.off[PGM_P_CRITIC_B1] + t];
        S.b2[t] = prm[L.off[PGM_P_CRITIC_B2] + t];
    }
    if (t < K) S.bv[t] = prm[L.off[PGM_P_VALUE_B] + t];
    const int ntile = (a.R + 31) / 32, stride = gridDim.x * 4;
    const float* xg = a.obs + (size_t)p * a.R * O;
    float xr[XL];  // this lane's share of a tile's rows (contiguous in HBM), rows past R as zeros
    auto load_tile = [&](int tile) {
        const int nv = tile < ntile ? min(32, a.R - tile * 32) * O : 0;
#pragma unroll
        for (int j = 0; j < XL; ++j) {
            const int i = l + 64 * j;
            xr[j] = i < nv ? xg[(size_t)tile * 32 * O + i] : 0.f;
        }
    };
    int tile = blockIdx.x * 4 + w;
    load_tile(tile);
    __syncthreads();
    float* xs = S.x[w];
    float* scr = S.scr[w];
    for (; tile < ntile; tile += stride) {
#pragma unroll
        for (int j = 0; j < XL; ++j) {
            const int i = l + 64 * j;
            if (i < 32 * O) xs[(i / O) * XS + (i % O)] = xr[j];
        }
        wave_lds_fence();
        load_tile(tile + stride);  // next tile's rows in flight during this one
        f32x16 z[2] = {f32x16{0}, f32x16{0}};
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
            const int k = 2 * ks + h;
            const float av = k < O ? xs[c * XS + k] : 0.f;
#pragma unroll
            for (int hb = 0; hb < 2; ++hb) z[hb] = mfma(av, k < O ? S.W1t[k < O ? k : 0][hb * TS + c] : 0.f, z[hb]);
        }
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
            const float bias = S.b1[hb * TS + c];
#pragma unroll
            for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + hb * TS + c] = tanh_fast(z[hb][r] + bias);
        }
        wave_lds_fence();
        z[0] = z[1] = f32x16{0};
#pragma unroll 16
        for (int ks = 0; ks < H / 2; ++ks) {
            const int k = 2 * ks + h;
            const float av = scr[c * SCR + k];
#pragma unroll
            for (int ob = 0; ob < 2; ++ob) z[ob] = mfma(av, S.W2t[k][ob * TS + c], z[ob]);
        }
        f32x16 h2[2];
#pragma unroll
        for (int ob = 0; ob < 2; ++ob) {
            const float bias = S.b2[ob * TS + c];
#pragma unroll
            for (int r = 0; r < 16; ++r) h2[ob][r] = tanh_fast(z[ob][r] + bias);
        }
        wave_lds_fence();  // every lane finished reading the H1 tile
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
            for (int r = 0; r < 16; ++r) scr[rowof(r, h) * SCR + ob * TS + c] = h2[ob][r];
        wave_lds_fence();
        float v[K];
#pragma unroll
        for (int q = 0; q < K; ++q) v[q] = 0.f;
#pragma unroll 8
        for (int u = 0; u < TS; ++u) {
            const float hv = scr[c * SCR + h * TS + u];
#pragma unroll
            for (int q = 0; q < K; ++q) v[q] = fmaf(hv, S.Wv[q][h * TS + u], v[q]);
        }
        const int r = tile * 32 + c;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const float vq = half_sum(v[q]) + S.bv[q];
            if (h == 0 && r < a.R) a.values[((size_t)p * a.R + r) * K + q] = vq;
        }
        wave_lds_fence();  // the head's tile reads done before the next tile's x / scr writes
    }
}

// ------------------------------------------------------------------------------------------ evaluation
template <int O>
struct EvalSmem {
    double epi[64][4];  // per-episode objective sums
};
constexpr int EVAL_MAX_WAVES = 8, EVAL_MAX_EPISODES = 64;

template <int O, int A, int K>
__global__ __launch_bounds__(64 * EVAL_MAX_WAVES) void eval_wave_kernel(EvalArgs a) {
    static_assert(K <= 4, "epi rows hold 4 objectives");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    auto& S = *reinterpret_cast<EvalSmem<O>*>(smem_raw);
    const int p = blockIdx.x, l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const float* prm = a.params + (size_t)p * a.L.total;
    ActorLane<O, A> pol;
    pol.load(prm, a.L, l);
    EnvLane<O, A, K> env;
    env.load(a.spec, l);
    const bool fl = l < O;
    const int lo = fl ? l : 0;
    // mopg.py:37-38: fp64 normalisation with the snapshot ob_rms, fixed eps 1e-8 / clip 10, no fp32 round
    const double mean = a.use_ob ? a.ob_mean[(size_t)p * O + lo] : 0.0;
    const double inv = a.use_ob ? 1.0 / sqrt(a.ob_var[(size_t)p * O + lo] + 1e-8) : 1.0;
    const int maxs = a.spec.max_episode_steps;
    for (int ep = w; ep < a.eval_num; ep += nw) {
        double s = a.s0_eval[(size_t)ep * O + lo];
        double acc[K], g = 1.0;
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = 0.0;
        for (int st = 0; st < maxs; ++st) {  // SynthMO episodes end at the time limit
            float mu[A];
            double v = s;  // (lanes >= O: ignored by the broadcast)
            if (a.use_ob) v = clipd((v - mean) * inv, -10.0, 10.0);
            pol.forward_reg((float)v, mu);
            double ac[A], sq[A];
#pragma unroll
            for (int j = 0; j < A; ++j) {  // deterministic action = mean, clipped by the env
                ac[j] = clipd((double)mu[j], env.lo[j], env.hi[j]);
                sq[j] = ac[j] * ac[j];
            }
            const double e2 = tree_sum(sq);
            double objraw[K];
            s = env.step(s, ac, e2, objraw);
#pragma unroll
            for (int k = 0; k < K; ++k) acc[k] += g * objraw[k];
            if (!a.raw) g *= a.gamma;
        }
        if (l < K) S.epi[ep][l] = sel_lane_d(acc, l);
    }
    __syncthreads();
    if (threadIdx.x < K) {  // objs /= eval_num, episodes summed in order
        double sum = 0.0;
        for (int ep = 0; ep < a.eval_num; ++ep) sum += S.epi[ep][threadIdx.x];
        a.objs[(size_t)p * K + threadIdx.x] = sum / (double)a.eval_num;
    }
}

// ------------------------------------------------------------------------------------------ launchers
template <class Kern, class Args>
static int launch_k(Kern k, dim3 grid, dim3 block, size_t smem, hipStream_t s, const Args& args, const char* what) {
    if (smem > 160 * 1024) {
        set_error("%s: LDS image %zu bytes exceeds 160 KiB", what, smem);
        return PGM_E_UNSUPPORTED;
    }
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return hip_fail(e, what);
    hipLaunchKernelGGL(k, grid, block, smem, s, args);
    return launch_status(what);
}

static bool lanes_dims(int O, int K) { return O <= 48 && O + K + 1 <= 64; }

bool rollout_lanes_supported(const pgm_dims* d) {
    return lanes_dims(d->O, d->K) && (d->N == 1 || d->N == 2 || d->N == 4 || d->N == 8);
}

bool eval_waves_supported(const pgm_dims* d, int eval_num) {
    return lanes_dims(d->O, d->K) && d->K <= 4 && eval_num <= EVAL_MAX_EPISODES;
}

template <int O, int A, int K, int NN>
static int launch_rollout_n(const pgm_dims* d, const RolloutArgs& a, hipStream_t s) {
    constexpr int NW = NN < 4 ? NN : 4;
    if (int rc = launch_k(rollout_lane_kernel<O, A, K, NN>, dim3(d->P), dim3(2 * 64 * NW), sizeof(LaneSmem<O, A, NN>), s,
                          a, "pgm_rollout"))
        return rc;
    return launch_critic_values(d, a, s);
}

int launch_critic_values(const pgm_dims* d, const RolloutArgs& a, hipStream_t s) {
    return dispatch_dims(d->O, d->A, d->K, "pgm_rollout (critic values)", [&](auto o, auto, auto k) -> int {
        constexpr int O = decltype(o)::value, K = decltype(k)::value;
        const int R = (d->T + 1) * d->N;
        ValueArgs va{R, a.L, a.params, a.rb.obs, a.rb.values};
        if constexpr (O <= 32) {
            // persistent workgroups: two per CU over the tasks (>= 1 per task; two waves per SIMD hide the dependent
            // 32x32 MFMA chains of one tile), at most one per 4 tiles
            const int wg = max(1, min(2 * device_cu_count() / d->P, (R + 127) / 128));
            return launch_k(value_mfma_kernel<O, K>, dim3(wg, d->P), dim3(256), sizeof(CriticMSmem<O, K>), s, va,
                            "pgm_rollout (critic values)");
        }
        return launch_k(value_kernel<O, K>, dim3((R + 255) / 256, d->P), dim3(256), sizeof(CriticSmem<O, K>), s, va,
                        "pgm_rollout (critic values)");
    });
}

int launch_rollout_lanes(const pgm_dims* d, const RolloutArgs& a, hipStream_t stream) {
    return dispatch_dims(d->O, d->A, d->K, "pgm_rollout", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (!lanes_fit<O, K>()) {
            set_error("pgm_rollout: obs_dim %d outside the lane kernel", O);
            return PGM_E_UNSUPPORTED;
        } else {
            switch (d->N) {
                case 1: return launch_rollout_n<O, A, K, 1>(d, a, stream);
                case 2: return launch_rollout_n<O, A, K, 2>(d, a, stream);
                case 4: return launch_rollout_n<O, A, K, 4>(d, a, stream);
                case 8: return launch_rollout_n<O, A, K, 8>(d, a, stream);
            }
            set_error("pgm_rollout: N=%d outside the lane kernel (1, 2, 4, 8)", d->N);
            return PGM_E_UNSUPPORTED;
        }
    });
}

int launch_eval_waves(const pgm_dims* d, const EvalArgs& a, hipStream_t stream) {
    return dispatch_dims(d->O, d->A, d->K, "pgm_eval", [&](auto o, auto aa, auto k) -> int {
        constexpr int O = decltype(o)::value, A = decltype(aa)::value, K = decltype(k)::value;
        if constexpr (!lanes_fit<O, K>() || K > 4) {
            set_error("pgm_eval: dims outside the wave kernel");
            return PGM_E_UNSUPPORTED;
        } else {
            const int nw = a.eval_num < EVAL_MAX_WAVES ? a.eval_num : EVAL_MAX_WAVES;
            return launch_k(eval_wave_kernel<O, A, K>, dim3(d->P), dim3(64 * nw), sizeof(EvalSmem<O>), stream, a,
                            "pgm_eval");
        }
    });
}

}  // namespace pgm
