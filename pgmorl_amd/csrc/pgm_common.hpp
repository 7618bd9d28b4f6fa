// Shared device/host helpers for libpgm (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pgm_abi.h"

namespace pgm {

constexpr int H = 64;        // hidden width (model.py:202,250)
constexpr int H2 = 2 * H;    // critic columns [0,H), actor columns [H,2H) when both towers run together
constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;

// ---------------------------------------------------------------- host-side error plumbing
void set_error(const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);
int launch_status(const char* what);  // hipGetLastError() after a launch

struct Layout {
    int32_t off[PGM_NUM_PARAM_TENSORS];
    int32_t total;
};
Layout make_layout(int O, int A, int K, int Hd);
// pgm_ppo_update workspace: [2 PGM_NS_MAX P + 1] tagged 8-byte granules (tower-norm hand-offs of every
// (task, tower, row part); word 2P = timeout flag), padded to 256 bytes; the gradient exchange of the
// row-split updates, [P][2 towers][PGM_NS_MAX row parts][2 parities] slots of (tower image + 1) granules; then
// the packed sample table [P][T*N][RS] fp32 (obs | action | old logp | adv | old value | return, RS a power
// of 2)
inline int ppo_row_stride(int O, int A, int K) {
    const int n = O + A + 2 + 2 * K;
    return n <= 16 ? 16 : n <= 32 ? 32 : n <= 64 ? 64 : 128;
}
constexpr int ppo_img_floats(int O, int A, int K) {  // TowerImg<O, A, K> of pgm_ppo_mfma.hip
    const int Q = A > K ? A : K;
    return O * H + H * (H + 1) + Q * H + 2 * H + Q + A;
}
constexpr int PGM_NS_MAX = 4;  // workgroups per tower of the row-split updates
// granules: [0, 16 P + 1) the norm granules + timeout word of the MODE 2 / t16 / wide updates, then from 16 P + 8 the
// feature-split update's image / norm / parameter granules ([3][P][2][<= 16 parts][2 parities], pgm_ppo_fs.hip)
inline size_t ppo_flag_bytes(int P) { return ((size_t)(208 * P + 8) * 8 + 255) / 256 * 256; }
// norm granule of (task p, tower m, row part hs, step parity par): (row part 0, parity 0) below the timeout word
// (word 2P), the others above it.  Double-buffered by step parity like the image slots: a workgroup rewrites a
// granule only two steps later, after every reader has matched it, so a delayed poll can never miss its tag.
__host__ __device__ inline int ppo_norm_granule(int P, int p, int m, int hs, int par) {
    const int q = 2 * hs + par;
    return q == 0 ? 2 * p + m : 2 * P + 1 + 2 * P * (q - 1) + 2 * p + m;
}
inline int ppo_xslot(int O, int A, int K) { return (ppo_img_floats(O, A, K) + 1 + 31) / 32 * 32; }  // granules
inline size_t ppo_xbuf_bytes(const pgm_dims* d, int ns = PGM_NS_MAX) {
    return d->O <= 32 ? (size_t)d->P * 2 * ns * 2 * ppo_xslot(d->O, d->A, d->K) * 8 : 0;
}
int wide_xslot_words(int O, int A, int K);  // pgm_ppo_wide.hip: small image + dW1 + flag granule, 8-B words
inline size_t wide_xbuf_bytes(const pgm_dims* d) {
    return (size_t)d->P * 2 * PGM_NS_MAX * 2 * wide_xslot_words(d->O, d->A, d->K) * 8;
}
// the part of the workspace a launch expects zeroed: flags + exchange slots (every mode's, sized for PGM_NS_MAX)
inline size_t ppo_reset_bytes(const pgm_dims* d) {
    return ppo_flag_bytes(d->P) + (d->O > 32 ? wide_xbuf_bytes(d) : ppo_xbuf_bytes(d));
}
// pgm_ppo_update_reset marks a workspace as zeroed (up to n bytes, ordered by the caller's streams); a launch
// needing <= n zeroed bytes consumes the mark instead of issuing its own reset (pgm_ppo_update.hip)
bool ws_take_zeroed(const void* ws, size_t need);
// feature-split update (pgm_ppo_fs.hip): its exchange payload after the sample table (0 when it cannot run)
size_t fs_workspace_extra(const pgm_dims* d);
// obs_dim > 32 (wide kernel): flags, exchange slots [P][2 towers][NS parts][2 parities], every workgroup's
// layer-1 copy in k-quad layout [P][2 towers][NS parts][O H] (sized for PGM_NS_MAX parts)
inline size_t ppo_workspace_bytes(const pgm_dims* d) {
    if (d->O > 32)
        return ppo_flag_bytes(d->P) + wide_xbuf_bytes(d) +
               (size_t)d->P * 2 * PGM_NS_MAX * d->O * d->H * sizeof(float);
    return ppo_flag_bytes(d->P) + ppo_xbuf_bytes(d) +
           (size_t)d->P * d->T * d->N * ppo_row_stride(d->O, d->A, d->K) * sizeof(float) + fs_workspace_extra(d);
}
int device_cu_count();  // CUs of the current device (cached)

// Co-residency precondition of the persistent update kernels (their workgroups spin on each other's tagged
// flags, so every workgroup of the grid must be resident at once): the occupancy query for this kernel,
// block size and LDS must admit grid <= blocks-per-CU x CUs.  PGM_E_UNSUPPORTED (with the numbers) otherwise.
int check_coresident(const void* kern, int block, size_t smem, int grid, const char* what);

// Launch options with NULL = automatic, validated (pgm_abi.h pgm_launch_opts).
int read_opts(const pgm_launch_opts* o, pgm_launch_opts* out, const char* what);
// Row-split cap of opts->update_split: 4 (four per tower), 2, 1 (one per tower), 0 (one per task); 4 when automatic.
inline int split_cap(const pgm_launch_opts& o) {
    switch (o.update_split) {
        case PGM_SPLIT_TASK: return 0;
        case PGM_SPLIT_TOWER: return 1;
        case PGM_SPLIT_HALVES: return 2;
        default: return 4;
    }
}

// Exchange delay of the TEST build only (libpgm_test.so, -DPGM_TEST_HOOKS; the production library returns an inert
// delay and keeps no such hook): PGM_TEST_DELAY="step:block:where:cycles" -- workgroup `block` stalls `cycles` shader
// cycles at hand-off point `where` of Adam step `step` -- 0 before publishing its gradient image, 1 between its image
// flag store and its partner poll, 2 between its tower-norm granule store and its poll, 3 (feature-split) before its
// Adam step.  Provokes the delayed-poll orders the step-parity double buffering must survive.
struct DbgDelay {
    int step, block, where;
    unsigned cycles;
};
DbgDelay dbg_delay_hook();
__device__ __forceinline__ void dbg_delay(const DbgDelay& d, int nstep, int where) {
    if (d.cycles != 0u && nstep == d.step && (int)blockIdx.x == d.block && where == d.where) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < (unsigned long long)d.cycles) __builtin_amdgcn_s_sleep(8);
    }
}

// ---------------------------------------------------------------- device helpers
// Branch-free fp32 tanh (~14 VALU ops, rel. error ~3e-7): odd Taylor series through x^9 for |x| < 0.25
// (truncation < 3e-9), 1 - 2/(exp(2|x|) + 1) above, with the sign restored.  Both branches are always
// evaluated and blended arithmetically (s in {0, 1}: big + (poly - big) is exactly poly, the two being
// within a factor 2) -- a select would be turned into control flow around the exp / rcp, which
// serialises the surrounding MFMA work.  The polynomial argument is clamped so it stays finite.
__device__ __forceinline__ float tanh_f(float x) {
    const float ax = fabsf(x);
    const float xp = __builtin_amdgcn_fmed3f(x, -0.25f, 0.25f);
    const float x2 = xp * xp;
    const float poly = xp * fmaf(x2, fmaf(x2, fmaf(x2, fmaf(x2, 0.021869488536155203f, -0.05396825396825397f),
                                                   0.13333333333333333f), -0.3333333333333333f), 1.0f);
    const float e = __expf(2.0f * ax);
    const float big = copysignf(1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f), x);
    const float s = ax < 0.25f ? 1.0f : 0.0f;
    return fmaf(s, poly - big, big);
}

// 5-instruction fp32 tanh for MFMA-paced tiles: 1 - 2 / (exp(2x) + 1) on the hardware exp2 / rcp.
// Absolute error <= ~2e-7 everywhere (relative error grows below |x| ~ 1e-2, where the absolute one is
// what reaches the next layer); saturates cleanly to +-1 (exp overflow -> rcp(inf) = 0).
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // exp(2x)
    return fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

// xor-butterfly sum over aligned groups of W lanes (W power of two <= 64)
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int m = W / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}
template <int W>
__device__ __forceinline__ double group_sum_d(double v) {
#pragma unroll
    for (int m = W / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// 64-lane sum on the DPP path (no LDS round trip): rotate-add inside each 16-lane row, then add the
// four row totals through readlane.  The result is wave-uniform.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum64(float v) {
    v += dpp_f<0x128>(v);  // row_ror:8
    v += dpp_f<0x124>(v);  // row_ror:4
    v += dpp_f<0x122>(v);  // row_ror:2
    v += dpp_f<0x121>(v);  // row_ror:1
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}

// M <= 8 simultaneous 64-lane sums, results wave-uniform.  Transposing reduction: v_permlane32_swap folds
// lane halves of PAIRS of values (value a in lanes 0-31, b in 32-63 of one register), v_permlane16_swap
// folds rows of pairs of those (4 values, one per 16-lane row), then 4 DPP row rotations finish each
// row and one readlane per value makes it uniform: ~3.5 instructions per value instead of ~12.
__device__ __forceinline__ float pl32_fold(float a, float b) {  // lanes 0-31: a_lo + a_hi, 32-63: b_lo + b_hi
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float pl16_fold(float a, float b) {  // rows (0,1,2,3) <- a r0+r1, b r0+r1, a r2+r3, b r2+r3
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// (update_dpp with bound_ctrl set, every lane a valid source: the DPP combiner folds each into one v_add_f32_dpp)
__device__ __forceinline__ float row_sum16(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, true));  // row_ror:8
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, true));  // row_ror:4
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, true));  // row_ror:2
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, true));  // row_ror:1
    return v;
}
// sum over each 8-lane half of a 16-lane row (the result in every lane of the half): mirror, then two quad swaps
__device__ __forceinline__ float row_sum8(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, true));  // row_half_mirror
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, true));   // quad_perm 1,0,3,2
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, true));   // quad_perm 2,3,0,1
    return v;
}
// rows (optional, 128 floats of LDS): the two reduced rows stored by every lane, so that another wave reads value i at
// rows[(i / 4) * 64 + {0, 32, 16, 48}[i % 4]] without the readlanes
// grow (optional, 8 floats of global memory): value i stored by one lane as an sc1 store at grow[(i / 4) * 4 + {0, 2, 1, 3}[i % 4]]
template <int M>
__device__ __forceinline__ void wave_sum64_multi(const float (&v)[M], float (&out)[M], float* rows = nullptr,
                                                 float* grow = nullptr) {
    static_assert(M >= 1 && M <= 8, "1..8 values");
    auto at = [&](int i) { return i < M ? v[i] : 0.f; };
    const int ln = __lane_id();
    // level 1: pairs (0,1) (2,3) (4,5) (6,7); level 2: (s01, s23) -> rows [v0, v2, v1, v3], (s45, s67) likewise
    // (a pair wholly past M is the constant 0, not a fold of zeros: the compiler does not fold the permlane of 0)
    const float r0 = row_sum16(pl16_fold(pl32_fold(at(0), at(1)), M > 2 ? pl32_fold(at(2), at(3)) : 0.f));
    const int lane_of[4] = {0, 32, 16, 48};  // value i of a group sits in row {0, 2, 1, 3}[i]
#pragma unroll
    for (int i = 0; i < (M < 4 ? M : 4); ++i)
        out[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r0), lane_of[i]));
    if (rows) rows[ln] = r0;
    if (grow && (ln & 15) == 0) __hip_atomic_store(grow + (ln >> 4), r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (M > 4) {
        const float r1 = row_sum16(pl16_fold(pl32_fold(at(4), at(5)), M > 6 ? pl32_fold(at(6), at(7)) : 0.f));
        if (rows) rows[64 + ln] = r1;
        if (grow && (ln & 15) == 0) __hip_atomic_store(grow + 4 + (ln >> 4), r1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 4; i < M; ++i) out[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r1), lane_of[i - 4]));
    }
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                            __builtin_amdgcn_readlane(__double2loint(v), lane));
}
// fp64 64-lane sum, same reduction tree as wave_sum64 (deterministic)
__device__ __forceinline__ double wave_sum64_d(double v) {
    v += dpp_d<0x128>(v);
    v += dpp_d<0x124>(v);
    v += dpp_d<0x122>(v);
    v += dpp_d<0x121>(v);
    return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// ---------------------------------------------------------------- counter RNG (perf mode)
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// standard normal for element i of stream `seed` (Box-Muller on one 64-bit hash)
__device__ __forceinline__ float counter_normal(uint64_t seed, uint64_t i) {
    uint64_t h = splitmix64(splitmix64(seed * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull) ^ i);
    float u1 = ((uint32_t)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);          // (0,1)
    float u2 = (uint32_t)(h & 0xFFFFFFu) * (1.0f / 16777216.0f);             // [0,1)
    return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

}  // namespace pgm

// ---------------------------------------------------------------- diagnostic phase stamps
// Built only into libpgm_stamps.so (-DPGM_STAMPS): every wave accumulates s_memtime deltas per phase id
// (< 24); thread 0 of the sampled workgroup adds its totals to pgm_stamp_acc at the end; read back with pgm_debug_stamps().  Never in the shipped .so.
#ifdef PGM_STAMPS
// one accumulator array + reader per translation unit (no relocatable device code)
#define PGM_STAMP_UNIT(name)                                                                          \
    static __device__ unsigned long long pgm_stamp_acc[64];                                           \
    static __device__ int pgm_stamp_block;                                                            \
    extern "C" int pgm_debug_stamp_block_##name(int b) {                                              \
        return hipMemcpyToSymbol(HIP_SYMBOL(pgm_stamp_block), &b, sizeof(int)) == hipSuccess ? PGM_OK : PGM_E_HIP; \
    }                                                                                                 \
    extern "C" int pgm_debug_stamps_##name(unsigned long long* out, int reset) {                      \
        if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pgm_stamp_acc), sizeof(unsigned long long) * 64) !=  \
            hipSuccess)                                                                               \
            return PGM_E_HIP;                                                                         \
        if (reset) {                                                                                  \
            unsigned long long z[64] = {0};                                                           \
            if (hipMemcpyToSymbol(HIP_SYMBOL(pgm_stamp_acc), z, sizeof(z)) != hipSuccess) return PGM_E_HIP; \
        }                                                                                             \
        return PGM_OK;                                                                                \
    }
// deltas accumulate in registers (no memory traffic inside the measured loop: a global access there would
// add vmcnt waits that drain the kernel's own stores); PGM_STAMP_FLUSH at the kernel's end publishes them
#define PGM_STAMP_DECL                                                           \
    unsigned long long pgm_stamp_last = __builtin_amdgcn_s_memtime();            \
    unsigned long long pgm_stamp_reg[24] = {0};
#define PGM_STAMP(id)                                                            \
    do {                                                                         \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();            \
        pgm_stamp_reg[id] += now_ - pgm_stamp_last;                              \
        pgm_stamp_last = now_;                                                   \
    } while (0)
#define PGM_STAMP_FLUSH                                                          \
    do {                                                                         \
        if ((int)blockIdx.x == pgm_stamp_block && threadIdx.x == 0)              \
            for (int i_ = 0; i_ < 24; ++i_)                                      \
                if (pgm_stamp_reg[i_]) atomicAdd(&pgm_stamp_acc[i_], pgm_stamp_reg[i_]); \
    } while (0)
#else
#define PGM_STAMP_UNIT(name)
#define PGM_STAMP_DECL
#define PGM_STAMP(id) \
    do {              \
    } while (0)
#define PGM_STAMP_FLUSH \
    do {                \
    } while (0)
#endif
