// Shared pieces of the f32-MFMA PPO update kernels (pgm_ppo_mfma.hip: obs_dim <= 32, pgm_ppo_wide.hip:
// wider observations).  Tiles of 32 samples; samples on accumulator ROWS, features on COLUMNS:
//     lane l, register r  <->  (sample rowof(r, l>>5), feature l & 31),  rowof(r,h) = (r&3)+8(r>>2)+4h.
#pragma once
#include "pgm_common.hpp"

namespace pgm {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int MT = 256;     // threads: 4 waves
constexpr int TS = 32;      // samples per MFMA tile
constexpr int SCR = H + 1;  // per-wave transpose tile row stride (conflict-free column reads)

template <int A, int K>
constexpr int qmax() { return A > K ? A : K; }
template <int O, int A, int K>
constexpr int row_stride() {
    constexpr int n = O + A + 2 + 2 * K;
    return n <= 16 ? 16 : n <= 32 ? 32 : n <= 64 ? 64 : 128;
}

__device__ __forceinline__ int rowof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void wave_lds_fence() {  // this wave's LDS writes are visible to its own lanes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
// workgroup barrier that leaves in-flight LDS-DMA (vmcnt) alone
__device__ __forceinline__ void lds_sync_m() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// retire this wave's LDS-DMA / loads, then the barrier
__device__ __forceinline__ void dma_sync_m() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// v[l] + v[l ^ 32] in every lane: one v_permlane32_swap (VALU, no LDS round trip); the sum is
// commutative, so both halves get bit-identical results
__device__ __forceinline__ float half_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// 16x16x4 f32 MFMA: C/D lane l, register r <-> (row 4(l >> 4) + r, column l & 15); A: lane l holds
// A[i = l & 15][k = l >> 4]; B: lane l holds B[k = l >> 4][j = l & 15]
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// sum over the four 16-lane groups (lanes c, c + 16, c + 32, c + 48), result in all of them
__device__ __forceinline__ float group4_sum(float v) {
    v = half_sum(v);                   // l ^ 32 (v_permlane32_swap)
    return v + __shfl_xor(v, 16, 64);  // l ^ 16
}

// torch.min(a,b) / torch.max(a,b) backward weights for the first argument (ties split the gradient in half)
__device__ __forceinline__ float wmin2(float a, float b) { return a < b ? 1.f : (a == b ? 0.5f : 0.f); }
__device__ __forceinline__ float wmax2(float a, float b) { return a > b ? 1.f : (a == b ? 0.5f : 0.f); }

typedef float f2v __attribute__((ext_vector_type(2)));

// Elementwise tile math on register PAIRS through the packed fp32 ALU (v_pk_add / v_pk_mul / v_pk_fma_f32); per
// element the same operations as tanh_fast / the scalar tanh' product.
template <int N, typename V>
__device__ __forceinline__ void tanh_bias_pk(const V& z, float bias, V& out) {
#pragma unroll
    for (int r = 0; r < N; r += 2) {
        const f2v x = f2v{z[r], z[r + 1]} + f2v{bias, bias};
        const f2v y = x * f2v{2.8853900817779268f, 2.8853900817779268f};
        const f2v e = f2v{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
        const f2v d = e + f2v{1.f, 1.f};
        const f2v rc = f2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
        const f2v o = __builtin_elementwise_fma(f2v{-2.f, -2.f}, rc, f2v{1.f, 1.f});
        out[r] = o.x;
        out[r + 1] = o.y;
    }
}
// out = z * (1 - a * a) (tanh' chain rule), pairs
template <int N, typename V>
__device__ __forceinline__ void dtanh_pk(const V& z, const V& a, V& out) {
#pragma unroll
    for (int r = 0; r < N; r += 2) {
        const f2v av = f2v{a[r], a[r + 1]};
        const f2v o = f2v{z[r], z[r + 1]} * __builtin_elementwise_fma(-av, av, f2v{1.f, 1.f});
        out[r] = o.x;
        out[r + 1] = o.y;
    }
}

}  // namespace pgm
