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

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ float tanh_f(float x) { return tanhf(x); }

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
// Built only into libpgm_stamps.so (-DPGM_STAMPS): workgroup 0 / thread 0 accumulates s_memtime
// deltas per phase id into pgm_stamp_acc; read back with pgm_debug_stamps().  Never in the shipped .so.
#ifdef PGM_STAMPS
// one accumulator array + reader per translation unit (no relocatable device code)
#define PGM_STAMP_UNIT(name)                                                                          \
    static __device__ unsigned long long pgm_stamp_acc[64];                                           \
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
#define PGM_STAMP_DECL unsigned long long pgm_stamp_last = __builtin_amdgcn_s_memtime();
#define PGM_STAMP(id)                                                            \
    do {                                                                         \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                               \
            unsigned long long now_ = __builtin_amdgcn_s_memtime();              \
            atomicAdd(&pgm_stamp_acc[id], now_ - pgm_stamp_last);              \
            pgm_stamp_last = now_;                                               \
        }                                                                        \
    } while (0)
#else
#define PGM_STAMP_UNIT(name)
#define PGM_STAMP_DECL
#define PGM_STAMP(id) \
    do {              \
    } while (0)
#endif
