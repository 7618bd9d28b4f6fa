// Diagnostic probe (not part of libpgm): cycles per instruction of the rollout chain's instruction kinds on gfx950,
// one wave per SIMD (256 threads per workgroup) or two (512), 16-instruction asm blocks in a counted loop:
// throughput with 4 independent accumulators, latency with one.  hipcc -O3 --offload-arch=gfx950 valu_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

#define FMAC_DPP4                                                                    \
    "v_fmac_f32_dpp %0, %4, %5 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"     \
    "v_fmac_f32_dpp %1, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"     \
    "v_fmac_f32_dpp %2, %4, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"     \
    "v_fmac_f32_dpp %3, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
#define FMAC_DPP1 "v_fmac_f32_dpp %0, %4, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
#define FMAC4 "v_fmac_f32 %0, %4, %5\n\tv_fmac_f32 %1, %4, %5\n\tv_fmac_f32 %2, %4, %5\n\tv_fmac_f32 %3, %4, %5\n\t"
#define FMAC1 "v_fmac_f32 %0, %4, %5\n\t"

template <int V>
__global__ __launch_bounds__(512) void probe_f32(float* out, unsigned long long* cyc, int iters) {
    float a0 = threadIdx.x * 1e-3f, a1 = 0.f, a2 = 0.f, a3 = 0.f, x = 1e-6f * threadIdx.x, w = 0.5f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (V == 0) asm volatile("s_nop 1\n\t" R4(FMAC_DPP4) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 1) asm volatile("s_nop 1\n\t" R16(FMAC_DPP1) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 2) asm volatile(R4(FMAC4) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 3) asm volatile(R16(FMAC1) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        // row sum step: mov_dpp + add vs add_dpp (dependent, 4 per block x 4)
        if constexpr (V == 4)
            asm volatile(R16("v_mov_b32_dpp %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\tv_add_f32 %0, %0, %1\n\t")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 5)
            asm volatile(R16("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 6) asm volatile(R16("v_exp_f32 %0, %0\n\t") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 7)
            asm volatile(R16("v_permlane32_swap_b32 %0, %1\n\t") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 8)
            asm volatile(R16("v_readlane_b32 s0, %0, 5\n\tv_add_f32 %0, s0, %0\n\t")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w) : "s0");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
__global__ __launch_bounds__(512) void probe_f64(double* out, unsigned long long* cyc, int iters) {
    double a0 = threadIdx.x * 1e-3, a1 = 0.0, a2 = 0.0, a3 = 0.0, x = 1.0 + 1e-9 * threadIdx.x, w = 0.5;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (V == 0)
            asm volatile(R4("v_fma_f64 %0, %4, %5, %0\n\tv_fma_f64 %1, %4, %5, %1\n\tv_fma_f64 %2, %4, %5, %2\n\tv_fma_f64 %3, %4, %5, %3\n\t")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 1) asm volatile(R16("v_fma_f64 %0, %4, %5, %0\n\t") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 2) asm volatile(R16("v_rcp_f64 %0, %0\n\t") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 3) asm volatile(R16("v_rsq_f64 %0, %0\n\t") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 4) asm volatile(R16("v_add_f64 %0, %0, %4\n\t") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
        if constexpr (V == 5) asm volatile(R16("v_max_f64 %0, %0, %4\n\t") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(w));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// LDS read -> use latency: a dependent ds_read_b64 chain (address from the loaded value)
__global__ __launch_bounds__(512) void probe_lds(int* out, unsigned long long* cyc, int iters) {
    __shared__ int buf[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) buf[i] = 0;
    __syncthreads();
    int a = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it)
        asm volatile(R16("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\t") : "+v"(a) : : "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(512) void probe_barrier(int* out, unsigned long long* cyc, int iters) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) asm volatile(R16("s_barrier\n\t") ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x] = 0;
}

static double mean_cyc(unsigned long long* cyc) {
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    return m / 256;
}

int main() {
    void* out;
    unsigned long long* cyc;
    hipMalloc(&out, 256 * 512 * 8);
    hipMalloc(&cyc, 256 * 8);
    const int iters = 2000;
    const char* f32n[] = {"v_fmac_f32_dpp row_newbcast, 4 acc (+1 s_nop per 16)", "v_fmac_f32_dpp, 1 acc", "v_fmac_f32, 4 acc",
                          "v_fmac_f32, 1 acc", "mov_dpp + add_f32 (per pair)", "s_nop 1 + v_add_f32_dpp (per pair)",
                          "v_exp_f32 chain", "v_permlane32_swap", "v_readlane + v_add_f32 (per pair)"};
    const char* f64n[] = {"v_fma_f64, 4 acc", "v_fma_f64, 1 acc", "v_rcp_f64 chain", "v_rsq_f64 chain", "v_add_f64 chain",
                          "v_max_f64 chain"};
    for (int th : {256, 512}) {
        printf("== %d threads per workgroup (%d wave(s) per SIMD)\n", th, th / 256);
#define RUN32(V)                                                                                        \
    hipLaunchKernelGGL(probe_f32<V>, dim3(256), dim3(th), 0, 0, (float*)out, cyc, iters);               \
    hipDeviceSynchronize();                                                                             \
    hipLaunchKernelGGL(probe_f32<V>, dim3(256), dim3(th), 0, 0, (float*)out, cyc, iters);               \
    hipDeviceSynchronize();                                                                             \
    printf("  %-48s %6.2f cycles per instruction\n", f32n[V], mean_cyc(cyc) / (16.0 * iters));
        RUN32(0) RUN32(1) RUN32(2) RUN32(3) RUN32(4) RUN32(5) RUN32(6) RUN32(7) RUN32(8)
#define RUN64(V)                                                                                        \
    hipLaunchKernelGGL(probe_f64<V>, dim3(256), dim3(th), 0, 0, (double*)out, cyc, iters);              \
    hipDeviceSynchronize();                                                                             \
    hipLaunchKernelGGL(probe_f64<V>, dim3(256), dim3(th), 0, 0, (double*)out, cyc, iters);              \
    hipDeviceSynchronize();                                                                             \
    printf("  %-48s %6.2f cycles per instruction\n", f64n[V], mean_cyc(cyc) / (16.0 * iters));
        RUN64(0) RUN64(1) RUN64(2) RUN64(3) RUN64(4) RUN64(5)
        hipLaunchKernelGGL(probe_lds, dim3(256), dim3(th), 0, 0, (int*)out, cyc, iters);
        hipDeviceSynchronize();
        printf("  %-48s %6.2f cycles per read\n", "ds_read_b32 -> address chain", mean_cyc(cyc) / (16.0 * iters));
        hipLaunchKernelGGL(probe_barrier, dim3(256), dim3(th), 0, 0, (int*)out, cyc, iters);
        hipDeviceSynchronize();
        printf("  %-48s %6.2f cycles per barrier\n", "s_barrier (all waves arrive together)", mean_cyc(cyc) / (16.0 * iters));
    }
    return 0;
}
