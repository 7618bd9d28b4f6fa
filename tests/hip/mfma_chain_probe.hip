// Diagnostic probe (not part of libpgm): cycles per v_mfma_f32_32x32x2_f32 for 1, 2, 4 and 8 interleaved
// accumulator chains, one wave per SIMD.  hipcc -O3 --offload-arch=gfx950 mfma_chain_probe.hip -o probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int C>
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* cyc, int iters) {
    f32x16 acc[C];
#pragma unroll
    for (int i = 0; i < C; ++i) acc[i] = f32x16{0};
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 64 / C; ++k)
#pragma unroll
            for (int i = 0; i < C; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < C; ++i) s += acc[i][0] + acc[i][15];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int C>
void run(float* out, unsigned long long* cyc, int iters) {
    hipLaunchKernelGGL(probe<C>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    m /= 256;
    printf("chains %d: %.1f cycles per MFMA\n", C, m / (64.0 * iters));
}

int main() {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&cyc, 256 * 8);
    const int iters = 200;
    run<1>(out, cyc, iters);
    run<1>(out, cyc, iters);
    run<2>(out, cyc, iters);
    run<4>(out, cyc, iters);
    run<8>(out, cyc, iters);
    return 0;
}
