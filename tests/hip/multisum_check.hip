// Standalone device check of wave_sum64_multi's lane mapping (run on the GPU box; exit 0 = ok).
#include <cstdio>
#include <cmath>
#include "../../pgmorl_amd/csrc/pgm_common.hpp"

template <int M>
__global__ void k(const float* in, float* out) {
    float v[M], o[M];
    for (int i = 0; i < M; ++i) v[i] = in[i * 64 + threadIdx.x];
    pgm::wave_sum64_multi<M>(v, o);
    for (int i = 0; i < M; ++i) out[i * 64 + threadIdx.x] = o[i];
}

template <int M>
int run() {
    float h[8 * 64], r[8 * 64];
    for (int i = 0; i < M * 64; ++i) h[i] = (float)((i * 37) % 101) - 50.f;
    float *d_in, *d_out;
    hipMalloc(&d_in, sizeof(h));
    hipMalloc(&d_out, sizeof(h));
    hipMemcpy(d_in, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k<M>, dim3(1), dim3(64), 0, 0, d_in, d_out);
    hipMemcpy(r, d_out, sizeof(r), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < M; ++i) {
        double s = 0;
        for (int l = 0; l < 64; ++l) s += h[i * 64 + l];
        for (int l = 0; l < 64; ++l)
            if (fabs(r[i * 64 + l] - s) > 1e-3) ++bad;
    }
    printf("M=%d bad=%d\n", M, bad);
    hipFree(d_in);
    hipFree(d_out);
    return bad;
}

int main() { return run<1>() + run<2>() + run<3>() + run<4>() + run<6>() + run<8>() ? 1 : 0; }
