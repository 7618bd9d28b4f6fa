// Probe of the gfx950 f32 MFMA operand / accumulator layouts used by the PPO update kernel.
// Exact small-integer data, asymmetric A and B; prints OK/FAIL.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O2 tests/hip/mfma_layout_probe.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// D[32x32] = A[32xK] * B[Kx32] with K = 2*KS: lane l feeds A[l&31][2s + (l>>5)], B[2s + (l>>5)][l&31]
__global__ void mm32(const float* A, const float* B, float* D, int KS) {
    const int l = threadIdx.x;
    f32x16 acc = {0};
    for (int s = 0; s < KS; ++s) {
        const float a = A[(l & 31) * (2 * KS) + 2 * s + (l >> 5)];
        const float b = B[(2 * s + (l >> 5)) * 32 + (l & 31)];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        D[row * 32 + (l & 31)] = acc[r];
    }
}

// "accumulator as operand": W^T = X^T Y where X, Y are [32 x 32] tiles held in C layout (rows in
// registers): feeding register r of X as A and register r of Y as B sums over the row index.
__global__ void xty(const float* X, const float* Y, float* D) {
    const int l = threadIdx.x;
    f32x16 xr, yr;
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        xr[r] = X[row * 32 + (l & 31)];
        yr[r] = Y[row * 32 + (l & 31)];
    }
    f32x16 acc = {0};
    for (int r = 0; r < 16; ++r) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[r], yr[r], acc, 0, 0, 0);
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        D[row * 32 + (l & 31)] = acc[r];
    }
}

// 16x16x4: lane l feeds A[l&15][4s + (l>>4)], B[4s + (l>>4)][l&15]; D reg i -> row (l>>4)*4 + i, col l&15
__global__ void mm16(const float* A, const float* B, float* D, int KS) {
    const int l = threadIdx.x;
    f32x4 acc = {0};
    for (int s = 0; s < KS; ++s) {
        const float a = A[(l & 15) * (4 * KS) + 4 * s + (l >> 4)];
        const float b = B[(4 * s + (l >> 4)) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i) D[((l >> 4) * 4 + i) * 16 + (l & 15)] = acc[i];
}

static int check(const char* name, const float* got, const float* want, int n) {
    int bad = 0;
    for (int i = 0; i < n; ++i)
        if (got[i] != want[i]) ++bad;
    printf("%s: %s (%d/%d wrong)\n", name, bad ? "FAIL" : "OK", bad, n);
    return bad;
}

int main() {
    const int KS = 3, Kd = 2 * KS;
    float hA[32 * 6], hB[6 * 32], hD[32 * 32], ref[32 * 32];
    for (int i = 0; i < 32; ++i)
        for (int k = 0; k < Kd; ++k) hA[i * Kd + k] = (float)((i * 7 + k * 3) % 11 - 5);
    for (int k = 0; k < Kd; ++k)
        for (int j = 0; j < 32; ++j) hB[k * 32 + j] = (float)((k * 5 + j * 2 + 1) % 13 - 6);
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            float s = 0;
            for (int k = 0; k < Kd; ++k) s += hA[i * Kd + k] * hB[k * 32 + j];
            ref[i * 32 + j] = s;
        }
    float *dA, *dB, *dD, *dX, *dY;
    hipMalloc(&dA, sizeof(hA));
    hipMalloc(&dB, sizeof(hB));
    hipMalloc(&dD, sizeof(hD));
    hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mm32, dim3(1), dim3(64), 0, 0, dA, dB, dD, KS);
    hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
    int bad = check("32x32x2 A/B/C layout", hD, ref, 1024);

    float hX[1024], hY[1024];
    for (int i = 0; i < 1024; ++i) {
        hX[i] = (float)((i * 7) % 9 - 4);
        hY[i] = (float)((i * 5 + 3) % 7 - 3);
    }
    for (int i = 0; i < 32; ++i)  // (X^T Y)[i][j] = sum_s X[s][i] Y[s][j]
        for (int j = 0; j < 32; ++j) {
            float s = 0;
            for (int r = 0; r < 32; ++r) s += hX[r * 32 + i] * hY[r * 32 + j];
            ref[i * 32 + j] = s;
        }
    hipMalloc(&dX, sizeof(hX));
    hipMalloc(&dY, sizeof(hY));
    hipMemcpy(dX, hX, sizeof(hX), hipMemcpyHostToDevice);
    hipMemcpy(dY, hY, sizeof(hY), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(xty, dim3(1), dim3(64), 0, 0, dX, dY, dD);
    hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
    bad += check("X^T Y from C-layout registers", hD, ref, 1024);

    const int KS16 = 2, K16 = 4 * KS16;
    float a16[16 * 8], b16[8 * 16], d16[256], r16[256];
    for (int i = 0; i < 16; ++i)
        for (int k = 0; k < K16; ++k) a16[i * K16 + k] = (float)((i * 3 + k * 5) % 7 - 3);
    for (int k = 0; k < K16; ++k)
        for (int j = 0; j < 16; ++j) b16[k * 16 + j] = (float)((k * 11 + j) % 5 - 2);
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            float s = 0;
            for (int k = 0; k < K16; ++k) s += a16[i * K16 + k] * b16[k * 16 + j];
            r16[i * 16 + j] = s;
        }
    hipMemcpy(dA, a16, sizeof(a16), hipMemcpyHostToDevice);
    hipMemcpy(dB, b16, sizeof(b16), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mm16, dim3(1), dim3(64), 0, 0, dA, dB, dD, KS16);
    hipMemcpy(d16, dD, sizeof(d16), hipMemcpyDeviceToHost);
    bad += check("16x16x4 A/B/C layout", d16, r16, 256);
    printf(bad ? "PROBE FAIL\n" : "PROBE OK\n");
    return bad ? 1 : 0;
}
