// Diagnostic probe (not part of libpgm): accuracy of the gfx950 fp64 reciprocal / reciprocal-square-root
// estimates (v_rcp_f64, v_rsq_f64) with 0, 1 and 2 Newton steps, against the IEEE divide / sqrt, over the
// argument ranges the rollout uses (1 / (e + 1) with e = exp(2|y|) in [1, e^40]; 1 / sqrt(var + eps), var in
// [1e-8, 1e4]).  Prints the max relative error of each form in ulps of 2^-52.
//   hipcc -O3 --offload-arch=gfx950 tests/hip/f64_rcp_rsq_probe.hip -o /tmp/f64probe && /tmp/f64probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

__global__ void probe(int n, double* err) {  // err[form] = max relative error (atomics by max over bit patterns)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double u = (i + 0.5) / n;
    // rcp: x in [2, 1 + e^40] log-uniform
    const double x = 1.0 + exp(u * 40.0 + 0.693);
    const double q = 1.0 / x;  // IEEE
    double r0 = __builtin_amdgcn_rcp(x);
    double r1 = fma(r0, fma(-x, r0, 1.0), r0);
    double r2 = fma(r1, fma(-x, r1, 1.0), r1);
    // rsq: y in [1e-8, 1e4] log-uniform
    const double y = exp(log(1e-8) + u * (log(1e4) - log(1e-8)));
    const double s = 1.0 / sqrt(y);
    double s0 = __builtin_amdgcn_rsq(y);
    double e = fma(-y * s0, s0, 1.0);
    double s1 = fma(s0 * e, 0.5, s0);
    e = fma(-y * s1, s1, 1.0);
    double s2 = fma(s1 * e, 0.5, s1);
    const double v[6] = {fabs(r0 - q) / q, fabs(r1 - q) / q, fabs(r2 - q) / q,
                         fabs(s0 - s) / s, fabs(s1 - s) / s, fabs(s2 - s) / s};
    for (int f = 0; f < 6; ++f) {
        unsigned long long* p = reinterpret_cast<unsigned long long*>(err + f);
        atomicMax(p, (unsigned long long)__double_as_longlong(v[f]));  // non-negative doubles order as integers
    }
}

int main() {
    const int n = 1 << 24;
    double* d;
    hipMalloc(&d, 6 * sizeof(double));
    hipMemset(d, 0, 6 * sizeof(double));
    probe<<<n / 256, 256>>>(n, d);
    double h[6];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[6] = {"rcp", "rcp+1N", "rcp+2N", "rsq", "rsq+1N", "rsq+2N"};
    for (int f = 0; f < 6; ++f) printf("%-8s max rel err %.3e = %.2f ulp(2^-52)\n", names[f], h[f], h[f] / ldexp(1.0, -52));
    return 0;
}
