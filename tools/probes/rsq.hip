// Probe: accuracy of v_rsq_f64 + 2 Newton steps vs 1/sqrt over the fp64 exponent range.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
__global__ void k(const double* x, double* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double piv = x[i];
    double r0 = __builtin_amdgcn_rsq(piv);
    double inv = r0 * fma(-0.5 * piv, r0 * r0, 1.5);
    inv = inv * fma(-0.5 * piv, inv * inv, 1.5);
    o[3 * i] = r0; o[3 * i + 1] = inv; o[3 * i + 2] = 1.0 / sqrt(piv);
}
int main() {
    const int n = 4096;
    double hx[n];
    for (int i = 0; i < n; ++i) hx[i] = pow(10.0, -300.0 + 600.0 * i / (n - 1)) * (1.0 + 0.37 * (i % 7));
    double *dx, *dout; hipMalloc(&dx, sizeof(hx)); hipMalloc(&dout, 3 * sizeof(hx));
    hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 64), dim3(64), 0, 0, dx, dout, n);
    static double ho[3 * n]; hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
    double worst0 = 0, worst = 0; int wi = 0;
    for (int i = 0; i < n; ++i) {
        const double ref = 1.0 / std::sqrt(hx[i]);
        const double e0 = std::fabs(ho[3 * i] / ref - 1), e = std::fabs(ho[3 * i + 1] / ref - 1);
        if (!(e0 <= worst0)) worst0 = e0;
        if (!(e <= worst)) { worst = e; wi = i; }
    }
    printf("rsq estimate worst rel err %.3e; refined worst rel err %.3e at x=%.3e (got %.17e ref %.17e)\n", worst0,
           worst, hx[wi], ho[3 * wi + 1], 1.0 / std::sqrt(hx[wi]));
    for (int i = 0; i < n; i += 512) printf("x=%.3e est=%.3e refined=%.3e\n", hx[i], ho[3*i]*std::sqrt(hx[i]) - 1, ho[3*i+1]*std::sqrt(hx[i]) - 1);
    return 0;
}
