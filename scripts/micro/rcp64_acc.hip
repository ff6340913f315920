// Accuracy of v_rcp_f64 over [2^-30, 2^30] and of one quadratic Newton step after it: max relative
// error against IEEE 1/x (from the correctly rounded division), 16M log-uniform samples plus powers
// of two and their neighbours.  Used to size warp_rows_pj's reciprocal refinement.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>
__global__ void k(const double* x, double* e0, double* e1, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i];
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e, r0);
    const double q = 1.0 / d;   // IEEE
    e0[i] = fabs((r0 - q) / q);
    e1[i] = fabs((r1 - q) / q);
}
int main()
{
    const int n = 1 << 24;
    std::vector<double> x(n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < n; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) * 0x1p-53;
        x[i] = std::ldexp(1.0 + u, (int)(s % 61) - 30) * ((s >> 7) & 1 ? -1.0 : 1.0);
    }
    for (int j = 0; j < 64 && j < n; j++) x[j] = std::ldexp(1.0, j - 32);                  // powers of two
    for (int j = 64; j < 128; j++) x[j] = std::nextafter(std::ldexp(1.0, j - 96), 0.0);    // just below them
    double *dx, *de0, *de1;
    hipMalloc(&dx, n * 8); hipMalloc(&de0, n * 8); hipMalloc(&de1, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, de0, de1, n);
    std::vector<double> a(n), b(n);
    hipMemcpy(a.data(), de0, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), de1, n * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0;
    for (int i = 0; i < n; i++) { m0 = std::fmax(m0, a[i]); m1 = std::fmax(m1, b[i]); }
    printf("v_rcp_f64 max rel err %.3e (2^%.2f); after one quadratic Newton step %.3e (2^%.2f); %d samples\n", m0,
           std::log2(m0), m1, m1 > 0 ? std::log2(m1) : -1e9, n);
    return 0;
}
