// Latency of the first-4 perspective fit in isolation: the one-lane solve (dev_perspective_fit_s<1>,
// what k_fit ran before round 6's wave form) against dev_perspective_fit_wave, one 64-lane workgroup
// per case, timed inside the kernel with s_memtime (core clock) and the 100 MHz wall clock; the two
// results must be bit-identical.  Timed cases: collinear first-4 points (the bench's typical pick: one
// grid column), a general quadrilateral, a near-identity one; then 4096 more inputs (random quads,
// collinear picks, a repeated point, all-zero destinations, 8K-scale coordinates) compared bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Imotion_detection_amd/csrc \
//        scripts/micro/fit_time.hip -Lmotion_detection_amd/lib -lmdx -Wl,-rpath,$PWD/motion_detection_amd/lib
#include "../../motion_detection_amd/csrc/mdx_kernels.hip"
#include <cstdio>
#include <cstring>
#include <vector>

using namespace mdx;

__global__ __launch_bounds__(64) void k_time(const float* cases, double* out, long long* t, int mode)
{
    __shared__ double fw[kFitWorkDoubles > kFitWaveDoubles ? kFitWorkDoubles : kFitWaveDoubles];
    const float* src = cases + blockIdx.x * 16;
    const float* dst = src + 8;
    float s[8], d[8];
    for (int i = 0; i < 8; i++) { s[i] = src[i]; d[i] = dst[i]; }
    double H[9];
    __syncthreads();
    const long long c0 = clock64(), w0 = wall_clock64();
    if (mode == 0) {
        if (threadIdx.x == 0) dev_perspective_fit_s<1>(s, d, H, fw);
    } else {
        dev_perspective_fit_wave(s, d, H, fw);
    }
    __syncthreads();
    const long long c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) {
        for (int i = 0; i < 9; i++) out[blockIdx.x * 9 + i] = H[i];
        t[blockIdx.x * 2] = c1 - c0;
        t[blockIdx.x * 2 + 1] = w1 - w0;
    }
}

int main()
{
    const int nc = 3;
    float h[nc * 16] = {
        // collinear: one grid column, flow (1.3, -0.7) plus small noise
        30, 40, 30, 50, 30, 60, 30, 70, 31.3f, 39.31f, 31.28f, 49.3f, 31.33f, 59.29f, 31.3f, 69.32f,
        // general quadrilateral
        10, 20, 400, 30, 380, 300, 20, 280, 12.5f, 21.f, 401.f, 33.5f, 379.f, 304.f, 19.f, 283.f,
        // near identity
        0, 0, 100, 0, 100, 100, 0, 100, 0.1f, 0.05f, 100.2f, -0.1f, 99.9f, 100.1f, 0.05f, 99.8f,
    };
    float* dc;
    double* dout;
    long long* dt;
    hipMalloc(&dc, sizeof h);
    hipMalloc(&dout, nc * 9 * 8 * 2);
    hipMalloc(&dt, nc * 2 * 8 * 2);
    hipMemcpy(dc, h, sizeof h, hipMemcpyHostToDevice);
    double H[2][nc * 9];
    long long T[2][nc * 2];
    for (int rep = 0; rep < 3; rep++)
        for (int mode = 0; mode < 2; mode++) {
            hipLaunchKernelGGL(k_time, dim3(nc), dim3(64), 0, 0, dc, dout + mode * nc * 9, dt + mode * nc * 2, mode);
            hipDeviceSynchronize();
        }
    hipMemcpy(H, dout, sizeof H, hipMemcpyDeviceToHost);
    hipMemcpy(T, dt, sizeof T, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int c = 0; c < nc; c++) {
        const bool same = std::memcmp(&H[0][c * 9], &H[1][c * 9], 9 * 8) == 0;
        bad += !same;
        printf("case %d: one lane %7lld cycles %6.2f us | wave %7lld cycles %6.2f us | bit-identical %s\n", c, T[0][c * 2],
               T[0][c * 2 + 1] / 100.0, T[1][c * 2], T[1][c * 2 + 1] / 100.0, same ? "yes" : "NO");
    }
    // bit-identity over many inputs: random quadrilaterals, collinear picks (one grid column),
    // repeated points, all-zero destinations, large coordinates
    const int nr = 4096;
    std::vector<float> rc(nr * 16);
    uint64_t st = 0x243F6A8885A308D3ull;
    auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (double)(st >> 11) * 0x1p-53; };
    for (int c = 0; c < nr; c++) {
        float* f = &rc[c * 16];
        const int kind = c % 5;
        const double scale = kind == 4 ? 7680.0 : 1920.0;
        for (int i = 0; i < 4; i++) {
            float sx = (float)(10 * (int)(rnd() * scale / 10)), sy = (float)(10 * (int)(rnd() * scale / 10));
            if (kind == 1) { sx = f[0] = (i == 0 ? sx : f[0]); sy = (float)(10 * (int)(rnd() * 100) + 10 * i); }
            if (kind == 2 && i == 3) { sx = f[0]; sy = f[1]; }
            f[2 * i] = sx; f[2 * i + 1] = sy;
            const float dx = sx + (float)(rnd() * 6 - 3), dy = sy + (float)(rnd() * 6 - 3);
            f[8 + 2 * i] = kind == 3 ? 0.f : dx;
            f[8 + 2 * i + 1] = kind == 3 ? 0.f : dy;
        }
    }
    float* drc;
    double *dh0, *dh1;
    long long* dtt;
    hipMalloc(&drc, rc.size() * 4);
    hipMalloc(&dh0, nr * 9 * 8);
    hipMalloc(&dh1, nr * 9 * 8);
    hipMalloc(&dtt, nr * 2 * 8);
    hipMemcpy(drc, rc.data(), rc.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_time, dim3(nr), dim3(64), 0, 0, drc, dh0, dtt, 0);
    hipLaunchKernelGGL(k_time, dim3(nr), dim3(64), 0, 0, drc, dh1, dtt, 1);
    hipDeviceSynchronize();
    std::vector<double> h0(nr * 9), h1(nr * 9);
    hipMemcpy(h0.data(), dh0, nr * 9 * 8, hipMemcpyDeviceToHost);
    hipMemcpy(h1.data(), dh1, nr * 9 * 8, hipMemcpyDeviceToHost);
    int rbad = 0;
    for (int c = 0; c < nr; c++) rbad += std::memcmp(&h0[c * 9], &h1[c * 9], 72) != 0;
    printf("random cases: %d of %d bit-identical (random quads, collinear, repeated point, zero dst, 8K scale)\n",
           nr - rbad, nr);
    return bad + rbad;
}
