// Microbenchmark: the pyramid front end of one side of a 1080p x 32 batch -- k_front (gray + pad +
// level 1), k_front's level mode (levels 2+), k_gray_pad alone, and a plain copy of the level 0-1
// bytes as the ceiling.  (Round 2 measured the superseded k_gray_pad + per-level k_pyrdown path
// here at 107 + 42 us against 44 + 32 us; k_pyrdown has since been removed.)
// hipcc --offload-arch=gfx950 -O3 -I../../include -I../../motion_detection_amd/csrc front_bench.hip -o front_bench
#include "../../motion_detection_amd/csrc/mdx_kernels.hip"

#include <stdio.h>
#include <algorithm>
#include <vector>

using namespace mdx;
constexpr int W = 1920, H = 1080, B = 32;

static Geometry geom(int w, int h, int max_level)
{
    Geometry g{};
    int sw = w, sh = h;
    long long img = 0;
    for (int l = 0; l <= max_level; l++) {
        Level& L = g.lv[l];
        L.w = sw; L.h = sh;
        L.pitch = (kXOff + sw + kPad + 16 + 63) / 64 * 64;
        L.rows = kPad + sh + kPad;
        L.img_off = img;
        img += (long long)L.pitch * L.rows;
        g.nlev = l + 1;
        sw = (sw + 1) / 2; sh = (sh + 1) / 2;
        if (sw <= kWin || sh <= kWin) break;
    }
    g.img_bytes = (img + 255) / 256 * 256;
    return g;
}

__global__ void k_copy(const uint4* a, uint4* b, size_t n16)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

template <typename F>
static float timeit(F f, int reps = 20)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int i = 0; i < 3; i++) f();
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; i++) f();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / reps;
}

int main()
{
    Geometry g = geom(W, H, 5);
    uint8_t *in, *pyr;
    const size_t fb = (size_t)W * H;
    hipMalloc(&in, fb * B);
    hipMalloc(&pyr, g.img_bytes * B);
    std::vector<uint8_t> h(fb * B);
    uint32_t x = 12345;
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = x >> 24; }
    hipMemcpy(in, h.data(), h.size(), hipMemcpyHostToDevice);
    const size_t bytes = g.img_bytes * B;
    // (parity of these bytes with the oracle: tests/test_pyramid_gpu.py)
    const float us_gp = timeit([&] { launch_gray_pad(0, B, in, in, W, H, W, (long long)fb, 0, pyr, pyr, g, 1); });
    auto new_l01 = [&] { launch_front(0, B, in, in, W, H, W, (long long)fb, 0, pyr, pyr, g, 1); };
    auto new_rest = [&] { launch_pyr_levels(0, B, pyr, pyr, g, 1); };
    const float us_new01 = timeit(new_l01);
    const float us_new_rest = timeit(new_rest);
    const double mb = (double)fb * B + (double)B * (g.lv[0].rows * 16.0 * ((kXOff + W + kPad - 1) / 16) +
                                                     g.lv[1].rows * 16.0 * ((kXOff + g.lv[1].w + kPad - 1) / 16));
    printf("1080p x %d frames (one side), %d levels\n", B, g.nlev);
    printf("levels 0-1: k_front %7.1f us (%.2f TB/s of %.1f MB); level 0 alone (k_gray_pad) %7.1f us\n", us_new01,
           mb / us_new01 * 1e-6, mb * 1e-6, us_gp);
    printf("levels 2+:  k_front level mode %7.1f us\n", us_new_rest);
    uint8_t* cp;
    hipMalloc(&cp, (size_t)mb);
    const size_t n16 = (size_t)(mb / 2) / 16;
    const float us_cp = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (const uint4*)cp, (uint4*)(cp + n16 * 16), n16); });
    printf("copy of the level 0-1 bytes   %8.1f us  %6.2f TB/s\n", us_cp, mb / us_cp * 1e-6);
    return 0;
}
