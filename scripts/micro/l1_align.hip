// Microbenchmark: L1-resident per-lane vector loads, aligned vs 4-B-misaligned, by width and
// lane stride.  hipcc --offload-arch=gfx950 -O3 l1_align.hip -o l1_align && ./l1_align
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

struct __attribute__((aligned(4))) u4a4 { uint32_t x, y, z, w; };
struct __attribute__((aligned(4))) u2a4 { uint32_t x, y; };

template <int W>
__global__ __launch_bounds__(64) void k_load(const uint32_t* __restrict__ buf, uint32_t* out, int lane_stride_w,
                                             int shift_w, int iters, int region_w)
{
    const int lane = threadIdx.x;
    const uint32_t* base = buf + (blockIdx.x % 2) * region_w;   // 2 regions: L1-resident (2 x 20 KiB)
    uint32_t acc = 0;
    int row = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t* p = base + row * 256 + lane * lane_stride_w + shift_w;
        if (W == 4) {
            const u4a4 v = *reinterpret_cast<const u4a4*>(p);
            acc ^= v.x + v.y + v.z + v.w;
        } else if (W == 2) {
            const u2a4 v = *reinterpret_cast<const u2a4*>(p);
            acc ^= v.x + v.y;
        } else {
            acc ^= p[0];
        }
        row = (row + 1) & 15;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    const int region_w = 16 * 256 + 1024;   // 16 rows of 1 KiB + slack
    uint32_t *buf, *out;
    hipMalloc(&buf, 64 * region_w * 4 + 65536);
    hipMemset(buf, 1, 64 * region_w * 4 + 65536);
    hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 16, iters = 4096;
    struct Cfg { int w, stride, shift; const char* what; } cfgs[] = {
        {4, 4, 0, "x4 contiguous aligned"},  {4, 4, 1, "x4 contiguous +4B"},
        {4, 1, 0, "x4 stride 4B (quad overlap)"}, {4, 1, 1, "x4 stride 4B +4B"},
        {4, 10, 0, "x4 stride 40B (aligned/mis mix)"}, {4, 3, 0, "x4 stride 12B"},
        {2, 2, 0, "x2 contiguous aligned"},  {2, 2, 1, "x2 contiguous +4B"},
        {1, 1, 0, "x1 contiguous"},
    };
    for (auto& c : cfgs) {
        float best = 1e9;
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            if (c.w == 4) hipLaunchKernelGGL(k_load<4>, dim3(blocks), dim3(64), 0, 0, buf, out, c.stride, c.shift, iters, region_w);
            if (c.w == 2) hipLaunchKernelGGL(k_load<2>, dim3(blocks), dim3(64), 0, 0, buf, out, c.stride, c.shift, iters, region_w);
            if (c.w == 1) hipLaunchKernelGGL(k_load<1>, dim3(blocks), dim3(64), 0, 0, buf, out, c.stride, c.shift, iters, region_w);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double winstr = (double)blocks * iters;
        const double bytes = winstr * 64 * 4 * c.w;
        printf("%-34s %8.3f ms  %7.2f TB/s lane-bytes  %6.2f clk/wave-instr/CU (2.4GHz)\n", c.what, best,
               bytes / best / 1e9, best * 1e-3 * 2.4e9 * 256 / winstr);
    }
    return 0;
}
