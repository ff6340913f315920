// Microbenchmark: memory-only upper bounds for the warp+diff access pattern at 4K x 32 pairs
// (3 B/px: read gray1, read gray2, write mask).
//  (a) linear: every thread streams 16 B of each of the three arrays
//  (b) tile: the k_warp_diff pattern -- one 256-thread workgroup per 128 x 64 tile, lane l of
//      wave w owns 4 columns of rows 2w + (l >> 5) + 8i; gray1 and gray2 read as dwords at the
//      same position, mask = g1 ^ g2 stored as a dword (no gather, no LDS)
//  (c) tile + gray1 staged through LDS by 16-B loads over a 76-row x 256-B footprint (as the kernel)
// hipcc --offload-arch=gfx950 -O3 warp_mem.hip -o warp_mem && ./warp_mem
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, B = 32;

__global__ __launch_bounds__(256) void k_linear(const uint4* a, const uint4* b, uint4* m, size_t n16)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 x = a[i], y = b[i];
        m[i] = make_uint4(x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w);
    }
}

__global__ __launch_bounds__(256) void k_linear_nt(const uint4* a, const uint4* b, uint4* m, size_t n16)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const v4u x = __builtin_nontemporal_load((const v4u*)a + i), y = __builtin_nontemporal_load((const v4u*)b + i);
        __builtin_nontemporal_store(x ^ y, (v4u*)m + i);
    }
}

__global__ __launch_bounds__(256) void k_linear_ntst(const uint4* a, const uint4* b, uint4* m, size_t n16)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const v4u x = ((const v4u*)a)[i], y = ((const v4u*)b)[i];
        __builtin_nontemporal_store(x ^ y, (v4u*)m + i);
    }
}

__global__ __launch_bounds__(256) void k_read(const uint4* a, const uint4* b, uint4* m, size_t n16)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 x = a[i], y = b[i];
        acc ^= x.x ^ y.y ^ x.z ^ y.w;
    }
    if (acc == 0x12345678u) m[0] = make_uint4(acc, 0, 0, 0);
}

__global__ __launch_bounds__(256) void k_write(const uint4* a, const uint4* b, uint4* m, size_t n16)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) m[i] = make_uint4(i, 0, 0, 0);
}

template <bool STAGE>
__global__ __launch_bounds__(256) void k_tile(const uint8_t* g1, const uint8_t* g2, uint8_t* mask)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_src[76 * 256];
    const int nbx = gridDim.x, nby = gridDim.y;
    int bid = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    {
        const int total = nbx * nby * gridDim.z, xcd = bid & 7, q8 = total >> 3, r8 = total & 7;
        bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    }
    const int pair = bid / (nbx * nby), tile = bid - pair * (nbx * nby);
    const int tx = tile % nbx, ty = tile / nbx;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x0 = tx * 128, y0 = ty * 64, xs = x0 + 4 * (lane & 31), r0 = 2 * wave + (lane >> 5);
    const size_t fo = (size_t)pair * W * H;
    uint32_t acc = 0;
    if (STAGE) {
        // footprint rows y0-6 .. y0+69, columns x0-8 .. x0+136 (16-B chunks), clamped to the frame
        for (int c = tid; c < 76 * 9; c += 256) {
            const int r = c / 9, ch = c % 9;
            const int y = min(max(y0 - 6 + r, 0), H - 1), x = min(max(x0 - 16 + 16 * ch, 0), W - 16);
            *(uint4*)&s_src[r * 256 + 16 * ch] = *(const uint4*)(g1 + fo + (size_t)y * W + x);
        }
        __syncthreads();
    }
    for (int i = 0; i < 8; i++) {
        const int y = y0 + r0 + 8 * i;
        if (y >= H || xs >= W) continue;
        const uint32_t v1 = STAGE ? *(const uint32_t*)&s_src[(r0 + 8 * i + 6) * 256 + 16 + 4 * (lane & 31)]
                                  : *(const uint32_t*)(g1 + fo + (size_t)y * W + xs);
        const uint32_t v2 = *(const uint32_t*)(g2 + fo + (size_t)y * W + xs);
        *(uint32_t*)(mask + fo + (size_t)y * W + xs) = v1 ^ v2;
    }
}

int main()
{
    const size_t n = (size_t)W * H * B;
    uint8_t *a, *b, *m;
    hipMalloc(&a, n);
    hipMalloc(&b, n);
    hipMalloc(&m, n);
    hipMemset(a, 1, n);
    hipMemset(b, 2, n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 10; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("%-28s %8.1f us  %7.1f GB/s (3 B/px)\n", name, best * 1e3, 3.0 * n / (best * 1e-3) / 1e9);
    };
    timeit("linear 16B/thread", [&] { hipLaunchKernelGGL(k_linear, dim3(256 * 32), dim3(256), 0, 0, (const uint4*)a, (const uint4*)b, (uint4*)m, n / 16); });
    timeit("linear nt load+store", [&] { hipLaunchKernelGGL(k_linear_nt, dim3(256 * 32), dim3(256), 0, 0, (const uint4*)a, (const uint4*)b, (uint4*)m, n / 16); });
    timeit("linear nt store", [&] { hipLaunchKernelGGL(k_linear_ntst, dim3(256 * 32), dim3(256), 0, 0, (const uint4*)a, (const uint4*)b, (uint4*)m, n / 16); });
    timeit("read only (2 B/px moved)", [&] { hipLaunchKernelGGL(k_read, dim3(256 * 32), dim3(256), 0, 0, (const uint4*)a, (const uint4*)b, (uint4*)m, n / 16); });
    timeit("write only (1 B/px moved)", [&] { hipLaunchKernelGGL(k_write, dim3(256 * 32), dim3(256), 0, 0, (const uint4*)a, (const uint4*)b, (uint4*)m, n / 16); });
    timeit("linear 16B/thread again", [&] { hipLaunchKernelGGL(k_linear, dim3(256 * 64), dim3(256), 0, 0, (const uint4*)a, (const uint4*)b, (uint4*)m, n / 16); });
    const dim3 grid(W / 128, (H + 63) / 64, B);
    timeit("tile dwords", [&] { hipLaunchKernelGGL(k_tile<false>, grid, dim3(256), 0, 0, a, b, m); });
    timeit("tile + LDS staging", [&] { hipLaunchKernelGGL(k_tile<true>, grid, dim3(256), 0, 0, a, b, m); });
    return 0;
}
