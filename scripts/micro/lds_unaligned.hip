// Microtest: are unaligned ds_read_u16 / ds_read_b32 correct and unpenalised on gfx950?
// hipcc --offload-arch=gfx950 -O3 lds_unaligned.hip -o lds_unaligned && ./lds_unaligned
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE>   // 0: u16 aligned, 1: u16 odd, 2: b32 aligned, 3: b32 +1, 4: b32 +2, 5: u8
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, int* bad)
{
    __shared__ __attribute__((aligned(16))) uint8_t s[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) s[i] = (uint8_t)(i * 7 + (i >> 8));
    __syncthreads();
    uint32_t acc = 0;
    const int lane = threadIdx.x & 63;
    int base = lane * 4 + (MODE == 1 || MODE == 3 ? 1 : MODE == 4 ? 2 : 0);
    for (int it = 0; it < iters; it++) {
        const int a = (base + it * 256) & 4095;
        uint32_t v;
        if (MODE <= 1) v = *reinterpret_cast<const uint16_t*>(&s[a]);
        else if (MODE <= 4) v = *reinterpret_cast<const uint32_t*>(&s[a]);
        else v = s[a];
        if (it == 0) {
            uint32_t exp = 0;
            const int nb = MODE <= 1 ? 2 : MODE <= 4 ? 4 : 1;
            for (int b = 0; b < nb; b++) exp |= (uint32_t)(uint8_t)((a + b) * 7 + ((a + b) >> 8)) << (8 * b);
            if (v != exp) atomicAdd(bad, 1);
        }
        acc += v;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    uint32_t* out; int* bad;
    hipMalloc(&out, 4); hipMalloc(&bad, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const char* names[] = {"u16 aligned", "u16 odd", "b32 aligned", "b32 +1", "b32 +2", "u8"};
    for (int m = 0; m < 6; m++) {
        hipMemset(bad, 0, 4);
        float best = 1e9;
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            switch (m) {
            case 0: hipLaunchKernelGGL(k<0>, dim3(4096), dim3(256), 0, 0, out, 2048, bad); break;
            case 1: hipLaunchKernelGGL(k<1>, dim3(4096), dim3(256), 0, 0, out, 2048, bad); break;
            case 2: hipLaunchKernelGGL(k<2>, dim3(4096), dim3(256), 0, 0, out, 2048, bad); break;
            case 3: hipLaunchKernelGGL(k<3>, dim3(4096), dim3(256), 0, 0, out, 2048, bad); break;
            case 4: hipLaunchKernelGGL(k<4>, dim3(4096), dim3(256), 0, 0, out, 2048, bad); break;
            case 5: hipLaunchKernelGGL(k<5>, dim3(4096), dim3(256), 0, 0, out, 2048, bad); break;
            }
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        int hb = 0; hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
        const double wi = 4096.0 * 4 * 2048;
        printf("%-12s %7.3f ms  %5.2f clk/wave-instr/CU  wrong=%d\n", names[m], best, best * 1e-3 * 2.4e9 * 256 / wi, hb);
    }
    return 0;
}
