// Microbenchmark: issue rate of VALU op classes on gfx950 (FP64 add/fma vs int32 vs packed u16 vs
// dot2 vs perm), chip-wide.  hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, uint32_t seed)
{
    uint32_t a[8];
    double d[8];
    for (int i = 0; i < 8; i++) { a[i] = seed * (threadIdx.x + i + 1); d[i] = (double)a[i] * 1e-3; }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (OP == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
                if (OP == 1) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
                if (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if (OP == 3) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if (OP == 4) asm volatile("v_dot2_u32_u16 %0, %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if (OP == 6) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if (OP == 7) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d[i]) : "v"(d[(i + 1) & 7]));
                if (OP == 8) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[i]));
            }
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s += a[i] + (uint32_t)__double2loint(d[i]);
    if (s == 0x12345678u) out[0] = s;
}

template <int OP>
float run(const char* name, int iters)
{
    uint32_t* out;
    hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8 * 4;   // 8 waves/SIMD x 4 SIMDs... many rounds
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 2, 7u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double waveinstr = (double)blocks * 4 * iters * 16 * 8;
    // per SIMD: 1024 SIMDs; cycles at an assumed 2.4 GHz max clock
    const double ns_per = ms * 1e6 / (waveinstr / 1024.0);
    printf("%-16s %8.3f ms  %6.3f ns per wave-instr per SIMD (= %.2f cycles @2.4GHz)\n", name, ms, ns_per, ns_per * 2.4);
    hipFree(out);
    return ms;
}

int main()
{
    const int it = 200;
    run<0>("v_add_f64", it);
    run<1>("v_fma_f64", it);
    run<2>("v_add_u32", it);
    run<3>("v_pk_add_u16", it);
    run<4>("v_dot2_u32_u16", it);
    run<5>("v_perm_b32", it);
    run<6>("v_mad_u32_u24", it);
    run<7>("v_pk_fma_f32", it);
    run<8>("v_lshlrev_b32", it);
    return 0;
}
