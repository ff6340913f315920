// Microbenchmark: chip-wide issue cost of VALU op classes on gfx950 relative to v_fma_f32 (the
// guide's 2-cycle full-rate reference), 8 independent chains per wave, 8 waves per SIMD.
// hipcc --offload-arch=gfx950 -O3 valu_rate2.hip -o /tmp/valu_rate2 && /tmp/valu_rate2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define OPS(X)                                                                  \
    X(0, "v_fma_f32", "v_fma_f32 %0, %0, %1, %1", f)                            \
    X(1, "v_add_f32", "v_add_f32 %0, %0, %1", f)                                \
    X(2, "v_add_u32", "v_add_u32 %0, %0, %1", a)                                \
    X(3, "v_and_b32", "v_and_b32 %0, %0, %1", a)                                \
    X(4, "v_or_b32", "v_or_b32 %0, %0, %1", a)                                  \
    X(5, "v_lshlrev_b32", "v_lshlrev_b32 %0, 3, %0", a1)                        \
    X(6, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 16, %1", a)                    \
    X(7, "v_and_or_b32", "v_and_or_b32 %0, %0, %1, %1", a)                      \
    X(8, "v_bfe_u32", "v_bfe_u32 %0, %0, 3, %1", a)                             \
    X(9, "v_perm_b32", "v_perm_b32 %0, %0, %1, %1", a)                          \
    X(10, "v_alignbyte_b32", "v_alignbyte_b32 %0, %0, %1, %1", a)               \
    X(11, "v_mad_u32_u24", "v_mad_u32_u24 %0, %0, %1, %1", a)                   \
    X(12, "v_mul_u32_u24", "v_mul_u32_u24 %0, %0, %1", a)                       \
    X(13, "v_sad_u32", "v_sad_u32 %0, %0, %1, %1", a)                           \
    X(14, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1", a)                         \
    X(15, "v_pk_mul_lo_u16", "v_pk_mul_lo_u16 %0, %0, %1", a)                   \
    X(16, "v_pk_mad_u16", "v_pk_mad_u16 %0, %0, %1, %1", a)                     \
    X(17, "v_dot2_u32_u16", "v_dot2_u32_u16 %0, %0, %1, %0", a)                 \
    X(18, "v_dot4_u32_u8", "v_dot4_u32_u8 %0, %0, %1, %0", a)                   \
    X(19, "v_add_f64", "v_add_f64 %0, %0, %1", d)                               \
    X(20, "v_fma_f64", "v_fma_f64 %0, %0, %1, %1", d)                           \
    X(21, "v_pk_fma_f32", "v_pk_fma_f32 %0, %0, %1, %1", d)                     \
    X(22, "v_pk_add_f32", "v_pk_add_f32 %0, %0, %1", d)                         \
    X(23, "v_cvt_f32_u32", "v_cvt_f32_u32 %0, %1", a2)                          \
    X(24, "v_mul_f32", "v_mul_f32 %0, %0, %1", f)                               \
    X(25, "v_add3_u32", "v_add3_u32 %0, %0, %1, %1", a)                         \
    X(26, "v_lshl_add_u32", "v_lshl_add_u32 %0, %0, 2, %1", a)                  \
    X(27, "v_cndmask_b32", "v_cndmask_b32 %0, %0, %1, vcc", a)                  \
    X(28, "v_mul_lo_u32", "v_mul_lo_u32 %0, %0, %1", a)                         \
    X(29, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %1", a)                           \
    X(30, "v_max3_u32", "v_max3_u32 %0, %0, %1, %1", a)                         \
    X(31, "v_med3_i32", "v_med3_i32 %0, %0, %1, %1", a)

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, uint32_t seed)
{
    uint32_t a[8];
    float f[8];
    double d[8];
    for (int i = 0; i < 8; i++) {
        a[i] = seed * (threadIdx.x + i + 1);
        f[i] = (float)a[i] * 1e-9f;
        d[i] = (double)a[i] * 1e-9;
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
#define EMIT(n, name, text, kind)                                                                     \
    if (OP == n) {                                                                                    \
        if (#kind[0] == 'f') asm volatile(text : "+v"(f[i]) : "v"(f[(i + 1) & 7]));                   \
        if (#kind[0] == 'd') asm volatile(text : "+v"(d[i]) : "v"(d[(i + 1) & 7]));                   \
        if (#kind[0] == 'a' && #kind[1] == 0) asm volatile(text : "+v"(a[i]) : "v"(a[(i + 1) & 7]));   \
        if (#kind[0] == 'a' && #kind[1] == '1') asm volatile(text : "+v"(a[i]));                      \
        if (#kind[0] == 'a' && #kind[1] == '2') asm volatile(text : "+v"(f[i]) : "v"(a[(i + 1) & 7])); \
    }
                OPS(EMIT)
            }
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s += a[i] + (uint32_t)__float_as_uint(f[i]) + (uint32_t)__double2loint(d[i]);
    if (s == 0x12345678u) out[0] = s;
}

template <int OP>
void run(const char* name, int iters, double ref_ms)
{
    uint32_t* out;
    hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8 * 4;
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 2, 7u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double waveinstr = (double)blocks * 4 * iters * 16 * 8;
    const double ns_per = best * 1e6 / (waveinstr / 1024.0);
    printf("%-18s %8.3f ms  %6.3f ns/wave-instr/SIMD  %.2f x v_fma_f32\n", name, best, ns_per,
           ref_ms > 0 ? best / ref_ms : 1.0);
    hipFree(out);
}

static double g_ref = 0;
template <int OP>
double time_only(int iters)
{
    uint32_t* out;
    hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8 * 4;
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 2, 7u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    hipFree(out);
    return best;
}

int main()
{
    const int it = 100;
    g_ref = time_only<0>(it);
#define RUN(n, name, text, kind) run<n>(name, it, g_ref);
    OPS(RUN)
    return 0;
}
