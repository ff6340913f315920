// Microbenchmark: chip-wide issue cost of VALU op classes on gfx950 relative to v_fma_f32 (the
// guide's 2-cycle full-rate reference), 8 independent chains per wave, 8 waves per SIMD.
// hipcc --offload-arch=gfx950 -O3 valu_rate3.hip -o /tmp/valu_rate3 && /tmp/valu_rate3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define OPS(X)                                                                  \
    X(0, "v_fma_f32", "v_fma_f32 %0, %0, %1, %1", f)                            \
    X(1, "v_xor_b32", "v_xor_b32 %0, %0, %1", a)                                \
    X(2, "v_sub_u32", "v_sub_u32 %0, %0, %1", a)                                \
    X(3, "v_min_u32", "v_min_u32 %0, %0, %1", a)                                \
    X(4, "v_max_f32", "v_max_f32 %0, %0, %1", f)                                \
    X(5, "v_lshrrev_b32", "v_lshrrev_b32 %0, 3, %0", a1)                        \
    X(6, "v_lshrrev_b32_v", "v_lshrrev_b32 %0, %1, %0", a)                      \
    X(7, "v_ashrrev_i32", "v_ashrrev_i32 %0, %1, %0", a)                        \
    X(8, "v_mov_b32", "v_mov_b32 %0, %1", a)                                    \
    X(9, "v_cvt_f32_i32", "v_cvt_f32_i32 %0, %1", a2)                           \
    X(10, "v_cvt_f32_ubyte0", "v_cvt_f32_ubyte0 %0, %1", a2)                    \
    X(11, "v_pk_mul_f32", "v_pk_mul_f32 %0, %0, %1", d)                         \
    X(12, "v_sub_f32", "v_sub_f32 %0, %0, %1", f)                               \
    X(13, "v_fmac_f32", "v_fmac_f32 %0, %1, %1", f)                             \
    X(14, "v_mul_hi_u32", "v_mul_hi_u32 %0, %0, %1", a)                         \
    X(15, "v_add_co_u32", "v_add_co_u32 %0, vcc, %0, %1", a)                    \
    X(16, "v_addc_co_u32", "v_addc_co_u32 %0, vcc, %0, %1, vcc", a)             \
    X(17, "v_and_b32_k", "v_and_b32 %0, 0xf80000, %0", a1)                      \
    X(18, "v_add_u32_k", "v_add_u32 %0, 0x12345, %0", a1)                       \
    X(19, "v_mul_f32_k", "v_mul_f32 %0, 0x3f812345, %0", f1)                    \
    X(20, "v_cvt_i32_f32", "v_cvt_i32_f32 %0, %1", f3)                          \
    X(21, "v_rndne_f32", "v_rndne_f32 %0, %1", f)                               \
    X(22, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1", a)                         \
    X(23, "v_add_u16", "v_add_u16 %0, %0, %1", a)                               \
    X(24, "v_mul_lo_u16", "v_mul_lo_u16 %0, %0, %1", a)                         \
    X(25, "v_fma_f16", "v_fma_f16 %0, %0, %1, %1", a)                           \
    X(26, "v_pk_fma_f16", "v_pk_fma_f16 %0, %0, %1, %1", a)                     \
    X(27, "v_dot2_f32_f16", "v_dot2_f32_f16 %0, %0, %1, %0", a)                 \
    X(28, "v_min_f32", "v_min_f32 %0, %0, %1", f)                               \
    X(29, "v_cmp_vcc", "v_cmp_gt_u32 vcc, %0, %1", a)                           \
    X(30, "v_add_f16", "v_add_f16 %0, %0, %1", a)                               \
    X(31, "v_and_b32_sdwa", "v_and_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD", a)

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
        if (#kind[0] == 'f' && #kind[1] == 0) asm volatile(text : "+v"(f[i]) : "v"(f[(i + 1) & 7]));   \
        if (#kind[0] == 'd') asm volatile(text : "+v"(d[i]) : "v"(d[(i + 1) & 7]));                   \
        if (#kind[0] == 'a' && #kind[1] == 0) asm volatile(text : "+v"(a[i]) : "v"(a[(i + 1) & 7]));   \
        if (#kind[0] == 'a' && #kind[1] == '1') asm volatile(text : "+v"(a[i]));                      \
        if (#kind[0] == 'a' && #kind[1] == '2') asm volatile(text : "+v"(f[i]) : "v"(a[(i + 1) & 7])); \
        if (#kind[0] == 'f' && #kind[1] == '1') asm volatile(text : "+v"(f[i]));                      \
        if (#kind[0] == 'f' && #kind[1] == '3') asm volatile(text : "+v"(a[i]) : "v"(f[(i + 1) & 7])); \
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
