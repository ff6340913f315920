// Microbenchmark: chip-wide issue cost of the LK chain element's instruction classes on gfx950
// relative to v_fma_f32 (the guide's 2-cycle full-rate reference), 8 independent chains per
// wave, 8 waves per SIMD.
// hipcc --offload-arch=gfx950 -O3 valu_rate4.hip -o valu_rate4 && ./valu_rate4
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define OPS(X)                                                                  \
    X(0, "v_fma_f32", "v_fma_f32 %0, %0, %1, %1", f)                            \
    X(1, "v_dot2c_i32_i16", "v_dot2c_i32_i16 %0, %1, %1", a)                    \
    X(2, "v_dot2_i32_i16", "v_dot2_i32_i16 %0, %1, %1, %0", a)                  \
    X(3, "v_cvt_f32_i32_sdwa", "v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1", a2) \
    X(4, "v_ashrrev_i32_k", "v_ashrrev_i32 %0, 9, %0", a1)                      \
    X(5, "v_lshrrev_b32_k", "v_lshrrev_b32 %0, 9, %0", a1)                      \
    X(6, "v_pk_add_f32", "v_pk_add_f32 %0, %0, %1", d)                          \
    X(7, "v_pk_mul_f32", "v_pk_mul_f32 %0, %0, %1", d)                          \
    X(8, "v_mul_f32", "v_mul_f32 %0, %0, %1", f)                                \
    X(9, "v_add_f32", "v_add_f32 %0, %0, %1", f)                                \
    X(10, "v_cvt_f32_i32", "v_cvt_f32_i32 %0, %1", a2)                          \
    X(11, "v_perm_b32", "v_perm_b32 %0, %0, %1, %1", a)                         \
    X(12, "v_mul_i32_i24", "v_mul_i32_i24 %0, %0, %1", a)                       \
    X(13, "v_or_b32", "v_or_b32 %0, %0, %1", a)                                 \
    X(14, "v_cvt_f32_ubyte1", "v_cvt_f32_ubyte1 %0, %1", a2)                    \
    X(15, "v_ashrrev_i32_v", "v_ashrrev_i32 %0, %1, %0", a)                     \
    X(16, "v_bfe_i32", "v_bfe_i32 %0, %0, 16, 16", a1)                          \
    X(17, "v_mad_i32_i24", "v_mad_i32_i24 %0, %0, %1, %1", a)                   \
    X(18, "v_cvt_f32_i32_e64", "v_cvt_f32_i32_e64 %0, %1", a2)                  \
    X(19, "v_mul_f32_sdwa", "v_mul_f32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD", f)

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
