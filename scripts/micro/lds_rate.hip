// Microbenchmark: LDS read issue cost per wave-instruction on gfx950, chip-wide, for the access
// patterns of the warp kernel's taps (lane l reads column 4*(l&31)+k of row r0 + (l>>5): the two
// half-waves 256 B apart) and variants.  8 independent reads in flight per wave, 8 waves/SIMD.
// hipcc --offload-arch=gfx950 -O3 lds_rate.hip -o /tmp/lds_rate && /tmp/lds_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, int half_off)
{
    __shared__ __attribute__((aligned(16))) uint8_t s[16384];
    for (int i = threadIdx.x; i < 4096; i += 256) ((uint32_t*)s)[i] = i * 2654435761u;
    __syncthreads();
    const int l = threadIdx.x & 63;
    uint32_t base = 4 * (l & 31) + (l >> 5) * half_off + (threadIdx.x >> 6) * 2048;
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t a = (base + 1024 * (i & 1) + 8 * i + (acc & 0)) & 16383u;
            uint32_t v = 0, w = 0;
            if (OP == 0) asm volatile("ds_read_u8 %0, %1" : "=v"(v) : "v"(a + 1));
            if (OP == 1) asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a & ~3u));
            if (OP == 2) asm volatile("ds_read2_b32 %0, %1 offset1:1" : "=v"(*(uint64_t*)&v) : "v"(a & ~3u));
            if (OP == 3) asm volatile("ds_read_b64 %0, %1" : "=v"(*(uint64_t*)&v) : "v"(a & ~7u));
            if (OP == 4) asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(a & ~1u));
            if (OP == 5) asm volatile("ds_read_u8 %0, %1" : "=v"(v) : "v"((4 * l) & 255));   // one row, 64 lanes
            if (OP == 6) asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(8 * ((l * 7) & 31)));  // weight table: 32 entries
            if (OP == 7) asm volatile("ds_read_b128 %0, %1" : "=v"(*(__attribute__((ext_vector_type(4))) uint32_t*)&v) : "v"(a & ~15u));
            acc += v + w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int OP>
void run(const char* name, int iters, int half_off)
{
    uint32_t* out;
    hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 4 * 4;   // 4 blocks of 16 KB LDS per CU at a time (16 waves/CU)
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 2, half_off);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, half_off);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double waveinstr = (double)blocks * 4 * iters * 8;
    printf("%-22s half_off %4d  %8.3f ms  %6.3f ns per wave-instr per CU\n", name, half_off, best,
           best * 1e6 / (waveinstr / 256.0));
    hipFree(out);
}

int main()
{
    const int it = 2000;
    for (int ho : {256, 128}) {
        run<0>("ds_read_u8", it, ho);
        run<1>("ds_read_b32", it, ho);
        run<2>("ds_read2_b32", it, ho);
        run<3>("ds_read_b64", it, ho);
        run<4>("ds_read_u16", it, ho);
        run<7>("ds_read_b128", it, ho);
    }
    run<5>("ds_read_u8 one row", it, 0);
    run<6>("ds_read_b32 table", it, 0);
    return 0;
}
