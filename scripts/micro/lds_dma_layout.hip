// Probe: where buffer_load_dword{x3,x4} ... lds put each lane's bytes in LDS (gfx950).
// Source word i holds i; one wave loads 16 B (x4) or 12 B (x3) per lane from byte 16*lane / 12*lane.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void* lptr;
__global__ void k(const unsigned* g, unsigned* out)
{
    __shared__ __attribute__((aligned(16))) unsigned lds[2][512];
    for (int i = threadIdx.x; i < 1024; i += 64) (&lds[0][0])[i] = 0xffffffffu;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, 1 << 16, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr)&lds[0][0], 16, threadIdx.x * 16, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr)&lds[1][0], 12, threadIdx.x * 12, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = (&lds[0][0])[i];
}
int main()
{
    unsigned h[4096], o[1024];
    for (int i = 0; i < 4096; i++) h[i] = i;
    unsigned *dg, *dout;
    hipMalloc(&dg, sizeof(h)); hipMalloc(&dout, sizeof(o));
    hipMemcpy(dg, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dg, dout);
    hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    int bad4 = 0, bad3 = 0;
    for (int i = 0; i < 256; i++) bad4 += o[i] != (unsigned)i;
    for (int i = 0; i < 192; i++) bad3 += o[512 + i] != (unsigned)i;
    printf("x4: %d mismatches of 256; first words:", bad4);
    for (int i = 0; i < 12; i++) printf(" %d", (int)o[i]);
    printf("\nx3: %d mismatches of 192; first words:", bad3);
    for (int i = 0; i < 16; i++) printf(" %d", (int)o[512 + i]);
    printf("\nx3 words 192..200:");
    for (int i = 192; i < 200; i++) printf(" %d", (int)o[512 + i]);
    printf("\n");
    return 0;
}
