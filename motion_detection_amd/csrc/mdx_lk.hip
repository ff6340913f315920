// mdx_lk.hip -- pyramidal Lucas-Kanade (reference row A5: calcOpticalFlowPyrLK as called at
// optical_flow_calculator.cpp:71), restructured for CDNA4 while keeping OpenCV 2.4's x86 SSE2
// arithmetic bit for bit.  This is the "class plane" LK (MDX_LK_IMPL=2, default); the
// single-kernel k_lk in mdx_kernels.hip is the fallback for very sparse grids.
//
// Per pyramid level, from maxLevel down to 0, three kernels:
//
//  k_lk_class  The interpolated window values (I*32 descaled by 9 bits, Ix/Iy descaled by 14
//              bits) over the whole padded level, once per fractional-offset class.  At level L a
//              grid point's window origin prevPt - 19.5 has a fractional part fixed by
//              (P mod 2^L), so all points of a residue class share the bilinear weights: the
//              16x-overlapping per-window interpolation of the reference becomes one
//              interpolation per class and pixel.  Row-major (D, C) pairs per class and plane
//              column: D = (Ix | Iy << 16) and C = 256 - 512*I (the J-chain bias, see below).
//  k_lk_A      Per point: the gradient matrix sums A11/A12/A22 over the window and the minEig /
//              determinant tests.
//  k_lk_iter   The Newton iterations, on persistent waves fed from per-XCD work queues.
//
// The first two depend on the previous frame only, so they run ahead on an auxiliary stream
// (level L-1's class planes and A sums while level L iterates) and fill the iteration kernel's
// tail; every level keeps its own planes, A buffer and queue heads.
//
// Work mapping.  Lane k of a point owns SSE lane k (window columns x = 4g + k, g = 0..9, rows in
// order) and keeps its partial sums in registers; partials are combined across the lane quad in
// the reference's order (A: ((P0+P1)+P2)+P3, b: (P0+P2)+(P1+P3)).  Points are processed in
// groups of G (4 or 8) consecutive members of one residue class along one grid row (host-built
// class-grouped order, runs padded to G), so a group's windows share their rows and overlap in
// columns: per window row the group needs one contiguous "union" segment of UW columns of D
// and C.  The group's lanes load it with coalesced dwordx4, store it to a double-buffered LDS
// row, and every lane then reads its 10 chain elements from LDS.  That replaces the 6 scattered
// dwordx2/x4 loads per lane and row that bound a per-point design on the texture data path (TD
// busy 97%, VALU 38%).  J (the moving window in the next frame) differs per point: its row
// segment is loaded once per lane quad and read back from LDS by the quad's lanes.
//
// Arithmetic: J taps via v_perm_b32 + v_dot2_i32_i16 (signed weights: w11 may be -1);
// dot2(pa, W0, dot2(pb, W1, C)) >> 9 == ((S + 256) >> 9) - I exactly, because C = 256 - 512*I
// is a multiple-of-512 shift of the rounding bias.  Products are float multiplies of exactly
// converted integers (one rounding of the exact product == the reference's (float)(int
// product)).  Products/sums never go through a contracted FMA (-ffp-contract=off); k_lk_A's
// explicit FMAs multiply operands whose product is exact in float (|Ix|, |Iy| <= 4080), so they
// round like the separate multiply and add.
#include "mdx_internal.h"

#include <float.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>

namespace mdx {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
// 4-B aligned 8-byte loads (global_load_dwordx2 at dword-aligned addresses)
struct __attribute__((aligned(4))) u2a4 { uint32_t x, y; };
struct __attribute__((aligned(4))) u3a4 { uint32_t x, y, z; };
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v3u __attribute__((ext_vector_type(3)));
// raw buffer descriptor over [base, base + bytes) (cdna_hip_programming.md T8: built from
// wave-uniform values only); loads then take a 32-bit per-lane byte offset
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, long long bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                             (int)min(bytes, (long long)0x7fffffff), 0x00020000);
}
// the same for wave-uniform inputs and a size the host keeps below 2 GB: the inputs pass through
// readfirstlane so that the compiler can prove the descriptor uniform (scalar instructions, no
// waterfall loop around the memory op; cdna_hip_programming.md T8)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc32(const void* base, uint32_t bytes)
{
    const unsigned long long b = (unsigned long long)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    void* p = (void*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// residue-class tables: [level][axis][128]
__device__ __forceinline__ int class_of(const int16_t* cmap, int level, int axis, int res)
{
    return cmap[(level * 2 + axis) * 128 + res];
}
__device__ __forceinline__ int residue_of(const int16_t* rlist, int level, int axis, int cls)
{
    return rlist[(level * 2 + axis) * 128 + cls];
}

__device__ __forceinline__ void lk_weights(float fa, float fb, int& w00, int& w01, int& w10, int& w11)
{
    w00 = __float2int_rn((1.f - fa) * (1.f - fb) * 16384.f);
    w01 = __float2int_rn(fa * (1.f - fb) * 16384.f);
    w10 = __float2int_rn((1.f - fa) * fb * 16384.f);
    w11 = 16384 - w00 - w01 - w10;
}

// The window element of one class / point at a pixel: LKTrackerInvoker's integer sums
//   I*32 = (i00 w00 + i01 w01 + i10 w10 + i11 w11 + 256) >> 9,  Ix/Iy = (sum d w + 8192) >> 14,
// evaluated with v_dot2 on 16-bit pairs (tap bytes, Ix / Iy halves; signed weights, w11 may be -1)
// -- the same int32 sums without any 32-bit multiply (v_mul_lo_u32 is quarter rate).  (lo, hi)
// hold the bytes of the tap rows y / y+1 with taps at bytes Q, Q+1; d* are the derivative words.
template <int Q>
__device__ __forceinline__ void lk_interp(uint32_t lo0, uint32_t hi0, uint32_t lo1, uint32_t hi1, uint32_t d00,
                                          uint32_t d01, uint32_t d10, uint32_t d11, s2 W0, s2 W1, int& ival, int& ixv,
                                          int& iyv)
{
    static_assert(Q >= 0 && Q < 7, "tap byte");
    constexpr unsigned sel = 0x0c000c00u | (unsigned)Q | ((unsigned)(Q + 1) << 16);
    const s2 t0 = __builtin_bit_cast(s2, __builtin_amdgcn_perm(hi0, lo0, sel));
    const s2 t1 = __builtin_bit_cast(s2, __builtin_amdgcn_perm(hi1, lo1, sel));
    ival = __builtin_amdgcn_sdot2(t0, W0, __builtin_amdgcn_sdot2(t1, W1, 256, false), false) >> 9;
    const s2 x0 = __builtin_bit_cast(s2, __builtin_amdgcn_perm(d01, d00, 0x05040100u));
    const s2 x1 = __builtin_bit_cast(s2, __builtin_amdgcn_perm(d11, d10, 0x05040100u));
    const s2 y0 = __builtin_bit_cast(s2, __builtin_amdgcn_perm(d01, d00, 0x07060302u));
    const s2 y1 = __builtin_bit_cast(s2, __builtin_amdgcn_perm(d11, d10, 0x07060302u));
    ixv = __builtin_amdgcn_sdot2(x0, W0, __builtin_amdgcn_sdot2(x1, W1, 8192, false), false) >> 14;
    iyv = __builtin_amdgcn_sdot2(y0, W0, __builtin_amdgcn_sdot2(y1, W1, 8192, false), false) >> 14;
}

// broadcast lane j of this lane's quad (DPP quad_perm, no LDS)
template <int J>
__device__ __forceinline__ float quad_bcast(float v)
{
    constexpr int ctrl = J | (J << 2) | (J << 4) | (J << 6);
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xf, 0xf, false));
}
template <int J>
__device__ __forceinline__ uint32_t quad_bcast_u(uint32_t v)
{
    constexpr int ctrl = J | (J << 2) | (J << 4) | (J << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xf, 0xf, false);
}

// Ordering point between a window row's LDS staging writes and the next row's reads.  A
// workgroup is one wave and one wave's LDS instructions execute in order, so only the compiler
// must be kept from moving LDS accesses across it (no s_barrier, no forced vmcnt(0)).
__device__ __forceinline__ void wave_lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// k_lk_iter: 5 waves/SIMD (<= 102 VGPRs; measured 3% faster than 6 at <= 80)
#ifndef MDX_LK_WPE
#define MDX_LK_WPE 4
#endif
#ifndef MDX_LK_NB
#define MDX_LK_NB 2
#endif
// Dataflow waits are bounded (LkArgs::spin_max s_sleep(8) polls, ~0.1 s by default): past that a
// group proceeds regardless and its wave stops waiting, so the launch drains instead of hanging.
// Every such give-up is counted in LkArgs::err, which the host reads at its next sync point and
// turns into MDX_EHIP: a timed-out hand-off is never a silent wrong result.
#ifndef MDX_LK_RFIRST
#define MDX_LK_RFIRST 0
#endif
constexpr int kLkIterWavesPerEU = MDX_LK_WPE;
typedef __attribute__((address_space(3))) void* lds_ptr;
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
// volatile LDS views: each access stays one ds_read_b64 / ds_read_b128 (never merged into a
// half-rate read2 or narrowed)
typedef __attribute__((address_space(3))) volatile const v2u lds_u2v;
typedef __attribute__((address_space(3))) volatile const v4u lds_u4v;
// s_waitcnt vmcnt(0) (gfx9 encoding: expcnt / lgkmcnt left at their maxima), pinned in place
__device__ __forceinline__ void lk_vmcnt0()
{
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_sched_barrier(0);
}
// s_waitcnt vmcnt(N), N < 16
template <int N>
__device__ __forceinline__ void lk_vmcnt()
{
    static_assert(N >= 0 && N < 16, "vmcnt field");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70 | N);
    __builtin_amdgcn_sched_barrier(0);
}

// compile-time loop: f(integral_constant<I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f)
{
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// XCD-aware block order: blocks are dealt round-robin over the 8 XCDs; remap so that each
// XCD gets a contiguous range of waves (= a contiguous image band), whose class planes then
// stay in that XCD's L2.  Bijective for any count (cdna_hip_programming.md §5.5 T1).
__device__ __forceinline__ int xcd_remap(int b, int total)
{
    const int xcd = b & 7, q = total >> 3, r = total & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// Class-plane stores go non-temporal: a level's planes (tens of MB per batch) do not fit in L2 and
// are re-read from HBM/MALL by k_lk_A and k_lk_iter anyway, and these kernels run on the aux stream
// beside the coarser levels' iterations, whose row re-reads keep their L2 lines this way.  Whole
// path, alternating on two boxes: 7129 / 7106 vs 7071 / 7046 Mpx/s (6 runs each, 5 of 6 pairs ahead).
__device__ __forceinline__ void cls_store(uint4* o, const uint32_t (&dv)[4], const int (&cv)[4])
{
    typedef unsigned v4nt __attribute__((ext_vector_type(4)));
    const uint4 a = make_uint4(dv[0], (uint32_t)cv[0], dv[1], (uint32_t)cv[1]);
    const uint4 b = make_uint4(dv[2], (uint32_t)cv[2], dv[3], (uint32_t)cv[3]);
    __builtin_nontemporal_store(__builtin_bit_cast(v4nt, a), reinterpret_cast<v4nt*>(o));
    __builtin_nontemporal_store(__builtin_bit_cast(v4nt, b), reinterpret_cast<v4nt*>(o) + 1);
}

// ------------------------------------------------------------------ class planes
// grid: x -> 4 consecutive plane columns u per thread, y -> plane row v, z -> pair * nclass +
// class.  Element (u, v) is the window value at level core position (x, y) = (u - 40, v - 40)
// for the class's bilinear weights: (I*32, Ix, Iy) exactly as LKTrackerInvoker extracts them
// (CV_DESCALE by W_BITS1-5 = 9 and W_BITS1 = 14).  Outside the level's padded extent: 0.
__global__ __launch_bounds__(256) void k_lk_class(const uint8_t* __restrict__ pyr1, const uint32_t* __restrict__ der,
                                                  uint8_t* __restrict__ cls_out, LkClassArgs a)
{
    const int level = a.level;
    const ClassLevel& C = a.plan.lv[level];
    const int nclass = C.nrx * C.nry;
    const int pair = blockIdx.z / nclass, cls = blockIdx.z % nclass;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int v = C.vlo + blockIdx.y;                // only rows some planned window reaches
    // columns a window can reach: x = u - 40 <= w + 38; the rest of PW is union-load slack whose
    // values no lane uses, so it is left unwritten
    if (4 * j >= a.g.lv[level].w + 2 * kPad || v >= C.UH) return;
    const Level L = a.g.lv[level];
    const float scale = (float)(1. / (1 << level));
    const int rx = residue_of(a.rlist, level, 0, cls % C.nrx), ry = residue_of(a.rlist, level, 1, cls / C.nrx);
    const float ppx = (float)rx * scale - 19.5f, ppy = (float)ry * scale - 19.5f;
    const float fa = ppx - floorf(ppx), fb = ppy - floorf(ppy);
    int w00, w01, w10, w11;
    lk_weights(fa, fb, w00, w01, w10, w11);
    const uint8_t* I = pyr1 + (long long)pair * a.g.img_bytes + L.img_off + L.core();
    const uint32_t* D = der + (long long)pair * a.g.der_words + L.der_off + L.core();
    const int y = v - kPad;
    const int p = L.pitch;
    uint8_t* base = cls_out + (long long)pair * a.plan.bytes_per_pair + C.off + (long long)cls * C.class_bytes;
    uint32_t dv[4] = {0, 0, 0, 0};
    int cv[4];
    const int x0 = 4 * j - kPad;                     // first of this thread's 4 columns
    if (y < L.h + kPad - 1 && x0 < L.w + kPad - 1) {
        // rows y, y+1 of the padded level: 5 image bytes (one 8-B load) and 5 derivative words
        // (16-B + 4-B loads) per row; x0 is a multiple of 4 and the core is 64-B aligned
        const uint8_t* ip = I + (long long)y * p + x0;
        const uint32_t* dp = D + (long long)y * p + x0;
        uint32_t ib[2][2], dw[2][5];
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const u2a4 bi = *reinterpret_cast<const u2a4*>(ip + (long long)r * p);
            ib[r][0] = bi.x; ib[r][1] = bi.y;
            const uint4 d4 = *reinterpret_cast<const uint4*>(dp + (long long)r * p);
            dw[r][0] = d4.x; dw[r][1] = d4.y; dw[r][2] = d4.z; dw[r][3] = d4.w;
            dw[r][4] = dp[(long long)r * p + 4];
        }
        const s2 W0 = {(short)w00, (short)w01}, W1 = {(short)w10, (short)w11};
        static_for<0, 4>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            if (x0 + q >= L.w + kPad - 1) { cv[q] = 256; return; }
            int ival, ixv, iyv;
            lk_interp<q>(ib[0][0], ib[0][1], ib[1][0], ib[1][1], dw[0][q], dw[0][q + 1], dw[1][q], dw[1][q + 1], W0, W1,
                         ival, ixv, iyv);
            dv[q] = ((uint32_t)ixv & 0xffffu) | ((uint32_t)iyv << 16);
            cv[q] = 256 - 512 * ival;   // J-chain bias: (S + C) >> 9 == ((S + 256) >> 9) - I
        });
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) cv[q] = 256;
    }
    // (D, C) pairs, row-major: one 8-B element per plane column
    uint4* o = reinterpret_cast<uint4*>(base) + ((long long)v * C.PW + 4 * j) / 2;
    cls_store(o, dv, cv);
}

// Levels with at most 4 residue classes (the finest ones, whose Scharr planes are the largest):
// the same elements, with the Scharr derivatives computed here from the padded level image instead
// of read back from k_scharr's planes (lkpyramid.cpp calcSharrDeriv: t0 = 3(a+c)+10b, t1 = c-a,
// Ix = t0[x+1]-t0[x-1], Iy = 3(t1[x-1]+t1[x+1])+10 t1[x]; the padded level's reflect-101 rows and
// columns are OpenCV's neighbour clamping; 0 outside the level, the derivative planes' CONSTANT
// border).  One thread serves every class of its pair from one set of row loads, and the level's
// k_scharr launch (its plane writes and their reads) is skipped.
__device__ __forceinline__ int u8_at(const uint32_t (&w)[3], int b) { return (int)((w[b >> 2] >> (8 * (b & 3))) & 255u); }

__global__ __launch_bounds__(256) void k_lk_class_fused(const uint8_t* __restrict__ pyr1, uint8_t* __restrict__ cls_out,
                                                        LkClassArgs a)
{
    const int level = a.level;
    const ClassLevel& C = a.plan.lv[level];
    const int nclass = C.nrx * C.nry;                // <= 4 (host)
    const int pair = blockIdx.z;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int v = C.vlo + blockIdx.y;
    if (4 * j >= a.g.lv[level].w + 2 * kPad || v >= C.UH) return;
    const Level L = a.g.lv[level];
    const float scale = (float)(1. / (1 << level));
    const uint8_t* I = pyr1 + (long long)pair * a.g.img_bytes + L.img_off + L.core();
    const int y = v - kPad;
    const int p = L.pitch;
    const int x0 = 4 * j - kPad;
    const bool inside = y < L.h + kPad - 1 && x0 < L.w + kPad - 1;
    // image rows y-1 .. y+2, bytes x0-4 .. x0+7 (3 aligned dwords each); rows outside the padded
    // level are never used (their derivatives are 0) and read row y instead
    uint32_t rw[4][3];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int yy = y - 1 + r;
        const int ys = (yy < -kPad || yy >= L.h + kPad) ? y : yy;
        const u3a4 t = *reinterpret_cast<const u3a4*>(I + (long long)ys * p + x0 - 4);
        rw[r][0] = t.x; rw[r][1] = t.y; rw[r][2] = t.z;
    }
    // derivative words at columns x0 .. x0+4 of rows y, y+1 (k_lk_class's dw)
    uint32_t dw[2][5];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int yy = y + r;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            const int x = x0 + c;
            uint32_t d = 0;
            if (yy >= 0 && yy < L.h && x >= 0 && x < L.w) {
                const int bm = 3 + c, bc = 4 + c, bp = 5 + c;          // bytes x-1, x, x+1
                const int t0m = (u8_at(rw[r], bm) + u8_at(rw[r + 2], bm)) * 3 + u8_at(rw[r + 1], bm) * 10;
                const int t0p = (u8_at(rw[r], bp) + u8_at(rw[r + 2], bp)) * 3 + u8_at(rw[r + 1], bp) * 10;
                const int t1m = u8_at(rw[r + 2], bm) - u8_at(rw[r], bm), t1c = u8_at(rw[r + 2], bc) - u8_at(rw[r], bc);
                const int t1p = u8_at(rw[r + 2], bp) - u8_at(rw[r], bp);
                const int ix = t0p - t0m, iy = (t1m + t1p) * 3 + t1c * 10;
                d = (uint32_t)(uint16_t)(int16_t)ix | ((uint32_t)(uint16_t)(int16_t)iy << 16);
            }
            dw[r][c] = d;
        }
    }
    // the image bytes of rows y, y+1 at columns x0 .. x0+4 (k_lk_class's ib): bytes 4 .. 8
    for (int cls = 0; cls < nclass; cls++) {
        const int rx = residue_of(a.rlist, level, 0, cls % C.nrx), ry = residue_of(a.rlist, level, 1, cls / C.nrx);
        const float ppx = (float)rx * scale - 19.5f, ppy = (float)ry * scale - 19.5f;
        const float fa = ppx - floorf(ppx), fb = ppy - floorf(ppy);
        int w00, w01, w10, w11;
        lk_weights(fa, fb, w00, w01, w10, w11);
        uint32_t dv[4] = {0, 0, 0, 0};
        int cv[4] = {256, 256, 256, 256};
        if (inside) {
            const s2 W0 = {(short)w00, (short)w01}, W1 = {(short)w10, (short)w11};
            static_for<0, 4>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if (x0 + q >= L.w + kPad - 1) return;
                int ival, ixv, iyv;
                // taps at bytes 4+q, 5+q of rows y / y+1 (rw[1], rw[2]): bytes q, q+1 of words 1..2
                lk_interp<q>(rw[1][1], rw[1][2], rw[2][1], rw[2][2], dw[0][q], dw[0][q + 1], dw[1][q], dw[1][q + 1], W0,
                             W1, ival, ixv, iyv);
                dv[q] = ((uint32_t)ixv & 0xffffu) | ((uint32_t)iyv << 16);
                cv[q] = 256 - 512 * ival;
            });
        }
        uint8_t* base = cls_out + (long long)pair * a.plan.bytes_per_pair + C.off + (long long)cls * C.class_bytes;
        uint4* o = reinterpret_cast<uint4*>(base) + ((long long)v * C.PW + 4 * j) / 2;
        cls_store(o, dv, cv);
    }
}

// ------------------------------------------------------------------ one pyramid level
// Work units.  A GROUP is G consecutive members of one residue class along one grid row (host
// order: each class's run padded to a multiple of G with -1).  A SLOT is the 4G lanes holding one
// group, a lane quad per point.  Per window row a slot needs one contiguous "union" segment of UW
// plane columns, UW (D, C) pairs: staged in LDS, from where each lane reads its 10 chain pairs.
//
// Per level two kernels follow k_lk_class:
//  k_lk_A     static groups (one slot each): the gradient sums A11/A12/A22 and the minEig /
//             determinant tests, stored per point as (A11, A12, A22, 1/D) -- 1/D = 0 marks a point
//             the reference skips at this level.
//  k_lk_iter  the Newton iterations.  Points iterate 1..max_iters times; a slot whose G points
//             iterate in lockstep costs the max over the group, and a static wave the max over
//             all its groups.  So the waves are persistent and each slot, when its group retires,
//             takes the next group from a work queue: slots of one wave run out of step, only the
//             group-internal lockstep remains.
// UW is the exact-fit union width (even: a 16-B load carries two pairs); the last load of a
// slot's row and the last LDS-DMA piece of the wave's row are partial (lane-masked), so no byte
// beyond the union is moved.
template <int G, int UW>
struct LkShape {
    static constexpr int LPS = 4 * G;                         // lanes per slot
    static constexpr int S = 64 / LPS;                        // slots per wave
    static constexpr int NP = (UW + 2 * LPS - 1) / (2 * LPS); // A pass: 16-B (2-pair) loads per lane and row
    static constexpr int BYTES = S * UW * 8;                  // the wave's union row image
    static constexpr int ND = (BYTES + 1023) / 1024;          // iterations: LDS-DMA pieces per row
    static_assert(UW % 2 == 0 && UW >= kWin, "union width");
};

struct GroupGeom {
    int gx, gy;       // grid point of this lane quad
    bool valid;       // the quad holds a real point (not run padding / no group)
    int ipx, ipy;     // floor of the window origin at this level
    int off;          // the point's first column inside the union
    int v0;           // first window row in the class plane
    uint32_t ubase;   // byte offset in the pair's class slab of the union's first pair, plane row 0
};

// geometry of group g (-1 = none) for lane sl of its slot
template <int G, int UW>
__device__ __forceinline__ GroupGeom group_geom(const LkArgs& a, const ClassLevel& C, int level, int g, int sl)
{
    GroupGeom r;
    const int16_t* xo = a.ord + C.ord_off;
    const int16_t* yo = xo + C.nxp;
    const bool has = g >= 0;
    const int gg = has ? g : 0;
    const int cg = gg / a.nyg, row = gg - cg * a.nyg;   // column-group major: neighbours share rows
    const int e0 = cg * G;
    const int gxv = has ? xo[e0 + (sl >> 2)] : -1;
    r.valid = gxv >= 0;
    r.gx = r.valid ? gxv : 0;
    r.gy = yo[row];
    const float scale = (float)(1. / (1 << level));
    r.ipx = (int)floorf((float)(r.gx * a.pixel_step) * scale - 19.5f);
    r.ipy = (int)floorf((float)(r.gy * a.pixel_step) * scale - 19.5f);
    // a group's first entry is a real point (runs start at multiples of G, padding at their ends)
    // and its leftmost one (runs sorted by x)
    const int gx0 = has ? xo[e0] : 0;
    const int ipx0 = (int)floorf((float)(gx0 * a.pixel_step) * scale - 19.5f);
    const int m = (1 << level) - 1;
    const int cx = class_of(a.cmap, level, 0, (gx0 * a.pixel_step) & m);
    const int cy = class_of(a.cmap, level, 1, (r.gy * a.pixel_step) & m);
    const int ub = min(max(ipx0 + kPad, 0), C.PW - UW);            // union start column
    r.off = min(max(r.ipx + kPad - ub, 0), UW - kWin);
    r.v0 = min(max(r.ipy + kPad, 0), C.UH - kWin);
    r.ubase = (uint32_t)(C.off + (long long)(cy * C.nrx + cx) * C.class_bytes) + 8u * (uint32_t)ub;
    return r;
}

// ---- A pass.  grid: x -> wave (S static groups), y -> pair (XCD-remapped as one range).  Each
// lane loads 2 (D, C) pairs per 16-B load and stages the two D words; the chain reads are D only.
template <int G, int UW>
__global__ __launch_bounds__(64) void k_lk_A(LkArgs a, const uint8_t* __restrict__ cls, float4* __restrict__ Ab,
                                             int* __restrict__ qctr, int level, int ngroups)
{
    using Sh = LkShape<G, UW>;
    constexpr int LPS = Sh::LPS, S = Sh::S, ND = Sh::ND;
    constexpr int NB = 3;                                          // row images: NB - 1 rows in flight ahead
    constexpr float FLT_SCALE = 1.f / (1 << 20);
    // [slot][UW][D, C]: the wave's union row images, filled by LDS-DMA like k_lk_iter's; one
    // __shared__ array per buffer, so that no compiler wait ties a row's reads to later rows' DMA
    __shared__ __attribute__((aligned(16))) uint32_t img0[ND * 256];
    __shared__ __attribute__((aligned(16))) uint32_t img1[ND * 256];
    __shared__ __attribute__((aligned(16))) uint32_t img2[ND * 256];
    static_assert(NB == 3, "three row images");

    const int lane = threadIdx.x, k = lane & 3, slot = lane / LPS, sl = lane % LPS;
    const int nw = gridDim.x;
    const int bid = xcd_remap(blockIdx.x + nw * blockIdx.y, nw * gridDim.y);
    const int pair = bid / nw, w = bid % nw;
    if (bid == 0 && lane < 8) qctr[(level * 8 + lane) * kCtrPad] = 0;   // k_lk_iter's queue heads
    const ClassLevel& C = a.plan.lv[level];
    const Level L = a.g.lv[level];
    const int g = w * S + slot;
    const GroupGeom q = group_geom<G, UW>(a, C, level, g < ngroups ? g : -1, sl);
    bool ok = q.valid && !(q.ipx < -kWin || q.ipx >= L.w || q.ipy < -kWin || q.ipy >= L.h);

    const __amdgpu_buffer_rsrc_t crs = buf_rsrc(cls + (long long)pair * a.plan.bytes_per_pair, a.plan.bytes_per_pair);
    const uint32_t rowb = (uint32_t)C.PW * 8;
    // lane L of piece c fills image bytes 1024c + 16L: slot sp's union bytes wb (past the image:
    // an out-of-range offset, zeros)
    uint32_t uoff[ND];
    {
        const uint32_t mine = q.ubase + (uint32_t)q.v0 * rowb;
#pragma unroll
        for (int c = 0; c < ND; c++) {
            const int P = 1024 * c + 16 * lane;
            const int sp = P / (8 * UW), wb = P % (8 * UW);
            const uint32_t src = (uint32_t)__shfl((int)mine, (sp < S ? sp : 0) * LPS) + (uint32_t)wb;
            uoff[c] = sp < S ? src : 0x80000000u;
        }
    }
    auto ibuf = [&](auto bc) -> uint32_t* {
        constexpr int bb = decltype(bc)::value;
        if constexpr (bb == 0) return img0;
        else if constexpr (bb == 1) return img1;
        else return img2;
    };
    auto dma = [&](auto bc) {
        uint32_t* I = ibuf(bc);
#pragma unroll
        for (int c = 0; c < ND; c++) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(crs, (lds_ptr)(I + 256 * c), 16, (int)uoff[c], 0, 0, 0);
            uoff[c] += rowb;
        }
    };
    const int el = 2 * (slot * UW + q.off + k);

    // lane k owns SSE lane k (columns 4g+k), rows in order; ((P0+P1)+P2)+P3 across the quad
    f2 sd = {0.f, 0.f};
    float s12 = 0.f;
    constexpr int PF = NB - 1;                                     // rows in flight ahead
    dma(std::integral_constant<int, 0>{});
    dma(std::integral_constant<int, 1>{});
    static_for<0, kWin>([&](auto yc) {
        constexpr int y = decltype(yc)::value;
        // row y has landed once at most the later rows' pieces are outstanding
        constexpr int later = (y + PF - 1 < kWin - 1 ? y + PF - 1 : kWin - 1) - y;
        lk_vmcnt<later * ND>();
        // row y+PF into the image row y-1 used (its reads were consumed last iteration)
        if constexpr (y + PF < kWin) dma(std::integral_constant<int, (y + PF) % NB>{});
        __builtin_amdgcn_sched_barrier(0);
        lds_u2v* lE = (lds_u2v*)(ibuf(std::integral_constant<int, y % NB>{}) + el);
        uint32_t dw[10];
#pragma unroll
        for (int gi = 0; gi < 10; gi++) dw[gi] = lE[4 * gi].x;      // the D word of pair q.off + k + 4 gi
#pragma unroll
        for (int gi = 0; gi < 10; gi++) {
            const uint32_t d = dw[gi];
            const f2 f = {(float)(int16_t)d, (float)((int)d >> 16)};
            // the reference rounds each product to float, then adds (_mm_mul_ps, _mm_add_ps).
            // |Ix|, |Iy| <= 4080 (Scharr of u8, interpolated), so every product is below 2^24 and
            // exact in float: one fused multiply-add rounds exactly like the two operations
            sd = __builtin_elementwise_fma(f, f, sd);      // (Ix*Ix, Iy*Iy)
            s12 = __builtin_fmaf(f.x, f.y, s12);           // Ix*Iy
        }
    });
    const float a11 = ((quad_bcast<0>(sd.x) + quad_bcast<1>(sd.x)) + quad_bcast<2>(sd.x)) + quad_bcast<3>(sd.x);
    const float a12 = ((quad_bcast<0>(s12) + quad_bcast<1>(s12)) + quad_bcast<2>(s12)) + quad_bcast<3>(s12);
    const float a22 = ((quad_bcast<0>(sd.y) + quad_bcast<1>(sd.y)) + quad_bcast<2>(sd.y)) + quad_bcast<3>(sd.y);
    const float A11 = a11 * FLT_SCALE, A12 = a12 * FLT_SCALE, A22 = a22 * FLT_SCALE;
    float Dinv = 0.f;
    if (ok) {
        const float D = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - __builtin_sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                             (float)(2 * kWin * kWin);
        if (!(minEig < a.min_eig || D < FLT_EPSILON)) Dinv = 1.f / D;
    }
    if (q.valid && k == 0) Ab[(long long)pair * a.npts + q.gx * a.ny + q.gy] = make_float4(A11, A12, A22, Dinv);
}

// the gradient sums of one window (lane k: SSE lane k's partials) -> (A11, A12, A22, 1/D or 0),
// the quad combine ((P0+P1)+P2)+P3 and LKTrackerInvoker's minEig / determinant tests
__device__ __forceinline__ float4 lk_A_result(f2 sd, float s12, bool ok, float min_eig)
{
    constexpr float FLT_SCALE = 1.f / (1 << 20);
    const float a11 = ((quad_bcast<0>(sd.x) + quad_bcast<1>(sd.x)) + quad_bcast<2>(sd.x)) + quad_bcast<3>(sd.x);
    const float a12 = ((quad_bcast<0>(s12) + quad_bcast<1>(s12)) + quad_bcast<2>(s12)) + quad_bcast<3>(s12);
    const float a22 = ((quad_bcast<0>(sd.y) + quad_bcast<1>(sd.y)) + quad_bcast<2>(sd.y)) + quad_bcast<3>(sd.y);
    const float A11 = a11 * FLT_SCALE, A12 = a12 * FLT_SCALE, A22 = a22 * FLT_SCALE;
    float Dinv = 0.f;
    if (ok) {
        const float D = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - __builtin_sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                             (float)(2 * kWin * kWin);
        if (!(minEig < min_eig || D < FLT_EPSILON)) Dinv = 1.f / D;
    }
    return make_float4(A11, A12, A22, Dinv);
}

// ---- A pass per row strip.  Neighbouring grid rows of one residue class have windows that start
// `asp` plane rows apart (5 at pixel_step 10 above level 0, 10 at level 0), so every plane row lies
// in 40 / asp of them: k_lk_A re-reads each plane row that many times.  Here a wave owns S column
// groups (the G class members of a group, as in k_lk_A) over a strip of up to kAStripRows grid rows
// of one y-class, streams the strip's plane rows ONCE (same LDS-DMA row images), converts each
// element once, and adds it into the chains of every window containing the row: window j of the
// strip lives in accumulator slot j % NW (NW * asp >= 40, so a slot's windows never overlap) from
// its first row to its 40th, then is finished like k_lk_A's.  Each window's chains see exactly
// k_lk_A's operands in k_lk_A's order, so the sums are the same bits.
// grid: x -> (strip, column-group wave), y -> pair (XCD-remapped as one range)
template <int G, int UW, int NW>
__global__ __launch_bounds__(64) void k_lk_A_rows(LkArgs a, const uint8_t* __restrict__ cls, float4* __restrict__ Ab,
                                                  int* __restrict__ qctr, int level, int ncg)
{
    using Sh = LkShape<G, UW>;
    constexpr int LPS = Sh::LPS, S = Sh::S, ND = Sh::ND;
    __shared__ __attribute__((aligned(16))) uint32_t img0[ND * 256];
    __shared__ __attribute__((aligned(16))) uint32_t img1[ND * 256];
    __shared__ __attribute__((aligned(16))) uint32_t img2[ND * 256];

    const int lane = threadIdx.x, k = lane & 3, slot = lane / LPS, sl = lane % LPS;
    const int nw = gridDim.x;
    const int bid = xcd_remap(blockIdx.x + nw * blockIdx.y, nw * gridDim.y);
    const int pair = bid / nw, w = bid % nw;
    if (bid == 0 && lane < 8) qctr[(level * 8 + lane) * kCtrPad] = 0;   // k_lk_iter's queue heads
    const ClassLevel& C = a.plan.lv[level];
    const Level L = a.g.lv[level];
    const int ncw = (ncg + S - 1) / S;
    const int strip = w / ncw, cg = (w - strip * ncw) * S + slot;
    const int16_t* xo = a.ord + C.ord_off;
    const int16_t* yo = xo + C.nxp;
    const int r0 = a.ord[C.strip_off + 2 * strip], nr = a.ord[C.strip_off + 2 * strip + 1];
    const int asp = C.asp;
    const float scale = (float)(1. / (1 << level));
    const int m = (1 << level) - 1;
    // column geometry of this lane quad's point (group_geom's, with the strip's first row)
    const int gx0 = cg < ncg ? xo[cg * G] : -1;
    const int gxv = cg < ncg ? xo[cg * G + (sl >> 2)] : -1;
    const bool valid = gxv >= 0;
    const int gx = valid ? gxv : 0;
    const int ipx = (int)floorf((float)(gx * a.pixel_step) * scale - 19.5f);
    const int gy0 = yo[r0];
    const int ipx0 = (int)floorf((float)((gx0 >= 0 ? gx0 : 0) * a.pixel_step) * scale - 19.5f);
    const int cx = class_of(a.cmap, level, 0, ((gx0 >= 0 ? gx0 : 0) * a.pixel_step) & m);
    const int cy = class_of(a.cmap, level, 1, (gy0 * a.pixel_step) & m);
    const int ub = min(max(ipx0 + kPad, 0), C.PW - UW);
    const int off = min(max(ipx + kPad - ub, 0), UW - kWin);
    const uint32_t ubase = (uint32_t)(C.off + (long long)(cy * C.nrx + cx) * C.class_bytes) + 8u * (uint32_t)ub;
    const int ipy0 = (int)floorf((float)(gy0 * a.pixel_step) * scale - 19.5f);
    const int v00 = min(max(ipy0 + kPad, 0), C.UH - kWin);
    const int R = (nr - 1) * asp + kWin;                           // plane rows of the strip

    const __amdgpu_buffer_rsrc_t crs = buf_rsrc(cls + (long long)pair * a.plan.bytes_per_pair, a.plan.bytes_per_pair);
    const uint32_t rowb = (uint32_t)C.PW * 8;
    uint32_t uoff[ND];
    {
        const uint32_t mine = ubase + (uint32_t)v00 * rowb;
#pragma unroll
        for (int c = 0; c < ND; c++) {
            const int P = 1024 * c + 16 * lane;
            const int sp = P / (8 * UW), wb = P % (8 * UW);
            const uint32_t src = (uint32_t)__shfl((int)mine, (sp < S ? sp : 0) * LPS) + (uint32_t)wb;
            uoff[c] = sp < S ? src : 0x80000000u;
        }
    }
    auto ibuf = [&](auto bc) -> uint32_t* {
        constexpr int bb = decltype(bc)::value;
        if constexpr (bb == 0) return img0;
        else if constexpr (bb == 1) return img1;
        else return img2;
    };
    auto dma = [&](auto bc) {
        uint32_t* I = ibuf(bc);
#pragma unroll
        for (int c = 0; c < ND; c++) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(crs, (lds_ptr)(I + 256 * c), 16, (int)uoff[c], 0, 0, 0);
            uoff[c] += rowb;
        }
    };
    const int el = 2 * (slot * UW + off + k);

    // window slots: rin[s] = rows the slot's window has summed (-1: idle), jw[s] = its strip row
    f2 sd[NW];
    float s12[NW];
    int rin[NW], jw[NW];
#pragma unroll
    for (int s = 0; s < NW; s++) {
        sd[s] = f2{0.f, 0.f};
        s12[s] = 0.f;
        rin[s] = -1;
        jw[s] = 0;
    }
    int nextj = 0;
    auto finish = [&](int j, f2 sdv, float s12v) {
        const int gy = yo[r0 + j];
        const int ipy = (int)floorf((float)(gy * a.pixel_step) * scale - 19.5f);
        const bool ok = valid && !(ipx < -kWin || ipx >= L.w || ipy < -kWin || ipy >= L.h);
        const float4 r = lk_A_result(sdv, s12v, ok, a.min_eig);
        if (valid && k == 0) Ab[(long long)pair * a.npts + gx * a.ny + gy] = r;
    };
    // one plane row: its elements (loaded once), then every window that contains it
    auto row = [&](int t, auto bc) {
        // row t has landed once only row t + 1's pieces may be outstanding
        if (t + 1 < R) lk_vmcnt<ND>();
        else lk_vmcnt0();
        if (t + 2 < R) dma(std::integral_constant<int, (decltype(bc)::value + 2) % 3>{});
        __builtin_amdgcn_sched_barrier(0);
        lds_u2v* lE = (lds_u2v*)(ibuf(bc) + el);
        uint32_t dw[10];
#pragma unroll
        for (int gi = 0; gi < 10; gi++) dw[gi] = lE[4 * gi].x;
        f2 f[10];
#pragma unroll
        for (int gi = 0; gi < 10; gi++) f[gi] = f2{(float)(int16_t)dw[gi], (float)((int)dw[gi] >> 16)};
        if (nextj < nr && t == nextj * asp) {   // window nextj starts here (slot nextj % NW is free)
            static_for<0, NW>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if (nextj % NW == s) {
                    sd[s] = f2{0.f, 0.f};
                    s12[s] = 0.f;
                    rin[s] = 0;
                    jw[s] = nextj;
                }
            });
            nextj++;
        }
        static_for<0, NW>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            if (rin[s] >= 0) {
#pragma unroll
                for (int gi = 0; gi < 10; gi++) {
                    // products exact in float (|Ix|, |Iy| <= 4080): the FMA rounds like k_lk_A's
                    sd[s] = __builtin_elementwise_fma(f[gi], f[gi], sd[s]);
                    s12[s] = __builtin_fmaf(f[gi].x, f[gi].y, s12[s]);
                }
                if (++rin[s] == kWin) {
                    finish(jw[s], sd[s], s12[s]);
                    rin[s] = -1;
                }
            }
        });
    };
    dma(std::integral_constant<int, 0>{});
    if (R > 1) dma(std::integral_constant<int, 1>{});
#pragma unroll 1
    for (int t = 0; t < R; t += 3) {
        row(t, std::integral_constant<int, 0>{});
        if (t + 1 < R) row(t + 1, std::integral_constant<int, 1>{});
        if (t + 2 < R) row(t + 2, std::integral_constant<int, 2>{});
    }
}

// ---- Newton iterations.  grid: x -> persistent wave (a multiple of 8).  The level's work list
// is every pair's groups, pair-major; it is cut into 8 contiguous ranges, one per XCD (blocks are
// dealt to the XCDs round-robin), each with its own queue head.  An XCD's waves thus work on
// neighbouring groups of one pair at a time, whose class-plane rows its L2 holds -- per-pair
// queues spread every XCD over several pairs at once and doubled the L2 misses.  Levels run as
// separate launches from maxLevel down to 0; the position carried between them is next_pts (the
// reference's nextPts[ptidx], stored every level).
//
// Rows arrive by LDS-DMA (buffer_load ... lds), NB - 1 rows ahead, retired by an explicit vmcnt
// at the top of each row (the compiler does not track LDS-DMA completion; it only orders LDS
// reads after DMA into the same __shared__ object, hence one array per row buffer):
//  * the union rows of all S slots: ND pieces of 1 KiB.  A piece's LDS destination is fixed
//    (lane L writes bytes 16L..16L+15), so lane L of piece c loads the 16 B of whichever slot and
//    pair offset that position holds in the [slot][UW][D, C] image -- source offsets are
//    per-lane and refreshed once per iteration;
//  * each lane quad's J row segment (16 B per lane, 12 of the quad's 16 dwords used).
// A lane then reads its 10 chain pairs with ds_read_b64 (kept apart: a merged ds_read2_b64
// would halve the LDS rate) and the quad's J dwords with three ds_read_b128.  D and C travel as
// one pair, so a chain element is one 2-cycle LDS access (it was two read2_b32 halves).
template <int G, int UW, bool DF>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kLkIterWavesPerEU, 8))) void k_lk_iter(
    LkArgs a, const uint8_t* __restrict__ cls, const float4* __restrict__ Ab, int* __restrict__ qctr, int level,
    int ngroups, int batch)
{
    using Sh = LkShape<G, UW>;
    constexpr int LPS = Sh::LPS, S = Sh::S, ND = Sh::ND;
    constexpr float HALFW = 19.5f;
    constexpr float FLT_SCALE = 1.f / (1 << 20);
    constexpr int UB = S * UW;                                    // (D, C) pairs per union buffer
    // Row buffers: window rows are fetched NB - 1 ahead of the row being summed.  One __shared__
    // array per buffer, so that the compiler sees a row's LDS reads and the DMA into another
    // buffer as disjoint: with one [NB][...] array it put a vmcnt(0) -- a wait for the DMA just
    // issued -- in front of every read that followed a DMA, and no row overlapped its fetch.
    constexpr int NB = MDX_LK_NB;
    static_assert(NB == 2 || NB == 3, "row buffers");
    static_assert(kWin == 40, "row schedule (20 row pairs; 6 row sextets + 4)");
    __shared__ __attribute__((aligned(16))) uint32_t dU0[2 * UB];   // [slot][UW][D, C]
    __shared__ __attribute__((aligned(16))) uint32_t dU1[2 * UB];
    __shared__ __attribute__((aligned(16))) uint32_t dU2[NB > 2 ? 2 * UB : 4];
    __shared__ __attribute__((aligned(16))) uint32_t dJ0[256];      // [quad][16]
    __shared__ __attribute__((aligned(16))) uint32_t dJ1[256];
    __shared__ __attribute__((aligned(16))) uint32_t dJ2[NB > 2 ? 256 : 4];

    const int lane = threadIdx.x, k = lane & 3, slot = lane / LPS, sl = lane % LPS;
    const unsigned long long smask = ((1ull << LPS) - 1) << (slot * LPS);
    const unsigned long long t_start = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const int xcd = blockIdx.x & 7;
    // DF = false (levels in sequence, no dataflow, no recompute): the hand-off, give-up and recompute
    // code below folds away, so the plain kernel carries none of it
    int* const a_done = DF ? a.done : nullptr;
    int* const a_lflags = DF ? a.lflags : nullptr;
    const int a_redo = DF ? a.redo : 0;
    const int dep_groups = DF ? a.dep_groups : 0;
    const int dep_points = DF ? a.dep_points : 0;
    const long long T = (long long)batch * ngroups;
    const long long cb = T * xcd / 8, ce = T * (xcd + 1) / 8;     // this XCD's range of the work list
    const int p0 = (int)(cb / ngroups);
    const uint32_t off0 = (uint32_t)(cb - (long long)p0 * ngroups);   // cb's group within pair p0
    const int np = ce > cb ? (int)((ce - 1) / ngroups) - p0 + 1 : 1;
    int* ctr = qctr + (level * 8 + xcd) * kCtrPad;
    if (a_redo) {
        // the level's recompute: only if it gave up, or the coarser level was recomputed (its
        // carried points changed after this level read them); levels then run in sequence
        int need = __hip_atomic_load(a_lflags + (kLkFlagGiveup + level) * kCtrPad, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        if (level < a.maxl)
            need |= __hip_atomic_load(a_lflags + (kLkFlagRedone + level + 1) * kCtrPad, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
        if (!need) return;
        if (blockIdx.x == 0 && lane == 0) {
            __hip_atomic_store(a_lflags + (kLkFlagRedone + level) * kCtrPad, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(a.err + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ctr = a_lflags + (kLkFlagQueue + level * 8 + xcd) * kCtrPad;
    }
    // this level's give-up flag (dataflow): set by the first wait that gives up or by the gate
    int* const giveup = a_lflags ? a_lflags + (kLkFlagGiveup + level) * kCtrPad : nullptr;
    const ClassLevel& C = a.plan.lv[level];
    const Level L = a.g.lv[level];
    // buffer addressing: descriptors over the range's class slabs and next-frame pyramids (the
    // host keeps them below 2 GB), 32-bit lane offsets
    const uint8_t* const cls_base = cls + (long long)p0 * a.plan.bytes_per_pair;
    const uint32_t cls_bytes = (uint32_t)(np * a.plan.bytes_per_pair);
    const uint32_t rowb = (uint32_t)C.PW * 8;
    const int pitch = L.pitch;
    const uint8_t* const j_base = a.pyr2 + (long long)p0 * a.g.img_bytes;
    const uint32_t j_bytes = (uint32_t)(np * a.g.img_bytes);
    const uint32_t jbase = (uint32_t)(L.img_off + L.core());
    const float scale = (float)(1. / (1 << level));

    // slot state (uniform over the slot's lanes)
    bool live = false, dead = false;
    int j = 0;
    // point state
    GroupGeom q{};
    int pt = 0, pair = 0;
    long long po = 0;
    uint32_t jrel = 0;                                            // pair's pyramid in jrs
    float A11 = 0.f, A12 = 0.f, A22 = 0.f, Dinv = 0.f;
    float nx = 0.f, ny = 0.f, npx = 0.f, npy = 0.f, pdx = 0.f, pdy = 0.f;
    bool act = false, gave_up = false;
    int status = 1, iters = 0;

    auto retire = [&]() {
        if (level == 0 && q.valid && status) {
            const int fx = (int)floorf(npx - HALFW), fy = (int)floorf(npy - HALFW);
            if (fx < -kWin || fx >= L.w || fy < -kWin || fy >= L.h) status = 0;
        }
        if (q.valid && k == 0) {
            if (a.dbg)
                a.dbg[((long long)pair * a.g.nlev + level) * a.npts + pt] = make_float4(npx, npy, (float)iters, (float)status);
            const float2 v = make_float2(npx, npy);
            float* dst = (a.carry && level > 0) ? a.carry + level * a.carry_lstride : a.next_pts;
            if (a_done)   // read by the next level's launch while this one runs: write-through (sc1)
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst) + po,
                                   __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                reinterpret_cast<float2*>(dst)[po] = v;
            if (level == 0) a.status[po] = (uint8_t)status;
        }
        if (a_done && level > 0) {
            // the group's points have their level result: once this wave's stores are done, one
            // lane of the slot counts the group for its pair (MI355X_MICROARCH.md hand-off: sc1
            // stores, vmcnt(0), agent atomic; the reader polls and loads sc1) -- or, per-point
            // dataflow, each point's lane stamps the point with the call's epoch
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (dep_points) {
                if (q.valid && k == 0)
                    __hip_atomic_store(a.pflags + level * a.pf_lstride + po, a.epoch, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            } else if (sl == 0) {
                __hip_atomic_fetch_add(a_done + (level * a.done_stride + pair) * kCtrPad, 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    };

    for (;;) {
        // ---- refill: each slot without a live group takes the next one; a group with no point
        // left to iterate retires at once
        for (;;) {
            const bool need = !live && !dead;
            if (!__any(need)) break;
            if (need) {
                int gi = 0;
                if (sl == 0) gi = atomicAdd(ctr, 1);
                gi = __shfl(gi, slot * LPS);
                if (cb + gi >= ce) {
                    dead = true;
                } else {
                    // position in the XCD's range relative to its first pair: 32-bit division
                    const uint32_t r = off0 + (uint32_t)gi, dp = r / (uint32_t)ngroups;
                    pair = p0 + (int)dp;
                    q = group_geom<G, UW>(a, C, level, (int)(r - dp * (uint32_t)ngroups), sl);
                    q.ubase += (uint32_t)((long long)(pair - p0) * a.plan.bytes_per_pair);
                    jrel = (uint32_t)((long long)(pair - p0) * a.g.img_bytes);
                    pt = q.gx * a.ny + q.gy;
                    po = (long long)pair * a.npts + pt;
                    const float4 Av = q.valid ? Ab[po] : make_float4(0.f, 0.f, 0.f, 0.f);
                    A11 = Av.x;
                    A12 = Av.y;
                    A22 = Av.z;
                    Dinv = Av.w;
                    if (level == a.maxl) {
                        npx = (float)(q.gx * a.pixel_step) * scale;
                        npy = (float)(q.gy * a.pixel_step) * scale;
                    } else {
                        float2 p = make_float2(0.f, 0.f);
                        const float* src = a.carry ? a.carry + (level + 1) * a.carry_lstride : a.next_pts;
                        const bool wait_pt = dep_points && level < a.maxl;
                        if (dep_groups || wait_pt) {
                            // dataflow: the coarser level may still run -- wait until every group of
                            // this pair has retired there (per-point dataflow: until this lane's
                            // point has; bounded: the coarser level's waves are resident and drain
                            // their queue), then read the carried points past L1.  A wait that
                            // gives up abandons the level (every later wait sees the flag): its
                            // groups drain without computing, and its recompute launch
                            // (launch_lk_v2) runs it again once the coarser level is done.
                            const bool waiter = wait_pt ? (q.valid && k == 0) : (sl == 0);
                            if (waiter && !gave_up) {
                                // polls back off (1 .. 16 sleeps between loads): thousands of
                                // waiting waves polling one line would load its L2 channel
                                const int* d = wait_pt ? a.pflags + (level + 1) * a.pf_lstride + po
                                                       : a_done + ((level + 1) * a.done_stride + pair) * kCtrPad;
                                const int target = wait_pt ? a.epoch : dep_groups;
                                int slept = 0, gap = 1;
                                bool mine = false;
                                if (a.spin_max < 0) mine = true;   // fault injection (tests)
                                while (!mine &&
                                       __hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                                    if (slept >= a.spin_max) {
                                        mine = true;
                                        break;
                                    }
                                    if (__hip_atomic_load(giveup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0) {
                                        gave_up = true;   // another wait (or the gate) gave up
                                        break;
                                    }
                                    for (int i = 0; i < gap; i++) __builtin_amdgcn_s_sleep(8);
                                    slept += gap;
                                    gap = gap < 16 ? 2 * gap : 16;
                                }
                                if (mine) {
                                    gave_up = true;
                                    __hip_atomic_fetch_add(giveup, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    __hip_atomic_fetch_add(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                }
                            }
                            // The hand-off is MI355X_MICROARCH.md's measured form (table row 1):
                            // every carried point stored sc1, each storing wave's vmcnt(0) before
                            // one lane's agent atomic add, the consumer's sc1 poll, then sc1
                            // loads only -- no acquire fence needed.  This compiler-only fence
                            // (wavefront scope: no instruction) keeps the loads below the poll.
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                            if (q.valid)
                                p = __builtin_bit_cast(float2, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(src) + po,
                                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        } else if (q.valid) {
                            p = reinterpret_cast<const float2*>(src)[po];
                        }
                        npx = p.x * 2.f;
                        npy = p.y * 2.f;
                    }
                    act = Dinv > 0.f;   // real point, window inside, eigenvalue / determinant tests passed
                    // an abandoned level retires its groups at once (its recompute redoes them)
                    if ((dep_groups || dep_points) && (__ballot(gave_up) & smask)) act = false;
                    status = (level == 0 && q.valid && !act) ? 0 : 1;
                    nx = npx - HALFW;
                    ny = npy - HALFW;
                    pdx = 0.f;
                    pdy = 0.f;
                    iters = 0;
                    j = 0;
                    live = (__ballot(act) & smask) != 0 && a.max_iters > 0;
                    if (!live) retire();
                }
            }
        }
        if (!__any(live)) break;

        // ---- one Newton iteration of every live group.  Lanes that are not iterating (or fail
        // the bounds test) run the row loop on a safe address and drop the result, so the loop
        // is wave-uniform (it also carries every slot's staging).
        f2 acc = {0.f, 0.f};
        if (act) iters++;
        int inx = (int)floorf(nx), iny = (int)floorf(ny);
        if (act && (inx < -kWin || inx >= L.w || iny < -kWin || iny >= L.h)) {
            act = false;
            if (level == 0) status = 0;
        }
        if (!act) { inx = 0; iny = 0; }
        const float fa = nx - (float)inx, fb = ny - (float)iny;
        int v00, v01, v10, v11;
        lk_weights(fa, fb, v00, v01, v10, v11);
        // signed: w11 = 16384 - w00 - w01 - w10 can be -1 after rounding
        const s2 W0 = {(short)v00, (short)v01};
        const s2 W1 = {(short)v10, (short)v11};
        const int o = (inx & 3) + k;
        const unsigned sel = (unsigned)o | 0x0c00u | ((unsigned)(o + 1) << 16) | 0x0c000000u;
        // this lane's 16 J bytes: the quad's first 12 dwords cover every lane's taps
        uint32_t joff = jrel + jbase + (uint32_t)(iny * pitch + (inx & ~3) + 16 * k);
        // union sources: lane L of piece c fills image bytes 1024c + 16L, i.e. slot sp's pair bytes wb
        uint32_t uoff[ND];
        {
            const uint32_t mine = q.ubase + (uint32_t)q.v0 * rowb;
#pragma unroll
            for (int c = 0; c < ND; c++) {
                const int P = 1024 * c + 16 * lane;
                const int sp = P / (8 * UW), wb = P % (8 * UW);
                uoff[c] = (uint32_t)__shfl((int)mine, sp * LPS) + (uint32_t)wb;
            }
        }
        auto ubuf = [&](auto bc) -> uint32_t* {
            constexpr int bb = decltype(bc)::value;
            if constexpr (bb == 0) return dU0;
            else if constexpr (bb == 1) return dU1;
            else return dU2;
        };
        auto jbuf = [&](auto bc) -> uint32_t* {
            constexpr int bb = decltype(bc)::value;
            if constexpr (bb == 0) return dJ0;
            else if constexpr (bb == 1) return dJ1;
            else return dJ2;
        };
        // window row yr of the union / J images: the per-lane offsets stay fixed and the row
        // advance moves the descriptor's base (and shrinks its size by as much, so the range check
        // keeps the same end): scalar work instead of a VALU add per piece and row
        auto dma_union = [&](auto bc, int yr) {
            uint32_t* U = ubuf(bc);
            const uint32_t adv = (uint32_t)yr * rowb;
            const __amdgpu_buffer_rsrc_t r = buf_rsrc32(cls_base + adv, cls_bytes - adv);
#pragma unroll
            for (int c = 0; c < ND; c++) {
                if (c < ND - 1 || 1024 * c + 16 * lane < Sh::BYTES)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)(U + 256 * c), 16, (int)uoff[c], 0, 0, 0);
            }
        };
        auto dma_j = [&](auto bc, int yr) {
            // the quad's taps span 44 bytes: lanes 0-2 carry them, lane 3 stays idle
            const uint32_t adv = (uint32_t)(yr * pitch);
            const __amdgpu_buffer_rsrc_t r = buf_rsrc32(j_base + adv, j_bytes - adv);
            if (k < 3) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)jbuf(bc), 16, (int)joff, 0, 0, 0);
        };
        const int jl = (lane >> 2) * 16, el = 2 * (slot * UW + q.off + k);
        auto read_j = [&](auto bc, uint32_t (&rj)[11]) {
            lds_u4v* lJ = (lds_u4v*)(jbuf(bc) + jl);
            const v4u j0 = lJ[0], j1 = lJ[1], j2 = lJ[2];
            rj[0] = j0.x; rj[1] = j0.y; rj[2] = j0.z; rj[3] = j0.w;
            rj[4] = j1.x; rj[5] = j1.y; rj[6] = j1.z; rj[7] = j1.w;
            rj[8] = j2.x; rj[9] = j2.y; rj[10] = j2.z;
        };
        // union row r and J row r live in buffer r % NB
        constexpr int D = NB - 1;
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        // taps of the current window row (pa) are the previous row's lower taps (pb)
        s2 pa[10], pb[10];
        dma_union(I0{}, 0);
        dma_j(I0{}, 0);
        dma_j(I1{}, 1);
        if constexpr (D == 2) {
            dma_union(I1{}, 1);
            dma_j(I2{}, 2);
        }
        lk_vmcnt<(D - 1) * (ND + 1)>();
        {
            uint32_t rj[11];
            read_j(I0{}, rj);
#pragma unroll
            for (int gi = 0; gi < 10; gi++) pa[gi] = __builtin_bit_cast(s2, __builtin_amdgcn_perm(rj[gi + 1], rj[gi], sel));
        }
        // row y (y % period = R): wait until union row y and J row y+1 have landed -- the loads
        // issued for later rows (W of them) may stay in flight -- then fetch union row y+D and J
        // row y+D+1 into the buffers rows y-1 / y (already summed) used, and sum the row.  An
        // opaque use of acc pins each row's arithmetic before the next row's wait.
        auto row = [&](int y, auto Rc, auto Wc, s2 (&up)[10], s2 (&lo)[10]) {
            constexpr int R = decltype(Rc)::value, W = decltype(Wc)::value;
            if (y) lk_vmcnt<W>();
            auto fetch = [&]() {
                if (y + D < kWin) dma_union(std::integral_constant<int, (R + D) % NB>{}, y + D);
                if (y + D + 1 <= kWin) dma_j(std::integral_constant<int, (R + D + 1) % NB>{}, y + D + 1);
                __builtin_amdgcn_sched_barrier(0);
            };
#if !MDX_LK_RFIRST
            fetch();
#endif
            // the row's LDS reads back to back (their latencies overlap), then the arithmetic
            uint32_t rj[11];
            read_j(std::integral_constant<int, (R + 1) % NB>{}, rj);
            lds_u2v* lE = (lds_u2v*)(ubuf(std::integral_constant<int, R % NB>{}) + el);
            v2u dcs[10];
#pragma unroll
            for (int gi = 0; gi < 10; gi++) dcs[gi] = lE[4 * gi];
#if MDX_LK_RFIRST
            __builtin_amdgcn_sched_barrier(0);
            fetch();
#endif
#pragma unroll
            for (int gi = 0; gi < 10; gi++) {
                const v2u dc = dcs[gi];
                lo[gi] = __builtin_bit_cast(s2, __builtin_amdgcn_perm(rj[gi + 1], rj[gi], sel));
                // (J*32 - I*32) exactly as the reference's CV_DESCALE(...) - I
                const int jd = __builtin_amdgcn_sdot2(up[gi], W0, __builtin_amdgcn_sdot2(lo[gi], W1, (int)dc.y, false),
                                                      false) >> 9;
                const float fd = (float)jd;
                const f2 f = {(float)(int16_t)dc.x, (float)((int)dc.x >> 16)};
                acc = acc + f * fd;
            }
            asm volatile("" : "+v"(acc));
        };
        if constexpr (NB == 2) {
            using W = std::integral_constant<int, 0>;
#pragma unroll 1
            for (int y = 0; y < kWin; y += 2) {
                row(y, I0{}, W{}, pa, pb);
                row(y + 1, I1{}, W{}, pb, pa);
            }
        } else {
            using W = std::integral_constant<int, ND + 1>;
#pragma unroll 1
            for (int y = 0; y < 36; y += 6) {
                row(y, I0{}, W{}, pa, pb);
                row(y + 1, I1{}, W{}, pb, pa);
                row(y + 2, I2{}, W{}, pa, pb);
                row(y + 3, std::integral_constant<int, 3>{}, W{}, pb, pa);
                row(y + 4, std::integral_constant<int, 4>{}, W{}, pa, pb);
                row(y + 5, std::integral_constant<int, 5>{}, W{}, pb, pa);
            }
            row(36, I0{}, W{}, pa, pb);
            row(37, I1{}, W{}, pb, pa);
            row(38, I2{}, W{}, pa, pb);
            row(39, std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{}, pb, pa);
        }
        if (!act) acc = f2{0.f, 0.f};
        // b = (P0+P2) + (P1+P3) across the quad; inactive quads compute values they ignore
        const float b1s = (quad_bcast<0>(acc.x) + quad_bcast<2>(acc.x)) + (quad_bcast<1>(acc.x) + quad_bcast<3>(acc.x));
        const float b2s = (quad_bcast<0>(acc.y) + quad_bcast<2>(acc.y)) + (quad_bcast<1>(acc.y) + quad_bcast<3>(acc.y));
        if (act) {
            const float b1 = b1s * FLT_SCALE, b2 = b2s * FLT_SCALE;
            const float dx = (A12 * b2 - A22 * b1) * Dinv;
            const float dy = (A12 * b1 - A11 * b2) * Dinv;
            if (a.dbg && pt == a.dbg_pt && pair == 0) {
                float4* t = a.dbg + (long long)a.g.nlev * a.npts + (level * 16 + j) * 4;
                if (k == 0) { t[0] = make_float4(b1s, b2s, dx, dy); t[1] = make_float4(nx, ny, A11, Dinv); }
                t[2 + (k >> 1)] = make_float4(k & 1 ? 0.f : acc.x, k & 1 ? 0.f : acc.y, acc.x, acc.y);
            }
            nx = nx + dx;
            ny = ny + dy;
            npx = nx + HALFW;
            npy = ny + HALFW;
            if ((double)dx * dx + (double)dy * dy <= a.eps2) {
                act = false;
            } else if (j > 0 && fabs((double)fabsf(dx + pdx)) < 0.01 && fabs((double)fabsf(dy + pdy)) < 0.01) {
                npx = npx - dx * 0.5f;
                npy = npy - dy * 0.5f;
                act = false;
            }
            pdx = dx;
            pdy = dy;
        }
        if (live) {
            j++;
            if ((__ballot(act) & smask) == 0 || j >= a.max_iters) {
                live = false;
                retire();
            }
        }
    }
    if (a.dbg && lane == 0 && blockIdx.x < kLkDbgWaves) {   // debug mode only: wave lifetimes
        uint4* st = reinterpret_cast<uint4*>(a.dbg + (long long)batch * a.g.nlev * a.npts + kLkDbgStampOff) +
                    (long long)level * kLkDbgWaves + blockIdx.x;
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        *st = make_uint4((uint32_t)t_start, (uint32_t)(t_start >> 32), (uint32_t)t_end, (uint32_t)(t_end >> 32));
    }
}

// Dataflow gate: one wave, launched on the next level's stream right before that level's
// iteration launch.  It returns once, on every XCD, the coarser level's queue has been handed out
// (the start of its tail) and the first pair of the XCD's next-level range has finished the
// coarser level (its first groups can run at once).  The next level's persistent waves are then
// dispatched only into the slots the tail frees, and find ready work there.  Without the gate the
// next level, launched beside the coarser level's whole queue, took half the chip and spun (both
// launches ~2x slower); gated on the queues alone, one pair per XCD (4K x 8) left every next-level
// wave polling its pair's counter (LK 3x slower).  Bounded like the group waits, and counted the
// same way when the bound is hit (err[1]); the gated level is then abandoned at once (giveup: its
// flag), since its waits could only time out too, and its recompute launch runs it.
__global__ __launch_bounds__(64) void k_lk_gate(const int* __restrict__ qctr, long long T, const int* __restrict__ done,
                                                int dep_groups, int ngroups_next, long long T_next, int* __restrict__ err,
                                                int spin_max, int* __restrict__ giveup)
{
    const int x = threadIdx.x;
    bool ready = true;   // lanes 0..7: XCD x's ranges
    if (x < 8) {
        const long long cb = T * x / 8, ce = T * (x + 1) / 8;
        const long long cbn = T_next * x / 8;
        const int pf = cbn < T_next ? (int)(cbn / ngroups_next) : -1;
        ready = false;
        for (int t = 0; t < spin_max; t++) {
            const bool dry = __hip_atomic_load(qctr + x * kCtrPad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ce - cb;
            const bool first = pf < 0 || __hip_atomic_load(done + pf * kCtrPad, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) >= dep_groups;
            if (dry && first) {
                ready = true;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
    }
    if (!__all(ready) && x == 0) {   // one count per gate
        __hip_atomic_fetch_add(err + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(giveup, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// persistent waves for k_lk_iter: what the current device keeps resident at once (cached per
// device; contexts on several devices may launch from several host threads)
template <int G, int UW, bool DF>
static int lk_iter_resident()
{
    constexpr int kDevs = 64;
    static std::atomic<int> cached[kDevs];
    int dev = 0;
    (void)hipGetDevice(&dev);
    int v = dev >= 0 && dev < kDevs ? cached[dev].load(std::memory_order_relaxed) : 0;
    if (!v) {
        int ncu = 0, nb = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_lk_iter<G, UW, DF>, 64, 0);
        v = std::max(1, ncu) * std::max(1, nb);
        if (dev >= 0 && dev < kDevs) cached[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

template <int G, int UW>
static int lk_groups(const LkArgs& a, int l)
{
    return (a.plan.lv[l].nxp / G) * a.nyg;
}

template <int G, int UW>
static void launch_A(hipStream_t s, int batch, const LkArgs& a, const uint8_t* cls, float4* Ab, int* qctr, int l)
{
    constexpr int S = LkShape<G, UW>::S;
    const int ngroups = lk_groups<G, UW>(a, l);
    const dim3 grid((ngroups + S - 1) / S, batch);
    hipLaunchKernelGGL((k_lk_A<G, UW>), grid, dim3(64), 0, s, a, cls, Ab, qctr, l, ngroups);
}

template <int G, int UW>
static void launch_A_rows(hipStream_t s, int batch, const LkArgs& a, const uint8_t* cls, float4* Ab, int* qctr, int l)
{
    constexpr int S = LkShape<G, UW>::S;
    const ClassLevel& C = a.plan.lv[l];
    const int ncg = C.nxp / G;
    const dim3 grid(((ncg + S - 1) / S) * C.nstrip, batch);
    if (C.asp >= 10)
        hipLaunchKernelGGL((k_lk_A_rows<G, UW, 4>), grid, dim3(64), 0, s, a, cls, Ab, qctr, l, ncg);
    else
        hipLaunchKernelGGL((k_lk_A_rows<G, UW, 8>), grid, dim3(64), 0, s, a, cls, Ab, qctr, l, ncg);
}

template <int G, int UW>
static void launch_iter(hipStream_t s, int batch, const LkArgs& a, const uint8_t* cls, const float4* Ab, int* qctr,
                        int l)
{
    constexpr int S = LkShape<G, UW>::S;
    const int ngroups = lk_groups<G, UW>(a, l);
    // persistent waves, a multiple of 8 so that every XCD range has waves.  Dataflow: each launch
    // leaves part of the chip free, for the aux stream's class planes and A sums of the next level
    // (which must be done before that level's launch can start) and for the coarser level's
    // launch that this one may wait on
    const int need = (int)std::min<long long>(((long long)batch * ngroups + S - 1) / S, 1 << 30);
    const bool df = a.done || a.redo || a.lflags || a.dep_groups || a.dep_points;
    int res = df ? lk_iter_resident<G, UW, true>() : lk_iter_resident<G, UW, false>();
    if (a.done) res = res * std::min(std::max(a.flow_cap, 10), 100) / 100;   // the context's (MDX_LK_CAP)
    int W = std::max(8, std::min((need + 7) / 8, res / 8) * 8);
    if (a.redo) W = std::max(8, std::min(W, kLkRedoWaves));
    if (df) hipLaunchKernelGGL((k_lk_iter<G, UW, true>), dim3(W), dim3(64), 0, s, a, cls, Ab, qctr, l, ngroups, batch);
    else hipLaunchKernelGGL((k_lk_iter<G, UW, false>), dim3(W), dim3(64), 0, s, a, cls, Ab, qctr, l, ngroups, batch);
}

hipError_t launch_lk_v2(hipStream_t s, hipStream_t aux, hipEvent_t* ev, int batch, const LkArgs& a, uint8_t* cls,
                        float4* Ab, int* qctr, hipEvent_t prev_ready, hipStream_t s2, hipEvent_t* flow_ev, int* done,
                        hipEvent_t* lvl_done, int parity, hipEvent_t out_free, hipEvent_t* redo_ev)
{
    // An XCD range spans at most ceil(n/8) + 1 pairs; its class slabs (and pyramids) must stay
    // addressable by 32-bit buffer offsets, so very large batches of large frames run in
    // sub-batches (the plan already guarantees one pair's slab fits).
    const long long span = std::max(a.plan.bytes_per_pair, a.g.img_bytes);
    int sub = batch;
    while (sub > 1 && ((sub + 7) / 8 + 1) * span > 0x7fff0000LL) sub = std::max(1, sub / 2);
    if (a.max_sub > 0) sub = std::max(1, std::min(sub, a.max_sub));   // MDX_LK_SUB (tests), read at mdx_create
    if (sub < batch) parity = 0;   // sub-batches follow everything on s (their slabs are reused)
    // Class planes and A sums depend on the previous frame only, not on the flow: with an aux
    // stream they run ahead (level L-1's while level L iterates, filling that kernel's tail);
    // every level has its own class planes, A buffer and queue heads, so nothing is overwritten
    // while still in use.
    hipStream_t sa = aux ? aux : s;
    for (int p = 0, si = 0; p < batch; p += sub, si++) {
        const int nb = std::min(sub, batch - p);
        LkArgs b = a;
        b.pyr1 = a.pyr1 + (long long)p * a.g.img_bytes;
        b.pyr2 = a.pyr2 + (long long)p * a.g.img_bytes;
        b.der = a.der + (long long)p * a.g.der_words;
        b.next_pts = a.next_pts + (long long)p * a.npts * 2;
        b.carry = a.carry ? a.carry + (long long)p * a.npts * 2 : nullptr;   // carry_lstride: whole batch
        b.pflags = a.pflags ? a.pflags + (long long)p * a.npts : nullptr;      // pf_lstride: whole batch
        b.status = a.status + (long long)p * a.npts;
        if (p) b.dbg = nullptr;   // the trace covers the first sub-batch
        uint8_t* bcls = cls + (long long)p * a.plan.bytes_per_pair;
        int* bq = qctr + si * kMaxLevels * 8 * kCtrPad;
        if (aux) {
            hipEvent_t ready = prev_ready;
            if (!ready || p) {   // later sub-batches follow everything on s (their slabs are reused)
                if (hipError_t e = hipEventRecord(ev[kMaxLevels], s)) return e;
                ready = ev[kMaxLevels];
            }
            if (hipError_t e = hipStreamWaitEvent(sa, ready, 0)) return e;
        }
        for (int l = a.maxl; l >= 0; l--) {
            const ClassLevel& C = a.plan.lv[l];
            if (aux && lvl_done) {   // the previous call's level-l iterations read these planes / sums
                if (hipError_t e = hipStreamWaitEvent(sa, lvl_done[l], 0)) return e;
            }
            LkClassArgs ca;
            ca.g = a.g;
            ca.plan = a.plan;
            ca.rlist = a.rlist;
            ca.level = l;
            if (C.nrx * C.nry <= 4) {
                // the finest levels: derivatives computed inside the class kernel, no Scharr planes
                const dim3 grid(((a.g.lv[l].w + 2 * kPad) / 4 + 63) / 64, C.vhi - C.vlo, nb);
                hipLaunchKernelGGL(k_lk_class_fused, grid, dim3(64), 0, sa, b.pyr1, bcls, ca);
            } else {
                const dim3 grid(((a.g.lv[l].w + 2 * kPad) / 4 + 63) / 64, C.vhi - C.vlo, nb * C.nrx * C.nry);
                // this level's Scharr planes (the caller left them to us): on the aux stream, so
                // they too run while the coarser levels iterate
                // (the derivative rows the class planes read: v, v + 1 for plane rows v in [vlo, vhi))
                if (hipError_t e = launch_scharr(sa, nb, b.pyr1, const_cast<uint32_t*>(b.der), a.g, l, C.vlo, C.vhi + 1))
                    return e;
                hipLaunchKernelGGL(k_lk_class, grid, dim3(64), 0, sa, b.pyr1, b.der, bcls, ca);
            }
            float4* bA = Ab + ((long long)l * batch + p) * a.npts;
            const int G = C.G, UW = C.UW;
            switch (G * 1000 + UW) {
#define LK_CASE(g, uw)                                                              \
    case g * 1000 + uw:                                                             \
        if (C.asp) launch_A_rows<g, uw>(sa, nb, b, bcls, bA, bq, l);               \
        else launch_A<g, uw>(sa, nb, b, bcls, bA, bq, l);                          \
        break;
                LK_SHAPES
#undef LK_CASE
            default: return hipErrorInvalidValue;
            }
            if (aux) {
                if (hipError_t e = hipEventRecord(ev[l], sa)) return e;
            }
        }
        // dataflow: every XCD's work range must hold whole pairs (the hand-off stays in one L2) and
        // no two pairs' carried points may share a 128-B line; with one pair per XCD (batch 8) the
        // next level can only start once the whole level is done there, and the dataflow measured
        // 1.5% slower than levels in sequence, so it needs at least two
        const bool flow_ok = aux && s2 && flow_ev && done && redo_ev && a.err && b.carry &&
                             (reinterpret_cast<uintptr_t>(b.carry) & 127) == 0 && (a.carry_lstride % 32) == 0;
        // per pair (groups wait for their pair's whole coarser level) where every XCD range holds
        // two or more whole pairs; per point (groups wait for their own points) for small batches
        // -- a single pair's level would otherwise wait for the coarser level's slowest group
        const bool flow_pair = flow_ok && !a.pflow_force && nb % 8 == 0 && nb >= 16 && a.npts % 16 == 0 &&
                               (reinterpret_cast<uintptr_t>(b.next_pts) & 127) == 0;
        const bool flow_pt = flow_ok && !flow_pair && b.pflags;
        const bool flow = flow_pair || flow_pt;
        int* lflags = flow ? done + (long long)kMaxLevels * nb * kCtrPad : nullptr;
        // the even levels' stream (the first level's) and the odd levels'; parity 1 swaps them so
        // that this call's first level does not queue behind the previous call's fit / warp on s
        const bool swap = flow && parity && b.carry;
        hipStream_t s0 = swap ? s2 : s, s1 = swap ? s : s2;
        if (flow) {
            if (hipError_t e = hipMemsetAsync(done, 0, sizeof(int) * ((long long)kMaxLevels * nb + kLkFlagInts) * kCtrPad, s0))
                return e;
            if (hipError_t e = hipEventRecord(flow_ev[0], s0)) return e;   // counters zeroed, front end done
            if (hipError_t e = hipStreamWaitEvent(s1, flow_ev[0], 0)) return e;
        }
        for (int l = a.maxl; l >= 0; l--) {
            const ClassLevel& C = a.plan.lv[l];
            // levels alternate between the two streams: level l-1 is enqueued behind level l+1
            // only, so it starts as level l's waves leave
            hipStream_t st = flow && ((a.maxl - l) & 1) ? s1 : s0;
            if (aux) {
                if (hipError_t e = hipStreamWaitEvent(st, ev[l], 0)) return e;
            }
            // level 0 writes next_pts / status: the previous call's readers of them come first
            if (l == 0 && out_free) {
                if (hipError_t e = hipStreamWaitEvent(st, out_free, 0)) return e;
            }
            LkArgs bl = b;
            bl.done = flow ? done : nullptr;
            bl.done_stride = nb;
            bl.dep_groups = 0;
            bl.lflags = lflags;
            bl.redo = 0;
            bl.dep_points = flow_pt ? 1 : 0;
            if (flow_pair && l < a.maxl) {
                const ClassLevel& Cp = a.plan.lv[l + 1];
                bl.dep_groups = (Cp.nxp / Cp.G) * a.nyg;
            }
            if (flow && l < a.maxl) {   // start in the coarser level's tail, not beside its whole queue
                const ClassLevel& Cp = a.plan.lv[l + 1];
                const int ngc = (Cp.nxp / Cp.G) * a.nyg, ng = (C.nxp / C.G) * a.nyg;
                // per point: the coarser queue handed out is the whole condition (dep_groups 0)
                hipLaunchKernelGGL(k_lk_gate, dim3(1), dim3(64), 0, st, bq + (l + 1) * 8 * kCtrPad, (long long)nb * ngc,
                                   done + (l + 1) * nb * kCtrPad, bl.dep_groups, ng, (long long)nb * ng, a.err,
                                   a.spin_max, lflags + (kLkFlagGiveup + l) * kCtrPad);
            }
            const float4* bA = Ab + ((long long)l * batch + p) * a.npts;
            switch (C.G * 1000 + C.UW) {
#define LK_CASE(g, uw) case g * 1000 + uw: launch_iter<g, uw>(st, nb, bl, bcls, bA, bq, l); break;
                LK_SHAPES
#undef LK_CASE
            default: return hipErrorInvalidValue;
            }
            if (flow) {
                // the level's recompute, behind it on its stream and behind the coarser level's
                // (launch and recompute): exits at once unless the level gave up or the coarser
                // one was recomputed.  The planes / A sums it reads are released (lvl_done) after it.
                if (l < a.maxl) {
                    if (hipError_t e = hipStreamWaitEvent(st, redo_ev[l + 1], 0)) return e;
                    LkArgs br = bl;
                    br.done = nullptr;
                    br.dep_groups = 0;
                    br.dep_points = 0;
                    br.redo = 1;
                    br.dbg = nullptr;
                    switch (C.G * 1000 + C.UW) {
#define LK_CASE(g, uw) case g * 1000 + uw: launch_iter<g, uw>(st, nb, br, bcls, bA, bq, l); break;
                        LK_SHAPES
#undef LK_CASE
                    default: return hipErrorInvalidValue;
                    }
                }
                if (hipError_t e = hipEventRecord(redo_ev[l], st)) return e;
            }
            if (lvl_done) {
                if (hipError_t e = hipEventRecord(lvl_done[l], st)) return e;
            }
        }
        if (flow) {   // join: everything after the LK (and the next sub-batch) follows both streams
            if (hipError_t e = hipEventRecord(flow_ev[1], s2)) return e;
            if (hipError_t e = hipStreamWaitEvent(s, flow_ev[1], 0)) return e;
        }
    }
    return hipGetLastError();
}

}  // namespace mdx
