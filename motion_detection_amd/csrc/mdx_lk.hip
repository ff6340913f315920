// mdx_lk.hip -- pyramidal Lucas-Kanade (reference row A5: calcOpticalFlowPyrLK as called at
// optical_flow_calculator.cpp:71), restructured for CDNA4 while keeping OpenCV 2.4's x86 SSE2
// arithmetic bit for bit.  This is the "class plane" LK (MDX_LK_IMPL=2, default); the
// single-kernel k_lk in mdx_kernels.hip is the general fallback.
//
// Per pyramid level, from maxLevel down to 0, two kernels:
//
//  k_lk_class  The interpolated window values (I*32 descaled by 9 bits, Ix/Iy descaled by 14
//              bits) over the whole padded level, once per fractional-offset class.  At level L a
//              grid point's window origin prevPt - 19.5 has a fractional part fixed by
//              (P mod 2^L), so all points of a residue class share the bilinear weights: the
//              16x-overlapping per-window interpolation of the reference becomes one
//              interpolation per class and pixel.  Natural row-major layout, two arrays per
//              class: D = (Ix | Iy << 16) and C = 256 - 512*I (the J-chain bias, see below).
//  k_lk_level  Per point: the gradient matrix sums A11/A12/A22 over the window, the minEig /
//              determinant tests, then the Newton iterations.
//
// Work mapping of k_lk_level.  A wave = 16 points x 4 lanes: lane k of a point owns SSE lane k
// (window columns x = 4g + k, g = 0..9, rows in order) and keeps its partial sums in registers;
// partials are combined across the lane quad in the reference's order (A: ((P0+P1)+P2)+P3,
// b: (P0+P2)+(P1+P3)).  The 16 points of a wave are two groups of 8 consecutive members of one
// residue class along one grid row (host-built class-grouped order, runs padded to 8), so a
// group's windows share their rows and overlap in columns: per window row the group needs one
// contiguous "union" segment of <= 128*NCH columns of D and C.  Each half-wave loads its
// group's segment with one coalesced dwordx4 per array and lane, stores it to a double-buffered
// LDS row, and every lane then reads its 10 chain elements with ds_read_b32.  That replaces the
// 6 scattered dwordx2/x4 loads per lane and row that bound the previous design on the texture
// data path (TD busy 97%, VALU 38%).  J (the moving window in the next frame) differs per point:
// its row segment is loaded once per lane quad (3 dwords per lane) and shared by DPP.
//
// Arithmetic: J taps via v_perm_b32 + v_dot2_i32_i16 (signed weights: w11 may be -1);
// dot2(pa, W0, dot2(pb, W1, C)) >> 9 == ((S + 256) >> 9) - I exactly, because C = 256 - 512*I
// is a multiple-of-512 shift of the rounding bias.  Products are float multiplies of exactly
// converted integers (one rounding of the exact product == the reference's (float)(int
// product)).  Products/sums never go through FMA (-ffp-contract=off).
#include "mdx_internal.h"

#include <float.h>

namespace mdx {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
// 4-B aligned multi-dword loads (global_load_dwordx4/x3 at dword-aligned addresses)
struct __attribute__((aligned(4))) u4a4 { uint32_t x, y, z, w; };
struct __attribute__((aligned(4))) u3a4 { uint32_t x, y, z; };
struct __attribute__((aligned(4))) u2a4 { uint32_t x, y; };
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v3u __attribute__((ext_vector_type(3)));
// raw buffer descriptor over [base, base + bytes) (cdna_hip_programming.md T8: built from
// wave-uniform values only); loads then take a 32-bit per-lane byte offset
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, long long bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                             (int)min(bytes, (long long)0x7fffffff), 0x00020000);
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

// One J row segment of a point's window, shared by its lane quad: the 11 dwords from the
// 4-B aligned column B = inx & ~3 cover every lane's taps (lane k needs bytes o + 4g and
// o + 4g + 1 with o = (inx & 3) + k <= 6, i.e. inside dwords g, g+1).  Each lane loads 3 of
// them and DPP broadcasts assemble the row in every lane: 12 B of L1 traffic per lane, not 48.
__device__ __forceinline__ u3a4 load_jrow_part(const uint32_t* seg, int k)
{
    return *reinterpret_cast<const u3a4*>(seg + 3 * k);
}
__device__ __forceinline__ void bcast_jrow(const u3a4 m, uint32_t (&r)[11])
{
    r[0] = quad_bcast_u<0>(m.x); r[1] = quad_bcast_u<0>(m.y); r[2] = quad_bcast_u<0>(m.z);
    r[3] = quad_bcast_u<1>(m.x); r[4] = quad_bcast_u<1>(m.y); r[5] = quad_bcast_u<1>(m.z);
    r[6] = quad_bcast_u<2>(m.x); r[7] = quad_bcast_u<2>(m.y); r[8] = quad_bcast_u<2>(m.z);
    r[9] = quad_bcast_u<3>(m.x); r[10] = quad_bcast_u<3>(m.y);
}
__device__ __forceinline__ void load_jrow_quad(const uint32_t* seg, int k, uint32_t (&r)[11])
{
    bcast_jrow(load_jrow_part(seg, k), r);
}

// Ordering point between a window row's LDS staging writes and the next row's reads.  A
// workgroup is one wave and one wave's LDS instructions execute in order, so only the compiler
// must be kept from moving LDS accesses across it (no s_barrier, no forced vmcnt(0)).
__device__ __forceinline__ void wave_lds_fence()
{
#ifdef LKX_SYNC
    __syncthreads();
#else
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

// XCD-aware block order: blocks are dealt round-robin over the 8 XCDs; remap so that each
// XCD gets a contiguous range of waves (= a contiguous image band), whose class planes then
// stay in that XCD's L2.  Bijective for any count (cdna_hip_programming.md §5.5 T1).
__device__ __forceinline__ int xcd_remap(int b, int total)
{
    const int xcd = b & 7, q = total >> 3, r = total & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
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
    const int v = blockIdx.y;
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
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (x0 + q >= L.w + kPad - 1) { cv[q] = 256; continue; }
            const int i00 = (ib[0][q >> 2] >> (8 * (q & 3))) & 255, i01 = (ib[0][(q + 1) >> 2] >> (8 * ((q + 1) & 3))) & 255;
            const int i10 = (ib[1][q >> 2] >> (8 * (q & 3))) & 255, i11 = (ib[1][(q + 1) >> 2] >> (8 * ((q + 1) & 3))) & 255;
            const int ival = (i00 * w00 + i01 * w01 + i10 * w10 + i11 * w11 + 256) >> 9;
            const uint32_t d00 = dw[0][q], d01 = dw[0][q + 1], d10 = dw[1][q], d11 = dw[1][q + 1];
            const int ixv = ((int)(int16_t)d00 * w00 + (int)(int16_t)d01 * w01 + (int)(int16_t)d10 * w10 +
                             (int)(int16_t)d11 * w11 + 8192) >> 14;
            const int iyv = (((int)d00 >> 16) * w00 + ((int)d01 >> 16) * w01 + ((int)d10 >> 16) * w10 +
                             ((int)d11 >> 16) * w11 + 8192) >> 14;
            dv[q] = ((uint32_t)ixv & 0xffffu) | ((uint32_t)iyv << 16);
            cv[q] = 256 - 512 * ival;   // J-chain bias: (S + C) >> 9 == ((S + 256) >> 9) - I
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) cv[q] = 256;
    }
    const long long o = (long long)v * C.PW + 4 * j;
    *reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(base) + o) = make_uint4(dv[0], dv[1], dv[2], dv[3]);
    *reinterpret_cast<int4*>(reinterpret_cast<int32_t*>(base) + (long long)C.UH * C.PW + o) =
        make_int4(cv[0], cv[1], cv[2], cv[3]);
}

// ------------------------------------------------------------------ one pyramid level
// grid: x -> wave (16 points), y -> pair (XCD-remapped as one linear range).  Levels run as
// separate launches from maxLevel down to 0; the position carried between them is next_pts
// (the reference's nextPts[ptidx], stored every level).
template <int NCH>
#ifdef LKX_WPE   // timing variants: occupancy request
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LKX_WPE, 8)))
#else
__global__ __launch_bounds__(64)
#endif
void k_lk_level(LkArgs a, const uint8_t* __restrict__ cls, int level)
{
    constexpr int UW = NCH * 128;           // union columns per group
    constexpr float HALFW = 19.5f;
    constexpr float FLT_SCALE = 1.f / (1 << 20);
    // [buf][group][D, C][UW]: a window row's union segment, double-buffered across rows
    __shared__ __attribute__((aligned(16))) uint32_t lds[2][2][2][UW];

    const int lane = threadIdx.x, k = lane & 3, grp = lane >> 5, gl = lane & 31;
    const int nw = gridDim.x;
    const int bid = xcd_remap(blockIdx.x + nw * blockIdx.y, nw * gridDim.y);
    const int pair = bid / nw, w = bid % nw;
    const ClassLevel& C = a.plan.lv[level];
    const Level L = a.g.lv[level];
    const int16_t* xo = a.ord + C.ord_off;
    const int16_t* yo = xo + C.nxp;
    const int slot = (w / a.ny) * 16 + (lane >> 2);
    const int gxv = slot < C.nxp ? xo[slot] : -1;
    const bool valid = gxv >= 0;
    const int gx = valid ? gxv : 0, gy = yo[w % a.ny];
    const int pt = gx * a.ny + gy;
    const long long po = (long long)pair * a.npts + pt;

    const float scale = (float)(1. / (1 << level));
    const float px0 = (float)(gx * a.pixel_step), py0 = (float)(gy * a.pixel_step);
    const float ppx = px0 * scale - HALFW, ppy = py0 * scale - HALFW;
    const int ipx = (int)floorf(ppx), ipy = (int)floorf(ppy);
    bool ok = valid && !(ipx < -kWin || ipx >= L.w || ipy < -kWin || ipy >= L.h);

    // group (8 points) geometry: its first slot holds its leftmost point (runs sorted by x)
    const int slot0 = (w / a.ny) * 16 + grp * 8;
    const int gx0v = slot0 < C.nxp ? xo[slot0] : -1;
    const int gx0 = gx0v >= 0 ? gx0v : 0;
    const int ipx0 = (int)floorf((float)(gx0 * a.pixel_step) * scale - HALFW);
    const int m = (1 << level) - 1;
    const int cx = class_of(a.cmap, level, 0, (gx0 * a.pixel_step) & m);
    const int cy = class_of(a.cmap, level, 1, (gy * a.pixel_step) & m);
    const uint8_t* cbase = cls + (long long)pair * a.plan.bytes_per_pair + C.off +
                           (long long)(cy * C.nrx + cx) * C.class_bytes;
    const int ub = min(max(ipx0 + kPad, 0), C.PW - UW);          // union start column
    const int off = min(max(ipx + kPad - ub, 0), UW - kWin);     // this point's column in it
    const uint32_t* gD = reinterpret_cast<const uint32_t*>(cbase) + ub + 4 * gl;
    [[maybe_unused]] const uint32_t* gC = gD + (long long)C.UH * C.PW;
    // buffer addressing: descriptor over this pair's class slab, 32-bit lane offsets; the C
    // array sits a constant UH*PW*4 bytes after D (scalar offset field)
    const uint8_t* cslab = cls + (long long)pair * a.plan.bytes_per_pair;
    const __amdgpu_buffer_rsrc_t crs = buf_rsrc(cslab, a.plan.bytes_per_pair);
    const uint32_t dlane = (uint32_t)(reinterpret_cast<const uint8_t*>(gD) - cslab);
    const int csoff = C.UH * C.PW * 4;
    const uint32_t rowb = (uint32_t)C.PW * 4;
    const int v0 = min(max(ipy + kPad, 0), C.UH - kWin);          // first window row (wave-uniform)
    const uint32_t* lD0 = &lds[0][grp][0][off + k];
    const uint32_t* lC0 = &lds[0][grp][1][off + k];
    constexpr int LBUF = 2 * 2 * UW;                              // words per buffer

    float npx, npy;
    if (level == a.maxl) {
        npx = px0 * scale;
        npy = py0 * scale;
    } else {
        const float2 q = valid ? reinterpret_cast<const float2*>(a.next_pts)[po] : make_float2(0.f, 0.f);
        npx = q.x * 2.f;
        npy = q.y * 2.f;
    }
    int status = 1;
    if (valid && !ok && level == 0) status = 0;

    uint4 rd[NCH], rc[NCH];
    auto gload = [&](int v, bool withC) {
#pragma unroll
        for (int c = 0; c < NCH; c++) {
#ifdef LKX_NOBUF
            const u4a4 t = *reinterpret_cast<const u4a4*>(gD + (long long)v * C.PW + 128 * c);
            rd[c] = make_uint4(t.x, t.y, t.z, t.w);
            if (withC) {
                const u4a4 s = *reinterpret_cast<const u4a4*>(gC + (long long)v * C.PW + 128 * c);
                rc[c] = make_uint4(s.x, s.y, s.z, s.w);
            }
#else
            const uint32_t vo = dlane + (uint32_t)v * rowb + 512u * c;
            const v4u t = __builtin_amdgcn_raw_buffer_load_b128(crs, (int)vo, 0, 0);
            rd[c] = make_uint4(t.x, t.y, t.z, t.w);
            if (withC) {
                const v4u q = __builtin_amdgcn_raw_buffer_load_b128(crs, (int)vo, csoff, 0);
                rc[c] = make_uint4(q.x, q.y, q.z, q.w);
            }
#endif
        }
    };
    auto lstore = [&](int buf, bool withC) {
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            *reinterpret_cast<uint4*>(&lds[buf][grp][0][128 * c + 4 * gl]) = rd[c];
            if (withC) *reinterpret_cast<uint4*>(&lds[buf][grp][1][128 * c + 4 * gl]) = rc[c];
        }
    };

    // ---- A sums: lane k owns SSE lane k (columns 4g+k), rows in order; ((P0+P1)+P2)+P3
    float A11, A12, A22;
    {
        f2 sd = {0.f, 0.f};
        float s12 = 0.f;
        gload(v0, false);
        lstore(0, false);
        wave_lds_fence();
#pragma unroll 2
        for (int y = 0; y < kWin; y++) {
            const int buf = y & 1;
            if (y + 1 < kWin) gload(v0 + y + 1, false);
            const uint32_t* ld = lD0 + buf * LBUF;
#pragma unroll
            for (int g = 0; g < 10; g++) {
                const uint32_t d = ld[4 * g];
                const f2 f = {(float)(int16_t)d, (float)((int)d >> 16)};
                sd = sd + f * f;                 // (Ix*Ix, Iy*Iy)
                s12 = s12 + f.x * f.y;           // Ix*Iy
            }
            if (y + 1 < kWin) lstore(buf ^ 1, false);
            wave_lds_fence();
        }
        const float a11 = ((quad_bcast<0>(sd.x) + quad_bcast<1>(sd.x)) + quad_bcast<2>(sd.x)) + quad_bcast<3>(sd.x);
        const float a12 = ((quad_bcast<0>(s12) + quad_bcast<1>(s12)) + quad_bcast<2>(s12)) + quad_bcast<3>(s12);
        const float a22 = ((quad_bcast<0>(sd.y) + quad_bcast<1>(sd.y)) + quad_bcast<2>(sd.y)) + quad_bcast<3>(sd.y);
        A11 = a11 * FLT_SCALE;
        A12 = a12 * FLT_SCALE;
        A22 = a22 * FLT_SCALE;
    }
    float Dinv = 0.f;
    if (ok) {
        const float D = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - __builtin_sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                             (float)(2 * kWin * kWin);
        if (minEig < a.min_eig || D < FLT_EPSILON) {
            ok = false;
            if (level == 0) status = 0;
        } else {
            Dinv = 1.f / D;
        }
    }

    // ---- Newton iterations
    const int pitch = L.pitch;
    const uint8_t* Jb = a.pyr2 + (long long)pair * a.g.img_bytes + L.img_off + L.core();
    const __amdgpu_buffer_rsrc_t jrs = buf_rsrc(a.pyr2 + (long long)pair * a.g.img_bytes, a.g.img_bytes);
    const uint32_t jbase = (uint32_t)(L.img_off + L.core());
    float nx = npx - HALFW, ny = npy - HALFW;
    float pdx = 0.f, pdy = 0.f;
    bool act = ok;
    int iters = 0;
    for (int j = 0; j < a.max_iters; j++) {
        if (!__any(act)) break;
        f2 acc = {0.f, 0.f};
        if (act) iters++;
        // Position, bounds and weights; lanes that are not iterating (or fail the bounds
        // test) run the row loop on a safe address and drop the result, so the loop below is
        // wave-uniform (it also carries the group's LDS staging).
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
        const uint32_t* jrow = reinterpret_cast<const uint32_t*>(Jb + (long long)iny * pitch + (inx & ~3));
        [[maybe_unused]] const int jstride = pitch >> 2;
        uint32_t joff = jbase + (uint32_t)(iny * pitch + (inx & ~3) + 12 * k);   // buffer offset of this lane's J dwords
        // taps of the current window row (pa) are the previous row's lower taps (pb)
        s2 pa[10], pb[10];
        {
            uint32_t rj[11];
            load_jrow_quad(jrow, k, rj);
#pragma unroll
            for (int g = 0; g < 10; g++) pa[g] = __builtin_bit_cast(s2, __builtin_amdgcn_perm(rj[g + 1], rj[g], sel));
        }
        gload(v0, true);
        lstore(0, true);
        wave_lds_fence();
#ifdef LKX_JPF
        // J rows are prefetched one row ahead (the DPP broadcast needs the data at once)
        jrow += jstride;
        u3a4 jnext = load_jrow_part(jrow, k);
#endif
#pragma unroll 2
        for (int y = 0; y < kWin; y++) {
            const int buf = y & 1;
            if (y + 1 < kWin) gload(v0 + y + 1, true);
            uint32_t rj[11];
#ifdef LKX_JPF
            const u3a4 jcur = jnext;
            jrow += jstride;
            if (y + 1 < kWin) jnext = load_jrow_part(jrow, k);
            bcast_jrow(jcur, rj);
#elif defined(LKX_NOBUF)
            jrow += jstride;
            load_jrow_quad(jrow, k, rj);
#else
            joff += (uint32_t)pitch;
            {
                const v3u m = __builtin_amdgcn_raw_buffer_load_b96(jrs, (int)joff, 0, 0);
                u3a4 mm;
                mm.x = m.x; mm.y = m.y; mm.z = m.z;
                bcast_jrow(mm, rj);
            }
#endif
            const uint32_t* ld = lD0 + buf * LBUF;
            const uint32_t* lc = lC0 + buf * LBUF;
#pragma unroll
            for (int g = 0; g < 10; g++) {
                pb[g] = __builtin_bit_cast(s2, __builtin_amdgcn_perm(rj[g + 1], rj[g], sel));
                // (J*32 - I*32) exactly as the reference's CV_DESCALE(...) - I
                const int jd = __builtin_amdgcn_sdot2(pa[g], W0, __builtin_amdgcn_sdot2(pb[g], W1, (int)lc[4 * g], false),
                                                      false) >> 9;
                const float fd = (float)jd;
                const uint32_t d = ld[4 * g];
                const f2 f = {(float)(int16_t)d, (float)((int)d >> 16)};
                acc = acc + f * fd;
                pa[g] = pb[g];
            }
            if (y + 1 < kWin) lstore(buf ^ 1, true);
            wave_lds_fence();
        }
        if (!act) acc = f2{0.f, 0.f};
        // b = (P0+P2) + (P1+P3) across the quad; inactive quads compute garbage they ignore
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
#ifdef LKX_FIXED   // timing-only builds (scripts/lk_variants.sh): a fixed iteration count
            if (j + 1 >= LKX_FIXED) act = false;
#else
            if ((double)dx * dx + (double)dy * dy <= a.eps2) {
                act = false;
            } else if (j > 0 && fabs((double)fabsf(dx + pdx)) < 0.01 && fabs((double)fabsf(dy + pdy)) < 0.01) {
                npx = npx - dx * 0.5f;
                npy = npy - dy * 0.5f;
                act = false;
            }
#endif
            pdx = dx;
            pdy = dy;
        }
    }
    if (level == 0 && valid && status) {
        const int fx = (int)floorf(npx - HALFW), fy = (int)floorf(npy - HALFW);
        if (fx < -kWin || fx >= L.w || fy < -kWin || fy >= L.h) status = 0;
    }
    if (a.dbg && valid && k == 0)
        a.dbg[((long long)pair * a.g.nlev + level) * a.npts + pt] = make_float4(npx, npy, (float)iters, (float)status);
    if (valid && k == 0) {
        reinterpret_cast<float2*>(a.next_pts)[po] = make_float2(npx, npy);
        if (level == 0) a.status[po] = (uint8_t)status;
    }
}

hipError_t launch_lk_v2(hipStream_t s, int batch, const LkArgs& a, uint8_t* cls)
{
    for (int l = a.maxl; l >= 0; l--) {
        // class planes of this level right before its use: they are still in L2 / MALL
        const ClassLevel& C = a.plan.lv[l];
        LkClassArgs ca;
        ca.g = a.g;
        ca.plan = a.plan;
        ca.rlist = a.rlist;
        ca.level = l;
        const dim3 grid(((a.g.lv[l].w + 2 * kPad) / 4 + 63) / 64, C.UH, batch * C.nrx * C.nry);
        hipLaunchKernelGGL(k_lk_class, grid, dim3(64), 0, s, a.pyr1, a.der, cls, ca);
        const dim3 lg(((C.nxp + 15) / 16) * a.ny, batch);
        switch (a.plan.nch) {
        case 1: hipLaunchKernelGGL(k_lk_level<1>, lg, dim3(64), 0, s, a, cls, l); break;
        case 2: hipLaunchKernelGGL(k_lk_level<2>, lg, dim3(64), 0, s, a, cls, l); break;
        case 4: hipLaunchKernelGGL(k_lk_level<4>, lg, dim3(64), 0, s, a, cls, l); break;
        default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}

}  // namespace mdx
