// mdx_lk.hip -- pyramidal Lucas-Kanade (reference row A5: calcOpticalFlowPyrLK as called at
// optical_flow_calculator.cpp:71), restructured for CDNA4 while keeping OpenCV 2.4's x86 SSE2
// arithmetic bit for bit.
//
// Three kernels per batch of frame pairs:
//
//  k_lk_class  For every level and every fractional-offset class, the interpolated window
//              values (I*32 descaled by 9 bits, Ix/Iy descaled by 14 bits) over the whole
//              padded level.  At level L a grid point's window origin prevPt - 19.5 has a
//              fractional part fixed by (P mod 2^L), so all points of a residue class share
//              the bilinear weights: the 16x-overlapping per-window interpolation of the
//              reference becomes one interpolation per class and pixel.  Stored de-interleaved
//              by column mod 4 ("planes"), so the 10 elements of one SSE lane's chain in a
//              window row are contiguous.
//  k_lk_A      Per point and level, the gradient matrix sums A11/A12/A22.  They depend only on
//              the original point and the level (not on tracking), so they are computed for all
//              levels at once.  4 lanes per point: lane k owns the SSE lane k chain (window
//              columns x = 4g+k, rows in order) and adds in registers; the four partials are
//              combined ((P0+P1)+P2)+P3 across the lane quad.
//  k_lk_track  Newton iterations level by level.  Same 4-lanes-per-point chain layout for
//              b1/b2 (combined (P0+P2)+(P1+P3)); J taps via v_perm_b32 + v_dot2_u32_u16; the
//              products are formed as float multiplies of exactly-converted integers (one
//              rounding of the exact product == the reference's (float)(int product)).
//
// Products/sums never go through FMA (-ffp-contract=off).
#include "mdx_internal.h"

#include <float.h>

namespace mdx {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint4 __attribute__((aligned(8))) uint4_a8;
typedef uint4 __attribute__((aligned(4))) uint4_a4;
typedef uint2 __attribute__((aligned(4))) uint2_a4;

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

// ------------------------------------------------------------------ class planes
// grid: x -> plane column j (elements u = 4j..4j+3, one per plane), y -> plane row v,
// z -> pair * nclass + class.  Element (u, v) is the window value at level core position
// (x, y) = (u - 40, v - 40) for the class's bilinear weights: (I*32, Ix, Iy) exactly as
// LKTrackerInvoker extracts them (CV_DESCALE by W_BITS1-5 = 9 and W_BITS1 = 14).
__global__ __launch_bounds__(256) void k_lk_class(const uint8_t* __restrict__ pyr1, const uint32_t* __restrict__ der,
                                                  uint8_t* __restrict__ cls_out, LkClassArgs a)
{
    const int level = a.level;
    const ClassLevel& C = a.plan.lv[level];
    const int nclass = C.nrx * C.nry;
    const int pair = blockIdx.z / nclass, cls = blockIdx.z % nclass;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int v = blockIdx.y;
    if (j >= C.PW || v >= C.UH) return;
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
    uint32_t* Dout = reinterpret_cast<uint32_t*>(base);
    uint16_t* Iout = reinterpret_cast<uint16_t*>(base + 16LL * C.UH * C.PW);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int x = 4 * j + q - kPad;
        uint32_t dv = 0;
        uint16_t iv = 0;
        if (x < L.w + kPad - 1 && y < L.h + kPad - 1) {
            const uint8_t* ip = I + (long long)y * p + x;
            const int ival = (ip[0] * w00 + ip[1] * w01 + ip[p] * w10 + ip[p + 1] * w11 + 256) >> 9;
            const uint32_t* dp = D + (long long)y * p + x;
            const uint32_t d00 = dp[0], d01 = dp[1], d10 = dp[p], d11 = dp[p + 1];
            const int ixv = ((int)(int16_t)d00 * w00 + (int)(int16_t)d01 * w01 + (int)(int16_t)d10 * w10 +
                             (int)(int16_t)d11 * w11 + 8192) >> 14;
            const int iyv = (((int)d00 >> 16) * w00 + ((int)d01 >> 16) * w01 + ((int)d10 >> 16) * w10 +
                             ((int)d11 >> 16) * w11 + 8192) >> 14;
            dv = ((uint32_t)ixv & 0xffffu) | ((uint32_t)iyv << 16);
            iv = (uint16_t)ival;
        }
        const long long o = ((long long)q * C.UH + v) * C.PW + j;
        Dout[o] = dv;
        Iout[o] = iv;
    }
}

// Point of lane `lane` in wave `w`: each wave takes 16 consecutive grid columns of ONE grid row
// (same iy), so at every window row the 64 lanes read the same image rows -> coalesced loads.
// XCD-aware block order: blocks are dealt round-robin over the 8 XCDs; remap so that each
// XCD gets a contiguous range of waves (= a contiguous image band), whose class planes then
// stay in that XCD's L2.  Bijective for any count (cdna_hip_programming.md §5.5 T1).
__device__ __forceinline__ int xcd_remap(int b, int total)
{
    const int xcd = b & 7, q = total >> 3, r = total & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

__device__ __forceinline__ void wave_point(const LkArgs& a, int w, int lane, int& pt, int& gx, int& gy, bool& valid)
{
    const int nx = (a.npts + a.ny - 1) / a.ny;
    gy = w % a.ny;
    gx = (w / a.ny) * 16 + (lane >> 2);
    valid = gx < nx;
    pt = gx * a.ny + gy;
    if (!valid) { gx = 0; pt = 0; }
}

// Window origin, class and plane addressing shared by k_lk_A and k_lk_track.
struct WinRef {
    bool ok;
    int ipx, ipy;
    const uint32_t* drow;   // this lane's chain start (D plane) in row 0 of the window
    const uint32_t* irow;   // 4-B aligned word holding its first I value (I plane)
    int ishift;             // 0 or 16: bit offset of the first I value in *irow
    int dstride, istride;   // row strides in words
};

__device__ __forceinline__ WinRef win_ref(const LkArgs& a, const uint8_t* cls, int pair, int level, int gx, int gy,
                                          float px0, float py0, int k, bool valid)
{
    WinRef r;
    const Level L = a.g.lv[level];
    const ClassLevel& C = a.plan.lv[level];
    const float scale = (float)(1. / (1 << level));
    const float ppx = px0 * scale - 19.5f, ppy = py0 * scale - 19.5f;
    r.ipx = (int)floorf(ppx);
    r.ipy = (int)floorf(ppy);
    r.ok = valid && !(r.ipx < -kWin || r.ipx >= L.w || r.ipy < -kWin || r.ipy >= L.h);
    r.dstride = C.PW;
    r.istride = C.PW >> 1;
    // lanes without a window read class 0, plane 0 from its origin (always in bounds) so that
    // the chain loops run wave-uniform; their sums are discarded.
    const uint8_t* base = cls + (long long)pair * a.plan.bytes_per_pair + C.off;
    long long eo = 0;
    if (r.ok) {
        const int m = (1 << level) - 1;
        const int cx = class_of(a.cmap, level, 0, (gx * a.pixel_step) & m);
        const int cy = class_of(a.cmap, level, 1, (gy * a.pixel_step) & m);
        const int u = r.ipx + kPad + k;
        const int q = u & 3, j0 = u >> 2;
        base += (long long)(cy * C.nrx + cx) * C.class_bytes;
        eo = ((long long)q * C.UH + (r.ipy + kPad)) * C.PW + j0;
    }
    r.drow = reinterpret_cast<const uint32_t*>(base) + eo;
    r.irow = reinterpret_cast<const uint32_t*>(base + 16LL * C.UH * C.PW) + (eo >> 1);
    r.ishift = (int)(eo & 1) * 16;
    return r;
}

// ------------------------------------------------------------------ A sums
// grid: x -> 16 points per 64-lane wave, y -> level, z -> pair.  Output per (pair, level,
// point): float4(A11, A12, A22, ok) with the FLT_SCALE already applied.
__global__ __launch_bounds__(64) void k_lk_A(LkArgs a, const uint8_t* __restrict__ cls, float4* __restrict__ Aout)
{
    const int lane = threadIdx.x, k = lane & 3;
    const int nw = gridDim.x, total = nw * gridDim.y * gridDim.z;
    const int bid = xcd_remap(blockIdx.x + nw * (blockIdx.y + gridDim.y * blockIdx.z), total);
    const int level = (bid / nw) % gridDim.y, pair = bid / (nw * gridDim.y);
    int pt, gx, gy;
    bool valid;
    wave_point(a, bid % nw, lane, pt, gx, gy, valid);
    const WinRef r = win_ref(a, cls, pair, level, gx, gy, (float)(gx * a.pixel_step), (float)(gy * a.pixel_step), k,
                             valid);
    f2 sd = {0.f, 0.f};
    float s12 = 0.f;
    const uint32_t* dp = r.drow;
    for (int y = 0; y < kWin; y++, dp += r.dstride) {
        uint32_t d[10];
        const uint4_a4* v4 = reinterpret_cast<const uint4_a4*>(dp);
        const uint4 w0 = v4[0], w1 = v4[1];
        const uint2 w2 = *reinterpret_cast<const uint2_a4*>(dp + 8);
        d[0] = w0.x; d[1] = w0.y; d[2] = w0.z; d[3] = w0.w;
        d[4] = w1.x; d[5] = w1.y; d[6] = w1.z; d[7] = w1.w;
        d[8] = w2.x; d[9] = w2.y;
#pragma unroll
        for (int g = 0; g < 10; g++) {
            const f2 f = {(float)(int16_t)d[g], (float)((int)d[g] >> 16)};
            sd = sd + f * f;                 // (Ix*Ix, Iy*Iy)
            s12 = s12 + f.x * f.y;           // Ix*Iy
        }
    }
    const float s11 = r.ok ? sd.x : 0.f, s22 = r.ok ? sd.y : 0.f;
    s12 = r.ok ? s12 : 0.f;
    // ((P0+P1)+P2)+P3 across the quad (SSE lanes 0..3)
    const float a11 = ((quad_bcast<0>(s11) + quad_bcast<1>(s11)) + quad_bcast<2>(s11)) + quad_bcast<3>(s11);
    const float a12 = ((quad_bcast<0>(s12) + quad_bcast<1>(s12)) + quad_bcast<2>(s12)) + quad_bcast<3>(s12);
    const float a22 = ((quad_bcast<0>(s22) + quad_bcast<1>(s22)) + quad_bcast<2>(s22)) + quad_bcast<3>(s22);
    if (valid && k == 0) {
        const float FS = 1.f / (1 << 20);
        Aout[((long long)pair * a.g.nlev + level) * a.npts + pt] =
            make_float4(a11 * FS, a12 * FS, a22 * FS, r.ok ? 1.f : 0.f);
    }
}

// ------------------------------------------------------------------ tracking
__global__ __launch_bounds__(64) void k_lk_track(LkArgs a, const uint8_t* __restrict__ cls, const float4* __restrict__ Ain)
{
    constexpr float HALFW = 19.5f;
    constexpr float FLT_SCALE = 1.f / (1 << 20);
    const int lane = threadIdx.x, k = lane & 3;
    const int nw = gridDim.x;
    const int bid = xcd_remap(blockIdx.x + nw * blockIdx.y, nw * gridDim.y);
    const int pair = bid / nw;
    int pt, gx, gy;
    bool valid;
    wave_point(a, bid % nw, lane, pt, gx, gy, valid);
    const float px0 = (float)(gx * a.pixel_step), py0 = (float)(gy * a.pixel_step);
    float npx = 0.f, npy = 0.f;
    int status = 1;
    const uint8_t* slab2 = a.pyr2 + (long long)pair * a.g.img_bytes;

    for (int level = a.maxl; level >= 0; --level) {
        const Level L = a.g.lv[level];
        const int pitch = L.pitch;
        const uint8_t* Jb = slab2 + L.img_off + L.core();
        const float scale = (float)(1. / (1 << level));
        const float ppx = px0 * scale, ppy = py0 * scale;
        if (level == a.maxl) { npx = ppx; npy = ppy; }
        else { npx = npx * 2.f; npy = npy * 2.f; }
        const WinRef r = win_ref(a, cls, pair, level, gx, gy, px0, py0, k, valid);
        bool ok = r.ok;
        if (valid && !ok && level == 0) status = 0;
        float A11 = 0.f, A12 = 0.f, A22 = 0.f, Dinv = 0.f;
        if (ok) {
            const float4 A = Ain[((long long)pair * a.g.nlev + level) * a.npts + pt];
            A11 = A.x; A12 = A.y; A22 = A.z;
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
        float nx = npx - HALFW, ny = npy - HALFW;
        float pdx = 0.f, pdy = 0.f;
        bool act = ok;
        int iters = 0;
        for (int j = 0; j < a.max_iters; j++) {
            if (!__any(act)) break;
            f2 acc = {0.f, 0.f};
            if (act) iters++;
            // Position, bounds and weights; lanes that are not iterating (or fail the bounds
            // test) run the chain loop on a safe address and drop the result, so the loop
            // below is wave-uniform.
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
            const int s = inx + k;
            const int o = s & 3;
            const unsigned sel = (unsigned)o | 0x0c00u | ((unsigned)(o + 1) << 16) | 0x0c000000u;
            const uint32_t* jrow = reinterpret_cast<const uint32_t*>(Jb + (long long)iny * pitch + (s - o));
            const int jstride = pitch >> 2;
            uint32_t r0[12], r1[12];
            {
                const uint4_a4* p4 = reinterpret_cast<const uint4_a4*>(jrow);
#pragma unroll
                for (int t = 0; t < 3; t++) {
                    const uint4 w = p4[t];
                    r0[4 * t] = w.x; r0[4 * t + 1] = w.y; r0[4 * t + 2] = w.z; r0[4 * t + 3] = w.w;
                }
            }
            const uint32_t* dp = r.drow;
            const uint32_t* ip = r.irow;
            for (int y = 0; y < kWin; y++, dp += r.dstride, ip += r.istride) {
                jrow += jstride;
                const uint4_a4* p4 = reinterpret_cast<const uint4_a4*>(jrow);
#pragma unroll
                for (int t = 0; t < 3; t++) {
                    const uint4 w = p4[t];
                    r1[4 * t] = w.x; r1[4 * t + 1] = w.y; r1[4 * t + 2] = w.z; r1[4 * t + 3] = w.w;
                }
                uint32_t d[10], iw[6], iv[5];
                {
                    const uint4_a4* v4 = reinterpret_cast<const uint4_a4*>(dp);
                    const uint4 w0 = v4[0], w1 = v4[1];
                    const uint2 w2 = *reinterpret_cast<const uint2_a4*>(dp + 8);
                    d[0] = w0.x; d[1] = w0.y; d[2] = w0.z; d[3] = w0.w;
                    d[4] = w1.x; d[5] = w1.y; d[6] = w1.z; d[7] = w1.w;
                    d[8] = w2.x; d[9] = w2.y;
                    const uint4 u0 = *reinterpret_cast<const uint4_a4*>(ip);
                    const uint2 u1 = *reinterpret_cast<const uint2_a4*>(ip + 4);
                    iw[0] = u0.x; iw[1] = u0.y; iw[2] = u0.z; iw[3] = u0.w; iw[4] = u1.x; iw[5] = u1.y;
#pragma unroll
                    for (int t = 0; t < 5; t++) iv[t] = __builtin_amdgcn_alignbit(iw[t + 1], iw[t], r.ishift);
                }
#pragma unroll
                for (int g = 0; g < 10; g++) {
                    const s2 pa = __builtin_bit_cast(s2, __builtin_amdgcn_perm(r0[g + 1], r0[g], sel));
                    const s2 pb = __builtin_bit_cast(s2, __builtin_amdgcn_perm(r1[g + 1], r1[g], sel));
                    const int jv = __builtin_amdgcn_sdot2(pa, W0, __builtin_amdgcn_sdot2(pb, W1, 256, false), false) >> 9;
                    const int ival = (g & 1) ? (int)(iv[g >> 1] >> 16) : (int)(iv[g >> 1] & 0xffffu);
                    const float fd = (float)(jv - ival);
                    const f2 f = {(float)(int16_t)d[g], (float)((int)d[g] >> 16)};
                    acc = acc + f * fd;
                }
#pragma unroll
                for (int t = 0; t < 12; t++) r0[t] = r1[t];
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
        }
        if (level == 0 && valid && status) {
            const int fx = (int)floorf(npx - HALFW), fy = (int)floorf(npy - HALFW);
            if (fx < -kWin || fx >= L.w || fy < -kWin || fy >= L.h) status = 0;
        }
        if (a.dbg && valid && k == 0)
            a.dbg[((long long)pair * a.g.nlev + level) * a.npts + pt] = make_float4(npx, npy, (float)iters, (float)status);
    }
    if (valid && k == 0) {
        const long long o = (long long)pair * a.npts + pt;
        a.next_pts[2 * o] = npx;
        a.next_pts[2 * o + 1] = npy;
        a.status[o] = (uint8_t)status;
    }
}

hipError_t launch_lk_v2(hipStream_t s, int batch, const LkArgs& a, uint8_t* cls, float4* Abuf)
{
    for (int l = 0; l <= a.maxl; l++) {
        const ClassLevel& C = a.plan.lv[l];
        LkClassArgs ca;
        ca.g = a.g;
        ca.plan = a.plan;
        ca.rlist = a.rlist;
        ca.level = l;
        const dim3 grid((C.PW + 63) / 64, C.UH, batch * C.nrx * C.nry);
        hipLaunchKernelGGL(k_lk_class, grid, dim3(64), 0, s, a.pyr1, a.der, cls, ca);
    }
    const int nx = (a.npts + a.ny - 1) / a.ny;
    const int nwaves = ((nx + 15) / 16) * a.ny;
    hipLaunchKernelGGL(k_lk_A, dim3(nwaves, a.maxl + 1, batch), dim3(64), 0, s, a, cls, Abuf);
    hipLaunchKernelGGL(k_lk_track, dim3(nwaves, batch), dim3(64), 0, s, a, cls, Abuf);
    return hipGetLastError();
}

}  // namespace mdx
