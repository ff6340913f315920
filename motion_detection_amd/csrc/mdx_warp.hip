// mdx_warp.hip -- rows A8-A10 fused: warpPerspective(gray1, M) + absdiff(., gray2) +
// threshold(., 190, 255, BINARY) (reference common/src/optical_flow_calculator.cpp:124-127),
// bit-exact to OpenCV 2.4's imgwarp.cpp WarpPerspectiveInvoker + remapBilinear<FixedPtCast> with
// BORDER_CONSTANT 0.
//
// Reference arithmetic per destination pixel (x, y), M = inverse of the fitted H:
//   blocks of bw0 x bh0 (bh0 = min(16, H), bw0 = min(1024 / bh0, W)); xb = bw0 * floor(x / bw0)
//   X0 = M0*xb + M1*y + M2,  W0 = M6*xb + M7*y + M8           (FP64, this evaluation order)
//   W  = W0 + M6*x1, Wd = W ? 32/W : 0,  x1 = x - xb
//   X  = cvRound(clamp((X0 + M0*x1) * Wd)),  Y likewise        (1/32-pixel fixed point)
//   sx = X >> 5, fx = X & 31, ...;  out = (sum v_i * w_i + 2^14) >> 15 with w_i from (fx, fy)
//   mask = |out - gray2| > thresh ? 255 : 0
//
// Fast path (affine M, bw0 == 64, the tile's source footprint small): one 256-thread workgroup
// per 64 x 64 destination tile (= one reference block column, four block rows).  Lane l of
// wave w owns the 4 columns x0 + 4*(l & 15) .. +3 of rows y0 + 16w + 4i + (l >> 4), i = 0..3,
// so gray2 loads / mask stores are dwords, 64 contiguous bytes per row.
//   * The tile's source footprint (exact: X, Y are monotone in x and y for affine M, so the
//     four corners bound it) is staged once into LDS as raw bytes with ds_write_b128, zero
//     outside the image (= BORDER_CONSTANT 0 per tap).  Row pitch 192 B (48 dwords = 16 mod 32):
//     the two rows a half-wave touches fall in disjoint banks; taps are 4 ds_read_u8 with
//     immediate offsets (0, 1, 192, 193).
//   * Per column, M0*x1 and M3*x1 stay in registers (4 columns per lane); per row, X0 and Y0 come
//     from a 64-entry LDS table.  Per pixel: two FP64 adds and two multiply-adds with the magic
//     constant 1.5*2^52 - 32*origin, whose low word is cvRound(.) relative to the staged origin
//     (round-half-even, exact for |X| < 2^30, checked per tile).  When 32/M8 is a power of two the
//     multiply is exact and fuses with the rounding add into one FMA.
//   * Bilinear: w = (32-fx)(32-fy)*32 ... factorises exactly: h0 = dot4(v00 v01 v10 v11, 32-fx fx 0 0),
//     h1 = dot4(., 0 0 32-fx fx), out = (dot2(h0 h1, 32-fy fy) + 512) >> 10.
//   * |out - g2| + (255 - thresh) has bit 8 set iff the pixel is moving (v_sad_u16); four such
//     bits are packed with v_perm and scaled by 255 into the mask dword.
// Everything else (perspective M, small frames, huge or far-away footprints) takes the general
// per-pixel path, exact for any input.
#include "mdx_internal.h"

#include <limits.h>

namespace mdx {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));


constexpr int kWTile = 64;              // tile = one reference block column (bw0 = 64)
constexpr int kHTile = 64;              // four reference block rows
constexpr int kSP = 192;                // staged row pitch, bytes (48 dwords = 16 mod 32)
constexpr int kSH = 96;                 // staged rows

__device__ __forceinline__ int clamp_int_from_double(double v)
{
    // std::max((double)INT_MIN, std::min((double)INT_MAX, v)) then cvRound
    double r = (v < (double)INT_MAX) ? v : (double)INT_MAX;
    r = ((double)INT_MIN < r) ? r : (double)INT_MIN;
    return (int)__builtin_rint(r);
}

// General path: one destination pixel, any M, reading gray1 straight from global memory.
__device__ __forceinline__ uint8_t warp_px_general(const double* M, const uint8_t* src, int pitch, int w, int h, int x,
                                                   int y, int bw0, int g2v, int thresh)
{
    const int xb = (x / bw0) * bw0, x1 = x - xb;
    const double X0 = M[0] * xb + M[1] * y + M[2];
    const double Y0 = M[3] * xb + M[4] * y + M[5];
    const double W0 = M[6] * xb + M[7] * y + M[8];
    const double Wv = W0 + M[6] * x1;
    const double Wd = Wv != 0.0 ? 32.0 / Wv : 0.0;
    const int X = clamp_int_from_double((X0 + M[0] * x1) * Wd);
    const int Y = clamp_int_from_double((Y0 + M[3] * x1) * Wd);
    const int sx = min(max(X >> 5, -32768), 32767), sy = min(max(Y >> 5, -32768), 32767);
    const int fx = X & 31, fy = Y & 31;
    // (0,0) cell of BilinearTab_i is {32767,0,0,1}; for 8-bit data it yields the same value as
    // {32768,0,0,0}, which is what the plain formula computes.
    const int wt0 = (32 - fx) * (32 - fy) * 32, wt1 = fx * (32 - fy) * 32;
    const int wt2 = (32 - fx) * fy * 32, wt3 = fx * fy * 32;
    const bool ix0 = (unsigned)sx < (unsigned)w, ix1 = (unsigned)(sx + 1) < (unsigned)w;
    const bool iy0 = (unsigned)sy < (unsigned)h, iy1 = (unsigned)(sy + 1) < (unsigned)h;
    const int cx0 = min(max(sx, 0), w - 1), cx1 = min(max(sx + 1, 0), w - 1);
    const int cy0 = min(max(sy, 0), h - 1), cy1 = min(max(sy + 1, 0), h - 1);
    const uint8_t* ra = src + (long long)cy0 * pitch;
    const uint8_t* rb = src + (long long)cy1 * pitch;
    const int v0 = (ix0 && iy0) ? ra[cx0] : 0;
    const int v1 = (ix1 && iy0) ? ra[cx1] : 0;
    const int v2 = (ix0 && iy1) ? rb[cx0] : 0;
    const int v3 = (ix1 && iy1) ? rb[cx1] : 0;
    int v = (v0 * wt0 + v1 * wt1 + v2 * wt2 + v3 * wt3 + (1 << 14)) >> 15;
    v = min(max(v, 0), 255);
    return abs(v - g2v) > thresh ? 255 : 0;
}

struct TileInfo {
    int fast;          // 1: fast path usable for this tile
    int sxa, sya;      // staged origin (sxa multiple of 16)
    int sw, sh, lp;    // staged width (bytes), height (rows), LDS row pitch
};

// Bounds of the tile's taps, computed on lanes 0..3 (one corner each) with the reference
// arithmetic; fast = every |X|, |Y| < 2^30 (no clamp, magic rounding exact) and the footprint fits.
__device__ TileInfo tile_info(const double* M, double Wd, int x0, int y0, int w, int h, int lane)
{
    const int cxl = min(kWTile - 1, w - 1 - x0), cyl = min(kHTile - 1, h - 1 - y0);
    const int c = lane & 3;
    const int x1 = (c & 1) ? cxl : 0, y = y0 + ((c & 2) ? cyl : 0);
    const double X0 = M[0] * x0 + M[1] * y + M[2];
    const double Y0 = M[3] * x0 + M[4] * y + M[5];
    const double px = (X0 + M[0] * x1) * Wd, py = (Y0 + M[3] * x1) * Wd;
    const double lim = 1073741824.0;   // 2^30
    int ok = (px > -lim && px < lim && py > -lim && py < lim) ? 1 : 0;
    int sx = 0, sy = 0;
    if (ok) {
        sx = ((int)__builtin_rint(px)) >> 5;
        sy = ((int)__builtin_rint(py)) >> 5;
    }
    int sx_lo = sx, sx_hi = sx, sy_lo = sy, sy_hi = sy;
#pragma unroll
    for (int m = 1; m <= 2; m <<= 1) {
        sx_lo = min(sx_lo, __shfl_xor(sx_lo, m, 4));
        sx_hi = max(sx_hi, __shfl_xor(sx_hi, m, 4));
        sy_lo = min(sy_lo, __shfl_xor(sy_lo, m, 4));
        sy_hi = max(sy_hi, __shfl_xor(sy_hi, m, 4));
        ok = min(ok, __shfl_xor(ok, m, 4));
    }
    TileInfo t;
    t.sxa = __builtin_amdgcn_readfirstlane(sx_lo) & ~15;
    t.sya = __builtin_amdgcn_readfirstlane(sy_lo);
    const int sxb = __builtin_amdgcn_readfirstlane(sx_hi), syb = __builtin_amdgcn_readfirstlane(sy_hi);
    t.sw = sxb - t.sxa + 2;                    // bytes: columns sxa .. sxb + 1
    t.sh = syb - t.sya + 2;                    // rows sya .. syb + 1
    t.lp = kSP;
    t.fast = __builtin_amdgcn_readfirstlane(ok) && t.sw > 0 && t.sh > 0 && t.sw <= kSP && t.sh <= kSH;
    return t;
}

// grid: x -> tile column, y -> tile row, z -> pair.  256 threads.
__global__ __launch_bounds__(256) void k_warp_diff(const uint8_t* __restrict__ g1, long long g1_stride, int g1_pitch,
                                                   const uint8_t* __restrict__ g2, long long g2_stride, int g2_pitch,
                                                   int w, int h, int bw0, const PairFit* __restrict__ fits,
                                                   uint8_t* __restrict__ mask, long long mask_stride, int thresh,
                                                   int vec_ok)
{
    __shared__ __attribute__((aligned(16))) double s_xy[kHTile][2];    // (X0, Y0) per tile row
    __shared__ __attribute__((aligned(16))) uint8_t s_src[kSH * kSP];

    const int pair = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x0 = blockIdx.x * kWTile, y0 = blockIdx.y * kHTile;
    const int cq = lane & 15, rr = lane >> 4;
    const int xs = x0 + 4 * cq;                     // this lane's 4 columns
    const int nx = max(0, min(4, w - xs));
    const uint8_t* g2p = g2 + (long long)pair * g2_stride;
    uint8_t* mp = mask + (long long)pair * mask_stride;
    const bool vec = vec_ok && nx == 4;

    const PairFit& f = fits[pair];
    if (f.fit_status != 0) {   // no fit: the reference produces no mask; ours is all zero
        for (int i = 0; i < 4; i++) {
            const int y = y0 + 16 * wave + 4 * i + rr;
            if (y >= h) break;
            uint8_t* m = mp + (long long)y * w + xs;
            if (vec) *reinterpret_cast<uint32_t*>(m) = 0u;
            else for (int k = 0; k < nx; k++) m[k] = 0;
        }
        return;
    }
    double M[9];
#pragma unroll
    for (int k = 0; k < 9; k++) M[k] = f.Hinv[k];
    const uint8_t* src = g1 + (long long)pair * g1_stride;
    const bool affine = (M[6] == 0.0) && (M[7] == 0.0);
    const double Wd = M[8] != 0.0 ? 32.0 / M[8] : 0.0;   // affine: W = M8 everywhere

    TileInfo t;
    t.fast = 0;
    if (affine && bw0 == kWTile) t = tile_info(M, Wd, x0, y0, w, h, lane);
    if (!t.fast) {
        // ---- general path: per pixel, global gathers
        for (int i = 0; i < 4; i++) {
            const int y = y0 + 16 * wave + 4 * i + rr;
            if (y >= h) break;
            const uint8_t* g2r = g2p + (long long)y * g2_pitch + xs;
            uint8_t* m = mp + (long long)y * w + xs;
            for (int k = 0; k < nx; k++) m[k] = warp_px_general(M, src, g1_pitch, w, h, xs + k, y, bw0, g2r[k], thresh);
        }
        return;
    }

    // ---- fast path: stage the footprint, rows sya.., columns sxa.. (16-B chunks)
    if (tid < kHTile) {
        const int y = y0 + tid;
        s_xy[tid][0] = M[0] * x0 + M[1] * y + M[2];
        s_xy[tid][1] = M[3] * x0 + M[4] * y + M[5];
    }
    {
        const int nch = (t.sw + 15) >> 4;
        for (int e = tid; e < nch * t.sh; e += 256) {
            const int r = e / nch, ch = e - r * nch;
            const int sy = t.sya + r, sx = t.sxa + 16 * ch;
            uint4 v;
            if ((unsigned)sy < (unsigned)h && sx >= 0 && sx + 16 <= w) {
                const uint8_t* p = src + (long long)sy * g1_pitch + sx;
                v = *reinterpret_cast<const uint4*>(p);
            } else {
                uint32_t d[4] = {0, 0, 0, 0};
                if ((unsigned)sy < (unsigned)h) {
                    const uint8_t* p = src + (long long)sy * g1_pitch;
                    for (int i = 0; i < 16; i++) {
                        const int xx = sx + i;
                        if ((unsigned)xx < (unsigned)w) d[i >> 2] |= (uint32_t)p[xx] << (8 * (i & 3));
                    }
                }
                v = make_uint4(d[0], d[1], d[2], d[3]);
            }
            *reinterpret_cast<uint4*>(&s_src[r * kSP + 16 * ch]) = v;
        }
    }
    __syncthreads();
    if (nx == 0) return;

    const double magic = 6755399441055744.0;                 // 1.5 * 2^52
    const double mX = magic - 32.0 * t.sxa, mY = magic - 32.0 * t.sya;
    // 32/M8 a power of two -> (X0 + M0*x1) * Wd is exact and fuses with the rounding add
    const bool pow2 = Wd != 0.0 && (__double_as_longlong(Wd) & 0x000fffffffffffffLL) == 0;
    const uint32_t bias = 255u - (uint32_t)thresh;
    double tx[4], ty[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        tx[k] = M[0] * (4 * cq + k);
        ty[k] = M[3] * (4 * cq + k);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int r = 16 * wave + 4 * i + rr;
        const int y = y0 + r;
        if (y >= h) break;
        const double2 xy = *reinterpret_cast<const double2*>(s_xy[r]);
        const uint8_t* g2r = g2p + (long long)y * g2_pitch + xs;
        uint32_t G;
        if (vec) {
            G = *reinterpret_cast<const uint32_t*>(g2r);
        } else {
            G = 0;
            for (int k = 0; k < nx; k++) G |= (uint32_t)g2r[k] << (8 * k);
        }
        uint32_t e4[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const double ax = xy.x + tx[k], ay = xy.y + ty[k];
            double rx, ry;
            if (pow2) {
                rx = __builtin_fma(ax, Wd, mX);
                ry = __builtin_fma(ay, Wd, mY);
            } else {
                rx = ax * Wd + mX;
                ry = ay * Wd + mY;
            }
            const uint32_t X = (uint32_t)__double2loint(rx);   // cvRound((...)*Wd) - 32*sxa, >= 0
            const uint32_t Y = (uint32_t)__double2loint(ry);
            const uint32_t fx = X & 31u, fy = Y & 31u;
            const uint8_t* tp = s_src + (Y >> 5) * kSP + (X >> 5);
            const uint32_t v00 = tp[0], v01 = tp[1], v10 = tp[kSP], v11 = tp[kSP + 1];
            const uint32_t P = v00 | (v01 << 8) | (v10 << 16) | (v11 << 24);
            const uint32_t wxb = fx * 255u + 32u;                 // bytes (32 - fx, fx)
            const uint32_t h0 = __builtin_amdgcn_udot4(P, wxb, 0u, false);
            const uint32_t h1 = __builtin_amdgcn_udot4(P, wxb << 16, 0u, false);
            const uint32_t wy = fy * 65535u + 32u;                // u16 (32 - fy, fy)
            const uint32_t sv = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, h0 | (h1 << 16)),
                                                       __builtin_bit_cast(u16x2, wy), 512u, false);
            const uint32_t v = sv >> 10;
            e4[k] = __builtin_amdgcn_sad_u16(v, (G >> (8 * k)) & 255u, bias);   // |v - g| + bias: bit 8 iff > thresh
        }
        // byte 1 of each e4[k] is 0 or 1 -> pack, scale by 255
        const uint32_t p01 = __builtin_amdgcn_perm(e4[1], e4[0], 0x0c0c0501u);
        const uint32_t p23 = __builtin_amdgcn_perm(e4[3], e4[2], 0x0c0c0501u);
        const uint32_t b = p01 | (p23 << 16);
        const uint32_t out = (b << 8) - b;
        uint8_t* m = mp + (long long)y * w + xs;
        if (vec) *reinterpret_cast<uint32_t*>(m) = out;
        else for (int k = 0; k < nx; k++) m[k] = (uint8_t)(out >> (8 * k));
    }
}

hipError_t launch_warp_diff(hipStream_t s, int batch, const uint8_t* g1, long long g1_stride, int g1_pitch,
                            const uint8_t* g2, long long g2_stride, int g2_pitch, int w, int h, const PairFit* fits,
                            uint8_t* mask, long long mask_stride, int thresh)
{
    const int bh0 = h < 16 ? h : 16;
    const int bw0 = (1024 / bh0) < w ? (1024 / bh0) : w;
    // dword loads of gray2 / stores of the mask need 4-B aligned rows
    const int vec_ok = ((uintptr_t)g2 % 4 == 0) && g2_stride % 4 == 0 && g2_pitch % 4 == 0 &&
                       ((uintptr_t)mask % 4 == 0) && mask_stride % 4 == 0 && w % 4 == 0;
    const dim3 grid((w + kWTile - 1) / kWTile, (h + kHTile - 1) / kHTile, batch);
    hipLaunchKernelGGL(k_warp_diff, grid, dim3(256), 0, s, g1, g1_stride, g1_pitch, g2, g2_stride, g2_pitch, w, h, bw0,
                       fits, mask, mask_stride, thresh, vec_ok);
    return hipGetLastError();
}

}  // namespace mdx
