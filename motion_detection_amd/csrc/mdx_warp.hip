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
// Fast path (affine M, bw0 == 64, full-width tile over dword-aligned buffers, the tile's source
// footprint small): one 256-thread workgroup per 64 x 128 destination tile (= one reference block
// column, eight block rows).  Lane l of wave w owns the 4 columns x0 + 4*(l & 15) .. +3 of rows
// y0 + 32w + 4i + (l >> 4), i = 0..7, so gray2 loads / mask stores are dwords, 64 contiguous bytes
// per row.  Wave 0 computes the footprint; the workgroup stages it.
//   * The tile's source footprint (exact: X, Y are monotone in x and y for affine M, so the
//     four corners bound it) is staged once into LDS as raw bytes with ds_write_b128, zero
//     outside the image (= BORDER_CONSTANT 0 per tap), row pitch kSP = 96 B; taps are 4 byte
//     reads with immediate offsets (0, 1, 96, 97).
//   * Per column, M0*x1 and M3*x1 stay in registers (4 columns per lane); per row, X0 and Y0 come
//     from a 128-entry LDS table.  Per pixel: two FP64 adds and two multiply-adds with the magic
//     constant 1.5*2^52 - 32*origin, whose low word is cvRound(.) relative to the staged origin
//     (round-half-even, exact for |X| < 2^30, checked per tile).  When 32/M8 is a power of two the
//     multiply is exact and fuses with the rounding add into one FMA.
//   * Bilinear: w = (32-fx)(32-fy)*32 ... factorises exactly into three v_dot2_u32_u16 on taps
//     loaded straight into u16 halves (ds_read_u8_d16/_hi): q0 = dot(v00 v10, 32-fy fy),
//     q1 = dot(v01 v11, .), out = (dot(q0 q1, 32-fx fx) + 512) >> 10.
//   * |out - g2| + (32767 - thresh) has bit 15 set iff the pixel is moving (v_sad_u16); v_perm's
//     sign-replicating selectors turn four such bits into the four 0x00/0xff mask bytes.
// Everything else (perspective M, small frames, huge or far-away footprints) takes the general
// per-pixel path, exact for any input.
#include "mdx_internal.h"

#include <limits.h>

namespace mdx {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));


constexpr int kWTile = 64;              // tile = one reference block column (bw0 = 64)
#ifndef WX_TH
#define WX_TH 128
#endif
constexpr int kHTile = WX_TH;           // 16 * reference block rows (default 8 block rows)
#ifndef WX_SP
#define WX_SP 96
#endif
// staged row pitch, bytes.  96 (24 dwords) leaves some 2-way bank conflicts between the two tap
// rows a half-wave reads, but 15 KiB of LDS per workgroup lets 8 workgroups share a CU, which
// hides the staging latency better than the conflict-free 192 (measured 258 vs 284 us, 4K x32).
constexpr int kSP = WX_SP;
constexpr int kSH = 136;                // staged rows (tile height + rotation/scale margin)

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
__device__ TileInfo tile_info(const double* M, double Wd, int x0, int y0, int w, int yend, int lane)
{
    const int cxl = min(kWTile - 1, w - 1 - x0), cyl = min(kHTile - 1, yend - 1 - y0);
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

typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
// LDS pointers stay 32-bit (address space 3) through the inlined helper
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const d2v lds_d2;

// Fast-path rows of one lane: 4 columns x nrows rows (every 4th tile row from r0).  The tile is
// full width and the buffers dword-aligned (checked by the caller), so loads/stores are dwords.
template <bool POW2>
__device__ __forceinline__ void warp_rows(lds_d2* s_xy, lds_u8* s_src, int r0, int nrows, int y0, int xs,
                                          const uint8_t* g2p, int g2_pitch, uint8_t* mp, int w, const double* tx,
                                          const double* ty, double Wd, double mX, double mY, uint32_t bias)
{
    const uint8_t* g2r = g2p + (long long)(y0 + r0) * g2_pitch + xs;
    uint8_t* mr = mp + (long long)(y0 + r0) * w + xs;   // mp: mask row 0 of the pair's band, shifted by -row0
    const long long g2s = 4LL * g2_pitch, ms = 4LL * w;
    for (int i = 0; i < nrows; i++, g2r += g2s, mr += ms) {
        const d2v xy = s_xy[r0 + 4 * i];
#ifndef WX_NO_G2   // WX_*: timing-only builds (scripts/warp_variants.sh), results invalid
        const uint32_t G = *reinterpret_cast<const uint32_t*>(g2r);
#else
        const uint32_t G = (uint32_t)i * 0x01010101u;
#endif
        uint32_t wxs[4], wys[4], c0s[4], c1s[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const double ax = xy.x + tx[k], ay = xy.y + ty[k];
            double rx, ry;
            if (POW2) {
                rx = __builtin_fma(ax, Wd, mX);
                ry = __builtin_fma(ay, Wd, mY);
            } else {
                rx = ax * Wd + mX;
                ry = ay * Wd + mY;
            }
            const uint32_t X = (uint32_t)__double2loint(rx);   // cvRound((...)*Wd) - 32*sxa, >= 0
            const uint32_t Y = (uint32_t)__double2loint(ry);
            const uint32_t fx = X & 31u, fy = Y & 31u;
            const uint32_t off = __umul24(Y >> 5, (uint32_t)kSP) + (X >> 5);   // v_mad_u32_u24
            wxs[k] = fx * 65535u + 32u;                 // u16 (32 - fx, fx)
            wys[k] = fy * 65535u + 32u;                 // u16 (32 - fy, fy)
#ifndef WX_NO_TAPS
#ifdef WX_D16
            // taps straight into u16 halves: c0 = (v00, v10), c1 = (v01, v11)
            const uint32_t a = (uint32_t)(uintptr_t)(s_src + off);
            uint32_t c0, c1;
            asm volatile("ds_read_u8_d16 %0, %2\n\t"
                         "ds_read_u8_d16_hi %0, %2 offset:%3\n\t"
                         "ds_read_u8_d16 %1, %2 offset:1\n\t"
                         "ds_read_u8_d16_hi %1, %2 offset:%4"
                         : "=&v"(c0), "=&v"(c1) : "v"(a), "i"(kSP), "i"(kSP + 1));
            c0s[k] = c0;
            c1s[k] = c1;
#else
            c0s[k] = (uint32_t)s_src[off] | ((uint32_t)s_src[off + kSP] << 16);
            c1s[k] = (uint32_t)s_src[off + 1] | ((uint32_t)s_src[off + kSP + 1] << 16);
#endif
#else
            c0s[k] = (off & 255) | (((off >> 3) & 255) << 16);
            c1s[k] = ((off >> 5) & 255) | (((off >> 7) & 255) << 16);
#endif
        }
#if defined(WX_D16) && !defined(WX_NO_TAPS)
        // the asm loads are invisible to the compiler's waitcnt pass: wait here, and make every
        // tap register an operand so no use can be scheduled above the wait
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(c0s[0]), "+v"(c0s[1]), "+v"(c0s[2]), "+v"(c0s[3]), "+v"(c1s[0]), "+v"(c1s[1]),
                       "+v"(c1s[2]), "+v"(c1s[3])
                     :
                     : "memory");
#endif
        uint32_t e4[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // vertical then horizontal: sum_i v_i (32-fx|fx)(32-fy|fy), exact in integers
            const uint32_t q0 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, c0s[k]), __builtin_bit_cast(u16x2v, wys[k]), 0u, false);
            const uint32_t q1 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, c1s[k]), __builtin_bit_cast(u16x2v, wys[k]), 0u, false);
            const uint32_t sv = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2v, q0 | (q1 << 16)),
                                                       __builtin_bit_cast(u16x2v, wxs[k]), 512u, false);
            const uint32_t v = sv >> 10;
            // |v - g| + 32767 - thresh: bit 15 set iff |v - g| > thresh (value < 2^16)
            e4[k] = __builtin_amdgcn_sad_u16(v, (G >> (8 * k)) & 255u, bias);
        }
        // v_perm selectors 8 / 10 replicate bit 15 / bit 47 of {src0:src1}: 0xff or 0x00 bytes
        const uint32_t e01 = e4[0] | (e4[1] << 16), e23 = e4[2] | (e4[3] << 16);
        const uint32_t out = __builtin_amdgcn_perm(e23, e01, 0x0b0a0908u);
#ifndef WX_NO_STORE
        *reinterpret_cast<uint32_t*>(mr) = out;
#else
        if (out == bias) *reinterpret_cast<uint32_t*>(mr) = out;   // runtime-false: keeps the work
#endif
    }
}

// grid: x -> tile column, y -> tile row of the band [row0, row1), z -> pair.  256 threads; lane l
// of wave q owns columns x0 + 4*(l & 15) .. +3 of tile rows 32q + (l >> 4) + 4i, i = 0..7.  The
// reference's blocking depends on the full height only through bw0, and each pixel's arithmetic
// on (x, y) only, so a band is exactly the full frame's rows.
__global__ __launch_bounds__(256) void k_warp_diff(const uint8_t* __restrict__ g1, long long g1_stride, int g1_pitch,
                                                   const uint8_t* __restrict__ g2, long long g2_stride, int g2_pitch,
                                                   int w, int h, int bw0, const PairFit* __restrict__ fits,
                                                   uint8_t* __restrict__ mask, long long mask_stride, int thresh,
                                                   int vec_ok, int row0, int row1)
{
    __shared__ __attribute__((aligned(16))) double s_xy[kHTile][2];    // (X0, Y0) per tile row
    __shared__ __attribute__((aligned(16))) uint8_t s_src[kSH * kSP];
    __shared__ TileInfo s_info;

    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs; remap the linear id so
    // each XCD walks a contiguous run of tiles (row-major), and horizontally adjacent tiles --
    // which share the 128-B lines of their gray1 footprints and gray2 / mask rows -- meet in
    // the same L2 at about the same time.
    const int nbx = gridDim.x, nby = gridDim.y;
    int bid = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    {
        const int total = nbx * nby * gridDim.z, xcd = bid & 7, q8 = total >> 3, r8 = total & 7;
        bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    }
    const int pair = bid / (nbx * nby), tile = bid - pair * (nbx * nby);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x0 = (tile % nbx) * kWTile, y0 = row0 + (tile / nbx) * kHTile;
    const int cq = lane & 15, rr = lane >> 4;
    const int xs = x0 + 4 * cq;                     // this lane's 4 columns
    const int r0 = (kHTile / 4) * wave + rr;        // this lane's first tile row
    const int nrows = max(0, min(kHTile / 16, (row1 - y0 - r0 + 3) >> 2));
    const uint8_t* g2p = g2 + (long long)pair * g2_stride;
    uint8_t* mp = mask + (long long)pair * mask_stride - (long long)row0 * w;   // indexed by frame row

    const PairFit& f = fits[pair];
    if (f.fit_status != 0) {   // no fit: the reference produces no mask; ours is all zero
        const int nx = max(0, min(4, w - xs));
        for (int i = 0; i < nrows; i++) {
            uint8_t* m = mp + (long long)(y0 + r0 + 4 * i) * w + xs;
            for (int k = 0; k < nx; k++) m[k] = 0;
        }
        return;
    }
    double M[9];
#pragma unroll
    for (int k = 0; k < 9; k++) M[k] = f.Hinv[k];
    const uint8_t* src = g1 + (long long)pair * g1_stride;
    const bool affine = (M[6] == 0.0) && (M[7] == 0.0);
    const double Wd = M[8] != 0.0 ? 32.0 / M[8] : 0.0;   // affine: W = M8 everywhere
    // fast path only for full-width tiles over dword-aligned rows (uniform per workgroup)
    const bool try_fast = affine && bw0 == kWTile && vec_ok && x0 + kWTile <= w;

    if (try_fast && wave == 0) {
        const TileInfo t = tile_info(M, Wd, x0, y0, w, row1, lane);
        if (lane == 0) s_info = t;
    }
    if (try_fast) __syncthreads();
    const TileInfo t = s_info;
    if (!try_fast || !t.fast) {
        // ---- general path: per pixel, global gathers
        const int nx = max(0, min(4, w - xs));
        for (int i = 0; i < nrows; i++) {
            const int y = y0 + r0 + 4 * i;
            const uint8_t* g2r = g2p + (long long)y * g2_pitch + xs;
            uint8_t* m = mp + (long long)y * w + xs;
            for (int k = 0; k < nx; k++) m[k] = warp_px_general(M, src, g1_pitch, w, h, xs + k, y, bw0, g2r[k], thresh);
        }
        return;
    }

    // ---- fast path: per-row X0/Y0, then stage the footprint (rows sya.., 16-B chunks from sxa)
    if (tid < kHTile) {
        const int y = y0 + tid;
        s_xy[tid][0] = M[0] * x0 + M[1] * y + M[2];
        s_xy[tid][1] = M[3] * x0 + M[4] * y + M[5];
    }
    {
        const int nch = (t.sw + 15) >> 4;                 // <= kSP / 16
        const int rpp = 256 / nch;                        // rows per pass
        const int ro = tid / nch, ch = tid - ro * nch;    // once per thread
        const int sx = t.sxa + 16 * ch;
        const bool xin = sx >= 0 && sx + 16 <= w;
        if (ro < rpp) {
            for (int r = ro; r < t.sh; r += rpp) {
                const int sy = t.sya + r;
                uint4 v;
#ifdef WX_NO_STAGE
                if (true) {
                    v = make_uint4(sy, sx, r, ch);
#else
                if ((unsigned)sy < (unsigned)h && xin) {
                    v = *reinterpret_cast<const uint4*>(src + (long long)sy * g1_pitch + sx);
#endif
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
    }
    __syncthreads();
    if (nrows == 0) return;

    const double magic = 6755399441055744.0;                 // 1.5 * 2^52
    const double mX = magic - 32.0 * t.sxa, mY = magic - 32.0 * t.sya;
    // 32/M8 a power of two -> (X0 + M0*x1) * Wd is exact and fuses with the rounding add
    const bool pow2 = Wd != 0.0 && (__double_as_longlong(Wd) & 0x000fffffffffffffLL) == 0;
    const uint32_t bias = 32767u - (uint32_t)thresh;
    double tx[4], ty[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        tx[k] = M[0] * (4 * cq + k);
        ty[k] = M[3] * (4 * cq + k);
        asm volatile("" : "+v"(tx[k]), "+v"(ty[k]));   // keep in registers (no per-row rematerialisation)
    }
    lds_d2* xyp = (lds_d2*)(&s_xy[0][0]);
    lds_u8* srcp = (lds_u8*)(&s_src[0]);
    if (pow2)
        warp_rows<true>(xyp, srcp, r0, nrows, y0, xs, g2p, g2_pitch, mp, w, tx, ty, Wd, mX, mY, bias);
    else
        warp_rows<false>(xyp, srcp, r0, nrows, y0, xs, g2p, g2_pitch, mp, w, tx, ty, Wd, mX, mY, bias);
}

hipError_t launch_warp_diff(hipStream_t s, int batch, const uint8_t* g1, long long g1_stride, int g1_pitch,
                            const uint8_t* g2, long long g2_stride, int g2_pitch, int w, int h, const PairFit* fits,
                            uint8_t* mask, long long mask_stride, int thresh, int row0, int row1)
{
    if (row1 < 0) row1 = h;
    if (row0 < 0 || row1 > h || row0 >= row1) return hipErrorInvalidValue;
    const int bh0 = h < 16 ? h : 16;
    const int bw0 = (1024 / bh0) < w ? (1024 / bh0) : w;
    // dword loads of gray2 / stores of the mask need 4-B aligned rows
    const int vec_ok = ((uintptr_t)g2 % 4 == 0) && g2_stride % 4 == 0 && g2_pitch % 4 == 0 &&
                       ((uintptr_t)mask % 4 == 0) && mask_stride % 4 == 0 && w % 4 == 0;
    const dim3 grid((w + kWTile - 1) / kWTile, (row1 - row0 + kHTile - 1) / kHTile, batch);
    hipLaunchKernelGGL(k_warp_diff, grid, dim3(256), 0, s, g1, g1_stride, g1_pitch, g2, g2_stride, g2_pitch, w, h, bw0,
                       fits, mask, mask_stride, thresh, vec_ok, row0, row1);
    return hipGetLastError();
}

}  // namespace mdx
