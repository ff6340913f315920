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
// Fast path (affine M, bw0 == 64, dword-aligned buffers, the tile's source footprint small): one
// 256-thread workgroup per 128 x 64 destination tile (two reference block columns; 64 rows
// measured best: 32 doubles the per-tile setup, 128 halves the workgroups a CU holds).  Lane l of
// wave w owns the 4 columns x0 + 4*(l & 31) .. +3 of rows y0 + 8i + 2w + (l >> 5), i = 0..7: a
// half-wave is one tile row, so gray2 loads / mask stores are dwords, 128 contiguous bytes.
//   * Footprint: X, Y are monotone in x and y inside a reference block for affine M, so the eight
//     block corners bound the tile's taps exactly.  It is staged once into LDS as raw bytes by
//     LDS-DMA (buffer_load ... lds, 16 B per lane, 4 staged rows per wave instruction), zero
//     outside the image (= BORDER_CONSTANT 0 per tap), at a row pitch of 256 B.
//   * Coordinates, per pixel: one FP64 add (per-row X0 from an LDS table + per-column M0*x1 in
//     registers) and one FMA with the magic constant 1.5*2^52 - 32*origin per axis, whose low word
//     is cvRound(32*(...)) - 32*origin (round-half-even, exact for |X| < 2^30, checked per tile).
//     When 32/M8 is not a power of two the product (...)*Wd is rounded first, as the reference
//     does, and the add only rounds it to an integer.
//   * Shifted left by 3, byte 1 of each low word is the staged source column (row) and bits 3..7
//     are 8*fx (8*fy): the tap address (row << 8 | col) is ONE v_perm, and 8*f indexes a 32-entry
//     LDS weight table (entry f: wy = (32-f, f), wx = 64*(32-f, f)).
//   * Taps: four byte reads per pixel, c0 = (v00, v01), c1 = (v10, v11) as u16 halves.  Vertical
//     with two packed u16 ops (op_sel splats the weight halves), q = c0*(32-fy) + c1*fy =
//     (q0, q1) <= 8160; horizontal with one v_dot2_u32_u16: s = 64*(q0 (32-fx) + q1 fx) + 32.
//   * Threshold without the >> 10: out = (S + 512) >> 10 with S = (s - 32)/64, and
//     |out - g| > t  <=>  |s - 65536 g| >= 65536 t + 32800 (exact).
//     v_sad_u32(s, g << 16, 2^31 - 65536 t - 32800) sets bit 31 iff the pixel moves (g << 16 is
//     one v_perm of the gray2 dword); v_perm's sign-replicating selectors turn the four flags
//     into the four 0x00/0xff mask bytes.
//   * gray2 loads / mask stores go through buffer descriptors: lanes past the right edge get an
//     out-of-range offset and rows past the band fall outside the mask descriptor, so the row
//     loop is branch-free.  ~17 VALU per pixel (4 of them FP64), vs ~23 for the 64x128-tile
//     design before it (rocprofv3 SQ_INSTS_VALU).
// Projective M (M6 or M7 != 0, e.g. every non-degenerate first-4 fit) takes the same tiles: the
// tile's footprint is the bounding box of its reference blocks' corner images (the homography maps
// the tile to a convex quadrilateral when W keeps one sign over it) widened by one pixel for the
// rounding of interior pixels; each pixel's coordinates come from a cheap estimate of the quotient,
// settled with the reference's exact expression when it lies near a rounding boundary (warp_rows_pj).
// Everything else (W changing sign over a tile, small frames, huge or far-away footprints) takes
// the general per-pixel path, exact for any input.
#include "mdx_internal.h"

#include <limits.h>

namespace mdx {

typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));

constexpr int kTW = 128;     // tile width: two reference block columns (bw0 = 64)
constexpr int kBW = 64;      // reference block width of the fast path
constexpr int kTH = 64;      // tile rows
constexpr int kSP = 256;     // staged row pitch: tap address = (row << 8) | col, one v_perm
constexpr int kSH = kTH + 12;   // staged rows (tile height + scale/rotation margin)

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
    double wd;         // 32 / M8 (affine: W = M8 everywhere), 0 when M8 == 0; projective: unused
    int fast;          // 1: fast path usable for this tile
    int sxa, sya;      // staged origin (sxa multiple of 16)
    int sw, sh;        // staged width (bytes), height (rows)
};

// Bounds of the tile's taps, from the reference arithmetic at the corners of its (one or two)
// reference blocks, one corner per lane of an aligned group of 8 (lane = its index in the group;
// every lane of the group returns the result); fast = every |X|, |Y| < 2^30 (no clamp, magic
// rounding exact) and the footprint fits the staging buffer.  Affine M: X and Y are monotone in x
// and y inside a block, so the corners bound every pixel's taps exactly.  Projective M: W is
// linear in (x, y), so if it has one sign (and a sane magnitude) at the corners it has it over the
// whole tile, the tile's image is the convex hull of the corner images, and X / W, Y / W take their
// extremes at the corners (linear-fractional); interior pixels' rounded coordinates can exceed the
// corners' by one 1/32 unit, so the footprint is widened by one pixel on every side.
__device__ TileInfo tile_info(const double* M, int x0, int y0, int w, int yend, int lane)
{
    const bool affine = M[6] == 0.0 && M[7] == 0.0;
    const int nb = (x0 + kBW < w) ? 2 : 1;                       // reference blocks in the tile
    const int b = ((lane >> 2) & 1) < nb ? ((lane >> 2) & 1) : 0;
    const int xb = x0 + kBW * b;
    const int cxl = min(kBW - 1, w - 1 - xb), cyl = min(kTH - 1, yend - 1 - y0);
    const int c = lane & 3;
    const int x1 = (c & 1) ? cxl : 0, y = y0 + ((c & 2) ? cyl : 0);
    const double X0 = M[0] * xb + M[1] * y + M[2];
    const double Y0 = M[3] * xb + M[4] * y + M[5];
    double Wd = M[8] != 0.0 ? 32.0 / M[8] : 0.0;
    int wsign = 1;
    if (!affine) {                                               // the reference's per-pixel W
        const double W0 = M[6] * xb + M[7] * y + M[8];
        const double Wv = W0 + M[6] * x1;
        Wd = Wv != 0.0 ? 32.0 / Wv : 0.0;
        const double aw = fabs(Wv);
        // W in [2^-100, 2^100] at every corner (so over the tile): div32's range; |W| >= 64 |M6|:
        // W0 + M6 * x1 does not cancel (warp_rows_pj's estimate)
        wsign = (aw >= 0x1p-100 && aw <= 0x1p100 && aw >= 64.0 * fabs(M[6])) ? (Wv > 0.0 ? 1 : 2) : 0;
    }
    const double px = (X0 + M[0] * x1) * Wd, py = (Y0 + M[3] * x1) * Wd;
    const double lim = affine ? 1073741824.0 : 16777216.0;   // 2^30; projective 2^24 (warp_rows_pj's bound)
    int ok = (px > -lim && px < lim && py > -lim && py < lim && wsign != 0) ? 1 : 0;
    int smin = wsign, smax = wsign;
    int sx = 0, sy = 0;
    if (ok) {
        sx = ((int)__builtin_rint(px)) >> 5;
        sy = ((int)__builtin_rint(py)) >> 5;
    }
    int sx_lo = sx, sx_hi = sx, sy_lo = sy, sy_hi = sy;
#pragma unroll
    for (int m = 1; m <= 4; m <<= 1) {
        sx_lo = min(sx_lo, __shfl_xor(sx_lo, m, 8));
        sx_hi = max(sx_hi, __shfl_xor(sx_hi, m, 8));
        sy_lo = min(sy_lo, __shfl_xor(sy_lo, m, 8));
        sy_hi = max(sy_hi, __shfl_xor(sy_hi, m, 8));
        ok = min(ok, __shfl_xor(ok, m, 8));
        smin = min(smin, __shfl_xor(smin, m, 8));
        smax = max(smax, __shfl_xor(smax, m, 8));
    }
    if (!affine) {
        ok = ok && smin == smax;                               // W keeps its sign over the tile
        sx_lo -= 1; sy_lo -= 1; sx_hi += 1; sy_hi += 1;        // interior rounding margin
    }
    TileInfo t;
    t.wd = Wd;
    t.sxa = sx_lo & ~15;
    t.sya = sy_lo;
    t.sw = sx_hi - t.sxa + 2;                  // bytes: columns sxa .. sx_hi + 1
    t.sh = sy_hi - t.sya + 2;                  // rows sya .. sy_hi + 1
    t.fast = ok && t.sw > 0 && t.sh > 0 && t.sw <= kSP && t.sh <= kSH;
    return t;
}

// LDS pointers stay 32-bit (address space 3) through the inlined helpers
typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef double d2v __attribute__((ext_vector_type(2)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const d2v lds_d2;

// raw buffer descriptor over [base, base + bytes): out-of-range loads return 0 and stores are
// dropped, which is how lanes past the right edge and rows past the band go quiet.
// (The clamp is done on the 32-bit halves: a 64-bit signed min has no scalar instruction, and
// the compiler put it on the VALU.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, long long bytes)
{
    uint32_t hi = (uint32_t)((unsigned long long)bytes >> 32), lo = (uint32_t)bytes;
    asm("" : "+s"(hi), "+s"(lo));   // keep the halves apart (else it is re-fused into a VALU compare)
    const int n = (int)min(lo | (0u - (uint32_t)(hi != 0u)), 0x7fffffffu);   // bytes >= 0
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, n, 0x00020000);
}

// Fast-path rows of one lane: 4 columns x 8 rows (tile rows r0 + 8i).  xyp points at this lane's
// (X0, Y0) of row r0 and block; tab8 at the weight table (entry f at byte 8f: (32-f, f), then
// 64*(32-f, f)); src_base is the staged footprint.  g2 / mask go through buffer descriptors whose
// per-lane offsets are out of range for idle lanes; ROWCHK (partial tiles) sends rows past the
// band to row r0's coordinates so every tap stays inside the footprint.
// Cache policy of the streamed operands: gray2 is read once and the mask written once, so both go
// non-temporal (nt).  The staged footprint keeps the default policy: adjacent tiles share its margin
// lines in L2.  4K x 32 launch, alternating on one box: 216-224 us with nt on gray2 + mask, 233-235
// without, 230-234 with nt on the footprint too, 222-224 with nt on the mask only; on a second box
// 211-220 with nt against 223-229 without.
constexpr int kCpStream = 2;   // buffer aux bit 1 = nt
// 32 / d correctly rounded, for |d| in [2^-100, 2^100] (tile_info keeps the fast path there): the
// compiler's IEEE double division without its v_div_scale / v_div_fixup steps, which only act on
// exponents far outside that range (huge quotients, denormals, inf / nan) -- two Newton steps on
// v_rcp_f64, the quotient, and the final FMA correction that rounds it correctly.  8 FP64
// instructions instead of 11.  tests/test_warp_gpu.py checks it bit for bit against IEEE division
// over that range (mdx_debug_div32).
__device__ __forceinline__ double div32(double d)
{
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0);
    const double r2 = __builtin_fma(r1, e1, r1);
    const double q0 = 32.0 * r2;
    const double rem = __builtin_fma(-d, q0, 32.0);
    return __builtin_fma(rem, r2, q0);
}
template <bool POW2, bool ROWCHK>
__device__ __forceinline__ void warp_rows(lds_d2* xyp, lds_u8* tab8, uint32_t src_base, int nvalid,
                                          __amdgpu_buffer_rsrc_t g2rs, uint32_t g2off, int g2s,
                                          __amdgpu_buffer_rsrc_t mrs, uint32_t moff, int ms, const double* tx,
                                          const double* ty, double Wd, double mX, double mY, uint32_t bias)
{
    uint32_t G[kTH / 8];
#pragma unroll
    for (int i = 0; i < kTH / 8; i++) G[i] = __builtin_amdgcn_raw_buffer_load_b32(g2rs, (int)g2off, i * g2s, kCpStream);
#pragma unroll
    for (int i = 0; i < kTH / 8; i++) {
        const int ri = ROWCHK ? (i < nvalid ? i : 0) : i;
        const d2v xy = xyp[16 * ri];                      // rows are 2 blocks x 16 B apart
        uint32_t xs_[4], ys_[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const double ax = xy.x + tx[k], ay = xy.y + ty[k];
            double rx, ry;
            if (POW2) {                            // (X0 + M0*x1) * Wd exact: one rounding
                rx = __builtin_fma(ax, Wd, mX);
                ry = __builtin_fma(ay, Wd, mY);
            } else {                                      // round the product, then to integer
                rx = ax * Wd + mX;
                ry = ay * Wd + mY;
            }
            xs_[k] = (uint32_t)__double2loint(rx);        // X - 32 * sxa
            ys_[k] = (uint32_t)__double2loint(ry);        // Y - 32 * sya
        }
        uint32_t ad[4], wys[4], wxs[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // 8X: byte 1 is the staged column (row), bits 3..7 index the 8-B weight table
            const uint32_t lx = xs_[k] << 3, ly = ys_[k] << 3;
            ad[k] = src_base + __builtin_amdgcn_perm(ly, lx, 0x0c0c0501u);   // (row << 8) | col
            wys[k] = *(lds_u32*)(tab8 + (ly & 0xf8u));       // (32 - fy, fy)
            wxs[k] = *(lds_u32*)(tab8 + (lx & 0xf8u) + 4);   // 64 * (32 - fx, fx)
        }
        // taps: four byte reads per pixel, c0 = (v00, v01), c1 = (v10, v11) as u16 halves.
        // (ds_read_*_d16_hi does not preserve the low half on gfx950 with SRAM ECC, and unaligned
        // ds_read_u16 is correct but ~4x slower here.)
        uint32_t c0s[4], c1s[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            lds_u8* p = (lds_u8*)(uintptr_t)ad[k];
            c0s[k] = (uint32_t)p[0] | ((uint32_t)p[1] << 16);
            c1s[k] = (uint32_t)p[kSP] | ((uint32_t)p[kSP + 1] << 16);
        }
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u16x2v c0 = __builtin_bit_cast(u16x2v, c0s[k]), c1 = __builtin_bit_cast(u16x2v, c1s[k]);
            const u16x2v wy = __builtin_bit_cast(u16x2v, wys[k]);
            const u16x2v q = c0 * wy.xx + c1 * wy.yy;     // (q0, q1): vertical, exact in u16
            const uint32_t s = __builtin_amdgcn_udot2(q, __builtin_bit_cast(u16x2v, wxs[k]), 32u, false);
            const uint32_t g16 = __builtin_amdgcn_perm(0u, G[i], 0x0c000c0cu | ((uint32_t)k << 16));   // g_k << 16
            asm("v_sad_u32 %0, %1, %2, %3" : "=v"(e[k]) : "v"(s), "v"(g16), "s"(bias));   // bit 31: moving
        }
        // v_perm selectors 9 / 11 replicate bit 31 of src1 / src0: 0xff or 0x00 bytes
        const uint32_t out = __builtin_amdgcn_perm(e[1], e[0], 0x0c0c0b09u) | __builtin_amdgcn_perm(e[3], e[2], 0x0b090c0cu);
        __builtin_amdgcn_raw_buffer_store_b32(out, mrs, (int)moff, i * ms, kCpStream);
    }
}

// Fixed-point rows (32/M8 a power of two, i.e. (X0 + M0*x1) * Wd exact).  The reference's
//   X = cvRound(Wd * fl(X0 + fl(M0*x1)))
// relative to the staged origin, plus 1/2, is held as a 32-bit fixed-point number
//   U = [ staged column (8 bits) | fx (5 bits) | fraction (19 bits) ]
// = A(row, block) + B(x1): A = floor(2^19 (Wd*X0 + 1/2 - 32*sxa)), B = floor(2^19 Wd fl(M0*x1)), so a
// pixel's coordinates are one 32-bit add per axis and floor(U / 2^19) = X - 32*sxa whenever the
// fraction of U lies in [1, 2^19 - 3]: the two truncations err by less than 2 units, the double
// rounding of fl(X0 + t1) by < 2^-17 units, so the true value is in (U - 1, U + 3) and cannot cross
// an integer (an exact tie, a true fraction of 0, is caught the same way).  Pixels outside that
// range (about 4 in 2^19) take the reference's FP64 expression.  They are found in two steps: the
// workgroup's per-axis bucket map marks every fraction of A that any column x1 of a block could
// turn bad (a row-block whose A falls in a marked bucket carries a flag in s_fx), and only lanes of
// flagged row-blocks test their four pixels.  Then, per pixel: the tap address is byte 3 of the two
// sums (one v_perm), the bilinear weight pairs come from fx, fy arithmetically (v_bfe + v_mad_u24:
// f * 65535 + 32 = (32 - f) | f << 16), and the rest is warp_rows's.
#ifndef MDX_WARP_BM_BITS
#define MDX_WARP_BM_BITS 13
#endif
constexpr int kBmBits = MDX_WARP_BM_BITS;     // bucket map: 2^kBmBits buckets of 2^(19 - kBmBits) units per axis
static_assert(kBmBits <= 16, "a bad range (5 units) must span at most two buckets");
typedef __attribute__((address_space(3))) const v4u lds_u4;
template <bool ROWCHK>
__device__ __forceinline__ void warp_rows_fx(lds_u4* fxp, lds_d2* xyp, uint32_t src_base, int nvalid,
                                             const uint32_t (&G)[kTH / 8], __amdgpu_buffer_rsrc_t mrs, uint32_t moff,
                                             int ms, const uint32_t (&bx)[4], const uint32_t (&by)[4], double M0,
                                             double M3, int x1b, double Wd, double mX, double mY, uint32_t bias)
{
    // loop constants held in registers once (gfx9 VOP3 takes no literals: otherwise each row would
    // rematerialise them with v_mov): the gray2 byte selectors in SGPRs, the wx multiplier in a VGPR
    uint32_t gsel[4], mulx;
    asm volatile("s_mov_b32 %0, 0x0c000c0c" : "=s"(gsel[0]));
    asm volatile("s_mov_b32 %0, 0x0c010c0c" : "=s"(gsel[1]));
    asm volatile("s_mov_b32 %0, 0x0c020c0c" : "=s"(gsel[2]));
    asm volatile("s_mov_b32 %0, 0x0c030c0c" : "=s"(gsel[3]));
    asm volatile("v_mov_b32 %0, 0x3fffc0" : "=v"(mulx));    // 64 * 65535
#pragma unroll
    for (int i = 0; i < kTH / 8; i++) {
        const int ri = ROWCHK ? (i < nvalid ? i : 0) : i;
        const v4u f = fxp[16 * ri];                     // (A_x, A_y, flag) of this lane's row and block
        uint32_t ux[4], uy[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            ux[k] = f.x + bx[k];
            uy[k] = f.y + by[k];
        }
        if (f.z) {
            // near a rounding boundary somewhere in this row-block: settle each pixel of this lane
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (((ux[k] & 0x7ffffu) - 1u) > 0x7fffcu || ((uy[k] & 0x7ffffu) - 1u) > 0x7fffcu) {
                    const d2v xy = xyp[16 * ri];
                    const double x1 = (double)(x1b + k);
                    const double ax = xy.x + M0 * x1, ay = xy.y + M3 * x1;
                    ux[k] = (uint32_t)__double2loint(__builtin_fma(ax, Wd, mX)) << 19;
                    uy[k] = (uint32_t)__double2loint(__builtin_fma(ay, Wd, mY)) << 19;
                }
            }
        }
        uint32_t ad[4], wys[4], wxs[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            ad[k] = src_base + __builtin_amdgcn_perm(uy[k], ux[k], 0x0c0c0703u);   // (row << 8) | col
            const uint32_t fx = __builtin_amdgcn_ubfe(ux[k], 19, 5), fy = __builtin_amdgcn_ubfe(uy[k], 19, 5);
            wys[k] = __umul24(fy, 65535u) + 32u;               // (32 - fy, fy)
            wxs[k] = __umul24(fx, mulx) + 2048u;               // 64 * (32 - fx, fx)
        }
        uint32_t c0s[4], c1s[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            lds_u8* p = (lds_u8*)(uintptr_t)ad[k];
            c0s[k] = (uint32_t)p[0] | ((uint32_t)p[1] << 16);
            c1s[k] = (uint32_t)p[kSP] | ((uint32_t)p[kSP + 1] << 16);
        }
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u16x2v c0 = __builtin_bit_cast(u16x2v, c0s[k]), c1 = __builtin_bit_cast(u16x2v, c1s[k]);
            const u16x2v wy = __builtin_bit_cast(u16x2v, wys[k]);
            const u16x2v q = c0 * wy.xx + c1 * wy.yy;
            const uint32_t s = __builtin_amdgcn_udot2(q, __builtin_bit_cast(u16x2v, wxs[k]), 32u, false);
            const uint32_t g16 = __builtin_amdgcn_perm(0u, G[i], gsel[k]);
            asm("v_sad_u32 %0, %1, %2, %3" : "=v"(e[k]) : "v"(s), "v"(g16), "s"(bias));
        }
        const uint32_t out = __builtin_amdgcn_perm(e[1], e[0], 0x0c0c0b09u) | __builtin_amdgcn_perm(e[3], e[2], 0x0b090c0cu);
        __builtin_amdgcn_raw_buffer_store_b32(out, mrs, (int)moff, i * ms, kCpStream);
    }
}

// Projective rows.  The reference's X = cvRound(fl(fl(X0 + fl(M0*x1)) * fl(32 / fl(W0 + fl(M6*x1))))) is
// taken in two steps.  First an estimate, in warp_rows_fx's fixed-point layout relative to the
// staged origin (U = [ staged column (8 bits) | fx (5 bits) | fraction (19 bits) ], U ~ 2^19 (X' + 1/2)):
// r ~ 2^24 / W from v_rcp_f64 and one quadratic Newton step (rcp's relative error e -> e^2:
// measured at most 2^-24.4 -> 2^-48.7 over 16 M values, scripts/micro/rcp64_acc.hip; round 5 used a
// cubic step), one reciprocal per four pixels (of the product of their W), then
// U = RN(ax * r + 2^18 - 2^24 sxa), one FMA per axis.  The estimate's operands need not be the
// reference's roundings: ax and W / 2^24 of column x1b + k come from the lane's column x1b by k
// adds of the per-column steps, so no per-column table is held in registers.  tile_info keeps projective fast tiles at |X|, |Y| <
// 2^24 (1/32 px units) and |W| >= 64 |M6| at the corners (no cancellation in W0 + M6 * x1), so the
// estimate stays within 2^24 * 2^19 * 2^-47 = 1/16 unit of 2^-19 of the exact quotient and the
// reference within 2^-9 unit (an rcp 16x less accurate than measured would still give < 8 units):
// whenever U's fraction is at least kPjGuard units from the boundary (0), floor(U / 2^19)
// is the reference's X' and not a tie.  The other pixels (64 of every 2^19 fractions per axis) take
// the exact form: W, the correctly rounded 32/W (div32) and the rounded product.  Then the taps,
// weights and threshold are warp_rows_fx's.
constexpr uint32_t kPjGuard = 32;
__device__ __forceinline__ bool pj_near(uint32_t u)
{
    return ((u + kPjGuard) & 0x7ffffu) < 2 * kPjGuard;
}
__device__ __forceinline__ void warp_rows_pj(lds_d2* xyp, lds_d2* wpp, uint32_t src_base, int nvalid,
                                             __amdgpu_buffer_rsrc_t g2rs, uint32_t g2off, int g2s,
                                             __amdgpu_buffer_rsrc_t mrs, uint32_t moff, int ms, double tx0, double ty0,
                                             double tws0, const double* M, int x1b, double mX, double mY, double mXs,
                                             double mYs, uint32_t bias)
{
    uint32_t G[kTH / 8];
#pragma unroll
    for (int i = 0; i < kTH / 8; i++) G[i] = __builtin_amdgcn_raw_buffer_load_b32(g2rs, (int)g2off, i * g2s, kCpStream);
    uint32_t gsel[4], mulx;
    asm volatile("s_mov_b32 %0, 0x0c000c0c" : "=s"(gsel[0]));
    asm volatile("s_mov_b32 %0, 0x0c010c0c" : "=s"(gsel[1]));
    asm volatile("s_mov_b32 %0, 0x0c020c0c" : "=s"(gsel[2]));
    asm volatile("s_mov_b32 %0, 0x0c030c0c" : "=s"(gsel[3]));
    asm volatile("v_mov_b32 %0, 0x3fffc0" : "=v"(mulx));    // 64 * 65535
    const double M6s = M[6] * 0x1p-24;
#pragma unroll
    for (int i = 0; i < kTH / 8; i++) {
        const int ri = i < nvalid ? i : 0;                // rows past the band: row r0's coordinates
        const d2v xy = xyp[16 * ri];                      // (X0, Y0) of this lane's row and block
        const d2v wv = wpp[16 * ri];                      // (W0, W0 / 2^24)
        const double ax0 = xy.x + tx0, ay0 = xy.y + ty0, ws0 = wv.y + tws0;
        uint32_t ux[4], uy[4];
        uint32_t fmin = 0xffffffffu;                      // the smallest guard-shifted fraction (x 2^13)
        // the four reciprocals from ONE v_rcp_f64 (a transcendental, several times an FMA's issue
        // cost) of the product of the four W: 1/W_k = (product of the other three) / P.  Six more
        // roundings of 2^-53 keep r within 2^-48 of 2^24 / W (the guard needs 2^-40, see above);
        // |W| in [2^-100, 2^100] (tile_info) keeps P inside FP64's range
        // column x1b + k by k adds of the per-column steps (the estimate needs accuracy, not the
        // reference's roundings: 3 more roundings of 2^-53), the steps are scalar operands
        double Ws[4];
        Ws[0] = ws0;                                      // ~ W / 2^24
#pragma unroll
        for (int k = 1; k < 4; k++) Ws[k] = Ws[k - 1] + M6s;
        const double P01 = Ws[0] * Ws[1], P23 = Ws[2] * Ws[3], P = P01 * P23;
        const double R0 = __builtin_amdgcn_rcp(P);
        const double R = __builtin_fma(R0, __builtin_fma(-P, R0, 1.0), R0);
        const double R01 = R * P23, R23 = R * P01;       // 1 / P01, 1 / P23
        const double rk[4] = {Ws[1] * R01, Ws[0] * R01, Ws[3] * R23, Ws[2] * R23};
        double ax = ax0, ay = ay0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (k) {
                ax = ax + M[0];
                ay = ay + M[3];
            }
            ux[k] = (uint32_t)__double2loint(__builtin_fma(ax, rk[k], mXs));
            uy[k] = (uint32_t)__double2loint(__builtin_fma(ay, rk[k], mYs));
            // ((u + G) & 0x7ffff) < 2G  <=>  (u << 13) + (G << 13) < 2G << 13 (mod 2^32): one
            // v_lshl_add_u32 per value instead of an add and an and
            fmin = min(fmin, min((ux[k] << 13) + (kPjGuard << 13), (uy[k] << 13) + (kPjGuard << 13)));
        }
        if (fmin < (2 * kPjGuard) << 13) {
            // within the guard of a rounding boundary (or on a tie): the reference's expression
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t uxk = ux[k], uyk = uy[k];
                asm volatile("" : "+v"(uxk), "+v"(uyk));   // tested here, per pixel, only on this rare path
                if (pj_near(uxk) || pj_near(uyk)) {
                    const double x1 = (double)(x1b + k);
                    const double Wk = div32(wv.x + M[6] * x1);   // 32 / W, correctly rounded
                    ux[k] = (uint32_t)__double2loint((xy.x + M[0] * x1) * Wk + mX) << 19;
                    uy[k] = (uint32_t)__double2loint((xy.y + M[3] * x1) * Wk + mY) << 19;
                }
            }
        }
        uint32_t ad[4], wys[4], wxs[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            ad[k] = src_base + __builtin_amdgcn_perm(uy[k], ux[k], 0x0c0c0703u);   // (row << 8) | col
            const uint32_t fx = __builtin_amdgcn_ubfe(ux[k], 19, 5), fy = __builtin_amdgcn_ubfe(uy[k], 19, 5);
            wys[k] = __umul24(fy, 65535u) + 32u;               // (32 - fy, fy)
            wxs[k] = __umul24(fx, mulx) + 2048u;               // 64 * (32 - fx, fx)
        }
        uint32_t c0s[4], c1s[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            lds_u8* p = (lds_u8*)(uintptr_t)ad[k];
            c0s[k] = (uint32_t)p[0] | ((uint32_t)p[1] << 16);
            c1s[k] = (uint32_t)p[kSP] | ((uint32_t)p[kSP + 1] << 16);
        }
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u16x2v c0 = __builtin_bit_cast(u16x2v, c0s[k]), c1 = __builtin_bit_cast(u16x2v, c1s[k]);
            const u16x2v wy = __builtin_bit_cast(u16x2v, wys[k]);
            const u16x2v q = c0 * wy.xx + c1 * wy.yy;
            const uint32_t s = __builtin_amdgcn_udot2(q, __builtin_bit_cast(u16x2v, wxs[k]), 32u, false);
            const uint32_t g16 = __builtin_amdgcn_perm(0u, G[i], gsel[k]);
            asm("v_sad_u32 %0, %1, %2, %3" : "=v"(e[k]) : "v"(s), "v"(g16), "s"(bias));
        }
        const uint32_t out = __builtin_amdgcn_perm(e[1], e[0], 0x0c0c0b09u) | __builtin_amdgcn_perm(e[3], e[2], 0x0b090c0cu);
        __builtin_amdgcn_raw_buffer_store_b32(out, mrs, (int)moff, i * ms, kCpStream);
    }
}

// footprint chunks that cross the image's left / right edge: byte by byte, 0 outside (kept out of
// line so its per-byte bounds are not computed on the interior path)
__device__ __noinline__ void stage_edge_chunks(const uint8_t* src, int pitch, int w, int h, int sya, int sx, int ro,
                                               int rpp, int sh, uint8_t* dst)
{
    for (int r = ro; r < sh; r += rpp) {
        const int sy = sya + r;
        uint32_t d[4] = {0, 0, 0, 0};
        if ((unsigned)sy < (unsigned)h) {
            const uint8_t* p = src + (long long)sy * pitch;
            for (int i = 0; i < 16; i++) {
                const int xx = sx + i;
                if ((unsigned)xx < (unsigned)w) d[i >> 2] |= (uint32_t)p[xx] << (8 * (i & 3));
            }
        }
        *reinterpret_cast<uint4*>(dst + r * kSP) = make_uint4(d[0], d[1], d[2], d[3]);
    }
}

#ifndef MDX_WARP_STAMP
#define MDX_WARP_STAMP 0
#endif
#if MDX_WARP_STAMP
// Diagnostic build only (-DMDX_WARP_STAMP=1, scripts/warp_burst.py): per launch, 64 sampled workgroups'
// thread 0 stamps s_memtime (shader clock) and s_memrealtime (100 MHz) at its start and end, so the
// in-kernel clock of every launch of a burst is Δmemtime / Δmemrealtime x 100 MHz
// (MI355X_MICROARCH.md DVFS item 6).  k_warp_prep counts the launches.
constexpr int kStampLaunches = 1024, kStampSamples = 64;
__device__ unsigned int g_warp_launch;
__device__ unsigned long long g_warp_stamps[kStampLaunches * kStampSamples * 4];
hipError_t debug_warp_stamps(void* dst, size_t bytes)
{
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_warp_stamps), bytes < sizeof(g_warp_stamps) ? bytes : sizeof(g_warp_stamps));
}
#define WARP_DIFF_FN __device__ __forceinline__ void warp_diff_tile
#else
#define WARP_DIFF_FN __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_warp_diff
#endif

// n / d for uniform n, d < 2^31 with m = udiv_magic_of(d) = floor(2^32 / d) (d >= 2; m = 0 for d = 1):
// the estimate mulhi(n, m) is q or q - 1, one correction makes it exact; all scalar instructions
static inline uint32_t udiv_magic_of(uint32_t d)
{
    return d > 1 ? (uint32_t)(0x100000000ull / d) : 0u;
}
__device__ __forceinline__ uint32_t udiv_magic(uint32_t n, uint32_t d, uint32_t m)
{
    if (d == 1) return n;
    uint32_t q = __umulhi(n, m);
    if (n - q * d >= d) q++;
    return q;
}

// Per-pair tables of the fixed-point path, made once per launch by k_warp_prep instead of once per
// tile: B(x1) = floor(2^19 Wd fl(M*x1)) per axis and column of a block, and the bucket maps (for
// column x1, A's fraction is bad iff it lies within -B(x1) - 3 .. -B(x1) + 1 mod 2^19; the buckets
// of those fractions are marked, one or two per column and axis).
struct WarpPrep {
    uint32_t B[2][kBW];
    uint32_t bm[2][(1 << kBmBits) / 32];
};

// floor(v) mod 2^32 for |v| < 2^51: the integer plus 1.5 * 2^52 is exact with ulp 1, so its low word
// is the two's-complement low word of floor(v) (a double -> int64 conversion is a multi-instruction
// sequence on gfx950)
__device__ __forceinline__ uint32_t floor_lo(double v)
{
    return (uint32_t)__double2loint(__builtin_floor(v) + 6755399441055744.0);
}

// grid: x -> 1 + tile groups, y -> pair.  Block 0 of a pair builds its WarpPrep; every other block
// takes 32 tiles, one aligned group of 8 lanes per tile, and writes their TileInfo.
__global__ __launch_bounds__(256) void k_warp_prep(const PairFit* __restrict__ fits, int w, int row0, int row1,
                                                   int nbx, int nby, TileInfo* __restrict__ tinfo,
                                                   WarpPrep* __restrict__ prep)
{
    const int pair = blockIdx.y, tid = threadIdx.x;
#if MDX_WARP_STAMP
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) g_warp_launch = g_warp_launch + 1;
#endif
    const PairFit& f = fits[pair];
    if (f.fit_status != 0) return;
    double M[9];
#pragma unroll
    for (int k = 0; k < 9; k++) M[k] = f.Hinv[k];
    if (blockIdx.x == 0) {
        __shared__ uint32_t s_bm[2][(1 << kBmBits) / 32];
        for (int i = tid; i < (1 << kBmBits) / 16; i += 256) (&s_bm[0][0])[i] = 0;
        __syncthreads();
        const double Wd = M[8] != 0.0 ? 32.0 / M[8] : 0.0;
        if (tid < 2 * kBW) {
            const int ax = tid >> 6, x1 = tid & 63;
            const double t1 = (ax ? M[3] : M[0]) * (double)x1;
            const uint32_t B = floor_lo(t1 * (Wd * 524288.0));
            prep[pair].B[ax][x1] = B;
            const uint32_t lo = (0u - B - 3u) & 0x7ffffu, hi = (0u - B + 1u) & 0x7ffffu;
            const uint32_t b0 = lo >> (19 - kBmBits), b1 = hi >> (19 - kBmBits);
            atomicOr(&s_bm[ax][b0 >> 5], 1u << (b0 & 31));
            atomicOr(&s_bm[ax][b1 >> 5], 1u << (b1 & 31));
        }
        __syncthreads();
        for (int i = tid; i < (1 << kBmBits) / 16; i += 256) (&prep[pair].bm[0][0])[i] = (&s_bm[0][0])[i];
        return;
    }
    const int tile = (blockIdx.x - 1) * 32 + (tid >> 3);
    if (tile >= nbx * nby) return;   // whole groups of 8 leave together
    const int tx = tile % nbx, ty = tile / nbx;
    const TileInfo t = tile_info(M, tx * kTW, row0 + ty * kTH, w, row1, tid & 7);
    if ((tid & 7) == 0) tinfo[(long long)pair * (nbx * nby) + tile] = t;
}

// grid: x -> tile column, y -> tile row of the band [row0, row1), z -> pair.  256 threads; lane l
// of wave q owns columns x0 + 4*(l & 31) .. +3 of tile rows 2q + (l >> 5) + 8i, i = 0..7.  The
// reference's blocking depends on the full height only through bw0, and each pixel's arithmetic
// on (x, y) only, so a band is exactly the full frame's rows.  The tile's footprint bounds and
// the pair's fixed-point tables come from k_warp_prep, so the setup has one barrier: footprint
// DMA, gray2 loads and the per-row-block table in flight together, then the row loop.
WARP_DIFF_FN(const uint8_t* __restrict__ g1, long long g1_stride, int g1_pitch,
                                                   const uint8_t* __restrict__ g2, long long g2_stride, int g2_pitch,
                                                   int w, int h, int bw0, const PairFit* __restrict__ fits,
                                                   uint8_t* __restrict__ mask, long long mask_stride, int thresh,
                                                   int vec_ok, int row0, int row1, const TileInfo* __restrict__ tinfo,
                                                   const WarpPrep* __restrict__ prep, uint32_t mt, uint32_t mx)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[64];             // weight table (FP64 rows)
    __shared__ __attribute__((aligned(16))) double s_xy[kTH][2][2];         // (X0, Y0) per row, block
    __shared__ __attribute__((aligned(16))) double s_w0[kTH][2][2];         // projective: (W0, W0 / 2^24) per row, block
    __shared__ __attribute__((aligned(16))) uint8_t s_src[kSH * kSP];
    __shared__ __attribute__((aligned(16))) uint4 s_fx[kTH][2];             // fixed point: (A_x, A_y, flag)

    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs; remap the linear id so
    // each XCD walks a contiguous run of tiles (row-major).  Horizontally adjacent tiles share the
    // 128-B lines at their footprints' margins: in one L2 they are fetched once (PMC: 529 MB read
    // per 4K x32 launch = 1.0x the algorithmic bytes; plain grid order, tiles of a row spread over
    // the XCDs: 803 MB).
    const int nbx = gridDim.x, nby = gridDim.y;
    int bid = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    {
        const int total = nbx * nby * gridDim.z, xcd = bid & 7, q8 = total >> 3, r8 = total & 7;
        bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    }
    // the divisions by uniform values with host magic numbers: scalar multiplies, no VALU
    const int pair = (int)udiv_magic((uint32_t)bid, (uint32_t)(nbx * nby), mt), tile = bid - pair * (nbx * nby);
    const int ty_ = (int)udiv_magic((uint32_t)tile, (uint32_t)nbx, mx), tx_ = tile - ty_ * nbx;
    // The tile's scalar operands (the pair's fit, the tile's TileInfo) in ONE round trip: left to
    // itself the compiler sinks each scalar load into the branch that first uses it, and the DMA
    // then waits behind five dependent scalar-load latencies (kernel arguments, fit status, more
    // arguments, M and TileInfo, TileInfo.wd).  The TileInfo of a pair with no fit is not written
    // by k_warp_prep; it is read (in bounds) and unused.
    const PairFit& f = fits[pair];
    const TileInfo t = tinfo[(long long)pair * (nbx * nby) + tile];   // uniform: scalar loads
    double M[9];
#pragma unroll
    for (int k = 0; k < 9; k++) M[k] = f.Hinv[k];
    const int fit_status = f.fit_status;
    asm volatile("" ::"s"(fit_status), "s"(t.wd), "s"(t.fast), "s"(t.sxa), "s"(t.sya), "s"(t.sw), "s"(t.sh),
                 "s"(M[0]), "s"(M[1]), "s"(M[2]), "s"(M[3]), "s"(M[4]), "s"(M[5]), "s"(M[6]), "s"(M[7]),
                 "s"(M[8]), "s"(g1), "s"(g2), "s"(mask), "s"(prep));
    // wave index in an SGPR: the staging loop's trip count and LDS addresses stay scalar
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int x0 = tx_ * kTW, y0 = row0 + ty_ * kTH;
    const int cq = lane & 31;
    const int xs = x0 + 4 * cq;                     // this lane's 4 columns
    const int r0 = 2 * wave + (lane >> 5);          // this lane's first tile row (then every 8th)
    const uint8_t* g2p = g2 + (long long)pair * g2_stride;
    uint8_t* mp = mask + (long long)pair * mask_stride - (long long)row0 * w;   // indexed by frame row

    if (fit_status != 0) {   // no fit: the reference produces no mask; ours is all zero
        const int nx = max(0, min(4, w - xs));
        for (int r = r0; r < kTH && y0 + r < row1; r += 8) {
            uint8_t* m = mp + (long long)(y0 + r) * w + xs;
            for (int k = 0; k < nx; k++) m[k] = 0;
        }
        return;
    }
    const uint8_t* src = g1 + (long long)pair * g1_stride;
    const bool affine = (M[6] == 0.0) && (M[7] == 0.0);
    // fast path only over dword-aligned rows with reference blocks of 64 (uniform per workgroup)
    const bool try_fast = bw0 == kBW && vec_ok;
    if (!try_fast || !t.fast) {
        // ---- general path: per pixel, global gathers
        const int nx = max(0, min(4, w - xs));
        for (int r = r0; r < kTH && y0 + r < row1; r += 8) {
            const int y = y0 + r;
            const uint8_t* g2r = g2p + (long long)y * g2_pitch + xs;
            uint8_t* m = mp + (long long)y * w + xs;
            for (int k = 0; k < nx; k++) m[k] = warp_px_general(M, src, g1_pitch, w, h, xs + k, y, bw0, g2r[k], thresh);
        }
        return;
    }

    // ---- fast path
    const double Wd = t.wd;
    // 32/M8 a power of two -> (X0 + M0*x1) * Wd is exact: the fixed-point rows (warp_rows_fx)
    const bool pow2 = affine && Wd != 0.0 && (__double_as_longlong(Wd) & 0x000fffffffffffffLL) == 0;
    if (affine && !pow2 && tid < 32) {
        s_tab[2 * tid] = (uint32_t)(32 - tid) | ((uint32_t)tid << 16);
        s_tab[2 * tid + 1] = (uint32_t)(64 * (32 - tid)) | ((uint32_t)(64 * tid) << 16);
    }
    const bool col_ok = xs < w;
    const uint32_t OOB = 0x80000000u;
    const __amdgpu_buffer_rsrc_t g2rs = buf_rsrc(g2p, (long long)h * g2_pitch);
    const uint32_t g2off = col_ok ? (uint32_t)((y0 + r0) * g2_pitch + xs) : OOB;
    // lanes past the right edge compute on a valid column of block 0 and store nothing
    const int cqe = col_ok ? cq : (cq & 15);
    const int blk = cqe >> 4, x1b = 4 * (cqe & 15);
    uint32_t G[kTH / 8];
    // LDS-DMA (buffer_load ... lds): one wave instruction fills 4 staged rows (lane L -> row
    // 4q + L/16, chunk L%16 at LDS byte 16L of the 1-KiB group), straight from memory to LDS.
    // Chunks past the footprint's width, and rows above / below the image, get an out-of-range
    // offset and land as zeros (BORDER_CONSTANT); chunks crossing the image's left / right edge
    // are rewritten byte by byte once the DMA has landed.
    const int nch = (t.sw + 15) >> 4;                 // <= kSP / 16
    const int ch = lane & 15, sx = t.sxa + 16 * ch;
    const bool inner = ch < nch && sx >= 0 && sx + 16 <= w;
    {
        const __amdgpu_buffer_rsrc_t srs = buf_rsrc(src, (long long)h * g1_pitch);
        // A group of 4 staged rows wholly inside the image and the footprint (all but the edge
        // tiles' first / last groups) needs no per-lane test: the lane's offset within the group is
        // loop-invariant and the group's row start is the scalar offset (0 VALU per DMA instead of 6)
        const uint32_t voff = inner ? (uint32_t)((lane >> 4) * g1_pitch + sx) : 0x80000000u;
        for (int q = wave; 4 * q < t.sh; q += 4) {
            const int y4 = t.sya + 4 * q;
            if (y4 >= 0 && y4 + 4 <= h && 4 * q + 4 <= t.sh) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(srs, (lds_ptr)&s_src[4 * q * kSP], 16, (int)voff,
                                                         y4 * g1_pitch, 0, 0);
            } else {
                const int r = 4 * q + (lane >> 4);
                const int sy = t.sya + r;
                const uint32_t off = (inner && r < t.sh && (unsigned)sy < (unsigned)h)
                                         ? (uint32_t)(sy * g1_pitch + sx) : 0x80000000u;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(srs, (lds_ptr)&s_src[4 * q * kSP], 16, (int)off, 0, 0, 0);
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    uint32_t bx[4] = {0, 0, 0, 0}, by[4] = {0, 0, 0, 0};
    if (pow2) {
        // gray2: this lane's dwords of its 8 rows; B(x1) of its four columns (the per-column half of U)
#pragma unroll
        for (int i = 0; i < kTH / 8; i++)
            G[i] = __builtin_amdgcn_raw_buffer_load_b32(g2rs, (int)g2off, i * 8 * g2_pitch, kCpStream);
        const v4u bxv = *reinterpret_cast<const v4u*>(&prep[pair].B[0][x1b]);
        const v4u byv = *reinterpret_cast<const v4u*>(&prep[pair].B[1][x1b]);
        bx[0] = bxv.x; bx[1] = bxv.y; bx[2] = bxv.z; bx[3] = bxv.w;
        by[0] = byv.x; by[1] = byv.y; by[2] = byv.z; by[3] = byv.w;
    }
    // per row and block: (X0, Y0) for the FP64 forms, and on the fixed-point path A and its flag
    // (the pair's bucket maps from k_warp_prep, read through L2)
    if (tid < 2 * kTH) {
        const int r = tid >> 1, b = tid & 1, y = y0 + r, xb = x0 + kBW * b;
        const double X0 = M[0] * xb + M[1] * y + M[2];
        const double Y0 = M[3] * xb + M[4] * y + M[5];
        s_xy[r][b][0] = X0;
        s_xy[r][b][1] = Y0;
        if (!affine) {
            const double W0 = M[6] * xb + M[7] * y + M[8];
            s_w0[r][b][0] = W0;
            s_w0[r][b][1] = W0 * 0x1p-24;
        }
        if (pow2) {
            const double fx_scale = 524288.0;                        // 2^19
            const uint32_t Ax = floor_lo((Wd * X0 + 0.5 - 32.0 * t.sxa) * fx_scale);
            const uint32_t Ay = floor_lo((Wd * Y0 + 0.5 - 32.0 * t.sya) * fx_scale);
            const uint32_t bx = (Ax & 0x7ffffu) >> (19 - kBmBits), by = (Ay & 0x7ffffu) >> (19 - kBmBits);
            const WarpPrep& P = prep[pair];
            const uint32_t flag = ((P.bm[0][bx >> 5] >> (bx & 31)) | (P.bm[1][by >> 5] >> (by & 31))) & 1u;
            s_fx[r][b] = make_uint4(Ax, Ay, flag, 0u);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0F70);               // vmcnt(0): this wave's DMA (and the rest) landed
    __builtin_amdgcn_sched_barrier(0);
    if (ch < nch && !inner)
        for (int q = wave; 4 * q < t.sh; q += 4) {
            const int r = 4 * q + (lane >> 4);
            if (r < t.sh) stage_edge_chunks(src, g1_pitch, w, h, t.sya, sx, r, t.sh, t.sh, &s_src[16 * ch]);
        }
    __syncthreads();

    const double magic = 6755399441055744.0;                 // 1.5 * 2^52: ulp 1
    const double mX = magic - 32.0 * t.sxa, mY = magic - 32.0 * t.sya;
    const int tc = min(max(thresh, -1), 255);                // t < 0: all moving; t >= 255: none
    const uint32_t bias = 0x80000000u - (uint32_t)(65536 * tc + 32800);
    lds_d2* xyp = (lds_d2*)(&s_xy[r0][blk][0]);
    lds_u8* tabp = (lds_u8*)(&s_tab[0]);
    const uint32_t src_base = (uint32_t)(uintptr_t)(lds_u8*)(&s_src[0]);
    // gray2 rows of this pair; mask rows [0, row1) of the frame (stores past the band drop)
    const __amdgpu_buffer_rsrc_t mrs = buf_rsrc(mp, (long long)row1 * w);
    const uint32_t moff = col_ok ? (uint32_t)((y0 + r0) * w + xs) : OOB;
    const int nvalid = (row1 - y0 - r0 + 7) >> 3;            // rows r0 + 8i inside the band: i < nvalid
    const bool rowchk = y0 + kTH > row1;
    if (pow2) {
        lds_u4* fxp = (lds_u4*)(&s_fx[r0][blk]);
        if (!rowchk)
            warp_rows_fx<false>(fxp, xyp, src_base, nvalid, G, mrs, moff, 8 * w, bx, by, M[0],
                                M[3], x1b, Wd, mX, mY, bias);
        else
            warp_rows_fx<true>(fxp, xyp, src_base, nvalid, G, mrs, moff, 8 * w, bx, by, M[0],
                               M[3], x1b, Wd, mX, mY, bias);
    } else if (affine) {
        double tx[4], ty[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            tx[k] = M[0] * (x1b + k);
            ty[k] = M[3] * (x1b + k);
            asm volatile("" : "+v"(tx[k]), "+v"(ty[k]));   // keep in registers (no per-row rematerialisation)
        }
        warp_rows<false, true>(xyp, tabp, src_base, nvalid, g2rs, g2off, 8 * g2_pitch, mrs, moff, 8 * w, tx, ty, Wd, mX,
                               mY, bias);
    } else {
        const double x1d = (double)x1b;
        double tx0 = M[0] * x1d, ty0 = M[3] * x1d, tws0 = (M[6] * x1d) * 0x1p-24;
        asm volatile("" : "+v"(tx0), "+v"(ty0), "+v"(tws0));   // held in registers across the rows
        const double mXs = magic + 262144.0 - 16777216.0 * t.sxa, mYs = magic + 262144.0 - 16777216.0 * t.sya;
        warp_rows_pj((lds_d2*)(&s_xy[r0][blk][0]), (lds_d2*)(&s_w0[r0][blk][0]), src_base, nvalid, g2rs, g2off,
                     8 * g2_pitch, mrs, moff, 8 * w, tx0, ty0, tws0, M, x1b, mX, mY, mXs, mYs, bias);
    }
}

#if MDX_WARP_STAMP
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_warp_diff(
    const uint8_t* __restrict__ g1, long long g1_stride, int g1_pitch, const uint8_t* __restrict__ g2,
    long long g2_stride, int g2_pitch, int w, int h, int bw0, const PairFit* __restrict__ fits,
    uint8_t* __restrict__ mask, long long mask_stride, int thresh, int vec_ok, int row0, int row1,
    const TileInfo* __restrict__ tinfo, const WarpPrep* __restrict__ prep, uint32_t mt, uint32_t mx)
{
    const unsigned total = gridDim.x * gridDim.y * gridDim.z;
    const unsigned bid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const unsigned step = (total + kStampSamples - 1) / kStampSamples;
    const bool stamp = threadIdx.x == 0 && bid % step == 0;
    unsigned long long* st = g_warp_stamps + ((size_t)(g_warp_launch % kStampLaunches) * kStampSamples + bid / step) * 4;
    if (stamp) {
        st[0] = __builtin_amdgcn_s_memtime();
        st[1] = __builtin_amdgcn_s_memrealtime();
    }
    warp_diff_tile(g1, g1_stride, g1_pitch, g2, g2_stride, g2_pitch, w, h, bw0, fits, mask, mask_stride, thresh,
                   vec_ok, row0, row1, tinfo, prep, mt, mx);
    if (stamp) {
        st[2] = __builtin_amdgcn_s_memtime();
        st[3] = __builtin_amdgcn_s_memrealtime();
    }
}
#endif

size_t warp_scratch_bytes(int batch, int w, int rows)
{
    const long long tiles = (long long)((w + kTW - 1) / kTW) * ((rows + kTH - 1) / kTH);
    return (size_t)batch * (sizeof(WarpPrep) + (size_t)tiles * sizeof(TileInfo)) + 256;
}

hipError_t launch_warp_diff(hipStream_t s, int batch, const uint8_t* g1, long long g1_stride, int g1_pitch,
                            const uint8_t* g2, long long g2_stride, int g2_pitch, int w, int h, const PairFit* fits,
                            uint8_t* mask, long long mask_stride, int thresh, void* scratch, size_t scratch_bytes,
                            int row0, int row1)
{
    if (row1 < 0) row1 = h;
    if (row0 < 0 || row1 > h || row0 >= row1) return hipErrorInvalidValue;
    if (!scratch || scratch_bytes < warp_scratch_bytes(batch, w, row1 - row0)) return hipErrorInvalidValue;
    const int bh0 = h < 16 ? h : 16;
    const int bw0 = (1024 / bh0) < w ? (1024 / bh0) : w;
    // dword loads of gray2 / stores of the mask need 4-B aligned rows
    const int vec_ok = ((uintptr_t)g2 % 4 == 0) && g2_stride % 4 == 0 && g2_pitch % 4 == 0 &&
                       ((uintptr_t)mask % 4 == 0) && mask_stride % 4 == 0 && w % 4 == 0;
    const dim3 grid((w + kTW - 1) / kTW, (row1 - row0 + kTH - 1) / kTH, batch);
    const int ntiles = (int)(grid.x * grid.y);
    WarpPrep* prep = reinterpret_cast<WarpPrep*>((reinterpret_cast<uintptr_t>(scratch) + 255) & ~(uintptr_t)255);
    TileInfo* tinfo = reinterpret_cast<TileInfo*>(prep + batch);
    hipLaunchKernelGGL(k_warp_prep, dim3(1 + (ntiles + 31) / 32, batch), dim3(256), 0, s, fits, w, row0, row1,
                       (int)grid.x, (int)grid.y, tinfo, prep);
    hipLaunchKernelGGL(k_warp_diff, grid, dim3(256), 0, s, g1, g1_stride, g1_pitch, g2, g2_stride, g2_pitch, w, h, bw0,
                       fits, mask, mask_stride, thresh, vec_ok, row0, row1, tinfo, prep, udiv_magic_of((uint32_t)ntiles),
                       udiv_magic_of(grid.x));
    return hipGetLastError();
}

// Test hook (mdx_debug_div32): div32 over n values.
__global__ void k_div32(const double* __restrict__ in, double* __restrict__ out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = div32(in[i]);
}

hipError_t launch_div32(hipStream_t s, const double* in, double* out, int n)
{
    hipLaunchKernelGGL(k_div32, dim3((n + 255) / 256), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

// Memory-ceiling probe (mdx_probe_stream3_dev): k_warp_diff's 3 B/px with no warp -- two frames
// read and one mask written linearly, 16 B per lane, non-temporal like the kernel's gray2 / mask.
__global__ __launch_bounds__(256) void k_stream3(const v4u* __restrict__ a, const v4u* __restrict__ b,
                                                  v4u* __restrict__ o, size_t n16, int t)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n16) return;
    const v4u x = __builtin_nontemporal_load(a + i), y = __builtin_nontemporal_load(b + i);
    v4u r;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        unsigned m = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int d = (int)((x[k] >> (8 * j)) & 255u) - (int)((y[k] >> (8 * j)) & 255u);
            m |= ((d > t || -d > t) ? 255u : 0u) << (8 * j);
        }
        r[k] = m;
    }
    __builtin_nontemporal_store(r, o + i);
}

hipError_t launch_stream3(hipStream_t s, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* o, int thresh)
{
    const size_t n16 = n / 16;
    hipLaunchKernelGGL(k_stream3, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s, (const v4u*)a,
                       (const v4u*)b, (v4u*)o, n16, thresh);
    return hipGetLastError();
}

}  // namespace mdx
