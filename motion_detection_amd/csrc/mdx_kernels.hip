// mdx_kernels.hip -- CDNA4 (gfx950) kernels of the flow + egomotion-warp + frame-diff path.
//
// Reference path: OpticalFlowCalculator::calculateOpticalFlow
// (common/src/optical_flow_calculator.cpp:30-130).  Every kernel reproduces the arithmetic
// of the OpenCV 2.4 routine the reference calls, bit for bit (integer stages exactly; float
// and double stages in the same evaluation order, compiled with -ffp-contract=off so no
// expression is fused into an FMA).  Stage map:
//   A1-A4   k_front          cvtColor(BGR2GRAY) + level-0 REFLECT_101 padding + pyrDown to level 1
//                            in one pass; in level mode pyrDown L -> L+1 for the coarser levels
//   A1      k_gray_pad       gray + level-0 padding alone (single-level pyramids)
//   A3      k_scharr         calcSharrDeriv + CONSTANT-0 padding (prev frame)
//   A5      k_lk             calcOpticalFlowPyrLK (LKTrackerInvoker, SSE2 summation order)
//   A6/A7   k_classify/k_fit Vec4d classification, first-4 getPerspectiveTransform, invert
//   A8-A10  k_warp_diff      warpPerspective + absdiff + threshold, fused (mdx_warp.hip)
#include "mdx_internal.h"

#include <float.h>
#include <limits.h>

#include <algorithm>

namespace mdx {

__device__ __forceinline__ int r101(int p, int len)
{
    // borderInterpolate(p, len, BORDER_REFLECT_101), any number of folds.
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// Front-end kernels (A1, A3, A4) work on aligned 16-byte chunks of each padded row (4 words
// for the derivative rows): a level's padded columns -40 .. w+39 sit at row bytes 24 .. 64+w+39
// and every row has >= 16 B of slack after them, so a chunk may spill into the unused margin.
// Interior chunks take vector loads; chunks that touch a border fall back to per-pixel
// reflect-101 addressing.  One aligned dwordx4 store per thread.
struct __attribute__((aligned(4))) u4a4k { uint32_t x, y, z, w; };
struct __attribute__((aligned(4))) u3a4k { uint32_t x, y, z; };
struct __attribute__((aligned(4))) u2a4k { uint32_t x, y; };
// a load from a global address held as an integer: through an address-space-1 pointer, so that it is
// a global_load (vmcnt only).  Through a generic pointer it is a flat_load, which also counts in
// lgkmcnt: every LDS wait would then wait for it, and a load issued ahead of use would be waited
// for at the next LDS access.
template <typename T>
__device__ __forceinline__ T gload(uintptr_t a)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return *reinterpret_cast<const __attribute__((address_space(1))) T*>(a);
#else
    return *reinterpret_cast<const T*>(a);   // the host pass only type-checks device code
#endif
}

__device__ __forceinline__ int gray_of(const uint8_t* s, int fmt)
{
    // color.cpp RGB2Gray<uchar>, blueIdx 0 on rgb8 data: R gets the blue weight
    if (fmt == 1) return (s[0] * 1868 + s[1] * 9617 + s[2] * 4899 + 8192) >> 14;
    return (s[2] * 1868 + s[1] * 9617 + s[0] * 4899 + 8192) >> 14;   // bgr8 -> converted to rgb8 first
}

// ------------------------------------------------------------------ A1: gray + pad
// color.cpp RGB2Gray<uchar> with blueIdx 0 on rgb8 data (node.cpp:271 then :50):
// gray = (R*1868 + G*9617 + B*4899 + 8192) >> 14.  mono8 passes through unchanged.
// grid: x -> pairs of adjacent 16-B chunks of the padded row, y -> padded row, z = 2*pair + which
// frame.  Both of a thread's loads are in flight before its first store: 0.146 ms per step
// against 0.158 with one chunk per thread (4 adjacent chunks: 0.247; chunks interleaved across
// lanes so each load instruction is 1 KiB contiguous: 0.164-0.171).
__device__ __forceinline__ void gray_chunk(const uint8_t* s, int px0, int w, int fmt, uint32_t (&o)[4])
{
    if (px0 >= 0 && px0 + 16 <= w && fmt == 0 && (((uintptr_t)(s + px0)) & 3) == 0) {
        const u4a4k v = *reinterpret_cast<const u4a4k*>(s + px0);
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    } else if (px0 >= 0 && px0 + 16 <= w && fmt != 0 && (((uintptr_t)(s + 3 * px0)) & 3) == 0) {
        uint32_t b[12];
        const u4a4k* q = reinterpret_cast<const u4a4k*>(s + 3 * px0);
#pragma unroll
        for (int t = 0; t < 3; t++) { const u4a4k v = q[t]; b[4 * t] = v.x; b[4 * t + 1] = v.y; b[4 * t + 2] = v.z; b[4 * t + 3] = v.w; }
        const uint8_t* bb = reinterpret_cast<const uint8_t*>(b);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            uint32_t d = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) d |= (uint32_t)gray_of(bb + 3 * (4 * t + i), fmt) << (8 * i);
            o[t] = d;
        }
    } else {
        for (int t = 0; t < 4; t++) {
            uint32_t d = 0;
            for (int i = 0; i < 4; i++) {
                const int px = px0 + 4 * t + i;
                if (px < -kPad || px >= w + kPad) continue;           // row margin: value unused
                const int sx = r101(px, w);
                d |= (uint32_t)(fmt == 0 ? s[sx] : gray_of(s + 3 * sx, fmt)) << (8 * i);
            }
            o[t] = d;
        }
    }
}

__global__ __launch_bounds__(256) void k_gray_pad(const uint8_t* __restrict__ in1, const uint8_t* __restrict__ in2,
                                                  int w, int h, int stride, long long frame_stride, int fmt,
                                                  uint8_t* __restrict__ pyr1, uint8_t* __restrict__ pyr2,
                                                  long long img_bytes, Level L, int nchunk, int fsel)
{
    const int which = fsel ? fsel - 1 : blockIdx.z & 1, pair = fsel ? blockIdx.z : blockIdx.z >> 1;
    const int c = 2 * (blockIdx.x * blockDim.x + threadIdx.x) + 1;   // chunk 0 is all margin
    const int py = blockIdx.y - kPad;
    if (c > nchunk) return;
    const uint8_t* src = (which ? in2 : in1) + (long long)pair * frame_stride;
    const uint8_t* s = src + (long long)r101(py, h) * stride;
    uint32_t o0[4], o1[4];
    gray_chunk(s, 16 * c - kXOff, w, fmt, o0);
    const bool two = c + 1 <= nchunk;
    if (two) gray_chunk(s, 16 * (c + 1) - kXOff, w, fmt, o1);
    uint8_t* row = (which ? pyr2 : pyr1) + (long long)pair * img_bytes + L.img_off + (long long)(py + kPad) * L.pitch;
    *reinterpret_cast<uint4*>(row + 16 * c) = make_uint4(o0[0], o0[1], o0[2], o0[3]);
    if (two) *reinterpret_cast<uint4*>(row + 16 * (c + 1)) = make_uint4(o1[0], o1[1], o1[2], o1[3]);
}

// ------------------------------------------------------------------ A1 + A3/A4: k_front
// buildOpticalFlowPyramid's images (lkpyramid.cpp, called at optical_flow_calculator.cpp:71):
// pyramids.cpp pyrDown_<FixPtCast<uchar,8>>: dst(x,y) = (sum_ij k_i k_j src(r101(2y+i-2),
// r101(2x+j-2)) + 128) >> 8, k = [1 4 6 4 1], on the source ROI's own size; every level carries a
// 40-px REFLECT_101 border of its own core (copyMakeBorder ... BORDER_REFLECT_101|BORDER_ISOLATED).
//
// Frame mode (MODE 0/1): gray + level-0 padding + level 1 in one pass.  A workgroup owns RB level-1
// core rows [Y0, Y0+RB) and the level-0 core rows [2 Y0, 2 Y0 + 2 RB):
//   1  stage level-0 padded rows 2 Y0 - 2 .. 2 Y0 + 2 RB (reflect-101 in both directions, gray of
//      rgb8 on the fly) in LDS: interior 16-B chunks by LDS-DMA (mono8; rgb8/bgr8 by vector loads,
//      K per thread in flight, and the gray conversion), the border bytes one per lane;
//   2  write the band's level-0 rows, and every border row that mirrors one of them, from LDS;
//   3a level-1 core rows into an LDS row buffer: a thread owns 4 level-1 columns and walks down
//      the band, each staged row's horizontal 5-tap sums (two chained v_dot4_u32_u8 per pixel)
//      computed once and reused by the up to three level-1 rows whose vertical window covers it;
//   3a' the row buffer's reflect-101 column borders, one byte per lane;
//   3b level-1 padded rows (and mirrored border rows) out, 16 B per lane.
// Level 0 thus crosses HBM once (written) instead of three times (written, read back by a
// separate pyrDown); source halo rows are shared with the neighbouring band through L2
// (consecutive bands go to the same XCD).  Level mode (MODE 2) runs the same band schedule from
// an already padded level to the next (phase 1 = LDS-DMA copies of the padded source rows, no
// phase 2).  Measured at 1080p x 32, one frame side (scripts/micro/front_bench.hip): levels 0-1
// 40 us (4.0 TB/s of 162 MB) and levels 2-4 20 us, against 107 + 42 us for the earlier
// k_gray_pad + per-level pyrDown kernels (44 + 30 us with vector loads instead of LDS-DMA).  Per-pixel reflect-101 gathers in the hot loops cost
// ~2-5 us per workgroup (measured): borders are built byte-per-lane from data already in LDS.
struct FrontArgs {
    const uint8_t* in1;
    const uint8_t* in2;
    int w, h, stride, fmt, fsel, nbands, nz;
    int band0;       // first band of the launch (row-band mode builds only the bands a band's LK reads)
    long long frame_stride, img_bytes;
    uint8_t* pyr1;
    uint8_t* pyr2;
    Level L0, L1;
    int nchunk0;     // last 16-B chunk of a level-0 row (chunk 0 is margin)
    int nchunk1_16;  // last 16-B chunk of a level-1 row (chunk 0 is margin)
    int aligned;     // every source row starts 4-B aligned (interior chunks take vector loads)
    int lp;          // LDS bytes per staged level-0 row (16 * (nchunk0 + 1))
    int lp1;         // LDS bytes per level-1 row of the row buffer (16 * (nchunk1_16 + 1))
};

// borderInterpolate(p, len, BORDER_REFLECT_101) for -len < p < 2 len - 1 (one fold), branch-free.
// k_front only runs when level 1 exists, i.e. w, h >= 81 and the level-1 sizes are >= 41, so
// every index it folds (at most 40 outside a row or column range) needs at most one fold.
__device__ __forceinline__ int r101s(int p, int len)
{
    const int q = p < 0 ? -p : p;
    return q >= len ? 2 * len - 2 - q : q;
}

__device__ __forceinline__ int fdiv(int a, int b, float rb)
{
    // a / b for 0 <= a < 2^20 (b > 0): float estimate, corrected
    int q = (int)((float)a * rb);
    if (q * b > a) q--;
    else if ((q + 1) * b <= a) q++;
    return q;
}

typedef __attribute__((address_space(3))) void* front_lds_ptr;

// MODE 0: mono8 frames, 1: rgb8/bgr8 frames (gray + pad + level 1, as above); MODE 2: one
// pyramid level L -> L+1 (a.L0 = source level, already padded in the slab, a.L1 = destination):
// the staged rows are plain 16-B copies of the padded source rows and phase 2 is skipped.
template <int RB, int MODE, int KM = 8>
__global__ __launch_bounds__(256) void k_front(FrontArgs a)
{
    constexpr bool COLOR = MODE == 1, FRAME = MODE != 2;
    constexpr int NR = 2 * RB + 3, K = COLOR ? 2 : KM, VW = COLOR ? 12 : 4, MAXOUT0 = 2 * RB + 80, MAXOUT1 = RB + 80;
    extern __shared__ uint32_t front_lds[];
    __shared__ int out0[MAXOUT0], out1[MAXOUT1], nout[2];
    uint8_t* lds = reinterpret_cast<uint8_t*>(front_lds);
    const int tid = threadIdx.x;

    // XCD-aware order: consecutive bands of a frame go to the same XCD (8 dispatch round-robin)
    const int nb = gridDim.x;
    int task = blockIdx.x;
    if ((nb & 7) == 0) task = (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
    const int band = a.band0 + task % a.nbands, z = task / a.nbands;
    const int which = a.fsel ? a.fsel - 1 : z & 1, pair = a.fsel ? z : z >> 1;
    const int w = a.w, h = a.h, w1 = a.L1.w, h1 = a.L1.h;
    const int Y0 = band * RB, e1 = min(Y0 + RB, h1), r0 = 2 * Y0, e0 = min(2 * Y0 + 2 * RB, h);
    const int fmt = a.fmt;
    const uint8_t* src = (which ? a.in2 : a.in1) + (long long)pair * a.frame_stride;
    uint8_t* slab = (which ? a.pyr2 : a.pyr1) + (long long)pair * a.img_bytes;

    // rows this band writes: level 0 padded rows whose core row is in [r0, e0), level 1 in [Y0, e1)
    if (tid < 2) nout[tid] = 0;
    __syncthreads();
    if (FRAME && tid < 80) {
        const int py = tid < 40 ? tid - 40 : h + tid - 40;
        const int r = r101s(py, h);
        if (r >= r0 && r < e0) out0[atomicAdd(&nout[0], 1)] = py;
    } else if (tid >= 128 && tid < 208) {
        const int t = tid - 128;
        const int py = t < 40 ? t - 40 : h1 + t - 40;
        const int r = r101s(py, h1);
        if (r >= Y0 && r < e1) out1[atomicAdd(&nout[1], 1)] = py;
    }
    __syncthreads();
    const int nb0 = nout[0], nb1 = nout[1];
    __syncthreads();
    if (FRAME && tid < e0 - r0) out0[nb0 + tid] = r0 + tid;
    if (tid >= 128 && tid - 128 < e1 - Y0) out1[nb1 + tid - 128] = Y0 + tid - 128;

    // phase 1: level-0 padded rows r0-2 .. r0+2RB into LDS (chunks 1 .. nchunk0).  Interior chunks
    // [cA, cB] (inside the source row, every row 4-B aligned per the host) take plain 16-B (mono8)
    // or 48-B (rgb8/bgr8) loads, K per thread in flight; the few border chunks go through the
    // per-pixel reflect-101 path in a loop of their own.
    const int nc0 = a.nchunk0;
    const int cA = kXOff / 16;
    int cB = a.aligned ? (w + kXOff - 16) / 16 : cA - 1;
    if (cB < cA) cB = cA - 1;
    const int ni = cB - cA + 1;
    if constexpr (MODE != 1) {
        // mono8 frames and level mode: LDS-DMA (buffer_load ... lds) straight into the staged rows.
        // Flat 16-B slot f is row f / (nc0 + 1), chunk f % (nc0 + 1) (LDS byte 16 f); one wave
        // instruction fills 64 consecutive slots.  Frame mode loads the interior chunks [cA, cB]
        // and leaves the rest to the border-byte pass below (an out-of-range offset lands zeros
        // there first); level mode copies whole padded rows.
        const int spr = nc0 + 1, nslot = NR * spr;
        const float rs = 1.f / (float)spr;
        const uint8_t* rbase = FRAME ? src : slab + a.L0.img_off;
        const long long rbytes = FRAME ? (long long)h * a.stride : (long long)a.L0.rows * a.L0.pitch;
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(rbase), (short)0, (int)min(rbytes, (long long)0x7fffffff), 0x00020000);
        const int wave = tid >> 6, wl = tid & 63;
        for (int b0 = 64 * wave; b0 < nslot; b0 += 256) {
            const int f = b0 + wl;
            if (f < nslot) {
                const int i = fdiv(f, spr, rs), c = f - i * spr;
                uint32_t off = 0x80000000u;
                if constexpr (FRAME) {
                    if (c >= cA && c <= cB) off = (uint32_t)(r101s(r0 - 2 + i, h) * a.stride + 16 * c - kXOff);
                } else {
                    off = (uint32_t)((r0 - 2 + i + kPad) * a.L0.pitch + 16 * c);
                }
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (front_lds_ptr)(lds + 16 * b0), 16, (int)off, 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0x0F70);               // vmcnt(0): this wave's DMA has landed
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (FRAME) __syncthreads();             // before any wave rewrites border slots
    }
    if (MODE == 1 && ni > 0) {
        const float rci = 1.f / (float)ni;
        const int n1 = NR * ni;
        for (int base = 0; base < n1; base += 256 * K) {
            uint32_t v[K][VW];
#pragma unroll
            for (int k = 0; k < K; k++) {
                const int item = base + k * 256 + tid;
                if (item < n1) {
                    const int i = fdiv(item, ni, rci), c = cA + item - i * ni;
                    const uint8_t* s = src + (long long)r101s(r0 - 2 + i, h) * a.stride + (16 * c - kXOff) * (COLOR ? 3 : 1);
                    const u4a4k* q = reinterpret_cast<const u4a4k*>(s);
                    const u4a4k t0 = q[0];
                    v[k][0] = t0.x; v[k][1] = t0.y; v[k][2] = t0.z; v[k][3] = t0.w;
                    if constexpr (COLOR) {
                        const u4a4k t1 = q[1], t2 = q[2];
                        v[k][4] = t1.x; v[k][5] = t1.y; v[k][6] = t1.z; v[k][7] = t1.w;
                        v[k][8] = t2.x; v[k][9] = t2.y; v[k][10] = t2.z; v[k][11] = t2.w;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < K; k++) {
                const int item = base + k * 256 + tid;
                if (item >= n1) continue;
                const int i = fdiv(item, ni, rci), c = cA + item - i * ni;
                uint32_t o[4] = {v[k][0], v[k][1], v[k][2], v[k][3]};
                if constexpr (COLOR) {
                    const uint8_t* bb = reinterpret_cast<const uint8_t*>(v[k]);
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        uint32_t d = 0;
#pragma unroll
                        for (int j = 0; j < 4; j++) d |= (uint32_t)gray_of(bb + 3 * (4 * t + j), fmt) << (8 * j);
                        o[t] = d;
                    }
                }
                *reinterpret_cast<uint4*>(lds + i * a.lp + 16 * c) = make_uint4(o[0], o[1], o[2], o[3]);
            }
        }
    }
    if constexpr (FRAME) {
        // border bytes one per lane: columns -48 .. 16 cA - 65 and 16 (cB + 1) - 64 .. 16 nc0 - 49
        const int nl = 16 * (cA - 1), nb = nl + 16 * (nc0 - cB);
        const float rcb = 1.f / (float)nb;
#pragma unroll 4
        for (int item = tid; item < NR * nb; item += 256) {
            const int i = fdiv(item, nb, rcb), e = item - i * nb;
            const int x = e < nl ? e - 48 : 16 * (cB + 1) - kXOff + (e - nl);
            const bool in = x >= -kPad && x < w + kPad;                     // row margin: left 0
            const uint8_t* sp = src + (long long)r101s(r0 - 2 + i, h) * a.stride;
            const int sx = in ? r101s(x, w) : 0;
            uint32_t v;
            if constexpr (COLOR) v = (uint32_t)gray_of(sp + 3 * sx, fmt);
            else v = sp[sx];
            lds[i * a.lp + kXOff + x] = (uint8_t)(in ? v : 0u);
        }
    }
    __syncthreads();

    // phase 2: level-0 rows out of LDS (core row r sits at LDS row r - r0 + 2)
    if constexpr (FRAME) {
        const int n0 = nb0 + (e0 - r0), n2 = n0 * nc0;
        const float rc0 = 1.f / (float)nc0;
        uint8_t* base0 = slab + a.L0.img_off;
        for (int item = tid; item < n2; item += 256) {
            const int j = fdiv(item, nc0, rc0), c = 1 + item - j * nc0;
            const int py = out0[j];
            const int i = r101s(py, h) - r0 + 2;
            *reinterpret_cast<uint4*>(base0 + (long long)(py + kPad) * a.L0.pitch + 16 * c) =
                *reinterpret_cast<const uint4*>(lds + i * a.lp + 16 * c);
        }
    }

    // phase 3a: the band's level-1 core rows into an LDS row buffer.  A thread owns one dword
    // chunk (4 level-1 pixels) of every row and walks down the band: each staged level-0 row's
    // horizontal 5-tap sums (two chained v_dot4_u32_u8 per pixel) are computed once and kept in
    // registers for the up to three level-1 rows whose vertical window covers it.
    uint8_t* l1buf = lds + NR * a.lp;
    {
        const int nq = (w1 + 3) >> 2;
        for (int q = tid; q < nq; q += 256) {
            const int px0 = 4 * q;
            const uint8_t* col = lds + kXOff + 2 * px0 - 4;      // level-0 columns 2 px0 - 4 .. 2 px0 + 11
            uint32_t hr[5][4];
            auto hsum = [&](int r, uint32_t (&o)[4]) {
                const uint32_t* p = reinterpret_cast<const uint32_t*>(col + r * a.lp);
                const uint32_t wd[4] = {p[0], p[1], p[2], p[3]};
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    const int b0 = 2 * jj + 2, qq = b0 >> 2;
                    const uint32_t lo = (b0 & 3) ? __builtin_amdgcn_alignbit(wd[qq + 1], wd[qq], 16) : wd[qq];
                    const uint32_t hi = (b0 & 3) ? (wd[qq + 1] >> 16) : wd[qq + 1];
                    o[jj] = __builtin_amdgcn_udot4(hi, 1u, __builtin_amdgcn_udot4(lo, 0x04060401u, 0u, false), false);
                }
            };
            hsum(0, hr[0]);
            hsum(1, hr[1]);
            hsum(2, hr[2]);
#pragma unroll
            for (int yy = 0; yy < RB; yy++) {
                if (Y0 + yy >= e1) break;
                hsum(2 * yy + 3, hr[3]);
                hsum(2 * yy + 4, hr[4]);
                uint32_t o = 0;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    const uint32_t acc = hr[0][jj] + hr[1][jj] * 4u + hr[2][jj] * 6u + hr[3][jj] * 4u + hr[4][jj];
                    o |= ((acc + 128) >> 8) << (8 * jj);
                }
                *reinterpret_cast<uint32_t*>(l1buf + yy * a.lp1 + kXOff + px0) = o;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    hr[0][jj] = hr[2][jj];
                    hr[1][jj] = hr[3][jj];
                    hr[2][jj] = hr[4][jj];
                }
            }
        }
    }
    __syncthreads();
    // phase 3a': the row buffer's reflect-101 borders (and zeroed margins), one byte per lane
    {
        const int nl = 48, nb = nl + 16 * (a.nchunk1_16 + 1) - kXOff - w1;   // columns -48..-1, w1..
        const float rcb = 1.f / (float)nb;
        const int nrow = e1 - Y0;
        for (int item = tid; item < nrow * nb; item += 256) {
            const int i = fdiv(item, nb, rcb), e = item - i * nb;
            const int x = e < nl ? e - 48 : w1 + (e - nl);
            const bool in = x >= -kPad && x < w1 + kPad;
            uint8_t* row = l1buf + i * a.lp1 + kXOff;
            const uint8_t v = row[in ? r101s(x, w1) : 0];
            row[x] = in ? v : (uint8_t)0;
        }
    }
    __syncthreads();

    // phase 3b: level-1 padded rows out of the row buffer, 16 B per lane (borders by reflect-101
    // in LDS; bytes 16..23 of a row are margin, written with zeros)
    {
        const int nc16 = a.nchunk1_16;                                // 16-B chunks 1 .. nc16
        const float rc16 = 1.f / (float)nc16;
        const int n3 = (nb1 + (e1 - Y0)) * nc16;
        uint8_t* base1 = slab + a.L1.img_off;
        for (int item = tid; item < n3; item += 256) {
            const int j = fdiv(item, nc16, rc16), c = 1 + item - j * nc16;
            const int py = out1[j];
            const uint8_t* row = l1buf + (r101s(py, h1) - Y0) * a.lp1 + kXOff;
            const int px0 = 16 * c - kXOff;
            const uint4 o = *reinterpret_cast<const uint4*>(row + px0);
            *reinterpret_cast<uint4*>(base1 + (long long)(py + kPad) * a.L1.pitch + 16 * c) = o;
        }
    }
}

// ------------------------------------------------------------------ A3: Scharr derivs
// lkpyramid.cpp calcSharrDeriv.  Vertical t0 = 3(a+c)+10b, t1 = c-a; horizontal
// Ix = t0[x+1]-t0[x-1], Iy = 3(t1[x-1]+t1[x+1])+10 t1[x].  OpenCV clamps the row/col
// neighbours as reflect-101 (row -1 -> 1, col cols -> cols-2), which is exactly the padded
// level's border, so the stencil reads the padded image directly.  Border = 0
// (copyMakeBorder ... BORDER_CONSTANT).  Per thread 4 pixels (one 16-B store); each of the
// three source rows is one dwordx3 load of bytes x0-4 .. x0+7.
__global__ __launch_bounds__(256) void k_scharr(const uint8_t* __restrict__ pyr1, uint32_t* __restrict__ der,
                                                long long img_bytes, long long der_words, Level L, int nchunk,
                                                int prow0)
{
    const int pair = blockIdx.z;
    const int c = blockIdx.x * blockDim.x + threadIdx.x + 4;         // word chunks 0..3 are margin
    const int py = prow0 + blockIdx.y - kPad;                        // padded rows prow0 + blockIdx.y
    if (c > nchunk) return;
    const int px0 = 4 * c - kXOff;
    uint32_t o[4] = {0, 0, 0, 0};
    if (py >= 0 && py < L.h && px0 + 4 > 0 && px0 < L.w) {
        const uint8_t* s = pyr1 + (long long)pair * img_bytes + L.img_off + L.core() + (long long)py * L.pitch + px0 - 4;
        const int p = L.pitch;
        uint32_t rw[3][3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const u3a4k v = *reinterpret_cast<const u3a4k*>(s + (long long)(r - 1) * p);
            rw[r][0] = v.x; rw[r][1] = v.y; rw[r][2] = v.z;
        }
        auto B = [&](int r, int b) -> int { return (int)((rw[r][b >> 2] >> (8 * (b & 3))) & 255u); };
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int px = px0 + i;
            if (px < 0 || px >= L.w) continue;
            const int bm = 3 + i, bc = 4 + i, bp = 5 + i;               // bytes x-1, x, x+1
            const int t0m = (B(0, bm) + B(2, bm)) * 3 + B(1, bm) * 10;
            const int t0p = (B(0, bp) + B(2, bp)) * 3 + B(1, bp) * 10;
            const int t1m = B(2, bm) - B(0, bm), t1c = B(2, bc) - B(0, bc), t1p = B(2, bp) - B(0, bp);
            const int ix = t0p - t0m;
            const int iy = (t1m + t1p) * 3 + t1c * 10;
            o[i] = (uint32_t)(uint16_t)(int16_t)ix | ((uint32_t)(uint16_t)(int16_t)iy << 16);
        }
    }
    uint32_t* row = der + (long long)pair * der_words + L.der_off + (long long)(py + kPad) * L.pitch;
    *reinterpret_cast<uint4*>(row + 4 * c) = make_uint4(o[0], o[1], o[2], o[3]);
}

// ------------------------------------------------------------------ A5: LK tracker
//
// One 64-lane wave = one workgroup tracks PPW = 64/LPP grid points through every pyramid
// level (LPP lanes per point).  Per level and point the 40x40 window is cut into 5 chunks of
// R = 8 rows; each lane owns EC = 320/LPP window elements per chunk and keeps its
// interpolated I*32, Ix, Iy for the whole level in registers (NE = 5*EC elements).
//
// Exact summation order.  OpenCV's SSE2 path accumulates every sum in four float lanes:
// lane k takes window columns x = 4g+k in (row, g) order; A = ((P0+P1)+P2)+P3 and
// b = (P0+P2)+(P1+P3).  A GPU reduction tree would round differently, so the kernel keeps
// the reference's order: the lanes compute the per-element products (exact integer
// products rounded once to float) in parallel and store them chain-ordered in LDS; then one
// lane per chain (12 chains for A11/A12/A22, 8 for b1/b2) adds its 80 terms of the chunk in
// order.  The result is bit-identical to the x86 reference, not merely within tolerance.
typedef short s2k __attribute__((ext_vector_type(2)));
// v_dot2_i32_i16 (VOP3P) with its accumulator in an SGPR.  The builtin with a constant accumulator
// compiles to v_mov + v_dot2c_i32_i16 (the constant rematerialised in a VGPR per dot product): one
// more VALU per chain (the trajectory LK's rounding biases 256 and 8192).
__device__ __forceinline__ int sdot2_sacc(s2k a, s2k b, int c)
{
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

// k_lk<LPP, true>: the chained trajectory passes (TrajChain); grid = nimg-1 passes x npts points,
// pass-major, one point per wave.
constexpr int kChainSpinMax = 1 << 19;   // ~0.1 s of s_sleep(8) polls: a lost hand-off gives wrong
                                         // results, never a hung launch

// four points per wave: each lane's 20 elements of a chunk as a block of 4 rows x 5 columns (1,
// round 6) or as 20 columns of one row (0).  The block shares tap rows between its rows: 5 row
// loads and 75 pair-building v_perm per chunk (I taps, Ix and Iy pairs) instead of 2 x 2 loads and
// 120, and its J rows for the next chunk are loaded while the current one is summed (ring callback
// 2.37 against 2.49 ms, profiles/r06_ab_traj_blk.txt)
#ifndef MDX_TRAJ_BLK
#define MDX_TRAJ_BLK 1
#endif
// two points per wave: 144 VGPRs, 3 waves per SIMD (MDX_LK32_WPE=4 squeezes 128 with spills)
#ifndef MDX_LK32_WPE
#define MDX_LK32_WPE 1
#endif
template <int LPP, bool CHAIN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LPP == 32 ? MDX_LK32_WPE : 1, 8))) void k_lk(LkArgs a, TrajChain t)
{
    constexpr int WIN = 40, R = 8, NCH = WIN / R, EC = R * WIN / LPP, NE = NCH * EC, PPW = 64 / LPP;
    constexpr int STRIDE = 88;                 // floats per chain (80 used; 4*odd => b128 conflict-free)
    constexpr int PT_FLOATS = 12 * STRIDE + 16;
    constexpr float HALFW = 19.5f;             // (winSize.width-1)*0.5f
    constexpr float FLT_SCALE = 1.f / (1 << 20);
    __shared__ float4 lds4[PPW * PT_FLOATS / 4];

    static_assert(!CHAIN || LPP == 64 || LPP == 32 || LPP == 16, "chain mode: one, two or four points per wave");
    // row runs: lane s owns RUN adjacent window columns of one row per chunk
    constexpr int RUN = LPP == 64 ? 5 : LPP == 32 ? 10 : LPP == 16 ? 20 : 0;
    constexpr int RW = (RUN + 1 + 3) / 4;      // words of a realigned run (taps x .. x + RUN)
    const int lane = threadIdx.x;
    const int p = lane / LPP, s = lane % LPP;
    // chain mode: block b = pass * nbp + points (dispatch order: every block a wave waits for was
    // dispatched before it, and pass 0 never waits, so the waits always drain)
    const unsigned nbp = (unsigned)((a.npts + PPW - 1) / PPW);       // blocks per pass
    const int pass = CHAIN ? (int)(blockIdx.x / nbp) : 0;
    const int pt = CHAIN ? (int)(blockIdx.x - (unsigned)pass * nbp) * PPW + p : (int)blockIdx.x * PPW + p;
    const int pair = CHAIN ? 0 : blockIdx.y;
    const bool valid = pt < a.npts;
    float* ch = reinterpret_cast<float*>(lds4) + p * PT_FLOATS;
    float* res = ch + 12 * STRIDE;

    // element geometry (level independent).  LPP 64: lane s owns a run of 5 adjacent window
    // columns of one row per 8-row chunk (row s >> 3, columns 5 (s & 7) .. +4), so its taps of a
    // chunk are two 12-B row loads (J: v_perm + v_dot2 tap pairs) instead of 4 byte loads per element
    static_assert(RUN == 0 || EC == RUN, "row runs of RUN columns");
    constexpr bool BLK = MDX_TRAJ_BLK && LPP == 16;   // lane s: rows 4 (s / 8) .. +3, columns 5 (s % 8) .. +4
    int woff[EC], ex[EC], ey[EC];
#pragma unroll
    for (int i = 0; i < EC; i++) {
        const int e = BLK ? (4 * (s / 8) + i / 5) * WIN + 5 * (s % 8) + i % 5
                    : RUN ? (s / (WIN / RUN)) * WIN + RUN * (s % (WIN / RUN)) + i : s + LPP * i;
        ey[i] = e / WIN;
        ex[i] = e % WIN;
        woff[i] = (ex[i] & 3) * STRIDE + ey[i] * 10 + (ex[i] >> 2);
    }
    // 12 bytes of a row from byte address p, realigned: (lo, hi) = bytes p .. p+7
    auto row8 = [](const uint8_t* p, uint32_t& lo, uint32_t& hi) {
        const uintptr_t u = reinterpret_cast<uintptr_t>(p);
        const u3a4k v = gload<u3a4k>(u & ~(uintptr_t)3);
        const uint32_t o = (uint32_t)(u & 3);
        lo = __builtin_amdgcn_alignbyte(v.y, v.x, o);
        hi = __builtin_amdgcn_alignbyte(v.z, v.y, o);
    };
    // 16 bytes of a row from byte address p, realigned: w[0..2] = bytes p .. p+11 (runs of 10)
    auto row12 = [](const uint8_t* p, uint32_t (&w)[3]) {
        const uintptr_t u = reinterpret_cast<uintptr_t>(p);
        const u4a4k v = gload<u4a4k>(u & ~(uintptr_t)3);
        const uint32_t o = (uint32_t)(u & 3);
        w[0] = __builtin_amdgcn_alignbyte(v.y, v.x, o);
        w[1] = __builtin_amdgcn_alignbyte(v.z, v.y, o);
        w[2] = __builtin_amdgcn_alignbyte(v.w, v.z, o);
    };
    // 28 bytes of a row from byte address p, realigned: w[0..5] = bytes p .. p+23 (runs of 20)
    auto row24 = [](const uint8_t* p, uint32_t (&w)[6]) {
        const uintptr_t u = reinterpret_cast<uintptr_t>(p);
        const u4a4k v = gload<u4a4k>(u & ~(uintptr_t)3);
        const u3a4k x = gload<u3a4k>((u & ~(uintptr_t)3) + 16);
        const uint32_t o = (uint32_t)(u & 3);
        w[0] = __builtin_amdgcn_alignbyte(v.y, v.x, o);
        w[1] = __builtin_amdgcn_alignbyte(v.z, v.y, o);
        w[2] = __builtin_amdgcn_alignbyte(v.w, v.z, o);
        w[3] = __builtin_amdgcn_alignbyte(x.x, v.w, o);
        w[4] = __builtin_amdgcn_alignbyte(x.y, x.x, o);
        w[5] = __builtin_amdgcn_alignbyte(x.z, x.y, o);
    };
    // (byte i, byte i + 1) of a realigned run as a 16-bit pair
    // (i is a constant once the element loops are unrolled)
    auto tap_pair = [](const uint32_t (&w)[RW > 0 ? RW : 1], int i) -> s2k {
        const unsigned sel = 0x0c000c00u | (unsigned)(i & 3) | ((unsigned)((i & 3) + 1) << 16);
        const uint32_t hi = (i >> 2) + 1 < RW ? w[(i >> 2) + 1 < RW ? (i >> 2) + 1 : RW - 1] : 0u;
        return __builtin_bit_cast(s2k, __builtin_amdgcn_perm(hi, w[i >> 2], sel));
    };

    const int gx = valid ? pt / a.ny : 0, gy = valid ? pt % a.ny : 0;
    float px0 = (float)(gx * a.pixel_step), py0 = (float)(gy * a.pixel_step);
    if constexpr (CHAIN) {
        // the point pass - 1 left (k_traj_init's grid point for pass 0): wait for that pass, then
        // read it past the caches (the MI355X_MICROARCH.md hand-off: the writer stores sc1, waits
        // vmcnt(0), then bumps the flag)
        if (valid) {
            if (pass > 0) {
                int n = 0;
                while (__hip_atomic_load(t.flag + pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < pass &&
                       n < kChainSpinMax) {
                    __builtin_amdgcn_s_sleep(8);
                    n++;
                }
                if (n >= kChainSpinMax && s == 0) atomicAdd(t.num + 1, 1);   // reported as an error by the host
                // the point's load stays below the poll (wavefront scope: no instruction; the load
                // is sc1 and issues only once the poll has matched)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            const float2 c = __builtin_bit_cast(
                float2, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(t.cur) + pt, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT));
            px0 = c.x;
            py0 = c.y;
        }
    } else if (a.prev_pts && valid) {   // trajectory passes: arbitrary start points (flags 0: nextPt = prevPt)
        const float* pp = a.prev_pts + ((long long)pair * a.npts + pt) * 2;
        px0 = pp[0];
        py0 = pp[1];
    }
    float npx = 0.f, npy = 0.f;   // nextPts[ptidx]
    int status = 1;

    uint32_t sd[NE];              // (Ix & 0xffff) | Iy << 16
    uint32_t si[(NE + 1) / 2];    // I*32 values, two per word

    const uint8_t* slab1 = CHAIN ? t.pyr[pass] : a.pyr1 + (long long)pair * a.g.img_bytes;
    const uint8_t* slab2 = CHAIN ? t.pyr[pass + 1] : a.pyr2 + (long long)pair * a.g.img_bytes;
    const uint32_t* dslab = CHAIN ? t.der[pass] : a.der + (long long)pair * a.g.der_words;

    for (int level = a.maxl; level >= 0; --level) {
        const Level L = a.g.lv[level];
        const int pitch = L.pitch;
        const uint8_t* Ib = slab1 + L.img_off + L.core();
        const uint8_t* Jb = slab2 + L.img_off + L.core();
        const uint32_t* Db = dslab + L.der_off + L.core();

        const float scale = (float)(1. / (1 << level));
        float ppx = px0 * scale, ppy = py0 * scale;
        if (level == a.maxl) { npx = ppx; npy = ppy; }
        else { npx = npx * 2.f; npy = npy * 2.f; }
        ppx = ppx - HALFW;
        ppy = ppy - HALFW;
        const int ipx = (int)floorf(ppx), ipy = (int)floorf(ppy);
        bool ok = valid && !(ipx < -WIN || ipx >= L.w || ipy < -WIN || ipy >= L.h);
        if (valid && !ok && level == 0) status = 0;

        int w00 = 0, w01 = 0, w10 = 0, w11 = 0;
        if (ok) {
            const float fa = ppx - (float)ipx, fb = ppy - (float)ipy;
            w00 = __float2int_rn((1.f - fa) * (1.f - fb) * 16384.f);
            w01 = __float2int_rn(fa * (1.f - fb) * 16384.f);
            w10 = __float2int_rn((1.f - fa) * fb * 16384.f);
            w11 = 16384 - w00 - w01 - w10;
        }
        int toff[EC];
#pragma unroll
        for (int i = 0; i < EC; i++) toff[i] = ey[i] * pitch + ex[i];
        const int ibase = ipy * pitch + ipx;

        // ---- window extraction + A sums (chains q*4+k, q: 0 A11, 1 A12, 2 A22)
        float acc = 0.f;
        u4a4k dpa[BLK ? 5 : 1] = {};
        u2a4k dpb[BLK ? 5 : 1] = {};
        if (BLK && ok)
#pragma unroll
            for (int ar = 0; ar < (BLK ? 5 : 1); ar++) {
                const uint32_t* q = Db + (ibase + toff[0]) + ar * pitch;
                dpa[ar] = *reinterpret_cast<const u4a4k*>(q);
                dpb[ar] = *reinterpret_cast<const u2a4k*>(q + 4);
            }
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if (ok && BLK) {
                // 4 x 5 block: rows a = 0 .. 4 of the block (4 element rows + the lower tap row),
                // each 6 I bytes and 6 derivative words; row a's tap / Ix / Iy pairs serve element row
                // a as its upper taps and element row a - 1 as its lower ones
                const int o = ibase + c * R * pitch + toff[0];
                const s2k W0 = {(short)w00, (short)w01}, W1 = {(short)w10, (short)w11};
                s2k pu[5], xu[5], yu[5];
#pragma unroll
                for (int ar = 0; ar <= 4; ar++) {
                    uint32_t lo, hi;
                    row8(Ib + o + ar * pitch, lo, hi);
                    const u4a4k v = dpa[BLK ? ar : 0];
                    const u2a4k w2 = dpb[BLK ? ar : 0];
                    const uint32_t d[6] = {v.x, v.y, v.z, v.w, w2.x, w2.y};
                    s2k pl[5], xl[5], yl[5];
#pragma unroll
                    for (int b = 0; b < 5; b++) {
                        const unsigned sel = 0x0c000c00u | (unsigned)b | ((unsigned)(b + 1) << 16);
                        pl[b] = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(hi, lo, sel));
                        xl[b] = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(d[b + 1], d[b], 0x05040100u));
                        yl[b] = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(d[b + 1], d[b], 0x07060302u));
                    }
                    if (ar > 0) {
#pragma unroll
                        for (int b = 0; b < 5; b++) {
                            const int i = 5 * (ar - 1) + b;
                            const int ival = __builtin_amdgcn_sdot2(pu[b], W0, sdot2_sacc(pl[b], W1, 256), false) >> 9;
                            const int ixv = __builtin_amdgcn_sdot2(xu[b], W0, sdot2_sacc(xl[b], W1, 8192), false) >> 14;
                            const int iyv = __builtin_amdgcn_sdot2(yu[b], W0, sdot2_sacc(yl[b], W1, 8192), false) >> 14;
                            const int k = c * EC + i;
                            sd[k] = ((uint32_t)ixv & 0xffffu) | ((uint32_t)iyv << 16);
                            if (k & 1) si[k >> 1] = (si[k >> 1] & 0xffffu) | ((uint32_t)ival << 16);
                            else si[k >> 1] = (uint32_t)ival;
                            float* wp = ch + woff[i];
                            wp[0] = (float)__mul24(ixv, ixv);
                            wp[4 * STRIDE] = (float)__mul24(ixv, iyv);
                            wp[8 * STRIDE] = (float)__mul24(iyv, iyv);
                        }
                    }
#pragma unroll
                    for (int b = 0; b < 5; b++) { pu[b] = pl[b]; xu[b] = xl[b]; yu[b] = yl[b]; }
                }
                if (c + 1 < NCH)
#pragma unroll
                    for (int ar = 0; ar < (BLK ? 5 : 1); ar++) {
                        const uint32_t* q = Db + (ibase + (c + 1) * R * pitch + toff[0]) + ar * pitch;
                        dpa[ar] = *reinterpret_cast<const u4a4k*>(q);
                        dpb[ar] = *reinterpret_cast<const u2a4k*>(q + 4);
                    }
            } else if (ok) {
                // LPP 64: the run's I bytes and derivative words of both tap rows, vector loads
                uint64_t r0 = 0, r1 = 0;
                uint32_t dr0[RUN >= 10 ? RUN + 1 : 6] = {}, dr1[RUN >= 10 ? RUN + 1 : 6] = {};
                uint32_t i0w[RW > 0 ? RW : 1] = {}, i1w[RW > 0 ? RW : 1] = {};
                if constexpr (LPP == 16) {
                    const int o = ibase + c * R * pitch + toff[0];
                    row24(Ib + o, i0w);
                    row24(Ib + o + pitch, i1w);
                    const uint32_t* dp = Db + o;
#pragma unroll
                    for (int rr = 0; rr < 2; rr++) {
                        uint32_t* dr = rr ? dr1 : dr0;
                        const uint32_t* q = dp + rr * pitch;
#pragma unroll
                        for (int b = 0; b < 5; b++) {
                            const u4a4k v = *reinterpret_cast<const u4a4k*>(q + 4 * b);
                            dr[4 * b] = v.x; dr[4 * b + 1] = v.y; dr[4 * b + 2] = v.z; dr[4 * b + 3] = v.w;
                        }
                        dr[20] = q[20];
                    }
                }
                if constexpr (LPP == 32) {
                    const int o = ibase + c * R * pitch + toff[0];
                    row12(Ib + o, i0w);
                    row12(Ib + o + pitch, i1w);
                    const uint32_t* dp = Db + o;
#pragma unroll
                    for (int rr = 0; rr < 2; rr++) {
                        uint32_t* dr = rr ? dr1 : dr0;
                        const uint32_t* q = dp + rr * pitch;
                        const u4a4k a0 = *reinterpret_cast<const u4a4k*>(q);
                        const u4a4k a1 = *reinterpret_cast<const u4a4k*>(q + 4);
                        const u3a4k a2 = *reinterpret_cast<const u3a4k*>(q + 8);
                        dr[0] = a0.x; dr[1] = a0.y; dr[2] = a0.z; dr[3] = a0.w;
                        dr[4] = a1.x; dr[5] = a1.y; dr[6] = a1.z; dr[7] = a1.w;
                        dr[8] = a2.x; dr[9] = a2.y; dr[10] = a2.z;
                    }
                }
                if constexpr (LPP == 64) {
                    const int o = ibase + c * R * pitch + toff[0];
                    uint32_t l0, h0, l1, h1;
                    row8(Ib + o, l0, h0);
                    row8(Ib + o + pitch, l1, h1);
                    r0 = ((uint64_t)h0 << 32) | l0;
                    r1 = ((uint64_t)h1 << 32) | l1;
                    const uint32_t* dp = Db + o;
                    const u4a4k a0 = *reinterpret_cast<const u4a4k*>(dp);
                    const u2a4k b0 = *reinterpret_cast<const u2a4k*>(dp + 4);
                    const u4a4k a1 = *reinterpret_cast<const u4a4k*>(dp + pitch);
                    const u2a4k b1 = *reinterpret_cast<const u2a4k*>(dp + pitch + 4);
                    dr0[0] = a0.x; dr0[1] = a0.y; dr0[2] = a0.z; dr0[3] = a0.w; dr0[4] = b0.x; dr0[5] = b0.y;
                    dr1[0] = a1.x; dr1[1] = a1.y; dr1[2] = a1.z; dr1[3] = a1.w; dr1[4] = b1.x; dr1[5] = b1.y;
                }
#pragma unroll
                for (int i = 0; i < EC; i++) {
                    const int o = ibase + c * R * pitch + toff[i];
                    const uint8_t* ip = Ib + o;
                    const uint32_t* dp = Db + o;
                    int ival;
                    uint32_t d00, d01, d10, d11;
                    int ixv, iyv;
                    if constexpr (RUN != 0) {
                        // the same integer sums as below through v_dot2 on 16-bit pairs (tap bytes,
                        // Ix / Iy halves; signed weights), no 32-bit multiplies
                        const s2k W0 = {(short)w00, (short)w01}, W1 = {(short)w10, (short)w11};
                        s2k t0, t1;
                        if constexpr (LPP == 64) {
                            const unsigned sel = 0x0c000c00u | (unsigned)i | ((unsigned)(i + 1) << 16);
                            t0 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm((uint32_t)(r0 >> 32), (uint32_t)r0, sel));
                            t1 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm((uint32_t)(r1 >> 32), (uint32_t)r1, sel));
                        } else {
                            t0 = tap_pair(i0w, i);
                            t1 = tap_pair(i1w, i);
                        }
                        ival = __builtin_amdgcn_sdot2(t0, W0, sdot2_sacc(t1, W1, 256), false) >> 9;
                        d00 = dr0[i]; d01 = dr0[i + 1]; d10 = dr1[i]; d11 = dr1[i + 1];
                        const s2k x0 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(d01, d00, 0x05040100u));
                        const s2k x1 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(d11, d10, 0x05040100u));
                        const s2k y0 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(d01, d00, 0x07060302u));
                        const s2k y1 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(d11, d10, 0x07060302u));
                        ixv = __builtin_amdgcn_sdot2(x0, W0, sdot2_sacc(x1, W1, 8192), false) >> 14;
                        iyv = __builtin_amdgcn_sdot2(y0, W0, sdot2_sacc(y1, W1, 8192), false) >> 14;
                    } else {
                        ival = (ip[0] * w00 + ip[1] * w01 + ip[pitch] * w10 + ip[pitch + 1] * w11 + 256) >> 9;
                        d00 = dp[0]; d01 = dp[1]; d10 = dp[pitch]; d11 = dp[pitch + 1];
                        ixv = ((int)(int16_t)d00 * w00 + (int)(int16_t)d01 * w01 + (int)(int16_t)d10 * w10 +
                               (int)(int16_t)d11 * w11 + 8192) >> 14;
                        iyv = (((int)d00 >> 16) * w00 + ((int)d01 >> 16) * w01 + ((int)d10 >> 16) * w10 +
                               ((int)d11 >> 16) * w11 + 8192) >> 14;
                    }
                    const int k = c * EC + i;
                    sd[k] = ((uint32_t)ixv & 0xffffu) | ((uint32_t)iyv << 16);
                    if (k & 1) si[k >> 1] = (si[k >> 1] & 0xffffu) | ((uint32_t)ival << 16);
                    else si[k >> 1] = (uint32_t)ival;
                    float* wp = ch + woff[i];
                    // |Ix|, |Iy| <= 4080: 24-bit multiplies (v_mul_i32_i24, full rate; a 32-bit
                    // v_mul_lo_u32 is quarter rate), products exact in int32
                    wp[0] = (float)__mul24(ixv, ixv);
                    wp[4 * STRIDE] = (float)__mul24(ixv, iyv);
                    wp[8 * STRIDE] = (float)__mul24(iyv, iyv);
                }
            }
            __syncthreads();
            if (ok && s < 12) {
                const float4* cp = reinterpret_cast<const float4*>(ch + s * STRIDE);
#pragma unroll
                for (int t = 0; t < 20; t++) {
                    const float4 v = cp[t];
                    acc = acc + v.x; acc = acc + v.y; acc = acc + v.z; acc = acc + v.w;
                }
            }
            __syncthreads();
        }
        if (ok && s < 12) res[s] = acc;
        __syncthreads();

        float A11 = 0.f, A12 = 0.f, A22 = 0.f, Dinv = 0.f;
        if (ok) {
            const float4 r0 = reinterpret_cast<const float4*>(res)[0];
            const float4 r1 = reinterpret_cast<const float4*>(res)[1];
            const float4 r2 = reinterpret_cast<const float4*>(res)[2];
            A11 = ((r0.x + r0.y) + r0.z) + r0.w;
            A12 = ((r1.x + r1.y) + r1.z) + r1.w;
            A22 = ((r2.x + r2.y) + r2.z) + r2.w;
            A11 = A11 * FLT_SCALE;
            A12 = A12 * FLT_SCALE;
            A22 = A22 * FLT_SCALE;
            const float D = A11 * A22 - A12 * A12;
            const float minEig = (A22 + A11 - __builtin_sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                                 (float)(2 * WIN * WIN);
            if (minEig < a.min_eig || D < FLT_EPSILON) {
                ok = false;
                if (level == 0) status = 0;
            } else {
                Dinv = 1.f / D;
            }
        }
        __syncthreads();   // res is rewritten by the iteration phase

        // ---- Newton iterations
        float nx = npx - HALFW, ny = npy - HALFW;
        float pdx = 0.f, pdy = 0.f;
        bool act = ok;
        for (int j = 0; j < a.max_iters; j++) {
            if (!__any(act)) break;
            int jbase = 0, v00 = 0, v01 = 0, v10 = 0, v11 = 0;
            if (act) {
                const int inx = (int)floorf(nx), iny = (int)floorf(ny);
                if (inx < -WIN || inx >= L.w || iny < -WIN || iny >= L.h) {
                    act = false;
                    if (level == 0) status = 0;
                } else {
                    const float fa = nx - (float)inx, fb = ny - (float)iny;
                    v00 = __float2int_rn((1.f - fa) * (1.f - fb) * 16384.f);
                    v01 = __float2int_rn(fa * (1.f - fb) * 16384.f);
                    v10 = __float2int_rn((1.f - fa) * fb * 16384.f);
                    v11 = 16384 - v00 - v01 - v10;
                    jbase = iny * pitch + inx;
                }
            }
            float bacc = 0.f;
            // BLK: the block's five J rows of chunk c + 1 are loaded while chunk c is summed (two waves
            // per SIMD hide little of a global load's latency); pitch is a multiple of 64, so one
            // realignment shift serves every row and chunk
            u3a4k jr[BLK ? 5 : 1] = {};
            uint32_t jsh = 0;
            const uint8_t* jb0 = nullptr;
            if (BLK && act) {
                const uintptr_t u = reinterpret_cast<uintptr_t>(Jb + (jbase + toff[0]));
                jsh = (uint32_t)(u & 3);
                jb0 = reinterpret_cast<const uint8_t*>(u & ~(uintptr_t)3);
#pragma unroll
                for (int ar = 0; ar < (BLK ? 5 : 1); ar++) jr[ar] = gload<u3a4k>(reinterpret_cast<uintptr_t>(jb0 + ar * pitch));
            }
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                if (act && BLK) {
                    const s2k W0 = {(short)v00, (short)v01}, W1 = {(short)v10, (short)v11};
                    s2k pu[5];
#pragma unroll
                    for (int ar = 0; ar <= 4; ar++) {
                        const uint32_t lo = __builtin_amdgcn_alignbyte(jr[BLK ? ar : 0].y, jr[BLK ? ar : 0].x, jsh);
                        const uint32_t hi = __builtin_amdgcn_alignbyte(jr[BLK ? ar : 0].z, jr[BLK ? ar : 0].y, jsh);
                        s2k pl[5];
#pragma unroll
                        for (int b = 0; b < 5; b++) {
                            const unsigned sel = 0x0c000c00u | (unsigned)b | ((unsigned)(b + 1) << 16);
                            pl[b] = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(hi, lo, sel));
                        }
                        if (ar > 0) {
#pragma unroll
                            for (int b = 0; b < 5; b++) {
                                const int i = 5 * (ar - 1) + b;
                                const int jv = __builtin_amdgcn_sdot2(pu[b], W0, sdot2_sacc(pl[b], W1, 256), false) >> 9;
                                const int k = c * EC + i;
                                const int iv = (k & 1) ? (int)(si[k >> 1] >> 16) : (int)(si[k >> 1] & 0xffffu);
                                const int diff = jv - iv;
                                const uint32_t dv = sd[k];
                                float* wp = ch + woff[i];
                                wp[0] = (float)__mul24(diff, (int)(int16_t)dv);
                                wp[4 * STRIDE] = (float)__mul24(diff, (int)dv >> 16);
                            }
                        }
#pragma unroll
                        for (int b = 0; b < 5; b++) pu[b] = pl[b];
                    }
                    if (c + 1 < NCH)
#pragma unroll
                        for (int ar = 0; ar < (BLK ? 5 : 1); ar++)
                            jr[ar] = gload<u3a4k>(reinterpret_cast<uintptr_t>(jb0 + ((c + 1) * R + ar) * pitch));
                } else if (act) {
                    uint32_t j0l = 0, j0h = 0, j1l = 0, j1h = 0;
                    uint32_t j0w[RW > 0 ? RW : 1] = {}, j1w[RW > 0 ? RW : 1] = {};
                    if constexpr (LPP == 16) {
                        const uint8_t* jp = Jb + (jbase + c * R * pitch + toff[0]);
                        row24(jp, j0w);
                        row24(jp + pitch, j1w);
                    } else if constexpr (LPP == 64) {
                        const uint8_t* jp = Jb + (jbase + c * R * pitch + toff[0]);
                        row8(jp, j0l, j0h);
                        row8(jp + pitch, j1l, j1h);
                    } else if constexpr (LPP == 32) {
                        const uint8_t* jp = Jb + (jbase + c * R * pitch + toff[0]);
                        row12(jp, j0w);
                        row12(jp + pitch, j1w);
                    }
#pragma unroll
                    for (int i = 0; i < EC; i++) {
                        int jv;
                        if constexpr (RUN != 0) {
                            // (J[x], J[x+1]) of both tap rows as 16-bit pairs; v_dot2 gives the
                            // reference's int sum j00*v00 + j01*v01 + j10*v10 + j11*v11 exactly
                            s2k t0, t1;
                            if constexpr (LPP == 64) {
                                const unsigned sel = 0x0c000c00u | (unsigned)i | ((unsigned)(i + 1) << 16);
                                t0 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(j0h, j0l, sel));
                                t1 = __builtin_bit_cast(s2k, __builtin_amdgcn_perm(j1h, j1l, sel));
                            } else {
                                t0 = tap_pair(j0w, i);
                                t1 = tap_pair(j1w, i);
                            }
                            const s2k W0 = {(short)v00, (short)v01}, W1 = {(short)v10, (short)v11};
                            jv = __builtin_amdgcn_sdot2(t0, W0, sdot2_sacc(t1, W1, 256), false) >> 9;
                        } else {
                            const uint8_t* jp = Jb + (jbase + c * R * pitch + toff[i]);
                            jv = (jp[0] * v00 + jp[1] * v01 + jp[pitch] * v10 + jp[pitch + 1] * v11 + 256) >> 9;
                        }
                        const int k = c * EC + i;
                        const int iv = (k & 1) ? (int)(si[k >> 1] >> 16) : (int)(si[k >> 1] & 0xffffu);
                        const int diff = jv - iv;
                        const uint32_t dv = sd[k];
                        float* wp = ch + woff[i];
                        // |diff| <= 8160, |Ix|, |Iy| <= 4080: exact 24-bit multiplies
                        wp[0] = (float)__mul24(diff, (int)(int16_t)dv);
                        wp[4 * STRIDE] = (float)__mul24(diff, (int)dv >> 16);
                    }
                }
                __syncthreads();
                if (act && s < 8) {
                    const float4* cp = reinterpret_cast<const float4*>(ch + s * STRIDE);
#pragma unroll
                    for (int t = 0; t < 20; t++) {
                        const float4 v = cp[t];
                        bacc = bacc + v.x; bacc = bacc + v.y; bacc = bacc + v.z; bacc = bacc + v.w;
                    }
                }
                __syncthreads();
            }
            if (act && s < 8) res[s] = bacc;
            __syncthreads();
            if (act) {
                const float4 q1 = reinterpret_cast<const float4*>(res)[0];
                const float4 q2 = reinterpret_cast<const float4*>(res)[1];
                float b1 = (q1.x + q1.z) + (q1.y + q1.w);
                float b2 = (q2.x + q2.z) + (q2.y + q2.w);
                b1 = b1 * FLT_SCALE;
                b2 = b2 * FLT_SCALE;
                const float dx = (A12 * b2 - A22 * b1) * Dinv;
                const float dy = (A12 * b1 - A11 * b2) * Dinv;
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
            __syncthreads();
        }

        if (level == 0 && valid && status) {
            // err pass of LKTrackerInvoker: its final bounds check is observable (status).
            const int fx = (int)floorf(npx - HALFW), fy = (int)floorf(npy - HALFW);
            if (fx < -WIN || fx >= L.w || fy < -WIN || fy >= L.h) status = 0;
        }
    }

    if constexpr (CHAIN) {
        // k_traj_update's bookkeeping for this point and pass (optical_flow_calculator.cpp:178-242)
        if (valid && s == 0) {
            const bool last = pass == t.nimg - 2;
            // outputs: the caller's mapped page-locked arrays when given, else the device ones
            float* tj = t.htraj ? t.htraj : t.traj;
            double* vv = t.hvec ? t.hvec : t.vectors;
            float* sp0 = t.hstart ? t.hstart : t.start_pts;
            double* v = (last && vv) ? vv + 4LL * pt : nullptr;
            if (t.htraj && pass == 0) {   // k_traj_init wrote the device row's start
                tj[(long long)pt * t.nimg * 2] = px0;
                tj[(long long)pt * t.nimg * 2 + 1] = py0;
            }
            if (last && sp0) {
                sp0[2 * pt] = px0;
                sp0[2 * pt + 1] = py0;
            }
            if (status) {
                const float ex = npx, ey = npy;
                if (last) {
                    const float xd = ex - px0, yd = ey - py0;
                    if (fabs((double)fabsf(xd)) > t.mvs || fabs((double)fabsf(yd)) > t.mvs) {
                        if (v) { v[0] = px0; v[1] = py0; v[2] = xd; v[3] = yd; }
                        atomicAdd(t.num, 1);
                    } else if (v) {
                        v[0] = px0; v[1] = py0; v[2] = 0.0; v[3] = 0.0;
                    }
                }
                if (ex > 10.0f && ey > 10.0f && ex < (float)(t.w - 10) && ey < (float)(t.h - 10)) {
                    __hip_atomic_store(reinterpret_cast<unsigned long long*>(t.cur) + pt,
                                       __builtin_bit_cast(unsigned long long, make_float2(ex, ey)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    const int l = __hip_atomic_load(t.tlen + pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    tj[((long long)pt * t.nimg + l) * 2] = ex;
                    tj[((long long)pt * t.nimg + l) * 2 + 1] = ey;
                    __hip_atomic_store(t.tlen + pt, l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else if (v) {
                v[0] = -1.0; v[1] = -1.0; v[2] = 0.0; v[3] = 0.0;
            }
            if (last && t.htraj) {
                // the mapped row's entries past traj_len (the device rows were zeroed by k_traj_init;
                // every entry of a mapped row is written once) and traj_len itself
                const int lf = __hip_atomic_load(t.tlen + pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (int k = lf; k < t.nimg; k++) {
                    tj[((long long)pt * t.nimg + k) * 2] = 0.f;
                    tj[((long long)pt * t.nimg + k) * 2 + 1] = 0.f;
                }
                t.htlen[pt] = lf;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(t.flag + pt, pass + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (valid && s == 0) {
        const long long o = (long long)pair * a.npts + pt;
        a.next_pts[2 * o] = npx;
        a.next_pts[2 * o + 1] = npy;
        a.status[o] = (uint8_t)status;
    }
}

// ------------------------------------------------------------------ A7: perspective fit
// fdlibm __ieee754_hypot (what OpenCV's JacobiSVD reaches through ::hypot on glibc).
__device__ double dev_hypot(double x, double y)
{
    auto hi = [](double d) { return (int)(__double_as_longlong(d) >> 32); };
    auto lo = [](double d) { return (unsigned)(__double_as_longlong(d) & 0xffffffffll); };
    auto set_hi = [](double d, int h) {
        unsigned long long u = (unsigned long long)__double_as_longlong(d);
        u = ((unsigned long long)(unsigned)h << 32) | (u & 0xffffffffull);
        return __longlong_as_double((long long)u);
    };
    double a, b, t1, t2, y1, y2, w;
    int j, k, ha, hb;
    ha = hi(x) & 0x7fffffff;
    hb = hi(y) & 0x7fffffff;
    if (hb > ha) { a = y; b = x; j = ha; ha = hb; hb = j; }
    else { a = x; b = y; }
    a = set_hi(a, ha);
    b = set_hi(b, hb);
    if ((ha - hb) > 0x3c00000) return a + b;
    k = 0;
    if (ha > 0x5f300000) {
        if (ha >= 0x7ff00000) {
            w = a + b;
            if (((ha & 0xfffff) | lo(a)) == 0) w = a;
            if ((((unsigned)hb ^ 0x7ff00000u) | lo(b)) == 0) w = b;
            return w;
        }
        ha -= 0x25800000; hb -= 0x25800000; k += 600;
        a = set_hi(a, ha);
        b = set_hi(b, hb);
    }
    if (hb < 0x20b00000) {
        if (hb <= 0x000fffff) {
            if ((hb | (int)lo(b)) == 0) return a;
            t1 = set_hi(0.0, 0x7fd00000);
            b *= t1;
            a *= t1;
            k -= 1022;
        } else {
            ha += 0x25800000; hb += 0x25800000; k -= 600;
            a = set_hi(a, ha);
            b = set_hi(b, hb);
        }
    }
    w = a - b;
    if (w > b) {
        t1 = set_hi(0.0, ha);
        t2 = a - t1;
        w = __builtin_sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
    } else {
        a = a + a;
        y1 = set_hi(0.0, hb);
        y2 = b - y1;
        t1 = set_hi(0.0, ha + 0x00100000);
        t2 = a - t1;
        w = __builtin_sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
    }
    if (k != 0) {
        t1 = set_hi(1.0, hi(1.0) + (k << 20));
        return t1 * w;
    }
    return w;
}

// getPerspectiveTransform(src, dst) = solve(A, b, DECOMP_SVD) on the 8x8 DLT system:
// lapack.cpp JacobiSVDImpl_<double> (one-sided Jacobi on A's columns, eps 10*DBL_EPSILON,
// max(m,30) sweeps, descending sort) then SVBkSb (threshold 2*DBL_EPSILON*sum(w)).
// One lane runs this solve (k_ransac_hyp: one hypothesis per lane); its working arrays (At[64],
// Vt[64], W[8], bv[8], x[8]) live in LDS, lane-interleaved: lane l's element e at fw[e * S + l]
// (S = lanes, conflict-free across lanes).  As private arrays they were scratch memory.
// k_fit / k_band_fit run the wave-parallel form below (dev_perspective_fit_wave).
constexpr int kFitWorkDoubles = 152;
template <int S>
__device__ __forceinline__ void dev_perspective_fit_s(const float* src, const float* dst, double* M, double* fw)
{
#define AT(e) fw[(e) * S]
#define VT(e) fw[(64 + (e)) * S]
#define WV(e) fw[(128 + (e)) * S]
#define BV(e) fw[(136 + (e)) * S]
#define XV(e) fw[(144 + (e)) * S]
    for (int i = 0; i < 64; i++) AT(i) = 0.0;
    for (int i = 0; i < 4; i++) {
        const float sx = src[2 * i], sy = src[2 * i + 1], dx = dst[2 * i], dy = dst[2 * i + 1];
        // A[i][c] stored as At[c*8 + i]; rows i (x equations) and i+4 (y equations)
        AT(0 * 8 + i) = sx; AT(1 * 8 + i) = sy; AT(2 * 8 + i) = 1.0;
        AT(3 * 8 + i + 4) = sx; AT(4 * 8 + i + 4) = sy; AT(5 * 8 + i + 4) = 1.0;
        AT(6 * 8 + i) = (double)(-sx * dx);
        AT(7 * 8 + i) = (double)(-sy * dx);
        AT(6 * 8 + i + 4) = (double)(-sx * dy);
        AT(7 * 8 + i + 4) = (double)(-sy * dy);
        BV(i) = dx;
        BV(i + 4) = dy;
    }
    const int m = 8, n = 8;
    const double eps = DBL_EPSILON * 10;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) { const double t = AT(i * m + k); sd += t * t; }
        WV(i) = sd;
        for (int k = 0; k < n; k++) VT(i * n + k) = 0;
        VT(i * n + i) = 1;
    }
    for (int iter = 0; iter < 30; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double aa = WV(i), p = 0, bb = WV(j);
                for (int k = 0; k < m; k++) p += AT(i * m + k) * AT(j * m + k);
                if (fabs(p) <= eps * __builtin_sqrt(aa * bb)) continue;
                p *= 2;
                const double beta = aa - bb, gamma = dev_hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = __builtin_sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = __builtin_sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                aa = bb = 0;
                for (int k = 0; k < m; k++) {
                    const double ai = AT(i * m + k), aj = AT(j * m + k);
                    const double t0 = c * ai + s * aj;
                    const double t1 = -s * ai + c * aj;
                    AT(i * m + k) = t0; AT(j * m + k) = t1;
                    aa += t0 * t0; bb += t1 * t1;
                }
                WV(i) = aa; WV(j) = bb;
                changed = true;
                for (int k = 0; k < n; k++) {
                    const double vi = VT(i * n + k), vj = VT(j * n + k);
                    const double t0 = c * vi + s * vj;
                    const double t1 = -s * vi + c * vj;
                    VT(i * n + k) = t0; VT(j * n + k) = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) { const double t = AT(i * m + k); sd += t * t; }
        WV(i) = __builtin_sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++) if (WV(j) < WV(k)) j = k;
        if (i != j) {
            double t = WV(i); WV(i) = WV(j); WV(j) = t;
            for (int k = 0; k < m; k++) { t = AT(i * m + k); AT(i * m + k) = AT(j * m + k); AT(j * m + k) = t; }
            for (int k = 0; k < n; k++) { t = VT(i * n + k); VT(i * n + k) = VT(j * n + k); VT(j * n + k) = t; }
        }
    }
    // Left singular vectors: rows with W[i] <= DBL_MIN are skipped by the back-substitution
    // threshold below, so only the normalisation of the others matters.
    for (int i = 0; i < n; i++) {
        if (WV(i) <= DBL_MIN) continue;
        const double s = 1 / WV(i);
        for (int k = 0; k < m; k++) AT(i * m + k) *= s;
    }
    double threshold = 0;
    for (int i = 0; i < n; i++) { XV(i) = 0; threshold += WV(i); }
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < n; i++) {
        double wi = WV(i);
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < m; j++) s += AT(i * m + j) * BV(j);
        s *= wi;
        for (int j = 0; j < n; j++) XV(j) = XV(j) + s * VT(i * n + j);
    }
    for (int i = 0; i < 8; i++) M[i] = XV(i);
    M[8] = 1.;
#undef AT
#undef VT
#undef WV
#undef BV
#undef XV
}
// The same solve by one wave (k_fit, k_band_fit: every lane of a 64-lane workgroup calls it with
// the same src / dst).  Each rotation, and every other step, computes what dev_perspective_fit_s
// does, in the same order within each sum, so the result is bit-identical; what changes is the
// schedule.  Rotation (i, j) of sweep s (r-th in the reference's order) needs only the latest
// earlier rotations on columns i and j, which puts it at dependency depth 8 s + d_r (d_r = 0..12):
// depth L holds sweep L/8's rotations at d = L%8 and sweep L/8 - 1's at d = L%8 + 8, at most four,
// on disjoint columns (kJacSlot: i | j << 3 | previous-sweep << 6).  A sweep is complete at depth
// 8 s + 12; if it changed nothing, the next sweep's rotations already run saw the same columns and
// skipped too, so stopping there leaves the reference's state.
// Element-parallel rotations: slot q of a depth runs on the 16-lane DPP row q, lane e holding
// element e of A's column (e < 8) or element e - 8 of Vt's row (e >= 8) for both columns, so the
// update is one step; the 8-term dot products (p, and the new column norms) are summed in the
// reference's order from row_newbcast broadcasts of lanes 0..7 (v_mov_b64 DPP, then the add), and
// the scalar part (hypot, square roots, divisions) runs once per row.  The column-wise steps after
// the sweeps run one lane per column.  fw: kFitWaveDoubles of LDS.  M: the 9 entries, in every lane.
__constant__ uint8_t kJacSlot[8][4] = {{0x08, 0x7a, 0x73, 0x6c}, {0x10, 0x7b, 0x74, 0xff}, {0x18, 0x11, 0x7c, 0x75},
                                       {0x20, 0x19, 0x7d, 0xff}, {0x28, 0x21, 0x1a, 0x7e}, {0x30, 0x29, 0x22, 0xff},
                                       {0x38, 0x31, 0x2a, 0x23}, {0x39, 0x32, 0x2b, 0xff}};
constexpr int kFitWaveDoubles = 168;   // X 8 x 16 (A column | Vt row), W 8, b 8, s 8, use 8, x 8
constexpr int kJacSweeps = 30;

// ((((0 + v0) + v1) + ...) + v7) over lanes 0..7 of the lane's 16-lane DPP row: a column's sum in the
// reference's order.  The eight broadcasts (v_mov_b64 row_newbcast; v_add_f64 has no DPP form on
// gfx950) in one block behind s_nop 4: five wait states cover both DPP hazards, a VALU write of the
// source VGPR (two) and of EXEC (five), whatever the compiler schedules before the block.
__device__ __forceinline__ double rowsum8(double v)
{
    double b0, b1, b2, b3, b4, b5, b6, b7;
    asm volatile("s_nop 4\n\t"
                 "v_mov_b64_dpp %0, %8 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %1, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %2, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %3, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %4, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %5, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %6, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %7, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf"
                 : "=&v"(b0), "=&v"(b1), "=&v"(b2), "=&v"(b3), "=&v"(b4), "=&v"(b5), "=&v"(b6), "=&v"(b7)
                 : "v"(v));
    double s = 0.0;
    s = s + b0; s = s + b1; s = s + b2; s = s + b3;
    s = s + b4; s = s + b5; s = s + b6; s = s + b7;
    return s;
}

__device__ void dev_perspective_fit_wave(const float* src, const float* dst, double* M, double* fw)
{
    double* X = fw;           // X[c * 16 + k]: A[k][c] (k < 8), Vt[c][k - 8] (k >= 8)
    double* W = fw + 128;
    double* bv = fw + 136;
    double* sv = fw + 144;    // back-substitution coefficient of row i
    double* uv = fw + 152;    // 1: row i passes the threshold
    double* xv = fw + 160;
    const int lane = threadIdx.x & 63, q = lane >> 4, e = lane & 15;
    const double eps = DBL_EPSILON * 10;
    if (lane < 8) {
        const int c = lane;
        for (int k = 0; k < 16; k++) X[c * 16 + k] = k == 8 + c ? 1.0 : 0.0;
    }
    __syncthreads();
    if (lane == 0) {
        for (int i = 0; i < 4; i++) {
            const float sx = src[2 * i], sy = src[2 * i + 1], dx = dst[2 * i], dy = dst[2 * i + 1];
            // A[i][c] at X[c * 16 + i]; rows i (x equations) and i + 4 (y equations)
            X[0 * 16 + i] = sx; X[1 * 16 + i] = sy; X[2 * 16 + i] = 1.0;
            X[3 * 16 + i + 4] = sx; X[4 * 16 + i + 4] = sy; X[5 * 16 + i + 4] = 1.0;
            X[6 * 16 + i] = (double)(-sx * dx);
            X[7 * 16 + i] = (double)(-sy * dx);
            X[6 * 16 + i + 4] = (double)(-sx * dy);
            X[7 * 16 + i + 4] = (double)(-sy * dy);
            bv[i] = dx;
            bv[i + 4] = dy;
        }
    }
    __syncthreads();
    if (lane < 8) {
        double sd = 0;
        for (int k = 0; k < 8; k++) { const double t = X[lane * 16 + k]; sd += t * t; }
        W[lane] = sd;
    }
    __syncthreads();
    bool chg_prev = false, chg_cur = false;
    for (int L = 0; L < 8 * (kJacSweeps - 1) + 13; L++) {
        const int ph = L & 7, sweep = L >> 3;
        const int ent = kJacSlot[ph][q];
        const bool prev = (ent >> 6) & 1;
        const int s_of = sweep - (int)prev;
        bool rot = false;
        if (ent != 0xff && s_of >= 0 && s_of < kJacSweeps) {   // uniform over the row
            const int i = ent & 7, j = (ent >> 3) & 7;
            const double xi = X[i * 16 + e], xj = X[j * 16 + e];
            const double aa0 = W[i], bb0 = W[j];
            double p = rowsum8(xi * xj);
            if (!(fabs(p) <= eps * __builtin_sqrt(aa0 * bb0))) {   // uniform over the row
                p *= 2;
                const double beta = aa0 - bb0, gamma = dev_hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = __builtin_sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = __builtin_sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                const double t0 = c * xi + s * xj;
                const double t1 = -s * xi + c * xj;
                X[i * 16 + e] = t0;
                X[j * 16 + e] = t1;
                const double aa = rowsum8(t0 * t0), bb = rowsum8(t1 * t1);
                if (e == 0) {
                    W[i] = aa;
                    W[j] = bb;
                }
                rot = true;
            }
        }
        chg_prev = chg_prev || __ballot(rot && prev) != 0;
        chg_cur = chg_cur || __ballot(rot && !prev) != 0;
        __syncthreads();
        if (ph == 4 && sweep >= 1 && !chg_prev) break;   // sweep - 1 complete, nothing changed
        if (ph == 7) { chg_prev = chg_cur; chg_cur = false; }
    }
    // singular values = column norms; descending selection sort (the reference's comparisons, on
    // every lane), applied as a permutation of the columns
    double w[8];
    int perm[8];
    if (lane < 8) {
        double sd = 0;
        for (int k = 0; k < 8; k++) { const double t = X[lane * 16 + k]; sd += t * t; }
        W[lane] = __builtin_sqrt(sd);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = W[i]; perm[i] = i; }
#pragma unroll
    for (int i = 0; i < 7; i++) {
        int j = i;
        double wj = w[i];
#pragma unroll
        for (int k = i + 1; k < 8; k++)
            if (wj < w[k]) { j = k; wj = w[k]; }
        int pj = perm[i];
#pragma unroll
        for (int k = i + 1; k < 8; k++)
            if (k == j) pj = perm[k];
#pragma unroll
        for (int k = i + 1; k < 8; k++)
            if (k == j) { w[k] = w[i]; perm[k] = perm[i]; }
        w[i] = wj;
        perm[i] = pj;
    }
    double a[8], v[8];
    if (lane < 8) {
        int src_c = perm[0];
#pragma unroll
        for (int k = 1; k < 8; k++) if (lane == k) src_c = perm[k];
#pragma unroll
        for (int k = 0; k < 8; k++) { a[k] = X[src_c * 16 + k]; v[k] = X[src_c * 16 + 8 + k]; }
    }
    __syncthreads();
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    if (lane < 8) {
        double wl = w[0];
#pragma unroll
        for (int k = 1; k < 8; k++) if (lane == k) wl = w[k];
        // left singular vectors (rows with W <= DBL_MIN fail the threshold below anyway)
        if (!(wl <= DBL_MIN)) {
            const double s = 1 / wl;
#pragma unroll
            for (int k = 0; k < 8; k++) a[k] *= s;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) X[lane * 16 + 8 + k] = v[k];
        const bool use = !(fabs(wl) <= threshold);
        double s = 0;
        if (use) {
            const double wi = 1 / wl;
#pragma unroll
            for (int k = 0; k < 8; k++) s += a[k] * bv[k];
            s *= wi;
        }
        sv[lane] = s;
        uv[lane] = use ? 1.0 : 0.0;
    }
    __syncthreads();
    if (lane < 8) {
        double x = 0;
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (uv[i] != 0.0) x = x + sv[i] * X[i * 16 + 8 + lane];
        xv[lane] = x;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; i++) M[i] = xv[i];
    M[8] = 1.;
}

// lapack.cpp invert(DECOMP_LU) for 3x3 CV_64F: cofactors times 1/det3; det == 0 -> zeros.
__device__ void dev_invert3x3(const double* m, double* out)
{
    const double d0 = m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
                      m[2] * (m[3] * m[7] - m[4] * m[6]);
    if (d0 != 0.) {
        const double d = 1. / d0;
        out[0] = (m[4] * m[8] - m[5] * m[7]) * d;
        out[1] = (m[2] * m[7] - m[1] * m[8]) * d;
        out[2] = (m[1] * m[5] - m[2] * m[4]) * d;
        out[3] = (m[5] * m[6] - m[3] * m[8]) * d;
        out[4] = (m[0] * m[8] - m[2] * m[6]) * d;
        out[5] = (m[2] * m[3] - m[0] * m[5]) * d;
        out[6] = (m[3] * m[7] - m[4] * m[6]) * d;
        out[7] = (m[1] * m[6] - m[0] * m[7]) * d;
        out[8] = (m[0] * m[4] - m[1] * m[3]) * d;
    } else {
        for (int i = 0; i < 9; i++) out[i] = 0.0;
    }
}

// A6 + A7: classify every grid point (optical_flow_calculator.cpp:78-117), count accepted
// vectors, pick the first four accepted in x-major order, fit and invert.  One 256-thread
// workgroup per pair; the first-4 search is a ballot scan that stops as soon as 4 are found
// (only the count needs the full sweep).
// Two kernels.  k_classify: one 256-point block per workgroup writes the Vec4d of its points
// and a summary {accepted count, first four accepted indices in block order}.  k_fit: one wave
// per pair prefix-sums the block counts (x-major block order = the reference's point order),
// picks the first four accepted points overall and runs the fit on lane 0.
struct BlockSummary {
    int count;
    int first[4];
    int pad_[3];
};

__global__ __launch_bounds__(256) void k_classify(const float* __restrict__ next_pts, const uint8_t* __restrict__ status,
                                                  int npts, int ny, int gy0, int gy1, int pixel_step, double mvs,
                                                  double* __restrict__ vectors, BlockSummary* __restrict__ summ)
{
    const int pair = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    __shared__ int s_wcnt[4];
    const int i = blk * 256 + tid;
    bool acc = false;
    const int gyi = i % ny;
    if (i < npts && gyi >= gy0 && gyi < gy1) {   // grid rows of the band (all rows: the full path)
        const float sx = (float)((i / ny) * pixel_step), sy = (float)((i % ny) * pixel_step);
        const float2 e = reinterpret_cast<const float2*>(next_pts)[(long long)pair * npts + i];
        double v0, v1, v2, v3;
        if (status[(long long)pair * npts + i]) {
            const float xd = e.x - sx, yd = e.y - sy;       // float differences (:82-83)
            if (fabs((double)fabsf(xd)) > mvs || fabs((double)fabsf(yd)) > mvs) {
                acc = true;
                v0 = sx; v1 = sy; v2 = xd; v3 = yd;
            } else {
                v0 = sx; v1 = sy; v2 = 0.0; v3 = 0.0;
            }
        } else {
            v0 = -1.0; v1 = -1.0; v2 = 0.0; v3 = 0.0;
        }
        if (vectors) {
            double4* v = reinterpret_cast<double4*>(vectors) + (long long)pair * npts + i;
            *v = make_double4(v0, v1, v2, v3);
        }
    }
    const unsigned long long bal = __ballot(acc);
    if (lane == 0) s_wcnt[wave] = __popcll(bal);
    __syncthreads();
    int before = 0;
    for (int w2 = 0; w2 < wave; w2++) before += s_wcnt[w2];
    const int rank = before + __popcll(bal & ((1ull << lane) - 1ull));
    BlockSummary& S = summ[(long long)pair * gridDim.x + blk];
    if (acc && rank < 4) S.first[rank] = i;
    if (tid == 0) S.count = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
}

__global__ __launch_bounds__(64) void k_fit(const float* __restrict__ next_pts, int npts, int ny, int pixel_step,
                                            BlockSummary* __restrict__ summ, int nblk, PairFit* __restrict__ fits,
                                            int fit_mode, const double* __restrict__ H_ext)
{
    const int pair = blockIdx.x, lane = threadIdx.x;
    BlockSummary* S = summ + (long long)pair * nblk;
    int carry = 0;          // accepted points in blocks before the current chunk
    int pick[4] = {-1, -1, -1, -1};
    for (int b0 = 0; b0 < nblk; b0 += 64) {
        const int b = b0 + lane;
        const int cnt = b < nblk ? S[b].count : 0;
        int incl = cnt;     // inclusive prefix over the chunk
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        const int excl = carry + incl - cnt;
        if (fit_mode == MDX_FIT_RANSAC && b < nblk) S[b].pad_[0] = excl;   // k_ransac_compact's block offsets
#pragma unroll
        for (int r = 0; r < 4; r++) {
            // the block holding overall rank r (one lane at most), then broadcast its index
            const bool here = cnt > 0 && r >= excl && r < excl + cnt;
            const unsigned long long m = __ballot(here);
            if (m) {
                const int src = __ffsll((long long)m) - 1;
                const int v = here ? S[b].first[r - excl] : 0;
                const int got = __shfl(v, src);
                if (pick[r] < 0) pick[r] = got;
            }
        }
        carry += __shfl(incl, 63);
    }
    // carry and pick are wave-uniform: the whole wave runs the fit, lane 0 writes the record
    __shared__ double fw[kFitWaveDoubles];
    PairFit& f = fits[pair];
    const int total = carry;
    if (fit_mode != MDX_FIT_EXTERNAL && fit_mode != MDX_FIT_RANSAC && total >= 4) {
        float src[8], dst[8];
        for (int r = 0; r < 4; r++) {
            const int i = pick[r];
            src[2 * r] = (float)((i / ny) * pixel_step);
            src[2 * r + 1] = (float)((i % ny) * pixel_step);
            const float2 e = reinterpret_cast<const float2*>(next_pts)[(long long)pair * npts + i];
            dst[2 * r] = e.x;
            dst[2 * r + 1] = e.y;
        }
        double H[9];
        dev_perspective_fit_wave(src, dst, H, fw);
        if (lane != 0) return;
        for (int k = 0; k < 9; k++) f.H[k] = H[k];
        dev_invert3x3(H, f.Hinv);
        f.fit_status = 0;
        f.num_vectors = total;
        return;
    }
    if (lane != 0) return;
    f.num_vectors = total;
    if (fit_mode == MDX_FIT_EXTERNAL) {
        for (int k = 0; k < 9; k++) f.H[k] = H_ext[(long long)pair * 9 + k];
        dev_invert3x3(f.H, f.Hinv);
        f.fit_status = 0;
    } else if (fit_mode == MDX_FIT_RANSAC && total >= 4) {
        f.fit_status = 0;                        // H / Hinv: k_ransac_pick
    } else {
        for (int k = 0; k < 9; k++) { f.H[k] = 0.0; f.Hinv[k] = 0.0; }
        f.fit_status = total == 0 ? 1 : 2;
    }
}

// ------------------------------------------------------------------ MDX_FIT_RANSAC (not in the reference)
// Deterministic RANSAC over every accepted vector (include/mdx.h MDX_FIT_RANSAC, DESIGN.md §7d;
// restated by oracle/mdx_oracle.c ora_fit_ransac, which the GPU equals bit for bit):
//   k_ransac_compact  the accepted vectors' grid indices in x-major order (the reference's
//                     src / dst order, optical_flow_calculator.cpp:78-117), from k_fit's block offsets
//   k_ransac_hyp      one lane per hypothesis: 4 distinct draws from splitmix64(seed, h, draw, retry)
//                     and the reference's getPerspectiveTransform on them (dev_perspective_fit_s,
//                     the lane's working set interleaved in LDS)
//   k_ransac_score    every accepted vector against every hypothesis: inlier iff
//                     |H src - dst * w|^2 <= t^2 w^2 in FP64 (w the projective denominator), counts
//                     added per workgroup
//   k_ransac_pick     the hypothesis with the most inliers (lowest index on ties), its inverse
__device__ __forceinline__ uint64_t ransac_mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// the reference's acceptance test of grid point i (k_classify's)
__device__ __forceinline__ bool ransac_accepted(const float* next_pts, const uint8_t* status, long long o, int i, int ny,
                                                int pixel_step, double mvs, float& sx, float& sy, float2& e)
{
    sx = (float)((i / ny) * pixel_step);
    sy = (float)((i % ny) * pixel_step);
    e = reinterpret_cast<const float2*>(next_pts)[o];
    if (!status[o]) return false;
    const float xd = e.x - sx, yd = e.y - sy;
    return fabs((double)fabsf(xd)) > mvs || fabs((double)fabsf(yd)) > mvs;
}

__global__ __launch_bounds__(256) void k_ransac_compact(const float* __restrict__ next_pts,
                                                        const uint8_t* __restrict__ status, int npts, int ny,
                                                        int pixel_step, double mvs,
                                                        const BlockSummary* __restrict__ summ, int* __restrict__ list)
{
    const int pair = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    __shared__ int s_wcnt[4];
    const int i = blk * 256 + tid;
    bool acc = false;
    if (i < npts) {
        float sx, sy;
        float2 e;
        acc = ransac_accepted(next_pts, status, (long long)pair * npts + i, i, ny, pixel_step, mvs, sx, sy, e);
    }
    const unsigned long long bal = __ballot(acc);
    if (lane == 0) s_wcnt[wave] = __popcll(bal);
    __syncthreads();
    int before = 0;
    for (int w2 = 0; w2 < wave; w2++) before += s_wcnt[w2];
    const int rank = before + __popcll(bal & ((1ull << lane) - 1ull));
    const int off = summ[(long long)pair * gridDim.x + blk].pad_[0];
    if (acc) list[(long long)pair * npts + off + rank] = i;
}

constexpr int kRansacLanes = 32;   // hypotheses per workgroup (LDS: 32 interleaved fit working sets)
__global__ __launch_bounds__(64) void k_ransac_hyp(const float* __restrict__ next_pts, int npts, int ny, int pixel_step,
                                                   const int* __restrict__ list, const PairFit* __restrict__ fits,
                                                   int iters, uint32_t seed, double* __restrict__ hyps,
                                                   int* __restrict__ counts)
{
    __shared__ double s_fw[kFitWorkDoubles * kRansacLanes];
    const int pair = blockIdx.y, lane = threadIdx.x, h = blockIdx.x * kRansacLanes + lane;
    if (lane >= kRansacLanes || h >= iters) return;
    counts[(long long)pair * iters + h] = 0;
    const int n = fits[pair].num_vectors;
    if (fits[pair].fit_status != 0 || n < 4) return;
    int idx[4];
    for (int j = 0; j < 4; j++) {
        for (uint32_t c = 0;; c++) {
            const uint64_t x = ((uint64_t)seed << 32) | ((uint64_t)h << 20) | ((uint64_t)j << 16) | (uint64_t)(c & 0xffffu);
            const int v = (int)(ransac_mix64(x) % (uint64_t)n);
            bool dup = false;
            for (int q = 0; q < j; q++) dup = dup || idx[q] == v;
            if (!dup || c >= 0xffffu) {
                idx[j] = v;
                break;
            }
        }
    }
    float src[8], dst[8];
    for (int j = 0; j < 4; j++) {
        const int i = list[(long long)pair * npts + idx[j]];
        src[2 * j] = (float)((i / ny) * pixel_step);
        src[2 * j + 1] = (float)((i % ny) * pixel_step);
        const float2 e = reinterpret_cast<const float2*>(next_pts)[(long long)pair * npts + i];
        dst[2 * j] = e.x;
        dst[2 * j + 1] = e.y;
    }
    double Hh[9];
    dev_perspective_fit_s<kRansacLanes>(src, dst, Hh, s_fw + lane);
    for (int k = 0; k < 9; k++) hyps[((long long)pair * iters + h) * 9 + k] = Hh[k];
}

__global__ __launch_bounds__(256) void k_ransac_score(const float* __restrict__ next_pts,
                                                     const uint8_t* __restrict__ status, int npts, int ny,
                                                     int pixel_step, double mvs, const double* __restrict__ hyps,
                                                     int iters, double t2, const PairFit* __restrict__ fits,
                                                     int* __restrict__ counts)
{
    __shared__ int s_cnt[kRansacMaxIters];
    const int pair = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
    if (fits[pair].fit_status != 0 || fits[pair].num_vectors < 4) return;   // uniform per workgroup
    for (int h = tid; h < iters; h += 256) s_cnt[h] = 0;
    __syncthreads();
    const int i = blockIdx.x * 256 + tid;
    bool acc = false;
    double sx = 0.0, sy = 0.0, dx = 0.0, dy = 0.0;
    if (i < npts) {
        float fsx, fsy;
        float2 e;
        acc = ransac_accepted(next_pts, status, (long long)pair * npts + i, i, ny, pixel_step, mvs, fsx, fsy, e);
        sx = fsx; sy = fsy; dx = e.x; dy = e.y;
    }
    const double* Hp = hyps + (long long)pair * iters * 9;
    for (int h = 0; h < iters; h++) {
        const double* H = Hp + 9 * h;                 // uniform: scalar loads
        const double nx = H[0] * sx + H[1] * sy + H[2];
        const double nyv = H[3] * sx + H[4] * sy + H[5];
        const double dd = H[6] * sx + H[7] * sy + H[8];
        const double ex = nx - dx * dd, ey = nyv - dy * dd;
        const bool in = acc && ex * ex + ey * ey <= t2 * (dd * dd);
        const unsigned long long bal = __ballot(in);
        if (lane == 0 && bal) atomicAdd(&s_cnt[h], __popcll(bal));
    }
    __syncthreads();
    for (int h = tid; h < iters; h += 256)
        if (s_cnt[h]) atomicAdd(&counts[(long long)pair * iters + h], s_cnt[h]);
}

__global__ __launch_bounds__(64) void k_ransac_pick(const double* __restrict__ hyps, const int* __restrict__ counts,
                                                    int iters, PairFit* __restrict__ fits)
{
    const int pair = blockIdx.x, lane = threadIdx.x;
    PairFit& f = fits[pair];
    if (f.fit_status != 0 || f.num_vectors < 4) return;
    int bc = -1, bh = 0;
    for (int h = lane; h < iters; h += 64) {
        const int cnt = counts[(long long)pair * iters + h];
        if (cnt > bc) { bc = cnt; bh = h; }            // first max of this lane's (increasing) h
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const int oc = __shfl_xor(bc, m), oh = __shfl_xor(bh, m);
        if (oc > bc || (oc == bc && oh < bh)) { bc = oc; bh = oh; }
    }
    if (lane != 0) return;
    for (int k = 0; k < 9; k++) f.H[k] = hyps[((long long)pair * iters + bh) * 9 + k];
    dev_invert3x3(f.H, f.Hinv);
}

// Row-band mode: the same block scan as k_fit, but the band's count and first four accepted
// points go to its record (the fit waits for every band's record, k_band_fit).
__global__ __launch_bounds__(64) void k_band_record(const float* __restrict__ next_pts, int npts, int ny, int pixel_step,
                                                    const BlockSummary* __restrict__ summ, int nblk,
                                                    mdx_band_cand* __restrict__ cand)
{
    const int pair = blockIdx.x, lane = threadIdx.x;
    const BlockSummary* S = summ + (long long)pair * nblk;
    int carry = 0;
    int pick[4] = {-1, -1, -1, -1};
    for (int b0 = 0; b0 < nblk; b0 += 64) {
        const int b = b0 + lane;
        const int cnt = b < nblk ? S[b].count : 0;
        int incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        const int excl = carry + incl - cnt;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const bool here = cnt > 0 && r >= excl && r < excl + cnt;
            const unsigned long long m = __ballot(here);
            if (m) {
                const int src = __ffsll((long long)m) - 1;
                const int v = here ? S[b].first[r - excl] : 0;
                const int got = __shfl(v, src);
                if (pick[r] < 0) pick[r] = got;
            }
        }
        carry += __shfl(incl, 63);
    }
    if (lane != 0) return;
    mdx_band_cand& c = cand[pair];
    c.count = carry;
    c.n = carry < 4 ? carry : 4;
    for (int r = 0; r < 4; r++) {
        const int i = r < c.n ? pick[r] : -1;
        c.idx[r] = i;
        if (i >= 0) {
            c.src[2 * r] = (float)((i / ny) * pixel_step);
            c.src[2 * r + 1] = (float)((i % ny) * pixel_step);
            const float2 e = reinterpret_cast<const float2*>(next_pts)[(long long)pair * npts + i];
            c.dst[2 * r] = e.x;
            c.dst[2 * r + 1] = e.y;
        } else {
            c.src[2 * r] = c.src[2 * r + 1] = c.dst[2 * r] = c.dst[2 * r + 1] = 0.f;
        }
    }
    c.pad_[0] = c.pad_[1] = 0;
}

// Merge the bands' records: the four smallest indices over all records are the frame's first four
// accepted points (each band lists its own first four, and bands partition the points), so the
// fit below is bit-identical to the full path's k_fit.
// Frame-1 rows the warp of destination rows [y0, y1) reads: under M (= Hinv) a rectangle whose
// corners all have W of one sign maps to the convex quadrilateral of the corners' images, so
// their Y bound the source rows (+-2 for the reference's 1/32-px rounding and the lower tap);
// otherwise every row.  M all zero (singular fit): the constant warp reads row 0 (and 1).
__device__ void band_source_rows(const double* M, int w, int h, int y0, int y1, int& r0, int& r1)
{
    bool zero = true;
    for (int k = 0; k < 9; k++) zero = zero && M[k] == 0.0;
    r0 = 0;
    r1 = h;
    if (zero) {
        r1 = min(h, 2);
        return;
    }
    double ymin = 0.0, ymax = 0.0;
    int sgn = 0;
    for (int q = 0; q < 4; q++) {
        const double x = (q & 1) ? (double)(w - 1) : 0.0, y = (q & 2) ? (double)(y1 - 1) : (double)y0;
        const double W = M[6] * x + M[7] * y + M[8];
        const int sq = W > 0.0 ? 1 : W < 0.0 ? -1 : 0;
        if (sq == 0 || (q && sq != sgn)) return;
        sgn = sq;
        const double Y = (M[3] * x + M[4] * y + M[5]) / W;
        if (!(Y == Y) || __builtin_isinf(Y)) return;
        ymin = q ? fmin(ymin, Y) : Y;
        ymax = q ? fmax(ymax, Y) : Y;
    }
    if (ymax < -4.0 || ymin > (double)h + 4.0) {   // footprint outside the frame: nothing to read
        r0 = r1 = 0;
        return;
    }
    r0 = (int)fmax(0.0, floor(ymin) - 2.0);
    r1 = (int)fmin((double)h, floor(ymax) + 3.0);
    if (r1 < r0) r1 = r0;
}

__global__ __launch_bounds__(64) void k_band_fit(const mdx_band_cand* __restrict__ cands, int nrec,
                                                 PairFit* __restrict__ fit, int w, int h, int y0, int y1)
{
    // every lane merges the records (uniform loads), the wave runs the fit, lane 0 writes
    int total = 0;
    int best[4] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX};
    float bs[8] = {}, bd[8] = {};
    for (int r = 0; r < nrec; r++) {
        const mdx_band_cand& c = cands[r];
        total += c.count;
        for (int q = 0; q < c.n && q < 4; q++) {
            int i = c.idx[q];
            float sx = c.src[2 * q], sy = c.src[2 * q + 1], dx = c.dst[2 * q], dy = c.dst[2 * q + 1];
            for (int k = 0; k < 4; k++) {   // insertion into the sorted four
                if (i < best[k]) {
                    const int ti = best[k];
                    const float t0 = bs[2 * k], t1 = bs[2 * k + 1], t2 = bd[2 * k], t3 = bd[2 * k + 1];
                    best[k] = i; bs[2 * k] = sx; bs[2 * k + 1] = sy; bd[2 * k] = dx; bd[2 * k + 1] = dy;
                    i = ti; sx = t0; sy = t1; dx = t2; dy = t3;
                }
            }
        }
    }
    PairFit& f = *fit;
    __shared__ double fw[kFitWaveDoubles];
    if (total >= 4) {
        double H[9];
        dev_perspective_fit_wave(bs, bd, H, fw);
        if (threadIdx.x != 0) return;
        f.num_vectors = total;
        for (int k = 0; k < 9; k++) f.H[k] = H[k];
        dev_invert3x3(H, f.Hinv);
        f.fit_status = 0;
        band_source_rows(f.Hinv, w, h, y0, y1, f.src_y0, f.src_y1);
    } else {
        if (threadIdx.x != 0) return;
        f.num_vectors = total;
        for (int k = 0; k < 9; k++) { f.H[k] = 0.0; f.Hinv[k] = 0.0; }
        f.fit_status = total == 0 ? 1 : 2;
        f.src_y0 = f.src_y1 = 0;   // no warp (zero mask)
    }
}

// Rows [fit->src_y0, fit->src_y1) of frame 1 -> gray, into the padded level-0 core (what k_front
// writes there): block (bx, by) converts 256 columns of rows src_y0 + by, + gridDim.y, ...
__global__ __launch_bounds__(64) void k_gray_rows(const uint8_t* __restrict__ img1, int w, int stride, int fmt,
                                                  uint8_t* __restrict__ g, int pitch, const PairFit* __restrict__ fit,
                                                  int built0, int built1)
{
    const int r0 = fit->src_y0, r1 = fit->src_y1;
    const int x = (blockIdx.x * 64 + threadIdx.x) * 4;
    if (x >= w) return;
    for (int y = r0 + (int)blockIdx.y; y < r1; y += gridDim.y) {
        if (y >= built0 && y < built1) continue;   // the band's flow built these rows

        const uint8_t* sp = img1 + (long long)y * stride;
        uint8_t* dp = g + (long long)y * pitch + x;
        const int n = min(4, w - x);
        uint32_t d = 0;
        for (int i = 0; i < n; i++) {
            const int v = fmt == 0 ? sp[x + i] : gray_of(sp + 3 * (x + i), fmt);
            d |= (uint32_t)v << (8 * i);
        }
        if (n == 4) *reinterpret_cast<uint32_t*>(dp) = d;   // x and the core are 4-B aligned
        else for (int i = 0; i < n; i++) dp[i] = (uint8_t)(d >> (8 * i));
    }
}

hipError_t launch_gray_rows(hipStream_t s, const uint8_t* img1, int w, int h, int stride, int fmt, uint8_t* gray1_l0,
                            int pitch, const PairFit* fit, int built0, int built1)
{
    (void)h;
    const dim3 grid((w + 255) / 256, 64);
    hipLaunchKernelGGL(k_gray_rows, grid, dim3(64), 0, s, img1, w, stride, fmt, gray1_l0, pitch, fit, built0, built1);
    return hipGetLastError();
}

__global__ void k_set_fit_external(const double* __restrict__ H_ext, PairFit* __restrict__ fits, int batch)
{
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= batch) return;
    PairFit& f = fits[pair];
    for (int k = 0; k < 9; k++) f.H[k] = H_ext[(long long)pair * 9 + k];
    dev_invert3x3(f.H, f.Hinv);
    f.num_vectors = 0;
    f.fit_status = 0;
}

__global__ void k_export_fit(const PairFit* __restrict__ fits, int batch, double* H, int* num)
{
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= batch) return;
    if (H) for (int k = 0; k < 9; k++) H[(long long)pair * 9 + k] = fits[pair].H[k];
    if (num) num[pair] = fits[pair].num_vectors;
}

// A8-A10 (warp + absdiff + threshold) lives in mdx_warp.hip.

// ------------------------------------------------------------------ launchers
// last 16-B chunk index of a padded row (columns -40 .. w+39 at row bytes 24 .. 64+w+39)
static inline int last_chunk16(int w) { return (kXOff + w + kPad - 1) / 16; }

hipError_t launch_gray_pad(hipStream_t s, int batch, const uint8_t* in1, const uint8_t* in2, int w, int h, int stride,
                           long long frame_stride, int fmt, uint8_t* pyr1, uint8_t* pyr2, const Geometry& g, int fsel)
{
    const int nchunk = last_chunk16(w);
    const dim3 grid((nchunk + 127) / 128, h + 2 * kPad, fsel ? batch : 2 * batch);   // two chunks per thread
    hipLaunchKernelGGL(k_gray_pad, grid, dim3(64), 0, s, in1, in2, w, h, stride, frame_stride, fmt, pyr1, pyr2,
                       g.img_bytes, g.lv[0], nchunk, fsel);
    return hipGetLastError();
}

// k_front's band height: 4 destination rows at 1080p (27 KB of LDS, 5-6 bands per CU): one frame
// side of gray + pad + level 1 takes 44 us there against 56 with 8 rows and 107 for the earlier
// k_gray_pad + k_pyrdown (scripts/micro/front_bench.hip).
static hipError_t launch_front_bands(hipStream_t s, FrontArgs& a, int mode, int rlo = 0, int rhi = -1)
{
    // the band height: 4 destination rows while a band's LDS fits 32 KB, else 2 (8K frames: 62 KB),
    // else 1; beyond 64 KB (rows wider than ~8.7K px at RB = 1) the launch asks for the larger
    // dynamic LDS explicitly (up to the CU's 160 KB)
    auto lds_of = [&](int rb) { return (size_t)(2 * rb + 3) * a.lp + (size_t)rb * a.lp1; };
    int rb = lds_of(4) <= 32 * 1024 ? 4 : lds_of(2) <= 64 * 1024 ? 2 : 1;
    // a single frame (the live ring's push): 4-row bands are a few hundred workgroups, under two
    // per CU; one-row bands re-read more source rows (5 per destination row against 2.75) but
    // spread the frame over the chip
    if (rb == 4 && (long long)a.nz * ((a.L1.h + 3) / 4) < 512) rb = 1;
    const size_t lds = lds_of(rb);
    // k_front's static arrays (out0, out1, nout) share the CU's 160 KB with the dynamic rows
    const size_t lds_static = (size_t)(2 * rb + 80 + rb + 80 + 2) * sizeof(int);
    if (lds + lds_static > 160 * 1024) return hipErrorInvalidValue;   // rows wider than ~31K px
    // destination rows [rlo, rhi) of the level built (all by default): the bands covering them
    if (rhi < 0 || rhi > a.L1.h) rhi = a.L1.h;
    rlo = std::max(0, std::min(rlo, rhi));
    a.band0 = rlo / rb;
    a.nbands = (rhi + rb - 1) / rb - a.band0;
    if (a.nbands <= 0) return hipSuccess;
    const dim3 grid((unsigned)(a.nbands * a.nz));
#define MDX_FRONT_CASE(M, R)                                                                             \
    if (mode == M && rb == R) {                                                                          \
        if (lds + lds_static > 64 * 1024)                                                                \
            if (hipError_t e = hipFuncSetAttribute((const void*)k_front<R, M>,                           \
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) \
                return e;                                                                                \
        hipLaunchKernelGGL((k_front<R, M>), grid, dim3(256), lds, s, a);                                 \
    }
    MDX_FRONT_CASE(0, 4) MDX_FRONT_CASE(0, 2) MDX_FRONT_CASE(0, 1)
    MDX_FRONT_CASE(1, 4) MDX_FRONT_CASE(1, 2) MDX_FRONT_CASE(1, 1)
    MDX_FRONT_CASE(2, 4) MDX_FRONT_CASE(2, 2) MDX_FRONT_CASE(2, 1)
#undef MDX_FRONT_CASE
    return hipGetLastError();
}

static FrontArgs front_args(int batch, uint8_t* pyr1, uint8_t* pyr2, const Geometry& g, int src_level, int fsel)
{
    FrontArgs a{};
    a.fsel = fsel;
    a.img_bytes = g.img_bytes;
    a.pyr1 = pyr1;
    a.pyr2 = pyr2;
    a.L0 = g.lv[src_level];
    a.L1 = g.lv[src_level + 1];
    a.w = a.L0.w;
    a.h = a.L0.h;
    a.nchunk0 = last_chunk16(a.L0.w);
    a.nchunk1_16 = last_chunk16(a.L1.w);
    a.lp = 16 * (a.nchunk0 + 1);
    a.lp1 = 16 * (a.nchunk1_16 + 1);
    a.nz = fsel ? batch : 2 * batch;
    return a;
}

hipError_t launch_front(hipStream_t s, int batch, const uint8_t* in1, const uint8_t* in2, int w, int h, int stride,
                        long long frame_stride, int fmt, uint8_t* pyr1, uint8_t* pyr2, const Geometry& g, int fsel,
                        const RowSpan* rows)
{
    if (g.nlev < 2) return launch_gray_pad(s, batch, in1, in2, w, h, stride, frame_stride, fmt, pyr1, pyr2, g, fsel);
    FrontArgs a = front_args(batch, pyr1, pyr2, g, 0, fsel);
    a.in1 = in1;
    a.in2 = in2;
    a.stride = stride;
    a.fmt = fmt;
    a.frame_stride = frame_stride;
    a.aligned = ((((uintptr_t)in1 | (uintptr_t)in2) & 3) == 0 && (stride & 3) == 0 && (frame_stride & 3) == 0) ? 1 : 0;
    // level-1 rows: those wanted at level 1 and those whose bands write the wanted level-0 rows
    int r1lo = 0, r1hi = -1;
    if (rows) {
        r1lo = std::min(rows[1].lo, rows[0].lo / 2);
        r1hi = std::max(rows[1].hi, (rows[0].hi + 1) / 2);
    }
    return launch_front_bands(s, a, fmt == MDX_FMT_GRAY8 ? 0 : 1, r1lo, r1hi);
}

hipError_t launch_pyr_levels(hipStream_t s, int batch, uint8_t* pyr1, uint8_t* pyr2, const Geometry& g, int fsel,
                             const RowSpan* rows)
{
    for (int l = 2; l < g.nlev; l++) {
        FrontArgs a = front_args(batch, pyr1, pyr2, g, l - 1, fsel);
        if (hipError_t e = launch_front_bands(s, a, 2, rows ? rows[l].lo : 0, rows ? rows[l].hi : -1)) return e;
    }
    return hipSuccess;
}

// Every level's Scharr planes in one launch (blockIdx.y runs over the levels' padded rows, level by
// level): the live ring's push builds one frame's five levels, whose launches are each a few
// microseconds of mostly launch overhead.
struct ScharrLevels {
    Level L[kMaxLevels];
    int nchunk[kMaxLevels];
    int row0[kMaxLevels + 1];   // first blockIdx.y of each level
    int nlev;
};
__global__ __launch_bounds__(256) void k_scharr_levels(const uint8_t* __restrict__ pyr1, uint32_t* __restrict__ der,
                                                       long long img_bytes, long long der_words, ScharrLevels sl)
{
    int l = 0;
    while (l + 1 < sl.nlev && (int)blockIdx.y >= sl.row0[l + 1]) l++;
    const Level L = sl.L[l];
    const int nchunk = sl.nchunk[l];
    const int pair = blockIdx.z;
    const int c = blockIdx.x * blockDim.x + threadIdx.x + 4;         // word chunks 0..3 are margin
    const int py = (int)blockIdx.y - sl.row0[l] - kPad;
    if (c > nchunk) return;
    const int px0 = 4 * c - kXOff;
    uint32_t o[4] = {0, 0, 0, 0};
    if (py >= 0 && py < L.h && px0 + 4 > 0 && px0 < L.w) {
        const uint8_t* s = pyr1 + (long long)pair * img_bytes + L.img_off + L.core() + (long long)py * L.pitch + px0 - 4;
        const int p = L.pitch;
        uint32_t rw[3][3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const u3a4k v = *reinterpret_cast<const u3a4k*>(s + (long long)(r - 1) * p);
            rw[r][0] = v.x; rw[r][1] = v.y; rw[r][2] = v.z;
        }
        auto B = [&](int r, int b) -> int { return (int)((rw[r][b >> 2] >> (8 * (b & 3))) & 255u); };
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int px = px0 + i;
            if (px < 0 || px >= L.w) continue;
            const int bm = 3 + i, bc = 4 + i, bp = 5 + i;               // bytes x-1, x, x+1
            const int t0m = (B(0, bm) + B(2, bm)) * 3 + B(1, bm) * 10;
            const int t0p = (B(0, bp) + B(2, bp)) * 3 + B(1, bp) * 10;
            const int t1m = B(2, bm) - B(0, bm), t1c = B(2, bc) - B(0, bc), t1p = B(2, bp) - B(0, bp);
            const int ix = t0p - t0m;
            const int iy = (t1m + t1p) * 3 + t1c * 10;
            o[i] = (uint32_t)(uint16_t)(int16_t)ix | ((uint32_t)(uint16_t)(int16_t)iy << 16);
        }
    }
    uint32_t* row = der + (long long)pair * der_words + L.der_off + (long long)(py + kPad) * L.pitch;
    *reinterpret_cast<uint4*>(row + 4 * c) = make_uint4(o[0], o[1], o[2], o[3]);
}

hipError_t launch_scharr_levels(hipStream_t s, int batch, const uint8_t* pyr1, uint32_t* der, const Geometry& g)
{
    ScharrLevels sl{};
    sl.nlev = g.nlev;
    int rows = 0, maxc = 0;
    for (int l = 0; l < g.nlev; l++) {
        sl.L[l] = g.lv[l];
        sl.nchunk[l] = (kXOff + g.lv[l].w + kPad - 1) / 4;
        sl.row0[l] = rows;
        rows += g.lv[l].rows;
        maxc = std::max(maxc, sl.nchunk[l]);
    }
    sl.row0[g.nlev] = rows;
    if (rows == 0) return hipSuccess;
    const dim3 grid((maxc - 4 + 1 + 63) / 64, rows, batch);
    hipLaunchKernelGGL(k_scharr_levels, grid, dim3(64), 0, s, pyr1, der, g.img_bytes, g.der_words, sl);
    return hipGetLastError();
}

hipError_t launch_scharr(hipStream_t s, int batch, const uint8_t* pyr1, uint32_t* der, const Geometry& g, int level,
                         int prow0, int prow1)
{
    const Level& L = g.lv[level];
    const int nchunk = (kXOff + L.w + kPad - 1) / 4;                 // last 4-word chunk
    if (prow1 < 0 || prow1 > L.rows) prow1 = L.rows;
    prow0 = std::max(0, std::min(prow0, prow1));
    if (prow1 == prow0) return hipSuccess;
    const dim3 grid((nchunk - 4 + 1 + 63) / 64, prow1 - prow0, batch);
    hipLaunchKernelGGL(k_scharr, grid, dim3(64), 0, s, pyr1, der, g.img_bytes, g.der_words, L, nchunk, prow0);
    return hipGetLastError();
}

// ------------------------------------------------------------ trajectory tracking
// OpticalFlowCalculator::calculateOpticalFlowTrajectory (optical_flow_calculator.cpp:133-257).
// init: points = the grid (:148-158, x-major), every trajectory = its grid point.
__global__ void k_traj_init(int npts, int ny, int pixel_step, int nimg, float* __restrict__ cur,
                            float* __restrict__ traj, int* __restrict__ tlen, int* __restrict__ num,
                            int* __restrict__ flag)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        num[0] = 0;
        if (flag) num[1] = 0;   // chain mode: hand-off timeouts
    }
    if (i >= npts) return;
    if (flag) flag[i] = 0;
    const float x = (float)((i / ny) * pixel_step), y = (float)((i % ny) * pixel_step);
    cur[2 * i] = x;
    cur[2 * i + 1] = y;
    traj[(long long)i * nimg * 2] = x;
    traj[(long long)i * nimg * 2 + 1] = y;
    for (int k = 2; k < 2 * nimg; k++) traj[(long long)i * nimg * 2 + k] = 0.f;   // entries past traj_len: 0
    tlen[i] = 1;
}

// One pass j -> j+1 (:178-242): a tracked point moves (and its trajectory grows) only when it lands
// strictly inside the 10-px border; lost or border points stay.  On the last pass the Vec4d of
// :183-206 / :220-230 per point and num_vectors (order-free integer count).
__global__ void k_traj_update(int npts, const float* __restrict__ next_pts, const uint8_t* __restrict__ status,
                              float* __restrict__ cur, float* __restrict__ traj, int* __restrict__ tlen, int nimg, int w,
                              int h, int last, double min_vector_size, double* __restrict__ vectors,
                              float* __restrict__ start_pts, int* __restrict__ num)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npts) return;
    const float sx = cur[2 * i], sy = cur[2 * i + 1];
    double* v = (last && vectors) ? vectors + 4LL * i : nullptr;
    if (last && start_pts) {
        start_pts[2 * i] = sx;
        start_pts[2 * i + 1] = sy;
    }
    if (status[i]) {
        const float ex = next_pts[2 * i], ey = next_pts[2 * i + 1];
        if (last) {
            const float xd = ex - sx, yd = ey - sy;
            if (fabs((double)fabsf(xd)) > min_vector_size || fabs((double)fabsf(yd)) > min_vector_size) {
                if (v) { v[0] = sx; v[1] = sy; v[2] = xd; v[3] = yd; }
                atomicAdd(num, 1);
            } else if (v) {
                v[0] = sx; v[1] = sy; v[2] = 0.0; v[3] = 0.0;
            }
        }
        if (ex > 10.0f && ey > 10.0f && ex < (float)(w - 10) && ey < (float)(h - 10)) {
            cur[2 * i] = ex;
            cur[2 * i + 1] = ey;
            const int l = tlen[i];
            traj[((long long)i * nimg + l) * 2] = ex;
            traj[((long long)i * nimg + l) * 2 + 1] = ey;
            tlen[i] = l + 1;
        }
    } else if (v) {
        v[0] = -1.0; v[1] = -1.0; v[2] = 0.0; v[3] = 0.0;
    }
}

hipError_t launch_traj_init(hipStream_t s, int npts, int ny, int pixel_step, int nimg, float* cur, float* traj,
                            int* tlen, int* num, int* flag)
{
    hipLaunchKernelGGL(k_traj_init, dim3((npts + 255) / 256 > 0 ? (npts + 255) / 256 : 1), dim3(256), 0, s, npts, ny,
                       pixel_step, nimg, cur, traj, tlen, num, flag);
    return hipGetLastError();
}

hipError_t launch_lk_chain(hipStream_t s, const LkArgs& a, const TrajChain& t, int ppw)
{
    const long long blocks = (long long)(t.nimg - 1) * ((a.npts + ppw - 1) / ppw);
    if (t.nimg < 2 || t.nimg > kMaxTrajImgs || a.npts <= 0 || blocks > 0x7fffffffLL || (ppw != 1 && ppw != 2 && ppw != 4))
        return hipErrorInvalidValue;
    if (ppw == 4) hipLaunchKernelGGL((k_lk<16, true>), dim3((unsigned)blocks), dim3(64), 0, s, a, t);
    else if (ppw == 2) hipLaunchKernelGGL((k_lk<32, true>), dim3((unsigned)blocks), dim3(64), 0, s, a, t);
    else hipLaunchKernelGGL((k_lk<64, true>), dim3((unsigned)blocks), dim3(64), 0, s, a, t);
    return hipGetLastError();
}

hipError_t launch_traj_update(hipStream_t s, int npts, const float* next_pts, const uint8_t* status, float* cur,
                              float* traj, int* tlen, int nimg, int w, int h, int last, double min_vector_size,
                              double* vectors, float* start_pts, int* num)
{
    if (npts <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_traj_update, dim3((npts + 255) / 256), dim3(256), 0, s, npts, next_pts, status, cur, traj,
                       tlen, nimg, w, h, last, min_vector_size, vectors, start_pts, num);
    return hipGetLastError();
}

hipError_t launch_lk(hipStream_t s, int batch, const LkArgs& a)
{
    // one point per wave: 124 VGPRs, 4 waves per SIMD (two points per wave took 172 VGPRs, 2 waves
    // per SIMD, and ran the trajectory passes 1.5x slower)
    constexpr int LPP = 64, PPW = 64 / LPP;
    const dim3 grid((a.npts + PPW - 1) / PPW, batch);
    hipLaunchKernelGGL((k_lk<LPP, false>), grid, dim3(64), 0, s, a, TrajChain{});
    return hipGetLastError();
}

hipError_t launch_classify_fit(hipStream_t s, int batch, const float* next_pts, const uint8_t* status, int npts,
                               int ny, int gy0, int gy1, int pixel_step, double mvs, double* vectors, PairFit* fits,
                               int fit_mode, const double* H_external, void* scratch, mdx_band_cand* cand,
                               const RansacArgs* ransac)
{
    const int nblk = (npts + 255) / 256;
    BlockSummary* summ = reinterpret_cast<BlockSummary*>(scratch);
    if (nblk > 0)
        hipLaunchKernelGGL(k_classify, dim3(nblk, batch), dim3(256), 0, s, next_pts, status, npts, ny, gy0, gy1,
                           pixel_step, mvs, vectors, summ);
    if (cand)
        hipLaunchKernelGGL(k_band_record, dim3(batch), dim3(64), 0, s, next_pts, npts, ny, pixel_step, summ, nblk, cand);
    else
        hipLaunchKernelGGL(k_fit, dim3(batch), dim3(64), 0, s, next_pts, npts, ny, pixel_step, summ, nblk, fits,
                           fit_mode, H_external);
    if (fit_mode == MDX_FIT_RANSAC && !cand) {
        if (!ransac || nblk == 0 || ransac->iters < 1 || ransac->iters > kRansacMaxIters) return hipErrorInvalidValue;
        const RansacArgs& r = *ransac;
        hipLaunchKernelGGL(k_ransac_compact, dim3(nblk, batch), dim3(256), 0, s, next_pts, status, npts, ny, pixel_step,
                           mvs, summ, r.list);
        hipLaunchKernelGGL(k_ransac_hyp, dim3((r.iters + kRansacLanes - 1) / kRansacLanes, batch), dim3(64), 0, s,
                           next_pts, npts, ny, pixel_step, r.list, fits, r.iters, r.seed, r.hyps, r.counts);
        hipLaunchKernelGGL(k_ransac_score, dim3(nblk, batch), dim3(256), 0, s, next_pts, status, npts, ny, pixel_step,
                           mvs, r.hyps, r.iters, r.thresh * r.thresh, fits, r.counts);
        hipLaunchKernelGGL(k_ransac_pick, dim3(batch), dim3(64), 0, s, r.hyps, r.counts, r.iters, fits);
    }
    return hipGetLastError();
}

hipError_t launch_band_fit(hipStream_t s, int nrec, const mdx_band_cand* cands, PairFit* fit, int w, int h, int y0,
                           int y1)
{
    hipLaunchKernelGGL(k_band_fit, dim3(1), dim3(64), 0, s, cands, nrec, fit, w, h, y0, y1);
    return hipGetLastError();
}

hipError_t launch_set_fit_external(hipStream_t s, int batch, const double* H_external, PairFit* fits)
{
    hipLaunchKernelGGL(k_set_fit_external, dim3((batch + 63) / 64), dim3(64), 0, s, H_external, fits, batch);
    return hipGetLastError();
}

hipError_t launch_export_fit(hipStream_t s, int batch, const PairFit* fits, double* H, int* num)
{
    hipLaunchKernelGGL(k_export_fit, dim3((batch + 63) / 64), dim3(64), 0, s, fits, batch, H, num);
    return hipGetLastError();
}

}  // namespace mdx
