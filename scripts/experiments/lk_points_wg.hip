// EXPERIMENT (not built; measured slower than k_lk).  Was
// motion_detection_amd/csrc/mdx_lkpt.hip, launched instead of k_lk with MDX_LK_PTS=1; bit-exact in
// tests/test_trajectory.py and tests/test_ring.py.  Live callback (5 x 1080p rgb8, ring): k_lk 3.96 ms;
// this kernel 7.40 (8 points / 512 lanes), 5.85 (4 / 256), 6.38 (2 / 128) ms: the chain-summing wave's
// barriers leave the SIMDs waiting (SQ_WAIT_ANY 72% of wave cycles, VALU 41% busy vs k_lk's 97%).
//
// mdx_lkpt.hip -- pyramidal Lucas-Kanade for arbitrary start points (reference row A5 as run by
// calculateOpticalFlowTrajectory, optical_flow_calculator.cpp:172, on the points the previous pass
// left: the node's live chain, motion_detection_node.cpp:94-110; also sparse grids whose class
// planes would not pay).  Same arithmetic as mdx_lk.hip, bit for bit: OpenCV 2.4's x86 SSE2
// LKTrackerInvoker -- 14-bit fixed-point bilinear weights (cvRound, half-even), window descales,
// float sums in four interleaved chains (lane k: window columns 4g+k, rows in order), combined as
// A: ((P0+P1)+P2)+P3 and b: (P0+P2)+(P1+P3), minEig/(2*1600), eps^2 in double, the oscillation
// half-step, and the err pass's final bounds check.  Nothing is fused into an FMA
// (-ffp-contract=off) except products that are exact in float.
//
// Why a second kernel.  The class-plane LK shares one interpolation per fractional class among
// the grid points; a trajectory point sits anywhere, so its window (I*32, Ix, Iy at the point's own
// weights) is interpolated per point, and its sums are four strictly ordered float chains.  One
// point per wave (k_lk) leaves 56 of 64 lanes idle while the chains are summed (400 dependent adds
// per Newton step).  Here a 512-lane workgroup tracks NP = 8 points:
//  * products: each point owns 64 lanes, each lane 25 window elements (5 per 8-row chunk), whose
//    interpolated values stay in registers for the level; per chunk the lanes write their
//    products chain-ordered to LDS;
//  * sums: one wave adds the chunk's 80 products of every chain of all 8 points in one instruction
//    stream (the b chains of all points with one v_pk_add_f32 per product), taking the partial
//    sums over from the previous chunk's wave through LDS; the chunks rotate over the 8 waves, so
//    one wave sums while the others compute the next chunk's products (double-buffered);
//  * J: per Newton step the 8 moving 41 x 41 windows are staged byte-aligned in LDS (3 x 16-B
//    loads + v_alignbyte per row), so a lane reads each tap pair with one 8-byte LDS access and one
//    v_perm, its byte position fixed by its lane (x & 3 == lane & 3).
#include "mdx_internal.h"

#include <float.h>

namespace mdx {

namespace {

typedef short s2p __attribute__((ext_vector_type(2)));
typedef float f2p __attribute__((ext_vector_type(2)));

#ifndef LKPT_NP
#define LKPT_NP 4
#endif
#ifndef LKPT_W
#define LKPT_W 4                       // waves per SIMD the register budget is sized for
#endif
constexpr int kNP = LKPT_NP;           // points per workgroup (one wave each)
constexpr int kWG = 64 * kNP;          // lanes per workgroup
constexpr int kTPP = kWG / kNP;        // lanes per point (64)
constexpr int kRC = 8;                 // window rows per chunk
constexpr int kNCH = kWin / kRC;       // chunks (5)
constexpr int kEPC = kRC * kWin / kTPP;   // elements per lane and chunk (5)
constexpr int kNE = kNCH * kEPC;       // elements per lane (25)
constexpr int kPOS = kRC * kWin / 4;   // chain positions per chunk (80)
// chain strides padded to 4 x odd dwords: the summing wave's lanes (one chain each) then read
// their 16-B pieces from distinct banks (an unpadded f2p chain of 160 dwords put 32 lanes on 2 banks)
constexpr int kPS2 = kPOS + 2;         // f2p chain stride (164 dwords)
constexpr int kPS1 = kPOS + 4;         // float chain stride (84 dwords)
constexpr int kJW = 12;                // dwords per staged J row (44 bytes used)

struct __attribute__((aligned(4))) u4al { uint32_t x, y, z, w; };
typedef __attribute__((address_space(3))) const uint32_t* lcu;
typedef __attribute__((address_space(3))) f2p* lf2;
typedef __attribute__((address_space(3))) float* lfl;

__device__ __forceinline__ void lkpt_weights(float fa, float fb, int& w00, int& w01, int& w10, int& w11)
{
    w00 = __float2int_rn((1.f - fa) * (1.f - fb) * 16384.f);
    w01 = __float2int_rn(fa * (1.f - fb) * 16384.f);
    w10 = __float2int_rn((1.f - fa) * fb * 16384.f);
    w11 = 16384 - w00 - w01 - w10;
}

struct LkPtShared {
    // chain-ordered products of one chunk, double-buffered: (b1, b2) or (Ix*Ix, Iy*Iy) per element
    f2p pab[2][kNP][4][kPS2];
    union {
        float p12[2][kNP][4][kPS1];                   // A phase: Ix*Iy
        uint32_t jwin[kNP][kWin + 1][kJW];           // Newton steps: the J windows, byte-aligned
    } u;
    f2p acc2[kNP][4];                                 // running (A11, A22) / (b1, b2) per chain
    float acc1[kNP][4];                               // running A12 per chain
    int4 jpos[kNP];                                   // per point: inx, iny, active
    int anyact;
};

}  // namespace

// grid: x -> 8 consecutive points, y -> pair.  Start points from a.prev_pts (trajectory passes,
// flags 0: nextPt = prevPt) or the pixel_step grid.
__global__ __launch_bounds__(64 * LKPT_NP, LKPT_W) void k_lk_pts(LkArgs a)
{
    constexpr float HALFW = 19.5f;             // (winSize.width-1)*0.5f
    constexpr float FLT_SCALE = 1.f / (1 << 20);
    __shared__ LkPtShared sh;

    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int i = t / kTPP, s = t % kTPP;      // this lane's point and its rank among the point's lanes
    const int pt = blockIdx.x * kNP + i;
    const int pair = blockIdx.y;
    const bool valid = pt < a.npts;

    // element m of a chunk (8 window rows x 40 columns, 5 per lane): m < 4 -> row 2m + (s >> 5),
    // column s & 31; m == 4 -> row s >> 3, column 32 + (s & 7).  Every element's chain
    // (column & 3) is s & 3, so its LDS positions are a per-lane base plus a constant.
    auto ey = [&](int m) { return m < 4 ? 2 * m + (s >> 5) : (s >> 3); };
    auto ex = [&](int m) { return m < 4 ? (s & 31) : 32 + (s & 7); };
    const int kq = s & 3;
    // J tap pair (x, x+1) of a staged row: bytes (x & 3), (x & 3) + 1 of the dword pair at x & ~3
    const unsigned jsel = (unsigned)kq | 0x0c00u | ((unsigned)(kq + 1) << 16) | 0x0c000000u;

    float px0 = 0.f, py0 = 0.f;
    if (valid) {
        if (a.prev_pts) {
            const float* pp = a.prev_pts + ((long long)pair * a.npts + pt) * 2;
            px0 = pp[0];
            py0 = pp[1];
        } else {
            px0 = (float)((pt / a.ny) * a.pixel_step);
            py0 = (float)((pt % a.ny) * a.pixel_step);
        }
    }
    float npx = 0.f, npy = 0.f;
    int status = 1;

    uint32_t sd[kNE];                  // (Ix & 0xffff) | Iy << 16 of each element
    uint32_t si[(kNE + 1) / 2];        // I*32 (descaled), two per word

    const uint8_t* slab1 = a.pyr1 + (long long)pair * a.g.img_bytes;
    const uint8_t* slab2 = a.pyr2 + (long long)pair * a.g.img_bytes;
    const uint32_t* dslab = a.der + (long long)pair * a.g.der_words;

    // the summing lanes of a wave: lane = point * 8 + chain slot; the summing wave of chunk c is
    // (c + rot) & 7, rot advancing by one phase's chunks, so the 8 waves take turns
    const int sp = lane >> 3, sq = lane & 7;
    int rot = 0;

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
        bool ok = valid && !(ipx < -kWin || ipx >= L.w || ipy < -kWin || ipy >= L.h);
        if (valid && !ok && level == 0) status = 0;
        int w00 = 0, w01 = 0, w10 = 0, w11 = 0;
        if (ok) lkpt_weights(ppx - (float)ipx, ppy - (float)ipy, w00, w01, w10, w11);
        const int ibase = ipy * pitch + ipx;
        // LDS element bases of this lane (m < 4 / m == 4), opaque so that the compiler derives every
        // element's address as base + constant instead of hoisting 50 addresses into registers
        const int pos0 = (s >> 5) * 10 + ((s & 31) >> 2), pos4 = (s >> 3) * 10 + 8 + ((s & 7) >> 2);
        uint32_t pa0 = (uint32_t)(uintptr_t)&sh.pab[0][i][kq][pos0];
        uint32_t pa4 = (uint32_t)(uintptr_t)&sh.pab[0][i][kq][pos4];
        uint32_t pc0 = (uint32_t)(uintptr_t)&sh.u.p12[0][i][kq][pos0];
        uint32_t pc4 = (uint32_t)(uintptr_t)&sh.u.p12[0][i][kq][pos4];
        asm volatile("" : "+v"(pa0), "+v"(pa4), "+v"(pc0), "+v"(pc4));

        // ---- window extraction and the A sums (per chunk: products to LDS; the chunk's wave sums)
#pragma unroll
        for (int c = 0; c < kNCH; c++) {
            const int b = c & 1;
            __builtin_amdgcn_sched_barrier(0);   // keep each chunk's work in place (register pressure)
#pragma unroll
            for (int m = 0; m < kEPC; m++) {
                const int k = c * kEPC + m;
                __builtin_amdgcn_sched_barrier(0);   // one element's 8 loads in flight at a time
                int ival = 0, ixv = 0, iyv = 0;
                if (ok) {
                    const int o = ibase + (c * kRC + ey(m)) * pitch + ex(m);
                    const uint8_t* ip = Ib + o;
                    ival = (ip[0] * w00 + ip[1] * w01 + ip[pitch] * w10 + ip[pitch + 1] * w11 + 256) >> 9;
                    const uint32_t* dp = Db + o;
                    const uint32_t d00 = dp[0], d01 = dp[1], d10 = dp[pitch], d11 = dp[pitch + 1];
                    ixv = ((int)(int16_t)d00 * w00 + (int)(int16_t)d01 * w01 + (int)(int16_t)d10 * w10 +
                           (int)(int16_t)d11 * w11 + 8192) >> 14;
                    iyv = (((int)d00 >> 16) * w00 + ((int)d01 >> 16) * w01 + ((int)d10 >> 16) * w10 +
                           ((int)d11 >> 16) * w11 + 8192) >> 14;
                }
                sd[k] = ((uint32_t)ixv & 0xffffu) | ((uint32_t)iyv << 16);
                if (k & 1) si[k >> 1] = (si[k >> 1] & 0xffffu) | ((uint32_t)ival << 16);
                else si[k >> 1] = (uint32_t)ival;
                const float fx = (float)ixv, fy = (float)iyv;
                // products of integers below 2^24: exact in float (== the reference's rounding)
                const uint32_t mo = (uint32_t)(m < 4 ? m * 20 : 0);
                *(lf2)(uintptr_t)((m < 4 ? pa0 : pa4) + 8u * ((uint32_t)(b * kNP * 4 * kPS2) + mo)) = f2p{fx * fx, fy * fy};
                *(lfl)(uintptr_t)((m < 4 ? pc0 : pc4) + 4u * ((uint32_t)(b * kNP * 4 * kPS1) + mo)) = fx * fy;
            }
            __syncthreads();
            if (wave == ((c + rot) % kNP) && sp < kNP) {
                // lanes sq < 4: the (A11, A22) chain sq of point sp; sq >= 4: its A12 chain sq - 4
                if (sq < 4) {
                    f2p acc = c ? sh.acc2[sp][sq] : f2p{0.f, 0.f};
                    const f2p* src = sh.pab[b][sp][sq];
#pragma unroll 1
                    for (int q0 = 0; q0 < kPOS; q0 += 8) {   // 8 products in flight: few registers
#pragma unroll
                        for (int q = q0; q < q0 + 8; q++) acc = acc + src[q];
                    }
                    sh.acc2[sp][sq] = acc;
                } else {
                    float acc = c ? sh.acc1[sp][sq - 4] : 0.f;
                    const float* src = sh.u.p12[b][sp][sq - 4];
#pragma unroll 1
                    for (int q0 = 0; q0 < kPOS; q0 += 8) {   // 8 products in flight: few registers
#pragma unroll
                        for (int q = q0; q < q0 + 8; q++) acc = acc + src[q];
                    }
                    sh.acc1[sp][sq - 4] = acc;
                }
            }
        }
        __syncthreads();
        rot += kNCH;
        float A11 = 0.f, A12 = 0.f, A22 = 0.f, Dinv = 0.f;
        if (ok) {
            const f2p a0 = sh.acc2[i][0], a1 = sh.acc2[i][1], a2 = sh.acc2[i][2], a3 = sh.acc2[i][3];
            A11 = ((a0.x + a1.x) + a2.x) + a3.x;
            A22 = ((a0.y + a1.y) + a2.y) + a3.y;
            A12 = ((sh.acc1[i][0] + sh.acc1[i][1]) + sh.acc1[i][2]) + sh.acc1[i][3];
            A11 = A11 * FLT_SCALE;
            A12 = A12 * FLT_SCALE;
            A22 = A22 * FLT_SCALE;
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
        float nx = npx - HALFW, ny = npy - HALFW;
        float pdx = 0.f, pdy = 0.f;
        bool act = ok;
        for (int j = 0; j < a.max_iters; j++) {
            int inx = 0, iny = 0;
            if (act) {
                inx = (int)floorf(nx);
                iny = (int)floorf(ny);
                if (inx < -kWin || inx >= L.w || iny < -kWin || iny >= L.h) {
                    act = false;
                    if (level == 0) status = 0;
                }
            }
            if (s == 0) sh.jpos[i] = make_int4(inx, iny, act ? 1 : 0, 0);
            if (!__syncthreads_or(act)) break;
            // the window values are loop-invariant; keep the compiler from hoisting what it derives
            // from them (their floats, the J biases: 150 registers) out of the Newton loop
#pragma unroll
            for (int q = 0; q < kNE; q++) asm volatile("" : "+v"(sd[q]));
#pragma unroll
            for (int q = 0; q < (kNE + 1) / 2; q++) asm volatile("" : "+v"(si[q]));
            uint32_t jb0 = (uint32_t)(uintptr_t)&sh.u.jwin[i][s >> 5][(s & 31) >> 2];
            uint32_t jb4 = (uint32_t)(uintptr_t)&sh.u.jwin[i][s >> 3][8 + ((s & 7) >> 2)];
            uint32_t pb0 = pa0, pb4 = pa4;
            asm volatile("" : "+v"(jb0), "+v"(jb4), "+v"(pb0), "+v"(pb4));
            int v00 = 0, v01 = 0, v10 = 0, v11 = 0;
            if (act) lkpt_weights(nx - (float)inx, ny - (float)iny, v00, v01, v10, v11);
            // signed: w11 = 16384 - w00 - w01 - w10 can be -1 after rounding
            const s2p W0 = {(short)v00, (short)v01};
            const s2p W1 = {(short)v10, (short)v11};
            // stage every active point's 41 J rows, bytes inx .. inx+43, dword-aligned in LDS
            for (int r = t; r < kNP * (kWin + 1); r += kWG) {
                const int pp = r / (kWin + 1), row = r % (kWin + 1);
                const int4 jp = sh.jpos[pp];
                if (!jp.z) continue;
                // 4-byte aligned 16-B loads (rows are 64-B aligned, jp.x & ~3 a multiple of 4)
                const u4al* src = reinterpret_cast<const u4al*>(Jb + (long long)(jp.y + row) * pitch + (jp.x & ~3));
                const u4al q0 = src[0], q1 = src[1], q2 = src[2];
                const uint32_t d[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
                const unsigned shb = (unsigned)(jp.x & 3);
                uint32_t o[kJW];
#pragma unroll
                for (int n = 0; n < 11; n++) o[n] = __builtin_amdgcn_alignbyte(d[n + 1], d[n], shb);
                o[11] = 0;
                uint4* dst = reinterpret_cast<uint4*>(sh.u.jwin[pp][row]);
                dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
                dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
                dst[2] = make_uint4(o[8], o[9], o[10], o[11]);
            }
            __syncthreads();
#pragma unroll
            for (int c = 0; c < kNCH; c++) {
                const int b = c & 1;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < kEPC; m++) {
                    const int k = c * kEPC + m;
                    const lcu r0 = (lcu)(uintptr_t)((m < 4 ? jb0 : jb4) + 4u * (uint32_t)((c * kRC + (m < 4 ? 2 * m : 0)) * kJW));
                    const lcu r1 = r0 + kJW;
                    const s2p ta = __builtin_bit_cast(s2p, __builtin_amdgcn_perm(r0[1], r0[0], jsel));
                    const s2p tb = __builtin_bit_cast(s2p, __builtin_amdgcn_perm(r1[1], r1[0], jsel));
                    const int iv = (int)((k & 1) ? (si[k >> 1] >> 16) : (si[k >> 1] & 0xffffu));
                    // (J*32 - I*32) exactly as the reference's CV_DESCALE(...) - I: the bias
                    // 256 - 512*I folds the rounding and the subtraction into the dot product
                    const int jd = __builtin_amdgcn_sdot2(ta, W0, __builtin_amdgcn_sdot2(tb, W1, 256 - 512 * iv, false),
                                                          false) >> 9;
                    const float fd = (float)jd;
                    const uint32_t dv = sd[k];
                    const f2p f = {(float)(int16_t)dv, (float)((int)dv >> 16)};
                    *((lf2)(uintptr_t)((m < 4 ? pb0 : pb4) + 8u * (uint32_t)(b * kNP * 4 * kPS2 + (m < 4 ? m * 20 : 0)))) = f * fd;
                }
                __syncthreads();
                if (wave == ((c + rot) % kNP) && sp < kNP && sq < 4) {
                    f2p acc = c ? sh.acc2[sp][sq] : f2p{0.f, 0.f};
                    const f2p* src = sh.pab[b][sp][sq];
#pragma unroll 1
                    for (int q0 = 0; q0 < kPOS; q0 += 8) {   // 8 products in flight: few registers
#pragma unroll
                        for (int q = q0; q < q0 + 8; q++) acc = acc + src[q];
                    }
                    sh.acc2[sp][sq] = acc;
                }
            }
            __syncthreads();
            rot += kNCH;
            if (act) {
                const f2p q0 = sh.acc2[i][0], q1 = sh.acc2[i][1], q2 = sh.acc2[i][2], q3 = sh.acc2[i][3];
                float b1 = (q0.x + q2.x) + (q1.x + q3.x);
                float b2 = (q0.y + q2.y) + (q1.y + q3.y);
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
            // jpos / acc2 are rewritten by the next step only after its first barrier
        }
        __syncthreads();   // LDS (J windows) is reused by the next level's products

        if (level == 0 && valid && status) {
            // err pass of LKTrackerInvoker: its final bounds check is observable (status).
            const int fx = (int)floorf(npx - HALFW), fy = (int)floorf(npy - HALFW);
            if (fx < -kWin || fx >= L.w || fy < -kWin || fy >= L.h) status = 0;
        }
    }

    if (valid && s == 0) {
        const long long o = (long long)pair * a.npts + pt;
        a.next_pts[2 * o] = npx;
        a.next_pts[2 * o + 1] = npy;
        a.status[o] = (uint8_t)status;
    }
}

hipError_t launch_lk_pts(hipStream_t s, int batch, const LkArgs& a)
{
    const dim3 grid((a.npts + kNP - 1) / kNP, batch);
    hipLaunchKernelGGL(k_lk_pts, grid, dim3(kWG), 0, s, a);
    return hipGetLastError();
}

}  // namespace mdx
