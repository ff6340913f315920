/*
 * mdx_oracle_sse2.c -- SSE2-intrinsics restatement of the two hot loops of the CPU oracle.
 * TEST INFRASTRUCTURE ONLY (the timed CPU baseline, `cpu_baseline.kind == "port-sse2"`): the
 * product path never links or calls this file.
 *
 * The reference runs OpenCV 2.4's x86 build of calcOpticalFlowPyrLK (called at reference
 * common/src/optical_flow_calculator.cpp:71) and warpPerspective (:124), whose inner loops are
 * SSE2.  The scalar oracle (mdx_oracle.c) already follows their 4-lane evaluation order; this file
 * evaluates the same order with 128-bit integer / float vectors, so the CPU baseline is a fair
 * stand-in for the reference's own speed:
 *   - LK window extraction + gradient sums: 4 window columns per step, the bilinear taps as
 *     pmaddwd of (tap, tap+1) x (w00, w01) + (tap', tap'+1) x (w10, w11) pairs, the descale by
 *     arithmetic shift, and three __m128 partial sums whose lane k holds columns x = 4g + k in row
 *     order (A = ((P0+P1)+P2)+P3 is done by the caller);
 *   - LK iteration sums: J taps the same way, It = J*32 - I*32 as int32, the products It*Ix and
 *     It*Iy as exact int32 (pmullw / pmulhw halves), converted and added into two __m128 sums whose
 *     lanes hold (Ix, Iy) products of columns 4g + {0, 1} and 4g + {2, 3}: b = (P0+P2)+(P1+P3);
 *   - warp bilinear (remapBilinear, 15-bit fixed point): four destination pixels per step whose
 *     taps are all inside, as pmaddwd of tap pairs and the BilinearTab weights.
 * Every float operation is a separate multiply or add (no FMA on x86-64 SSE2), so the results are
 * bit-identical to the scalar oracle's (tests/test_oracle.py checks it).
 */
#include <emmintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "mdx_oracle.h"

static inline __m128i load4_u8(const uint8_t* p)
{
    int v;
    memcpy(&v, p, 4);
    return _mm_unpacklo_epi8(_mm_cvtsi32_si128(v), _mm_setzero_si128());   /* 4 x u16 in the low half */
}

/* bilinear of 4 adjacent u8 taps at p (row r) and p + step (row r+1), weights as int16 pairs */
static inline __m128i interp4_u8(const uint8_t* p, ptrdiff_t step, __m128i qw0, __m128i qw1)
{
    const __m128i a0 = load4_u8(p), a1 = load4_u8(p + 1), b0 = load4_u8(p + step), b1 = load4_u8(p + step + 1);
    return _mm_add_epi32(_mm_madd_epi16(_mm_unpacklo_epi16(a0, a1), qw0),
                         _mm_madd_epi16(_mm_unpacklo_epi16(b0, b1), qw1));
}

void ora_sse2_window_sums(const uint8_t* I, int stepI, const int16_t* D, int dstep, int win, int iw00, int iw01,
                          int iw10, int iw11, int16_t* Iwin, int16_t* dIwin, float qA11[4], float qA12[4],
                          float qA22[4])
{
    const __m128i qw0 = _mm_set1_epi32((iw00 & 0xffff) | (iw01 << 16));
    const __m128i qw1 = _mm_set1_epi32((iw10 & 0xffff) | (iw11 << 16));
    const __m128i di = _mm_set1_epi32(1 << 8), dd = _mm_set1_epi32(1 << 13);
    __m128 a11 = _mm_setzero_ps(), a12 = _mm_setzero_ps(), a22 = _mm_setzero_ps();
    for (int y = 0; y < win; y++) {
        const uint8_t* src = I + (ptrdiff_t)y * stepI;
        const int16_t* ds = D + (ptrdiff_t)y * dstep;
        for (int x = 0; x < win; x += 4) {
            const __m128i t = _mm_srai_epi32(_mm_add_epi32(interp4_u8(src + x, stepI, qw0, qw1), di), 9);
            _mm_storel_epi64((__m128i*)(Iwin + y * win + x), _mm_packs_epi32(t, t));
            /* (Ix, Iy) pairs of columns x .. x+3 and their right neighbours, rows y and y+1 */
            const __m128i d00 = _mm_loadu_si128((const __m128i*)(ds + 2 * x));
            const __m128i d01 = _mm_loadu_si128((const __m128i*)(ds + 2 * x + 2));
            const __m128i d10 = _mm_loadu_si128((const __m128i*)(ds + dstep + 2 * x));
            const __m128i d11 = _mm_loadu_si128((const __m128i*)(ds + dstep + 2 * x + 2));
            __m128i lo = _mm_add_epi32(_mm_madd_epi16(_mm_unpacklo_epi16(d00, d01), qw0),
                                       _mm_madd_epi16(_mm_unpacklo_epi16(d10, d11), qw1));
            __m128i hi = _mm_add_epi32(_mm_madd_epi16(_mm_unpackhi_epi16(d00, d01), qw0),
                                       _mm_madd_epi16(_mm_unpackhi_epi16(d10, d11), qw1));
            lo = _mm_srai_epi32(_mm_add_epi32(lo, dd), 14);   /* Ix0 Iy0 Ix1 Iy1 */
            hi = _mm_srai_epi32(_mm_add_epi32(hi, dd), 14);   /* Ix2 Iy2 Ix3 Iy3 */
            const __m128i v = _mm_packs_epi32(lo, hi);
            _mm_storeu_si128((__m128i*)(dIwin + 2 * (y * win + x)), v);
            const __m128 fx = _mm_cvtepi32_ps(_mm_srai_epi32(_mm_slli_epi32(v, 16), 16));
            const __m128 fy = _mm_cvtepi32_ps(_mm_srai_epi32(v, 16));
            a11 = _mm_add_ps(a11, _mm_mul_ps(fx, fx));
            a12 = _mm_add_ps(a12, _mm_mul_ps(fx, fy));
            a22 = _mm_add_ps(a22, _mm_mul_ps(fy, fy));
        }
    }
    _mm_storeu_ps(qA11, a11);
    _mm_storeu_ps(qA12, a12);
    _mm_storeu_ps(qA22, a22);
}

void ora_sse2_iter_sums(const uint8_t* J, int stepJ, const int16_t* Iwin, const int16_t* dIwin, int win, int iw00,
                        int iw01, int iw10, int iw11, float q1[4], float q2[4])
{
    const __m128i qw0 = _mm_set1_epi32((iw00 & 0xffff) | (iw01 << 16));
    const __m128i qw1 = _mm_set1_epi32((iw10 & 0xffff) | (iw11 << 16));
    const __m128i di = _mm_set1_epi32(1 << 8);
    __m128 s01 = _mm_setzero_ps(), s23 = _mm_setzero_ps();   /* (Ix It, Iy It) of columns 4g+0,1 / 4g+2,3 */
    for (int y = 0; y < win; y++) {
        const uint8_t* Jp = J + (ptrdiff_t)y * stepJ;
        const int16_t* Ip = Iwin + y * win;
        const int16_t* dIp = dIwin + 2 * y * win;
        for (int x = 0; x < win; x += 4) {
            const __m128i jv = _mm_srai_epi32(_mm_add_epi32(interp4_u8(Jp + x, stepJ, qw0, qw1), di), 9);
            const __m128i iv = _mm_srai_epi32(_mm_unpacklo_epi16(_mm_loadl_epi64((const __m128i*)(Ip + x)),
                                                                 _mm_loadl_epi64((const __m128i*)(Ip + x))), 16);
            const __m128i it = _mm_sub_epi32(jv, iv);                      /* |It| <= 8160: int16 */
            const __m128i it16 = _mm_packs_epi32(it, it);
            const __m128i itp = _mm_unpacklo_epi16(it16, it16);            /* It0 It0 It1 It1 ... */
            const __m128i d = _mm_loadu_si128((const __m128i*)(dIp + 2 * x));
            const __m128i pl = _mm_mullo_epi16(d, itp), ph = _mm_mulhi_epi16(d, itp);
            s01 = _mm_add_ps(s01, _mm_cvtepi32_ps(_mm_unpacklo_epi16(pl, ph)));
            s23 = _mm_add_ps(s23, _mm_cvtepi32_ps(_mm_unpackhi_epi16(pl, ph)));
        }
    }
    float a[4], b[4];
    _mm_storeu_ps(a, s01);
    _mm_storeu_ps(b, s23);
    q1[0] = a[0]; q2[0] = a[1]; q1[1] = a[2]; q2[1] = a[3];
    q1[2] = b[0]; q2[2] = b[1]; q1[3] = b[2]; q2[3] = b[3];
}

/* Four interior destination pixels: taps p[k], p[k]+1 (row sy) and p[k]+stride, +stride+1, 15-bit
 * weights w[k][0..3] (BilinearTab_i, every entry <= 32767); out = (sum + 2^14) >> 15 as u8. */
void ora_sse2_bilinear4(const uint8_t* const p[4], int stride, const int w[4][4], uint8_t out[4])
{
    const __m128i t0 = _mm_setr_epi16(p[0][0], p[0][1], p[1][0], p[1][1], p[2][0], p[2][1], p[3][0], p[3][1]);
    const __m128i t1 = _mm_setr_epi16(p[0][stride], p[0][stride + 1], p[1][stride], p[1][stride + 1], p[2][stride],
                                      p[2][stride + 1], p[3][stride], p[3][stride + 1]);
    const __m128i w0 = _mm_setr_epi16(w[0][0], w[0][1], w[1][0], w[1][1], w[2][0], w[2][1], w[3][0], w[3][1]);
    const __m128i w1 = _mm_setr_epi16(w[0][2], w[0][3], w[1][2], w[1][3], w[2][2], w[2][3], w[3][2], w[3][3]);
    __m128i s = _mm_add_epi32(_mm_madd_epi16(t0, w0), _mm_madd_epi16(t1, w1));
    s = _mm_srai_epi32(_mm_add_epi32(s, _mm_set1_epi32(1 << 14)), 15);
    const __m128i b = _mm_packus_epi16(_mm_packs_epi32(s, s), _mm_setzero_si128());
    const int v = _mm_cvtsi128_si32(b);
    memcpy(out, &v, 4);
}
