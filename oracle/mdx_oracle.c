/*
 * mdx_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
 * product.  See mdx_oracle.h for scope and the parity-unpinned statement.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; x86-64 => SSE2 float, no x87 excess
 * precision, matching an x86-64 OpenCV 2.4 build).  Every float/double expression below is
 * written in the evaluation order of the OpenCV 2.4.8 source it restates; contraction
 * into FMA must stay off or the LK sums and warp coordinates change.
 */
#include "mdx_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

void ora_default_params(ora_params* p)
{
    /* optical_flow_calculator.cpp:40-44, :71, :127; node.cpp:44; bag.launch:27 */
    p->win = 40;
    p->max_level = 5;
    p->max_iters = 10;
    p->eps = 0.03;
    p->min_eig = 0.001f;
    p->thresh = 190;
    p->pixel_step = 10;
    p->min_vector_size = 1.0;
    p->fit_mode = ORA_FIT_FIRST4;
    p->ransac_iters = 128;
    p->ransac_thresh = 3.0;
    p->ransac_seed = 20141105u;
}

/* OpenCV borderInterpolate(p, len, BORDER_REFLECT_101) (core/src/copy.cpp). */
int ora_reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;               /* -p - 1 + delta, delta = 1 */
        else p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

/* ---------------------------------------------------------------- A1: cvtColor ------- */
/* color.cpp RGB2Gray<uchar>, CV_BGR2GRAY (blueIdx 0): tab-based
 *   gray = (s0*B2Y + s1*G2Y + s2*R2Y + (1<<13)) >> 14, B2Y=1868 G2Y=9617 R2Y=4899.
 * The node converts every frame to rgb8 first (motion_detection_node.cpp:271), so s0 is
 * R: effective weights R*1868 + G*9617 + B*4899.  A bgr8 message is converted to rgb8 by
 * cv_bridge before that, so the same weights apply to its true R/G/B; mono8 is replicated
 * to 3 channels, which gives gray == input exactly. */
void ora_to_gray(const uint8_t* src, int w, int h, int stride, int fmt, uint8_t* dst)
{
    for (int y = 0; y < h; y++) {
        const uint8_t* s = src + (size_t)y * stride;
        uint8_t* d = dst + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            if (fmt == ORA_FMT_GRAY8) {
                int v = s[x];
                d[x] = (uint8_t)((v * 1868 + v * 9617 + 8192 + v * 4899) >> 14);
            } else {
                int r, g, b;
                if (fmt == ORA_FMT_RGB8) { r = s[3 * x]; g = s[3 * x + 1]; b = s[3 * x + 2]; }
                else { b = s[3 * x]; g = s[3 * x + 1]; r = s[3 * x + 2]; }
                d[x] = (uint8_t)((r * 1868 + g * 9617 + (8192 + b * 4899)) >> 14);
            }
        }
    }
}

/* ---------------------------------------------------------------- A3: pyrDown -------- */
/* pyramids.cpp pyrDown_<FixPtCast<uchar,8>>: separable [1 4 6 4 1] on the ROI with
 * BORDER_REFLECT_101 on the ROI's own size (borderInterpolate on ssize), +128 >> 8. */
void ora_pyrdown(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh, int dstride)
{
    int* row = (int*)malloc(sizeof(int) * 5 * (size_t)dw);
    int* tab = (int*)malloc(sizeof(int) * 5 * (size_t)dw);
    for (int x = 0; x < dw; x++)
        for (int k = 0; k < 5; k++) tab[x * 5 + k] = ora_reflect101(2 * x + k - 2, sw);
    for (int y = 0; y < dh; y++) {
        for (int k = 0; k < 5; k++) {
            const uint8_t* s = src + (size_t)ora_reflect101(2 * y + k - 2, sh) * sstride;
            int* r = row + (size_t)k * dw;
            for (int x = 0; x < dw; x++) {
                const int* t = tab + x * 5;
                r[x] = s[t[2]] * 6 + (s[t[1]] + s[t[3]]) * 4 + s[t[0]] + s[t[4]];
            }
        }
        uint8_t* d = dst + (size_t)y * dstride;
        for (int x = 0; x < dw; x++) {
            int v = row[2 * dw + x] * 6 + (row[dw + x] + row[3 * dw + x]) * 4 + row[x] + row[4 * dw + x];
            d[x] = (uint8_t)((v + 128) >> 8);
        }
    }
    free(row);
    free(tab);
}

/* ---------------------------------------------------------------- A3: Scharr --------- */
/* lkpyramid.cpp calcSharrDeriv: vertical t0 = 3(a+c)+10b, t1 = c-a with rows clamped as
 * reflect-101 (y-1 -> 1 at y=0), then horizontal Ix = t0[x+1]-t0[x-1],
 * Iy = 3(t1[x-1]+t1[x+1]) + 10 t1[x] with cols reflect-101; int16 interleaved (Ix, Iy). */
void ora_scharr(const uint8_t* src, int w, int h, int sstride, int16_t* dst, int dstride)
{
    int16_t* t0 = (int16_t*)malloc(sizeof(int16_t) * (size_t)(w + 2));
    int16_t* t1 = (int16_t*)malloc(sizeof(int16_t) * (size_t)(w + 2));
    for (int y = 0; y < h; y++) {
        const uint8_t* s0 = src + (size_t)(y > 0 ? y - 1 : h > 1 ? 1 : 0) * sstride;
        const uint8_t* s1 = src + (size_t)y * sstride;
        const uint8_t* s2 = src + (size_t)(y < h - 1 ? y + 1 : h > 1 ? h - 2 : 0) * sstride;
        int16_t* d = dst + (size_t)y * dstride;
        for (int x = 0; x < w; x++) {
            t0[x + 1] = (int16_t)((s0[x] + s2[x]) * 3 + s1[x] * 10);
            t1[x + 1] = (int16_t)(s2[x] - s0[x]);
        }
        int x0 = w > 1 ? 1 : 0, x1 = w > 1 ? w - 2 : 0;
        t0[0] = t0[x0 + 1]; t0[w + 1] = t0[x1 + 1];
        t1[0] = t1[x0 + 1]; t1[w + 1] = t1[x1 + 1];
        for (int x = 0; x < w; x++) {
            d[2 * x] = (int16_t)(t0[x + 2] - t0[x]);
            d[2 * x + 1] = (int16_t)((t1[x + 2] + t1[x]) * 3 + t1[x + 1] * 10);
        }
    }
    free(t0);
    free(t1);
}

/* ---------------------------------------------------------------- buildOpticalFlowPyramid */
/* lkpyramid.cpp buildOpticalFlowPyramid(img, pyr, Size(win,win), maxLevel, withDerivatives,
 * BORDER_REFLECT_101, BORDER_CONSTANT): level 0 = img padded by win (REFLECT_101); level
 * l+1 = pyrDown(level l ROI) padded REFLECT_101|ISOLATED; derivs = calcSharrDeriv(level)
 * padded CONSTANT 0.  Stops (returns level) when the next size is <= win on either side. */
static void pad_reflect_u8(uint8_t* buf, int w, int h, int pad)
{
    int pitch = w + 2 * pad;
    for (int y = -pad; y < h + pad; y++) {
        uint8_t* r = buf + (size_t)(y + pad) * pitch;
        const uint8_t* sr = buf + (size_t)(ora_reflect101(y, h) + pad) * pitch;
        for (int x = -pad; x < w + pad; x++) {
            if (x >= 0 && x < w && y >= 0 && y < h) continue;
            r[x + pad] = sr[ora_reflect101(x, w) + pad];
        }
    }
}

int ora_build_pyramid(const uint8_t* gray, int w, int h, int win, int max_level, int with_deriv, ora_pyramid* out)
{
    memset(out, 0, sizeof(*out));
    out->pad = win;
    int sw = w, sh = h;
    int level;
    for (level = 0; level <= max_level && level < ORA_MAX_LEVELS; level++) {
        int pitch = sw + 2 * win;
        uint8_t* buf = (uint8_t*)calloc((size_t)pitch * (sh + 2 * win), 1);
        uint8_t* core = buf + (size_t)win * pitch + win;
        if (level == 0) {
            for (int y = 0; y < sh; y++) memcpy(core + (size_t)y * pitch, gray + (size_t)y * w, (size_t)sw);
        } else {
            int pw = out->w[level - 1], pp = pw + 2 * win;
            const uint8_t* pcore = out->img[level - 1] + (size_t)win * pp + win;
            ora_pyrdown(pcore, pw, out->h[level - 1], pp, core, sw, sh, pitch);
        }
        pad_reflect_u8(buf, sw, sh, win);
        out->img[level] = buf;
        out->w[level] = sw;
        out->h[level] = sh;
        if (with_deriv) {
            int16_t* d = (int16_t*)calloc((size_t)pitch * (sh + 2 * win) * 2, sizeof(int16_t));
            ora_scharr(core, sw, sh, pitch, d + ((size_t)win * pitch + win) * 2, pitch * 2);
            out->deriv[level] = d;  /* border stays 0: BORDER_CONSTANT */
        }
        out->nlevels = level + 1;
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win || sh <= win) return level;
    }
    return max_level;
}

void ora_free_pyramid(ora_pyramid* p)
{
    for (int l = 0; l < p->nlevels; l++) {
        free(p->img[l]);
        free(p->deriv[l]);
    }
    memset(p, 0, sizeof(*p));
}

/* ---------------------------------------------------------------- A5: LK tracker ------ */
/* cvRound(float) == _mm_cvtss_si32 (round half to even); cvFloor via double. */
static inline int cv_round_f(float v) { return (int)lrintf(v); }

static int g_simd = 0;
void ora_set_simd(int on) { g_simd = on != 0; }
static inline int cv_floor_f(float v) { return (int)floor((double)v); }

typedef struct {
    const ora_pyramid* prev;
    const ora_pyramid* next;
    int level, max_level;
    const float* prev_pts;
    float* next_pts;
    uint8_t* status;
    const ora_params* prm;
    int begin, end;
} lk_job;

/*
 * LKTrackerInvoker::operator() for one level, x86-64 SSE2 code path.  The float sums are
 * accumulated exactly as the SSE2 code does it (winSize.width = 40 is a multiple of 8, so
 * the scalar tails never run):
 *   A11/A12/A22: four partials, lane k takes x = 4g+k (g = 0..9) over rows y = 0..39 in
 *                order; A = ((P0+P1)+P2)+P3.
 *   b1/b2:       four partials per quantity, lane k takes x = 4g+k in the same order;
 *                b = (P0+P2) + (P1+P3)   (qb0+qb1 then bbuf[0]+bbuf[2]).
 * Each term is the exact integer product rounded once to float.
 */
static void lk_level_range(const lk_job* jb)
{
    const int win = jb->prm->win;
    const int level = jb->level;
    const float halfw = (float)(win - 1) * 0.5f;
    const int pad = jb->prev->pad;
    const int Iw = jb->prev->w[level], Ih = jb->prev->h[level];
    const int Jw = jb->next->w[level], Jh = jb->next->h[level];
    const int stepI = Iw + 2 * pad, stepJ = Jw + 2 * pad, dstep = stepI * 2;
    const uint8_t* I0 = jb->prev->img[level] + (size_t)pad * stepI + pad;
    const int16_t* D0 = jb->prev->deriv[level] + ((size_t)pad * stepI + pad) * 2;
    const uint8_t* J0 = jb->next->img[level] + (size_t)pad * stepJ + pad;
    const int W_BITS = 14;
    const float FLT_SCALE = 1.f / (1 << 20);
    const double eps2 = jb->prm->eps * jb->prm->eps;   /* criteria.epsilon *= epsilon */
    const float minEigThr = jb->prm->min_eig;
    int maxCount = jb->prm->max_iters;
    if (maxCount < 0) maxCount = 0;
    if (maxCount > 100) maxCount = 100;

    int16_t* Iwin = (int16_t*)malloc(sizeof(int16_t) * (size_t)win * win);
    int16_t* dIwin = (int16_t*)malloc(sizeof(int16_t) * (size_t)win * win * 2);

    for (int ptidx = jb->begin; ptidx < jb->end; ptidx++) {
        float scale = (float)(1. / (1 << level));
        float px = jb->prev_pts[2 * ptidx] * scale, py = jb->prev_pts[2 * ptidx + 1] * scale;
        float nx, ny;
        if (level == jb->max_level) { nx = px; ny = py; }
        else { nx = jb->next_pts[2 * ptidx] * 2.f; ny = jb->next_pts[2 * ptidx + 1] * 2.f; }
        jb->next_pts[2 * ptidx] = nx;
        jb->next_pts[2 * ptidx + 1] = ny;

        px -= halfw; py -= halfw;
        int ipx = cv_floor_f(px), ipy = cv_floor_f(py);
        if (ipx < -win || ipx >= Iw || ipy < -win || ipy >= Ih) {
            if (level == 0) jb->status[ptidx] = 0;
            continue;
        }
        float a = px - (float)ipx, b = py - (float)ipy;
        int iw00 = cv_round_f((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
        int iw01 = cv_round_f(a * (1.f - b) * (float)(1 << W_BITS));
        int iw10 = cv_round_f((1.f - a) * b * (float)(1 << W_BITS));
        int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

        float qA11[4] = {0, 0, 0, 0}, qA12[4] = {0, 0, 0, 0}, qA22[4] = {0, 0, 0, 0};
        if (g_simd && win % 4 == 0)
            ora_sse2_window_sums(I0 + (ptrdiff_t)ipy * stepI + ipx, stepI, D0 + (ptrdiff_t)ipy * dstep + (ptrdiff_t)ipx * 2,
                                 dstep, win, iw00, iw01, iw10, iw11, Iwin, dIwin, qA11, qA12, qA22);
        else
        for (int y = 0; y < win; y++) {
            const uint8_t* src = I0 + (ptrdiff_t)(y + ipy) * stepI + ipx;
            const int16_t* dsrc = D0 + (ptrdiff_t)(y + ipy) * dstep + (ptrdiff_t)ipx * 2;
            for (int x = 0; x < win; x++) {
                int ival = (src[x] * iw00 + src[x + 1] * iw01 + src[x + stepI] * iw10 +
                            src[x + stepI + 1] * iw11 + (1 << 8)) >> 9;
                const int16_t* ds = dsrc + 2 * x;
                int ixval = (ds[0] * iw00 + ds[2] * iw01 + ds[dstep] * iw10 + ds[dstep + 2] * iw11 +
                             (1 << 13)) >> 14;
                int iyval = (ds[1] * iw00 + ds[3] * iw01 + ds[dstep + 1] * iw10 + ds[dstep + 3] * iw11 +
                             (1 << 13)) >> 14;
                Iwin[y * win + x] = (int16_t)ival;
                dIwin[2 * (y * win + x)] = (int16_t)ixval;
                dIwin[2 * (y * win + x) + 1] = (int16_t)iyval;
                int k = x & 3;
                qA11[k] = qA11[k] + (float)(ixval * ixval);
                qA12[k] = qA12[k] + (float)(ixval * iyval);
                qA22[k] = qA22[k] + (float)(iyval * iyval);
            }
        }
        float A11 = ((qA11[0] + qA11[1]) + qA11[2]) + qA11[3];
        float A12 = ((qA12[0] + qA12[1]) + qA12[2]) + qA12[3];
        float A22 = ((qA22[0] + qA22[1]) + qA22[2]) + qA22[3];
        A11 *= FLT_SCALE;
        A12 *= FLT_SCALE;
        A22 *= FLT_SCALE;

        float D = A11 * A22 - A12 * A12;
        float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                       (float)(2 * win * win);
        if (minEig < minEigThr || D < FLT_EPSILON) {
            if (level == 0) jb->status[ptidx] = 0;
            continue;
        }
        D = 1.f / D;

        nx -= halfw; ny -= halfw;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < maxCount; j++) {
            int inx = cv_floor_f(nx), iny = cv_floor_f(ny);
            if (inx < -win || inx >= Jw || iny < -win || iny >= Jh) {
                if (level == 0) jb->status[ptidx] = 0;
                break;
            }
            a = nx - (float)inx;
            b = ny - (float)iny;
            iw00 = cv_round_f((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
            iw01 = cv_round_f(a * (1.f - b) * (float)(1 << W_BITS));
            iw10 = cv_round_f((1.f - a) * b * (float)(1 << W_BITS));
            iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
            float q1[4] = {0, 0, 0, 0}, q2[4] = {0, 0, 0, 0};
            if (g_simd && win % 4 == 0)
                ora_sse2_iter_sums(J0 + (ptrdiff_t)iny * stepJ + inx, stepJ, Iwin, dIwin, win, iw00, iw01, iw10, iw11, q1, q2);
            else
            for (int y = 0; y < win; y++) {
                const uint8_t* Jp = J0 + (ptrdiff_t)(y + iny) * stepJ + inx;
                const int16_t* Ip = Iwin + y * win;
                const int16_t* dIp = dIwin + 2 * y * win;
                for (int x = 0; x < win; x++) {
                    int diff = ((Jp[x] * iw00 + Jp[x + 1] * iw01 + Jp[x + stepJ] * iw10 +
                                 Jp[x + stepJ + 1] * iw11 + (1 << 8)) >> 9) - Ip[x];
                    int k = x & 3;
                    q1[k] = q1[k] + (float)(diff * dIp[2 * x]);
                    q2[k] = q2[k] + (float)(diff * dIp[2 * x + 1]);
                }
            }
            float b1 = (q1[0] + q1[2]) + (q1[1] + q1[3]);
            float b2 = (q2[0] + q2[2]) + (q2[1] + q2[3]);
            b1 *= FLT_SCALE;
            b2 *= FLT_SCALE;
            float dx = (A12 * b2 - A22 * b1) * D;
            float dy = (A12 * b1 - A11 * b2) * D;
            nx += dx;
            ny += dy;
            jb->next_pts[2 * ptidx] = nx + halfw;
            jb->next_pts[2 * ptidx + 1] = ny + halfw;
            if ((double)dx * dx + (double)dy * dy <= eps2) break;
            if (j > 0 && fabs((double)fabsf(dx + pdx)) < 0.01 && fabs((double)fabsf(dy + pdy)) < 0.01) {
                jb->next_pts[2 * ptidx] -= dx * 0.5f;
                jb->next_pts[2 * ptidx + 1] -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }

        /* err pass (err is requested at :71): only its final bounds check is observable. */
        if (jb->status[ptidx] && level == 0) {
            float fx = jb->next_pts[2 * ptidx] - halfw, fy = jb->next_pts[2 * ptidx + 1] - halfw;
            int ix = cv_floor_f(fx), iy = cv_floor_f(fy);
            if (ix < -win || ix >= Jw || iy < -win || iy >= Jh) jb->status[ptidx] = 0;
        }
    }
    free(Iwin);
    free(dIwin);
}

static void* lk_thread(void* arg)
{
    lk_level_range((const lk_job*)arg);
    return NULL;
}

void ora_lk(const ora_pyramid* prev, const ora_pyramid* next, int max_level,
            const float* prev_pts, float* next_pts, uint8_t* status, int npts,
            const ora_params* prm, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    for (int i = 0; i < npts; i++) status[i] = 1;
    lk_job* jobs = (lk_job*)malloc(sizeof(lk_job) * (size_t)nthreads);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int level = max_level; level >= 0; level--) {
        for (int t = 0; t < nthreads; t++) {
            lk_job* jb = &jobs[t];
            jb->prev = prev; jb->next = next; jb->level = level; jb->max_level = max_level;
            jb->prev_pts = prev_pts; jb->next_pts = next_pts; jb->status = status; jb->prm = prm;
            jb->begin = (int)((long long)npts * t / nthreads);
            jb->end = (int)((long long)npts * (t + 1) / nthreads);
        }
        if (nthreads == 1) {
            lk_level_range(&jobs[0]);
        } else {
            for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, lk_thread, &jobs[t]);
            for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
        }
    }
    free(jobs);
    free(th);
}

/* ---------------------------------------------------------------- A7: perspective fit - */
/* fdlibm __ieee754_hypot (glibc <= 2.34 dbl-64/e_hypot.c), which OpenCV's JacobiSVD calls
 * through ::hypot.  Restated so CPU and GPU builds round identically. */
static inline uint32_t hi_word(double d) { uint64_t u; memcpy(&u, &d, 8); return (uint32_t)(u >> 32); }
static inline uint32_t lo_word(double d) { uint64_t u; memcpy(&u, &d, 8); return (uint32_t)u; }
static inline double set_hi(double d, uint32_t hi)
{
    uint64_t u; memcpy(&u, &d, 8);
    u = ((uint64_t)hi << 32) | (u & 0xffffffffu);
    memcpy(&d, &u, 8);
    return d;
}

static double ora_hypot(double x, double y)
{
    double a, b, t1, t2, y1, y2, w;
    int32_t j, k, ha, hb;
    ha = (int32_t)(hi_word(x) & 0x7fffffff);
    hb = (int32_t)(hi_word(y) & 0x7fffffff);
    if (hb > ha) { a = y; b = x; j = ha; ha = hb; hb = j; }
    else { a = x; b = y; }
    a = set_hi(a, (uint32_t)ha);
    b = set_hi(b, (uint32_t)hb);
    if ((ha - hb) > 0x3c00000) return a + b;
    k = 0;
    if (ha > 0x5f300000) {
        if (ha >= 0x7ff00000) {
            w = a + b;
            if (((ha & 0xfffff) | lo_word(a)) == 0) w = a;
            if ((((uint32_t)hb ^ 0x7ff00000u) | lo_word(b)) == 0) w = b;
            return w;
        }
        ha -= 0x25800000; hb -= 0x25800000; k += 600;
        a = set_hi(a, (uint32_t)ha);
        b = set_hi(b, (uint32_t)hb);
    }
    if (hb < 0x20b00000) {
        if (hb <= 0x000fffff) {
            if ((hb | (int32_t)lo_word(b)) == 0) return a;
            t1 = set_hi(0.0, 0x7fd00000);
            b *= t1;
            a *= t1;
            k -= 1022;
        } else {
            ha += 0x25800000; hb += 0x25800000; k -= 600;
            a = set_hi(a, (uint32_t)ha);
            b = set_hi(b, (uint32_t)hb);
        }
    }
    w = a - b;
    if (w > b) {
        t1 = set_hi(0.0, (uint32_t)ha);
        t2 = a - t1;
        w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
    } else {
        a = a + a;
        y1 = set_hi(0.0, (uint32_t)hb);
        y2 = b - y1;
        t1 = set_hi(0.0, (uint32_t)(ha + 0x00100000));
        t2 = a - t1;
        w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
    }
    if (k != 0) {
        t1 = set_hi(1.0, hi_word(1.0) + (uint32_t)(k << 20));
        return t1 * w;
    }
    return w;
}

/* cv::RNG::next (core/include/opencv2/core/operations.hpp): multiply-with-carry. */
static inline uint32_t rng_next(uint64_t* state)
{
    *state = (uint64_t)(uint32_t)*state * 4164903690u + (uint32_t)(*state >> 32);
    return (uint32_t)*state;
}

/* The two readings of JacobiSVDImpl_ under CV_SSE2.  VBLAS<double>::givens (the Vt
 * rotations) computes every element exactly as the scalar loop, so it needs no restatement.  If
 * the column dot product and the rotated columns' norms went through VBLAS<double>::dot / givensx,
 * they would accumulate in two-lane SSE2 partials: dot over 4-element steps into two __m128d
 * accumulators, result ((s0 + s1)[0] + (s0 + s1)[1]) then a scalar tail; givensx over 2-element
 * steps, norms (lane 0 + lane 1) then a scalar tail.  g_svd_vblas = 1 selects that reading;
 * 0 (default, what the GPU restates) the scalar loops. */
static int g_svd_vblas = 0;
void ora_set_svd_vblas(int on) { g_svd_vblas = on != 0; }

static double vblas_dot(const double* a, const double* b, int n)
{
    if (n < 4) {
        double p = 0;
        for (int k = 0; k < n; k++) p += a[k] * b[k];
        return p;
    }
    double s00 = 0, s01 = 0, s10 = 0, s11 = 0;
    int k = 0;
    for (; k <= n - 4; k += 4) {
        s00 = s00 + a[k] * b[k];
        s01 = s01 + a[k + 1] * b[k + 1];
        s10 = s10 + a[k + 2] * b[k + 2];
        s11 = s11 + a[k + 3] * b[k + 3];
    }
    double p = (s00 + s10) + (s01 + s11);
    for (; k < n; k++) p += a[k] * b[k];
    return p;
}

/* lapack.cpp JacobiSVDImpl_<double>(At, W, Vt, m, n, n1=n, minval=DBL_MIN, eps=10*DBL_EPSILON).
 * At: n rows of length m (rows are columns of A); Vt: n x n. */
static void jacobi_svd(double* At, int m, int n, double* Wout, double* Vt)
{
    double W[16];
    int i, j, k, iter, max_iter = m > 30 ? m : 30;
    const double eps = DBL_EPSILON * 10, minval = DBL_MIN;
    double c, s, sd;
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
        W[i] = sd;
        for (k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (i = 0; i < n - 1; i++)
            for (j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                if (g_svd_vblas) p = vblas_dot(Ai, Aj, m);
                else
                    for (k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = ora_hypot(p, beta);
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                k = 0;
                if (g_svd_vblas) {   /* givensx: two lanes, then lane 0 + lane 1 */
                    double a0 = 0, a1 = 0, b0 = 0, b1 = 0;
                    for (; k <= m - 2; k += 2) {
                        double t00 = Ai[k] * c + Aj[k] * s, t01 = Ai[k + 1] * c + Aj[k + 1] * s;
                        double t10 = Aj[k] * c - Ai[k] * s, t11 = Aj[k + 1] * c - Ai[k + 1] * s;
                        Ai[k] = t00; Ai[k + 1] = t01; Aj[k] = t10; Aj[k + 1] = t11;
                        a0 = a0 + t00 * t00; a1 = a1 + t01 * t01;
                        b0 = b0 + t10 * t10; b1 = b1 + t11 * t11;
                    }
                    a = a0 + a1;
                    b = b0 + b1;
                }
                for (; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0; Aj[k] = t1;
                    a += t0 * t0; b += t1 * t1;
                }
                W[i] = a; W[j] = b;
                changed = 1;
                double *Vi = Vt + i * n, *Vj = Vt + j * n;
                for (k = 0; k < n; k++) {
                    double t0 = c * Vi[k] + s * Vj[k];
                    double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0; Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
        W[i] = sqrt(sd);
    }
    for (i = 0; i < n - 1; i++) {
        j = i;
        for (k = i + 1; k < n; k++) if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (k = 0; k < m; k++) { t = At[i * m + k]; At[i * m + k] = At[j * m + k]; At[j * m + k] = t; }
            for (k = 0; k < n; k++) { t = Vt[i * n + k]; Vt[i * n + k] = Vt[j * n + k]; Vt[j * n + k] = t; }
        }
    }
    for (i = 0; i < n; i++) Wout[i] = W[i];
    uint64_t rng = 0x12345678;
    for (i = 0; i < n; i++) {
        sd = i < n ? W[i] : 0;
        while (sd <= minval) {
            const double val0 = 1. / m;
            for (k = 0; k < m; k++) At[i * m + k] = (rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (iter = 0; iter < 2; iter++)
                for (j = 0; j < i; j++) {
                    sd = 0;
                    for (k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
                    double asum = 0;
                    for (k = 0; k < m; k++) {
                        double t = At[i * m + k] - sd * At[j * m + k];
                        At[i * m + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum != 0 ? 1 / asum : 0;
                    for (k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (k = 0; k < m; k++) { double t = At[i * m + k]; sd += t * t; }
            sd = sqrt(sd);
        }
        s = 1 / sd;
        for (k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

/* imgwarp.cpp getPerspectiveTransform + lapack.cpp solve(DECOMP_SVD) -> SVBkSb (nb == 1). */
void ora_get_perspective_transform(const float src[8], const float dst[8], double M[9])
{
    double a[8][8], bvec[8];
    for (int i = 0; i < 4; ++i) {
        float sx = src[2 * i], sy = src[2 * i + 1], dx = dst[2 * i], dy = dst[2 * i + 1];
        a[i][0] = a[i + 4][3] = sx;
        a[i][1] = a[i + 4][4] = sy;
        a[i][2] = a[i + 4][5] = 1;
        a[i][3] = a[i][4] = a[i][5] = a[i + 4][0] = a[i + 4][1] = a[i + 4][2] = 0;
        a[i][6] = (double)(-sx * dx);      /* float products (Point2f members) */
        a[i][7] = (double)(-sy * dx);
        a[i + 4][6] = (double)(-sx * dy);
        a[i + 4][7] = (double)(-sy * dy);
        bvec[i] = dx;
        bvec[i + 4] = dy;
    }
    const int m = 8, n = 8;
    double At[64], Vt[64], W[8], x[8];
    for (int i = 0; i < n; i++)
        for (int k = 0; k < m; k++) At[i * m + k] = a[k][i];   /* transpose(src, a) */
    jacobi_svd(At, m, n, W, Vt);
    double threshold = 0;
    for (int i = 0; i < n; i++) x[i] = 0;
    for (int i = 0; i < n; i++) threshold += W[i];
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < n; i++) {
        double wi = W[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < m; j++) s += At[i * m + j] * bvec[j];
        s *= wi;
        for (int j = 0; j < n; j++) x[j] = x[j] + s * Vt[i * n + j];
    }
    for (int i = 0; i < 8; i++) M[i] = x[i];
    M[8] = 1.;
}

/* lapack.cpp invert(DECOMP_LU), n == 3, CV_64F: cofactors / det3; det == 0 -> all zero. */
int ora_invert3x3(const double m[9], double out[9])
{
#define Md(i, j) m[(i) * 3 + (j)]
    double d = Md(0, 0) * (Md(1, 1) * Md(2, 2) - Md(1, 2) * Md(2, 1)) -
               Md(0, 1) * (Md(1, 0) * Md(2, 2) - Md(1, 2) * Md(2, 0)) +
               Md(0, 2) * (Md(1, 0) * Md(2, 1) - Md(1, 1) * Md(2, 0));
    if (d != 0.) {
        double t[9];
        d = 1. / d;
        t[0] = (Md(1, 1) * Md(2, 2) - Md(1, 2) * Md(2, 1)) * d;
        t[1] = (Md(0, 2) * Md(2, 1) - Md(0, 1) * Md(2, 2)) * d;
        t[2] = (Md(0, 1) * Md(1, 2) - Md(0, 2) * Md(1, 1)) * d;
        t[3] = (Md(1, 2) * Md(2, 0) - Md(1, 0) * Md(2, 2)) * d;
        t[4] = (Md(0, 0) * Md(2, 2) - Md(0, 2) * Md(2, 0)) * d;
        t[5] = (Md(0, 2) * Md(1, 0) - Md(0, 0) * Md(1, 2)) * d;
        t[6] = (Md(1, 0) * Md(2, 1) - Md(1, 1) * Md(2, 0)) * d;
        t[7] = (Md(0, 1) * Md(2, 0) - Md(0, 0) * Md(2, 1)) * d;
        t[8] = (Md(0, 0) * Md(1, 1) - Md(0, 1) * Md(1, 0)) * d;
        memcpy(out, t, sizeof(t));
        return 1;
    }
    for (int i = 0; i < 9; i++) out[i] = 0;
    return 0;
#undef Md
}

/* ---------------------------------------------------------------- A8: warpPerspective -- */
/* BilinearTab_i (imgwarp.cpp initInterTab2D(INTER_LINEAR, fixpt)): w = v*32768 saturated to
 * short, sum corrected to 32768; the (0,0) entry becomes {32767,0,0,1} (its correction
 * lands on tap 3, the max/min search reading still-zero entries of the next cell). */
static void bilinear_tab(int fx, int fy, int w[4])
{
    if (fx == 0 && fy == 0) { w[0] = 32767; w[1] = 0; w[2] = 0; w[3] = 1; return; }
    w[0] = (32 - fx) * (32 - fy) * 32;
    w[1] = fx * (32 - fy) * 32;
    w[2] = (32 - fx) * fy * 32;
    w[3] = fx * fy * 32;
}

static inline int sat_short(int v) { return v < -32768 ? -32768 : v > 32767 ? 32767 : v; }

typedef struct {
    const uint8_t* src; int w, h, sstride; const double* M; uint8_t* dst; int dstride;
    int y0, y1;
} warp_job;

/* warpPerspectiveInvoker (BLOCK_SZ 32: bh0 = min(16,H), bw0 = min(1024/bh0, W)) computes
 * per block row X0 = M0*xb + M1*y + M2 (xb = block origin), W = W0 + M6*x1,
 * W = W ? 32/W : 0, X = cvRound(clamp((X0 + M0*x1)*W)); then remapBilinear with
 * BORDER_CONSTANT 0.  y-blocking does not change any value; x-blocking does (xb). */
static void warp_rows(const warp_job* jb)
{
    const double* M = jb->M;
    int W = jb->w, H = jb->h;
    int bh0 = 16 < H ? 16 : H;
    int bw0 = 1024 / bh0 < W ? 1024 / bh0 : W;
    for (int y = jb->y0; y < jb->y1; y++) {
        uint8_t* d = jb->dst + (size_t)y * jb->dstride;
        for (int xb = 0; xb < W; xb += bw0) {
            int bw = W - xb < bw0 ? W - xb : bw0;
            double X0 = M[0] * xb + M[1] * y + M[2];
            double Y0 = M[3] * xb + M[4] * y + M[5];
            double W0 = M[6] * xb + M[7] * y + M[8];
            for (int x1 = 0; x1 < bw; x1++) {
                if (g_simd && x1 + 4 <= bw) {
                    /* four pixels at once when all their taps are inside (remapBilinear's vector
                     * loop over interior runs); otherwise this pixel takes the scalar code below */
                    const uint8_t* pp[4];
                    int wt4[4][4], k;
                    for (k = 0; k < 4; k++) {
                        double Wk = W0 + M[6] * (x1 + k);
                        Wk = Wk != 0 ? 32.0 / Wk : 0;
                        double fX = (X0 + M[0] * (x1 + k)) * Wk, fY = (Y0 + M[3] * (x1 + k)) * Wk;
                        fX = fX < (double)INT_MIN ? (double)INT_MIN : fX > (double)INT_MAX ? (double)INT_MAX : fX;
                        fY = fY < (double)INT_MIN ? (double)INT_MIN : fY > (double)INT_MAX ? (double)INT_MAX : fY;
                        int X = (int)lrint(fX), Y = (int)lrint(fY);
                        int sx = sat_short(X >> 5), sy = sat_short(Y >> 5);
                        if (!((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1))) break;
                        pp[k] = jb->src + (size_t)sy * jb->sstride + sx;
                        bilinear_tab(X & 31, Y & 31, wt4[k]);
                    }
                    if (k == 4) {
                        ora_sse2_bilinear4(pp, jb->sstride, (const int(*)[4])wt4, d + xb + x1);
                        x1 += 3;
                        continue;
                    }
                }
                double Wd = W0 + M[6] * x1;
                Wd = Wd != 0 ? 32.0 / Wd : 0;
                double fX = (X0 + M[0] * x1) * Wd;
                double fY = (Y0 + M[3] * x1) * Wd;
                fX = fX < (double)INT_MIN ? (double)INT_MIN : fX > (double)INT_MAX ? (double)INT_MAX : fX;
                fY = fY < (double)INT_MIN ? (double)INT_MIN : fY > (double)INT_MAX ? (double)INT_MAX : fY;
                int X = (int)lrint(fX), Y = (int)lrint(fY);
                int sx = sat_short(X >> 5), sy = sat_short(Y >> 5);
                int wt[4];
                bilinear_tab(X & 31, Y & 31, wt);
                int v;
                const uint8_t* S = jb->src;
                int st = jb->sstride;
                if ((unsigned)sx < (unsigned)(W - 1) && (unsigned)sy < (unsigned)(H - 1)) {
                    const uint8_t* p = S + (size_t)sy * st + sx;
                    v = p[0] * wt[0] + p[1] * wt[1] + p[st] * wt[2] + p[st + 1] * wt[3];
                    v = (v + (1 << 14)) >> 15;
                } else if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
                    v = 0;
                } else {
                    int x0 = sx, x1p = sx + 1, y0 = sy, y1p = sy + 1;
                    int in_x0 = (unsigned)x0 < (unsigned)W, in_x1 = (unsigned)x1p < (unsigned)W;
                    int in_y0 = (unsigned)y0 < (unsigned)H, in_y1 = (unsigned)y1p < (unsigned)H;
                    int v0 = in_x0 && in_y0 ? S[(size_t)y0 * st + x0] : 0;
                    int v1 = in_x1 && in_y0 ? S[(size_t)y0 * st + x1p] : 0;
                    int v2 = in_x0 && in_y1 ? S[(size_t)y1p * st + x0] : 0;
                    int v3 = in_x1 && in_y1 ? S[(size_t)y1p * st + x1p] : 0;
                    v = (v0 * wt[0] + v1 * wt[1] + v2 * wt[2] + v3 * wt[3] + (1 << 14)) >> 15;
                }
                d[xb + x1] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        }
    }
}

static void* warp_thread(void* arg)
{
    warp_rows((const warp_job*)arg);
    return NULL;
}

void ora_warp_perspective(const uint8_t* src, int w, int h, int sstride, const double M[9],
                          uint8_t* dst, int dstride, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    warp_job* jobs = (warp_job*)malloc(sizeof(warp_job) * (size_t)nthreads);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) {
        warp_job* jb = &jobs[t];
        jb->src = src; jb->w = w; jb->h = h; jb->sstride = sstride; jb->M = M;
        jb->dst = dst; jb->dstride = dstride;
        jb->y0 = (int)((long long)h * t / nthreads);
        jb->y1 = (int)((long long)h * (t + 1) / nthreads);
    }
    if (nthreads == 1) warp_rows(&jobs[0]);
    else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, warp_thread, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    free(jobs);
    free(th);
}

/* A9 + A10: absdiff then threshold(thresh, 255, THRESH_BINARY): dst = src > thresh ? 255 : 0 */
void ora_absdiff_threshold(const uint8_t* a, const uint8_t* b, int n, int thresh, uint8_t* mask)
{
    for (int i = 0; i < n; i++) {
        int d = a[i] > b[i] ? a[i] - b[i] : b[i] - a[i];
        mask[i] = d > thresh ? 255 : 0;
    }
}

/* ---------------------------------------------------------------- A2: grid ----------- */
int ora_grid_count(int w, int h, int ps)
{
    return ((w + ps - 1) / ps) * ((h + ps - 1) / ps);
}

void ora_grid_points(int w, int h, int ps, float* pts)
{
    int k = 0;
    for (int i = 0; i < w; i += ps)
        for (int j = 0; j < h; j += ps) {
            pts[2 * k] = (float)i;
            pts[2 * k + 1] = (float)j;
            k++;
        }
}

/* ---------------------------------------------------------------- RANSAC option -------- */
/* The product's MDX_FIT_RANSAC (not in the reference): see mdx_oracle.h. */
static uint64_t ransac_mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int ora_fit_ransac(const float* src, const float* dst, int n, int iters, double thresh, uint32_t seed, double H[9],
                   int* best_h)
{
    if (n < 4 || iters < 1) return -1;
    const double t2 = thresh * thresh;
    int bc = -1, bh = 0;
    double Hb[9] = {0};
    for (int h = 0; h < iters; h++) {
        int idx[4];
        for (int j = 0; j < 4; j++) {
            for (uint32_t c = 0;; c++) {
                const uint64_t x = ((uint64_t)seed << 32) | ((uint64_t)h << 20) | ((uint64_t)j << 16) | (uint64_t)(c & 0xffffu);
                const int v = (int)(ransac_mix64(x) % (uint64_t)n);
                int dup = 0;
                for (int q = 0; q < j; q++) dup = dup || idx[q] == v;
                if (!dup || c >= 0xffffu) {
                    idx[j] = v;
                    break;
                }
            }
        }
        float s4[8], d4[8];
        for (int j = 0; j < 4; j++) {
            s4[2 * j] = src[2 * idx[j]];
            s4[2 * j + 1] = src[2 * idx[j] + 1];
            d4[2 * j] = dst[2 * idx[j]];
            d4[2 * j + 1] = dst[2 * idx[j] + 1];
        }
        double Hh[9];
        ora_get_perspective_transform(s4, d4, Hh);
        int cnt = 0;
        for (int k = 0; k < n; k++) {
            const double sx = src[2 * k], sy = src[2 * k + 1], dx = dst[2 * k], dy = dst[2 * k + 1];
            const double nx = Hh[0] * sx + Hh[1] * sy + Hh[2];
            const double ny = Hh[3] * sx + Hh[4] * sy + Hh[5];
            const double dd = Hh[6] * sx + Hh[7] * sy + Hh[8];
            const double ex = nx - dx * dd, ey = ny - dy * dd;
            if (ex * ex + ey * ey <= t2 * (dd * dd)) cnt++;
        }
        if (cnt > bc) {
            bc = cnt;
            bh = h;
            memcpy(Hb, Hh, sizeof(Hb));
        }
    }
    memcpy(H, Hb, sizeof(Hb));
    if (best_h) *best_h = bh;
    return bc;
}

/* ---------------------------------------------------------------- whole path ---------- */
int ora_calculate_optical_flow(const uint8_t* img1, const uint8_t* img2, int w, int h, int stride,
                               int fmt, const ora_params* prm, int nthreads,
                               float* next_pts_out, uint8_t* status_out, double* vectors,
                               uint8_t* mask, double* H, double* Hinv, int* fit_status)
{
    uint8_t* g1 = (uint8_t*)malloc((size_t)w * h);
    uint8_t* g2 = (uint8_t*)malloc((size_t)w * h);
    ora_to_gray(img1, w, h, stride, fmt, g1);
    ora_to_gray(img2, w, h, stride, fmt, g2);

    int npts = ora_grid_count(w, h, prm->pixel_step);
    float* pts1 = (float*)malloc(sizeof(float) * 2 * (size_t)(npts > 0 ? npts : 1));
    float* pts2 = (float*)malloc(sizeof(float) * 2 * (size_t)(npts > 0 ? npts : 1));
    uint8_t* st = (uint8_t*)malloc((size_t)(npts > 0 ? npts : 1));
    ora_grid_points(w, h, prm->pixel_step, pts1);

    ora_pyramid P1, P2;
    int ml = ora_build_pyramid(g1, w, h, prm->win, prm->max_level, 1, &P1);
    ml = ora_build_pyramid(g2, w, h, prm->win, ml, 0, &P2);
    ora_lk(&P1, &P2, ml, pts1, pts2, st, npts, prm, nthreads);

    int num = 0;
    float src4[8], dst4[8];
    const int ransac = prm->fit_mode == ORA_FIT_RANSAC;
    float* srcs = ransac ? (float*)malloc(sizeof(float) * 2 * (size_t)(npts > 0 ? npts : 1)) : NULL;
    float* dsts = ransac ? (float*)malloc(sizeof(float) * 2 * (size_t)(npts > 0 ? npts : 1)) : NULL;
    for (int i = 0; i < npts; i++) {
        float sx = pts1[2 * i], sy = pts1[2 * i + 1];
        float ex = pts2[2 * i], ey = pts2[2 * i + 1];
        double* v = vectors ? vectors + 4 * (size_t)i : NULL;
        if (st[i]) {
            float xd = ex - sx, yd = ey - sy;
            if (fabs((double)fabsf(xd)) > prm->min_vector_size || fabs((double)fabsf(yd)) > prm->min_vector_size) {
                if (v) { v[0] = sx; v[1] = sy; v[2] = xd; v[3] = yd; }
                if (num < 4) {
                    src4[2 * num] = sx; src4[2 * num + 1] = sy;
                    dst4[2 * num] = ex; dst4[2 * num + 1] = ey;
                }
                if (ransac) {
                    srcs[2 * num] = sx; srcs[2 * num + 1] = sy;
                    dsts[2 * num] = ex; dsts[2 * num + 1] = ey;
                }
                num++;
            } else if (v) { v[0] = sx; v[1] = sy; v[2] = 0.0; v[3] = 0.0; }
        } else if (v) { v[0] = -1.0; v[1] = -1.0; v[2] = 0.0; v[3] = 0.0; }
    }
    if (next_pts_out) memcpy(next_pts_out, pts2, sizeof(float) * 2 * (size_t)npts);
    if (status_out) memcpy(status_out, st, (size_t)npts);

    double Hm[9] = {0}, Hi[9] = {0};
    int fs;
    if (num >= 4) {
        fs = 0;
        if (ransac)
            ora_fit_ransac(srcs, dsts, num, prm->ransac_iters, prm->ransac_thresh, prm->ransac_seed, Hm, NULL);
        else
            ora_get_perspective_transform(src4, dst4, Hm);
        ora_invert3x3(Hm, Hi);
        if (mask) {
            uint8_t* warped = (uint8_t*)malloc((size_t)w * h);
            ora_warp_perspective(g1, w, h, w, Hi, warped, w, nthreads);
            ora_absdiff_threshold(warped, g2, w * h, prm->thresh, mask);
            free(warped);
        }
    } else {
        fs = num == 0 ? 1 : 2;
        if (mask) memset(mask, 0, (size_t)w * h);
    }
    if (H) memcpy(H, Hm, sizeof(Hm));
    if (Hinv) memcpy(Hinv, Hi, sizeof(Hi));
    if (fit_status) *fit_status = fs;

    ora_free_pyramid(&P1);
    ora_free_pyramid(&P2);
    free(g1); free(g2); free(pts1); free(pts2); free(st); free(srcs); free(dsts);
    return num;
}

/* ------------------------------------------------- trajectory tracking - */
/* OpticalFlowCalculator::calculateOpticalFlowTrajectory (reference
 * common/src/optical_flow_calculator.cpp:133-257), restated.  Per consecutive pair j -> j+1
 * (:161): gray both frames (:166-167), pyramid of frame j with derivatives (:170), LK of the
 * current points (:172, flags 0: each pass starts from the point itself).  Per point (:178-236):
 *   status set: on the last pair (:183-206) the Vec4d (x, y, dx, dy) if |dx| or |dy| exceeds
 *     min_vector_size (num_vectors++), else (x, y, 0, 0), with (x, y) the point before the pass;
 *     then if 10 < x' < cols-10 and 10 < y' < rows-10 (:207-208) the point moves to x' and its
 *     trajectory grows by x' (:210-211), else it stays (:215);
 *   status clear: on the last pair (-1, -1, 0, 0) (:220-230); the point stays (:234).
 * traj[i] holds the init_traj_list entries (:143-158, :211), traj_len[i] their count; a
 * trajectory is reported by the reference iff traj_len == nimg (:244-249).  start_pts receives
 * the points entering the last pass (the Vec4d's buffer position).  Returns num_vectors. */
int ora_flow_trajectory(const uint8_t* const* imgs, int nimg, int w, int h, int stride, int fmt,
                        const ora_params* prm, int nthreads, float* traj, int* traj_len,
                        float* start_pts, double* vectors)
{
    const int npts = ora_grid_count(w, h, prm->pixel_step);
    const size_t np1 = (size_t)(npts > 0 ? npts : 1);
    float* cur = (float*)malloc(sizeof(float) * 2 * np1);
    float* nxt = (float*)malloc(sizeof(float) * 2 * np1);
    uint8_t* st = (uint8_t*)malloc(np1);
    int* len = (int*)malloc(sizeof(int) * np1);
    uint8_t* g1 = (uint8_t*)malloc((size_t)w * h);
    uint8_t* g2 = (uint8_t*)malloc((size_t)w * h);
    ora_grid_points(w, h, prm->pixel_step, cur);
    for (int i = 0; i < npts; i++) {
        len[i] = 1;
        if (traj) { traj[(size_t)i * nimg * 2] = cur[2 * i]; traj[(size_t)i * nimg * 2 + 1] = cur[2 * i + 1]; }
    }
    int num = 0;
    for (int j = 0; j + 1 < nimg; j++) {
        const int last = (j == nimg - 2);
        ora_to_gray(imgs[j], w, h, stride, fmt, g1);
        ora_to_gray(imgs[j + 1], w, h, stride, fmt, g2);
        ora_pyramid P1, P2;
        int ml = ora_build_pyramid(g1, w, h, prm->win, prm->max_level, 1, &P1);
        ml = ora_build_pyramid(g2, w, h, prm->win, ml, 0, &P2);
        ora_lk(&P1, &P2, ml, cur, nxt, st, npts, prm, nthreads);
        ora_free_pyramid(&P1);
        ora_free_pyramid(&P2);
        for (int i = 0; i < npts; i++) {
            const float sx = cur[2 * i], sy = cur[2 * i + 1];
            double* v = (last && vectors) ? vectors + 4 * (size_t)i : NULL;
            if (last && start_pts) { start_pts[2 * i] = sx; start_pts[2 * i + 1] = sy; }
            if (st[i]) {
                const float ex = nxt[2 * i], ey = nxt[2 * i + 1];
                if (last) {
                    const float xd = ex - sx, yd = ey - sy;
                    if (fabs((double)fabsf(xd)) > prm->min_vector_size || fabs((double)fabsf(yd)) > prm->min_vector_size) {
                        if (v) { v[0] = sx; v[1] = sy; v[2] = xd; v[3] = yd; }
                        num++;
                    } else if (v) { v[0] = sx; v[1] = sy; v[2] = 0.0; v[3] = 0.0; }
                }
                if (ex > 10.0f && ey > 10.0f && ex < (float)(w - 10) && ey < (float)(h - 10)) {
                    cur[2 * i] = ex; cur[2 * i + 1] = ey;
                    if (traj) {
                        traj[((size_t)i * nimg + len[i]) * 2] = ex;
                        traj[((size_t)i * nimg + len[i]) * 2 + 1] = ey;
                    }
                    len[i]++;
                }
            } else if (v) { v[0] = -1.0; v[1] = -1.0; v[2] = 0.0; v[3] = 0.0; }
        }
    }
    if (traj_len) memcpy(traj_len, len, sizeof(int) * (size_t)npts);
    free(cur); free(nxt); free(st); free(len); free(g1); free(g2);
    return num;
}

/* ----------------------------------------- trajectory subspace RANSAC - */
/* glibc rand() (random_r TYPE_3: x[i] = x[i-3] + x[i-31], output x >> 1, after the 310-value
 * warm-up srand does), the generator the reference draws its hypotheses from
 * (outlier_detector.cpp:17 srand(time(NULL)), :226 rand() % cols).  Restated so runs are
 * reproducible from a seed; pinned against this machine's libc in tests/test_subspace.py. */
void ora_srand(ora_rand_state* s, uint32_t seed)
{
    int32_t r[34];
    r[0] = (int32_t)(seed ? seed : 1);
    for (int i = 1; i < 31; i++) {
        const int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int64_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    for (int i = 0; i < 34; i++) s->x[i] = (uint32_t)r[i];
    s->i = 34;
    for (int k = 0; k < 310; k++) (void)ora_rand(s);
}

int ora_rand(ora_rand_state* s)
{
    /* x[i] = x[i-31] + x[i-3] over a ring of 34 */
    const int i = s->i;
    const uint32_t v = s->x[(i - 31) % 34] + s->x[(i - 3) % 34];
    s->x[i % 34] = v;
    s->i = i + 1 >= 34 * 1024 ? (i + 1) % 34 + 34 : i + 1;
    return (int)(v >> 1);
}

/* Householder QR of the n x d sample (double, column-major, LAPACK dgeqr2-style reflectors with
 * beta = v'v) and the last n - d columns of Q = H_0 ... H_{d-1}: an orthonormal basis of the
 * complement of the first d left singular vectors' span, i.e. Pnd = I - U_d U_d' = Q2 Q2'
 * (outlier_detector.cpp:272-283; with a rank-deficient sample -- repeated indices -- the
 * completion is implementation-defined there too).  Shared verbatim-in-order with the GPU
 * kernel so both round identically.  q2: n x (n-d) column-major. */
static void subspace_basis(double* A, int n, int d, double* q2)
{
    double V[ORA_MAX_SUBSPACE * ORA_MAX_SUBSPACE];   /* reflector k in column k (rows k..n-1) */
    double beta[ORA_MAX_SUBSPACE];
    for (int k = 0; k < d; k++) {
        double nrm2 = 0.0;
        for (int r = k; r < n; r++) nrm2 = nrm2 + A[k * n + r] * A[k * n + r];
        const double nrm = sqrt(nrm2);
        const double x0 = A[k * n + k];
        const double alpha = x0 >= 0.0 ? -nrm : nrm;
        for (int r = k; r < n; r++) V[k * n + r] = A[k * n + r];
        V[k * n + k] = x0 - alpha;
        double b = 0.0;
        for (int r = k; r < n; r++) b = b + V[k * n + r] * V[k * n + r];
        beta[k] = b;
        if (b == 0.0) continue;
        for (int c = k; c < d; c++) {            /* A[k:, c] -= 2 v (v'a) / b */
            double dot = 0.0;
            for (int r = k; r < n; r++) dot = dot + V[k * n + r] * A[c * n + r];
            const double f = 2.0 * dot / b;
            for (int r = k; r < n; r++) A[c * n + r] = A[c * n + r] - f * V[k * n + r];
        }
    }
    for (int j = d; j < n; j++) {
        double* q = q2 + (size_t)(j - d) * n;
        for (int r = 0; r < n; r++) q[r] = r == j ? 1.0 : 0.0;
        for (int k = d - 1; k >= 0; k--) {
            if (beta[k] == 0.0) continue;
            double dot = 0.0;
            for (int r = k; r < n; r++) dot = dot + V[k * n + r] * q[r];
            const double f = 2.0 * dot / beta[k];
            for (int r = k; r < n; r++) q[r] = q[r] - f * V[k * n + r];
        }
    }
}

/* residual of one mean-subtracted trajectory column x (float, n): sum over the complement basis
 * of (q' x)^2, in double, fixed order */
static double subspace_residual(const double* q2, int n, int m, const float* x)
{
    double res = 0.0;
    for (int j = 0; j < m; j++) {
        double p = 0.0;
        for (int r = 0; r < n; r++) p = p + q2[(size_t)j * n + r] * (double)x[r];
        res = res + p * p;
    }
    return res;
}

/* Float mode (ORA_SUBSPACE_F32): the reference's float arithmetic shape (outlier_detector.cpp:
 * 243-290, every Eigen::MatrixXf/VectorXf quantity a float): the sample's basis from the same
 * Householder statement in float; Pnd formed explicitly as I - sum_idx u u' with the sum taken
 * idx by idx (:272-282: Pnd = Pnd + M, then Identity - Pnd); residual = |x' (Pnd x)| as the two
 * products of :286 (y = Pnd x with sequential b, then x'y with sequential a), float throughout.
 * Eigen's own JacobiSVD rotations and its vectorised GEMM order are not restated (Eigen is not in
 * the reference tree to pin against): this mode reproduces the precision, not Eigen's exact
 * bits, and the GPU kernel follows it operation for operation.  P: n x n row-major. */
static void subspace_pnd_f32(float* A, int n, int d, float* P)
{
    float V[ORA_MAX_SUBSPACE * ORA_MAX_SUBSPACE], beta[ORA_MAX_SUBSPACE], q[ORA_MAX_SUBSPACE];
    for (int k = 0; k < d; k++) {
        float nrm2 = 0.0f;
        for (int r = k; r < n; r++) nrm2 = nrm2 + A[k * n + r] * A[k * n + r];
        const float nrm = sqrtf(nrm2);
        const float x0 = A[k * n + k];
        const float alpha = x0 >= 0.0f ? -nrm : nrm;
        for (int r = k; r < n; r++) V[k * n + r] = A[k * n + r];
        V[k * n + k] = x0 - alpha;
        float b = 0.0f;
        for (int r = k; r < n; r++) b = b + V[k * n + r] * V[k * n + r];
        beta[k] = b;
        if (b == 0.0f) continue;
        for (int c = k; c < d; c++) {
            float dot = 0.0f;
            for (int r = k; r < n; r++) dot = dot + V[k * n + r] * A[c * n + r];
            const float f = 2.0f * dot / b;
            for (int r = k; r < n; r++) A[c * n + r] = A[c * n + r] - f * V[k * n + r];
        }
    }
    for (int e = 0; e < n * n; e++) P[e] = 0.0f;
    for (int j = 0; j < d; j++) {                  /* u_j = Q e_j, then Pnd = Pnd + u_j u_j' */
        for (int r = 0; r < n; r++) q[r] = r == j ? 1.0f : 0.0f;
        for (int k = d - 1; k >= 0; k--) {
            if (beta[k] == 0.0f) continue;
            float dot = 0.0f;
            for (int r = k; r < n; r++) dot = dot + V[k * n + r] * q[r];
            const float f = 2.0f * dot / beta[k];
            for (int r = k; r < n; r++) q[r] = q[r] - f * V[k * n + r];
        }
        for (int a = 0; a < n; a++)
            for (int b = 0; b < n; b++) P[a * n + b] = P[a * n + b] + q[a] * q[b];
    }
    for (int a = 0; a < n; a++)
        for (int b = 0; b < n; b++) P[a * n + b] = (a == b ? 1.0f : 0.0f) - P[a * n + b];
}

static float subspace_residual_f32(const float* P, int n, const float* x)
{
    float res = 0.0f;
    for (int a = 0; a < n; a++) {
        float y = 0.0f;
        for (int b = 0; b < n; b++) y = y + P[a * n + b] * x[b];
        res = res + x[a] * y;
    }
    return fabsf(res);
}

/* meanSubtract (outlier_detector.cpp:200-221): float sums of row 0 / row 1 in column order,
 * double mean, float constants; even rows minus the x mean, odd rows = y mean minus the row (the
 * reference's y flip).  data: N columns of n floats (column i = trajectory i). */
void ora_subspace_data(const float* traj, int N, int T, float* data)
{
    const int n = 2 * T;
    float xs = 0.0f, ys = 0.0f;
    for (int i = 0; i < N; i++) {
        xs = i ? xs + traj[(size_t)i * T * 2] : traj[0];
        ys = i ? ys + traj[(size_t)i * T * 2 + 1] : traj[1];
    }
    double xm = (double)xs, ym = (double)ys;
    xm /= N;
    ym /= N;
    const float xc = (float)xm, yc = (float)ym;
    for (int i = 0; i < N; i++)
        for (int r = 0; r < n; r++) {
            const float v = traj[(size_t)i * T * 2 + r];
            data[(size_t)i * n + r] = (r % 2 == 0) ? v - xc : yc - v;
        }
}

int ora_fit_subspace(const float* traj, int N, int T, int num_motions, double sigma, ora_rand_state* rng,
                     int* columns, uint8_t* is_outlier, double* residuals)
{
    return ora_fit_subspace_ex(traj, N, T, num_motions, sigma, rng, columns, is_outlier, residuals, ORA_SUBSPACE_F64);
}

int ora_fit_subspace_ex(const float* traj, int N, int T, int num_motions, double sigma, ora_rand_state* rng,
                        int* columns, uint8_t* is_outlier, double* residuals, int precision)
{
    const int n = 2 * T, d = 4 * num_motions;
    if (N <= 0 || d <= 0 || d > n || n > ORA_MAX_SUBSPACE || n - d == 10) return -1;
    float* data = (float*)malloc(sizeof(float) * (size_t)N * n);
    double* best_res = (double*)malloc(sizeof(double) * (size_t)N);
    double* q2 = (double*)malloc(sizeof(double) * (size_t)n * (n - d > 0 ? n - d : 1));
    double A[ORA_MAX_SUBSPACE * ORA_MAX_SUBSPACE];
    float Af[ORA_MAX_SUBSPACE * ORA_MAX_SUBSPACE], P[ORA_MAX_SUBSPACE * ORA_MAX_SUBSPACE];
    int cols[ORA_MAX_SUBSPACE];
    const int f32 = precision == ORA_SUBSPACE_F32;
    ora_subspace_data(traj, N, T, data);
    const double inlier_thr = (double)(n - d) * sigma * sigma;
    int max_points = 0, have = 0;
    for (int it = 0; it < 50; it++) {
        for (int k = 0; k < d; k++) {
            cols[k] = ora_rand(rng) % N;
            for (int r = 0; r < n; r++) {
                A[k * n + r] = (double)data[(size_t)cols[k] * n + r];
                Af[k * n + r] = data[(size_t)cols[k] * n + r];
            }
        }
        if (f32) subspace_pnd_f32(Af, n, d, P);
        else subspace_basis(A, n, d, q2);
#define ORA_RES(i) (f32 ? (double)subspace_residual_f32(P, n, data + (size_t)(i) * n) \
                        : subspace_residual(q2, n, n - d, data + (size_t)(i) * n))
        int np = 0;
        for (int i = 0; i < N; i++)
            if (ORA_RES(i) < inlier_thr) np++;
        if (np > max_points) {
            max_points = np;
            have = 1;
            for (int k = 0; k < d; k++) columns[k] = cols[k];
            for (int i = 0; i < N; i++) best_res[i] = ORA_RES(i);
        }
#undef ORA_RES
    }
    /* chi-square 99% table (:19-30), indexed by n - d */
    static const double p99[10] = {0.0, 0.020, 0.115, 0.297, 0.554, 0.872, 1.239, 1.646, 2.088, 2.558};
    double thr = 0.2;
    if (n - d < 11 && n - d > 0) {
        if (n - d == 10) { free(data); free(best_res); free(q2); return -1; }   /* vector::at(10) throws */
        thr = sigma * sigma * p99[n - d];
    }
    int nout = 0;
    for (int i = 0; i < N; i++) {
        const int o = have && best_res[i] > thr;
        if (is_outlier) is_outlier[i] = (uint8_t)o;
        if (residuals) residuals[i] = have ? best_res[i] : 0.0;
        nout += o;
    }
    free(data); free(best_res); free(q2);
    return have ? nout : 0;
}
