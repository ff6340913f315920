/*
 * mdx_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This header and oracle/mdx_oracle.c are the parity ORACLE for the MI355X path in
 * motion_detection_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product library never links it.
 *
 * What it restates: OpticalFlowCalculator::calculateOpticalFlow
 * (reference common/src/optical_flow_calculator.cpp:30-130) and the OpenCV calls it makes.
 * OpenCV is a third-party dependency that is NOT vendored in /root/reference and NOT
 * installed here.  The semantics restated are those of OpenCV 2.4.8 (ROS Indigo's
 * opencv2 package; the reference uses 2.4-only APIs) on an x86-64 SSE2 build:
 *   cvtColor(CV_BGR2GRAY)            color.cpp    RGB2Gray<uchar>            (call site :50-51)
 *   buildOpticalFlowPyramid          lkpyramid.cpp + pyramids.cpp pyrDown_   (:67)
 *   calcOpticalFlowPyrLK             lkpyramid.cpp LKTrackerInvoker, SSE2 order (:71)
 *   getPerspectiveTransform          imgwarp.cpp + lapack.cpp JacobiSVD/SVBkSb (:120)
 *   warpPerspective                  imgwarp.cpp warpPerspectiveInvoker + remapBilinear (:124)
 *   absdiff / threshold(190,255,BINARY)                                       (:125,:127)
 *
 * Parity status: UNPINNED against a real OpenCV 2.4 binary -- the reference ships no
 * tests, fixtures or golden vectors and OpenCV cannot be built or
 * imported here.  The oracle is pinned instead by known-answer tests and by an
 * independent numpy restatement (tests/golden/make_golden.py); see DESIGN.md §3.
 */
#ifndef MDX_ORACLE_H_
#define MDX_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_MAX_LEVELS 16

enum { ORA_FMT_GRAY8 = 0, ORA_FMT_RGB8 = 1, ORA_FMT_BGR8 = 2 };

typedef struct {
    int win;             /* window side, reference 40 (optical_flow_calculator.cpp:41) */
    int max_level;       /* reference MAX_LEVEL 5 (:40) */
    int max_iters;       /* TermCriteria count 10 (:44) */
    double eps;          /* TermCriteria eps 0.03 (:44) */
    float min_eig;       /* minEigThreshold 1e-3 (:71) */
    int thresh;          /* threshold 190 (:127) */
    int pixel_step;      /* ROS param pixel_step (motion_detection_node.cpp:29) */
    double min_vector_size; /* ROS param min_vector_size, default 1.0 (node.cpp:44) */
    /* NOT in the reference: the product's MDX_FIT_RANSAC option (include/mdx.h), restated below */
    int fit_mode;            /* ORA_FIT_FIRST4 (default, the reference) or ORA_FIT_RANSAC */
    int ransac_iters;        /* default 128 */
    double ransac_thresh;    /* default 3.0 px */
    uint32_t ransac_seed;    /* default 20141105 */
} ora_params;
#define ORA_FIT_FIRST4 0
#define ORA_FIT_RANSAC 2

void ora_default_params(ora_params* p);

/* One pyramid: per level a padded u8 image and (optionally) padded interleaved Ix,Iy int16. */
typedef struct {
    int nlevels;                 /* attained maxLevel + 1 */
    int pad;                     /* = win */
    int w[ORA_MAX_LEVELS], h[ORA_MAX_LEVELS];
    uint8_t* img[ORA_MAX_LEVELS];    /* (h+2pad) x (w+2pad), pitch w+2pad, REFLECT_101 border */
    int16_t* deriv[ORA_MAX_LEVELS];  /* (h+2pad) x (w+2pad) x 2, CONSTANT-0 border; NULL if none */
} ora_pyramid;

int  ora_reflect101(int p, int len);
void ora_to_gray(const uint8_t* src, int w, int h, int stride, int fmt, uint8_t* dst);
void ora_pyrdown(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh, int dstride);
void ora_scharr(const uint8_t* src, int w, int h, int sstride, int16_t* dst, int dstride);
int  ora_build_pyramid(const uint8_t* gray, int w, int h, int win, int max_level, int with_deriv, ora_pyramid* out);
void ora_free_pyramid(ora_pyramid* p);

/* calcOpticalFlowPyrLK over a prev pyramid (with derivs) and next pyramid; nthreads>=1. */
void ora_lk(const ora_pyramid* prev, const ora_pyramid* next, int max_level,
            const float* prev_pts, float* next_pts, uint8_t* status, int npts,
            const ora_params* prm, int nthreads);

/* 1: JacobiSVDImpl_ with SSE2 VBLAS dot/givensx partial sums (see mdx_oracle.c); 0: scalar (default) */
void ora_set_svd_vblas(int on);
/* 1: the LK window / iteration sums and the warp's interior bilinear run the SSE2-intrinsics
 * restatement (mdx_oracle_sse2.c, OpenCV 2.4's x86 4-lane order, bit-identical results); 0: the
 * scalar loops.  The timed CPU baseline uses 1. */
void ora_set_simd(int on);
/* mdx_oracle_sse2.c (internal) */
void ora_sse2_window_sums(const uint8_t* I, int stepI, const int16_t* D, int dstep, int win, int iw00, int iw01,
                          int iw10, int iw11, int16_t* Iwin, int16_t* dIwin, float qA11[4], float qA12[4],
                          float qA22[4]);
void ora_sse2_iter_sums(const uint8_t* J, int stepJ, const int16_t* Iwin, const int16_t* dIwin, int win, int iw00,
                        int iw01, int iw10, int iw11, float q1[4], float q2[4]);
void ora_sse2_bilinear4(const uint8_t* const p[4], int stride, const int w[4][4], uint8_t out[4]);
void ora_get_perspective_transform(const float src[8], const float dst[8], double M[9]);
int  ora_invert3x3(const double M[9], double Minv[9]);
void ora_warp_perspective(const uint8_t* src, int w, int h, int sstride, const double M[9],
                          uint8_t* dst, int dstride, int nthreads);
void ora_absdiff_threshold(const uint8_t* a, const uint8_t* b, int n, int thresh, uint8_t* mask);

/* Deterministic RANSAC homography (the product's MDX_FIT_RANSAC; no reference counterpart, so
 * parity with the reference is N/A -- this pins the GPU kernels k_ransac_*): over the n accepted
 * vectors (src, dst) in x-major order, `iters` hypotheses; hypothesis h draws 4 distinct indices
 * idx_j = splitmix64(seed << 32 | h << 20 | j << 16 | retry) % n and fits them with
 * ora_get_perspective_transform (the reference's 4-point solver); a vector is an inlier of H iff
 * ex^2 + ey^2 <= t^2 w^2 with w = H6 sx + H7 sy + H8, ex = (H0 sx + H1 sy + H2) - dx w, ey likewise
 * (FP64, this evaluation order, t = thresh); the first hypothesis with the most inliers is H.
 * Returns its inlier count (-1 when n < 4: H untouched); *best_h = its index if non-NULL. */
int ora_fit_ransac(const float* src, const float* dst, int n, int iters, double thresh, uint32_t seed, double H[9],
                   int* best_h);

/* Grid of the reference (optical_flow_calculator.cpp:56-64): x-major order. */
int  ora_grid_count(int w, int h, int pixel_step);
void ora_grid_points(int w, int h, int pixel_step, float* pts);

/*
 * Whole hot path.  Outputs (any may be NULL):
 *   next_pts  2*npts floats  (LK output points, x-major grid order)
 *   status    npts bytes
 *   vectors   4*npts doubles (x, y, dx, dy) / (x, y, 0, 0) / (-1, -1, 0, 0)  (:78-117)
 *   mask      w*h bytes      (only written when num_vectors >= 4, else zero-filled)
 *   H         9 doubles      (getPerspectiveTransform result; zero when no fit)
 *   Hinv      9 doubles      (matrix actually used by the warp: inverse or all-zero)
 * Returns num_vectors.  *fit_status: 0 = fitted, 1 = num_vectors==0 (no mask, :118),
 * 2 = 1..3 vectors (reference UB at :120; defined here as "no fit, zero mask").
 */
int ora_calculate_optical_flow(const uint8_t* img1, const uint8_t* img2, int w, int h, int stride,
                               int fmt, const ora_params* prm, int nthreads,
                               float* next_pts, uint8_t* status, double* vectors,
                               uint8_t* mask, double* H, double* Hinv, int* fit_status);

/*
 * Trajectory tracking (OpticalFlowCalculator::calculateOpticalFlowTrajectory,
 * optical_flow_calculator.cpp:133-257) over nimg >= 2 frames.  Outputs (any may be NULL):
 *   traj       npts*nimg*2 floats: point i's positions, entry 0 = its grid point, then every
 *              accepted move (only the first traj_len[i] entries are written)
 *   traj_len   npts ints (the reference keeps a trajectory iff traj_len == nimg)
 *   start_pts  2*npts floats: the points entering the last pair
 *   vectors    4*npts doubles: the last pair's Vec4d per point
 * Returns num_vectors (last pair only).
 */
int ora_flow_trajectory(const uint8_t* const* imgs, int nimg, int w, int h, int stride, int fmt,
                        const ora_params* prm, int nthreads, float* traj, int* traj_len,
                        float* start_pts, double* vectors);

/*
 * Trajectory subspace RANSAC (OutlierDetector::fitSubspace, outlier_detector.cpp:236-331).
 * traj: N trajectories of T points (x, y) (the complete ones of ora_flow_trajectory), n = 2T,
 * d = 4*num_motions (d <= n <= ORA_MAX_SUBSPACE).  50 hypotheses of d columns drawn with
 * ora_rand() % N; per hypothesis the residual of every trajectory against the complement of the
 * sample's span; the first hypothesis with the most residuals < (n-d) sigma^2 wins.  Outputs:
 * columns [d] (the winner's sample: the trajectories fitSubspace returns), is_outlier [N]
 * (winner residual > sigma^2 * chi2_99[n-d], or 0.2 when n-d is outside 1..10; the reference
 * reports trajectory[i][T-2] for each), residuals [N] (double).  Returns the outlier count
 * (0 and columns untouched when no hypothesis has an inlier), -1 on bad arguments.
 * Arithmetic: the reference's float meanSubtract, then double Householder QR + residuals (the
 * reference uses Eigen's float JacobiSVD; see DESIGN.md for the parity statement).
 */
#define ORA_MAX_SUBSPACE 32
typedef struct { uint32_t x[34]; int i; } ora_rand_state;
void ora_srand(ora_rand_state* s, uint32_t seed);
int  ora_rand(ora_rand_state* s);
void ora_subspace_data(const float* traj, int N, int T, float* data);
int  ora_fit_subspace(const float* traj, int N, int T, int num_motions, double sigma, ora_rand_state* rng,
                      int* columns, uint8_t* is_outlier, double* residuals);
/* precision: ORA_SUBSPACE_F64 (the default above: double basis and residuals) or ORA_SUBSPACE_F32
 * (the reference's float arithmetic shape, explicit Pnd; see subspace_pnd_f32) */
#define ORA_SUBSPACE_F64 0
#define ORA_SUBSPACE_F32 1
int  ora_fit_subspace_ex(const float* traj, int N, int T, int num_motions, double sigma, ora_rand_state* rng,
                         int* columns, uint8_t* is_outlier, double* residuals, int precision);

/* Synthetic-frame generator spec is in the product (motion_detection_amd/csrc/synth.cpp);
 * the oracle does not need one. */

#ifdef __cplusplus
}
#endif
#endif
