/*
 * mdx.h -- C-ABI of the MI355X-native motion-detection hot path.
 *
 * Drop-in boundary for the reference's in-process seam
 *   int OpticalFlowCalculator::calculateOpticalFlow(const cv::Mat& image1,
 *        const cv::Mat& image2, cv::Mat& optical_flow_vectors, int pixel_step,
 *        cv::Mat& comp, double min_vector_size)
 * declared at reference common/include/motion_detection/optical_flow_calculator.h:19 and
 * defined at common/src/optical_flow_calculator.cpp:30-130, called from
 * MotionDetectionNode::runOpticalFlow (ros/src/motion_detection_node.cpp:76-92, call :82).
 *
 * Plain C types only: pointers + sizes, no torch / OpenCV / HIP types in signatures.
 * Errors are integer codes; no C++ exception crosses this boundary.  A context owns one
 * HIP stream on one device; it is not thread-safe, but different contexts may be driven
 * concurrently from different host threads (one context per camera stream / GPU).
 */
#ifndef MDX_H_
#define MDX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDX_ABI_VERSION 4    /* 2: mdx_params.call_pipelining, mdx_input_ready.
                                3: mdx_lk_fallbacks; mdx_params grew ransac_iters, ransac_thresh and
                                   ransac_seed (16 more bytes: a caller built against ABI 2 passes a
                                   shorter struct); mdx_sync / mdx_device_sync return MDX_OK after an
                                   LK hand-off that gave up and was recomputed (ABI 2: MDX_EHIP).
                                4: mdx_abi_version and mdx_params_size: check both at start-up --
                                   a mismatch means the header and the library differ. */

/* Return codes */
#define MDX_OK           0
#define MDX_EINVAL      -1   /* bad argument (size, format, unsupported parameter) */
#define MDX_EHIP        -2   /* HIP runtime error (message in mdx_last_error) */
#define MDX_ENOMEM      -3   /* device allocation failed */
#define MDX_EDEGENERATE  1   /* success, but fewer than 4 accepted vectors: no fit, mask zeroed.
                                num_vectors == 0 is the reference's "no mask" branch
                                (optical_flow_calculator.cpp:118); 1..3 is reference UB (:120,
                                reads past src_points) and is defined here as "no fit". */

/* Pixel formats of the input frames (sensor_msgs/Image encodings the node accepts). */
#define MDX_FMT_GRAY8 0      /* mono8: cv_bridge rgb8 replication then BGR2GRAY == identity */
#define MDX_FMT_RGB8  1      /* rgb8 (node.cpp:271), BGR2GRAY weights land swapped (:50) */
#define MDX_FMT_BGR8  2      /* bgr8: cv_bridge converts to rgb8 first, same swapped weights */

/* Global-motion fit used for the back-warp. */
#define MDX_FIT_FIRST4   0   /* reference: getPerspectiveTransform on the first 4 accepted
                                vectors in x-major grid order (:120) */
#define MDX_FIT_EXTERNAL 1   /* caller supplies H (forward, frame1 -> frame2) per pair */
#define MDX_FIT_RANSAC   2   /* NOT in the reference (parity with it N/A): deterministic RANSAC over
                                all accepted vectors -- mdx_params.ransac_iters hypotheses, each the
                                reference's own 4-point getPerspectiveTransform on 4 accepted vectors
                                drawn by a counter-based generator (splitmix64 of ransac_seed,
                                hypothesis, draw); the hypothesis with the most inliers (reprojection
                                error <= ransac_thresh px; first on ties) is H, without a refit.
                                Restated in oracle/ and bit-exact there. */

/* mdx_fit_subspace arithmetic (see its comment below). */
#define MDX_SUBSPACE_F64 0   /* double Householder basis and residuals (stable; the default) */
#define MDX_SUBSPACE_F32 1   /* the reference's float arithmetic shape: Eigen::MatrixXf
                                (outlier_detector.cpp:243-290), Pnd formed explicitly in float */

typedef struct {
    int    win;              /* LK window side; reference hard-codes 40 (:41). Only 40 is supported. */
    int    max_level;        /* reference MAX_LEVEL = 5 (:40) */
    int    max_iters;        /* TermCriteria count = 10 (:44) */
    double eps;              /* TermCriteria epsilon = 0.03 (:44) */
    float  min_eig;          /* minEigThreshold = 1e-3 (:71) */
    int    thresh;           /* threshold(comp, comp, 190, 255, BINARY) (:127) */
    int    pixel_step;       /* ROS param pixel_step (node.cpp:29; 10 in bag.launch:27) */
    double min_vector_size;  /* ROS param min_vector_size, default 1.0 (node.cpp:44) */
    int    fit_mode;         /* MDX_FIT_FIRST4 (default), MDX_FIT_EXTERNAL or MDX_FIT_RANSAC */
    int    subspace_precision; /* mdx_fit_subspace arithmetic: MDX_SUBSPACE_F64 (default) or _F32 */
    int    call_pipelining;  /* 0 (default) or 1: consecutive device-entry calls overlap (below) */
    int    ransac_iters;     /* MDX_FIT_RANSAC hypotheses, 1..1024 (default 128) */
    double ransac_thresh;    /* MDX_FIT_RANSAC inlier reprojection error, px (default 3.0, as
                                OpenCV findHomography's ransacReprojThreshold) */
    uint32_t ransac_seed;    /* MDX_FIT_RANSAC generator seed (default 20141105) */
} mdx_params;

/*
 * Call pipelining (mdx_params.call_pipelining = 1).  The pyramid workspace holds two halves used by
 * alternate device-entry calls (mdx_flow_warp_diff_batch_dev, mdx_band_flow_dev), and a call's
 * front end (gray, pyramids) runs on the context's second stream, behind the previous call's
 * flow-independent LK work, so it overlaps that call's last LK level and its fit/warp.  The front
 * end then does NOT wait for earlier work on the context stream: the call's input frames must be
 * in HBM when it is made (mdx_memcpy_h2d returns after the copy), or the caller names the event
 * after which they are, with mdx_input_ready.  Outputs are unaffected; results are identical with
 * and without pipelining.  The workspace doubles its pyramid slabs while the flag is set.
 */

typedef struct mdx_ctx mdx_ctx;

/* Fill params with the reference's constants. */
void mdx_default_params(mdx_params* p);

/* The ABI version and sizeof(mdx_params) the library was built with.  A caller compares them with
 * MDX_ABI_VERSION and its own sizeof(mdx_params) before the first mdx_create: the struct is passed
 * by pointer, so a library newer than the caller's header would read past a shorter struct. */
int mdx_abi_version(void);
size_t mdx_params_size(void);

/* Number of grid points for a frame: ceil(w/ps) * ceil(h/ps) (:56-64, x-major order:
 * point k = ix*ny + iy sits at (ix*ps, iy*ps)). */
int mdx_grid_count(int w, int h, int pixel_step);

/* Create a context on HIP device `device`.  max_w/max_h/max_batch size the device
 * workspace (pyramids, derivatives, scratch) so that the per-frame path never allocates.
 * Returns NULL on failure; mdx_create_error() then holds the reason. */
mdx_ctx* mdx_create(int device, int max_w, int max_h, int max_batch, const mdx_params* p);
const char* mdx_create_error(void);
int mdx_destroy(mdx_ctx* ctx);
const char* mdx_last_error(const mdx_ctx* ctx);
int mdx_set_params(mdx_ctx* ctx, const mdx_params* p);
int mdx_get_params(const mdx_ctx* ctx, mdx_params* p);

/* The context's HIP stream (hipStream_t as void*) and device id; for interop only. */
void* mdx_stream(mdx_ctx* ctx);
int mdx_device(const mdx_ctx* ctx);
/* PCI bus id ("0000:xx:yy.z") of the context's device, so multi-GPU records can show which
 * distinct devices the ranks ran on. */
int mdx_device_pci(const mdx_ctx* ctx, char* buf, int len);
/* Build provenance: "src_sha256=<sha256 of the library's sources> arch=gfx950", compiled in by
 * csrc/Makefile.  tests/test_abi.py checks it against the sources in the tree. */
const char* mdx_build_info(void);
/* Wait for the context's work (and collect the LK fallback counts below). */
int mdx_sync(mdx_ctx* ctx);
/* hipDeviceSynchronize on the context's device (all streams); the same collection. */
int mdx_device_sync(mdx_ctx* ctx);
/* LK level dataflow fallbacks since mdx_create, as of the last mdx_sync / mdx_device_sync:
 *   counts[0]  group waits that gave up (a group of level l waits, bounded, for its pair's level
 *              l+1 groups, whose launch may not be dispatched in time: the device is preempted,
 *              shared, or serializes kernels as a counter-collecting profiler does)
 *   counts[1]  gate waits that gave up (the same, before a level's launch)
 *   counts[2]  levels recomputed
 * A level whose wait gave up is abandoned and recomputed in sequence within the same call, after
 * its coarser level, together with every finer level: the outputs are exact either way (the
 * reference call always returns a result, optical_flow_calculator.cpp:71).  The counts are
 * statistics, not errors. */
int mdx_lk_fallbacks(const mdx_ctx* ctx, long long counts[3]);
/* Name the input frames' producer: the next device-entry call (mdx_flow_warp_diff_batch_dev,
 * mdx_band_flow_dev, mdx_warp_diff_dev) makes its first stage wait for `hip_event` (a hipEvent_t
 * the caller recorded on its own stream after writing the frames) before reading them.  One-shot:
 * consumed by that call.  Needed with call pipelining whenever the frames are produced
 * asynchronously (a zero-copy producer on another stream); harmless without it. */
int mdx_input_ready(mdx_ctx* ctx, void* hip_event);

/*
 * Synchronous host-buffer entry: the direct replacement of calculateOpticalFlow.
 *   img1, img2  w x h frames, row pitch `stride` bytes, format `fmt`.
 *   next_pts    [2*npts] float  LK output positions (x-major grid order)        or NULL
 *   status      [npts]   uint8  LK status                                       or NULL
 *   vectors     [4*npts] double the reference's Vec4d per grid point:
 *               (x, y, dx, dy) accepted / (x, y, 0, 0) tracked / (-1, -1, 0, 0) lost
 *               (:78-117; stored densely per grid point)     or NULL
 *   mask        [w*h]    uint8  thresholded |warp(gray1) - gray2| (comp, :122-127) or NULL
 *   H           [9]      double perspective transform (first-4 fit or external)  or NULL
 *   H_external  [9]      double forward H when fit_mode == MDX_FIT_EXTERNAL, else NULL
 *   num_vectors          number of accepted vectors (the reference's return value)
 * Returns MDX_OK, MDX_EDEGENERATE, or a negative error.
 */
int mdx_flow_warp_diff(mdx_ctx* ctx, const uint8_t* img1, const uint8_t* img2,
                       int w, int h, int stride, int fmt,
                       float* next_pts, uint8_t* status, double* vectors,
                       uint8_t* mask, double* H, const double* H_external, int* num_vectors);

/*
 * Asynchronous batched device entry (zero-copy; everything stays in HBM).  Pair i reads
 * d_img1 + i*frame_stride and d_img2 + i*frame_stride.  Outputs (device pointers, each may
 * be NULL except where noted):
 *   d_next_pts  [batch][npts][2] float     d_status [batch][npts] uint8
 *   d_vectors   [batch][npts][4] double    d_mask   [batch][h][w] uint8
 *   d_H         [batch][9] double          d_num_vectors [batch] int32
 *   d_H_external[batch][9] double (input; required iff fit_mode == MDX_FIT_EXTERNAL)
 * Work is enqueued on the context stream; call mdx_sync (or sync the stream) before use.
 */
int mdx_flow_warp_diff_batch_dev(mdx_ctx* ctx, int batch,
                                 const uint8_t* d_img1, const uint8_t* d_img2,
                                 int w, int h, int stride, size_t frame_stride, int fmt,
                                 float* d_next_pts, uint8_t* d_status, double* d_vectors,
                                 uint8_t* d_mask, double* d_H, const double* d_H_external,
                                 int* d_num_vectors);

/*
 * The fused back-warp + absdiff + threshold kernel alone (rows A8-A10): for each pair,
 * mask = (|warpPerspective(gray1, H) - gray2| > thresh) * 255 with the reference's
 * warpPerspective arithmetic (inverse of H, FP64 coordinates, 1/32 px, BORDER_CONSTANT 0).
 * d_gray1/d_gray2: [batch] frames of w x h gray8, row pitch `stride`, frame pitch
 * `frame_stride`.  d_H: [batch][9] forward transforms (device).  d_mask: [batch][h][w].
 */
int mdx_warp_diff_dev(mdx_ctx* ctx, int batch, const uint8_t* d_gray1, const uint8_t* d_gray2,
                      int w, int h, int stride, size_t frame_stride,
                      const double* d_H, uint8_t* d_mask);

/*
 * Row-tiled path: one frame pair split by rows over several GPUs (8K RGB
 * over 8 GPUs).  No reference interface corresponds -- the reference runs the whole frame in one
 * calculateOpticalFlow call (optical_flow_calculator.cpp:30-130); this splits that call at its
 * only global step, the first-four-accepted getPerspectiveTransform input (:118-120).
 *
 * Rank r owns the destination rows [y0, y1) (the bands partition [0, h)) and the grid points
 * whose row y = gy*pixel_step lies in that band.  Per pair:
 *   1. every rank: mdx_band_flow_dev -- rows A1-A6 for the band's points.  next_pts / status /
 *      vectors are full-frame arrays ([npts]...); only the band's entries are written.  d_cand
 *      receives the band's mdx_band_cand record.
 *   2. the caller all-gathers the ranks' records (any transport: RCCL all_gather over xGMI, or
 *      host memory) into one device array, in any order.
 *   3. every rank: mdx_band_fit_warp_dev -- the first four accepted points overall are the four
 *      smallest indices over all records; the fit, its inverse and num_vectors are then exactly
 *      the full path's.  Writes mask rows [y0, y1) to d_mask_band (row pitch w) and, when
 *      non-NULL, d_H[9] and d_num_vectors.
 * Both entries are asynchronous on the context stream.  Step 3 reads the pyramids of the
 * context's latest mdx_band_flow_dev call, which must be of the same frame pair (several bands of
 * one pair may run step 1 one after another first), and converts from that call's d_img1 the
 * frame-1 rows its warp reads beyond the band, so d_img1 must still hold frame 1.  Any other entry
 * that rebuilds the context's pyramids in between (a pair or trajectory call) voids them: step 3
 * then returns MDX_EINVAL instead of warping another pair's frames.  fit_mode must be
 * MDX_FIT_FIRST4.  With call pipelining, consecutive band calls alternate the two pyramid halves;
 * step 3 reads (and then releases) only the latest call's half, the other half having been
 * released by its own call once its classification was queued.
 */
typedef struct mdx_band_cand {
    int32_t count;     /* accepted vectors (status && |d| > min_vector_size) in the band */
    int32_t n;         /* min(count, 4) */
    int32_t idx[4];    /* x-major grid index k = gx*ny + gy of the band's first n accepted points */
    float src[8];      /* their grid positions (x, y) */
    float dst[8];      /* their tracked positions next_pts[k] */
    int32_t pad_[2];
} mdx_band_cand;       /* 96 bytes */

int mdx_band_flow_dev(mdx_ctx* ctx, const uint8_t* d_img1, const uint8_t* d_img2,
                      int w, int h, int stride, int fmt, int y0, int y1,
                      float* d_next_pts, uint8_t* d_status, double* d_vectors,
                      mdx_band_cand* d_cand);
int mdx_band_fit_warp_dev(mdx_ctx* ctx, int nrec, const mdx_band_cand* d_cands, int y0, int y1,
                          uint8_t* d_mask_band, double* d_H, int* d_num_vectors);

/*
 * Trajectory tracking: replaces OpticalFlowCalculator::calculateOpticalFlowTrajectory
 * (optical_flow_calculator.h:20-21, optical_flow_calculator.cpp:133-257), the node's live caller
 * (motion_detection_node.cpp:94-110 over 2*num_motions+1 frames, :241).  Synchronous.
 *   imgs        nimg >= 2 host frames, each w x h, row pitch `stride`, format `fmt`.
 * The pixel_step grid is tracked through the nimg-1 consecutive pairs; each pass starts from the
 * points the previous one left (a point moves only when tracked and strictly inside the 10-px
 * border, :207-216).  Outputs (any may be NULL; npts = mdx_grid_count(w, h, pixel_step)):
 *   traj        [npts][nimg][2] float  point i's positions: its grid point, then each accepted
 *               move (entries past traj_len[i] are unspecified)
 *   traj_len    [npts] int32           the reference's init_traj_list[i].size(); it reports the
 *               trajectory iff traj_len[i] == nimg (:244-249)
 *   start_pts   [npts][2] float        the points entering the last pass (where the reference
 *               stores each Vec4d: optical_flow_vectors.at<Vec4d>((int)y, (int)x))
 *   vectors     [npts][4] double       the last pass's Vec4d per point (:183-206, :220-230)
 *   num_vectors                        the reference's return value (last pass only)
 * Grows the context's pyramid workspace to nimg - 1 slots (one per pair) when needed.
 */
int mdx_flow_trajectory(mdx_ctx* ctx, const uint8_t* const* imgs, int nimg, int w, int h, int stride,
                        int fmt, float* traj, int32_t* traj_len, float* start_pts, double* vectors,
                        int* num_vectors);

/*
 * One host block for a trajectory call's outputs.  With traj, start_pts, vectors and traj_len at
 * these byte offsets of one block (e.g. from mdx_host_alloc), mdx_flow_trajectory and
 * mdx_ring_trajectory read all four back with one copy instead of four.  offsets[] = {traj,
 * start_pts, vectors, traj_len}; returns the block size in bytes.  Any other placement works too.
 * Outputs that are all in page-locked memory (mdx_host_alloc) are written by the chained launch
 * itself through their device mapping, with no readback copy.  Either way traj's entries past
 * traj_len[i] are 0.
 */
size_t mdx_trajectory_layout(int npts, int nimg, size_t offsets[4]);

/*
 * Resident frame ring for the live chain: the node's raw_images_ deque (motion_detection_node.h:82,
 * filled at node.cpp:248-261), whose every frame the reference re-converts, re-uploads and
 * re-pyramids on each callback (:266-287, then optical_flow_calculator.cpp:166-170).  Here a frame
 * crosses PCIe and is pyramided (gray, padded levels, Scharr planes) once, when it enters the ring,
 * and stays in HBM while it is in it.
 *   mdx_ring_push        append a frame (w x h, row pitch `stride`, format `fmt`), then drop frames
 *                        from the front until at most `keep` remain (the deque's size after the
 *                        reference's push / pop at :248-261).  A frame of another size empties the
 *                        ring first.  Returns the number of frames held, or a negative error.
 *   mdx_ring_trajectory  calculateOpticalFlowTrajectory over the frames held (>= 2), outputs exactly
 *                        as mdx_flow_trajectory's (nimg = the ring size).
 *   mdx_ring_reset       empty the ring.
 * mdx_ring_push only queues the upload and the pyramid on the context's stream: the frame's host
 * memory (page-locked memory is read by DMA after the call returns) must stay unchanged until the
 * next mdx_ring_trajectory or mdx_sync returns.
 */
int mdx_ring_push(mdx_ctx* ctx, const uint8_t* img, int w, int h, int stride, int fmt, int keep);
int mdx_ring_trajectory(mdx_ctx* ctx, float* traj, int32_t* traj_len, float* start_pts, double* vectors,
                        int* num_vectors);
int mdx_ring_reset(mdx_ctx* ctx);

/*
 * Trajectory subspace RANSAC: replaces OutlierDetector::fitSubspace
 * (common/include/motion_detection/outlier_detector.h:21, outlier_detector.cpp:236-331), called
 * by the node on the complete trajectories (motion_detection_node.cpp:348).
 *   traj        [ntraj][traj_len][2] float host trajectories (mdx_flow_trajectory's complete ones)
 *   rng         the caller's generator: the reference draws 50 x 4*num_motions samples per call
 *               from one srand(time(NULL)) stream (outlier_detector.cpp:17, :226); seed it with
 *               mdx_srand (glibc rand() restated: the same stream for the same seed)
 * Outputs (any may be NULL):
 *   columns     [4*num_motions] the winning sample's trajectory indices (the return value of
 *               fitSubspace is those trajectories); -1 when no hypothesis had an inlier
 *   is_outlier  [ntraj] 1 where the winner's residual exceeds sigma^2 * chi2_99[n-d]
 *   residuals   [ntraj] double, the winner's residuals
 *   outlier_points [n_outliers][2] float: each outlier's second-to-last point (:322), in order
 * Arithmetic: the reference's float meanSubtract, then by mdx_params.subspace_precision:
 * MDX_SUBSPACE_F64 -- double Householder QR of each sample and double residuals; MDX_SUBSPACE_F32
 * -- the reference's float shape (float basis, explicit float Pnd = I - sum u u', float x'(Pnd x)).
 * The reference itself runs Eigen's float JacobiSVD, which neither mode restates rotation for
 * rotation.
 */
typedef struct mdx_rand_state { uint32_t x[34]; int32_t pos; } mdx_rand_state;
void mdx_srand(mdx_rand_state* st, uint32_t seed);
int  mdx_rand(mdx_rand_state* st);
int  mdx_fit_subspace(mdx_ctx* ctx, const float* traj, int ntraj, int traj_len, int num_motions, double sigma,
                      mdx_rand_state* rng, int* columns, uint8_t* is_outlier, double* residuals,
                      float* outlier_points, int* n_outliers);

/* Page-locked host memory for frames and outputs (e.g. the node's rgb8 staging buffer and its
 * trajectory outputs): copies between it and the device run as DMA at full link rate, while a
 * pageable buffer is staged by the runtime through bounce buffers.  Any entry taking host pointers
 * accepts either.  mdx_host_alloc returns NULL on failure. */
void* mdx_host_alloc(size_t bytes);
int mdx_host_free(void* p);

/* Device memory helpers so hosts without a HIP toolchain (ctypes, cgo, JNI) can stage
 * buffers: allocation on the context's device, copies ordered on its stream. */
void* mdx_dev_alloc(mdx_ctx* ctx, size_t bytes);
int mdx_dev_free(mdx_ctx* ctx, void* p);
int mdx_memcpy_h2d(mdx_ctx* ctx, void* dst, const void* src, size_t bytes);
int mdx_memcpy_d2h(mdx_ctx* ctx, void* dst, const void* src, size_t bytes);

/* Per-stage device time from HIP events recorded on the ctx stream around each stage.
 * mdx_enable_timing(ctx, 1) (re)starts recording; every later pipeline call records one
 * event set (up to 256 calls).  mdx_stage_ms returns the SUM over the recorded calls, in
 * milliseconds, of stage: 0 gray+pad, 1 pyramids, 2 Scharr, 3 LK, 4 classify+fit,
 * 5 warp+diff, 6 whole call; mdx_timing_calls returns how many calls were recorded. */
int mdx_enable_timing(mdx_ctx* ctx, int on);
int mdx_timing_calls(const mdx_ctx* ctx);
int mdx_stage_ms(mdx_ctx* ctx, int stage, float* ms);

/* Test hook: copy an internal buffer of the last call to the host (0: per-(pair, level,
 * point) float4 LK gradient sums; 1: per-level LK trace when MDX_LK_DEBUG=1 at create). */
int mdx_debug_copy(mdx_ctx* ctx, int which, void* dst, size_t bytes);
/* Test hook: d_out[i] = 32 / d_in[i] through the projective warp's FP64 division (device buffers,
 * queued on the context stream); equal to IEEE division for |d_in[i]| in [2^-100, 2^100]. */
int mdx_debug_div32(mdx_ctx* ctx, const double* d_in, double* d_out, int n);

/* Measurement probe, no reference counterpart: the memory ceiling of k_warp_diff's access mix.
 * d_mask[i] = |d_a[i] - d_b[i]| > thresh ? 255 : 0 over n bytes (n a multiple of 16, pointers
 * 16-byte aligned): the same 3 B/px (read two frames, write the mask) as a linear streaming pass,
 * 16 B per lane, non-temporal.  Queued on the context's stream and timed as its warp_diff stage
 * (mdx_stage_ms) when timing is on; bench.py reports its rate as roofline.copy_ceiling. */
int mdx_probe_stream3_dev(mdx_ctx* ctx, size_t n, const uint8_t* d_a, const uint8_t* d_b, uint8_t* d_mask,
                          int thresh);

/*
 * Synthetic frame-pair generator used by the benchmark and tests (host, deterministic,
 * byte-identical on every x86-64 host).  Spec in DESIGN.md §5: blurred value noise +
 * rectangles; frame 2 = frame 1 under the affine H_true (0.5 deg rotation about the
 * centre, scale 1.01, translation (3.2, -1.7)) + one moving patch (+8, +5) + +-2 LSB noise.
 * channels = 1 (gray) or 3 (rgb8).  H_true (9 doubles, forward) is written if non-NULL.
 */
int mdx_synth_pair(uint64_t seed, int w, int h, int channels, uint8_t* img1, uint8_t* img2,
                   double* H_true, int nthreads);

#ifdef __cplusplus
}
#endif
#endif /* MDX_H_ */
