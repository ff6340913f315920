// mdx_internal.h -- shared between the HIP kernels (mdx_kernels.hip) and the host API
// (mdx_api.cpp).  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mdx.h"

namespace mdx {

constexpr int kMaxLevels = 8;
// LK debug buffer (MDX_LK_DEBUG=1): after the per-point records, the traced point's iterations
// (kMaxLevels * 64 float4), then per level and persistent wave of k_lk_iter its {start, end}
// s_memrealtime stamps (100 MHz), for the wave-occupancy profile (scripts/lk_tail.py)
constexpr int kLkDbgStampOff = kMaxLevels * 64 + 64;
constexpr int kLkDbgWaves = 16384;
constexpr int kWin = 40;     // LK window side (reference optical_flow_calculator.cpp:41)
constexpr int kPad = 40;     // border rows/cols every pyramid level carries (= win)
constexpr int kXOff = 64;    // left margin of a level row: the core starts 64-B aligned

// One pyramid level inside a per-pair slab.  Images are u8; derivatives are uint32 words
// holding (Ix int16 | Iy int16 << 16), the little-endian image of OpenCV's interleaved
// CV_16SC2 derivative Mat.  Both use the same pitch (elements) and origin.
struct Level {
    int w, h;              // core size
    int pitch;             // elements per row (>= kXOff + w + kPad, multiple of 64)
    int rows;              // kPad + h + kPad
    long long img_off;     // byte offset of the level's padded buffer in the u8 slab
    long long der_off;     // word offset of the level's padded buffer in the deriv slab
    __host__ __device__ long long core() const { return (long long)kPad * pitch + kXOff; }
};

struct Geometry {
    int nlev;                // attained maxLevel + 1
    Level lv[kMaxLevels];
    long long img_bytes;     // bytes of one pyramid slab (all levels)
    long long der_words;     // words of one derivative slab (all levels)
};

// Per-pair result of the classify + fit stage.
struct PairFit {
    double H[9];      // getPerspectiveTransform output (or external H); zero when no fit
    double Hinv[9];   // matrix warpPerspective actually samples with (inverse or all-zero)
    int num_vectors;  // accepted vectors (reference return value)
    int fit_status;   // 0 fitted, 1 no vectors, 2 fewer than 4 vectors
    int src_y0, src_y1;   // row bands (k_band_fit): frame-1 rows the band's warp reads
};

// Residue-class planes of LK v2 (mdx_lk.hip): per level, one plane set per class of
// (P_x mod 2^L, P_y mod 2^L) present in the grid.  Each class holds one row-major UH x PW array of
// 8-B (D, C) pairs: D (uint32, Ix | Iy << 16) and C (int32, 256 - 512*I: the J-chain bias, see
// mdx_lk.hip).
struct ClassLevel {
    int nrx, nry;            // residue classes per axis
    int UH, PW;              // plane rows (h + 79), plane width in elements (multiple of 4)
    long long off;           // byte offset of this level inside a pair's class slab
    long long class_bytes;   // UH * PW * 8
    int nxp;                 // length of the padded class-grouped column order (multiple of G)
    int ord_off;             // offset of this level's order tables in LkArgs::ord
    int G;                   // points per LK group (4 or 8)
    int UW;                  // union columns per group (64, 128, 256 or 512)
    int vlo, vhi;            // plane rows the planned grid rows' windows reach (k_lk_class range)
    // A sums per row strip (k_lk_A_rows): the level's grid rows, in class order, cut into strips of
    // at most kAStripRows rows of one y-class whose windows start every `asp` plane rows; 0: the
    // per-group k_lk_A instead (spacing not uniform, or below 5 rows: too many windows overlap)
    int asp;
    int nstrip;              // strips (table at LkArgs::ord + strip_off: (first row index, rows) pairs)
    int strip_off;
};
constexpr int kAStripRows = 16;

// (G, UW) shapes of the LK level kernels (mdx_lk.hip instantiates these; the host plan picks the
// smallest UW >= a level's union span among the shapes of its G)
#define LK_SHAPES LK_CASE(4, 48) LK_CASE(4, 56) LK_CASE(4, 64) LK_CASE(4, 72) LK_CASE(4, 80) LK_CASE(4, 96) \
    LK_CASE(4, 128) LK_CASE(8, 80) LK_CASE(8, 112) LK_CASE(8, 128) LK_CASE(8, 256) LK_CASE(8, 512)
constexpr int kLkUW4[] = {48, 56, 64, 72, 80, 96, 128};
constexpr int kLkUW8[] = {80, 112, 128, 256, 512};

struct ClassPlan {
    ClassLevel lv[kMaxLevels];
    long long bytes_per_pair;
    int nch;                 // 0: some group's union is wider than 512 columns (single-kernel LK)
};

struct LkClassArgs {
    Geometry g;
    ClassPlan plan;
    const int16_t* rlist;    // [level][axis][128] class index -> residue
    int level;
};

struct LkArgs {
    const uint8_t* pyr1;     // prev pyramid slabs
    const uint8_t* pyr2;     // next pyramid slabs
    const uint32_t* der;     // prev derivative slabs
    Geometry g;
    int maxl;                // attained max level used by LK
    int npts, ny, pixel_step;
    int nyg;                 // LK v2: grid rows in the group order (ny, or a row band's count)
    int max_iters;
    float min_eig;
    double eps2;
    float* next_pts;         // [batch][npts][2]
    float* carry;            // LK v2: per level l > 0 a [batch][npts][2] array (at carry + l *
                             // carry_lstride) of the points level l leaves for level l-1; level 0
                             // writes next_pts.  null: next_pts carries them (levels in sequence only)
    long long carry_lstride; // floats between two levels' carried-point arrays
    uint8_t* status;         // [batch][npts]
    ClassPlan plan;          // LK v2 only
    const int16_t* cmap;     // [level][axis][128] residue -> class index
    const int16_t* rlist;    // [level][axis][128] class index -> residue
    const int16_t* ord;      // per level: nxp padded grid columns (-1 = empty), then ny grid rows,
                             // both grouped by residue class (ClassLevel::ord_off)
    const float* prev_pts;   // k_lk only: [batch][npts][2] start points (trajectories); null = the grid
    int max_sub;             // > 0: at most this many pairs per LK sub-batch (MDX_LK_SUB, tests)
    int* done;               // LK v2 dataflow: [level][done_stride] groups retired per pair, each
                             // counter on its own 128-B line (kCtrPad ints); null:
                             // the level launches run one after another
    int done_stride;
    int dep_groups;          // > 0: groups per pair of the coarser level, which a group waits for
    int dep_points;          // 1: per-point dataflow -- a group waits only for its own points' coarser
                             // level results (pflags), not for the whole pair's level (small batches)
    int* pflags;             // per-point dataflow: [level][batch][npts] epoch of each point's last
                             // retirement at that level (this sub-batch's first pair)
    long long pf_lstride;    // ints between two levels of pflags
    int epoch;               // this call's epoch (> every earlier call's)
    int pflow_force;         // 1: per-point dataflow even where the per-pair form applies (MDX_LK_PFLOW)
    int* err;                // dataflow statistics, read and cleared at the context's sync points:
                             // [0] group waits and [1] gate waits that gave up, [2] levels recomputed
    int* lflags;             // dataflow: the call's per-level flags (kLkFlag* below, zeroed with
                             // `done`); null: no dataflow
    int redo;                // 1: this launch is level `level`'s conditional recompute (kLkFlag*)
    int spin_max;            // dataflow wait bound in s_sleep(8) polls; < 0: fault injection (every
                             // wait counts as timed out at once; tests)
    int flow_cap;            // dataflow: percent of the resident waves one iteration launch takes
    float4* dbg;             // optional [batch][nlev][npts] (npx, npy, iters, status) at level end
    int dbg_pt;              // point whose per-iteration values are appended after dbg (pair 0)
};

// LK counters (queue heads per level and XCD, dataflow retire counts per level and pair): one per
// 128-B line.  Packed, a line held the counters of several levels (or pairs) that concurrently
// running launches update and poll, and the dataflow ran 1.4-3x slower wherever the batch did not
// fill whole lines (8, 16, 24, 40 pairs) -- the concurrent launches contending on shared lines.
constexpr int kCtrPad = 32;
// default dataflow wait bound: s_sleep(8) polls, ~0.1 s
constexpr int kLkSpinDefault = 1 << 19;
// Dataflow fallback flags of one call (LkArgs::lflags, ints kCtrPad apart, zeroed with the retire
// counters): level l's give-ups (a group wait or the gate before it gave up: the level's results may
// be wrong), whether level l was recomputed (so every finer level must be too), and the queue heads
// of the recompute launches ([level][XCD]).
constexpr int kLkFlagGiveup = 0;
constexpr int kLkFlagRedone = kMaxLevels;
constexpr int kLkFlagQueue = 2 * kMaxLevels;
constexpr int kLkFlagInts = kLkFlagQueue + 8 * kMaxLevels;
// persistent waves of a recompute launch: cheap when it exits at once (the common case), and a
// recompute of the finest level at 1080p x 32 still takes only tens of ms
#ifndef MDX_LK_REDO_WAVES
#define MDX_LK_REDO_WAVES 512
#endif
constexpr int kLkRedoWaves = MDX_LK_REDO_WAVES;

// Core rows [lo, hi) of one pyramid level (row-band mode: what a band's LK reads)
struct RowSpan {
    int lo, hi;
};

// Launchers (mdx_kernels.hip).  All enqueue on `s`.
// fsel: 0 both frames of every pair, 1 the first frame only, 2 the second frame only
hipError_t launch_gray_pad(hipStream_t s, int batch, const uint8_t* in1, const uint8_t* in2, int w, int h,
                           int stride, long long frame_stride, int fmt, uint8_t* pyr1, uint8_t* pyr2,
                           const Geometry& g, int fsel = 0);
// gray + pad of level 0 and pyrDown to level 1 in one pass (k_front; launch_gray_pad when nlev == 1);
// launch_pyr_levels then builds levels 2 .. nlev-1 (k_front in level mode, one launch per level)
// rows (may be null = all): [nlev] core rows wanted per level; only the bands covering them are built
hipError_t launch_front(hipStream_t s, int batch, const uint8_t* in1, const uint8_t* in2, int w, int h, int stride,
                        long long frame_stride, int fmt, uint8_t* pyr1, uint8_t* pyr2, const Geometry& g,
                        int fsel = 0, const RowSpan* rows = nullptr);
hipError_t launch_pyr_levels(hipStream_t s, int batch, uint8_t* pyr1, uint8_t* pyr2, const Geometry& g, int fsel = 0,
                             const RowSpan* rows = nullptr);
// padded rows [prow0, prow1) of the level's derivative planes (default: all)
// every level's Scharr planes, whole levels, one launch
hipError_t launch_scharr_levels(hipStream_t s, int batch, const uint8_t* pyr1, uint32_t* der, const Geometry& g);
hipError_t launch_scharr(hipStream_t s, int batch, const uint8_t* pyr1, uint32_t* der, const Geometry& g, int level,
                         int prow0 = 0, int prow1 = -1);
hipError_t launch_lk(hipStream_t s, int batch, const LkArgs& a);

// Trajectory passes in one launch (k_lk chain mode): pass j of point p tracks frame j -> j+1 from
// the point pass j-1 left, waiting for it through flag[p]; the pass bookkeeping of
// calculateOpticalFlowTrajectory (k_traj_update's) is done by the point's own wave.
constexpr int kMaxTrajImgs = 16;
struct TrajChain {
    const uint8_t* pyr[kMaxTrajImgs];    // padded pyramid slab of each frame
    const uint32_t* der[kMaxTrajImgs];   // its Scharr planes
    int nimg, w, h;
    float* cur;                          // [npts][2] current points (atomic hand-off between passes)
    float* traj;                         // [npts][nimg][2]
    int* tlen;                           // [npts]
    int* flag;                           // [npts] passes done (zeroed by k_traj_init)
    double* vectors;                     // [npts][4] Vec4d of the last pass, or null
    float* start_pts;                    // [npts][2] start points of the last pass, or null
    int* num;                            // [0] num_vectors, [1] hand-off waits that timed out
    double mvs;                          // min_vector_size
    // the caller's page-locked outputs, device-mapped (or null): the passes write traj, traj_len,
    // start_pts and vectors straight into them, and no readback copy follows
    float* htraj;
    int* htlen;
    float* hstart;
    double* hvec;
};
// ppw: points per wave (1: 64 lanes per point, 2: 32, 4: 16)
hipError_t launch_lk_chain(hipStream_t s, const LkArgs& a, const TrajChain& t, int ppw);
// Trajectory subspace RANSAC (fitSubspace): mean-subtracted data, nhyp hypotheses of d columns
// (cols: [nhyp][d]), winner's residuals / outlier flags; best[0] = winner or -1.  Scratch: data
// [N][2T] floats + 2 (the means), qbuf [nhyp][2T][2T-d] doubles (MDX_SUBSPACE_F32: [nhyp][2T][2T] floats), counts [nhyp].
hipError_t launch_subspace(hipStream_t s, const float* traj, int N, int T, int d, const int* cols, int nhyp,
                           double sigma, float* data, double* qbuf, int* counts, double* residuals,
                           uint8_t* is_outlier, int* best, int precision);
// Trajectory tracking (calculateOpticalFlowTrajectory): grid init and the per-pass point update.
hipError_t launch_traj_init(hipStream_t s, int npts, int ny, int pixel_step, int nimg, float* cur, float* traj,
                            int* tlen, int* num, int* flag = nullptr);
hipError_t launch_traj_update(hipStream_t s, int npts, const float* next_pts, const uint8_t* status, float* cur,
                              float* traj, int* tlen, int nimg, int w, int h, int last, double min_vector_size,
                              double* vectors, float* start_pts, int* num);
// Ab: [nlev][batch][npts] per-point (A11, A12, A22, 1/D); qctr: [batch][kMaxLevels][8] (x kCtrPad) queue
// heads.  aux (may be null): second stream for the flow-independent class / A kernels; ev: kMaxLevels
// + 1 events (no timing) used to order the two streams.  prev_ready (may be null): recorded by the
// caller once the first frames' pyramids exist; the aux work waits on it instead of on everything
// enqueued on s so far (the second frames' pyramids may still be in flight on s).
// Dataflow (s2 and flow_ev[2] non-null, done: kMaxLevels x batch + kLkFlagInts counters): the level launches alternate
// between s and s2, so level L-1 starts in level L's tail; its groups wait for their pair's level-L
// groups (done counters).  Used when every XCD's work range holds two or more whole pairs (batch a
// multiple of 8, at least 16) and pairs' next_pts do not share 128-B lines (npts % 16 == 0).
// lvl_done (may be null: calls do not overlap): [kMaxLevels] events, re-recorded after each level's
// iteration launch; the aux stream waits for the previous call's before rewriting that level's
// class planes, A sums and queue heads (call pipelining lets the aux stream run a call ahead).
// Cross-call overlap (call pipelining): parity 1 swaps which of s / s2 carries the even levels, so
// the next call's first level can start on the other stream while this call's classify / fit / warp
// run on s; qctr and done must then be the parity's own counters and a.carry non-null, and out_free
// (the previous call's outputs read) is waited for before level 0 writes next_pts / status.
// Dataflow fallback: a group whose wait gives up (the coarser level's launch was not dispatched in
// time: a preempted, shared or serialized device) abandons its level, which then drains without
// computing; right behind each level's launch, on its stream and after the coarser level's (redo_ev,
// kMaxLevels events), a recompute launch re-runs the level in sequence if it gave up or the coarser
// level was recomputed, and exits at once otherwise.  Results are then always exact.
hipError_t launch_lk_v2(hipStream_t s, hipStream_t aux, hipEvent_t* ev, int batch, const LkArgs& a, uint8_t* cls,
                        float4* Ab, int* qctr, hipEvent_t prev_ready = nullptr, hipStream_t s2 = nullptr,
                        hipEvent_t* flow_ev = nullptr, int* done = nullptr, hipEvent_t* lvl_done = nullptr,
                        int parity = 0, hipEvent_t out_free = nullptr, hipEvent_t* redo_ev = nullptr);
// MDX_FIT_RANSAC (mdx_kernels.hip k_ransac_*): device scratch and parameters
constexpr int kRansacMaxIters = 1024;
struct RansacArgs {
    int iters;
    double thresh;
    uint32_t seed;
    int* list;       // [batch][npts] accepted grid indices, x-major
    double* hyps;    // [batch][iters][9]
    int* counts;     // [batch][iters]
};
inline size_t ransac_scratch_bytes(int batch, int npts, int iters)
{
    return (size_t)batch * npts * 4 + (size_t)batch * iters * 72 + (size_t)batch * iters * 4 + 256;
}
// Grid rows [gy0, gy1) only (a row band; others are neither written nor counted).  cand != null:
// row-band mode -- the band's count and first four accepted points go to *cand (one record per
// pair) instead of a fit.
hipError_t launch_classify_fit(hipStream_t s, int batch, const float* next_pts, const uint8_t* status, int npts,
                               int ny, int gy0, int gy1, int pixel_step, double min_vector_size, double* vectors,
                               PairFit* fits, int fit_mode, const double* H_external, void* scratch,
                               mdx_band_cand* cand, const RansacArgs* ransac = nullptr);
// Merge nrec band records (first four accepted overall = four smallest indices) and fit
hipError_t launch_band_fit(hipStream_t s, int nrec, const mdx_band_cand* cands, PairFit* fit, int w, int h, int y0,
                           int y1);
// bytes of the scratch launch_classify_fit needs
inline size_t classify_scratch_bytes(int batch, int npts) { return (size_t)batch * ((npts + 255) / 256) * 32; }
// Row bands: frame-1 gray rows [fit->src_y0, fit->src_y1) into the padded level 0 of pyr1 (the
// band's warp may read rows its own pyramid build skipped), except the rows [built0, built1) the
// pyramid build wrote.  gray1_l0: level-0 core, pitch bytes.
hipError_t launch_gray_rows(hipStream_t s, const uint8_t* img1, int w, int h, int stride, int fmt, uint8_t* gray1_l0,
                            int pitch, const PairFit* fit, int built0 = 0, int built1 = 0);
hipError_t launch_set_fit_external(hipStream_t s, int batch, const double* H_external, PairFit* fits);
// Destination rows [row0, row1) of every pair (row1 <= h); mask row y is at mask + (y - row0) * w.
// scratch: warp_scratch_bytes(batch, w, rows of the band) of device memory for the per-pair and
// per-tile tables of k_warp_prep (the launch's own; reused by the next launch on the stream)
size_t warp_scratch_bytes(int batch, int w, int rows);
hipError_t launch_warp_diff(hipStream_t s, int batch, const uint8_t* g1, long long g1_stride, int g1_pitch,
                            const uint8_t* g2, long long g2_stride, int g2_pitch, int w, int h,
                            const PairFit* fits, uint8_t* mask, long long mask_stride, int thresh, void* scratch,
                            size_t scratch_bytes, int row0 = 0, int row1 = -1);
hipError_t launch_div32(hipStream_t s, const double* in, double* out, int n);   // test hook
hipError_t launch_stream3(hipStream_t s, size_t n, const uint8_t* a, const uint8_t* b, uint8_t* o, int thresh);
hipError_t launch_export_fit(hipStream_t s, int batch, const PairFit* fits, double* H, int* num_vectors);

}  // namespace mdx
