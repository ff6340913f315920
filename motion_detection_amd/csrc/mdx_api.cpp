// mdx_api.cpp -- host side of the C-ABI (include/mdx.h): context, device workspace sized
// once at create time, and the per-call pipeline
//   gray+pad -> pyrDown x L (both frames) -> Scharr x (L+1) -> LK -> classify+fit -> warp+diff
// enqueued on the context's HIP stream.  Replaces OpticalFlowCalculator::calculateOpticalFlow
// (reference common/src/optical_flow_calculator.cpp:30-130); no allocation on the per-frame
// path once the workspace fits the frame size.
#include "../../include/mdx.h"
#include "mdx_internal.h"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cmath>

using namespace mdx;

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    template <typename T> T* as() const { return static_cast<T*>(p); }
};

struct mdx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t aux = nullptr;               // LK class / A kernels run ahead here (MDX_LK_AUX=0: off)
    hipEvent_t lkev[kMaxLevels + 2] = {};    // launch_lk_v2's + the first frames' pyramids ready
    hipStream_t iter2 = nullptr;             // LK dataflow: every other level's iteration launch (MDX_LK_FLOW)
    hipEvent_t flowev[2] = {};
    // Call pipelining (mdx_params.call_pipelining): the pyramid slabs have two halves used by
    // alternate calls, and a call's front end runs on the aux stream right behind the previous
    // call's last class planes and A sums, so it overlaps that call's last LK level and fit/warp.
    // (A stream of its own measured 1.9x slower: a process gets 4 hardware queues, and a fifth
    // stream shares one, so its event waits block the work queued behind them.)
    hipEvent_t front_ev = nullptr;
    hipEvent_t pyr_free[2] = {};             // on `stream`, after the last reader of each half
    hipEvent_t lvl_done[kMaxLevels] = {};    // the last call's iteration launch of each level
    hipEvent_t redo_ev[kMaxLevels] = {};     // LK dataflow: each level's launch + recompute done (fallback order)
    int pyr_half = 0;                        // the half the next pipelined call writes
    hipEvent_t input_ev = nullptr;           // mdx_input_ready: the next device call's inputs (caller-owned)
    uint8_t* last_pyr1 = nullptr;            // the last pair call's pyramids (debug copies)
    uint8_t* last_pyr2 = nullptr;
    // the latest mdx_band_flow_dev's pyramids, which its fit/warp reads (band_w == 0: none, or
    // voided by another call that rebuilt the slabs since)
    uint8_t* band_pyr1 = nullptr;
    uint8_t* band_pyr2 = nullptr;
    int band_half = 0;
    const uint8_t* band_img1 = nullptr;      // the last mdx_band_flow_dev's frame 1 (its fit/warp reads it)
    int band_built[2] = {0, 0};              // level-0 rows of frame 1 that call's pyramid build wrote
    int band_stride = 0, band_fmt = 0;
    // LK dataflow fallback statistics ([0] group waits and [1] gate waits that gave up, [2] levels
    // recomputed), read back and cleared at the sync points, accumulated in lk_fallback
    DevBuf errw;
    int* err_host = nullptr;                 // pinned readback
    int* tcnt_host = nullptr;                // pinned readback of the trajectory counts
    long long lk_fallback[3] = {0, 0, 0};
    int spin_max = kLkSpinDefault;           // MDX_LK_SPIN_MAX (debug: < 0 injects timeouts)
    // MDX_LK_CAP: dataflow launch share of the resident waves (%).  75: the aux stream's next-level
    // class planes and A sums pace the level hand-offs (round 6, profiles/r06_ab_lk_w5_cap.txt: 60 -3%,
    // 70 / 80 / 85 within 1%, 75 best and steadiest, 95 -1.2%)
    int lk_cap = 75;
    // pipelined calls alternate the LK stream parity (MDX_LK_XCALL=1): the next call's first level
    // then need not queue behind this call's fit / warp.  Measured +0.5% (within noise; the chip is
    // already saturated by the aux work in that gap), and it moves the LK stage events, so it is off
    bool lk_xcall = false;
    int lk_parity = 0;                       // the next pipelined call's LK stream parity
    mdx_params prm{};
    int max_w = 0, max_h = 0, max_batch = 0;
    DevBuf pyr1, pyr2, der, fits;            // pyramid / derivative / fit workspace
    DevBuf in1, in2, np, st, vec, mask, H, Hext, num;   // host-path staging
    DevBuf bnp, bst;                         // LK outputs the batched caller did not ask for
    DevBuf cls, Abuf, ctab;                  // LK v2: class planes, A sums, residue tables
    DevBuf dbg;                              // LK v2 per-level trace (MDX_LK_DEBUG=1)
    DevBuf csum;                             // classify: per-block summaries
    DevBuf tin, tcur, tnp, tst, ttraj, tnum, tflag;   // trajectory tracking (ttraj: the four outputs, one block)
    DevBuf straj, sdata, sq, scnt, scols, sres, sout, sbest;      // subspace RANSAC
    DevBuf ring_pyr, ring_der, rin;          // resident frame ring (mdx_ring_*)
    DevBuf wscr;                             // k_warp_prep's per-pair / per-tile tables
    DevBuf rsc;                              // MDX_FIT_RANSAC scratch (list, hypotheses, counts)
    std::vector<int> ring_order;             // held slots, oldest first
    int ring_cap = 0, ring_w = 0, ring_h = 0, ring_ml = -1;
    bool lk_debug = false;
    bool traj_chain = true;                  // trajectory passes in one launch (MDX_TRAJ_CHAIN=0: per pass)
    int traj_ppw = 4;                        // trajectory LK points per wave (MDX_TRAJ_PPW: 1, 2 or 4)
    int lk_impl = 2;                         // 1 = single-kernel LK (k_lk), 2 = class planes
    int lk_g = 0;                            // LK group size: 0 = per level, 4 or 8 (MDX_LK_G)
    int lk_sub = 0;                          // > 0: LK sub-batch cap (MDX_LK_SUB, tests)
    bool lk_arows = true;                    // A sums per row strip where the plan allows (MDX_LK_AROWS=0: per group)
    int lk_astrip = 0;                       // grid rows per A-sum strip (MDX_LK_ASTRIP; 0: kAStripRows)
    // MDX_LK_PFLOW: 1 per-point dataflow wherever the per-pair form does not apply (small batches,
    // row bands), 2 everywhere; 0 (default) never -- measured slower for row bands
    int lk_pflow = 0;
    int lk_epoch = 0;                        // per-point dataflow: the last call's epoch
    void* pflag_mem = nullptr;               // the Abuf allocation and layout whose per-point flags were zeroed
    size_t pflag_at = 0, pflag_bytes = 0, pflag_per = 0;
    int plan_w = -1, plan_h = -1, plan_ps = -1, plan_ml = -1, plan_gy0 = -1, plan_gy1 = -1;
    int band_w = 0, band_h = 0;              // frame of the last mdx_band_flow_dev (its pyramids are live)
    ClassPlan plan{};
    bool timing = false;
    static constexpr int kSlots = 256;     // timed calls kept between mdx_enable_timing and readout
    hipEvent_t* ev = nullptr;              // kSlots x 7 events
    int ncalls = 0;                        // calls recorded since enable
    int cur = -1;                          // slot of the call in flight
    std::string err;
};

static thread_local std::string g_create_err;

static int set_err(mdx_ctx* c, int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIP_OR_RETURN(c, expr)                                                                 \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return set_err((c), MDX_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));      \
    } while (0)

extern "C" void mdx_default_params(mdx_params* p)
{
    p->win = 40;
    p->max_level = 5;
    p->max_iters = 10;
    p->eps = 0.03;
    p->min_eig = 0.001f;
    p->thresh = 190;
    p->pixel_step = 10;
    p->min_vector_size = 1.0;
    p->fit_mode = MDX_FIT_FIRST4;
    p->subspace_precision = MDX_SUBSPACE_F64;
    p->call_pipelining = 0;
    p->ransac_iters = 128;
    p->ransac_thresh = 3.0;
    p->ransac_seed = 20141105u;
}

extern "C" int mdx_grid_count(int w, int h, int ps)
{
    if (w <= 0 || h <= 0 || ps <= 0) return 0;
    return ((w + ps - 1) / ps) * ((h + ps - 1) / ps);
}

static int check_params(const mdx_params* p, std::string* why)
{
    if (p->win != kWin) { *why = "only win == 40 (the reference constant) is supported"; return 0; }
    if (p->max_level < 0 || p->max_level >= kMaxLevels) { *why = "max_level out of range [0, 7]"; return 0; }
    if (p->pixel_step <= 0) { *why = "pixel_step must be > 0 (reference leaves it unset: UB)"; return 0; }
    if (p->fit_mode != MDX_FIT_FIRST4 && p->fit_mode != MDX_FIT_EXTERNAL && p->fit_mode != MDX_FIT_RANSAC) {
        *why = "bad fit_mode";
        return 0;
    }
    if (p->ransac_iters < 1 || p->ransac_iters > kRansacMaxIters) { *why = "ransac_iters must be in [1, 1024]"; return 0; }
    if (!(p->ransac_thresh >= 0.0) || !(p->ransac_thresh < 1e6)) { *why = "ransac_thresh must be in [0, 1e6)"; return 0; }
    if (p->subspace_precision != MDX_SUBSPACE_F64 && p->subspace_precision != MDX_SUBSPACE_F32) {
        *why = "bad subspace_precision";
        return 0;
    }
    if (p->call_pipelining != 0 && p->call_pipelining != 1) { *why = "call_pipelining must be 0 or 1"; return 0; }
    return 1;
}

// buildOpticalFlowPyramid level count and the padded slab layout for a w x h frame.
static Geometry make_geometry(int w, int h, int max_level)
{
    Geometry g{};
    int sw = w, sh = h;
    long long img = 0, der = 0;
    int lvl;
    for (lvl = 0; lvl <= max_level; lvl++) {
        Level& L = g.lv[lvl];
        L.w = sw;
        L.h = sh;
        L.pitch = (kXOff + sw + kPad + 16 + 63) / 64 * 64;   // +16: slack for 16-B row loads
        L.rows = kPad + sh + kPad;
        L.img_off = img;
        L.der_off = der;
        img += (long long)L.pitch * L.rows;
        der += (long long)L.pitch * L.rows;
        g.nlev = lvl + 1;
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= kWin || sh <= kWin) break;
    }
    g.img_bytes = (img + 255) / 256 * 256;
    g.der_words = (der + 63) / 64 * 64;
    return g;
}

static int ensure(mdx_ctx* c, DevBuf& b, size_t need)
{
    if (need == 0) need = 1;
    if (b.p && b.cap >= need) return MDX_OK;
    if (b.p) {
        (void)hipStreamSynchronize(c->stream);   // the aux stream's work is always joined by c->stream
        (void)hipFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    if (hipMalloc(&b.p, need) != hipSuccess) {
        b.p = nullptr;
        return set_err(c, MDX_ENOMEM, "hipMalloc(%zu) failed", need);
    }
    b.cap = need;
    return MDX_OK;
}

// With call pipelining the pyramid slabs hold two halves (ensure_workspace(.., two = true) makes the
// slab at least twice one call's pyramids); other users take the slab from its start.
static size_t pyr_half_bytes(const DevBuf& b) { return b.cap / 2 / 256 * 256; }

static int ensure_workspace(mdx_ctx* c, const Geometry& g, int batch, bool two)
{
    int rc;
    const size_t half = ((size_t)g.img_bytes * batch + 255) / 256 * 256;
    if ((rc = ensure(c, c->pyr1, two ? 2 * half : half)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->pyr2, two ? 2 * half : half)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->der, (size_t)g.der_words * 4 * batch)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->fits, sizeof(PairFit) * (size_t)batch)) != MDX_OK) return rc;
    return MDX_OK;
}

// Page-locked blocks handed out by mdx_host_alloc: [base, base + bytes).  The trajectory entry
// writes its outputs straight into them only when a whole output range lies inside one block.
static std::mutex g_host_mu;
static std::map<uintptr_t, size_t> g_host_blocks;
static bool host_block_holds(const void* p, size_t bytes)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_blocks.upper_bound(a);
    if (it == g_host_blocks.begin()) return false;
    --it;
    return a >= it->first && bytes <= it->second && a - it->first <= it->second - bytes;
}

// Residue classes of the grid at each level (see mdx_lk.hip), the class-grouped point order and
// the class-plane layout.  Rebuilt and uploaded only when frame size / pixel_step / levels change.
// plan.nch == 0 means some group's union is wider than 512 columns (pixel_step >~ 66) or a pair's
// class slab exceeds 2 GB: the caller then runs the single-kernel LK instead.
static int ensure_class_plan(mdx_ctx* c, const Geometry& g, int w, int h, int ps, int batch, int gy0, int gy1)
{
    int rc;
    if (c->plan_w != w || c->plan_h != h || c->plan_ps != ps || c->plan_ml != g.nlev || c->plan_gy0 != gy0 ||
        c->plan_gy1 != gy1) {
        const int nx = (w + ps - 1) / ps, ny = (h + ps - 1) / ps;
        static_assert(kMaxLevels <= 8, "residue tables sized for 2^7 residues");
        std::vector<int16_t> tab(2 * kMaxLevels * 2 * 128, (int16_t)-1);
        std::vector<int16_t> ord;
        int16_t* cmap = tab.data();
        int16_t* rlist = tab.data() + kMaxLevels * 2 * 128;
        ClassPlan P{};
        bool usable = true;
        for (int l = 0; l < g.nlev; l++) {
            const int m = (1 << l) - 1;
            int n[2] = {0, 0};
            for (int axis = 0; axis < 2; axis++) {
                const int cnt = axis == 0 ? nx : ny;
                for (int i = 0; i < cnt; i++) {
                    const int r = (i * ps) & m;
                    int16_t& slot = cmap[(l * 2 + axis) * 128 + r];
                    if (slot < 0) {
                        slot = (int16_t)n[axis];
                        rlist[(l * 2 + axis) * 128 + n[axis]] = (int16_t)r;
                        n[axis]++;
                    }
                    if (n[axis] == m + 1) break;
                }
            }
            ClassLevel& C = P.lv[l];
            C.nrx = n[0];
            C.nry = n[1];
            // columns: each class's members in x order.  Group size per level: 4 points when a
            // 4-group's union fits 64 columns (no extra union loads), else 8 (MDX_LK_G forces one)
            C.ord_off = (int)ord.size();
            const int16_t* cmx = cmap + (l * 2 + 0) * 128;
            const float scale = (float)(1. / (1 << l));
            auto ipx_of = [&](int gx) { return (int)std::floor((float)(gx * ps) * scale - 19.5f); };
            std::vector<std::vector<int16_t>> runs(n[0]);
            for (int i = 0; i < nx; i++) runs[cmx[(i * ps) & m]].push_back((int16_t)i);
            auto union_of = [&](int G) {
                int u = 0;
                for (const auto& r : runs)
                    for (size_t q = 0; q < r.size(); q += G)
                        u = std::max(u, ipx_of(r[std::min(r.size(), q + G) - 1]) - ipx_of(r[q]) + kWin);
                return u;
            };
            // group size 4 (less lockstep) unless 8 stages a row with fewer DMA pieces; union
            // width = the smallest kernel shape that fits (MDX_LK_G=4/8 forces the group size)
            const int u4 = union_of(4), u8 = union_of(8);
            auto fit = [](const int* uws, int n, int u) {
                for (int i = 0; i < n; i++)
                    if (uws[i] >= u) return uws[i];
                return 0;
            };
            const int uw4 = fit(kLkUW4, (int)(sizeof(kLkUW4) / sizeof(int)), u4);
            const int uw8 = fit(kLkUW8, (int)(sizeof(kLkUW8) / sizeof(int)), u8);
            // a row's staging cost goes by LDS-DMA pieces (1 KiB, one per 64 lanes x 16 B): the
            // wave's union row is 4 slots x uw4 or 2 slots x uw8 pairs of 8 B
            auto pieces = [](int slots, int uw) { return (slots * uw * 8 + 1023) / 1024; };
            const bool g4 = c->lk_g == 4 ? uw4 > 0
                          : c->lk_g == 8 ? false
                          : uw4 > 0 && (uw8 == 0 || pieces(4, uw4) <= pieces(2, uw8));
            if (g4) {
                C.G = 4;
                C.UW = uw4;
            } else {
                C.G = 8;
                C.UW = uw8;
            }
            if (C.UW == 0) usable = false;
            for (const auto& r : runs) {   // each run padded to a multiple of G with -1
                ord.insert(ord.end(), r.begin(), r.end());
                for (size_t q = r.size(); q % C.G; q++) ord.push_back((int16_t)-1);
            }
            C.nxp = (int)ord.size() - C.ord_off;
            // rows of the band [gy0, gy1): grouped by class the same way (no padding: a group is
            // one row)
            const size_t r0 = ord.size();
            for (int i = gy0; i < gy1; i++) ord.push_back((int16_t)i);
            const int16_t* cmy = cmap + (l * 2 + 1) * 128;
            std::stable_sort(ord.begin() + r0, ord.end(),
                             [&](int16_t u, int16_t v) { return cmy[(u * ps) & m] < cmy[(v * ps) & m]; });
            // A-sum strips (k_lk_A_rows): runs of one y-class cut into kAStripRows rows; the first
            // window rows v0 = ipy + 40 of a class's rows must be evenly spaced (asp rows apart)
            const size_t r1 = ord.size();
            auto v0_row = [&](int gy) { return (int)std::floor((float)(gy * ps) * scale - 19.5f) + kPad; };
            int asp = 0;
            bool uniform = true;
            std::vector<int16_t> strips;
            for (size_t i = r0; i < r1;) {
                size_t e = i + 1;
                const int cls = cmy[(ord[i] * ps) & m];
                while (e < r1 && cmy[(ord[e] * ps) & m] == cls) {
                    const int d = v0_row(ord[e]) - v0_row(ord[e - 1]);
                    if (asp == 0) asp = d;
                    if (d != asp) uniform = false;
                    e++;
                }
                // small-batch contexts (C4 row bands: one pair per call) take short strips: more
                // waves in flight for the few pairs' A sums, which then finish sooner (one band
                // 1.196-1.197 against 1.217-1.226 ms at 16, profiles/r05_ab_astrip.txt); at batch 32
                // 4..16 rows measured within noise
                const size_t srows = c->lk_astrip > 0 ? (size_t)c->lk_astrip
                                                      : (size_t)(c->max_batch <= 4 ? 4 : kAStripRows);
                for (size_t s = i; s < e; s += srows) {
                    strips.push_back((int16_t)(s - r0));
                    strips.push_back((int16_t)std::min<size_t>(srows, e - s));
                }
                i = e;
            }
            if (asp == 0) asp = kWin;   // one row per class: windows never overlap
            C.asp = uniform && asp >= 5 && c->lk_arows ? asp : 0;
            C.nstrip = (int)strips.size() / 2;
            C.strip_off = (int)ord.size();
            ord.insert(ord.end(), strips.begin(), strips.end());
        }
        (void)ny;
        long long off = 0;
        for (int l = 0; l < g.nlev; l++) {
            ClassLevel& C = P.lv[l];
            C.UH = g.lv[l].h + 79;
            C.PW = (g.lv[l].w + kPad + std::max(C.UW, 64) + 3) & ~3;
            // plane rows the band's windows read: first rows v0 = clamp(ipy + 40, 0, UH - 40) of
            // its first and last grid rows (ipy is monotone in gy), 40 rows each
            const float scale = (float)(1. / (1 << l));
            auto v0_of = [&](int gy) {
                const int ipy = (int)std::floor((float)(gy * ps) * scale - 19.5f);
                return std::min(std::max(ipy + kPad, 0), C.UH - kWin);
            };
            C.vlo = v0_of(gy0);
            C.vhi = v0_of(gy1 - 1) + kWin;
            C.class_bytes = (long long)C.UH * C.PW * 8;
            C.off = off;
            off += (long long)C.nrx * C.nry * C.class_bytes;
        }
        // the kernels address a pair's slab with 32-bit buffer offsets
        if (off > 0x7fff0000LL) usable = false;
        P.nch = usable ? 1 : 0;
        P.bytes_per_pair = (off + 255) / 256 * 256;
        tab.insert(tab.end(), ord.begin(), ord.end());
        if ((rc = ensure(c, c->ctab, tab.size() * sizeof(int16_t))) != MDX_OK) return rc;
        // kernels of earlier calls may still read the old tables: the copy waits for them (the
        // stream is non-blocking, so a plain hipMemcpy would not)
        HIP_OR_RETURN(c, hipStreamSynchronize(c->stream));
        HIP_OR_RETURN(c, hipMemcpy(c->ctab.p, tab.data(), tab.size() * sizeof(int16_t), hipMemcpyHostToDevice));
        c->plan = P;
        c->plan_w = w;
        c->plan_h = h;
        c->plan_ps = ps;
        c->plan_ml = g.nlev;
        c->plan_gy0 = gy0;
        c->plan_gy1 = gy1;
    }
    if (c->plan.nch == 0) return MDX_OK;
    if ((rc = ensure(c, c->cls, (size_t)c->plan.bytes_per_pair * batch + 64)) != MDX_OK) return rc;
    return MDX_OK;
}

extern "C" const char* mdx_create_error(void) { return g_create_err.c_str(); }
extern "C" int mdx_abi_version(void) { return MDX_ABI_VERSION; }
extern "C" size_t mdx_params_size(void) { return sizeof(mdx_params); }

extern "C" mdx_ctx* mdx_create(int device, int max_w, int max_h, int max_batch, const mdx_params* p)
{
    g_create_err.clear();
    mdx_params prm;
    if (p) prm = *p;
    else mdx_default_params(&prm);
    std::string why;
    if (!check_params(&prm, &why)) { g_create_err = why; return nullptr; }
    if (max_w <= 0 || max_h <= 0 || max_batch <= 0) { g_create_err = "max_w/max_h/max_batch must be > 0"; return nullptr; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { g_create_err = "no HIP device visible"; return nullptr; }
    if (device < 0 || device >= ndev) { g_create_err = "device index out of range"; return nullptr; }
    if (hipSetDevice(device) != hipSuccess) { g_create_err = "hipSetDevice failed"; return nullptr; }
    mdx_ctx* c = new mdx_ctx();
    c->device = device;
    c->prm = prm;
    c->max_w = max_w;
    c->max_h = max_h;
    c->max_batch = max_batch;
    if (const char* e = std::getenv("MDX_LK_IMPL")) c->lk_impl = std::atoi(e) == 1 ? 1 : 2;
    if (const char* e = std::getenv("MDX_LK_G")) c->lk_g = std::atoi(e);
    if (const char* e = std::getenv("MDX_LK_SUB")) c->lk_sub = std::atoi(e);
    if (const char* e = std::getenv("MDX_LK_AROWS")) c->lk_arows = std::atoi(e) != 0;
    if (const char* e = std::getenv("MDX_LK_ASTRIP")) c->lk_astrip = std::max(0, std::min(std::atoi(e), 64));
    if (const char* e = std::getenv("MDX_LK_PFLOW")) c->lk_pflow = std::atoi(e);
    if (const char* e = std::getenv("MDX_LK_DEBUG")) c->lk_debug = std::atoi(e) != 0;
    if (const char* e = std::getenv("MDX_TRAJ_CHAIN")) c->traj_chain = std::atoi(e) != 0;
    if (const char* e = std::getenv("MDX_TRAJ_PPW")) c->traj_ppw = std::atoi(e) == 1 ? 1 : std::atoi(e) == 2 ? 2 : 4;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        g_create_err = "hipStreamCreate failed";
        delete c;
        return nullptr;
    }
    const char* ea = std::getenv("MDX_LK_AUX");
    if (!ea || std::atoi(ea) != 0) {
        // MDX_AUX_PRIO=1: the aux stream (class planes, A sums, pipelined front ends) gets the
        // greatest dispatch priority, so its waves take slots ahead of a persistent iteration launch
        int least = 0, greatest = 0;
        const char* ep = std::getenv("MDX_AUX_PRIO");
        const bool prio = ep && std::atoi(ep) != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess;
        bool ok = (prio ? hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, greatest)
                        : hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking)) == hipSuccess;
        for (int i = 0; ok && i <= kMaxLevels + 1; i++)
            ok = hipEventCreateWithFlags(&c->lkev[i], hipEventDisableTiming) == hipSuccess;
        const char* ef = std::getenv("MDX_LK_FLOW");
        if (ok && (!ef || std::atoi(ef) != 0)) {
            ok = hipStreamCreateWithFlags(&c->iter2, hipStreamNonBlocking) == hipSuccess;
            for (int i = 0; ok && i < 2; i++) ok = hipEventCreateWithFlags(&c->flowev[i], hipEventDisableTiming) == hipSuccess;
            for (int i = 0; ok && i < kMaxLevels; i++)
                ok = hipEventCreateWithFlags(&c->redo_ev[i], hipEventDisableTiming) == hipSuccess;
        }
        // call pipelining's events (mdx_params.call_pipelining may be switched on at any call)
        ok = ok && hipEventCreateWithFlags(&c->front_ev, hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < 2; i++) ok = hipEventCreateWithFlags(&c->pyr_free[i], hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < kMaxLevels; i++)
            ok = hipEventCreateWithFlags(&c->lvl_done[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            g_create_err = "aux stream / event creation failed";
            mdx_destroy(c);
            return nullptr;
        }
    }
    if (const char* e = std::getenv("MDX_LK_CAP")) c->lk_cap = std::min(std::max(std::atoi(e), 10), 100);
    if (const char* e = std::getenv("MDX_LK_SPIN_MAX")) c->spin_max = std::atoi(e);
    if (const char* e = std::getenv("MDX_LK_XCALL")) c->lk_xcall = std::atoi(e) != 0;
    if (ensure(c, c->errw, 16) != MDX_OK || hipMemset(c->errw.p, 0, 16) != hipSuccess ||
        hipHostMalloc((void**)&c->err_host, 16, hipHostMallocDefault) != hipSuccess) {
        g_create_err = "error-word allocation failed";
        mdx_destroy(c);
        return nullptr;
    }
    Geometry g = make_geometry(max_w, max_h, prm.max_level);
    if (ensure_workspace(c, g, max_batch, prm.call_pipelining != 0) != MDX_OK) {
        g_create_err = c->err;
        mdx_destroy(c);
        return nullptr;
    }
    return c;
}

extern "C" int mdx_destroy(mdx_ctx* c)
{
    if (!c) return MDX_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->aux) (void)hipStreamSynchronize(c->aux);          // pipelined front ends
    if (c->iter2) (void)hipStreamSynchronize(c->iter2);
    DevBuf* bufs[] = {&c->pyr1, &c->pyr2, &c->der, &c->fits, &c->in1, &c->in2, &c->np, &c->st,
                      &c->vec, &c->mask, &c->H, &c->Hext, &c->num, &c->bnp, &c->bst,
                      &c->cls, &c->Abuf, &c->ctab, &c->dbg, &c->csum, &c->tin, &c->tcur, &c->tnp, &c->tst,
                      &c->ttraj, &c->tnum, &c->tflag, &c->straj, &c->sdata, &c->sq,
                      &c->scnt, &c->scols, &c->sres, &c->sout, &c->sbest, &c->ring_pyr, &c->ring_der, &c->rin,
                      &c->errw, &c->wscr, &c->rsc};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    if (c->err_host) (void)hipHostFree(c->err_host);
    if (c->tcnt_host) (void)hipHostFree(c->tcnt_host);
    if (c->ev) {
        for (int i = 0; i < mdx_ctx::kSlots * 7; i++) (void)hipEventDestroy(c->ev[i]);
        delete[] c->ev;
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    if (c->iter2) (void)hipStreamDestroy(c->iter2);
    if (c->front_ev) (void)hipEventDestroy(c->front_ev);
    for (hipEvent_t e : c->pyr_free)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->lvl_done)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->lkev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->flowev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->redo_ev)
        if (e) (void)hipEventDestroy(e);
    delete c;
    return MDX_OK;
}

extern "C" const char* mdx_last_error(const mdx_ctx* c) { return c ? c->err.c_str() : "null context"; }
extern "C" void* mdx_stream(mdx_ctx* c) { return c ? (void*)c->stream : nullptr; }
extern "C" int mdx_device(const mdx_ctx* c) { return c ? c->device : -1; }
extern "C" int mdx_device_pci(const mdx_ctx* c, char* buf, int len)
{
    if (!c || !buf || len < 16) return MDX_EINVAL;
    return hipDeviceGetPCIBusId(buf, len, c->device) == hipSuccess ? MDX_OK : MDX_EHIP;
}

extern "C" int mdx_set_params(mdx_ctx* c, const mdx_params* p)
{
    if (!c || !p) return MDX_EINVAL;
    std::string why;
    if (!check_params(p, &why)) return set_err(c, MDX_EINVAL, "%s", why.c_str());
    c->prm = *p;
    return MDX_OK;
}

extern "C" int mdx_get_params(const mdx_ctx* c, mdx_params* p)
{
    if (!c || !p) return MDX_EINVAL;
    *p = c->prm;
    return MDX_OK;
}

// The LK dataflow's fallbacks since the last check: queue the statistics word's readback on the
// context stream (every LK launch of a call is joined into it); after the caller's sync
// lk_err_result adds them to the context's totals (mdx_lk_fallbacks) and clears the word.  A wait
// that gave up is not an error: its level was recomputed in sequence within the same call.
static int queue_lk_err(mdx_ctx* c)
{
    HIP_OR_RETURN(c, hipMemcpyAsync(c->err_host, c->errw.p, 12, hipMemcpyDeviceToHost, c->stream));
    return MDX_OK;
}

static int lk_err_result(mdx_ctx* c)
{
    const int groups = c->err_host[0], gates = c->err_host[1], redone = c->err_host[2];
    if (groups == 0 && gates == 0 && redone == 0) return MDX_OK;
    c->err_host[0] = c->err_host[1] = c->err_host[2] = 0;
    c->lk_fallback[0] += groups;
    c->lk_fallback[1] += gates;
    c->lk_fallback[2] += redone;
    HIP_OR_RETURN(c, hipMemsetAsync(c->errw.p, 0, 12, c->stream));
    HIP_OR_RETURN(c, hipStreamSynchronize(c->stream));
    // a give-up (a group wait or a gate) is always followed by its level's recompute (launch_lk_v2):
    // one without it would be a scheduling bug, and its outputs could be wrong
    if (groups + gates > 0 && redone == 0)
        return set_err(c, MDX_EHIP, "LK dataflow: %d wait(s) and %d gate(s) gave up but no level was recomputed",
                       groups, gates);
    return MDX_OK;
}

extern "C" int mdx_lk_fallbacks(const mdx_ctx* c, long long* counts)
{
    if (!c || !counts) return MDX_EINVAL;
    for (int i = 0; i < 3; i++) counts[i] = c->lk_fallback[i];
    return MDX_OK;
}

extern "C" int mdx_sync(mdx_ctx* c)
{
    if (!c) return MDX_EINVAL;
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    int rc = queue_lk_err(c);
    if (rc != MDX_OK) return rc;
    HIP_OR_RETURN(c, hipStreamSynchronize(c->stream));
    return lk_err_result(c);
}

extern "C" int mdx_device_sync(mdx_ctx* c)
{
    if (!c) return MDX_EINVAL;
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    int rc = queue_lk_err(c);
    if (rc != MDX_OK) return rc;
    HIP_OR_RETURN(c, hipDeviceSynchronize());
    return lk_err_result(c);
}

extern "C" int mdx_input_ready(mdx_ctx* c, void* hip_event)
{
    if (!c) return MDX_EINVAL;
    c->input_ev = static_cast<hipEvent_t>(hip_event);
    return MDX_OK;
}

// The next device call's first stage waits for the caller's input event (mdx_input_ready), once.
static int wait_input(mdx_ctx* c, hipStream_t st)
{
    if (!c->input_ev) return MDX_OK;
    hipEvent_t e = c->input_ev;
    c->input_ev = nullptr;
    HIP_OR_RETURN(c, hipStreamWaitEvent(st, e, 0));
    return MDX_OK;
}

extern "C" int mdx_enable_timing(mdx_ctx* c, int on)
{
    if (!c) return MDX_EINVAL;
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    if (on && !c->ev) {
        c->ev = new hipEvent_t[mdx_ctx::kSlots * 7];
        for (int i = 0; i < mdx_ctx::kSlots * 7; i++) HIP_OR_RETURN(c, hipEventCreate(&c->ev[i]));
    }
    c->timing = on != 0;
    c->ncalls = 0;
    c->cur = -1;
    return MDX_OK;
}

extern "C" int mdx_timing_calls(const mdx_ctx* c) { return c ? c->ncalls : 0; }

// Sum over the recorded calls of the time between the stage's bracketing events.
extern "C" int mdx_stage_ms(mdx_ctx* c, int stage, float* ms)
{
    if (!c || !ms || stage < 0 || stage > 6) return MDX_EINVAL;
    if (!c->timing || !c->ev) return set_err(c, MDX_EINVAL, "timing not enabled");
    if (c->ncalls > mdx_ctx::kSlots) return set_err(c, MDX_EINVAL, "more than %d timed calls", mdx_ctx::kSlots);
    float total = 0.f;
    for (int k = 0; k < c->ncalls; k++) {
        hipEvent_t* e = c->ev + k * 7;
        HIP_OR_RETURN(c, hipEventSynchronize(e[6]));
        float t = 0.f;
        if (stage == 6) HIP_OR_RETURN(c, hipEventElapsedTime(&t, e[0], e[6]));
        else HIP_OR_RETURN(c, hipEventElapsedTime(&t, e[stage], e[stage + 1]));
        total += t;
    }
    *ms = total;
    return MDX_OK;
}

static inline void mark(mdx_ctx* c, int i, hipStream_t st = nullptr)
{
    if (!c->timing || !c->ev) return;
    if (i == 0) {
        c->cur = c->ncalls < mdx_ctx::kSlots ? c->ncalls : -1;
        c->ncalls++;
    }
    if (c->cur >= 0) (void)hipEventRecord(c->ev[c->cur * 7 + i], st ? st : c->stream);
}

// Non-pipelined users of the pyramid / derivative slabs (from the slab start, any size): the next
// pipelined call's front end and aux work wait for them through both halves' events.
static void release_pyr_all(mdx_ctx* c)
{
    for (hipEvent_t e : c->pyr_free)
        if (e) (void)hipEventRecord(e, c->stream);
}

// The LK of a batch of pairs on the context's stream.  Grid start points (a.prev_pts null) on a
// dense enough grid take the class-plane kernels, which launch each level's Scharr planes
// themselves; otherwise the single kernel, after the Scharr planes unless the caller already
// computed them (have_scharr).  a: every field but the class-plan ones.
static int run_lk(mdx_ctx* c, const Geometry& g, LkArgs& a, int batch, int w, int h, int gy0, int gy1,
                  bool have_scharr, hipEvent_t prev_ready = nullptr, int parity = -1, hipEvent_t out_free = nullptr)
{
    int rc;
    hipStream_t s = c->stream;
    bool v2 = c->lk_impl == 2 && a.prev_pts == nullptr;
    if (v2) {
        if ((rc = ensure_class_plan(c, g, w, h, c->prm.pixel_step, batch, gy0, gy1)) != MDX_OK) return rc;
        v2 = c->plan.nch != 0;   // very sparse grids: the single-kernel LK
    }
    if (!v2) {
        if (gy0 != 0 || gy1 != a.ny)
            return set_err(c, MDX_EINVAL, "row bands need the class-plane LK (pixel_step too large)");
        if (!have_scharr)
            for (int l = 0; l < g.nlev; l++)
                HIP_OR_RETURN(c, launch_scharr(s, batch, a.pyr1, const_cast<uint32_t*>(a.der), g, l));
        HIP_OR_RETURN(c, launch_lk(s, batch, a));
        return MDX_OK;
    }
    a.plan = c->plan;
    a.max_sub = c->lk_sub;
    a.err = c->errw.as<int>();
    a.spin_max = c->spin_max;
    a.flow_cap = c->lk_cap;
    a.cmap = c->ctab.as<int16_t>();
    a.rlist = c->ctab.as<int16_t>() + kMaxLevels * 2 * 128;
    a.ord = c->ctab.as<int16_t>() + 2 * kMaxLevels * 2 * 128;
    const int npts = a.npts;
    if (c->lk_debug) {
        if ((rc = ensure(c, c->dbg, ((size_t)npts * g.nlev * batch + kLkDbgStampOff + kMaxLevels * kLkDbgWaves) * 16)) !=
            MDX_OK)
            return rc;
        a.dbg = c->dbg.as<float4>();
        const char* e = std::getenv("MDX_LK_DEBUG_PT");
        a.dbg_pt = e ? std::atoi(e) : -1;
    }
    // A sums, then per parity (parity < 0: no cross-call overlap, parity 0's) the queue heads
    // ([sub-batch][level][XCD]), the dataflow counters ([level][pair]) and the points carried
    // between levels ([pair][point]; cross-call overlap only: the next call's coarse levels then
    // never touch the next_pts this call's classify still reads)
    const size_t abytes = (size_t)g.nlev * batch * npts * sizeof(float4);
    const size_t qbytes = (size_t)batch * kMaxLevels * 8 * kCtrPad * sizeof(int);
    const size_t dbytes = ((size_t)kMaxLevels * batch + kLkFlagInts) * kCtrPad * sizeof(int);
    const size_t lbytes = ((size_t)batch * npts * 8 + 127) / 128 * 128;   // one level's carried points
    const size_t cbytes = lbytes * g.nlev;
    // per-point dataflow flags: [level][pair][point] epochs, per parity (zeroed once per allocation;
    // every call's epoch exceeds the earlier ones', so stale stamps never satisfy a wait)
    const size_t fbytes = ((size_t)batch * npts * 4 + 127) / 128 * 128;
    const size_t pbytes = fbytes * g.nlev;
    const size_t per = qbytes + dbytes + cbytes + pbytes;
    if ((rc = ensure(c, c->Abuf, abytes + 2 * per)) != MDX_OK) return rc;
    // (re)zeroed whenever the flags move: stale bytes of another layout (A sums, carried points)
    // could read as large epochs
    const size_t pf_at = abytes + qbytes + dbytes + cbytes;
    if (c->lk_epoch >= (1 << 30)) {   // epochs wrap: start again from zeroed flags
        c->lk_epoch = 0;
        c->pflag_mem = nullptr;
    }
    if (c->pflag_mem != c->Abuf.p || c->pflag_at != pf_at || c->pflag_bytes != pbytes || c->pflag_per != per) {
        // only the flag regions: the aux stream may already write the A sums of this allocation;
        // the flags' writers and readers (the iteration launches) follow c->stream
        for (int q = 0; q < 2; q++)
            HIP_OR_RETURN(c, hipMemsetAsync(c->Abuf.as<uint8_t>() + abytes + q * per + qbytes + dbytes + cbytes, 0,
                                            pbytes, c->stream));
        // the coarsest level may run on the second iteration stream (MDX_LK_XCALL, parity 1), which
        // does not follow c->stream: finish the zeroing before any launch reads the flags (this runs
        // only when the flag regions move, i.e. on a reallocation or a layout change)
        HIP_OR_RETURN(c, hipStreamSynchronize(c->stream));
        c->pflag_mem = c->Abuf.p;
        c->pflag_at = pf_at;
        c->pflag_bytes = pbytes;
        c->pflag_per = per;
    }
    const int par = parity < 0 ? 0 : parity;
    uint8_t* base = c->Abuf.as<uint8_t>() + abytes + par * per;
    a.carry = reinterpret_cast<float*>(base + qbytes + dbytes);
    a.carry_lstride = (long long)(lbytes / sizeof(float));
    a.pflags = c->lk_pflow <= 0 ? nullptr : reinterpret_cast<int*>(base + qbytes + dbytes + cbytes);
    a.pf_lstride = (long long)(fbytes / sizeof(int));
    a.epoch = ++c->lk_epoch;
    a.pflow_force = c->lk_pflow > 1 ? 1 : 0;
    HIP_OR_RETURN(c, launch_lk_v2(s, c->aux, c->lkev, batch, a, c->cls.as<uint8_t>(), c->Abuf.as<float4>(),
                                  reinterpret_cast<int*>(base), prev_ready, c->iter2, c->flowev,
                                  reinterpret_cast<int*>(base + qbytes), c->prm.call_pipelining ? c->lvl_done : nullptr,
                                  par, out_free, c->iter2 ? c->redo_ev : nullptr));
    return MDX_OK;
}

// Row-band mode: the previous frame's (pyr1) core rows a band's class planes read at each level --
// padded rows [vlo - 1, vhi + 2) of the planes' source (k_lk_class_fused reads y-1 .. y+2, the
// Scharr planes behind k_lk_class the same), reflect-101 border rows folded onto the core rows they
// mirror -- and the rows the next level's pyrDown reads from it (pyramids.cpp: dst row r reads rows
// 2r-2 .. 2r+2).  Only those rows of pyr1 are built; the next frame's pyramid stays whole, since J
// may be read anywhere in it.
static void band_rows(const Geometry& g, const ClassPlan& P, RowSpan* rows)
{
    for (int l = g.nlev - 1; l >= 0; l--) {
        const int h = g.lv[l].h;
        const int lo = P.lv[l].vlo - 1 - kPad, hi = P.lv[l].vhi + 2 - kPad;   // core coordinates
        int clo = std::max(lo, 0), chi = std::min(hi, h);
        if (lo < 0) chi = std::max(chi, std::min(h, 1 - lo));                 // rows lo..-1 mirror 1..-lo
        if (hi > h) clo = std::min(clo, std::max(0, 2 * h - 1 - hi));         // rows h..hi-1 mirror down to 2h-1-hi
        if (l + 1 < g.nlev) {
            clo = std::min(clo, std::max(0, 2 * rows[l + 1].lo - 2));
            chi = std::max(chi, std::min(h, 2 * rows[l + 1].hi + 2));
        }
        rows[l] = RowSpan{clo, std::max(clo, chi)};
    }
}

// The pipeline on device buffers.  d_np/d_st must be valid (LK writes them).
// Row-band mode (cand != null, batch 1): LK and classification for grid rows [gy0, gy1) only, the
// band's record to *cand, no fit and no mask.
static int run_pipeline(mdx_ctx* c, int batch, const uint8_t* d_img1, const uint8_t* d_img2, int w, int h, int stride,
                        size_t frame_stride, int fmt, float* d_np, uint8_t* d_st, double* d_vec, uint8_t* d_mask,
                        double* d_H, const double* d_Hext, int* d_num, int gy0 = 0, int gy1 = -1,
                        mdx_band_cand* cand = nullptr, bool may_overlap = false)
{
    const mdx_params& P = c->prm;
    if (w <= 0 || h <= 0 || batch <= 0) return set_err(c, MDX_EINVAL, "bad frame size or batch");
    if (fmt < MDX_FMT_GRAY8 || fmt > MDX_FMT_BGR8) return set_err(c, MDX_EINVAL, "bad pixel format %d", fmt);
    const int cn = fmt == MDX_FMT_GRAY8 ? 1 : 3;
    if (stride < w * cn) return set_err(c, MDX_EINVAL, "stride %d < w*channels %d", stride, w * cn);
    if (batch > 1 && frame_stride < (size_t)stride * h) return set_err(c, MDX_EINVAL, "frame_stride too small");
    if (P.fit_mode == MDX_FIT_EXTERNAL && !d_Hext) return set_err(c, MDX_EINVAL, "fit_mode EXTERNAL needs H_external");
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    // call pipelining: this call's pyramids go to the half the previous call did not use, and its
    // front end runs on the front stream once that half's last reader (two calls back) is done
    const bool pipe = may_overlap && P.call_pipelining && c->aux && c->lk_impl == 2;
    Geometry g = make_geometry(w, h, P.max_level);
    int rc = ensure_workspace(c, g, batch, pipe);
    if (rc != MDX_OK) return rc;
    const int npts = mdx_grid_count(w, h, P.pixel_step);
    const int ny = (h + P.pixel_step - 1) / P.pixel_step;
    if (gy1 < 0) gy1 = ny;
    const int nyb = gy1 - gy0;
    hipStream_t s = c->stream;
    uint8_t* pyr1 = c->pyr1.as<uint8_t>();
    uint8_t* pyr2 = c->pyr2.as<uint8_t>();
    uint32_t* der = c->der.as<uint32_t>();
    PairFit* fits = c->fits.as<PairFit>();
    hipStream_t fs_ = s;
    int half = 0;
    if (pipe) {
        half = c->pyr_half;
        c->pyr_half ^= 1;
        pyr1 += half * pyr_half_bytes(c->pyr1);
        pyr2 += half * pyr_half_bytes(c->pyr2);
        fs_ = c->aux;
        HIP_OR_RETURN(c, hipStreamWaitEvent(fs_, c->pyr_free[half], 0));
    }
    if ((rc = wait_input(c, fs_)) != MDX_OK) return rc;
    c->last_pyr1 = pyr1;
    c->last_pyr2 = pyr2;
    // a row band's fit/warp reads these pyramids; any other call voids the band's
    if (cand) {
        c->band_pyr1 = pyr1;
        c->band_pyr2 = pyr2;
        c->band_half = half;
    } else {
        c->band_w = c->band_h = 0;
    }

    mark(c, 0, fs_);
    // The class planes and A sums need only the first frames' pyramids: build those first and let
    // the aux stream start on them while the second frames' pyramids are built.  Stage "gray_pad"
    // = gray + pad + level 1 of the first frames (k_front), "pyrdown" = the rest of the pyramids.
    hipEvent_t prev_ready = nullptr;
    const long long fs = (long long)frame_stride;
    // a row band (batch 1): the rows of the previous frame's pyramid its class planes read
    RowSpan rows[kMaxLevels];
    const RowSpan* prows = nullptr;
    if (cand && c->lk_impl == 2 && npts > 0 && nyb > 0 && nyb < ny) {
        if ((rc = ensure_class_plan(c, g, w, h, P.pixel_step, batch, gy0, gy1)) != MDX_OK) return rc;
        if (c->plan.nch != 0) {
            band_rows(g, c->plan, rows);
            prows = rows;
        }
    }
    // level-0 rows of frame 1 this call builds (mdx_band_fit_warp_dev converts the others it needs);
    // k_front writes whole level-1 bands, i.e. level-0 rows 2*lo1 .. 2*hi1 of the widened range
    c->band_built[0] = 0;
    c->band_built[1] = h;
    if (prows) {
        const int lo1 = std::min(rows[1].lo, rows[0].lo / 2), hi1 = std::max(rows[1].hi, (rows[0].hi + 1) / 2);
        c->band_built[0] = std::max(0, 2 * lo1);
        c->band_built[1] = std::min(h, 2 * hi1);
    }
    if (c->aux && c->lk_impl == 2) {
        HIP_OR_RETURN(c, launch_front(fs_, batch, d_img1, d_img2, w, h, stride, fs, fmt, pyr1, pyr2, g, 1, prows));
        mark(c, 1, fs_);
        HIP_OR_RETURN(c, launch_pyr_levels(fs_, batch, pyr1, pyr2, g, 1, prows));
        HIP_OR_RETURN(c, hipEventRecord(c->lkev[kMaxLevels + 1], fs_));
        prev_ready = c->lkev[kMaxLevels + 1];
        HIP_OR_RETURN(c, launch_front(fs_, batch, d_img1, d_img2, w, h, stride, fs, fmt, pyr1, pyr2, g, 2));
        HIP_OR_RETURN(c, launch_pyr_levels(fs_, batch, pyr1, pyr2, g, 2));
        if (pipe) {
            mark(c, 2, fs_);
            HIP_OR_RETURN(c, hipEventRecord(c->front_ev, fs_));
            HIP_OR_RETURN(c, hipStreamWaitEvent(s, c->front_ev, 0));
        }
    } else {
        HIP_OR_RETURN(c, launch_front(s, batch, d_img1, d_img2, w, h, stride, fs, fmt, pyr1, pyr2, g));
        mark(c, 1);
        HIP_OR_RETURN(c, launch_pyr_levels(s, batch, pyr1, pyr2, g));
    }
    if (!pipe) mark(c, 2);
    // Scharr derivatives feed only the LK.  The class-plane LK launches them itself, on its
    // aux stream right before each level's class planes, so they overlap the coarser levels'
    // iterations; the single-kernel LK needs them up front.
    mark(c, 3);
    if (npts > 0 && nyb > 0) {
        LkArgs a{};
        a.pyr1 = pyr1;
        a.pyr2 = pyr2;
        a.der = der;
        a.g = g;
        a.maxl = g.nlev - 1;
        a.npts = npts;
        a.ny = ny;
        a.nyg = nyb;
        a.pixel_step = P.pixel_step;
        a.max_iters = std::min(std::max(P.max_iters, 0), 100);
        a.min_eig = P.min_eig;
        const double e = std::min(std::max(P.eps, 0.), 10.);
        a.eps2 = e * e;
        a.next_pts = d_np;
        a.status = d_st;
        // pipelined calls alternate the LK's stream parity (cross-call overlap: this call's first
        // level need not wait for the previous call's classify / fit / warp on the context stream);
        // level 0 waits for the previous call's warp (pyr_free of its half) before writing outputs
        int parity = -1;
        hipEvent_t out_free = nullptr;
        if (pipe && c->lk_xcall) {
            parity = c->lk_parity;
            c->lk_parity ^= 1;
            out_free = c->pyr_free[half ^ 1];
        }
        if ((rc = run_lk(c, g, a, batch, w, h, gy0, gy1, false, prev_ready, parity, out_free)) != MDX_OK) return rc;
    }
    mark(c, 4);
    if ((rc = ensure(c, c->csum, classify_scratch_bytes(batch, npts))) != MDX_OK) return rc;
    RansacArgs ra{};
    if (P.fit_mode == MDX_FIT_RANSAC && !cand) {
        if ((rc = ensure(c, c->rsc, ransac_scratch_bytes(batch, npts, P.ransac_iters))) != MDX_OK) return rc;
        uint8_t* base = c->rsc.as<uint8_t>();
        ra.iters = P.ransac_iters;
        ra.thresh = P.ransac_thresh;
        ra.seed = P.ransac_seed;
        ra.list = reinterpret_cast<int*>(base);
        ra.hyps = reinterpret_cast<double*>(base + (((size_t)batch * npts * 4 + 7) & ~(size_t)7));
        ra.counts = reinterpret_cast<int*>(reinterpret_cast<uint8_t*>(ra.hyps) + (size_t)batch * P.ransac_iters * 72);
    }
    HIP_OR_RETURN(c, launch_classify_fit(s, batch, d_np, d_st, npts, ny, gy0, gy1, P.pixel_step, P.min_vector_size, d_vec,
                                         fits, P.fit_mode, d_Hext, c->csum.p, cand, &ra));
    mark(c, 5);
    if (cand) {
        // mdx_band_fit_warp_dev reads the latest band call's pyramids (same frame pair), whichever
        // half they are in, and records their release again after its warp
        if (pipe) HIP_OR_RETURN(c, hipEventRecord(c->pyr_free[half], s));
        else release_pyr_all(c);
        mark(c, 6);
        return MDX_OK;
    }
    if (d_mask) {
        const Level& L0 = g.lv[0];
        const uint8_t* g1 = pyr1 + L0.img_off + L0.core();
        const uint8_t* g2 = pyr2 + L0.img_off + L0.core();
        const size_t wsb = warp_scratch_bytes(batch, w, h);
        if ((rc = ensure(c, c->wscr, wsb)) != MDX_OK) return rc;
        HIP_OR_RETURN(c, launch_warp_diff(s, batch, g1, g.img_bytes, L0.pitch, g2, g.img_bytes, L0.pitch, w, h, fits,
                                          d_mask, (long long)w * h, P.thresh, c->wscr.p, wsb));
    }
    if (d_H || d_num) HIP_OR_RETURN(c, launch_export_fit(s, batch, fits, d_H, d_num));
    if (pipe) HIP_OR_RETURN(c, hipEventRecord(c->pyr_free[half], s));
    else release_pyr_all(c);
    mark(c, 6);
    return MDX_OK;
}

extern "C" int mdx_flow_warp_diff_batch_dev(mdx_ctx* c, int batch, const uint8_t* d_img1, const uint8_t* d_img2,
                                            int w, int h, int stride, size_t frame_stride, int fmt, float* d_next_pts,
                                            uint8_t* d_status, double* d_vectors, uint8_t* d_mask, double* d_H,
                                            const double* d_H_external, int* d_num_vectors)
{
    if (!c) return MDX_EINVAL;
    if (!d_img1 || !d_img2 || batch <= 0) return set_err(c, MDX_EINVAL, "null frame pointer or batch <= 0");
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    const size_t need = (size_t)mdx_grid_count(w, h, c->prm.pixel_step) * batch;
    int rc;
    if (!d_next_pts) {
        if ((rc = ensure(c, c->bnp, need * 8)) != MDX_OK) return rc;
        d_next_pts = c->bnp.as<float>();
    }
    if (!d_status) {
        if ((rc = ensure(c, c->bst, need)) != MDX_OK) return rc;
        d_status = c->bst.as<uint8_t>();
    }
    return run_pipeline(c, batch, d_img1, d_img2, w, h, stride, frame_stride, fmt, d_next_pts, d_status, d_vectors,
                        d_mask, d_H, d_H_external, d_num_vectors, 0, -1, nullptr, true);
}

extern "C" int mdx_flow_warp_diff(mdx_ctx* c, const uint8_t* img1, const uint8_t* img2, int w, int h, int stride,
                                  int fmt, float* next_pts, uint8_t* status, double* vectors, uint8_t* mask, double* H,
                                  const double* H_external, int* num_vectors)
{
    if (!c) return MDX_EINVAL;
    if (!img1 || !img2) return set_err(c, MDX_EINVAL, "null frame pointer");
    if (w <= 0 || h <= 0) return set_err(c, MDX_EINVAL, "bad frame size");
    if (fmt < MDX_FMT_GRAY8 || fmt > MDX_FMT_BGR8) return set_err(c, MDX_EINVAL, "bad pixel format %d", fmt);
    const int cn = fmt == MDX_FMT_GRAY8 ? 1 : 3;
    if (stride < w * cn) return set_err(c, MDX_EINVAL, "stride %d < w*channels %d", stride, w * cn);
    if (c->prm.fit_mode == MDX_FIT_EXTERNAL && !H_external)
        return set_err(c, MDX_EINVAL, "fit_mode EXTERNAL needs H_external");
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    const size_t in_bytes = (size_t)stride * h;
    const int npts = mdx_grid_count(w, h, c->prm.pixel_step);
    const size_t pts = (size_t)(npts > 0 ? npts : 1);
    int rc;
    if ((rc = ensure(c, c->in1, in_bytes)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->in2, in_bytes)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->np, pts * 8)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->st, pts)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->vec, pts * 32)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->mask, (size_t)w * h)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->H, 72)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->Hext, 72)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->num, 4)) != MDX_OK) return rc;

    hipStream_t s = c->stream;
    HIP_OR_RETURN(c, hipMemcpyAsync(c->in1.p, img1, in_bytes, hipMemcpyHostToDevice, s));
    HIP_OR_RETURN(c, hipMemcpyAsync(c->in2.p, img2, in_bytes, hipMemcpyHostToDevice, s));
    if (H_external) HIP_OR_RETURN(c, hipMemcpyAsync(c->Hext.p, H_external, 72, hipMemcpyHostToDevice, s));
    rc = run_pipeline(c, 1, c->in1.as<uint8_t>(), c->in2.as<uint8_t>(), w, h, stride, in_bytes, fmt, c->np.as<float>(),
                      c->st.as<uint8_t>(), vectors ? c->vec.as<double>() : nullptr,
                      mask ? c->mask.as<uint8_t>() : nullptr, c->H.as<double>(),
                      H_external ? c->Hext.as<double>() : nullptr, c->num.as<int>());
    if (rc != MDX_OK) return rc;
    int num = 0;
    if (next_pts && npts > 0) HIP_OR_RETURN(c, hipMemcpyAsync(next_pts, c->np.p, (size_t)npts * 8, hipMemcpyDeviceToHost, s));
    if (status && npts > 0) HIP_OR_RETURN(c, hipMemcpyAsync(status, c->st.p, (size_t)npts, hipMemcpyDeviceToHost, s));
    if (vectors && npts > 0) HIP_OR_RETURN(c, hipMemcpyAsync(vectors, c->vec.p, (size_t)npts * 32, hipMemcpyDeviceToHost, s));
    if (mask) HIP_OR_RETURN(c, hipMemcpyAsync(mask, c->mask.p, (size_t)w * h, hipMemcpyDeviceToHost, s));
    if (H) HIP_OR_RETURN(c, hipMemcpyAsync(H, c->H.p, 72, hipMemcpyDeviceToHost, s));
    HIP_OR_RETURN(c, hipMemcpyAsync(&num, c->num.p, 4, hipMemcpyDeviceToHost, s));
    HIP_OR_RETURN(c, hipStreamSynchronize(s));
    if (num_vectors) *num_vectors = num;
    if (c->prm.fit_mode != MDX_FIT_EXTERNAL && num < 4) return MDX_EDEGENERATE;
    return MDX_OK;
}

// The trajectory passes of calculateOpticalFlowTrajectory (optical_flow_calculator.cpp:143-257) over
// nimg frames whose padded pyramids and Scharr planes are on the device already: pass j tracks the
// points the previous pass left from frame j (pyr[j], der[j]) to frame j + 1 (pyr[j + 1]).  Every
// pass runs the point LK from the carried points: for one pair it is faster than the class-plane
// kernels even on the grid start points of pass 0, whose per-level tails one pair cannot fill.
extern "C" size_t mdx_trajectory_layout(int npts, int nimg, size_t offsets[4])
{
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t p = (size_t)(npts > 0 ? npts : 1), n = (size_t)(nimg > 0 ? nimg : 1);
    size_t o[4];
    o[0] = 0;
    o[1] = al(p * n * 8);
    o[2] = o[1] + al(p * 8);
    o[3] = o[2] + al(p * 32);
    if (offsets)
        for (int i = 0; i < 4; i++) offsets[i] = o[i];
    return o[3] + p * 4;
}

static int trajectory_passes(mdx_ctx* c, const Geometry& g, int nimg, int w, int h, const uint8_t* const* pyr,
                             const uint32_t* const* der, float* traj, int32_t* traj_len, float* start_pts,
                             double* vectors, int* num_vectors)
{
    const mdx_params& P = c->prm;
    const int npts = mdx_grid_count(w, h, P.pixel_step);
    const int ny = (h + P.pixel_step - 1) / P.pixel_step;
    const size_t pts = (size_t)(npts > 0 ? npts : 1);
    int rc;
    if ((rc = ensure(c, c->tcur, pts * 8)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->tnp, pts * 8)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->tst, pts)) != MDX_OK) return rc;
    // the four outputs in one block, laid out as mdx_trajectory_layout says (one readback copy
    // when the host block matches)
    size_t off[4];
    const size_t obytes = mdx_trajectory_layout(npts, nimg, off);
    if ((rc = ensure(c, c->ttraj, obytes)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->tnum, 8)) != MDX_OK) return rc;
    if (!c->tcnt_host && hipHostMalloc((void**)&c->tcnt_host, 16, hipHostMallocDefault) != hipSuccess) {
        c->tcnt_host = nullptr;
        return set_err(c, MDX_ENOMEM, "trajectory passes: hipHostMalloc(counts)");
    }
    hipStream_t s = c->stream;
    float* cur = c->tcur.as<float>();
    uint8_t* ob = c->ttraj.as<uint8_t>();
    float* tr = reinterpret_cast<float*>(ob + off[0]);
    float* tstart = reinterpret_cast<float*>(ob + off[1]);
    double* tvec = reinterpret_cast<double*>(ob + off[2]);
    int* tl = reinterpret_cast<int*>(ob + off[3]);
    int* dnum = c->tnum.as<int>();
    const bool chain = c->traj_chain && nimg <= kMaxTrajImgs && npts > 0;
    bool direct = false;   // the chained launch writes the caller's mapped outputs itself
    if (chain && (rc = ensure(c, c->tflag, pts * 4)) != MDX_OK) return rc;
    HIP_OR_RETURN(c, launch_traj_init(s, npts, ny, P.pixel_step, nimg, cur, tr, tl, dnum,
                                      chain ? c->tflag.as<int>() : nullptr));
    if (chain) {
        // every pass in one launch: pass j + 1 of a point starts as soon as its pass j is done, so
        // the passes' launch tails overlap (the per-pass launches below leave each tail idle)
        LkArgs a{};
        a.g = g;
        a.maxl = g.nlev - 1;
        a.npts = npts;
        a.ny = ny;
        a.nyg = ny;
        a.pixel_step = P.pixel_step;
        a.max_iters = std::min(std::max(P.max_iters, 0), 100);
        a.min_eig = P.min_eig;
        const double e = std::min(std::max(P.eps, 0.), 10.);
        a.eps2 = e * e;
        TrajChain t{};
        for (int j = 0; j < nimg; j++) {
            t.pyr[j] = pyr[j];
            t.der[j] = der[j];
        }
        t.nimg = nimg;
        t.w = w;
        t.h = h;
        t.cur = cur;
        t.traj = tr;
        t.tlen = tl;
        t.flag = c->tflag.as<int>();
        t.vectors = tvec;
        t.start_pts = tstart;
        // the caller's outputs in mapped page-locked memory (mdx_host_alloc): the launch writes them
        if (npts > 0 && traj && traj_len && start_pts && vectors) {
            // only whole ranges inside one mdx_host_alloc block qualify (a partly pinned or short
            // buffer takes the copy path, which reports its errors); pageable memory is never queried
            const size_t pn = (size_t)npts, nn = (size_t)nimg;
            auto mapped = [&](void* p, size_t bytes) -> void* {
                if (!host_block_holds(p, bytes)) return nullptr;
                hipPointerAttribute_t at{};
                if (hipPointerGetAttributes(&at, p) != hipSuccess) {
                    (void)hipGetLastError();
                    return nullptr;
                }
                return at.type == hipMemoryTypeHost ? at.devicePointer : nullptr;
            };
            void* m[4] = {mapped(traj, pn * nn * 8), mapped(traj_len, pn * 4), mapped(start_pts, pn * 8),
                          mapped(vectors, pn * 32)};
            if (m[0] && m[1] && m[2] && m[3]) {
                t.htraj = static_cast<float*>(m[0]);
                t.htlen = static_cast<int*>(m[1]);
                t.hstart = static_cast<float*>(m[2]);
                t.hvec = static_cast<double*>(m[3]);
                direct = true;
            }
        }
        t.num = dnum;
        t.mvs = P.min_vector_size;
        HIP_OR_RETURN(c, launch_lk_chain(s, a, t, c->traj_ppw));
    }
    for (int j = 0; !chain && j + 1 < nimg && npts > 0; j++) {
        LkArgs a{};
        a.pyr1 = pyr[j];
        a.pyr2 = pyr[j + 1];
        a.der = der[j];
        a.g = g;
        a.maxl = g.nlev - 1;
        a.npts = npts;
        a.ny = ny;
        a.nyg = ny;
        a.pixel_step = P.pixel_step;
        a.max_iters = std::min(std::max(P.max_iters, 0), 100);
        a.min_eig = P.min_eig;
        const double e = std::min(std::max(P.eps, 0.), 10.);
        a.eps2 = e * e;
        a.next_pts = c->tnp.as<float>();
        a.status = c->tst.as<uint8_t>();
        a.prev_pts = cur;
        if ((rc = run_lk(c, g, a, 1, w, h, 0, ny, true)) != MDX_OK) return rc;
        HIP_OR_RETURN(c, launch_traj_update(s, npts, c->tnp.as<float>(), c->tst.as<uint8_t>(), cur, tr, tl, nimg, w, h,
                                            j == nimg - 2, P.min_vector_size, tvec, tstart, dnum));
    }
    int num = 0;
    if (npts > 0 && !direct) {
        uint8_t* hb = reinterpret_cast<uint8_t*>(traj);
        const bool one_block = traj && start_pts && vectors && traj_len &&
                               reinterpret_cast<uint8_t*>(start_pts) == hb + off[1] &&
                               reinterpret_cast<uint8_t*>(vectors) == hb + off[2] &&
                               reinterpret_cast<uint8_t*>(traj_len) == hb + off[3];
        if (one_block) {
            HIP_OR_RETURN(c, hipMemcpyAsync(hb, ob, off[3] + (size_t)npts * 4, hipMemcpyDeviceToHost, s));
        } else {
            if (traj) HIP_OR_RETURN(c, hipMemcpyAsync(traj, tr, (size_t)npts * nimg * 8, hipMemcpyDeviceToHost, s));
            if (traj_len) HIP_OR_RETURN(c, hipMemcpyAsync(traj_len, tl, (size_t)npts * 4, hipMemcpyDeviceToHost, s));
            if (start_pts) HIP_OR_RETURN(c, hipMemcpyAsync(start_pts, tstart, (size_t)npts * 8, hipMemcpyDeviceToHost, s));
            if (vectors) HIP_OR_RETURN(c, hipMemcpyAsync(vectors, tvec, (size_t)npts * 32, hipMemcpyDeviceToHost, s));
        }
    }
    c->tcnt_host[0] = c->tcnt_host[1] = 0;
    HIP_OR_RETURN(c, hipMemcpyAsync(c->tcnt_host, dnum, chain ? 8 : 4, hipMemcpyDeviceToHost, s));
    HIP_OR_RETURN(c, hipStreamSynchronize(s));
    num = c->tcnt_host[0];
    if (chain && c->tcnt_host[1] != 0)
        return set_err(c, MDX_EHIP, "trajectory passes: %d point hand-off(s) timed out", c->tcnt_host[1]);
    if (num_vectors) *num_vectors = num;
    return MDX_OK;
}

static int check_frame(mdx_ctx* c, const char* who, int w, int h, int stride, int fmt)
{
    if (w <= 0 || h <= 0) return set_err(c, MDX_EINVAL, "%s: bad frame size", who);
    if (fmt < MDX_FMT_GRAY8 || fmt > MDX_FMT_BGR8) return set_err(c, MDX_EINVAL, "%s: bad pixel format %d", who, fmt);
    const int cn = fmt == MDX_FMT_GRAY8 ? 1 : 3;
    if (stride < w * cn) return set_err(c, MDX_EINVAL, "%s: stride %d < w*channels %d", who, stride, w * cn);
    return MDX_OK;
}

// calculateOpticalFlowTrajectory (optical_flow_calculator.cpp:133-257) on host frames.  Pair slot j
// holds frames (j, j+1): the gray / pyramid / Scharr stages run batched over all slots in one
// launch each (the reference rebuilds each frame's pyramid twice, :166-170; these are the same
// images), then the nimg-1 LK passes run in order on the points the previous pass left.
extern "C" int mdx_flow_trajectory(mdx_ctx* c, const uint8_t* const* imgs, int nimg, int w, int h, int stride,
                                   int fmt, float* traj, int32_t* traj_len, float* start_pts, double* vectors,
                                   int* num_vectors)
{
    if (!c) return MDX_EINVAL;
    if (!imgs || nimg < 2) return set_err(c, MDX_EINVAL, "mdx_flow_trajectory: need >= 2 frames");
    for (int i = 0; i < nimg; i++)
        if (!imgs[i]) return set_err(c, MDX_EINVAL, "mdx_flow_trajectory: null frame %d", i);
    int rc = check_frame(c, "mdx_flow_trajectory", w, h, stride, fmt);
    if (rc != MDX_OK) return rc;
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    const int npairs = nimg - 1;
    const Geometry g = make_geometry(w, h, c->prm.max_level);
    if ((rc = ensure_workspace(c, g, npairs, false)) != MDX_OK) return rc;
    c->band_w = c->band_h = 0;   // the slabs are rebuilt: a pending band fit/warp has nothing to read
    const size_t fbytes = (size_t)stride * h;
    if ((rc = ensure(c, c->tin, fbytes * nimg)) != MDX_OK) return rc;
    hipStream_t s = c->stream;
    uint8_t* din = c->tin.as<uint8_t>();
    for (int i = 0; i < nimg; i++)
        HIP_OR_RETURN(c, hipMemcpyAsync(din + fbytes * i, imgs[i], fbytes, hipMemcpyHostToDevice, s));
    uint8_t* pyr1 = c->pyr1.as<uint8_t>();
    uint8_t* pyr2 = c->pyr2.as<uint8_t>();
    uint32_t* der = c->der.as<uint32_t>();
    HIP_OR_RETURN(c, launch_front(s, npairs, din, din + fbytes, w, h, stride, (long long)fbytes, fmt, pyr1, pyr2, g));
    HIP_OR_RETURN(c, launch_pyr_levels(s, npairs, pyr1, pyr2, g));
    HIP_OR_RETURN(c, launch_scharr_levels(s, npairs, pyr1, der, g));
    // frame j's pyramid is slot j of pyr1 (j < nimg-1) and the last frame's slot nimg-2 of pyr2
    std::vector<const uint8_t*> fp(nimg);
    std::vector<const uint32_t*> fd(nimg);
    for (int j = 0; j < npairs; j++) {
        fp[j] = pyr1 + (size_t)g.img_bytes * j;
        fd[j] = der + (size_t)g.der_words * j;
    }
    fp[npairs] = pyr2 + (size_t)g.img_bytes * (npairs - 1);
    fd[npairs] = nullptr;
    rc = trajectory_passes(c, g, nimg, w, h, fp.data(), fd.data(), traj, traj_len, start_pts, vectors, num_vectors);
    release_pyr_all(c);
    return rc;
}

// The resident ring (include/mdx.h): slot k of ring_pyr / ring_der holds one frame's padded pyramid
// and Scharr planes; ring_order lists the held slots oldest first.
static int ring_grow(mdx_ctx* c, const Geometry& g, int cap)
{
    if (cap <= c->ring_cap) return MDX_OK;
    DevBuf np, nd;
    auto fail = [&](const char* what) {
        if (np.p) (void)hipFree(np.p);
        if (nd.p) (void)hipFree(nd.p);
        return set_err(c, MDX_ENOMEM, "mdx_ring_push: %s", what);
    };
    if (hipMalloc(&np.p, (size_t)g.img_bytes * cap) != hipSuccess) return fail("hipMalloc(pyramids)");
    if (hipMalloc(&nd.p, (size_t)g.der_words * 4 * cap) != hipSuccess) return fail("hipMalloc(derivatives)");
    np.cap = (size_t)g.img_bytes * cap;
    nd.cap = (size_t)g.der_words * 4 * cap;
    // the held frames move to slots 0 .. n-1, in order; the context's state changes only once
    // every copy has landed (a failed copy leaves the old ring intact and frees the new buffers)
    std::vector<int> order(c->ring_order.size());
    for (size_t k = 0; k < c->ring_order.size(); k++) {
        const int o = c->ring_order[k];
        if (hipMemcpyAsync(np.as<uint8_t>() + (size_t)g.img_bytes * k, c->ring_pyr.as<uint8_t>() + (size_t)g.img_bytes * o,
                           g.img_bytes, hipMemcpyDeviceToDevice, c->stream) != hipSuccess ||
            hipMemcpyAsync(nd.as<uint8_t>() + (size_t)g.der_words * 4 * k,
                           c->ring_der.as<uint8_t>() + (size_t)g.der_words * 4 * o, (size_t)g.der_words * 4,
                           hipMemcpyDeviceToDevice, c->stream) != hipSuccess) {
            (void)hipStreamSynchronize(c->stream);
            return fail("slot copy failed");
        }
        order[k] = (int)k;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return fail("slot copy failed");
    c->ring_order = order;
    if (c->ring_pyr.p) (void)hipFree(c->ring_pyr.p);
    if (c->ring_der.p) (void)hipFree(c->ring_der.p);
    c->ring_pyr = np;
    c->ring_der = nd;
    c->ring_cap = cap;
    return MDX_OK;
}

extern "C" int mdx_ring_reset(mdx_ctx* c)
{
    if (!c) return MDX_EINVAL;
    c->ring_order.clear();
    return MDX_OK;
}

extern "C" int mdx_ring_push(mdx_ctx* c, const uint8_t* img, int w, int h, int stride, int fmt, int keep)
{
    if (!c) return MDX_EINVAL;
    if (!img) return set_err(c, MDX_EINVAL, "mdx_ring_push: null frame");
    if (keep < 1) return set_err(c, MDX_EINVAL, "mdx_ring_push: keep must be >= 1");
    int rc = check_frame(c, "mdx_ring_push", w, h, stride, fmt);
    if (rc != MDX_OK) return rc;
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    if (w != c->ring_w || h != c->ring_h || c->prm.max_level != c->ring_ml) {   // another geometry: start over
        c->ring_order.clear();
        if (c->ring_pyr.p) (void)hipStreamSynchronize(c->stream);
        if (c->ring_pyr.p) (void)hipFree(c->ring_pyr.p);
        if (c->ring_der.p) (void)hipFree(c->ring_der.p);
        c->ring_pyr = DevBuf{};
        c->ring_der = DevBuf{};
        c->ring_cap = 0;
        c->ring_w = w;
        c->ring_h = h;
        c->ring_ml = c->prm.max_level;
    }
    const Geometry g = make_geometry(w, h, c->prm.max_level);
    const int n = (int)c->ring_order.size();
    if ((rc = ring_grow(c, g, std::max(n + 1, std::max(keep, 4)))) != MDX_OK) return rc;
    // a free slot: the lowest one no held frame uses
    std::vector<char> used(c->ring_cap, 0);
    for (int o : c->ring_order) used[o] = 1;
    int slot = 0;
    while (used[slot]) slot++;
    const size_t fbytes = (size_t)stride * h;
    if ((rc = ensure(c, c->rin, fbytes)) != MDX_OK) return rc;
    hipStream_t s = c->stream;
    HIP_OR_RETURN(c, hipMemcpyAsync(c->rin.p, img, fbytes, hipMemcpyHostToDevice, s));
    uint8_t* pyr = c->ring_pyr.as<uint8_t>() + (size_t)g.img_bytes * slot;
    uint32_t* der = c->ring_der.as<uint32_t>() + (size_t)g.der_words * slot;
    HIP_OR_RETURN(c, launch_front(s, 1, c->rin.as<uint8_t>(), c->rin.as<uint8_t>(), w, h, stride, (long long)fbytes, fmt,
                                  pyr, pyr, g, 1));
    HIP_OR_RETURN(c, launch_pyr_levels(s, 1, pyr, pyr, g, 1));
    HIP_OR_RETURN(c, launch_scharr_levels(s, 1, pyr, der, g));
    c->ring_order.push_back(slot);
    while ((int)c->ring_order.size() > keep) c->ring_order.erase(c->ring_order.begin());
    return (int)c->ring_order.size();
}

extern "C" int mdx_ring_trajectory(mdx_ctx* c, float* traj, int32_t* traj_len, float* start_pts, double* vectors,
                                   int* num_vectors)
{
    if (!c) return MDX_EINVAL;
    const int nimg = (int)c->ring_order.size();
    if (nimg < 2) return set_err(c, MDX_EINVAL, "mdx_ring_trajectory: the ring holds %d frame(s), need >= 2", nimg);
    if (c->prm.max_level != c->ring_ml)
        return set_err(c, MDX_EINVAL, "mdx_ring_trajectory: max_level changed since the frames were pushed");
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    const Geometry g = make_geometry(c->ring_w, c->ring_h, c->prm.max_level);
    std::vector<const uint8_t*> fp(nimg);
    std::vector<const uint32_t*> fd(nimg);
    for (int j = 0; j < nimg; j++) {
        fp[j] = c->ring_pyr.as<uint8_t>() + (size_t)g.img_bytes * c->ring_order[j];
        fd[j] = c->ring_der.as<uint32_t>() + (size_t)g.der_words * c->ring_order[j];
    }
    return trajectory_passes(c, g, nimg, c->ring_w, c->ring_h, fp.data(), fd.data(), traj, traj_len, start_pts, vectors,
                             num_vectors);
}

// glibc rand() (random_r TYPE_3), the generator of fitSubspace's samples
// (outlier_detector.cpp:17 srand(time(NULL)), :226 rand() % data.cols()).
extern "C" void mdx_srand(mdx_rand_state* st, uint32_t seed)
{
    int32_t r[34];
    r[0] = (int32_t)(seed ? seed : 1u);
    for (int i = 1; i < 31; i++) {
        const int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int64_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    for (int i = 0; i < 34; i++) st->x[i] = (uint32_t)r[i];
    st->pos = 34;
    for (int k = 0; k < 310; k++) (void)mdx_rand(st);
}

extern "C" int mdx_rand(mdx_rand_state* st)
{
    const int i = st->pos;                       // ring of 34: x[i] = x[i-31] + x[i-3]
    const uint32_t v = st->x[(i - 31) % 34] + st->x[(i - 3) % 34];
    st->x[i % 34] = v;
    st->pos = (i + 1) % 34 + 34;
    return (int)(v >> 1);
}

// fitSubspace (outlier_detector.cpp:236-331): samples drawn on the host from the caller's
// generator state (the reference's OutlierDetector keeps one stream across calls), the rest on
// the device (mdx_subspace.hip).
extern "C" int mdx_fit_subspace(mdx_ctx* c, const float* traj, int ntraj, int traj_len, int num_motions, double sigma,
                                mdx_rand_state* rng, int* columns, uint8_t* is_outlier, double* residuals,
                                float* outlier_points, int* n_outliers)
{
    if (!c) return MDX_EINVAL;
    const int n = 2 * traj_len, d = 4 * num_motions;
    if (!traj || !rng || ntraj <= 0 || traj_len < 1 || num_motions < 1)
        return set_err(c, MDX_EINVAL, "mdx_fit_subspace: bad argument (the reference needs >= 1 trajectory: rand() %% 0)");
    if (d > n) return set_err(c, MDX_EINVAL, "mdx_fit_subspace: 4*num_motions > 2*traj_len (reference reads U past its columns)");
    if (n > 32) return set_err(c, MDX_EINVAL, "mdx_fit_subspace: trajectories longer than 16 points");
    if (n - d == 10) return set_err(c, MDX_EINVAL, "mdx_fit_subspace: n - d == 10 (reference chi_square_table.at(10) throws)");
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    constexpr int kHyp = 50;                      // num_iterations (:250)
    std::vector<int> cols((size_t)kHyp * d);
    for (auto& v : cols) v = mdx_rand(rng) % ntraj;   // fillSubset, hypothesis by hypothesis (:223-230)
    const size_t N = (size_t)ntraj;
    int rc;
    if ((rc = ensure(c, c->straj, N * n * 4)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->sdata, (N * n + 2) * 4)) != MDX_OK) return rc;   // + the two means
    const size_t qb = std::max((size_t)n * std::max(n - d, 1) * 8, (size_t)n * n * 4);   // F64 basis / F32 Pnd
    if ((rc = ensure(c, c->sq, (size_t)kHyp * qb)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->scnt, kHyp * 4)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->scols, cols.size() * 4)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->sres, N * 8)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->sout, N)) != MDX_OK) return rc;
    if ((rc = ensure(c, c->sbest, 4)) != MDX_OK) return rc;
    hipStream_t s = c->stream;
    HIP_OR_RETURN(c, hipMemcpyAsync(c->straj.p, traj, N * n * 4, hipMemcpyHostToDevice, s));
    HIP_OR_RETURN(c, hipMemcpyAsync(c->scols.p, cols.data(), cols.size() * 4, hipMemcpyHostToDevice, s));
    HIP_OR_RETURN(c, launch_subspace(s, c->straj.as<float>(), ntraj, traj_len, d, c->scols.as<int>(), kHyp, sigma,
                                     c->sdata.as<float>(), c->sq.as<double>(), c->scnt.as<int>(), c->sres.as<double>(),
                                     c->sout.as<uint8_t>(), c->sbest.as<int>(), c->prm.subspace_precision));
    std::vector<uint8_t> out(N);
    int best = -1;
    HIP_OR_RETURN(c, hipMemcpyAsync(out.data(), c->sout.p, N, hipMemcpyDeviceToHost, s));
    if (residuals) HIP_OR_RETURN(c, hipMemcpyAsync(residuals, c->sres.p, N * 8, hipMemcpyDeviceToHost, s));
    HIP_OR_RETURN(c, hipMemcpyAsync(&best, c->sbest.p, 4, hipMemcpyDeviceToHost, s));
    HIP_OR_RETURN(c, hipStreamSynchronize(s));
    int nout = 0;
    for (size_t i = 0; i < N; i++) {
        if (!out[i]) continue;
        if (outlier_points) {     // the trajectory's second-to-last point (:322)
            const int j = traj_len >= 2 ? traj_len - 2 : 0;
            outlier_points[2 * nout] = traj[(i * traj_len + j) * 2];
            outlier_points[2 * nout + 1] = traj[(i * traj_len + j) * 2 + 1];
        }
        nout++;
    }
    if (is_outlier) std::memcpy(is_outlier, out.data(), N);
    if (columns) {
        if (best >= 0)
            std::memcpy(columns, cols.data() + (size_t)best * d, (size_t)d * 4);
        else
            for (int k = 0; k < d; k++) columns[k] = -1;
    }
    if (n_outliers) *n_outliers = nout;
    return MDX_OK;
}

extern "C" int mdx_warp_diff_dev(mdx_ctx* c, int batch, const uint8_t* d_gray1, const uint8_t* d_gray2, int w, int h,
                                 int stride, size_t frame_stride, const double* d_H, uint8_t* d_mask)
{
    if (!c) return MDX_EINVAL;
    if (!d_gray1 || !d_gray2 || !d_H || !d_mask || batch <= 0 || w <= 0 || h <= 0 || stride < w)
        return set_err(c, MDX_EINVAL, "mdx_warp_diff_dev: bad argument");
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    int rc = ensure(c, c->fits, sizeof(PairFit) * (size_t)batch);
    if (rc != MDX_OK) return rc;
    hipStream_t s = c->stream;
    PairFit* fits = c->fits.as<PairFit>();
    if ((rc = wait_input(c, s)) != MDX_OK) return rc;
    for (int i = 0; i < 5; i++) mark(c, i);
    HIP_OR_RETURN(c, launch_set_fit_external(s, batch, d_H, fits));
    mark(c, 5);
    const size_t wsb = warp_scratch_bytes(batch, w, h);
    if ((rc = ensure(c, c->wscr, wsb)) != MDX_OK) return rc;
    HIP_OR_RETURN(c, launch_warp_diff(s, batch, d_gray1, (long long)frame_stride, stride, d_gray2,
                                      (long long)frame_stride, stride, w, h, fits, d_mask, (long long)w * h,
                                      c->prm.thresh, c->wscr.p, wsb));
    mark(c, 6);
    return MDX_OK;
}

extern "C" int mdx_probe_stream3_dev(mdx_ctx* c, size_t n, const uint8_t* d_a, const uint8_t* d_b, uint8_t* d_mask,
                                     int thresh)
{
    if (!c) return MDX_EINVAL;
    if (!d_a || !d_b || !d_mask || n == 0 || n % 16 || ((uintptr_t)d_a | (uintptr_t)d_b | (uintptr_t)d_mask) % 16)
        return set_err(c, MDX_EINVAL, "mdx_probe_stream3_dev: bad argument");
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    for (int i = 0; i < 6; i++) mark(c, i);
    HIP_OR_RETURN(c, launch_stream3(c->stream, n, d_a, d_b, d_mask, thresh));
    mark(c, 6);
    return MDX_OK;
}

extern "C" int mdx_band_flow_dev(mdx_ctx* c, const uint8_t* d_img1, const uint8_t* d_img2, int w, int h, int stride,
                                 int fmt, int y0, int y1, float* d_next_pts, uint8_t* d_status, double* d_vectors,
                                 mdx_band_cand* d_cand)
{
    if (!c) return MDX_EINVAL;
    if (!d_img1 || !d_img2 || !d_next_pts || !d_status || !d_cand)
        return set_err(c, MDX_EINVAL, "mdx_band_flow_dev: null pointer");
    if (w <= 0 || h <= 0 || y0 < 0 || y1 > h || y0 >= y1) return set_err(c, MDX_EINVAL, "bad band [%d, %d) of %d rows", y0, y1, h);
    if (c->prm.fit_mode != MDX_FIT_FIRST4) return set_err(c, MDX_EINVAL, "row bands need fit_mode FIRST4");
    const int ps = c->prm.pixel_step;
    // grid rows whose y = gy*ps lies in [y0, y1)
    const int gy0 = (y0 + ps - 1) / ps, gy1 = (y1 + ps - 1) / ps;
    c->band_w = c->band_h = 0;
    const int rc = run_pipeline(c, 1, d_img1, d_img2, w, h, stride, (size_t)stride * h, fmt, d_next_pts, d_status,
                                d_vectors, nullptr, nullptr, nullptr, nullptr, gy0, gy1, d_cand, true);
    if (rc == MDX_OK) {
        c->band_w = w;
        c->band_h = h;
        c->band_img1 = d_img1;
        c->band_stride = stride;
        c->band_fmt = fmt;
    }
    return rc;
}

extern "C" int mdx_band_fit_warp_dev(mdx_ctx* c, int nrec, const mdx_band_cand* d_cands, int y0, int y1,
                                     uint8_t* d_mask_band, double* d_H, int* d_num_vectors)
{
    if (!c) return MDX_EINVAL;
    if (nrec <= 0 || !d_cands || !d_mask_band) return set_err(c, MDX_EINVAL, "mdx_band_fit_warp_dev: bad argument");
    const int w = c->band_w, h = c->band_h;
    if (w <= 0 || h <= 0)
        return set_err(c, MDX_EINVAL, "mdx_band_fit_warp_dev: no mdx_band_flow_dev before, or another call rebuilt "
                                      "the context's pyramids since");
    if (y0 < 0 || y1 > h || y0 >= y1) return set_err(c, MDX_EINVAL, "bad band [%d, %d) of %d rows", y0, y1, h);
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    const Geometry g = make_geometry(w, h, c->prm.max_level);
    hipStream_t s = c->stream;
    PairFit* fits = c->fits.as<PairFit>();
    if (!c->band_pyr1 || !c->band_img1) return set_err(c, MDX_EINVAL, "mdx_band_fit_warp_dev: no mdx_band_flow_dev before");
    HIP_OR_RETURN(c, launch_band_fit(s, nrec, d_cands, fits, w, h, y0, y1));
    const Level& L0 = g.lv[0];
    // the band's flow built frame 1's pyramid for its own rows only: the rows this band's warp
    // reads beyond them (the fit is known now) are converted from the frame
    HIP_OR_RETURN(c, launch_gray_rows(s, c->band_img1, w, h, c->band_stride, c->band_fmt,
                                      c->band_pyr1 + L0.img_off + L0.core(), L0.pitch, fits, c->band_built[0],
                                      c->band_built[1]));
    const uint8_t* g1 = c->band_pyr1 + L0.img_off + L0.core();
    const uint8_t* g2 = c->band_pyr2 + L0.img_off + L0.core();
    const size_t wsb = warp_scratch_bytes(1, w, y1 - y0);
    if (const int erc = ensure(c, c->wscr, wsb); erc != MDX_OK) return erc;
    HIP_OR_RETURN(c, launch_warp_diff(s, 1, g1, g.img_bytes, L0.pitch, g2, g.img_bytes, L0.pitch, w, h, fits, d_mask_band,
                                      (long long)w * (y1 - y0), c->prm.thresh, c->wscr.p, wsb, y0, y1));
    if (d_H || d_num_vectors) HIP_OR_RETURN(c, launch_export_fit(s, 1, fits, d_H, d_num_vectors));
    // the band's pyramids have been read: the pipelined call two calls on may overwrite them
    if (c->prm.call_pipelining) HIP_OR_RETURN(c, hipEventRecord(c->pyr_free[c->band_half], s));
    else release_pyr_all(c);
    return MDX_OK;
}

// Test hook: copy an internal LK v2 buffer to the host (0 = A sums, 1 = per-level trace).
#if MDX_WARP_STAMP
namespace mdx { hipError_t debug_warp_stamps(void* dst, size_t bytes); }
#endif
extern "C" int mdx_debug_copy(mdx_ctx* c, int which, void* dst, size_t bytes)
{
    if (!c || !dst) return MDX_EINVAL;
#if MDX_WARP_STAMP
    if (which == 99) {   // diagnostic build: the warp's in-kernel clock stamps (scripts/warp_burst.py)
        HIP_OR_RETURN(c, hipDeviceSynchronize());
        HIP_OR_RETURN(c, debug_warp_stamps(dst, bytes));
        return MDX_OK;
    }
#endif
    DevBuf& b = which == 0 ? c->Abuf : which == 1 ? c->dbg : which == 2 ? c->pyr1 : which == 3 ? c->pyr2
              : which == 4 ? c->der : c->cls;
    if (!b.p) return set_err(c, MDX_EINVAL, "debug buffer %d unavailable", which);
    HIP_OR_RETURN(c, hipStreamSynchronize(c->stream));
    // pyramids: the half the last pair call wrote
    const uint8_t* src = static_cast<const uint8_t*>(b.p);
    if (which == 2 && c->last_pyr1) src = c->last_pyr1;
    if (which == 3 && c->last_pyr2) src = c->last_pyr2;
    const size_t avail = b.cap - (size_t)(src - static_cast<const uint8_t*>(b.p));
    HIP_OR_RETURN(c, hipMemcpy(dst, src, bytes < avail ? bytes : avail, hipMemcpyDeviceToHost));
    return MDX_OK;
}

extern "C" int mdx_debug_div32(mdx_ctx* c, const double* d_in, double* d_out, int n)
{
    if (!c || !d_in || !d_out || n <= 0) return MDX_EINVAL;
    HIP_OR_RETURN(c, hipSetDevice(c->device));
    HIP_OR_RETURN(c, launch_div32(c->stream, d_in, d_out, n));
    return MDX_OK;
}

extern "C" void* mdx_host_alloc(size_t bytes)
{
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_blocks[reinterpret_cast<uintptr_t>(p)] = bytes ? bytes : 1;
    return p;
}

extern "C" int mdx_host_free(void* p)
{
    if (!p) return MDX_OK;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        g_host_blocks.erase(reinterpret_cast<uintptr_t>(p));
    }
    return hipHostFree(p) == hipSuccess ? MDX_OK : MDX_EHIP;
}

extern "C" void* mdx_dev_alloc(mdx_ctx* c, size_t bytes)
{
    if (!c) return nullptr;
    (void)hipSetDevice(c->device);
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        set_err(c, MDX_ENOMEM, "hipMalloc(%zu) failed", bytes);
        return nullptr;
    }
    return p;
}

extern "C" int mdx_dev_free(mdx_ctx* c, void* p)
{
    if (!c) return MDX_EINVAL;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    HIP_OR_RETURN(c, hipFree(p));
    return MDX_OK;
}

extern "C" int mdx_memcpy_h2d(mdx_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c) return MDX_EINVAL;
    HIP_OR_RETURN(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_OR_RETURN(c, hipStreamSynchronize(c->stream));
    return MDX_OK;
}

extern "C" int mdx_memcpy_d2h(mdx_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c) return MDX_EINVAL;
    HIP_OR_RETURN(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_OR_RETURN(c, hipStreamSynchronize(c->stream));
    return MDX_OK;
}
