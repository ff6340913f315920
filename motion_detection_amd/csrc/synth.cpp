// synth.cpp -- deterministic synthetic frame pairs for the benchmark and tests
// (mdx_synth_pair in include/mdx.h; spec in DESIGN.md §5).  Host-only, integer + IEEE
// double arithmetic compiled with -ffp-contract=off, so every x86-64 host produces the
// same bytes for the same (seed, w, h, channels).
#include "../../include/mdx.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline uint64_t hash2(uint64_t seed, uint64_t i) { return mix64(mix64(seed) ^ (i * 0xD1B54A32D192ED03ull)); }

inline int reflect(int p, int n)
{
    if (n == 1) return 0;
    const int period = 2 * n - 2;
    p %= period;
    if (p < 0) p += period;
    return p < n ? p : period - p;
}

template <typename F>
void parallel_rows(int h, int nthreads, F&& fn)
{
    nthreads = std::max(1, std::min(nthreads, h));
    if (nthreads == 1) { fn(0, h); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) {
        const int y0 = (int)((long long)h * t / nthreads), y1 = (int)((long long)h * (t + 1) / nthreads);
        th.emplace_back([&fn, y0, y1] { fn(y0, y1); });
    }
    for (auto& x : th) x.join();
}

// Blurred value noise (7-tap binomial, sigma ~1.2 px), contrast x3 around 128, then
// rectangles drawn in order.  One channel.
void make_texture(uint64_t seed, int w, int h, uint8_t* out, int nthreads)
{
    static const int k[7] = {1, 6, 15, 20, 15, 6, 1};
    std::vector<int> hor((size_t)w * h);
    parallel_rows(h, nthreads, [&](int y0, int y1) {
        for (int y = y0; y < y1; y++)
            for (int x = 0; x < w; x++) {
                int acc = 0;
                for (int t = 0; t < 7; t++) {
                    const int xx = reflect(x + t - 3, w);
                    acc += k[t] * (int)(hash2(seed, (uint64_t)y * (uint64_t)w + (uint64_t)xx) >> 56);
                }
                hor[(size_t)y * w + x] = acc;
            }
    });
    parallel_rows(h, nthreads, [&](int y0, int y1) {
        for (int y = y0; y < y1; y++)
            for (int x = 0; x < w; x++) {
                int acc = 0;
                for (int t = 0; t < 7; t++) acc += k[t] * hor[(size_t)reflect(y + t - 3, h) * w + x];
                const int b = (acc + 2048) >> 12;
                out[(size_t)y * w + x] = (uint8_t)std::min(255, std::max(0, 128 + (b - 128) * 3));
            }
    });
    const uint64_t rs = mix64(seed ^ 0x5EC7A9u);
    const int nrect = 16;
    for (int r = 0; r < nrect; r++) {
        const uint64_t a = hash2(rs, (uint64_t)r * 4), b = hash2(rs, (uint64_t)r * 4 + 1);
        const uint64_t c = hash2(rs, (uint64_t)r * 4 + 2), d = hash2(rs, (uint64_t)r * 4 + 3);
        const int maxs = std::max(8, std::min(w, h) / 8);
        const int rw = 8 + (int)(c % (uint64_t)maxs), rh = 8 + (int)(d % (uint64_t)maxs);
        const int x0 = (int)(a % (uint64_t)w), y0 = (int)(b % (uint64_t)h);
        const uint8_t v = (uint8_t)(hash2(rs, 1000 + (uint64_t)r) >> 56);
        for (int y = y0; y < std::min(h, y0 + rh); y++)
            for (int x = x0; x < std::min(w, x0 + rw); x++) out[(size_t)y * w + x] = v;
    }
}

}  // namespace

extern "C" int mdx_synth_pair(uint64_t seed, int w, int h, int channels, uint8_t* img1, uint8_t* img2, double* H_true,
                              int nthreads)
{
    if (w <= 0 || h <= 0 || (channels != 1 && channels != 3) || !img1 || !img2) return MDX_EINVAL;
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
    // H_true: p2 = s R(theta) (p1 - c) + c + t, theta = 0.5 deg, s = 1.01, t = (3.2, -1.7)
    const double cth = 0.99996192306417131, sth = 0.0087265354983739347;  // cos/sin(0.5 deg)
    const double sc = 1.01, cx = w * 0.5, cy = h * 0.5, tx = 3.2, ty = -1.7;
    const double a = sc * cth, b = sc * sth;
    const double Hf[9] = {a, -b, cx - a * cx + b * cy + tx, b, a, cy - b * cx - a * cy + ty, 0.0, 0.0, 1.0};
    if (H_true) std::memcpy(H_true, Hf, sizeof(Hf));
    // inverse map used to render frame 2: p1 = R^-1 (p2 - c - t) / s + c
    const double ia = cth / sc, ib = sth / sc;
    // moving patch: ~10% of the area, moved by (+8, +5) between the frames
    const int mx0 = (int)(w * 0.55), mx1 = std::min(w, mx0 + (int)(w * 0.30));
    const int my0 = (int)(h * 0.30), my1 = std::min(h, my0 + (int)(h * 0.33));
    std::vector<uint8_t> plane((size_t)w * h), warped((size_t)w * h);
    for (int ch = 0; ch < channels; ch++) {
        make_texture(seed * 7919u + (uint64_t)ch * 104729u + 1u, w, h, plane.data(), nthreads);
        parallel_rows(h, nthreads, [&](int y0, int y1) {
            for (int y = y0; y < y1; y++)
                for (int x = 0; x < w; x++) {
                    int v;
                    if (x >= mx0 && x < mx1 && y >= my0 && y < my1) {
                        const int sx = std::max(0, x - 8), sy = std::max(0, y - 5);
                        v = plane[(size_t)sy * w + sx];
                    } else {
                        const double dx = x - cx - tx, dy = y - cy - ty;
                        const double sxf = ia * dx + ib * dy + cx;
                        const double syf = -ib * dx + ia * dy + cy;
                        const double fx = std::floor(sxf), fy = std::floor(syf);
                        const int ix = (int)fx, iy = (int)fy;
                        const int ax = (int)((sxf - fx) * 256.0), ay = (int)((syf - fy) * 256.0);
                        const int x0 = std::min(std::max(ix, 0), w - 1), x1 = std::min(std::max(ix + 1, 0), w - 1);
                        const int y0_ = std::min(std::max(iy, 0), h - 1), y1_ = std::min(std::max(iy + 1, 0), h - 1);
                        const int p00 = plane[(size_t)y0_ * w + x0], p01 = plane[(size_t)y0_ * w + x1];
                        const int p10 = plane[(size_t)y1_ * w + x0], p11 = plane[(size_t)y1_ * w + x1];
                        const int top = p00 * (256 - ax) + p01 * ax, bot = p10 * (256 - ax) + p11 * ax;
                        v = (top * (256 - ay) + bot * ay + 32768) >> 16;
                    }
                    const int noise = (int)(hash2(seed ^ 0xA5A5A5A5ull, ((uint64_t)ch << 40) + (uint64_t)y * w + x) % 5) - 2;
                    warped[(size_t)y * w + x] = (uint8_t)std::min(255, std::max(0, v + noise));
                }
        });
        for (size_t i = 0; i < (size_t)w * h; i++) {
            img1[i * channels + ch] = plane[i];
            img2[i * channels + ch] = warped[i];
        }
    }
    return MDX_OK;
}
