// C4 one-band timer for same-box A/B of libmdx.so builds from different revisions (the band API
// has been unchanged since ABI 2).  Mirrors bench.py main_c4's one_band_ms leg: one 8K RGB pair,
// F contexts (frames in flight), band b of K; per repetition every context queues its band flow,
// then every context its band fit + warp; time per band and frame after a warmup.
// Build (CPU side): g++ -O2 -std=c++17 -I include scripts/micro/c4_band_timer.cpp -ldl -o scripts/micro/bin/c4_band_timer
// Run (GPU box):    scripts/micro/bin/c4_band_timer <libmdx.so> [reps] [F] [band] [K]
#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mdx.h"

#define SYM(name) auto name = reinterpret_cast<decltype(&::name)>(dlsym(h, #name)); \
    if (!name) { std::fprintf(stderr, "missing %s\n", #name); return 2; }

int main(int argc, char** argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: %s libmdx.so [reps] [F] [band] [K]\n", argv[0]); return 2; }
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    const int F = argc > 3 ? std::atoi(argv[3]) : 2;
    const int band = argc > 4 ? std::atoi(argv[4]) : 0;
    const int K = argc > 5 ? std::atoi(argv[5]) : 8;
    void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) { std::fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
    SYM(mdx_default_params) SYM(mdx_create) SYM(mdx_create_error) SYM(mdx_dev_alloc) SYM(mdx_memcpy_h2d)
    SYM(mdx_synth_pair) SYM(mdx_band_flow_dev) SYM(mdx_band_fit_warp_dev) SYM(mdx_device_sync) SYM(mdx_destroy)
    SYM(mdx_grid_count) SYM(mdx_last_error) SYM(mdx_memcpy_d2h)
    const int w = 7680, hh = 4320, ps = 10;
    std::vector<uint8_t> a((size_t)w * hh * 3), b((size_t)w * hh * 3);
    if (mdx_synth_pair(20141105ull + 4, w, hh, 3, a.data(), b.data(), nullptr, 16) != 0) return 3;
    alignas(16) unsigned char prm[1024] = {};   // larger than any revision's mdx_params
    mdx_default_params(reinterpret_cast<mdx_params*>(prm));
    reinterpret_cast<mdx_params*>(prm)->pixel_step = ps;
    reinterpret_cast<mdx_params*>(prm)->min_vector_size = 1.0;
    const int n = mdx_grid_count(w, hh, ps);
    const int y0 = (hh * band) / K, y1 = (hh * (band + 1)) / K;
    struct Ctx { mdx_ctx* c; uint8_t *i1, *i2, *st, *mask; float* np; mdx_band_cand *cand, *cands; int* num; };
    std::vector<Ctx> cs(F);
    for (auto& x : cs) {
        x.c = mdx_create(0, w, hh, 1, reinterpret_cast<mdx_params*>(prm));
        if (!x.c) { std::fprintf(stderr, "create: %s\n", mdx_create_error()); return 3; }
        x.i1 = (uint8_t*)mdx_dev_alloc(x.c, a.size());
        x.i2 = (uint8_t*)mdx_dev_alloc(x.c, b.size());
        x.np = (float*)mdx_dev_alloc(x.c, (size_t)n * 8);
        x.st = (uint8_t*)mdx_dev_alloc(x.c, n);
        x.cand = (mdx_band_cand*)mdx_dev_alloc(x.c, 96);
        x.cands = (mdx_band_cand*)mdx_dev_alloc(x.c, 96 * K);
        x.mask = (uint8_t*)mdx_dev_alloc(x.c, (size_t)w * hh);
        x.num = (int*)mdx_dev_alloc(x.c, 4);
        mdx_memcpy_h2d(x.c, x.i1, a.data(), a.size());
        mdx_memcpy_h2d(x.c, x.i2, b.data(), b.size());
        std::vector<unsigned char> zero(96 * K, 0);
        mdx_memcpy_h2d(x.c, x.cands, zero.data(), zero.size());
    }
    auto rep = [&]() {
        for (auto& x : cs)
            if (mdx_band_flow_dev(x.c, x.i1, x.i2, w, hh, w * 3, MDX_FMT_RGB8, y0, y1, x.np, x.st, nullptr, x.cand) < 0)
                return false;
        for (auto& x : cs)
            if (mdx_band_fit_warp_dev(x.c, K, x.cands, y0, y1, x.mask + (size_t)y0 * w, nullptr, x.num) < 0)
                return false;
        return true;
    };
    // the records every band's fit sees: all K bands' real records (bench.py's exchange), made once
    std::vector<unsigned char> recs(96 * K);
    for (int k = 0; k < K; k++) {
        const int b0 = (hh * k) / K, b1 = (hh * (k + 1)) / K;
        if (mdx_band_flow_dev(cs[0].c, cs[0].i1, cs[0].i2, w, hh, w * 3, MDX_FMT_RGB8, b0, b1, cs[0].np, cs[0].st,
                              nullptr, cs[0].cand) < 0)
            return 4;
        mdx_device_sync(cs[0].c);
        mdx_memcpy_d2h(cs[0].c, recs.data() + 96 * k, cs[0].cand, 96);
    }
    for (auto& x : cs) mdx_memcpy_h2d(x.c, x.cands, recs.data(), recs.size());
    for (int i = 0; i < 3; i++) if (!rep()) { std::fprintf(stderr, "call: %s\n", mdx_last_error(cs[0].c)); return 4; }
    for (auto& x : cs) mdx_device_sync(x.c);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; i++) if (!rep()) { std::fprintf(stderr, "call: %s\n", mdx_last_error(cs[0].c)); return 4; }
    for (auto& x : cs) mdx_device_sync(x.c);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%s band %d of %d F=%d: %.3f ms per band and frame\n", argv[1], band, K, F, ms / (reps * F));
    for (auto& x : cs) mdx_destroy(x.c);
    return 0;
}
