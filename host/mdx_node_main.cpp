// mdx_node -- drives mdx_host::MotionDetectionNode (C++, over libmdx.so) from a recorded frame stream,
// the way ros::spin delivers ~input_image to imageCallback (node.cpp:63, :575).
//
//   mdx_node <frames.bin> <outdir> [pixel_step=10] [min_vector_size=1.0] [skip_frames=1]
//            [num_motions=2] [egomotion=1] [live_path=1] [sigma=0.5] [seed=1] [device=0]
//            [subspace_precision=0]   (0 double, 1 the reference's float arithmetic shape)
//
// frames.bin: "MDXF", u32 count, then per frame u32 height, u32 width, u32 step, u32 len, the
// encoding (len bytes) and step * height data bytes (a sensor_msgs/Image each).
// For the k-th processed frame it writes to <outdir>:
//   pub_<k>_<topic>.rgb8          every published image (raw RGB8, step 3 * width)
//   res_<k>.bin                   i32 num_vectors, rc, w, h, npts, ntraj, traj_len, nout; f64 H[9];
//                                 pair: f32 next_pts[2 npts], u8 status[npts], u8 mask[w h];
//                                 live: f32 trajectories[ntraj][traj_len][2], f32 outliers[nout][2],
//                                 i32 ncols, i32 columns[ncols]
//   flow_<k>_h, flow_<k>_f        writeFlow of the node's vector image (optical_flow_calculator.cpp:509)
//   traj_<k>                      writeTrajectories (live path, :543)
// (The reference's MotionLogger logs the live branch's cluster rectangles, node.cpp:431-434; the
// clustering is out of scope, so no motion.log is written.)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "mdx_host.h"

using namespace mdx_host;

static std::vector<Image> read_frames(const char* path)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) throw std::runtime_error(std::string("cannot open ") + path);
    char magic[4];
    uint32_t n = 0;
    if (std::fread(magic, 1, 4, f) != 4 || std::memcmp(magic, "MDXF", 4) != 0 || std::fread(&n, 4, 1, f) != 1)
        throw std::runtime_error("bad frames header");
    std::vector<Image> out(n);
    for (uint32_t i = 0; i < n; i++) {
        uint32_t hdr[4];
        if (std::fread(hdr, 4, 4, f) != 4) throw std::runtime_error("truncated frame header");
        Image& im = out[i];
        im.height = hdr[0];
        im.width = hdr[1];
        im.step = hdr[2];
        im.encoding.resize(hdr[3]);
        im.data.resize((size_t)im.step * im.height);
        if (std::fread(&im.encoding[0], 1, hdr[3], f) != hdr[3] ||
            std::fread(im.data.data(), 1, im.data.size(), f) != im.data.size())
            throw std::runtime_error("truncated frame data");
    }
    std::fclose(f);
    return out;
}

static void write_bytes(const std::string& path, const void* p, size_t n)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(p, 1, n, f) != n) throw std::runtime_error("cannot write " + path);
    std::fclose(f);
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <frames.bin> <outdir> [key=value ...]\n", argv[0]);
        return 2;
    }
    std::map<std::string, std::string> kv;
    for (int i = 3; i < argc; i++) {
        const char* eq = std::strchr(argv[i], '=');
        if (!eq) {
            std::fprintf(stderr, "bad argument %s\n", argv[i]);
            return 2;
        }
        kv[std::string(argv[i], eq - argv[i])] = eq + 1;
    }
    auto get = [&](const char* k, const char* d) { return kv.count(k) ? kv[k] : std::string(d); };
    try {
        Params p;
        p.pixel_step = std::atoi(get("pixel_step", "10").c_str());
        p.min_vector_size = std::atof(get("min_vector_size", "1.0").c_str());
        p.skip_frames = std::atoi(get("skip_frames", "1").c_str());
        p.num_motions = std::atoi(get("num_motions", "2").c_str());
        p.egomotion = std::atoi(get("egomotion", "1").c_str()) != 0;
        p.live_path = std::atoi(get("live_path", "1").c_str()) != 0;
        p.sigma = std::atof(get("sigma", "0.5").c_str());
        p.seed = (uint32_t)std::strtoul(get("seed", "1").c_str(), nullptr, 10);
        p.subspace_precision = std::atoi(get("subspace_precision", "0").c_str());
        const int device = std::atoi(get("device", "0").c_str());
        const std::string out = argv[2];
        const std::vector<Image> frames = read_frames(argv[1]);
        if (frames.empty()) throw std::runtime_error("no frames");

        int k = 0;
        Publisher pub = [&](const std::string& topic, const Image& im) {
            write_bytes(out + "/pub_" + std::to_string(k) + "_" + topic + ".rgb8", im.data.data(), im.data.size());
        };
        MotionDetectionNode node(p, device, (int)frames[0].width, (int)frames[0].height, pub);
        for (size_t fi = 0; fi < frames.size(); fi++) {
            FrameResult r;
            if (!node.image_callback(frames[fi], &r)) continue;
            const int traj_len = r.trajectories.empty() ? 0 : (int)r.trajectories[0].size() / 2;
            int32_t hdr[8] = {r.num_vectors, r.rc, r.w, r.h, r.npts, (int32_t)r.trajectories.size(), traj_len,
                              (int32_t)(r.outlier_points.size() / 2)};
            std::vector<uint8_t> buf((uint8_t*)hdr, (uint8_t*)hdr + sizeof(hdr));
            auto put = [&](const void* q, size_t n) { buf.insert(buf.end(), (const uint8_t*)q, (const uint8_t*)q + n); };
            put(r.H, sizeof(r.H));
            if (!p.live_path) {
                put(r.next_pts.data(), r.next_pts.size() * 4);
                put(r.status.data(), r.status.size());
                put(r.mask.data(), r.mask.size());
            } else {
                for (const auto& t : r.trajectories) put(t.data(), t.size() * 4);
                put(r.outlier_points.data(), r.outlier_points.size() * 4);
                const int32_t nc = (int32_t)r.subspace_columns.size();
                put(&nc, 4);
                put(r.subspace_columns.data(), r.subspace_columns.size() * 4);
                write_trajectories(r.trajectories, out + "/traj_" + std::to_string(k));
            }
            write_bytes(out + "/res_" + std::to_string(k) + ".bin", buf.data(), buf.size());
            write_flow(r.vector_image, r.w, r.h, p.pixel_step, out + "/flow_" + std::to_string(k));
            std::printf("frame %zu -> processed %d: num_vectors %d%s\n", fi, k, r.num_vectors,
                        p.live_path ? (", trajectories " + std::to_string(r.trajectories.size()) + ", outliers " +
                                       std::to_string(r.outlier_points.size() / 2)).c_str()
                                    : "");
            k++;
        }
        std::printf("processed %d of %zu frames\n", k, frames.size());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "mdx_node: %s\n", e.what());
        return 1;
    }
    return 0;
}
