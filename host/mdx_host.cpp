// mdx_host.cpp -- see mdx_host.h.  Reference sites cited per function.
#include "mdx_host.h"

#include <cmath>
#include <cstring>
#include <stdexcept>

namespace mdx_host {

Image to_rgb8(const Image& msg)
{
    int cn;
    if (msg.encoding == "mono8") cn = 1;
    else if (msg.encoding == "rgb8" || msg.encoding == "bgr8") cn = 3;
    else throw std::invalid_argument("unsupported encoding " + msg.encoding);
    if (msg.step < msg.width * (uint32_t)cn || msg.data.size() < (size_t)msg.step * msg.height)
        throw std::invalid_argument("image buffer smaller than step * height");
    Image out;
    out.height = msg.height;
    out.width = msg.width;
    out.encoding = "rgb8";
    out.step = 3 * msg.width;
    out.data.resize((size_t)out.step * out.height);
    for (uint32_t y = 0; y < msg.height; y++) {
        const uint8_t* s = msg.data.data() + (size_t)y * msg.step;
        uint8_t* d = out.data.data() + (size_t)y * out.step;
        for (uint32_t x = 0; x < msg.width; x++) {
            if (cn == 1) {
                d[3 * x] = d[3 * x + 1] = d[3 * x + 2] = s[x];
            } else if (msg.encoding == "bgr8") {
                d[3 * x] = s[3 * x + 2];
                d[3 * x + 1] = s[3 * x + 1];
                d[3 * x + 2] = s[3 * x];
            } else {
                d[3 * x] = s[3 * x];
                d[3 * x + 1] = s[3 * x + 1];
                d[3 * x + 2] = s[3 * x + 2];
            }
        }
    }
    return out;
}

MotionDetectionNode::MotionDetectionNode(const Params& p, int device, int max_w, int max_h, Publisher pub)
    : p_(p), pub_(std::move(pub))
{
    // the library must match the header this node was built against (ABI 4)
    if (mdx_abi_version() != MDX_ABI_VERSION || mdx_params_size() != sizeof(mdx_params))
        throw std::runtime_error("libmdx.so does not match include/mdx.h (ABI / mdx_params size)");
    mdx_params mp;
    mdx_default_params(&mp);
    mp.pixel_step = p_.pixel_step;
    mp.min_vector_size = p_.min_vector_size;
    mp.subspace_precision = p_.subspace_precision;
    ctx_ = mdx_create(device, max_w, max_h, 1, &mp);
    if (!ctx_) throw std::runtime_error(std::string("mdx_create: ") + mdx_create_error());
    mdx_srand(&rng_, p_.seed);
}

MotionDetectionNode::~MotionDetectionNode()
{
    if (ctx_) mdx_destroy(ctx_);
}

void MotionDetectionNode::publish(const std::string& topic, const Image& img) const
{
    if (pub_) pub_(topic, img);
}

// imageCallback (node.cpp:235-455): the frame counter advances on every call -- on a skipped
// frame at :247, on a kept one at :454 (or :315 when no trajectory survives).
bool MotionDetectionNode::image_callback(const Image& msg, FrameResult* out)
{
    const int skip = p_.skip_frames > 0 ? p_.skip_frames : 1;
    if (global_frame_count_ % skip != 0) {
        global_frame_count_++;
        return false;
    }
    const size_t ts = (size_t)trajectory_size();
    if (raw_images_.size() < ts) {                               // :248-261
        raw_images_.push_back(msg);
        if (raw_images_.size() == ts) image_received_ = true;
    } else {
        raw_images_.push_back(msg);
        raw_images_.pop_front();
        image_received_ = true;
    }
    if (p_.live_path) {
        // the device ring mirrors raw_images_: this frame is converted, uploaded and pyramided once
        // (the reference re-converts every ring frame on every callback, :266-287)
        last_rgb_ = to_rgb8(msg);
        const int rc = mdx_ring_push(ctx_, last_rgb_.data.data(), (int)last_rgb_.width, (int)last_rgb_.height,
                                     (int)last_rgb_.step, MDX_FMT_RGB8, (int)raw_images_.size());
        if (rc < 0) throw std::runtime_error(std::string("mdx_ring_push: ") + mdx_last_error(ctx_));
    }
    bool done = false;
    if (p_.use_all_frames && image_received_) {                  // :262
        mdx_params mp;
        mdx_get_params(ctx_, &mp);
        mp.pixel_step = p_.pixel_step;                           // re-read every frame (:264)
        mp.min_vector_size = p_.min_vector_size;
        if (mdx_set_params(ctx_, &mp) != MDX_OK) throw std::runtime_error(mdx_last_error(ctx_));
        FrameResult local;
        FrameResult* r = out ? out : &local;
        if (p_.live_path) {
            run_live((int)raw_images_.size(), r);
        } else {
            // toCvCopy(*iter, "rgb8") (:271) of the two frames the pair path reads
            run_pair(to_rgb8(raw_images_[raw_images_.size() - 2]), to_rgb8(raw_images_.back()), r);
        }
        done = true;
    }
    global_frame_count_++;
    return done;
}

// runOpticalFlow (node.cpp:76-92) -> calculateOpticalFlow (optical_flow_calculator.cpp:30-130)
void MotionDetectionNode::run_pair(const Image& a, const Image& b, FrameResult* r)
{
    const int w = (int)a.width, h = (int)a.height, ps = p_.pixel_step;
    if (b.width != a.width || b.height != a.height) throw std::invalid_argument("frame sizes differ");
    const int npts = mdx_grid_count(w, h, ps), ny = (h + ps - 1) / ps;
    r->w = w;
    r->h = h;
    r->npts = npts;
    r->next_pts.assign((size_t)2 * npts, 0.f);
    r->status.assign(npts, 0);
    r->mask.assign((size_t)w * h, 0);
    std::vector<double> vec((size_t)4 * npts);
    r->rc = mdx_flow_warp_diff(ctx_, a.data.data(), b.data.data(), w, h, (int)a.step, MDX_FMT_RGB8, r->next_pts.data(),
                               r->status.data(), vec.data(), r->mask.data(), r->H, nullptr, &r->num_vectors);
    if (r->rc < 0) throw std::runtime_error(std::string("mdx_flow_warp_diff: ") + mdx_last_error(ctx_));
    // optical_flow_vectors = zeros(rows, cols) (:81), the calculator's Vec4d at each grid point
    r->vector_image.assign((size_t)w * h * 4, 0.0);
    for (int k = 0; k < npts; k++) {
        const int x = (k / ny) * ps, y = (k % ny) * ps;          // x-major grid (:56-64)
        std::memcpy(&r->vector_image[((size_t)y * w + x) * 4], &vec[(size_t)4 * k], 32);
    }
    publish(kTopicFlowMarkers, flow_image(a, r->vector_image, ps, p_.min_vector_size));   // (not :83-85's arrows)
    publish(kTopicMask, mask_image(r->mask, w, h));
}

// runOpticalFlowTrajectory (node.cpp:94-110) over the nimg ring frames already on the device, and,
// with egomotion, fitSubspace (:341-348)
void MotionDetectionNode::run_live(int nimg, FrameResult* r)
{
    const int w = (int)last_rgb_.width, h = (int)last_rgb_.height, ps = p_.pixel_step;
    for (const Image& m : raw_images_)
        if (m.width != last_rgb_.width || m.height != last_rgb_.height) throw std::invalid_argument("frame sizes differ");
    const int npts = mdx_grid_count(w, h, ps);
    r->w = w;
    r->h = h;
    r->npts = npts;
    std::vector<float> traj((size_t)npts * nimg * 2), start((size_t)npts * 2);
    std::vector<int32_t> tlen(npts);
    std::vector<double> vec((size_t)npts * 4);
    const int rc = mdx_ring_trajectory(ctx_, traj.data(), tlen.data(), start.data(), vec.data(), &r->num_vectors);
    if (rc < 0) throw std::runtime_error(std::string("mdx_ring_trajectory: ") + mdx_last_error(ctx_));
    // optical_flow_vectors = zeros (:98); the last pass stores each point's Vec4d at
    // ((int)y, (int)x) of its position entering that pass, in point order
    r->vector_image.assign((size_t)w * h * 4, 0.0);
    for (int k = 0; k < npts; k++) {
        const int x = (int)start[2 * k], y = (int)start[2 * k + 1];
        if (x >= 0 && x < w && y >= 0 && y < h) std::memcpy(&r->vector_image[((size_t)y * w + x) * 4], &vec[4 * k], 32);
    }
    r->trajectories.clear();
    for (int k = 0; k < npts; k++)                              // full-length ones only (:244-249)
        if (tlen[k] == nimg) r->trajectories.emplace_back(&traj[(size_t)k * nimg * 2], &traj[(size_t)(k + 1) * nimg * 2]);
    publish(kTopicFlowMarkers, flow_image(last_rgb_, r->vector_image, ps, p_.min_vector_size));   // (not :101-103's arrows)
    r->outlier_points.clear();
    r->subspace_columns.clear();
    if (r->trajectories.empty() || !p_.egomotion) return;       // :296-318 / :357-389 (clustering: out of scope)
    const int nt = (int)r->trajectories.size(), d = 4 * p_.num_motions;
    std::vector<float> flat((size_t)nt * nimg * 2);
    for (int i = 0; i < nt; i++) std::memcpy(&flat[(size_t)i * nimg * 2], r->trajectories[i].data(), (size_t)nimg * 8);
    std::vector<int> cols(d);
    std::vector<float> outl((size_t)nt * 2);
    int nout = 0;
    const int frc = mdx_fit_subspace(ctx_, flat.data(), nt, nimg, p_.num_motions, p_.sigma, &rng_, cols.data(), nullptr,
                                     nullptr, outl.data(), &nout);
    if (frc < 0) throw std::runtime_error(std::string("mdx_fit_subspace: ") + mdx_last_error(ctx_));
    r->outlier_points.assign(outl.begin(), outl.begin() + 2 * nout);
    for (int c : cols)
        if (c >= 0) r->subspace_columns.push_back(c);
}

Image mask_image(const std::vector<uint8_t>& mask, int w, int h)
{
    Image im;
    im.width = w;
    im.height = h;
    im.encoding = "rgb8";                                      // publishImage's encoding (:220)
    im.step = 3 * w;
    im.data.resize((size_t)3 * w * h);
    for (size_t i = 0; i < (size_t)w * h; i++) im.data[3 * i] = im.data[3 * i + 1] = im.data[3 * i + 2] = mask[i];
    return im;
}

Image flow_image(const Image& rgb, const std::vector<double>& vi, int pixel_step, double mvs)
{
    Image im = rgb;
    const int w = (int)rgb.width, h = (int)rgb.height;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const double* e = &vi[((size_t)y * w + x) * 4];
            // the vectors showOpticalFlowVectors draws (optical_flow_visualizer.cpp:37)
            if ((std::fabs(e[2]) > mvs || std::fabs(e[3]) > mvs) && std::fabs(e[2]) < pixel_step * 5 &&
                std::fabs(e[3]) < pixel_step * 5) {
                const int sx = (int)e[0], sy = (int)e[1];
                if (sx < 0 || sx >= w || sy < 0 || sy >= h) continue;
                uint8_t* p = &im.data[(size_t)sy * im.step + 3 * (size_t)sx];
                p[0] = 0;
                p[1] = 0;
                p[2] = 255;                                    // CV_RGB(0, 0, 255) in an rgb8 image
            }
        }
    return im;
}

// writeFlow (optical_flow_calculator.cpp:509-541): grid rows i = 0, ps, .. and columns j = 0, ps, ..
// of the Vec4d image; a lost point (x == -1) writes 0.0
void write_flow(const std::vector<double>& vi, int w, int h, int ps, const std::string& filename)
{
    std::ofstream hf(filename + "_h"), vf(filename + "_f");
    for (int i = 0; i < h; i += ps) {
        for (int j = 0; j < w; j += ps) {
            if (j) {
                hf << ", ";
                vf << ", ";
            }
            const double* e = &vi[((size_t)i * w + j) * 4];
            if (e[0] == -1.0) {
                hf << 0.0;
                vf << 0.0;
            } else {
                hf << e[2];
                vf << e[3];
            }
        }
        hf << std::endl;
        vf << std::endl;
    }
}

// writeTrajectories (:543-562): "x0, y0, x1, y1, ..." per trajectory, float32 values
void write_trajectories(const std::vector<std::vector<float>>& trajectories, const std::string& filename)
{
    std::ofstream tf(filename);
    for (const auto& t : trajectories) {
        for (size_t j = 0; j + 1 < t.size(); j += 2) {
            if (j) tf << ", ";
            tf << t[j] << ", " << t[j + 1];
        }
        tf << std::endl;
    }
}

// MotionLogger::writeContour / writeBoundingBox (motion_logger.cpp:31-47); cv::Rect br() = tl + size
void MotionLogger::write_contour(const std::vector<int>& xy, int frame_number, int contour_id)
{
    out_ << frame_number << ", " << contour_id;
    for (size_t i = 0; i + 1 < xy.size(); i += 2) out_ << ", " << xy[i] << ", " << xy[i + 1];
    out_ << std::endl;
}

void MotionLogger::write_bounding_box(int x, int y, int width, int height, int frame_number, int contour_id)
{
    out_ << frame_number << ", " << contour_id << ", " << x << ", " << y << ", " << x + width << ", " << y + height
         << std::endl;
}

}  // namespace mdx_host
